#!/usr/bin/env python3
"""Build the native core of the framework for MI355X (gfx950).

Compiles every C++/HIP source under csrc/ with hipcc (parallel, mtime-cached
objects under build/obj) and links the pybind11 extension
``open-gpu-kernel-modules_amd/_ogkm<EXT_SUFFIX>`` in-tree, so the built .so
travels with the repo snapshot to the GPU box.

    python tools/build_native.py [--debug] [--clean] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "open-gpu-kernel-modules_amd"
CSRC = ROOT / "csrc"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def ext_path() -> Path:
    return PKG / ("_ogkm" + sysconfig.get_config_var("EXT_SUFFIX"))


def sources() -> list[Path]:
    out = []
    for sub in ("core", "kernels", "python"):
        for p in sorted((CSRC / sub).glob("*")):
            if p.suffix in (".cpp", ".hip"):
                out.append(p)
    return out


def headers_mtime() -> float:
    return max((p.stat().st_mtime for p in (CSRC / "include").rglob("*.hpp")), default=0.0)


def compile_one(src: Path, obj: Path, flags: list[str], hdr_mtime: float) -> tuple[Path, str]:
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr_mtime):
        return obj, ""
    obj.parent.mkdir(parents=True, exist_ok=True)
    # hipcc compiles .cpp as HIP too: every TU targets gfx950 only.
    cmd = [str(ROCM / "bin" / "hipcc")] + flags + [f"--offload-arch={ARCH}"]
    if src.suffix == ".hip":
        cmd += ["-x", "hip"]
    cmd += ["-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(debug: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    flags = [
        "-std=c++17",
        "-fPIC",
        "-O1" if debug else "-O3",
        "-g" if debug else "-g0",
        "-Wall",
        "-Wno-unused-result",
        "-Wno-unused-variable",
        "-Wno-unused-function",
        "-Wno-sign-compare",
        "-fvisibility=hidden",
        f"-I{CSRC / 'include'}",
        f"-I{py_inc}",
        f"-I{pybind11.get_include()}",
        f"-I{ROCM / 'include'}",
    ]
    if debug:
        flags.append("-DOGKM_DEBUG")
    objdir = ROOT / "build" / ("obj-debug" if debug else "obj")
    hdr = headers_mtime()
    srcs = sources()
    jobs = jobs or min(8, os.cpu_count() or 4)
    objs = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(compile_one, s, objdir / (s.stem + s.suffix.replace(".", "_") + ".o"), flags, hdr): s
                for s in srcs}
        for f in cf.as_completed(futs):
            obj, log = f.result()
            if verbose and log:
                print(log, file=sys.stderr)
            objs.append(obj)
    out = ext_path()
    newest = max(o.stat().st_mtime for o in objs)
    if out.exists() and out.stat().st_mtime >= newest:
        return out
    # link to a temporary file and rename it over the old library: processes
    # that have the old one mapped (a running test suite) keep their inode
    tmp = out.with_name(out.name + ".tmp")
    link = [str(ROCM / "bin" / "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp)]
    link += [str(o) for o in sorted(objs)]
    link += [f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}", "-lamdhip64", "-lhsa-runtime64",
             "-lrocprofiler-sdk-roctx", "-lnuma",
             "-lpthread"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(link)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    if a.clean:
        shutil.rmtree(ROOT / "build" / "obj", ignore_errors=True)
        shutil.rmtree(ROOT / "build" / "obj-debug", ignore_errors=True)
        if ext_path().exists():
            ext_path().unlink()
    print(build(debug=a.debug, jobs=a.j, verbose=a.v))


if __name__ == "__main__":
    main()
