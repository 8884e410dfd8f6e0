"""Build and run the native core unit tests (tests/native/test_core.cpp) with
g++ under AddressSanitizer + UndefinedBehaviorSanitizer and under
ThreadSanitizer - host code only, the fake backend replaces HIP (GPU sanitizers
are not available on this pool). Mirrors the reference's UBSAN build option
(kernel-open/Kbuild:55-58) and its lock-order checker tests (uvm_lock_test.c)."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CORE = [p for p in sorted((ROOT / "csrc" / "core").glob("*.cpp"))
        if p.name not in ("backend_hip.cpp",)]


def _build(kind: str, flags: list[str]) -> Path:
    out_dir = ROOT / "build" / f"native-{kind}"
    out_dir.mkdir(parents=True, exist_ok=True)
    exe = out_dir / "test_core"
    srcs = CORE + [ROOT / "tests" / "native" / "test_core.cpp"]
    hdrs = list((ROOT / "csrc" / "include").rglob("*.hpp"))
    newest = max(p.stat().st_mtime for p in srcs + hdrs)
    if exe.exists() and exe.stat().st_mtime >= newest:
        return exe
    cxx = shutil.which("g++") or "g++"
    objs = []
    procs = []
    for s in srcs:
        o = out_dir / (s.stem + ".o")
        objs.append(o)
        if o.exists() and o.stat().st_mtime >= max(s.stat().st_mtime, max(p.stat().st_mtime for p in hdrs)):
            continue
        procs.append(subprocess.Popen([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags,
                                       f"-I{ROOT / 'csrc' / 'include'}", "-c", str(s), "-o", str(o)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        if len(procs) >= 8:
            for p in procs:
                _, err = p.communicate()
                assert p.returncode == 0, err
            procs = []
    for p in procs:
        _, err = p.communicate()
        assert p.returncode == 0, err
    r = subprocess.run([cxx, *flags, *map(str, objs), "-o", str(exe), "-lnuma", "-lpthread"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def _run(exe: Path, env_extra: dict) -> None:
    env = dict(os.environ, **env_extra)
    env.pop("LD_PRELOAD", None) if "LD_PRELOAD" in env and "asan" in env.get("LD_PRELOAD", "") else None
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "ALL NATIVE TESTS PASSED" in r.stderr, r.stderr[-6000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_core_asan_ubsan():
    exe = _build("asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    _run(exe, {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:allow_user_segv_handler=1", "UBSAN_OPTIONS": "print_stacktrace=1",
               "RT_LOG": "error"})


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_core_tsan():
    exe = _build("tsan", ["-fsanitize=thread"])
    _run(exe, {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1", "RT_LOG": "error"})
