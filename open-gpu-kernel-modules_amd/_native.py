"""Loader for the native core (``_ogkm`` pybind11 extension, built in-tree).

The extension is built by ``tools/build_native.py`` (also run by
``__graft_entry__.build()``). There is deliberately no Python fallback: if the
extension is missing the import fails loudly, so a GPU run can never silently
measure a pure-Python path.
"""
from __future__ import annotations

import importlib
import os
import sysconfig
from pathlib import Path

_PKG_DIR = Path(__file__).resolve().parent
SO_PATH = _PKG_DIR / ("_ogkm" + sysconfig.get_config_var("EXT_SUFFIX"))


def _load():
    # PyTorch-ROCm bundles its own libamdhip64 / libhsa-runtime64 (same sonames as
    # /opt/rocm). Import torch first so the extension binds to the copy torch
    # already loaded: two HIP runtimes in one process cannot share the GPU.
    import torch  # noqa: F401

    if not SO_PATH.exists():
        if os.environ.get("OGKM_AUTOBUILD", "1") == "1":
            import subprocess
            import sys

            root = _PKG_DIR.parent
            subprocess.run([sys.executable, str(root / "tools" / "build_native.py")], check=True)
        if not SO_PATH.exists():
            raise ImportError(f"native core not built: {SO_PATH} (run python tools/build_native.py)")
    return importlib.import_module(__package__ + "._ogkm")


lib = _load()
RuntimeStatusError = lib.RuntimeStatusError
