"""Importable alias for the ``open-gpu-kernel-modules_amd`` package (whose
directory name is not a Python identifier): ``import ogkm`` works from the repo
root and resolves every submodule to the same module objects."""
import importlib as _importlib
import sys as _sys

_pkg = _importlib.import_module("open-gpu-kernel-modules_amd")
_sys.modules[__name__] = _pkg
