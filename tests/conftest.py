"""Test configuration.

Markers
  gpu   needs a real MI355X (HIP backend); everything else runs on the CPU with
        the fake backend (memfd "HBM", worker-thread streams, memcpy copies) -
        the analog of the reference's fake CE HAL (uvm_page_tree_test.c:65-100).
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# Test models are tiny: no unit-size floor, so their FFN matrices still split
# into several streamed row parts (the multi-part path stays covered).
os.environ.setdefault("OGKM_UNIT_MIN_MB", "0")

import ogkm  # noqa: E402  (builds/loads the native core)
from ogkm import rt  # noqa: E402
from ogkm._native import lib  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (HIP backend)")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def fake_rt():
    """A runtime on the fake backend: 2 devices x 64 MB HBM, lock checker on."""
    if lib.is_initialized():
        lib.shutdown()
    lib.config_reset()
    lib.clear_fatal_for_test()
    # packed host copies off: tests that count link bytes see raw transfers
    # (tests/test_packing*.py turn it on)
    rt.init("fake", fake_devices=2, fake_hbm_mb=64, lock_check=1, host_budget_mb=1024, pack_host_copies=0)
    lib.reset_lock_violations()
    lib.reset_counters()
    yield rt
    violations = lib.lock_violations()
    lib.shutdown()
    lib.config_reset()
    lib.clear_fatal_for_test()
    assert violations == 0, f"lock order violations: {violations}"


@pytest.fixture
def gpu_rt():
    if not gpu_available():
        pytest.skip("no GPU")
    if lib.is_initialized():
        lib.shutdown()
    lib.config_reset()
    lib.clear_fatal_for_test()
    rt.init("hip", lock_check=1, host_budget_mb=16384, hbm_budget={0: 2 << 30}, pack_host_copies=0)
    lib.reset_lock_violations()
    lib.reset_counters()
    yield rt
    violations = lib.lock_violations()
    lib.shutdown()
    lib.config_reset()
    assert violations == 0, f"lock order violations: {violations}"
