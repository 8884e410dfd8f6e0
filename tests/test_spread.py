"""Runtime-decided keep / stream classes (csrc/core/spread.cpp, ogkm/spread.hpp)
on the fake backend: a cyclic access sequence 1.5x the HBM arena, hinted with
next uses only - no caller-side classes. The runtime finds the cycle, sizes a
keep class to its arena and spreads it over the use order; each pass then
streams only the stream class and keeps the keep class resident. Reference:
residency chosen by the runtime from faults and policy (uvm_va_block.c:
11560-11760; victim order uvm_pmm_gpu.c:1460-1500)."""
from __future__ import annotations

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20
UNIT_MB = 2
N_UNITS = 48          # 96 MB cycle
ARENA_MB = 64         # 32 chunks: the cycle is 1.5x the arena


def _run_cycle(passes: int, spread: bool, window: int = 2, after_pass=None):
    lib.configure("perf_spread_enable", 1 if spread else 0)
    lib.configure("arena_victim_rerank", 1)  # exact next-use victim order (the fake arena is tiny)
    lib.init_device(0, ARENA_MB * MB)
    units = []
    for i in range(N_UNITS):
        b = rt.malloc_managed(UNIT_MB * MB, f"unit{i}", cpu_view=False)
        b.set_preferred_location("gpu:0")
        b.set_read_mostly(True)
        b.write(torch.full((UNIT_MB * MB,), i % 251, dtype=torch.uint8))
        units.append(b)
    lib.reset_op_clock(0)
    n = len(units)
    per_pass, keep_ev = [], []
    for p in range(passes):
        h0 = lib.stats()["bytes_xfer_htd"]
        for j, u in enumerate(units):
            t = p * n + j
            lib.set_op_clock(0, t)
            for k in range(1, window + 1):  # the prefetch window, floored at each unit's own use
                try:
                    units[(j + k) % n].prefetch("gpu:0", needed_at=t + k)
                except lib.RuntimeStatusError:
                    break
            lease = u.acquire(0, rt.READ)
            lease.wait(0)
            lease.release(0)
            u.hint_next_use(t + n)
        per_pass.append(lib.stats()["bytes_xfer_htd"] - h0)
        keep_ev.append(lib.spread_stats(0)["keep_evictions"])
        if after_pass:
            after_pass(p)
    resident = [u.resident_bytes("gpu:0") == u.size for u in units]
    st = lib.spread_stats(0)
    ok = all(bytes(u.read()[:4]) == bytes([i % 251] * 4) for i, u in enumerate(units))
    for u in units:
        u.free()
    st["keep_evictions_per_pass"] = [b - a for a, b in zip([0] + keep_ev, keep_ev)]
    return st, per_pass, resident, ok


def test_runtime_spread_reaches_keep_share_on_cyclic_hints(fake_rt):
    st, per_pass, resident, ok = _run_cycle(passes=6, spread=True)
    assert ok
    assert st["ready"] and st["passes"] >= 4 and st["ranges"] == N_UNITS
    cap = ARENA_MB * MB
    # the runtime held back its observed prefetch window (2 units ahead + the one in use)
    assert st["window_reserve"] == 3 * UNIT_MB * MB, st
    # keep class = 97 % of the rest of the arena (nothing pinned between uses), within one unit of diffusion
    want = 0.97 * (cap - st["window_reserve"])
    assert want - UNIT_MB * MB <= st["keep_bytes"] <= want + UNIT_MB * MB, st
    # the discovery pass and the one after it move data between the classes; then the keep class stays put
    assert st["adaptations"] == 0 and sum(st["keep_evictions_per_pass"][3:]) == 0, st
    # steady passes stream about the stream class (what does not fit), not the whole cycle
    stream_bytes = N_UNITS * UNIT_MB * MB - st["keep_bytes"]
    for b in per_pass[-3:]:
        assert b <= stream_bytes + 6 * UNIT_MB * MB, (per_pass, st)
    # the resident set is spread over the cycle: no long run of streamed units
    run, longest = 0, 0
    for r in resident + resident:
        run = 0 if r else run + 1
        longest = max(longest, run)
    assert longest <= 4, resident


def test_runtime_spread_off_keeps_one_contiguous_run(fake_rt):
    """Without the classes, plain Belady keeps one contiguous stretch of the
    cycle resident - the pattern the spread classes exist to break up."""
    st, per_pass, resident, ok = _run_cycle(passes=5, spread=False)
    assert ok
    assert st["ranges"] == 0  # the policy never saw a hint
    run, longest = 0, 0
    for r in resident + resident:
        run = 0 if r else run + 1
        longest = max(longest, run)
    assert longest >= 8, resident


def test_spread_adapts_down_on_keep_evictions(fake_rt):
    """Capacity the classes did not account for disappears (another user pins
    8 MB of the arena after the classes were set): keep-class data is evicted,
    and after that pass the runtime shrinks the keep class (online adaptation
    from refaults) until it fits again."""
    held = []
    lib.configure("perf_spread_adapt", 1)

    def squeeze(p):
        if p == 3:
            held.append(lib.torch_alloc(8 * MB, 0))  # pinned allocator chunks

    st, per_pass, resident, ok = _run_cycle(passes=12, spread=True, after_pass=squeeze)
    for ptr in held:
        lib.torch_free(ptr, 0)
    assert ok
    assert st["adaptations"] >= 1, st
    assert st["keep_bytes"] < 0.97 * (ARENA_MB * MB - st["window_reserve"]) - UNIT_MB * MB, st
    # settled: the last passes evict no keep-class data
    assert sum(st["keep_evictions_per_pass"][-2:]) == 0, st


def test_reset_op_clock_forgets_the_cycle(fake_rt):
    st, _, _, _ = _run_cycle(passes=2, spread=True)
    assert st["ranges"] == N_UNITS
    lib.reset_op_clock(0)
    assert lib.spread_stats(0)["ranges"] == 0


@pytest.mark.parametrize("spread", [True, False])
def test_partial_victim_ranking_matches_full(fake_rt, spread):
    """A victim-cache rebuild that ranks only the best few chunks (the default
    ranks 4096 - here 1, so the 32-chunk arena takes the partial path on every
    rebuild) picks the same victims as ranking every chunk: identical traffic
    per pass and the same resident set."""
    lib.configure("arena_victim_cache_ops", 4)
    lib.configure("arena_victim_rank_top", 0)
    full = _run_cycle(passes=4, spread=spread)
    lib.configure("arena_victim_rank_top", 1)
    part = _run_cycle(passes=4, spread=spread)
    assert full[3] and part[3]
    assert full[1] == part[1] and full[2] == part[2]
