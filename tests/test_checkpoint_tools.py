"""Residency-map checkpoint, tools event queues / counters, config system."""
from __future__ import annotations

import os

import torch

from ogkm import checkpoint, rt, tools
from ogkm._native import lib

MB = 1 << 20


def test_checkpoint_roundtrip_with_data(fake_rt, tmp_path):
    a = rt.malloc_managed(5 * MB + 100, "weights")
    da = torch.randint(0, 256, (a.size,), dtype=torch.uint8)
    a.write(da)
    a.set_read_mostly(True)
    a.prefetch("gpu:0").wait()            # read-duplicated on gpu0 + host
    b = rt.malloc_managed(3 * MB, "kv")
    b.set_preferred_location("gpu:1")
    db = torch.randint(0, 256, (b.size,), dtype=torch.uint8)
    b.write(db)
    p = tmp_path / "rmap.bin"
    checkpoint.save(p, with_data=True)
    desc = checkpoint.describe(p)
    assert desc["with_data"] and [r["name"] for r in desc["ranges"]] == ["weights", "kv"]
    blk0 = desc["ranges"][0]["blocks"][0]
    assert blk0["read_dup"] and {x["loc"] for x in blk0["resident"]} == {"host:0", "gpu:0"}
    assert desc["ranges"][1]["blocks"][0]["preferred"] == "gpu:1"
    a.free()
    b.free()
    ids = checkpoint.load(p, with_data=True)
    na, nb = rt.ManagedBuffer(ids[0]), rt.ManagedBuffer(ids[1])
    assert torch.equal(na.read(), da) and torch.equal(nb.read(), db)
    assert {(r["tier"], r["id"]) for r in na.residency(0)["resident_on"]} == {("host", 0), ("gpu", 0)}
    assert nb.residency(0)["preferred"] == {"tier": "gpu", "id": 1}
    assert ("gpu", 1) in {(r["tier"], r["id"]) for r in nb.residency(0)["resident_on"]}
    assert "weights" in checkpoint.to_json(p)


def test_checkpoint_map_only(fake_rt, tmp_path):
    a = rt.malloc_managed(2 * MB, "x")
    a.fill(3)
    p = tmp_path / "m.bin"
    checkpoint.save(p, with_data=False)
    assert not checkpoint.describe(p)["with_data"]
    ids = checkpoint.load(p, with_data=False)
    assert len(ids) == 1 and lib.range_info(ids[0])["size"] == 2 * MB


def test_in_place_restore_is_all_or_nothing(fake_rt, tmp_path):
    """An in-place restore whose second range's id / address is taken fails
    without leaving the first range behind; the relocating restore the caller
    falls back to then creates exactly one copy of each range."""
    import pytest

    a = rt.malloc_managed(2 * MB, "first")
    a.fill(1)
    b = rt.malloc_managed(2 * MB, "second")
    b.fill(2)
    p = tmp_path / "ip.bin"
    checkpoint.save(p, with_data=True)
    a_id = a.id
    a.free()  # the first range's id and addresses are free again, the second's are not
    with pytest.raises(Exception, match="BUSY"):
        checkpoint.load(p, with_data=True, in_place=True)
    with pytest.raises(Exception):
        lib.range_info(a_id)  # rolled back, not leaked
    ids = checkpoint.load(p, with_data=True)
    assert len(ids) == 2
    assert int(rt.ManagedBuffer(ids[0]).read()[0]) == 1 and int(rt.ManagedBuffer(ids[1]).read()[0]) == 2
    b.free()


def test_tools_event_queue(fake_rt):
    q = tools.EventQueue(entries=1024, events=["Migration", "Eviction", "ReadDuplicate"])
    b = rt.malloc_managed(4 * MB, "ev")
    b.fill(1)
    b.migrate("gpu:0")
    ev = q.read_dicts()
    mig = [e for e in ev if e["type"] == "Migration" and e["dst"] == "gpu:0"]
    assert sum(e["bytes"] for e in mig) == 4 * MB
    assert all(e["range_id"] == b.id for e in mig)
    # overflow accounting
    small = tools.EventQueue(entries=2, events=["Migration"])
    b.migrate("host:0")
    b.migrate("gpu:1")
    assert small.dropped().get("Migration", 0) > 0
    q.close()
    small.close()


def test_tools_queue_shm_visible(fake_rt):
    name = f"/ogkm-test-{os.getpid()}"
    q = tools.EventQueue(entries=64, shm_name=name)
    assert os.path.exists("/dev/shm" + name)
    q.close()
    assert not os.path.exists("/dev/shm" + name)


def test_counters_and_prometheus(fake_rt):
    b = rt.malloc_managed(2 * MB, "c")
    b.fill(1)
    b.migrate("gpu:0")
    c = tools.counters()
    assert c["bytes_xfer_htd"] == 2 * MB
    txt = tools.prometheus_text()
    assert "ogkm_bytes_xfer_htd 2097152" in txt
    tools.reset_counters()
    assert tools.counters()["bytes_xfer_htd"] == 0


def test_config_knobs_match_reference_defaults(fake_rt):
    names = rt.config_names()
    expect = {"perf_prefetch_threshold": 51, "perf_thrashing_threshold": 3, "perf_thrashing_pin_threshold": 10,
              "perf_thrashing_lapse_usec": 500, "perf_fault_batch_count": 256,
              "perf_access_counter_threshold": 256, "channel_num_gpfifo_entries": 1024, "cxl_max_buffers": 256,
              "cxl_pin_budget_pct": 90}
    for k, v in expect.items():
        assert k in names and rt.get_config(k) == v
    rt.configure(perf_prefetch_threshold=75)
    assert rt.get_config("perf_prefetch_threshold") == 75


def test_config_env_override(tmp_path):
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, %r); import ogkm; from ogkm._native import lib; "
            "print(lib.get_config('perf_prefetch_threshold'))") % os.path.dirname(os.path.dirname(__file__))
    env = dict(os.environ, RT_PERF_PREFETCH_THRESHOLD="77")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.stdout.strip().endswith("77"), out.stderr


def test_tools_process_memory_read_write(fake_rt):
    """Read / write managed memory by address wherever it lives (host, HBM)."""
    b = rt.malloc_managed(4 * MB, "pm")
    ref = torch.arange(MB, dtype=torch.int32)
    b.write(ref)
    b.migrate("gpu:0", 2 * MB, 2 * MB)                 # second half lives in HBM
    got = tools.read_process_memory(b.addr + 2 * MB - 8, 16)
    assert torch.equal(torch.frombuffer(bytearray(got), dtype=torch.int32), ref[MB // 2 - 2:MB // 2 + 2])
    tools.write_process_memory(b.addr + 3 * MB, torch.tensor([7, 8], dtype=torch.int32).numpy().tobytes())
    back = b.read().view(torch.int32)
    assert back[(3 * MB) // 4].item() == 7 and back[(3 * MB) // 4 + 1].item() == 8
    b.free()


def test_tools_prefetch_and_page_size_change_events(fake_rt):
    q = tools.EventQueue(events=["Prefetch", "PageSizeChange"])
    b = rt.malloc_managed(4 * MB, "ev")
    b.write(torch.ones(4 * MB, dtype=torch.uint8))
    lib.device_table(b.id)                               # the GPU view of the range
    b.prefetch("gpu:0").wait()
    lib.poll_device_faults(0)
    b.migrate("host:0")
    types = [e["type"] for e in q.read_dicts()]
    q.close()
    assert "Prefetch" in types
    assert types.count("PageSizeChange") >= 2            # 2 MB mapping on, then off
    b.free()
