"""Residency-map checkpoint.

The reference has no user-visible residency checkpoint; its closest artifacts
are UVM_TEST_VA_RESIDENCY_INFO (uvm_test_ioctl.h:626-674) and FB save/restore
(FBSR, fbsr.c:37-104, ``FBSR_TYPE_FILE``). This format combines both:

  header   "OGKMRMAP" | u32 version=2 | u32 flags (bit0 = data present) | u64 nranges
  range    u64 id | u32 type | u32 flags | u64 size | u64 nblocks | u32 name_len | name
           | u64 group_id | u8 group_migratable
           | (v2) u64 cpu_view_addr | u64 stable_dev_va | i32 stable_dev
  block*   u64 index | u32 npages | u8 read_dup | u8 has_preferred | u8 pref_tier | i16 pref_id
           | u64 accessed_by | u8 thrash_pinned | u32 nres
           | nres x (u8 tier | i16 id | 64 B resident page mask over the 512 4 KB pages)
  data     (flags bit0) nblocks x block bytes, appended after each range's block table

``save`` quiesces the rings first (the uvm_suspend analog, uvm_global.c:272-415).
"""
from __future__ import annotations

import json
import struct
from pathlib import Path

from ._native import lib

TIERS = {0: "gpu", 1: "host", 2: "cxl"}


def save(path: str | Path, with_data: bool = False) -> None:
    lib.checkpoint_save(str(path), with_data)


def load(path: str | Path, with_data: bool = True, in_place: bool = False) -> list[int]:
    """Recreate the recorded ranges (ids returned in file order), their
    policies, and - with data - their contents at the recorded locations.
    ``in_place``: the ranges keep their recorded ids, CPU windows and stable
    device VAs (a resumed process finds its pointers valid); fails with BUSY
    if one is taken. Otherwise ranges get new ids and VAs."""
    return list(lib.checkpoint_load(str(path), with_data, in_place))


def describe(path: str | Path) -> dict:
    """Pure-Python parser of the binary format (no native code needed)."""
    b = Path(path).read_bytes()
    pos = 0

    def take(fmt):
        nonlocal pos
        v = struct.unpack_from("<" + fmt, b, pos)
        pos += struct.calcsize("<" + fmt)
        return v if len(v) > 1 else v[0]

    magic = b[:8]
    if magic != b"OGKMRMAP":
        raise ValueError("not a residency map")
    pos = 8
    version, flags, n = take("I"), take("I"), take("Q")
    out = {"version": version, "with_data": bool(flags & 1), "ranges": []}
    for _ in range(n):
        rid, rtype, rflags, size, nblocks, nl = take("Q"), take("I"), take("I"), take("Q"), take("Q"), take("I")
        name = b[pos:pos + nl].decode()
        pos += nl
        gid, gm = take("Q"), take("B")
        addrs = {}
        if version >= 2:
            addrs = {"cpu_view": take("Q"), "dev_va": take("Q"), "stable_dev": take("i")}
        blocks = []
        for _ in range(nblocks):
            idx, npages, rd, hp, pt, pid, ab, pinned, nres = (take("Q"), take("I"), take("B"), take("B"), take("B"),
                                                              take("h"), take("Q"), take("B"), take("I"))
            res = []
            for _ in range(nres):
                t, lid = take("B"), take("h")
                words = struct.unpack_from("<8Q", b, pos)
                pos += 64
                res.append({"loc": f"{TIERS.get(t, t)}:{lid}", "pages": sum(bin(w).count("1") for w in words)})
            blocks.append({"index": idx, "npages": npages, "read_dup": bool(rd),
                           "preferred": f"{TIERS.get(pt, pt)}:{pid}" if hp else None, "accessed_by": ab,
                           "thrash_pinned": bool(pinned), "resident": res})
        if flags & 1:
            pos += size
        out["ranges"].append({"id": rid, "type": rtype, "flags": rflags, "size": size, "name": name,
                              "group": gid, "group_migratable": bool(gm), "blocks": blocks, **addrs})
    return out


def to_json(path: str | Path) -> str:
    return json.dumps(describe(path), indent=1)
