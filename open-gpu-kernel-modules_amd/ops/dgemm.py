"""Decode GEMM: ``out = epilogue(x @ W^T)`` for decode batches on the MFMA cores,
reading W straight from the format it rests in (csrc/kernels/decode_gemm.hip).

W is stored in *fragment order* (16 x 32 tiles, 1 KB each, lane-major = the
A-operand fragment of v_mfma_f32_16x16x32_bf16), either as raw bf16 or inside a
BF11 packed stream (ops/bf12.py, "bf11s": BF11-or-raw chunks) that the kernel
decodes in registers - the packed bytes are the only weight bytes read from HBM
and no bf16 staging copy exists. Epilogues are fused into the split-K sum
(in-kernel for raw weights: the last-arriving wave of each output group runs
it; a k_dgemm_reduce launch otherwise):
``store``, ``resid`` (out = resid + x @ W^T, in place allowed) and ``silu_mul``
(W = [gate; up] rows, out = silu(gate) * up).

This replaces the library GEMM the reference-free design started with
(hipBLASLt at M = 64 moved only ~0.3-0.9 TB/s of weights; profiles/).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from .._native import lib
from . import bf12

EPI = {"store": 0, "resid": 1, "silu_mul": 2}
# Waves per GEMM (~3 per CU): fewer K splits keep the f32 split-K partials
# small - measured best at Llama-3 8B and 70B decode shapes (profiles/r2_dgemm_sweep.txt:
# 768 -> 2.71 / 3.86 TB/s vs 2048 -> 2.19 / 3.45 TB/s).
TARGET_UNITS = int(os.environ.get("OGKM_DGEMM_UNITS", "768"))
# Packed (BF11) weights decode in registers - ALU-heavy, they need the waves:
TARGET_UNITS_PACKED = int(os.environ.get("OGKM_DGEMM_UNITS_PACKED", "2048"))
# Raw weights: k_dgemm_lds (row tile per wave, activations shared in LDS, 4x
# fewer K splits at equal waves). Round 2 measured it 8-13% ahead at N <= 8192;
# against k_dgemm_pipe it no longer wins at 8B shapes and loses 35% on the 70B
# down projection (8192 x 28672: 172 vs 127 us; profiles/r3_dgemm_sweep.txt).
# -1 = auto (N <= 8192), 0 off (default), 1 on.
LDS_X = int(os.environ.get("OGKM_DGEMM_LDS", "0"))
LDS_MAX_N = 8192
UNROLL = int(os.environ.get("OGKM_DGEMM_UNROLL", "0"))  # K steps per pipelined block (0 = kernel default)
# Raw weights on the split-K path: k_dgemm_pipe (two-deep register pipeline,
# unconditional loads) instead of k_dgemm<RAW>, in one-wave workgroups (a
# GEMM's few hundred units spread over all 256 CUs; 4-wave workgroups leave
# CUs idle), 768 waves per GEMM (1024 for matrices of >= 400 M elements).
# Measured, graph-timed incl. the reduce (profiles/r3_dgemm_sweep.txt):
# 8B layer 0.155 -> 0.144 ms (3.04 TB/s), 70B layer 0.430 -> 0.408 ms (4.19 TB/s).
PIPE = int(os.environ.get("OGKM_DGEMM_PIPE", "1"))
WG_WAVES = int(os.environ.get("OGKM_DGEMM_WG", "1"))
TARGET_UNITS_PIPE = int(os.environ.get("OGKM_DGEMM_UNITS_PIPE", "768"))
TARGET_UNITS_PIPE_LARGE = int(os.environ.get("OGKM_DGEMM_UNITS_PIPE_LARGE", "1024"))
LARGE_ELEMS = 400 << 20
# Pipelined raw path kernel: 0 = auto (below), 4 = k_dgemm_pipe (two register
# sets of 2 K steps), 10 D = k_dgemm_lring (LDS ring of D K steps, D = 3..7).
# (A register ring of 3+ sets was tried and dropped: profiles/r3_dgemm_xfrag.md.)
DEPTH = int(os.environ.get("OGKM_DGEMM_DEPTH", "0"))
# Auto: the LDS ring (5 slots = 20 KB of weights in flight per wave) at 512
# waves when each wave's K range is short (<= LRING_MAX_STEPS 32-wide steps:
# ramp-dominated units - every decode shape of Llama-3 8B and the 70B
# attention projections), else k_dgemm_pipe at TARGET_UNITS_PIPE(_LARGE).
# Measured per shape, graph-timed incl. the reduce (profiles/r3_dgemm_depth.txt):
# 8B layer 0.143 -> 0.110 ms; 70B q/k/v+o 0.087 -> 0.066 ms; the long-K units
# (70B gate/up with one K split, down with 224 steps) stay on k_dgemm_pipe.
LRING_DEPTH = int(os.environ.get("OGKM_DGEMM_LRING_DEPTH", "50"))
LRING_UNITS = int(os.environ.get("OGKM_DGEMM_LRING_UNITS", "512"))
LRING_MAX_STEPS = int(os.environ.get("OGKM_DGEMM_LRING_MAX_STEPS", "96"))
# Split-K fixup inside the pipelined raw kernels (the last-arriving wave of an
# output group sums the splits and runs the epilogue) instead of a
# k_dgemm_reduce launch; 0 = always launch the reduce.
# Measured slower on config 2 (7.84 vs 6.43 ms/step, profiles/r4_config2.md):
# every wave's agent-scope release writes its XCD's L2 back - off by default.
FIXUP = int(os.environ.get("OGKM_DGEMM_FIXUP", "0"))
# One K split (the LM head's row blocks outnumber the waves): the kernel
# writes the store / resid epilogue from its accumulators - no partials.
DIRECT = int(os.environ.get("OGKM_DGEMM_DIRECT", "1"))
FIX_SLOTS = 1 << 16  # arrival counters per (device, stream): grid.y x row blocks


def frag_permute(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> flat fragment order (N % 16 == 0, K % 32 == 0)."""
    n, k = w.shape
    if n % 16 or k % 32:
        raise ValueError(f"fragment order needs N % 16 == 0 and K % 32 == 0, got {tuple(w.shape)}")
    # W[16 rt + r][32 ks + 8 h + j] -> offset ((rt * K/32 + ks) * 64 + 16 h + r) * 8 + j
    return w.reshape(n // 16, 16, k // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(-1)


def frag_unpermute(flat: torch.Tensor, n: int, k: int) -> torch.Tensor:
    """Inverse of frag_permute: flat fragment order -> [N, K]."""
    return flat.reshape(n // 16, k // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(n, k)


def frag_rows(m: int) -> int:
    """Rows of a fragment-ordered activation buffer holding m rows (16-row tiles)."""
    return (m + 15) // 16 * 16


def to_frag(x: torch.Tensor) -> torch.Tensor:
    """[M, K] activation -> fragment-ordered [frag_rows(M), K] buffer (csrc
    frag_index: the MFMA B-operand tiles, as the producers write them)."""
    m, k = x.shape
    pad = torch.zeros(frag_rows(m), k, dtype=x.dtype, device=x.device)
    pad[:m] = x
    return frag_permute(pad).view(frag_rows(m), k)


def from_frag(xf: torch.Tensor, m: int) -> torch.Tensor:
    """Inverse of to_frag: the first m rows, row-major."""
    return frag_unpermute(xf.reshape(-1), xf.shape[0], xf.shape[1])[:m]


MODE_RAW, MODE_PACKED, MODE_PACKED_BF11 = 0, 1, 2


def packed_mode(stream_cpu: torch.Tensor) -> int:
    """Kernel mode for a packed stream: the fast phase-pipelined path needs every
    chunk to be BF11; raw chunks (incompressible data / odd tails) take the
    generic path; BF12 chunks cannot be read by the GEMM at all."""
    kinds = bf12.chunk_kinds(stream_cpu)
    if 1 in kinds:
        raise ValueError("decode GEMM streams must be packed with fmt='bf11s' (no BF12 chunks)")
    return MODE_PACKED_BF11 if kinds <= {2} else MODE_PACKED


@dataclass(frozen=True)
class WeightRef:
    """Where a [N, K] fragment-ordered weight lives: raw bf16 at ``ptr`` + 2 * off
    (mode MODE_RAW), or value offset ``off`` inside the packed stream at ``ptr``."""
    ptr: int
    off: int
    n: int
    k: int
    mode: int = MODE_RAW
    chunk_shift: int = 20

    @property
    def packed(self) -> bool:
        return self.mode != MODE_RAW


class _Workspace:
    def __init__(self):
        self.buf: dict = {}

    def get(self, device: torch.device, nbytes: int) -> torch.Tensor:
        key = str(device)
        t = self.buf.get(key)
        if t is None or t.numel() * 4 < nbytes:
            t = torch.empty((nbytes + 3) // 4 + (1 << 20), dtype=torch.float32, device=device)
            self.buf[key] = t
        return t


_WS = _Workspace()
_PLANS: dict = {}
_FIX: dict = {}


def _fix_counters(device: torch.device, stream: int) -> torch.Tensor:
    """The zeroed arrival-counter slab of the in-kernel fixup for one stream
    (kernels on one stream never overlap; each last arrival re-zeroes its own)."""
    key = (str(device), stream)
    t = _FIX.get(key)
    if t is None:
        t = _FIX[key] = torch.zeros(FIX_SLOTS, dtype=torch.int32, device=device)
    return t


_PIPE_PLANS: dict = {}


def _launch_cfg(w: "WeightRef", lds: int | None) -> tuple:
    """(waves, unroll, lds_x, depth) of one decode GEMM launch."""
    lds = LDS_X if lds is None else int(lds)
    if lds < 0:
        lds = int(w.mode == MODE_RAW and w.n <= LDS_MAX_N)
    units = TARGET_UNITS if w.mode == MODE_RAW else TARGET_UNITS_PACKED
    unroll = UNROLL
    if lds and w.mode == MODE_RAW:
        units *= 2  # waves; the kernel runs 4 per K split
    depth = 0
    if w.mode == MODE_RAW and PIPE and not UNROLL and not lds:
        units, depth = _pipe_plan(w.n, w.k)  # unroll 1 selects the pipelined raw kernels
        unroll = 1
    return units, unroll, lds, depth


def _ksplit(w: "WeightRef", units: int, lds: int) -> int:
    raw_lds = bool(lds) and w.mode == MODE_RAW
    ks = _PLANS.get((w.n, w.k, units, raw_lds))
    if ks is None:  # the binding plans the launch with the same function: one source of truth
        ks = _PLANS[(w.n, w.k, units, raw_lds)] = lib.dgemm_plan(w.n, w.k, units, raw_lds)[0]
    return ks


def _pipe_plan(n: int, k: int) -> tuple:
    """(waves, depth code) of the pipelined raw path for an [n, k] weight."""
    key = (n, k, DEPTH, LRING_DEPTH, LRING_UNITS, LRING_MAX_STEPS, TARGET_UNITS_PIPE, TARGET_UNITS_PIPE_LARGE)
    p = _PIPE_PLANS.get(key)
    if p is None:
        pipe_units = TARGET_UNITS_PIPE_LARGE if n * k >= LARGE_ELEMS else TARGET_UNITS_PIPE
        if DEPTH >= 30:
            p = (LRING_UNITS, DEPTH)
        elif DEPTH:
            p = (pipe_units, DEPTH)
        else:
            ks, klen = lib.dgemm_plan(n, k, LRING_UNITS, False)
            p = (LRING_UNITS, LRING_DEPTH) if klen // 32 <= LRING_MAX_STEPS else (pipe_units, 4)
        _PIPE_PLANS[key] = p
    return p


@dataclass(frozen=True)
class Deferred:
    """A decode GEMM whose split-K sum and epilogue run in its consumer's launch
    (``linear(..., defer=True)``): ``part`` = f32 [ksplit][M][N] in the shared
    per-device workspace, valid until the next ``linear`` call (``gen``)."""
    part: int
    ksplit: int
    m: int
    n: int
    gen: int

    def check(self, m: int, n: int) -> None:
        if (m, n) != (self.m, self.n):
            raise ValueError(f"deferred GEMM is [{self.m}, {self.n}], consumer wants [{m}, {n}]")
        if _GEN[0] != self.gen:
            raise RuntimeError("deferred GEMM partials were overwritten by a later dgemm.linear call")


_GEN = [0]


def linear(x: torch.Tensor, w: WeightRef, epi: str = "store", resid: torch.Tensor | None = None,
           out: torch.Tensor | None = None, device_index: int = 0, lds: int | None = None,
           defer: bool = False, x_rows: int | None = None, out_frag: bool = False, out_col0: int = 0):
    """x: [M, K] bf16 (row stride % 8 == 0). Returns out [M, N] (silu_mul: [M, N/2]).
    Raw weights run the pipelined kernels (k_dgemm_lring / k_dgemm_pipe, see
    _pipe_plan; ``lds``=1: k_dgemm_lds), packed ones k_dgemm's in-register decode;
    the pipelined raw kernels sum the K splits and run the epilogue themselves
    (FIXUP: the last-arriving wave of each output group), the others leave it
    to a k_dgemm_reduce launch. ``defer``: no
    reduce launch - returns a Deferred whose consumer (fused.rms_norm's
    residual form, fused.rope_kv) sums the splits and applies the epilogue.
    ``x_rows``: x is a fragment-ordered [frag_rows(x_rows), K] buffer (to_frag)
    with x_rows valid rows. ``out_frag``: out is a fragment-ordered
    [frag_rows(M), C] buffer and this GEMM writes its columns out_col0 ..
    out_col0 + N (silu_mul: N/2)."""
    _GEN[0] += 1
    xf = x_rows is not None
    if x.dtype != torch.bfloat16 or x.dim() != 2 or x.stride(1) != 1 or x.shape[1] != w.k:
        raise ValueError("dgemm.linear: x must be a row-major bf16 [M, K] view")
    if xf and (not x.is_contiguous() or x.shape[0] != frag_rows(x_rows)):
        raise ValueError("dgemm.linear: fragment-ordered x must be a contiguous [frag_rows(M), K] buffer")
    m = x_rows if xf else x.shape[0]
    ldx = w.k if xf else x.stride(0)
    units, unroll, lds_, depth = _launch_cfg(w, lds)
    ks = _ksplit(w, units, lds_)
    part = _WS.get(x.device, ks * m * w.n * 4)
    stream = int(torch.cuda.current_stream(device_index).cuda_stream) if x.is_cuda else 0
    if defer:
        lib.dgemm(device_index, stream, w.ptr, w.off, w.mode, w.chunk_shift, x.data_ptr(), ldx, m, w.n, w.k,
                  part.data_ptr(), part.numel() * 4, 0, 0, 0, 0, 0, units, unroll, lds_, WG_WAVES, depth, False, xf)
        return Deferred(part.data_ptr(), ks, m, w.n, _GEN[0])
    nout = w.n // 2 if epi == "silu_mul" else w.n
    if out is None:
        out = torch.empty(frag_rows(m) if out_frag else m, nout, dtype=torch.bfloat16, device=x.device)
    if out_frag:
        if out.dtype != torch.bfloat16 or not out.is_contiguous() or out.shape[0] != frag_rows(m) or epi == "resid":
            raise ValueError("dgemm.linear: bad fragment-ordered out")
    elif out.dtype != torch.bfloat16 or out.stride(1) != 1 or tuple(out.shape) != (m, nout):
        raise ValueError("dgemm.linear: bad out")
    if epi == "resid":
        if resid is None or resid.shape != out.shape or resid.stride(1) != 1:
            raise ValueError("dgemm.linear: resid must match out")
    inkernel = unroll == 1 and not lds_ and w.mode == MODE_RAW
    fix = _fix_counters(x.device, stream) if FIXUP and inkernel else None
    lib.dgemm(device_index, stream, w.ptr, w.off, w.mode, w.chunk_shift, x.data_ptr(), ldx, m, w.n, w.k,
              part.data_ptr(), part.numel() * 4, EPI[epi], resid.data_ptr() if resid is not None else 0,
              resid.stride(0) if resid is not None else 0, out.data_ptr(), out.stride(0), units, unroll, lds_,
              WG_WAVES, depth, True, xf, out_frag, out.shape[1] if out_frag else 0, out_col0,
              fix.data_ptr() if fix is not None else 0, FIX_SLOTS if fix is not None else 0,
              bool(DIRECT and inkernel and epi != "silu_mul"))
    return out
