"""Decode GEMM: ``out = epilogue(x @ W^T)`` for decode batches on the MFMA cores,
reading W straight from the format it rests in (csrc/kernels/decode_gemm.hip).

W is stored in *fragment order* (16 x 32 tiles, 1 KB each, lane-major = the
A-operand fragment of v_mfma_f32_16x16x32_bf16), either as raw bf16 or inside a
BF11 packed stream (ops/bf12.py, "bf11s": BF11-or-raw chunks) that the kernel
decodes in registers - the packed bytes are the only weight bytes read from HBM
and no bf16 staging copy exists. Epilogues are fused into the split-K reduce:
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


def linear(x: torch.Tensor, w: WeightRef, epi: str = "store", resid: torch.Tensor | None = None,
           out: torch.Tensor | None = None, device_index: int = 0, lds: int | None = None) -> torch.Tensor:
    """x: [M, K] bf16 (row stride % 8 == 0). Returns out [M, N] (silu_mul: [M, N/2]).
    Raw weights run k_dgemm_pipe (``lds``=1: k_dgemm_lds), packed ones k_dgemm's
    in-register decode; k_dgemm_reduce sums the K splits and runs the epilogue."""
    if x.dtype != torch.bfloat16 or x.dim() != 2 or x.stride(1) != 1 or x.shape[1] != w.k:
        raise ValueError("dgemm.linear: x must be a row-major bf16 [M, K] view")
    m = x.shape[0]
    nout = w.n // 2 if epi == "silu_mul" else w.n
    if out is None:
        out = torch.empty(m, nout, dtype=torch.bfloat16, device=x.device)
    if out.dtype != torch.bfloat16 or out.stride(1) != 1 or tuple(out.shape) != (m, nout):
        raise ValueError("dgemm.linear: bad out")
    if epi == "resid":
        if resid is None or resid.shape != out.shape or resid.stride(1) != 1:
            raise ValueError("dgemm.linear: resid must match out")
    stream = int(torch.cuda.current_stream(device_index).cuda_stream) if x.is_cuda else 0
    lds = LDS_X if lds is None else int(lds)
    if lds < 0:
        lds = int(w.mode == MODE_RAW and w.n <= LDS_MAX_N)
    units = TARGET_UNITS if w.mode == MODE_RAW else TARGET_UNITS_PACKED
    unroll = UNROLL
    if lds and w.mode == MODE_RAW:
        units *= 2  # waves; the kernel runs 4 per K split
    elif w.mode == MODE_RAW and PIPE and not UNROLL:
        # unroll 1 selects k_dgemm_pipe; the largest matrices take more splits
        units = TARGET_UNITS_PIPE_LARGE if w.n * w.k >= LARGE_ELEMS else TARGET_UNITS_PIPE
        unroll = 1
    raw_lds = bool(lds) and w.mode == MODE_RAW
    ks = _PLANS.get((w.n, w.k, units, raw_lds))
    if ks is None:  # the binding plans the launch with the same function: one source of truth
        ks = _PLANS[(w.n, w.k, units, raw_lds)] = lib.dgemm_plan(w.n, w.k, units, raw_lds)[0]
    part = _WS.get(x.device, ks * m * w.n * 4)
    lib.dgemm(device_index, stream, w.ptr, w.off, w.mode, w.chunk_shift, x.data_ptr(), x.stride(0), m, w.n, w.k,
              part.data_ptr(), part.numel() * 4, EPI[epi], resid.data_ptr() if resid is not None else 0,
              resid.stride(0) if resid is not None else 0, out.data_ptr(), out.stride(0), units, unroll, lds, WG_WAVES)
    return out
