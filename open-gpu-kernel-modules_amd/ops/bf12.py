"""BF12 packed tensors: lossless ~0.75x bf16 storage for data that rests in any
tier - host, CXL *and HBM* - and is unpacked into a bf16 staging buffer right
before use.

Why: at 2x oversubscription a decode step is bound by the bytes that cross
PCIe per step. Keeping the weights packed where they rest shrinks both the
streamed bytes and the HBM each resident layer occupies, so more of the model
stays resident (the managed footprint the runtime moves is the packed one).
The unpack (csrc/kernels/bf12_kernels.hip k_bf12_unpack) runs HBM->HBM at a
few TB/s, i.e. well under a millisecond per 70B layer.

Format: codec.hpp "BFS1" stream = header + chunk table + 256-B aligned chunks,
each one of
  * BF11 (default): sign|mantissa bytes + a 2-bit primary exponent code (the
    chunk's three most frequent exponents) + a 4-bit secondary code only for the
    values that escape it, ~11 bits/value (~0.69x) for weight-like data;
  * BF12: sign|mantissa bytes + 4-bit exponent codes relative to a per-chunk
    base, 12 bits/value (0.75x);
  * ANS1 ("ans"): sign|mantissa bytes + the exponents entropy-coded with
    interleaved rANS (one wave decodes 32 Ki values; csrc/kernels/ans_kernels.hip),
    ~10.65 bits/value (~0.667x) for weight-like data;
  * raw bf16 (incompressible chunks / odd tails).
BF11/BF12 carry an exception list for exponents outside their code space and
ANS codes every exponent, so every bf16 bit pattern round-trips.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

import torch

from .._native import lib

CHUNK_VALUES = 1 << 20  # 2 MB of bf16 per chunk (32 decode tiles)
HEADER = struct.Struct("<IIIIQQ")
MAGIC = 0x31534642


@dataclass
class PackedInfo:
    n_values: int
    nbytes: int          # stream size
    nchunks: int
    chunk_values: int
    fmt: int = 0         # PackFormat the stream was packed with (4 = ANS)

    @property
    def ratio(self) -> float:
        return self.nbytes / max(1, self.n_values * 2)


def _threads() -> int:
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))


FORMATS = {"bf12": 1, "bf11": 2, "bf11s": 3, "ans": 4}  # bf11s: BF11-or-raw chunks (decode-GEMM weights)
FMT_ANS = 4


def pack(t: torch.Tensor, chunk_values: int = CHUNK_VALUES, out: torch.Tensor | None = None, fmt: str = "bf11"
         ) -> tuple[torch.Tensor, PackedInfo]:
    """Pack a bf16 tensor (any device; encoded on the host) -> (uint8 CPU stream, info).
    ``fmt``: "bf11" (per chunk the smaller of BF11 / BF12 / raw) or "bf12"."""
    if t.dtype != torch.bfloat16:
        raise TypeError("pack expects bf16")
    src = t.detach().reshape(-1).contiguous().cpu()
    n = src.numel()
    bound = lib.bf12_pack_bound(n, chunk_values)
    if out is None or out.numel() < bound:
        out = torch.empty(bound, dtype=torch.uint8)
    total = lib.bf12_pack(src.data_ptr(), n, out.data_ptr(), bound, chunk_values, _threads(), FORMATS[fmt])
    return out[:total], info_of(out[:64])


def info_of(stream_head: torch.Tensor) -> PackedInfo:
    """Parse a stream header (the first 32 bytes, CPU tensor or bytes)."""
    raw = bytes(stream_head[:HEADER.size].cpu().numpy()) if isinstance(stream_head, torch.Tensor) else stream_head
    magic, nch, cv, fmt, n, nbytes = HEADER.unpack(raw[:HEADER.size])
    if magic != MAGIC:
        raise ValueError("not a BF12 stream")
    return PackedInfo(n, nbytes, nch, cv, fmt)


def unpack_host(stream: torch.Tensor, info: PackedInfo) -> torch.Tensor:
    """CPU reference unpack -> bf16 tensor of info.n_values."""
    out = torch.empty(info.n_values, dtype=torch.bfloat16)
    s = stream.contiguous()
    lib.bf12_unpack_host(s.data_ptr(), out.data_ptr(), info.n_values)
    return out


def unpack_into(dst: torch.Tensor, src_ptr: int, info: PackedInfo, device: int = 0, stream: int | None = None,
                workgroups: int = 0, dst_stride: int = 0, row_chunks: int = 1) -> torch.Tensor:
    """Unpack the stream at device address ``src_ptr`` into ``dst`` (bf16) on
    ``stream`` (default: the current torch stream of ``device``). ``dst_stride``:
    rows of ``row_chunks`` consecutive chunks (a power of two) land at element
    row * dst_stride (0 = contiguous), e.g. KV row blocks into a cache with room
    for more tokens per row - a row longer than the largest chunk (1 Mi values)
    is several chunks."""
    if row_chunks < 1 or row_chunks & (row_chunks - 1):
        raise ValueError("row_chunks must be a power of two")
    row = row_chunks * info.chunk_values
    rows = -(-info.nchunks // row_chunks)
    need = info.n_values if not dst_stride else (rows - 1) * dst_stride + (info.n_values - (rows - 1) * row)
    if dst_stride and dst_stride < row:
        raise ValueError("dst_stride must be >= row_chunks * chunk_values")
    if dst.dtype != torch.bfloat16 or dst.numel() < need:
        raise ValueError("dst must be bf16 with room for the unpacked chunks")
    if stream is None:
        stream = int(torch.cuda.current_stream(device).cuda_stream) if dst.is_cuda else 0
    fn = lib.ans_unpack if info.fmt == FMT_ANS else lib.bf12_unpack
    fn(device, src_ptr, dst.data_ptr(), info.nchunks, info.chunk_values, info.n_values, stream, workgroups, dst_stride,
       row_chunks.bit_length() - 1)
    return dst


def chunk_kinds(stream: torch.Tensor) -> set:
    """Chunk encodings present in a (CPU) stream: 0 raw, 1 BF12, 2 BF11, 3 ANS1."""
    info = info_of(stream[:64])
    table = stream[32:32 + 16 * info.nchunks].view(torch.int32).view(-1, 4)
    return set(int(k) for k in table[:, 3].unique().tolist())
