// Launchers for the hand-written CDNA4 (gfx950) kernels of the migration data
// plane (csrc/kernels/copy_kernels.hip). Each kernel replaces a Copy-Engine
// method the reference encodes into pushbuffers:
//   k_batch_copy      <- ce_hal->memcopy / memcopy_v_to_v  (uvm_volta_ce.c:119-181)
//   k_gather_pages    <- staged pack of scattered pages     (uvm_va_block.c:3673-3860)
//   k_scatter_pages   <- staged unpack
//   k_memset32        <- ce_hal->memset_4                   (uvm_volta_ce.c:259-300)
//   k_signal          <- semaphore_release                  (uvm_hal.h:789-792)
//   k_managed_gather  <- replayable-fault producer + access counters (device side)
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ogkm/dgemm.hpp"
#include "ogkm/fault_abi.hpp"

namespace ogkm {

struct KCopyDesc {      // device-side copy descriptor (24 B)
  uint64_t dst;
  uint64_t src;
  uint64_t bytes;
};

constexpr int kInlineDescs = 32;
struct KInlineDescs {   // passed by value as a kernel argument for small batches
  KCopyDesc d[kInlineDescs];
  uint64_t piece_start[kInlineDescs + 1];
};

// Copies n descriptors. `d_descs`/`d_piece_start` are device pointers (large
// batches) or null with `inl` used. piece_bytes must be a multiple of 4096.
hipError_t launch_batch_copy(const KCopyDesc* d_descs, const uint64_t* d_piece_start, const KInlineDescs* inl,
                             uint32_t n, uint64_t total_pieces, uint32_t piece_bytes, uint32_t workgroups,
                             hipStream_t s, bool nt_loads = true);
// k_peer_push: source-GPU push of up to kInlineDescs copies (typically into a
// peer's HBM over xGMI) with a bounded grid of `workgroups`.
hipError_t launch_peer_push(const KInlineDescs& inl, uint32_t n, uint64_t total_pieces, uint32_t piece_bytes,
                            uint32_t workgroups, hipStream_t s);
hipError_t launch_gather_pages(uint64_t base, uint64_t contig, const uint32_t* d_idx, uint32_t npages,
                               uint32_t page_bytes, bool scatter, uint32_t workgroups, hipStream_t s);
hipError_t launch_memset32(uint64_t dst, uint32_t pattern, uint64_t bytes, hipStream_t s);
// Page-list copy of one 2 MB block's scattered 4 KiB pages, staged through LDS
// with global_load_lds (16 pages = 64 KiB in flight per workgroup).
struct KPageList {
  uint16_t idx[512];
};
hipError_t launch_page_copy(uint64_t dst_base, uint64_t src_base, const KPageList& pl, uint32_t npages,
                            uint32_t workgroups, hipStream_t s);
hipError_t launch_signal(uint64_t* host_addr, uint64_t value, hipStream_t s);
hipError_t launch_acquire(hipStream_t s);  // system-scope cache acquire on every XCD (k_acquire)

// Fused copy + BF12 decode of up to kInlineDescs encoded blocks (codec.hpp).
struct KBf12Desc {
  uint64_t src;        // encoded block (pinned host / CXL)
  uint64_t dst;        // bf16 output (HBM)
  uint32_t n_values;
  uint32_t pad;
};
struct KBf12Descs {
  KBf12Desc d[kInlineDescs];
  uint64_t item_start[kInlineDescs + 1];  // prefix sum of 32768-value tiles
};
hipError_t launch_bf12_decode(const KBf12Descs& inl, uint32_t n, uint32_t workgroups, hipStream_t s);
// Unpack a whole BF12 stream (codec.hpp) that lives in device memory into bf16
// at `dst` (chunk c at dst + c * dst_stride values; 0 = contiguous): one
// launch, one work item per 32768-value tile of every chunk.
// Destination of chunk c: (c >> row_shift) * dst_stride + (c & (2^row_shift - 1)) * chunk_values
// (row_shift 0: c * dst_stride) - a row of 2^row_shift chunks, e.g. a KV row block
// longer than the largest chunk, lands contiguously in a strided cache row.
hipError_t launch_bf12_unpack(const void* stream, void* dst, uint32_t nchunks, uint32_t chunk_values,
                              uint32_t workgroups, hipStream_t s, uint64_t dst_stride = 0, uint32_t row_shift = 0);
// Unpack an ANS stream (ANS1 or raw chunks, codec.hpp) in device memory into
// bf16 (csrc/kernels/ans_kernels.hip): one wave per 32 Ki-value rANS segment.
// err: optional host-coherent {count, stream, chunk, freq sum} record of corrupt chunks.
hipError_t launch_ans_unpack(const void* stream, void* dst, uint32_t nchunks, uint32_t chunk_values,
                             uint32_t workgroups, hipStream_t s, uint64_t dst_stride = 0, uint64_t* err = nullptr,
                             uint32_t row_shift = 0);
// Decode a batch of single-chunk ANS1 blocks (the runtime's packed host copies,
// staged in HBM by the migration ring): block i at src[i] -> n_values[i] bf16
// at dst[i]. One launch, one work item per 4 segments of every block.
constexpr int kAnsInlineBlocks = 64;
struct KAnsBlocks {
  uint64_t src[kAnsInlineBlocks];
  uint64_t dst[kAnsInlineBlocks];
  uint32_t n_values[kAnsInlineBlocks];
  uint32_t item_start[kAnsInlineBlocks + 1];
};
hipError_t launch_ans_blocks(const KAnsBlocks& b, uint32_t n, hipStream_t s, uint64_t* err = nullptr);
// Single-segment ANS1 chunks (32 Ki values each: segmented packed host copies),
// one wave per chunk.
constexpr int kAnsInlineSegs = 128;
struct KAnsSegs {
  uint64_t src[kAnsInlineSegs];
  uint64_t dst[kAnsInlineSegs];
};
hipError_t launch_ans_segs(const KAnsSegs& d, uint32_t n, hipStream_t s, uint64_t* err = nullptr);

// Decode GEMM (csrc/kernels/decode_gemm.hip); argument structs in ogkm/dgemm.hpp.
hipError_t launch_dgemm(const DGemmArgs& a, int mode, hipStream_t s);
hipError_t launch_dgemm_reduce(const DGemmReduceArgs& a, hipStream_t s);
// Fused decode-step ops (csrc/kernels/decode_ops.hip).
hipError_t launch_rmsnorm(const ResidNormArgs& a, hipStream_t s);
hipError_t launch_rope_kv(const RopeKvArgs& a, hipStream_t s);
hipError_t launch_attn_decode(AttnArgs a, hipStream_t s);

// Device fault buffer (GET/PUT ring, ogkm/fault_abi.hpp) as kernels see it.
struct KFaultBuf {
  FaultBufHeader* hdr;
  DeviceFaultRecord* recs;
  uint32_t entries;   // power of two
};

// Gather `nrows` rows (row_bytes each) of a managed table through its device
// residency table; misses read zero and are recorded as faults, remote hits are
// recorded as access-counter notifications.
hipError_t launch_managed_gather(const uint64_t* table, uint64_t range_id, const int64_t* rows, uint32_t nrows,
                                 uint32_t row_bytes, void* out, KFaultBuf fb, uint32_t proc, hipStream_t s);

// Fault gate (replayable-fault stall + replay): one wave checks blocks
// [b0, b0 + nblocks) of a range in its device residency table; every block not
// resident in HBM is recorded as a fault and the wave waits for the host's
// replay token (re-recording every ~1 ms), then re-checks. Work queued behind
// the gate on the stream runs once every block is resident. status[0]:
// kGateResolved, kGateTimeout (gave up after `timeout_us`; the kernel always
// exits) or kGateCancelled (the host cancelled this channel's faults: precise
// cancel, fault_abi.hpp); status[1] = number of replays the gate waited for.
hipError_t launch_fault_gate(const uint64_t* table, uint64_t range_id, uint32_t b0, uint32_t nblocks, KFaultBuf fb,
                             uint32_t proc, uint32_t access, uint32_t timeout_us, uint32_t* status, hipStream_t s);

// Table-indirect fetch: copy [off, off + bytes) of a range into `out`, block by
// block through the device residency table (HBM entry, else the remote entry).
// Meant to run behind a fault gate on a registered table stream.
hipError_t launch_table_fetch(const uint64_t* table, uint64_t off, uint64_t bytes, void* out, uint32_t workgroups,
                              hipStream_t s);

// Fault-buffer stress producer (tests): `waves` x 64 lanes append
// `per_lane` records each, retrying while the ring is full (bounded).
hipError_t launch_fault_stress(KFaultBuf fb, uint32_t waves, uint32_t per_lane, uint32_t* gave_up, hipStream_t s);

}  // namespace ogkm
