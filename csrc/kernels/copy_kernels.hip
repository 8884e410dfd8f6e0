// Migration data-plane kernels for MI355X (gfx950, CDNA4).
//
// Design notes (measured on the box, profiles/probe_gpu_r1.txt):
//  * PCIe Gen5 x16 H2D saturates at ~57.4 GB/s with as few as 64 workgroups of
//    256 threads issuing 16-B non-temporal loads; more workgroups only add
//    contention. Copies therefore run with a small CU budget
//    (config copy_workgroups, default 64 = 1/4 of the CUs, one WG each) and leave
//    the rest of the chip to the model.
//  * Work is split into fixed-size pieces (default 64 KB = one 16-B load per
//    lane x 16) over a batch of descriptors; a workgroup walks pieces
//    grid-stride so a batch of thousands of 2 MB block copies is ONE launch
//    (vs one CE LAUNCH_DMA per contiguous run in the reference,
//    uvm_va_block.c:4278-4326). Each wave keeps 4 dwordx4 loads in flight
//    before storing (HBM/PCIe latency hiding without LDS).
//  * PCIe-bound ring copies default to the SDMA engines (config copy_engine=3,
//    driven from the ring's worker thread, backend_hip.cpp): this kernel reading
//    host memory slows concurrent HBM-bound kernels 3-7x (2.5x less with plain
//    instead of non-temporal loads, copy_nt_loads=0; measured,
//    profiles/r1_copy_engine_interference.md), SDMA 1.06x. These kernels serve
//    HBM<->HBM copies, page gather/scatter, the fused copy+decode path,
//    k_peer_push (GPU->GPU, peer_copy_engine=0) and copy_engine=0.
//  * Small batches pass their descriptors by value in the kernarg segment
//    (scalar loads, no extra upload); big batches read them from device memory.
#include <hip/hip_runtime.h>

#include "ogkm/kernels.hpp"

namespace ogkm {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kUnroll = 4;

// Copy `len` bytes with 256 threads. Fast path: 16-B aligned src/dst.
// NT_LOAD: non-temporal source loads (config copy_nt_loads); stores are always
// non-temporal.
template <bool NT_LOAD = true>
__device__ __forceinline__ void copy_span(uint64_t dst, uint64_t src, uint64_t len) {
  const int t = threadIdx.x;
  if (((dst | src) & 15) == 0) {
    const u32x4* __restrict__ s = reinterpret_cast<const u32x4*>(src);
    u32x4* __restrict__ d = reinterpret_cast<u32x4*>(dst);
    uint64_t n16 = len >> 4;
    uint64_t i = t;
    for (; i + (kUnroll - 1) * kThreads < n16; i += kUnroll * kThreads) {
      u32x4 v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) v[u] = NT_LOAD ? __builtin_nontemporal_load(s + i + u * kThreads) : s[i + u * kThreads];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) __builtin_nontemporal_store(v[u], d + i + u * kThreads);
    }
    for (; i < n16; i += kThreads) __builtin_nontemporal_store(NT_LOAD ? __builtin_nontemporal_load(s + i) : s[i], d + i);
    uint64_t tail = n16 << 4;
    for (uint64_t b = tail + t; b < len; b += kThreads)
      reinterpret_cast<uint8_t*>(dst)[b] = reinterpret_cast<const uint8_t*>(src)[b];
  } else if (((dst | src) & 3) == 0) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    uint64_t n4 = len >> 2;
    for (uint64_t i = t; i < n4; i += kThreads) d[i] = s[i];
    for (uint64_t b = (n4 << 2) + t; b < len; b += kThreads)
      reinterpret_cast<uint8_t*>(dst)[b] = reinterpret_cast<const uint8_t*>(src)[b];
  } else {
    for (uint64_t b = t; b < len; b += kThreads)
      reinterpret_cast<uint8_t*>(dst)[b] = reinterpret_cast<const uint8_t*>(src)[b];
  }
}

template <bool INLINE, bool NT_LOAD>
__global__ void __launch_bounds__(kThreads)
    k_batch_copy(const KCopyDesc* __restrict__ descs, const uint64_t* __restrict__ piece_start, KInlineDescs inl,
                 uint32_t n, uint64_t total_pieces, uint32_t piece_bytes) {
  __shared__ uint32_t s_desc;
  uint32_t hint = 0;
  for (uint64_t p = blockIdx.x; p < total_pieces; p += gridDim.x) {
    if (threadIdx.x == 0) {
      // Pieces are visited in increasing order: advance from the last hit,
      // fall back to binary search on a big jump.
      const uint64_t* ps = INLINE ? inl.piece_start : piece_start;
      uint32_t i = hint;
      if (!(ps[i] <= p && p < ps[i + 1])) {
        uint32_t lo = 0, hi = n;
        while (hi - lo > 1) {
          uint32_t mid = (lo + hi) >> 1;
          if (ps[mid] <= p) lo = mid;
          else hi = mid;
        }
        i = lo;
      }
      s_desc = i;
    }
    __syncthreads();
    uint32_t i = s_desc;
    hint = i;
    KCopyDesc d = INLINE ? inl.d[i] : descs[i];
    uint64_t ps_i = INLINE ? inl.piece_start[i] : piece_start[i];
    uint64_t off = (p - ps_i) * (uint64_t)piece_bytes;
    uint64_t len = d.bytes - off;
    if (len > piece_bytes) len = piece_bytes;
    copy_span<NT_LOAD>(d.dst + off, d.src + off, len);
    __syncthreads();
  }
}

hipError_t launch_batch_copy(const KCopyDesc* d_descs, const uint64_t* d_piece_start, const KInlineDescs* inl,
                             uint32_t n, uint64_t total_pieces, uint32_t piece_bytes, uint32_t workgroups,
                             hipStream_t s, bool nt_loads) {
  if (n == 0 || total_pieces == 0) return hipSuccess;
  uint32_t grid = (uint32_t)(total_pieces < workgroups ? total_pieces : workgroups);
  if (grid == 0) grid = 1;
  KInlineDescs dummy;
  const KInlineDescs& d = inl ? *inl : dummy;
  if (inl && nt_loads)
    hipLaunchKernelGGL((k_batch_copy<true, true>), dim3(grid), dim3(kThreads), 0, s, nullptr, nullptr, d, n,
                       total_pieces, piece_bytes);
  else if (inl)
    hipLaunchKernelGGL((k_batch_copy<true, false>), dim3(grid), dim3(kThreads), 0, s, nullptr, nullptr, d, n,
                       total_pieces, piece_bytes);
  else if (nt_loads)
    hipLaunchKernelGGL((k_batch_copy<false, true>), dim3(grid), dim3(kThreads), 0, s, d_descs, d_piece_start, d,
                       n, total_pieces, piece_bytes);
  else
    hipLaunchKernelGGL((k_batch_copy<false, false>), dim3(grid), dim3(kThreads), 0, s, d_descs, d_piece_start, d,
                       n, total_pieces, piece_bytes);
  return hipGetLastError();
}

// k_peer_push: the SOURCE GPU pushes its HBM into a peer's HBM over xGMI (the
// reference pushes peer copies from the source GPU's channel,
// uvm_va_block.c:3390-3460). A bounded grid (config peer_push_wgs = the CU
// budget taken from compute); each workgroup streams whole 64 KB pieces with 8
// 16-B loads in flight per lane (non-temporal: read once locally, written once
// remotely), so the remote-write latency of the link is covered.
__global__ void __launch_bounds__(kThreads)
    k_peer_push(KInlineDescs inl, uint32_t n, uint64_t total_pieces, uint32_t piece_bytes) {
  constexpr int kU = 8;
  uint32_t i = 0;
  for (uint64_t p = blockIdx.x; p < total_pieces; p += gridDim.x) {
    while (i + 1 < n && inl.piece_start[i + 1] <= p) ++i;  // pieces visited in increasing order
    const KCopyDesc d = inl.d[i];
    const uint64_t off = (p - inl.piece_start[i]) * (uint64_t)piece_bytes;
    uint64_t len = d.bytes - off;
    if (len > piece_bytes) len = piece_bytes;
    const uint64_t dst = d.dst + off, src = d.src + off;
    if (((dst | src | len) & 15) == 0) {
      const u32x4* s16 = reinterpret_cast<const u32x4*>(src);
      u32x4* d16 = reinterpret_cast<u32x4*>(dst);
      const uint64_t n16 = len >> 4;
      uint64_t j = threadIdx.x;
      for (; j + (kU - 1) * kThreads < n16; j += kU * kThreads) {
        u32x4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) v[u] = __builtin_nontemporal_load(s16 + j + u * kThreads);
#pragma unroll
        for (int u = 0; u < kU; ++u) __builtin_nontemporal_store(v[u], d16 + j + u * kThreads);
      }
      for (; j < n16; j += kThreads) __builtin_nontemporal_store(__builtin_nontemporal_load(s16 + j), d16 + j);
    } else {
      copy_span(dst, src, len);
    }
  }
}

hipError_t launch_peer_push(const KInlineDescs& inl, uint32_t n, uint64_t total_pieces, uint32_t piece_bytes,
                            uint32_t workgroups, hipStream_t s) {
  if (n == 0 || total_pieces == 0) return hipSuccess;
  if (n > (uint32_t)kInlineDescs || piece_bytes % 4096 || inl.piece_start[n] != total_pieces) return hipErrorInvalidValue;
  uint32_t grid = (uint32_t)(total_pieces < workgroups ? total_pieces : workgroups);
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(k_peer_push, dim3(grid), dim3(kThreads), 0, s, inl, n, total_pieces, piece_bytes);
  return hipGetLastError();
}

// Pack (gather) / unpack (scatter) of a page list: page i <-> base + idx[i]*page_bytes.
__global__ void __launch_bounds__(kThreads)
    k_gather_pages(uint64_t base, uint64_t contig, const uint32_t* __restrict__ idx, uint32_t npages,
                   uint32_t page_bytes, int scatter) {
  for (uint32_t p = blockIdx.x; p < npages; p += gridDim.x) {
    uint64_t sparse = base + (uint64_t)idx[p] * page_bytes;
    uint64_t packed = contig + (uint64_t)p * page_bytes;
    if (scatter) copy_span(sparse, packed, page_bytes);
    else copy_span(packed, sparse, page_bytes);
  }
}

hipError_t launch_gather_pages(uint64_t base, uint64_t contig, const uint32_t* d_idx, uint32_t npages,
                               uint32_t page_bytes, bool scatter, uint32_t workgroups, hipStream_t s) {
  if (npages == 0) return hipSuccess;
  uint32_t grid = npages < workgroups ? npages : workgroups;
  hipLaunchKernelGGL(k_gather_pages, dim3(grid), dim3(kThreads), 0, s, base, contig, d_idx, npages, page_bytes,
                     scatter ? 1 : 0);
  return hipGetLastError();
}

// Scattered pages of one block: every workgroup stages up to kStagePages pages
// (4 KiB = 256 lanes x 16 B each) global -> LDS with global_load_lds (no VGPR
// round trip, all of them in flight at once - what hides the PCIe latency of a
// host-resident source), then writes them out with non-temporal 16-B stores.
// The LDS image is lane-linear per wave (each wave-instruction fills 1 KiB).
constexpr uint32_t kStagePages = 16;  // 64 KiB of the 160 KiB LDS

__global__ void __launch_bounds__(kThreads)
    k_page_copy_lds(uint64_t dst_base, uint64_t src_base, KPageList pl, uint32_t npages) {
  __shared__ u32x4 stage[kStagePages * kThreads];
  const uint32_t t = threadIdx.x, wave = t >> 6;
  for (uint32_t first = blockIdx.x * kStagePages; first < npages; first += gridDim.x * kStagePages) {
    const uint32_t n = npages - first < kStagePages ? npages - first : kStagePages;
    for (uint32_t j = 0; j < n; ++j) {
      const u32x4* src = reinterpret_cast<const u32x4*>(src_base + ((uint64_t)pl.idx[first + j] << 12)) + t;
      __builtin_amdgcn_global_load_lds(src, &stage[j * kThreads + wave * 64], 16, 0, 0);
    }
    __syncthreads();  // vmcnt(0): every staged page has landed in LDS
    for (uint32_t j = 0; j < n; ++j) {
      u32x4* dst = reinterpret_cast<u32x4*>(dst_base + ((uint64_t)pl.idx[first + j] << 12)) + t;
      __builtin_nontemporal_store(stage[j * kThreads + t], dst);
    }
    __syncthreads();  // the stage is rewritten by the next round
  }
}

hipError_t launch_page_copy(uint64_t dst_base, uint64_t src_base, const KPageList& pl, uint32_t npages,
                            uint32_t workgroups, hipStream_t s) {
  if (npages == 0) return hipSuccess;
  if (npages > 512 || ((dst_base | src_base) & 4095)) return hipErrorInvalidValue;
  uint32_t grid = (npages + kStagePages - 1) / kStagePages;
  if (grid > workgroups) grid = workgroups;
  hipLaunchKernelGGL(k_page_copy_lds, dim3(grid), dim3(kThreads), 0, s, dst_base, src_base, pl, npages);
  return hipGetLastError();
}

__global__ void __launch_bounds__(kThreads) k_memset32(uint32_t* __restrict__ dst, uint32_t pattern, uint64_t n4) {
  u32x4 v = {pattern, pattern, pattern, pattern};
  uint64_t n16 = n4 >> 2;
  u32x4* d = reinterpret_cast<u32x4*>(dst);
  for (uint64_t i = blockIdx.x * (uint64_t)kThreads + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * kThreads)
    __builtin_nontemporal_store(v, d + i);
  for (uint64_t i = (n16 << 2) + blockIdx.x * (uint64_t)kThreads + threadIdx.x; i < n4;
       i += (uint64_t)gridDim.x * kThreads)
    dst[i] = pattern;
}

hipError_t launch_memset32(uint64_t dst, uint32_t pattern, uint64_t bytes, hipStream_t s) {
  uint64_t n4 = bytes >> 2;
  if (n4 == 0) return hipSuccess;
  uint64_t grid = (n4 / 4 + kThreads - 1) / kThreads;
  if (grid > 2048) grid = 2048;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(k_memset32, dim3((uint32_t)grid), dim3(kThreads), 0, s, reinterpret_cast<uint32_t*>(dst),
                     pattern, n4);
  return hipGetLastError();
}

// Tracking-semaphore release: all prior work on the stream has completed when
// this kernel runs; publish the value with system scope so the host sees it.
__global__ void k_signal(uint64_t* addr, uint64_t value) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(addr, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t launch_signal(uint64_t* host_addr, uint64_t value, hipStream_t s) {
  hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, s, host_addr, value);
  return hipGetLastError();
}

// Consumer-side acquire after a GPU-side wait on a ring's tracking value: the
// data the ring delivered (SDMA copies, decodes on the ring's own stream) must
// not be read through a line an XCD's L2 still holds from the chunk's previous
// contents. Every workgroup runs a system-scope acquire (vector cache
// invalidate of its CU and its XCD's L2); 256 workgroups cover every XCD
// (workgroups go round-robin over the 8 XCDs) and every CU.
__global__ void __launch_bounds__(64) k_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

hipError_t launch_acquire(hipStream_t s) {
  hipLaunchKernelGGL(k_acquire, dim3(256), dim3(64), 0, s);
  return hipGetLastError();
}

// ---------------------------------------------------------------- fault buffer
// Producer side of the GET/PUT fault ring (ogkm/fault_abi.hpp): drop on a
// full ring at first look (may_drop), else reserve a slot with one atomic add
// on PUT, wait (bounded, ~1 s) for the host to consume the slot's previous lap,
// fill the record and publish it by storing seq = slot + 1 with release
// semantics at system scope. All stores are vector stores.
__device__ bool fb_append(KFaultBuf fb, uint64_t range_id, uint32_t block, uint32_t page, uint32_t access,
                          uint32_t kind, uint32_t proc, bool may_drop = true) {
  FaultBufHeader* h = fb.hdr;
  if (may_drop && __hip_atomic_load(&h->put, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                          __hip_atomic_load(&h->get, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >=
                      fb.entries) {
    __hip_atomic_fetch_add(&h->overflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return false;
  }
  const uint32_t p = __hip_atomic_fetch_add(&h->put, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock64();
  while (p - __hip_atomic_load(&h->get, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >= fb.entries) {
    if (wall_clock64() - t0 > 100000000ull) {  // 1 s: overwrite, the older record counts as lost
      __hip_atomic_fetch_add(&h->overflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  DeviceFaultRecord* r = fb.recs + (p & (fb.entries - 1));
  r->range_id = range_id;
  r->block = block;
  r->page = (uint16_t)page;
  r->access = (uint8_t)access;
  r->kind = (uint8_t)kind;
  r->proc = proc;
  __hip_atomic_store(&r->seq, p + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  return true;
}

// Device-side residency check + gather. table[2*b] = HBM address of block b (0 if
// not resident on this GPU), table[2*b+1] = remote (host/CXL) address. One
// workgroup per row; lane 0 resolves the source and records misses / remote
// accesses into the fault buffer (software replayable-fault + access-counter
// producer).
__global__ void __launch_bounds__(kThreads)
    k_managed_gather(const uint64_t* __restrict__ table, uint64_t range_id, const int64_t* __restrict__ rows,
                     uint32_t nrows, uint32_t row_bytes, uint8_t* __restrict__ out, KFaultBuf fb, uint32_t proc) {
  __shared__ uint64_t s_src;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    if (threadIdx.x == 0) {
      uint64_t off = (uint64_t)rows[r] * row_bytes;
      uint64_t b = off >> 21;
      uint64_t in_blk = off & ((1ull << 21) - 1);
      uint64_t hbm = __hip_atomic_load(table + 2 * b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      uint64_t rem = __hip_atomic_load(table + 2 * b + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      uint64_t src = hbm ? hbm + in_blk : (rem ? rem + in_blk : 0);
      if (!hbm && fb.hdr) fb_append(fb, range_id, (uint32_t)b, (uint32_t)(in_blk >> 12), 1, rem ? 1 : 0, proc);
      s_src = src;
    }
    __syncthreads();
    uint64_t src = s_src;
    uint64_t dst = reinterpret_cast<uint64_t>(out) + (uint64_t)r * row_bytes;
    if (src) {
      copy_span(dst, src, row_bytes);
    } else {
      for (uint32_t b = threadIdx.x * 4; b < row_bytes; b += kThreads * 4)
        *reinterpret_cast<uint32_t*>(dst + b) = 0;
    }
    __syncthreads();
  }
}

hipError_t launch_managed_gather(const uint64_t* table, uint64_t range_id, const int64_t* rows, uint32_t nrows,
                                 uint32_t row_bytes, void* out, KFaultBuf fb, uint32_t proc, hipStream_t s) {
  if (nrows == 0) return hipSuccess;
  uint32_t grid = nrows < 1024 ? nrows : 1024;
  hipLaunchKernelGGL(k_managed_gather, dim3(grid), dim3(kThreads), 0, s, table, range_id, rows, nrows, row_bytes,
                     reinterpret_cast<uint8_t*>(out), fb, proc);
  return hipGetLastError();
}

// One wave. The wall clock (100 MHz constant counter) bounds every wait, so
// the kernel exits even if the host never services the faults.
__global__ void __launch_bounds__(64)
    k_fault_gate(const uint64_t* __restrict__ table, uint64_t range_id, uint32_t b0, uint32_t nblocks, KFaultBuf fb,
                 uint32_t proc, uint32_t access, uint64_t timeout_ticks, uint32_t* status) {
  const uint32_t lane = threadIdx.x;
  const uint64_t t0 = wall_clock64();
  uint32_t replays = 0;
  // Precise cancel: the host bumps this channel's word before the replay token
  // when it gives up on the channel's faults (fault_abi.hpp).
  uint32_t* cancel_word = fb.hdr->cancel + ((proc >> 16) % kFaultCancelSlots);
  const uint32_t cancel0 = __hip_atomic_load(cancel_word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    const uint64_t token = __hip_atomic_load(&fb.hdr->replay, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (__hip_atomic_load(cancel_word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != cancel0) {
      if (lane == 0) {
        status[0] = kGateCancelled;
        status[1] = replays;
      }
      return;
    }
    int miss = 0;
    for (uint32_t b = b0 + lane; b < b0 + nblocks; b += 64) {
      uint64_t hbm = __hip_atomic_load(table + 2 * (uint64_t)b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (!hbm) {
        miss = 1;
        fb_append(fb, range_id, b, kFaultWholeBlock, access, 0, proc);
      }
    }
    if (!__any(miss)) {
      if (lane == 0) {
        status[0] = kGateResolved;
        status[1] = replays;
      }
      return;
    }
    // Stall until the host replays (or ~1 ms passes: re-record, a record may
    // have been dropped on a full ring), bounded by the timeout.
    const uint64_t t_rec = wall_clock64();
    for (;;) {
      __builtin_amdgcn_s_sleep(32);
      uint64_t now = wall_clock64();
      if (now - t0 > timeout_ticks) {
        if (lane == 0) {
          status[0] = kGateTimeout;
          status[1] = replays;
        }
        return;
      }
      if (__hip_atomic_load(&fb.hdr->replay, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != token) {
        ++replays;
        break;
      }
      if (now - t_rec > 100000) break;  // 1 ms at 100 MHz
    }
  }
}

hipError_t launch_fault_gate(const uint64_t* table, uint64_t range_id, uint32_t b0, uint32_t nblocks, KFaultBuf fb,
                             uint32_t proc, uint32_t access, uint32_t timeout_us, uint32_t* status, hipStream_t s) {
  if (!fb.hdr || !table || !status) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fault_gate, dim3(1), dim3(64), 0, s, table, range_id, b0, nblocks, fb, proc, access,
                     (uint64_t)timeout_us * 100, status);
  return hipGetLastError();
}

// Table-indirect copy: work item = (block, 64 KB piece); source resolved per
// block from the residency table at run time.
__global__ void __launch_bounds__(kThreads)
    k_table_fetch(const uint64_t* __restrict__ table, uint64_t off, uint64_t bytes, uint8_t* __restrict__ out) {
  constexpr uint64_t kPiece = 64 << 10;
  const uint64_t npieces = (bytes + kPiece - 1) / kPiece;
  for (uint64_t p = blockIdx.x; p < npieces; p += gridDim.x) {
    uint64_t o = off + p * kPiece;
    uint64_t len = bytes - p * kPiece < kPiece ? bytes - p * kPiece : kPiece;
    // a piece never crosses a block when off is 64 KB aligned; split otherwise
    while (len) {
      uint64_t b = o >> 21, in_blk = o & ((1ull << 21) - 1);
      uint64_t n = (1ull << 21) - in_blk < len ? (1ull << 21) - in_blk : len;
      uint64_t hbm = __hip_atomic_load(table + 2 * b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      uint64_t base = hbm ? hbm : __hip_atomic_load(table + 2 * b + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      uint64_t dst = reinterpret_cast<uint64_t>(out) + (o - off);
      if (base) {
        copy_span(dst, base + in_blk, n);
      } else {
        for (uint64_t k = threadIdx.x * 4; k < n; k += kThreads * 4) *reinterpret_cast<uint32_t*>(dst + k) = 0;
      }
      o += n;
      len -= n;
    }
  }
}

hipError_t launch_table_fetch(const uint64_t* table, uint64_t off, uint64_t bytes, void* out, uint32_t workgroups,
                              hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  if ((off | bytes | reinterpret_cast<uint64_t>(out)) & 3) return hipErrorInvalidValue;
  uint64_t pieces = (bytes + (64 << 10) - 1) / (64 << 10);
  uint32_t grid = pieces < workgroups ? (uint32_t)pieces : workgroups;
  hipLaunchKernelGGL(k_table_fetch, dim3(grid), dim3(kThreads), 0, s, table, off, bytes,
                     reinterpret_cast<uint8_t*>(out));
  return hipGetLastError();
}

// Every lane appends per_lane records (block = global lane id, page = i),
// never dropping: each append waits for ring space (the host drains).
__global__ void __launch_bounds__(64) k_fault_stress(KFaultBuf fb, uint32_t per_lane, uint32_t* gave_up) {
  const uint32_t id = blockIdx.x * 64 + threadIdx.x;
  const uint32_t ov0 = __hip_atomic_load(&fb.hdr->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (uint32_t i = 0; i < per_lane; ++i) fb_append(fb, 7, id, i, 1, 0, id, false);
  // a bounded wait that expired shows up as an overflow
  if (__hip_atomic_load(&fb.hdr->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != ov0 && threadIdx.x == 0)
    __hip_atomic_fetch_add(gave_up, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

hipError_t launch_fault_stress(KFaultBuf fb, uint32_t waves, uint32_t per_lane, uint32_t* gave_up, hipStream_t s) {
  if (!fb.hdr || !gave_up || waves == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fault_stress, dim3(waves), dim3(64), 0, s, fb, per_lane, gave_up);
  return hipGetLastError();
}

}  // namespace ogkm
