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
//  * PCIe-bound ring copies default to hipMemcpyAsync (config copy_engine=1):
//    this kernel reading host memory slows concurrent HBM-bound kernels 3-7x
//    (2.5x less with plain instead of non-temporal loads, copy_nt_loads=0;
//    measured, profiles/r1_copy_engine_interference.md). These kernels serve HBM<->HBM
//    copies, page gather/scatter, the fused copy+decode path and copy_engine=0.
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

// Device-side residency check + gather. table[2*b] = HBM address of block b (0 if
// not resident on this GPU), table[2*b+1] = remote (host/CXL) address. One
// workgroup per row; lane 0 resolves the source and records misses / remote
// accesses into the fault buffer (software replayable-fault + access-counter
// producer).
struct DevFaultRec {
  uint64_t range_id;
  uint32_t block;
  uint16_t page;
  uint8_t access;
  uint8_t kind;
  uint32_t proc;
  uint32_t pad;
};

__global__ void __launch_bounds__(kThreads)
    k_managed_gather(const uint64_t* __restrict__ table, uint64_t range_id, const int64_t* __restrict__ rows,
                     uint32_t nrows, uint32_t row_bytes, uint8_t* __restrict__ out, KFaultBuf fb, uint32_t proc) {
  __shared__ uint64_t s_src;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    if (threadIdx.x == 0) {
      uint64_t off = (uint64_t)rows[r] * row_bytes;
      uint64_t b = off >> 21;
      uint64_t in_blk = off & ((1ull << 21) - 1);
      uint64_t hbm = __hip_atomic_load(table + 2 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      uint64_t rem = __hip_atomic_load(table + 2 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      uint64_t src = hbm ? hbm + in_blk : (rem ? rem + in_blk : 0);
      if (!hbm && fb.put) {
        uint32_t slot = __hip_atomic_fetch_add(fb.put, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (slot < fb.entries) {
          DevFaultRec rec;
          rec.range_id = range_id;
          rec.block = (uint32_t)b;
          rec.page = (uint16_t)(in_blk >> 12);
          rec.access = 1;
          rec.kind = rem ? 1 : 0;
          rec.proc = proc;
          rec.pad = 0;
          reinterpret_cast<DevFaultRec*>(fb.recs)[slot] = rec;
        }
      }
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

}  // namespace ogkm
