// Backend = the runtime's hardware abstraction (analog of the UVM HAL tables,
// uvm_hal.h:779-883, and of the nvUvmInterface bridge, nv_uvm_interface.c:142-1740).
//
// Two implementations:
//   * HipBackend  - MI355X (gfx950): HBM slabs / VMM handles, hipHostRegister'd
//                   host tiers, side hipStreams, hand-written CDNA4 copy kernels
//                   (csrc/kernels/copy_kernels.hip) with an SDMA comparator.
//   * FakeBackend - CPU-only "devices" whose HBM is a memfd and whose streams are
//                   worker threads doing memcpy (the fake CE HAL of
//                   uvm_page_tree_test.c:65-100, generalised). Used by the CPU
//                   test-suite and by the CPU-only north-star config.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "ogkm/common.hpp"
#include "ogkm/dgemm.hpp"

namespace ogkm {

// One contiguous copy. Addresses are device-usable pointers (HBM, registered host/CXL).
struct CopyDesc {
  uint64_t dst;
  uint64_t src;
  uint64_t bytes;
  uint32_t engine = 0;  // dma_copy: SDMA engine bit to use (0 = the backend picks by direction / channel)
};

// Page-list pack/unpack (k_gather_pages / k_scatter_pages): copies `npages`
// pages of `page_bytes` each; page i goes from src_base + idx[i]*page_bytes to
// dst (contiguous) for gather, or the reverse for scatter.
struct PageListDesc {
  uint64_t base;        // sparse side
  uint64_t contig;      // packed side
  const uint32_t* idx;  // host pointer to page indices (copied by the backend)
  uint32_t npages;
  uint32_t page_bytes;
};

// One fused copy+decode of a BF12-encoded block (codec.hpp) into raw bf16.
struct DecodeDesc {
  uint64_t src;       // encoded block (device-readable host / CXL memory)
  uint64_t dst;       // raw bf16 output (HBM)
  uint32_t n_values;
  uint32_t fmt = 0;   // staged ring decodes: 0 = ANS1 block, 1 = BF12 block
};

enum class LinkType : int { NONE = 0, SELF = 1, PCIE = 2, XGMI = 3 };

class Backend {
 public:
  virtual ~Backend() = default;
  virtual const char* name() const = 0;
  virtual bool is_fake() const = 0;
  virtual int device_count() = 0;
  virtual int device_numa_node(int dev) = 0;
  virtual Status device_mem_info(int dev, size_t* free_b, size_t* total_b) = 0;
  virtual Status set_device(int dev) = 0;

  // ---- HBM slab provider (one large allocation carved into 2 MB root chunks)
  virtual Status hbm_alloc(int dev, size_t bytes, void** ptr) = 0;
  // Device memory of a coherence kind: 0 = as hbm_alloc (coarse-grained),
  // 1 = fine-grained, 2 = uncached (loads never hit a stale L2 line after
  // another agent - an SDMA engine - wrote it).
  virtual Status hbm_alloc_kind(int dev, size_t bytes, void** ptr, int kind) {
    (void)kind;
    return hbm_alloc(dev, bytes, ptr);
  }
  virtual void hbm_free(int dev, void* ptr, size_t bytes) = 0;
  // ---- VMM provider (stable VA): physical 2 MB handles mapped into reserved VA
  virtual bool vmm_supported(int dev) = 0;
  virtual Status vmm_create(int dev, size_t bytes, uint64_t* handle) = 0;
  virtual void vmm_release(uint64_t handle) = 0;
  // `want` != null: reserve exactly there (in-place checkpoint restore) or fail with BUSY.
  virtual Status va_reserve(size_t bytes, void** va, void* want = nullptr) = 0;
  virtual void va_free(void* va, size_t bytes) = 0;
  virtual Status vmm_map(void* va, size_t bytes, uint64_t handle, int dev) = 0;
  virtual Status vmm_unmap(void* va, size_t bytes) = 0;
  // A stable-VA range's reservation, before its first vmm_map / after its last
  // vmm_unmap: the HIP backend remaps such VAs through ROCr
  // (hsa_amd_vmem_map / unmap: 5.3 + 2.3 us per 2 MB block against HIP's
  // 7.6 + 14.0, tools/probe_vmm_rocr_path.hip) and keeps HIP's own view of the
  // VA mapped to a per-device placeholder handle, so HIP copies on it resolve.
  virtual Status stable_va_prepare(void* va, size_t bytes, int dev) { return Status::OK; }
  virtual void stable_va_release(void* va, size_t bytes) {}
  // RAS error counters of a GPU (ECC of HBM / on-chip SRAM and xGMI link
  // errors): the analog of the reference's ECC error notifier and NVLink error
  // checks (uvm_gpu.c:1328-1354, 2087-2104). -1 = not reported by the platform.
  struct Health {
    int64_t ue = -1, ce = -1;            // uncorrectable / correctable, all blocks but xGMI
    int64_t link_ue = -1, link_ce = -1;  // xGMI (WAFL / PCS) link errors
    std::string source;                  // where the counters were read
  };
  virtual Status device_health(int dev, Health* out) {
    (void)dev;
    (void)out;
    return Status::NOT_SUPPORTED;
  }
  // Invalidate the process's cached GPU translations on `dev`. Needed after a
  // VA that was mapped to one handle is mapped to another: on this driver stack
  // (gfx950) hipMemUnmap / hipMemMap leave the old translation live, so the VA
  // keeps reading the previous chunk (tools/probe_vmm_tlb.hip).
  virtual Status tlb_flush(int dev) {
    (void)dev;
    return Status::OK;
  }

  // ---- host memory pinning (device-visible at the same address)
  virtual Status host_register(void* p, size_t bytes) = 0;
  virtual void host_unregister(void* p) = 0;
  // Fine-grained, coherent host memory for completion queues / fault rings.
  virtual Status host_alloc_coherent(size_t bytes, void** p) = 0;
  virtual void host_free_coherent(void* p) = 0;

  // ---- streams and events
  virtual void* stream_create(int dev, int priority) = 0;
  virtual void stream_destroy(void* s) = 0;
  virtual Status stream_sync(void* s) = 0;
  virtual void* event_create(int dev) = 0;
  virtual void event_destroy(void* e) = 0;
  virtual Status event_record(void* e, void* stream) = 0;
  virtual bool event_query(void* e) = 0;
  virtual Status event_sync(void* e) = 0;
  virtual Status stream_wait_event(void* stream, void* e) = 0;

  // ---- work submission (ordered on `stream`)
  // engine: 0 = copy kernel with the PCIe CU budget, 1 = hipMemcpyAsync, 2 = copy
  // kernel with the whole chip (HBM<->HBM), 4 = k_peer_push (source GPU writes
  // the peer's HBM over xGMI with config().peer_push_wgs workgroups).
  virtual Status copy_batch(int dev, const CopyDesc* d, size_t n, void* stream, int engine) = 0;
  // ---- DMA copy engines (SDMA), driven from a ring's worker thread: no CU, no
  // stream. `channel` picks the engine (one per ring kind and direction).
  // dma_copy returns once every copy of the batch has completed.
  virtual bool dma_supported(int dev) { (void)dev; return false; }
  virtual Status dma_copy(int dev, const CopyDesc* d, size_t n, int channel) {
    (void)dev; (void)d; (void)n; (void)channel;
    return Status::NOT_SUPPORTED;
  }
  // Split form of dma_copy for a pipelined ring worker: issue a batch on the
  // calling thread's completion slot (0 / 1) and return at once; dma_complete
  // waits for that slot. Default: synchronous (dma_copy, nothing to wait for).
  virtual Status dma_issue(int dev, const CopyDesc* d, size_t n, int channel, int slot) {
    (void)slot;
    return dma_copy(dev, d, n, channel);
  }
  virtual Status dma_complete(int slot) {
    (void)slot;
    return Status::OK;
  }
  // SDMA engines of `src_dev` able to copy src_dev -> dst_dev (-1 = host
  // memory): the bitmask of hsa_amd_memory_copy_engine_status(dst, src) - per
  // GPU pair for xGMI peers (uvm_gpu.c:2332-2388 reads peer caps per pair).
  virtual uint32_t copy_engine_mask(int dst_dev, int src_dev) { (void)dst_dev; (void)src_dev; return 0; }
  // Bytes each SDMA engine of `dev` has copied (index = engine bit), for tests / stats.
  virtual void engine_bytes(int dev, uint64_t out[32]) {
    (void)dev;
    for (int i = 0; i < 32; ++i) out[i] = 0;
  }
  // workgroups = 0: config().decode_workgroups (sized for H2D streaming); HBM->HBM
  // unpacking passes a full-chip grid.
  virtual Status decode_bf12(int dev, const DecodeDesc* d, size_t n, void* stream, uint32_t workgroups = 0) = 0;
  // Decode single-chunk ANS1 blocks (codec.hpp; the runtime's packed host
  // copies) from device-readable memory into bf16: one launch per <= 64 blocks.
  virtual Status decode_ans_blocks(int dev, const DecodeDesc* d, size_t n, void* stream) = 0;
  // Unpack a device-resident BF12 stream (codec.hpp) of n_values into bf16 at dst.
  // Chunk c lands at dst + (c >> row_shift) * dst_stride + (c mod 2^row_shift) *
  // chunk_values values (dst_stride 0 = contiguous).
  virtual Status unpack_bf12_stream(int dev, uint64_t src, uint64_t dst, uint32_t nchunks, uint32_t chunk_values,
                                    uint64_t n_values, void* stream, uint32_t workgroups, uint64_t dst_stride = 0,
                                    uint32_t row_shift = 0) = 0;
  // Same for an ANS stream (ANS1 / raw chunks, k_ans_unpack). The default serves
  // backends whose stream unpack decodes every chunk kind (the fake CPU one).
  virtual Status unpack_ans_stream(int dev, uint64_t src, uint64_t dst, uint32_t nchunks, uint32_t chunk_values,
                                   uint64_t n_values, void* stream, uint32_t workgroups, uint64_t dst_stride = 0,
                                   uint32_t row_shift = 0) {
    return unpack_bf12_stream(dev, src, dst, nchunks, chunk_values, n_values, stream, workgroups, dst_stride,
                              row_shift);
  }
  // Corrupt packed chunks seen by the device decoders since the last reset:
  // out = {count, stream address, chunk index, detail}. Decoders zero-fill such
  // chunks and report them here instead of decoding garbage.
  virtual void decode_errors(uint64_t out[4], bool reset) {
    for (int i = 0; i < 4; ++i) out[i] = 0;
    (void)reset;
  }
  // Decode GEMM (ogkm/dgemm.hpp): split-K partials, then the fused epilogue.
  virtual Status dgemm(int dev, const DGemmArgs& a, int mode, void* stream) = 0;
  virtual Status dgemm_reduce(int dev, const DGemmReduceArgs& a, void* stream) = 0;
  // Fused decode-step ops (ogkm/dgemm.hpp).
  virtual Status rmsnorm(int dev, const ResidNormArgs& a, void* stream) = 0;
  virtual Status rope_kv(int dev, const RopeKvArgs& a, void* stream) = 0;
  virtual Status attn_decode(int dev, const AttnArgs& a, void* stream) = 0;
  virtual Status gather_pages(int dev, const PageListDesc& d, void* stream) = 0;
  virtual Status scatter_pages(int dev, const PageListDesc& d, void* stream) = 0;
  // Asynchronous error state of a stream after its work completed (a kernel or
  // copy that faulted): OK while fine or still running.
  virtual Status stream_check(void* stream) { (void)stream; return Status::OK; }
  // Profiler annotations (roctx ranges / marks on the HIP backend):
  // rocprofv3 --marker-trace shows them on the CPU timeline.
  virtual void range_push(const char* name) { (void)name; }
  virtual void range_pop() {}
  virtual void mark(const char* name) { (void)name; }
  // Scattered 4 KiB pages of one block (npages <= 512): page idx[i] of src_base
  // -> page idx[i] of dst_base (k_page_copy_lds; the index list travels in the
  // kernel arguments).
  virtual Status page_copy(int dev, uint64_t dst_base, uint64_t src_base, const uint32_t* idx, uint32_t npages,
                           void* stream) = 0;
  virtual Status memset32(int dev, uint64_t dst, uint32_t pattern, size_t bytes, void* stream) = 0;
  // Write `value` to *addr (host-coherent) once all prior work on `stream` is done,
  // with system-scope release (the tracking-semaphore release of uvm_channel.c:1484-1580).
  virtual Status signal(int dev, uint64_t* addr, uint64_t value, void* stream) = 0;
  // Make `stream` wait until *addr >= value (GPU-side wait, no CPU involvement).
  virtual Status wait_value(void* stream, uint64_t* addr, uint64_t value) = 0;
  // Invalidate the GPU's caches for the work queued on `stream` after this
  // point (data another engine wrote since). Default: nothing to do.
  virtual Status acquire_caches(void* stream) {
    (void)stream;
    return Status::OK;
  }
  // Test hook (fake backend): a "kernel" on `stream` that sleeps delay_us and
  // then reads (and with `write`, increments) one word of every 4 KB page of
  // [ptr, ptr+bytes) - an access through an unmapped VA is a SIGSEGV on the
  // stream's thread.
  virtual Status debug_touch(void* /*stream*/, uint64_t /*ptr*/, uint64_t /*bytes*/, uint32_t /*delay_us*/,
                             bool /*write*/) {
    return Status::NOT_SUPPORTED;
  }

  // ---- peers
  virtual LinkType link_type(int a, int b) = 0;
  virtual bool can_access_peer(int a, int b) = 0;
  virtual Status enable_peer(int a, int b) = 0;

  // ---- export (dma-buf for NICs / importers; IPC for peer processes)
  virtual Status export_dmabuf(void* p, size_t bytes, int* fd, uint64_t* offset) = 0;
  // Importer side of a dma-buf (a third-party exporter, or our own export in
  // another process): map the fd into device `dev`'s address space.
  virtual Status import_dmabuf(int dev, int fd, void** ptr, size_t* bytes) {
    (void)dev; (void)fd; (void)ptr; (void)bytes;
    return Status::NOT_SUPPORTED;
  }
  virtual Status unimport_dmabuf(void* ptr) { (void)ptr; return Status::NOT_SUPPORTED; }
  virtual Status ipc_handle(void* p, std::string* handle) = 0;
  virtual Status ipc_open(const std::string& handle, void** p) = 0;
  virtual void ipc_close(void* p) = 0;

  virtual std::string last_error() { return ""; }
};

// Creates the best available backend: HIP when a gfx950 GPU is visible and
// RT_BACKEND != "fake", else the fake backend.
std::unique_ptr<Backend> make_backend(const std::string& want);
std::unique_ptr<Backend> make_fake_backend(int ndev, size_t hbm_bytes_per_dev);
std::unique_ptr<Backend> make_hip_backend();  // nullptr when unavailable

}  // namespace ogkm
