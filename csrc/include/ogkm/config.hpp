// Runtime configuration: one flat table of integer knobs, loaded
// defaults -> RT_<NAME> environment variables -> rt.configure(**kw).
//
// Knob names and defaults intentionally match the reference's UVM module
// parameters so behaviour is comparable:
//   prefetch   uvm_perf_prefetch.c:37-61
//   thrashing  uvm_perf_thrashing.c:241-318
//   faults     uvm_gpu_replayable_faults.c:65-116
//   access ctr uvm_gpu_access_counters.c:40-84
//   pmm        uvm_pmm_gpu.c:183-192
//   channels   uvm_channel.c:82-85, uvm_channel.h:49
//   CXL fork   p2p_cxl.c:137-144, nv-p2p.c:1049,1079-1080, kern_bus_ctrl.c:769-774
#pragma once

#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace ogkm {

#define OGKM_CONFIG_KNOBS(X)                                                                          \
  /* prefetch heuristic */                                                                           \
  X(perf_prefetch_enable, 1, "enable the bitmap-tree prefetcher")                                    \
  X(perf_prefetch_threshold, 51, "percent of a subregion resident+faulted before it is prefetched")  \
  X(perf_prefetch_min_faults, 1, "faults to a block by the same processor before prefetching")       \
  /* thrashing detection */                                                                          \
  X(perf_thrashing_enable, 1, "enable thrashing detection")                                          \
  X(perf_thrashing_threshold, 3, "migrations within lapse that count as thrashing")                  \
  X(perf_thrashing_pin_threshold, 10, "throttles before a block is pinned")                          \
  X(perf_thrashing_lapse_usec, 500, "thrashing detection window (us)")                               \
  X(perf_thrashing_nap, 1, "throttle nap in lapses")                                                 \
  X(perf_thrashing_epoch, 2000, "lapses before thrashing state resets")                              \
  X(perf_thrashing_pin, 300, "pin duration in lapses")                                               \
  X(perf_thrashing_max_resets, 4, "max thrashing resets per block")                                  \
  X(perf_map_remote_on_native_atomics_fault, 0, "map remotely on atomics faults")                    \
  /* fault service */                                                                                \
  X(perf_fault_batch_count, 256, "faults fetched per batch")                                         \
  X(perf_fault_replay_policy, 2, "0=BLOCK 1=BATCH 2=BATCH_FLUSH 3=ONCE")                            \
  X(perf_fault_replay_update_put_ratio, 50, "duplicate percent that forces a put update")            \
  X(perf_fault_max_batches_per_service, 20, "batches per service call")                              \
  X(perf_fault_max_throttle_per_service, 5, "throttled faults tolerated per service call")           \
  X(perf_fault_coalesce, 1, "coalesce duplicate faults")                                             \
  X(perf_reenable_prefetch_faults_lapse_msec, 1000, "re-enable prefetch faults after (ms)")          \
  /* access counters */                                                                              \
  X(perf_access_counter_migration_enable, -1, "-1=auto 0=off 1=on")                                  \
  X(perf_access_counter_batch_count, 256, "notifications per batch")                                 \
  X(perf_access_counter_threshold, 256, "remote accesses to a 2MB region before migration")          \
  /* physical memory managers */                                                                     \
  X(global_oversubscription, 1, "allow eviction from HBM under pressure")                            \
  X(perf_pma_batch_nonpinned_order, 6, "log2 of chunks evicted per batch")                           \
  X(perf_workingset_active_pct, 95, "HBM chunks of refaulted GPU-preferred blocks (plus pinned chunks) protected from eviction, percent of the arena (0 = plain LRU)") \
  X(hbm_budget_mb, 0, "per-GPU HBM budget for the arena in MB (0 = 90% of free)")                   \
  X(hbm_provider, 0, "0=slab (one hipMalloc) 1=vmm (hipMemCreate handles, enables stable VA)")       \
  X(stable_lazy_unmap, 0, "stable VAs of evicted blocks stay mapped to their old chunk until the block returns (saves the unmap; a stray access reads stale data instead of faulting)") \
  X(stable_batch_blocks, 32, "stable-VA placement: 2 MB blocks per eviction / fill / remap group (pipelined)") \
  X(arena_reuse_cooldown, 0, "next-use eviction: data used within this many op-clock steps is kept (its readers may still be queued)") \
  X(arena_dead_cooldown, 0, "next-use eviction: freed data used within this many op-clock steps ranks as just used, not as the first victim") \
  X(perf_spread_enable, 1, "next-use eviction: the runtime splits cyclically hinted data into a keep class (error-diffused over the use order, sized to the arena) and a stream class evicted first (ogkm/spread.hpp); hints that carry their own class flag are left alone") \
  X(perf_spread_keep_pct, 97, "spread classes: percent of the HBM arena's unpinned capacity the keep class may fill") \
  X(perf_spread_adapt, 0, "spread classes: a pass that evicted keep-class data shrinks the keep class (online, from refaults). Off by default: on the 70B headline the keep-class evictions are structural (contiguous extents), shrinking the class only streams more (123.1 vs 129.4 tok/s, profiles/r5_spread.md)") \
  X(perf_spread_step_pct, 2, "spread classes: keep-share reduction per adaptation (percent)") \
  X(arena_victim_rank_top, 4096, "next-use eviction: a periodic victim-cache rebuild ranks only this many best chunks (at least 8x the request; the fallback pass ranks all; 0 = always all)") \
  X(arena_victim_cache_ops, 16, "next-use eviction: rebuild the ranked victim list after the op clock moved this far (0 = full scan per call)") \
  X(lease_fast_path, 1, "acquire: a GPU read of data resident in one contiguous extent only pins, touches and waits (no placement pass)") \
  X(unit_hold, 1, "UnitStream: after a pass with no eviction and no streaming, released units keep their leases until their next use (dropped at the first eviction / refused prefetch)") \
  X(unit_release_batch, 1, "UnitStream: released units are handed back in groups of this many behind one event (fewer event records on the consumer stream)") \
  X(ring_wait_issued, 1, "a GPU-side wait on a DMA ring value is enqueued only once that value's copies are on the engines (Ring::issued_seq; prevents an SDMA-engine cycle with HIP's own copies)") \
  X(arena_class_sides, 0, "spread classes: HBM extents of keep-class ranges are placed from the arena's low end, stream-class ones from its high end (less fragmentation of kept data by the stream turnover)") \
  X(arena_victim_rerank, 0, "next-use eviction: chunks whose key rose since the victim cache was built (re-hinted) are ranked ahead of its stale order. Off by default: the 70B headline is unchanged (129.5 vs 129.4) and the transparent 8B lost 12 % with it (profiles/r5_spread.md)") \
  X(ring_pipeline, 1, "DMA ring workers issue the next batch of plain copies before the previous one completed (two completion slots)") \
  X(vmm_rocr_remap, 1, "stable-VA remaps through ROCr hsa_amd_vmem_* (HIP keeps a placeholder mapping of the VA); 0 = hipMemMap / hipMemUnmap") \
  X(torch_persistent_ops, 128, "transparent mode: a managed tensor held again this many ops after its first hold is long-lived (keys the op-trace prefetcher)") \
  X(evict_clean_first, 0, "HBM LRU: GPU-preferred data with a valid copy elsewhere (clean) is evicted before data only in HBM (dirty: a copy-out plus a refill). Off: on the stock-torch managed 8B it protected every activation and thrashed the weights (193 -> 47 tok/s)") \
  X(torch_async_prefetch, 0, "transparent mode: op-trace prefetches (their evictions, stable-VA remaps and translation flushes) run on a per-GPU worker thread instead of the dispatching thread (measured slower on the stock 8B: 117 vs 197 tok/s - lock contention with the dispatching thread; 0 = inline)") \
  X(torch_alloc_empty_slabs, 2, "pluggable allocator: empty small-size slabs kept per size class for reuse (the rest go back to the HBM arena)") \
  X(torch_alloc_extent_cache_mb, 1024, "pluggable allocator: freed extents (> 1 MB) kept for same-size reuse on the freeing stream without a fence; handed back to the arena beyond this or under pressure") \
  X(torch_alloc_cache_mb, 256, "pluggable allocator: freed managed ranges kept (by size) for reuse at the same stable VA - no VA reserve / remap / translation flush per activation (0 = off)") \
  X(torch_alloc_managed_min_mb, 0, "pluggable allocator: allocations >= this many MB are evictable stable-VA managed ranges (0 = off; needs hbm_provider=1)") \
  X(host_node, -1, "NUMA node for the host tier (-1 = NUMA node of the first local GPU)")             \
  X(local_devices, 0, "bitmask of the GPUs this process manages (0 = all; one process per GPU: 1<<rank)") \
  X(fake_numa_nodes, 1, "fake backend: NUMA nodes the fake GPUs are spread over (GPU d on node d*n/ndev)") \
  X(host_budget_mb, 0, "host-tier arena limit in MB (0 = the node budget)")                          \
  X(node_ledger, 1, "host / CXL arenas reserve their segments in a node-wide shared-memory ledger (every runtime process on the machine; OGKM_NODE_LEDGER = its path)") \
  X(node_budget_mb, 0, "per-NUMA-node byte budget of the node ledger in MB (0 = the node's MemTotal x cxl_pin_budget_pct)") \
  X(pack_host_copies, 1, "keep lossless ANS1-packed host / CXL copies of read-mostly managed blocks (H2D moves the packed bytes; the ring decodes them in HBM)") \
  X(pack_auto_clean_evictions, 2, "a block whose HBM copy was evicted this many times without a copy-out counts as read-mostly and gets packed (0 = only SET_READ_MOSTLY blocks)") \
  X(pack_min_saving_pct, 8, "a block is kept packed only when its packed form saves at least this share of its bytes") \
  X(pack_read_dup_clean_evictions, 1, "clean HBM evictions after which a READ_MOSTLY block's host copy is packed") \
  X(pack_segments, 0, "segmented packed host copies (64 KB ANS1 segments, fmt 3) for blocks that are written: a write-back expands only the segments it touches, the rest stay packed (0 = whole blocks only). Off by default: on the stock 70B under ogkm.managed() it saves 2.5 of 63 GB/step H2D but costs more ring / host time than that (38.4 vs 49.6 tok/s, profiles/r6_segmented.md)") \
  X(pack_seg_min, 4, "a written block's host copy is segment-packed when at least this many of its 64 KB segments were untouched by its latest write-back") \
  X(pack_threads, 4, "host encoder threads of the packer") \
  X(ans_stage_mb, 128, "per-H2D-ring HBM staging buffer the packed bytes land in before the decode kernel (0: the kernel reads the host copy over PCIe)") \
  X(bf12_stage, 0, "H2D ring: BF12 blocks are staged into HBM by SDMA (4 engines) and decoded there, as ANS1 blocks are (0: the fused kernel reads the host copy over PCIe). Measured on 1 GiB, best of 3, across boxes: fused 70.9-73.9 GB/s of bf16 every run; staged 72-73 on some processes and 41-42 on others of the same build (tools/diag_bf12_refill.py, profiles/r6_bf12_refill.md)") \
  X(ring_defer_decodes, 1, "H2D ring: packed-block decodes overlap the next batch (two staging halves, deferred publish); 0 = drain after each batch's decodes") \
  X(ring_stage_overlap, 1, "H2D ring: a staging half's copies are issued before the host waits for the previous half's and launches its decode (0 = issue, wait, decode per half)") \
  X(ring_merge_packed_mb, 0, "H2D ring: queued batches of packed-block decodes run as one batch up to this many packed MB (0 = one batch at a time) Off by default: with it on, the packed transparent-mode training test read another block's decoded weights in a gradient, 6/6 runs, unresolved (profiles/r6_ring_merge_fix)") \
  X(gpu_wait_acquire, 0, "after a stream's GPU-side wait on a ring tracking value, a system-scope cache acquire kernel on that stream (every XCD's L2)") \
  X(debug_check_copy_owner, 0, "diagnostics: every copy into an HBM chunk asserts the chunk's arena owner is the destination block") \
  X(tlb_flush_repeat, 1, "diagnostics: translation flushes issued per flush_translations call") \
  X(ans_stage_mem, 0, "H2D ring staging buffer memory: 0 coarse-grained (hipMalloc), 1 fine-grained, 2 uncached") \
  X(ans_stage_engines, 0xF, "SDMA engines (mask) the H2D ring spreads packed-block staging copies over (0 = the ring's own engine)") \
  X(host_segment_mb, 1024, "host / CXL arenas populate, pin and reserve their memory in segments of this many MB") \
  /* channels / ring */                                                                              \
  X(channel_num_gpfifo_entries, 1024, "SQ/CQ entries per ring")                                      \
  X(copy_engine, 3, "PCIe/xGMI ring copies: 3=SDMA engines driven by the ring's worker (default) 1=hipMemcpyAsync 0=our CU copy kernels") \
  X(sdma_pcie_mask, 0, "SDMA engines used for host/CXL <-> HBM copies (bitmask; 0 = ROCr's preferred set, else engines 0-3)") \
  X(dma_spin_us, 20, "SDMA worker: spin this long on a batch's completion signal, then block")             \
  X(peer_copy_engine, 3, "GPU->GPU ring copies: 3=SDMA split over the pair's xGMI engines 0=k_peer_push CU kernel") \
  X(peer_split_min_mb, 8, "GPU->GPU copies >= 2x this are split into pieces over the pair's SDMA engines") \
  X(peer_push_wgs, 64, "workgroups (CU budget) of one k_peer_push launch")                             \
  X(copy_workgroups, 16, "workgroups per copy-kernel launch (CU budget; 16 saturate PCIe, more starve HBM-bound compute)") \
  X(copy_piece_kb, 64, "bytes per copy work item (KB)")                                              \
  X(copy_nt_loads, 1, "copy kernels: non-temporal source loads (0 = plain loads)")                      \
  X(trace_ranges, 1, "emit roctx ranges around runtime operations (fault batches, migrations, evictions)") \
  X(copy_page_list_min_runs, 4, "a block copy with at least this many page runs is one LDS-staged page-list kernel") \
  X(decode_workgroups, 256, "workgroups per fused copy+BF12-decode launch")                           \
  X(peer_copy, 1, "0=phys 1=virt peer addressing")                                                   \
  /* misc UVM knobs */                                                                               \
  X(fault_force_sysmem, 0, "always service faults in system memory")                                 \
  X(perf_map_remote_on_eviction, 0, "map evicted blocks remotely instead of refaulting")             \
  X(block_cpu_to_cpu_copy_with_ce, 0, "use the copy engine for CPU->CPU copies")                     \
  /* CXL fork constants */                                                                           \
  X(cxl_max_buffers, 256, "max registered CXL buffers")                                              \
  X(cxl_max_buffer_gb, 1024, "max single CXL buffer (GB)")                                           \
  X(cxl_pin_budget_pct, 90, "max pinned bytes as percent of system RAM")                             \
  X(cxl_max_dma_mb, 4095, "single CXL DMA request clamp (MB)")                                       \
  X(cxl_emulate_node, -1, "treat this NUMA node as CXL when no CXL hardware (-1 = off)")             \
  X(cxl_emulate_mask, 0, "bitmask of NUMA nodes treated as CXL pools when no CXL hardware")          \
  /* debug */                                                                                        \
  X(lock_check, 0, "enable the lock-order checker")                                                  \
  X(debug_copy_host_wait, 0, "diagnostics: a copy into a chunk host-waits for the chunk's reuse fence and the block's pending work before it is queued (1 = copies to a GPU, 2 = every copy)") \
  X(fake_race_check, 0, "fake backend: report kernels (debug_touch) that touch a chunk an engine copy is using") \
  X(fake_dma_delay_us, 0, "fake backend: microseconds every SDMA batch takes (ordering tests)")       \
  X(fake_kernel_delay_us, 0, "fake backend: each packed-block decode launch sleeps this long on its stream (tests)") \
  X(leak_check, 1, "track outstanding arena bytes")                                                  \
  X(release_asserts, 1, "release asserts set the sticky fatal error")                                \
  X(tools_queue_entries, 4096, "entries per tools event queue")

struct Config {
#define OGKM_DECL(name, def, doc) int64_t name = def;
  OGKM_CONFIG_KNOBS(OGKM_DECL)
#undef OGKM_DECL

  bool set(const std::string& name, int64_t v);
  bool get(const std::string& name, int64_t* v) const;
  void load_env();  // RT_<UPPER_NAME>
  void reset() {
    *this = Config();
    load_env();
  }
  std::vector<std::string> names() const;
  std::string doc(const std::string& name) const;
};

Config& config();
std::mutex& config_mutex();

}  // namespace ogkm
