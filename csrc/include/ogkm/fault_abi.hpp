// Device fault buffer ABI shared by the runtime (host, g++ or hipcc) and the
// HIP kernels that produce records.
//
// The buffer is a GET/PUT ring in host-coherent memory, the analog of the
// replayable fault buffer (uvm_gpu_replayable_faults.c:558 write_get,
// :844-988 fetch):
//   * a producer (kernel lane) drops the record and counts an overflow when the
//     ring is full at a first look (the faulting kernel re-records after the
//     next replay, like a fault dropped on buffer overflow); otherwise it
//     reserves a slot with ONE atomic add on PUT (a CAS loop would serialise
//     every producer at the PCIe root complex), waits until the host has
//     consumed the slot's previous lap (GET > slot - entries), fills the record
//     and publishes it by storing seq = slot + 1 with release semantics;
//   * the host consumes in order from GET, accepts a record once its seq
//     matches (acquire) and re-checks seq after copying it (a producer that gave
//     up waiting may overwrite a slot: the older record then counts as lost,
//     never as garbage), and hands slots back by advancing GET (release).
// PUT is never reset, so a record appended while the host drains is never lost.
//
// Replay: after a serviced batch has LANDED (its copies complete and the device
// residency tables refreshed) the host bumps `replay`; a kernel stalled on a
// fault (k_fault_gate) waits for the token to move, then re-checks residency -
// the replay policy BATCH_FLUSH of uvm_gpu_replayable_faults.c:2986-3022.
//
// Precise cancel (cancel_faults_precise, uvm_gpu_replayable_faults.c:2863):
// when servicing a channel's fault fails (or the fault is fatal: freed range,
// out of bounds), the host bumps `cancel[channel]` (ids 1..kFaultCancelSlots-1;
// unattributed faults, channel 0, are never cancelled) BEFORE
// the replay token. A gate snapshots its channel's word at entry and, once the
// replay wakes it, exits with status kGateCancelled instead of re-recording.
#pragma once

#include <cstdint>

namespace ogkm {

constexpr uint16_t kFaultWholeBlock = 0xffff;  // record.page: the access needs the whole 2 MB block
constexpr uint32_t kFaultCancelSlots = 64;      // per-channel cancel words (channel ids 1..63; 0 = no channel)
// k_fault_gate status[0]
constexpr uint32_t kGateResolved = 0, kGateTimeout = 2, kGateCancelled = 3;

struct DeviceFaultRecord {
  uint64_t range_id;
  uint32_t block;
  uint16_t page;
  uint8_t access;   // 1 read 2 write
  uint8_t kind;     // 0 miss (fault), 1 remote access (access counter)
  uint32_t proc;
  uint32_t seq;     // slot + 1, stored last (release): the record is valid
};
static_assert(sizeof(DeviceFaultRecord) == 24, "device fault record layout");

// One field per 64 B line: device atomics on PUT and the host's GET stores do
// not share a line.
struct FaultBufHeader {
  uint32_t put;        // slots reserved by producers (monotonic, wraps at 2^32)
  uint32_t pad0[15];
  uint32_t get;        // slots consumed by the host (monotonic)
  uint32_t pad1[15];
  uint32_t overflow;   // records dropped on a full ring (producer atomics)
  uint32_t pad2[15];
  uint64_t replay;     // bumped by the host after each serviced batch landed
  uint64_t pad3[7];
  uint32_t cancel[kFaultCancelSlots];  // bumped (before `replay`) when a channel's faults are cancelled
};
static_assert(sizeof(FaultBufHeader) == 256 + 4 * kFaultCancelSlots, "fault buffer header layout");

// Host-side producer with the device protocol (fake backend, tests, CPU
// emulation of a faulting processor). `entries` is a power of two. `may_drop`:
// a full ring drops the record (counted) instead of waiting for space.
bool fault_buf_produce(FaultBufHeader* h, DeviceFaultRecord* recs, uint32_t entries, DeviceFaultRecord rec,
                       bool may_drop = true);

}  // namespace ogkm
