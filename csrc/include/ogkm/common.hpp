// Common vocabulary of the ogkm tiering runtime: status codes, memory locations,
// processor masks, 4 KB page masks over a 2 MB block, logging and assertions.
//
// Parity notes (reference = NVIDIA open-gpu-kernel-modules + CXL fork):
//  * 2 MB block / 4 KB page geometry mirrors UVM_VA_BLOCK_BITS=21
//    (kernel-open/nvidia-uvm/uvm_va_block_types.h:42-50).
//  * Status::MORE_PROCESSING_REQUIRED is the allocation-retry protocol status
//    (NV_ERR_MORE_PROCESSING_REQUIRED, uvm_va_block.c:2088-2101).
//  * Assertions follow UVM_ASSERT / UVM_ASSERT_RELEASE semantics
//    (uvm_common.h:166-200): debug asserts compile out, release asserts set the
//    sticky fatal status.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace ogkm {

constexpr uint32_t kPageShift = 12;
constexpr uint64_t kPageSize = 1ull << kPageShift;          // 4 KB
constexpr uint32_t kBlockShift = 21;
constexpr uint64_t kBlockSize = 1ull << kBlockShift;        // 2 MB
constexpr uint32_t kPagesPerBlock = kBlockSize / kPageSize;  // 512
constexpr int kMaxGpus = 32;
constexpr int kMaxNodes = 32;
constexpr int kMaxLocs = kMaxGpus + kMaxNodes;  // memory locations (64 -> one u64 mask)
constexpr int kCpuProc = 32;                    // processor id of the CPU (GPUs are 0..31)

enum class Status : int {
  OK = 0,
  NO_MEMORY = 1,
  MORE_PROCESSING_REQUIRED = 2,  // allocation retry after eviction
  INVALID_ARGUMENT = 3,
  NOT_FOUND = 4,
  BUSY = 5,
  NOT_SUPPORTED = 6,
  IO_ERROR = 7,
  LIMIT_EXCEEDED = 8,
  INJECTED_ERROR = 9,   // returned by fault-injection hooks
  PEER_LINK_DOWN = 10,
  FATAL = 11,
  TIMEOUT = 12,
};
const char* status_str(Status s);

// Memory tier of a location. HBM is per GPU; HOST and CXL are per NUMA node.
enum class Tier : uint8_t { HBM = 0, HOST = 1, CXL = 2 };
const char* tier_str(Tier t);

// A memory location = (tier, id). Encoded in one byte-sized slot for masks:
// HBM of GPU g -> slot g; NUMA node n (HOST or CXL) -> slot 32+n.
struct Loc {
  Tier tier = Tier::HOST;
  int16_t id = 0;
  static Loc gpu(int g) { return Loc{Tier::HBM, (int16_t)g}; }
  static Loc host(int n) { return Loc{Tier::HOST, (int16_t)n}; }
  static Loc cxl(int n) { return Loc{Tier::CXL, (int16_t)n}; }
  int slot() const { return tier == Tier::HBM ? id : kMaxGpus + id; }
  bool is_gpu() const { return tier == Tier::HBM; }
  bool operator==(const Loc& o) const { return tier == o.tier && id == o.id; }
  bool operator!=(const Loc& o) const { return !(*this == o); }
  std::string str() const;
};
using LocMask = uint64_t;   // bit = Loc::slot()
using ProcMask = uint64_t;  // bit g = GPU g, bit 32 = CPU
inline LocMask loc_bit(const Loc& l) { return 1ull << l.slot(); }

// 512-bit page mask over a 2 MB block.
struct PageMask {
  uint64_t w[kPagesPerBlock / 64] = {0};
  void set(uint32_t p) { w[p >> 6] |= 1ull << (p & 63); }
  void clear(uint32_t p) { w[p >> 6] &= ~(1ull << (p & 63)); }
  bool test(uint32_t p) const { return (w[p >> 6] >> (p & 63)) & 1; }
  void set_range(uint32_t first, uint32_t n);
  void clear_range(uint32_t first, uint32_t n);
  uint32_t count_range(uint32_t first, uint32_t n) const;  // set pages in [first, first+n)
  void fill() { for (auto& x : w) x = ~0ull; }
  void zero() { for (auto& x : w) x = 0; }
  bool empty() const { for (auto x : w) if (x) return false; return true; }
  bool full() const { for (auto x : w) if (x != ~0ull) return false; return true; }
  uint32_t count() const { uint32_t c = 0; for (auto x : w) c += __builtin_popcountll(x); return c; }
  PageMask operator&(const PageMask& o) const { PageMask r; for (int i = 0; i < 8; ++i) r.w[i] = w[i] & o.w[i]; return r; }
  PageMask operator|(const PageMask& o) const { PageMask r; for (int i = 0; i < 8; ++i) r.w[i] = w[i] | o.w[i]; return r; }
  PageMask operator~() const { PageMask r; for (int i = 0; i < 8; ++i) r.w[i] = ~w[i]; return r; }
  PageMask andnot(const PageMask& o) const { PageMask r; for (int i = 0; i < 8; ++i) r.w[i] = w[i] & ~o.w[i]; return r; }
  PageMask& operator|=(const PageMask& o) { for (int i = 0; i < 8; ++i) w[i] |= o.w[i]; return *this; }
  PageMask& operator&=(const PageMask& o) { for (int i = 0; i < 8; ++i) w[i] &= o.w[i]; return *this; }
  bool operator==(const PageMask& o) const { return memcmp(w, o.w, sizeof w) == 0; }
  bool intersects(const PageMask& o) const { for (int i = 0; i < 8; ++i) if (w[i] & o.w[i]) return true; return false; }
  // Next set bit at or after p, or kPagesPerBlock.
  uint32_t next_set(uint32_t p) const;
  uint32_t next_clear(uint32_t p) const;
  // Iterate maximal runs [first, first+len) of set pages: coalesced copies
  // (analog of the contiguous-run coalescing at uvm_va_block.c:4278-4326).
  template <class F> void for_each_run(F&& f) const {
    uint32_t p = next_set(0);
    while (p < kPagesPerBlock) {
      uint32_t e = next_clear(p);
      f(p, e - p);
      p = next_set(e);
    }
  }
  // Number of maximal runs of set pages (rising edges of the 512-bit mask).
  uint32_t runs() const {
    uint32_t r = 0;
    uint64_t carry = 0;  // bit 63 of the previous word
    for (int i = 0; i < 8; ++i) {
      r += __builtin_popcountll(w[i] & ~((w[i] << 1) | carry));
      carry = w[i] >> 63;
    }
    return r;
  }
  static PageMask all() { PageMask m; m.fill(); return m; }
  static PageMask range(uint32_t first, uint32_t n) { PageMask m; m.set_range(first, n); return m; }
};

// ---------------------------------------------------------------- logging
enum class LogLevel : int { ERROR = 0, WARN = 1, INFO = 2, DEBUG = 3 };
LogLevel log_level();
void set_log_level(LogLevel l);
void log_msg(LogLevel l, const char* file, int line, const char* fmt, ...) __attribute__((format(printf, 4, 5)));

#define RT_LOG(lvl, ...)                                                                   \
  do {                                                                                     \
    if ((int)(lvl) <= (int)::ogkm::log_level()) ::ogkm::log_msg(lvl, __FILE__, __LINE__, __VA_ARGS__); \
  } while (0)
#define RT_ERR(...) RT_LOG(::ogkm::LogLevel::ERROR, __VA_ARGS__)
#define RT_WARN(...) RT_LOG(::ogkm::LogLevel::WARN, __VA_ARGS__)
#define RT_INFO(...) RT_LOG(::ogkm::LogLevel::INFO, __VA_ARGS__)
#define RT_DBG(...) RT_LOG(::ogkm::LogLevel::DEBUG, __VA_ARGS__)

// Sticky global status (uvm_global_set_fatal_error_impl, uvm_global.c:420-438).
Status global_status();
void set_fatal(Status s, const char* why);
void clear_fatal_for_test();
const char* fatal_reason();  // why the sticky status was set ("" when OK)

void assert_fail(const char* cond, const char* file, int line, bool release);
#define RT_ASSERT_RELEASE(c) \
  do { if (!(c)) ::ogkm::assert_fail(#c, __FILE__, __LINE__, true); } while (0)
#ifdef OGKM_DEBUG
#define RT_ASSERT(c) do { if (!(c)) ::ogkm::assert_fail(#c, __FILE__, __LINE__, false); } while (0)
#else
#define RT_ASSERT(c) do { (void)sizeof(c); } while (0)
#endif

inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) & ~(a - 1); }
inline uint64_t align_down(uint64_t x, uint64_t a) { return x & ~(a - 1); }

}  // namespace ogkm
