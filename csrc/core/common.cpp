// Common utilities: status strings, page-mask helpers, leveled logging, sticky fatal status.
#include <execinfo.h>
#include "ogkm/common.hpp"

#include <cstdarg>
#include <cstdlib>
#include <mutex>

#include "ogkm/config.hpp"

namespace ogkm {

const char* status_str(Status s) {
  switch (s) {
    case Status::OK: return "OK";
    case Status::NO_MEMORY: return "NO_MEMORY";
    case Status::MORE_PROCESSING_REQUIRED: return "MORE_PROCESSING_REQUIRED";
    case Status::INVALID_ARGUMENT: return "INVALID_ARGUMENT";
    case Status::NOT_FOUND: return "NOT_FOUND";
    case Status::BUSY: return "BUSY";
    case Status::NOT_SUPPORTED: return "NOT_SUPPORTED";
    case Status::IO_ERROR: return "IO_ERROR";
    case Status::LIMIT_EXCEEDED: return "LIMIT_EXCEEDED";
    case Status::INJECTED_ERROR: return "INJECTED_ERROR";
    case Status::PEER_LINK_DOWN: return "PEER_LINK_DOWN";
    case Status::FATAL: return "FATAL";
    case Status::TIMEOUT: return "TIMEOUT";
  }
  return "UNKNOWN";
}

const char* tier_str(Tier t) {
  switch (t) {
    case Tier::HBM: return "gpu";
    case Tier::HOST: return "host";
    case Tier::CXL: return "cxl";
  }
  return "?";
}

std::string Loc::str() const { return std::string(tier_str(tier)) + ":" + std::to_string(id); }

void PageMask::set_range(uint32_t first, uint32_t n) {
  uint32_t end = first + n;
  if (end > kPagesPerBlock) end = kPagesPerBlock;
  for (uint32_t p = first; p < end;) {
    uint32_t wi = p >> 6, bi = p & 63;
    uint32_t take = 64 - bi;
    if (take > end - p) take = end - p;
    uint64_t m = take == 64 ? ~0ull : (((1ull << take) - 1) << bi);
    w[wi] |= m;
    p += take;
  }
}

uint32_t PageMask::count_range(uint32_t first, uint32_t n) const {
  uint32_t end = first + n, c = 0;
  if (end > kPagesPerBlock) end = kPagesPerBlock;
  for (uint32_t p = first; p < end;) {
    uint32_t wi = p >> 6, bi = p & 63;
    uint32_t take = 64 - bi;
    if (take > end - p) take = end - p;
    uint64_t m = take == 64 ? ~0ull : (((1ull << take) - 1) << bi);
    c += (uint32_t)__builtin_popcountll(w[wi] & m);
    p += take;
  }
  return c;
}

void PageMask::clear_range(uint32_t first, uint32_t n) {
  uint32_t end = first + n;
  if (end > kPagesPerBlock) end = kPagesPerBlock;
  for (uint32_t p = first; p < end;) {
    uint32_t wi = p >> 6, bi = p & 63;
    uint32_t take = 64 - bi;
    if (take > end - p) take = end - p;
    uint64_t m = take == 64 ? ~0ull : (((1ull << take) - 1) << bi);
    w[wi] &= ~m;
    p += take;
  }
}

uint32_t PageMask::next_set(uint32_t p) const {
  while (p < kPagesPerBlock) {
    uint32_t wi = p >> 6;
    uint64_t x = w[wi] >> (p & 63);
    if (x) return p + __builtin_ctzll(x);
    p = (wi + 1) << 6;
  }
  return kPagesPerBlock;
}

uint32_t PageMask::next_clear(uint32_t p) const {
  while (p < kPagesPerBlock) {
    uint32_t wi = p >> 6;
    uint64_t x = (~w[wi]) >> (p & 63);
    if (x) {
      uint32_t r = p + __builtin_ctzll(x);
      return r < kPagesPerBlock ? r : kPagesPerBlock;
    }
    p = (wi + 1) << 6;
  }
  return kPagesPerBlock;
}

// ---------------------------------------------------------------- logging
static std::atomic<int> g_level{-1};

LogLevel log_level() {
  int l = g_level.load(std::memory_order_relaxed);
  if (l < 0) {
    const char* e = getenv("RT_LOG");
    l = 1;
    if (e) {
      std::string s(e);
      if (s == "error") l = 0;
      else if (s == "warn") l = 1;
      else if (s == "info") l = 2;
      else if (s == "debug") l = 3;
    }
    g_level.store(l);
  }
  return (LogLevel)l;
}

void set_log_level(LogLevel l) { g_level.store((int)l); }

void log_msg(LogLevel l, const char* file, int line, const char* fmt, ...) {
  static std::mutex m;
  static const char* names[] = {"ERROR", "WARN", "INFO", "DEBUG"};
  const char* base = strrchr(file, '/');
  base = base ? base + 1 : file;
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> g(m);
  fprintf(stderr, "[ogkm %s %s:%d] %s\n", names[(int)l], base, line, buf);
}

// ---------------------------------------------------------------- fatal status
static std::atomic<int> g_status{0};
static char g_fatal_why[256];

Status global_status() { return (Status)g_status.load(std::memory_order_acquire); }

void set_fatal(Status s, const char* why) {
  int expected = 0;
  if (g_status.compare_exchange_strong(expected, (int)s)) {
    snprintf(g_fatal_why, sizeof g_fatal_why, "%s", why ? why : "");
    RT_ERR("sticky fatal error %s: %s", status_str(s), g_fatal_why);
  }
}

void clear_fatal_for_test() { g_status.store(0); }

const char* fatal_reason() { return global_status() == Status::OK ? "" : g_fatal_why; }

#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
extern "C" void __sanitizer_print_stack_trace();
#endif

void assert_fail(const char* cond, const char* file, int line, bool release) {
  log_msg(LogLevel::ERROR, file, line, "assertion failed: %s", cond);
  {
    // where the invariant broke (symbolize the offsets with llvm-symbolizer --obj=<.so>)
    void* frames[32];
    const int n = backtrace(frames, 32);
    backtrace_symbols_fd(frames, n, 2);
  }
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
  __sanitizer_print_stack_trace();  // sanitizer test builds: where the broken invariant was hit
#endif
  if (release && config().release_asserts) set_fatal(Status::FATAL, cond);
#ifdef OGKM_DEBUG
  if (!release) abort();
#endif
}

}  // namespace ogkm
