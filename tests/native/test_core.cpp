// Native unit tests of the runtime core on the fake backend (analog of the
// reference's in-module UVM tests: uvm_pmm_test.c, uvm_range_tree_test.c,
// uvm_channel_test.c, uvm_lock_test.c). Built with g++ and run under
// AddressSanitizer + UBSan and under ThreadSanitizer by tests/test_native.py.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "ogkm/arena.hpp"
#include "ogkm/codec.hpp"
#include "ogkm/lock_order.hpp"
#include "ogkm/runtime.hpp"

namespace ogkm {
// This test binary has no HIP: the runtime falls back to the fake backend.
std::unique_ptr<Backend> make_hip_backend() { return nullptr; }
}  // namespace ogkm

using namespace ogkm;

static int g_fail = 0;
#define CHECK(c)                                                           \
  do {                                                                     \
    if (!(c)) {                                                            \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                            \
    }                                                                      \
  } while (0)
#define RUN(t)                            \
  do {                                    \
    fprintf(stderr, "[ RUN  ] %s\n", #t); \
    t();                                  \
  } while (0)

static void test_pagemask() {
  PageMask m;
  CHECK(m.empty());
  m.set_range(3, 70);
  CHECK(m.count() == 70 && m.test(3) && m.test(72) && !m.test(73) && !m.test(2));
  CHECK(m.next_set(0) == 3 && m.next_clear(3) == 73);
  m.clear_range(10, 5);
  int runs = 0;
  uint32_t total = 0;
  m.for_each_run([&](uint32_t, uint32_t n) {
    runs++;
    total += n;
  });
  CHECK(runs == 2 && total == 65);
  PageMask a = PageMask::all();
  CHECK(a.full() && a.count() == kPagesPerBlock);
  CHECK((a.andnot(m)).count() == kPagesPerBlock - 65);
}

struct TestArena : ChunkArena {
  explicit TestArena(uint32_t n) : ChunkArena("test", Loc::gpu(0), LockOrder::HBM_ARENA) {
    init_chunks(1ull << 40, n);
  }
};

static void test_arena_alloc_reserve() {
  TestArena a(64);
  uint32_t f1, f2, f3;
  CHECK(a.alloc(16, nullptr, -1, &f1) == Status::OK);
  CHECK(a.alloc(16, nullptr, -1, &f2) == Status::OK);
  CHECK(a.alloc(32, nullptr, -1, &f3) == Status::OK);
  uint32_t x;
  CHECK(a.alloc(1, nullptr, -1, &x) == Status::NO_MEMORY);
  CHECK(a.check().empty());
  // f1's chunks are the coldest: an 8-chunk reservation evicts inside them.
  for (uint32_t i = 0; i < 16; ++i) a.touch(f2 + i, true);
  for (uint32_t i = 0; i < 32; ++i) a.touch(f3 + i, true);
  Reservation r;
  CHECK(a.reserve(8, &r) == Status::OK);
  CHECK(r.first >= f1 && r.first + 8 <= f1 + 16 && r.victims.size() == 8);
  for (uint32_t v : r.victims) a.evicted(v);
  a.commit(r);
  CHECK(a.check().empty());
  // pinned chunks are never victims
  for (uint32_t i = 0; i < 64; ++i) a.pin(i);
  Reservation r2;
  CHECK(a.reserve(1, &r2) == Status::NO_MEMORY);
  for (uint32_t i = 0; i < 64; ++i) a.unpin(i);
  a.free(f2, 16);
  a.free(f3, 32);
  a.free((uint32_t)r.first, 8);
  for (uint32_t i = 0; i < 16; ++i)
    if ((int64_t)(f1 + i) < r.first || f1 + i >= r.first + 8) a.free(f1 + i, 1);
  CHECK(a.outstanding_bytes() == 0);
  CHECK(a.check().empty());
  CHECK(a.largest_free_run() == 64);
}

static void test_arena_random() {
  TestArena a(256);
  std::mt19937 rng(42);
  std::vector<std::pair<uint32_t, uint32_t>> live;
  for (int it = 0; it < 5000; ++it) {
    if (live.empty() || rng() % 3) {
      uint32_t n = 1 + rng() % 8, f;
      if (a.alloc(n, nullptr, -1, &f) == Status::OK) live.emplace_back(f, n);
    } else {
      size_t k = rng() % live.size();
      a.free(live[k].first, live[k].second);
      live.erase(live.begin() + k);
    }
  }
  CHECK(a.check().empty());
  for (auto& l : live) a.free(l.first, l.second);
  CHECK(a.outstanding_bytes() == 0 && a.largest_free_run() == 256);
}

static void test_codec() {
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 0.02f);
  const uint32_t n = 1u << 20;
  std::vector<uint16_t> in(n), out(n);
  for (uint32_t i = 0; i < n; ++i) {
    float f = nd(rng);
    uint32_t bits;
    memcpy(&bits, &f, 4);
    in[i] = (uint16_t)(bits >> 16);
  }
  const uint16_t specials[] = {0x0000, 0x8000, 0x7F80, 0xFF80, 0x7FC0, 0x0001, 0x3F80, 0xC2F7};
  for (uint32_t i = 0; i < 8; ++i) in[i * 1000 + 5] = specials[i];
  std::vector<uint8_t> enc(kBlockSize);
  uint64_t sz = bf12_encode(in.data(), n, enc.data(), enc.size());
  CHECK(sz > 0 && sz < (uint64_t)(0.76 * 2 * n));
  CHECK(bf12_decode(enc.data(), out.data(), n));
  CHECK(memcmp(in.data(), out.data(), 2ull * n) == 0);
  // incompressible (uniform random bits) -> refused, caller stores raw
  for (auto& v : in) v = (uint16_t)rng();
  CHECK(bf12_encode(in.data(), n, enc.data(), enc.size()) == 0);
}

static void test_codec_bf11() {
  std::mt19937 rng(11);
  std::normal_distribution<float> nd(0.f, 0.02f);
  for (uint32_t n : {1u << 20, 8u, 520u, 32768u + 512u + 8u}) {
    std::vector<uint16_t> in(n), out(n);
    for (uint32_t i = 0; i < n; ++i) {
      float f = nd(rng);
      uint32_t bits;
      memcpy(&bits, &f, 4);
      in[i] = (uint16_t)(bits >> 16);
    }
    const uint16_t specials[] = {0x0000, 0x8000, 0x7F80, 0xFF80, 0x7FC0, 0x0001, 0x3F80, 0xC2F7};
    for (uint32_t i = 0; i < 8 && i * 61 < n; ++i) in[i * 61] = specials[i];
    std::vector<uint8_t> enc(2ull * n + 4096);
    uint64_t sz = bf11_encode(in.data(), n, enc.data(), enc.size());
    CHECK(sz > 0);
    if (n == (1u << 20)) CHECK(sz < (uint64_t)(0.70 * 2 * n));
    std::fill(out.begin(), out.end(), 0xAAAA);
    CHECK(bf11_decode(enc.data(), out.data(), n));
    CHECK(memcmp(in.data(), out.data(), 2ull * n) == 0);
  }
  // streams: BF11 chunks, an incompressible chunk and a raw odd tail
  const uint64_t n = (3u << 20) + 6;
  std::vector<uint16_t> in(n), out(n);
  for (uint64_t i = 0; i < n; ++i) {
    float f = nd(rng);
    uint32_t bits;
    memcpy(&bits, &f, 4);
    in[i] = (uint16_t)(bits >> 16);
  }
  for (uint64_t i = 1u << 20; i < (2u << 20); ++i) in[i] = (uint16_t)rng();
  std::vector<uint8_t> st(bf12_pack_bound(n, 1u << 20));
  uint64_t total = bf12_pack(in.data(), n, 1u << 20, st.data(), st.size(), 4, PackFormat::BF11);
  CHECK(total > 0 && total < 2 * n);
  CHECK(bf12_unpack(st.data(), out.data(), n));
  CHECK(memcmp(in.data(), out.data(), 2 * n) == 0);
}

static void test_lockcheck() {
  lockcheck::set_enabled(true);
  uint64_t v0 = lockcheck::violations();
  OrderedMutex blk(LockOrder::VA_BLOCK), ar(LockOrder::HBM_ARENA);
  blk.lock();
  ar.lock();  // in order
  ar.unlock();
  blk.unlock();
  CHECK(lockcheck::violations() == v0);
  // Inverted order. A second mutex pair keeps TSan's own deadlock detector
  // (which would flag the real inversion) out of this deliberate violation.
  OrderedMutex blk2(LockOrder::VA_BLOCK), ar2(LockOrder::HBM_ARENA);
  ar2.lock();
  blk2.lock();
  blk2.unlock();
  ar2.unlock();
  CHECK(lockcheck::violations() == v0 + 1);
  lockcheck::reset_violations();
}

static void test_runtime_end_to_end() {
  Runtime* rt = Runtime::init("fake", 2, 64ull << 20);
  CHECK(rt != nullptr);
  lockcheck::set_enabled(true);
  lockcheck::reset_violations();
  CHECK(rt->init_device(0, 16ull << 20) == Status::OK);  // 8 chunks
  std::vector<Range*> rs;
  for (int i = 0; i < 4; ++i) {
    Range* r = nullptr;
    CHECK(rt->malloc_managed(6ull << 20, 0, "r" + std::to_string(i), &r) == Status::OK);
    std::vector<uint8_t> data(6ull << 20, (uint8_t)(i + 1));
    CHECK(rt->write(r, 0, data.data(), data.size(), -1) == Status::OK);
    rs.push_back(r);
  }
  // oversubscribed round robin (3 chunks each, 8 chunk budget): evictions + data integrity
  for (int round = 0; round < 3; ++round)
    for (int i = 0; i < 4; ++i) {
      Lease* l = nullptr;
      CHECK(rt->acquire(rs[i], 0, rs[i]->size, 0, Access::WRITE, &l) == Status::OK);
      if (!l) continue;
      CHECK(l->ready.wait() == Status::OK);
      CHECK(((uint8_t*)l->dptr)[12345] == (uint8_t)(i + 1));
      CHECK(rt->release(l, nullptr) == Status::OK);
    }
  CHECK(rt->dev(0).hbm->check().empty());
  // concurrent leases from several threads (lock discipline under TSan)
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < 20; ++k) {
        Range* r = rs[(t + k) % 4];
        Lease* l = nullptr;
        Status s = rt->acquire(r, 0, 2ull << 20, t % 2, Access::READ, &l);
        if (s == Status::BUSY || s == Status::NO_MEMORY) continue;  // all chunks leased by others
        if (s != Status::OK || l->ready.wait() != Status::OK) {
          bad++;
          continue;
        }
        if (((uint8_t*)l->dptr)[7] != (uint8_t)((t + k) % 4 + 1)) bad++;
        rt->release(l, nullptr);
      }
    });
  for (auto& x : th) x.join();
  CHECK(bad.load() == 0);
  CHECK(lockcheck::violations() == 0);
  std::vector<uint8_t> back(6ull << 20);
  CHECK(rt->read(rs[2], 0, back.data(), back.size(), -1) == Status::OK);
  CHECK(back[0] == 3 && back.back() == 3);
  for (Range* r : rs) CHECK(rt->free_range(r) == Status::OK);
  CHECK(rt->dev(0).hbm->outstanding_bytes() == 0);
  Runtime::shutdown();
}

// A chunk's reuse fence must survive its first writer: a second writer on
// another ring (D2D relocation + H2D fill of one extent) still has to wait for
// the previous owner's readers (round-2 corrupt-chunk bug).
static void test_reuse_fence_not_consumed() {
  Runtime* rt = Runtime::init("fake", 1, 64ull << 20);
  TestArena a(8);
  uint32_t f;
  CHECK(a.alloc(1, nullptr, -1, &f) == Status::OK);
  Ring* ring = rt->ring(0, RingKind::CPU_TO_GPU);
  auto pending = std::make_shared<Fence>();
  pending->ring = ring;
  pending->seq = ring->pushed_seq() + 1000;  // never completes during the test
  a.add_reuse_fence(f, pending);
  CHECK(a.reuse_fence(f).size() == 1);
  CHECK(a.reuse_fence(f).size() == 1);  // still there for the next writer
  auto done = std::make_shared<Fence>();
  done->done.store(true);
  a.add_reuse_fence(f, done);  // completed fences are never kept
  CHECK(a.reuse_fence(f).size() == 1);
  a.free(f, 1);
  Runtime::shutdown();
}

// Concurrent extent placement vs eviction on a small arena: no HBM chunk may
// ever back two blocks (owner-less unpinned extent chunks were
// eviction victims of a concurrent reserve()).
static void test_no_shared_chunks_under_concurrency() {
  Runtime* rt = Runtime::init("fake", 1, 64ull << 20);
  lockcheck::set_enabled(true);
  CHECK(rt->init_device(0, 24ull << 20) == Status::OK);  // 12 chunks
  std::vector<Range*> rs;
  for (int i = 0; i < 6; ++i) {
    Range* r = nullptr;
    CHECK(rt->malloc_managed(8ull << 20, 0, "c" + std::to_string(i), &r) == Status::OK);
    std::vector<uint8_t> data(8ull << 20, (uint8_t)(0x40 + i));
    CHECK(rt->write(r, 0, data.data(), data.size(), -1) == Status::OK);
    rs.push_back(r);
  }
  std::atomic<int> bad{0}, shared{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> th;
  for (int t = 0; t < 3; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < 40; ++k) {
        const size_t idx = (t * 2 + k) % rs.size();
        Range* r = rs[idx];
        Lease* l = nullptr;
        Status s = rt->acquire(r, 0, r->size, 0, Access::READ, &l);
        if (s != Status::OK) continue;  // BUSY / NO_MEMORY under contention is fine
        const uint8_t want = (uint8_t)(0x40 + idx);
        if (l->ready.wait() != Status::OK) bad++;
        else if (((uint8_t*)l->dptr)[0] != want || ((uint8_t*)l->dptr)[r->size - 1] != want)
          bad++;
        rt->release(l, nullptr);
      }
    });
  std::thread checker([&] {
    // A consistent snapshot: every block locked at once (trylock, all or none -
    // two block locks are never waited for together).
    std::vector<Block*> all;
    for (Range* r : rs)
      for (auto& bp : r->blocks) all.push_back(bp.get());
    while (!stop.load()) {
      size_t got = 0;
      while (got < all.size() && all[got]->lock.try_lock()) ++got;
      if (got == all.size()) {
        std::vector<std::pair<ChunkArena*, int64_t>> seen;
        for (Block* b : all)
          for (auto& x : b->res)
            if (x.loc.is_gpu() && x.chunk >= 0) seen.emplace_back(x.arena, x.chunk);
        std::sort(seen.begin(), seen.end());
        if (std::adjacent_find(seen.begin(), seen.end()) != seen.end()) shared++;
      }
      for (size_t i = 0; i < got; ++i) all[i]->lock.unlock();
      std::this_thread::yield();
    }
  });
  for (auto& x : th) x.join();
  stop.store(true);
  checker.join();
  CHECK(bad.load() == 0);
  CHECK(shared.load() == 0);
  {
    std::string why = rt->dev(0).hbm->check();
    if (!why.empty()) fprintf(stderr, "hbm check: %s\n", why.c_str());
    CHECK(why.empty());
  }
  for (int i = 0; i < (int)rs.size(); ++i) {
    std::vector<uint8_t> back(rs[i]->size);
    CHECK(rt->read(rs[i], 0, back.data(), back.size(), -1) == Status::OK);
    CHECK(back.front() == (uint8_t)(0x40 + i) && back.back() == (uint8_t)(0x40 + i));
  }
  for (Range* r : rs) CHECK(rt->free_range(r) == Status::OK);
  CHECK(lockcheck::violations() == 0);
  Runtime::shutdown();
}

// Reads a managed CPU view. Not TSan-instrumented: TSan keeps no shadow for the
// view's PROT_NONE reservation (later mprotect'ed page by page by the runtime),
// so an instrumented access would fault inside TSan itself.
__attribute__((no_sanitize("thread"), noinline)) static uint32_t view_read(const uint32_t* p) {
  return *(const volatile uint32_t*)p;
}

// Many threads touch the CPU views of managed ranges (SIGSEGV -> service
// thread -> cpu_fault) while other threads lease the same ranges on a fake GPU
// and migrate them back and forth. Under TSan this also checks that the signal
// handler does nothing signal-unsafe (TSan reports malloc / locks in handlers).
static void test_cpu_faults_concurrent() {
  Runtime* rt = Runtime::init("fake", 1, 64ull << 20);
  CHECK(rt->init_device(0, 16ull << 20) == Status::OK);
  const int nr = 4;
  const uint64_t sz = 4ull << 20;
  std::vector<Range*> rs;
  for (int i = 0; i < nr; ++i) {
    Range* r = nullptr;
    CHECK(rt->malloc_managed(sz, 0, "cf" + std::to_string(i), &r) == Status::OK);
    std::vector<uint32_t> data(sz / 4);
    for (size_t k = 0; k < data.size(); ++k) data[k] = (uint32_t)(i * 0x1000000 + k);
    CHECK(rt->write(r, 0, data.data(), sz, -1) == Status::OK);
    rs.push_back(r);
  }
  // Move every range to the GPU first: the views lose their mappings, so the
  // readers' first touches fault.
  for (int i = 0; i < nr; ++i) {
    Lease* l = nullptr;
    CHECK(rt->acquire(rs[i], 0, sz, 0, Access::WRITE, &l) == Status::OK);
    if (!l) continue;
    l->ready.wait();
    rt->release(l, nullptr);
  }
  std::atomic<int> bad{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> th;
  for (int t = 0; t < 6; ++t)
    th.emplace_back([&, t] {  // CPU readers through the views (real page faults)
      for (int k = 0; k < 300; ++k) {
        int i = (t + k) % nr;
        const uint32_t* v = (const uint32_t*)rs[i]->addr();
        size_t idx = ((size_t)k * 7919 + t * 104729) % (sz / 4);
        uint32_t got = view_read(v + idx);
        if (got != (uint32_t)(i * 0x1000000 + idx)) {
          if (bad++ < 4)
            fprintf(stderr, "cpu-fault test: range %d idx %zu read %08x want %08x\n", i, idx, got,
                    (uint32_t)(i * 0x1000000 + idx));
        }
      }
    });
  std::thread gpu([&] {  // a GPU user pulling the ranges into (tiny) HBM and out again
    for (int k = 0; !stop.load() && k < 200; ++k) {
      Lease* l = nullptr;
      Range* r = rs[k % nr];
      // WRITE: the GPU copy becomes the only one, the CPU views lose their mapping
      if (rt->acquire(r, 0, sz, 0, Access::WRITE, &l) != Status::OK) continue;
      l->ready.wait();
      rt->release(l, nullptr);
      Tracker t;
      rt->prefetch(r, 0, sz, rt->cpu_loc(), &t);
      t.wait();
    }
  });
  for (auto& x : th) x.join();
  stop.store(true);
  gpu.join();
  CHECK(bad.load() == 0);
  uint64_t serviced = 0, passed = 0;
  cpu_fault_stats(&serviced, &passed);
  CHECK(serviced > 0);
  CHECK(passed == 0);
  for (Range* r : rs) CHECK(rt->free_range(r) == Status::OK);
  Runtime::shutdown();
}


// Writes into ranges that prefer HBM while HBM is oversubscribed (the
// planner-off model init): each write stages on the host, then migrates to the
// GPU, evicting earlier ranges.
static void test_write_preferred_gpu_oversubscribed() {
  Runtime* rt = Runtime::init("fake", 1, 64ull << 20);
  CHECK(rt->init_device(0, 16ull << 20) == Status::OK);
  std::vector<Range*> rs;
  for (int i = 0; i < 10; ++i) {
    Range* r = nullptr;
    CHECK(rt->malloc_managed((3ull << 20) + 4096 * i, 0, "pg" + std::to_string(i), &r) == Status::OK);
    CHECK(rt->mem_advise(r, 0, r->size, Advice::SET_PREFERRED_LOCATION, Loc::gpu(0), 0) == Status::OK);
    CHECK(rt->mem_advise(r, 0, r->size, Advice::SET_READ_MOSTLY, Loc{}, 0) == Status::OK);
    std::vector<uint8_t> data(r->size, (uint8_t)(0x30 + i));
    CHECK(rt->write(r, 0, data.data(), data.size(), -1) == Status::OK);
    rs.push_back(r);
  }
  for (int i = 0; i < 10; ++i) {
    std::vector<uint8_t> back(rs[i]->size);
    CHECK(rt->read(rs[i], 0, back.data(), back.size(), -1) == Status::OK);
    CHECK(back.front() == (uint8_t)(0x30 + i) && back.back() == (uint8_t)(0x30 + i));
  }
  CHECK(rt->dev(0).hbm->check().empty());
  for (Range* r : rs) CHECK(rt->free_range(r) == Status::OK);
  Runtime::shutdown();
}

int main() {
  RUN(test_pagemask);
  RUN(test_arena_alloc_reserve);
  RUN(test_arena_random);
  RUN(test_codec);
  RUN(test_codec_bf11);
  RUN(test_lockcheck);
  RUN(test_runtime_end_to_end);
  RUN(test_reuse_fence_not_consumed);
  RUN(test_no_shared_chunks_under_concurrency);
  RUN(test_cpu_faults_concurrent);
  RUN(test_write_preferred_gpu_oversubscribed);
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  fprintf(stderr, "ALL NATIVE TESTS PASSED\n");
  return 0;
}
