// Host-runtime self test, built with sanitizers by scripts/sanitize_native.sh (ASan + UBSan, and TSan for
// the concurrent paths). Exercises the TCAP parser, the slab allocator, page files, and the buffer manager
// under concurrent pin/unpin from several threads plus WorkerQueue prefetch/flush work.
// Exit code 0 = every check passed; a sanitizer report or a failed CHECK exits non-zero.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

using namespace nsdb_rt;

#define CHECK(c)                                                           \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(2);                                                        \
    }                                                                      \
  } while (0)

static void test_tcap() {
  const char* text =
      "in(a) <= SCAN ('db', 's', 'Scan_0')\n"
      "b(a, k) <= APPLY (in(a), in(a), 'Sel_1', 'attAccess_0')\n"
      "c(a) <= FILTER (b(k), b(a), 'Sel_1')\n"
      "h(a, hk) <= HASHLEFT (b(k), b(a), 'Join_2', '==_1')\n"
      "out() <= OUTPUT (c(a), 'db', 'o', 'Write_3')\n";
  auto atoms = parse_tcap(text);
  CHECK(atoms.size() == 5);
  CHECK(atoms[1].type == "APPLY" && atoms[1].lambda == "attAccess_0");
  CHECK(atoms[4].type == "OUTPUT" && atoms[4].set == "o");
  bool threw = false;
  try {
    parse_tcap("x(a) <= BOGUS (y(a), 'c')");
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_slab() {
  SlabAllocator s(1 << 20, 256);
  std::vector<int64_t> offs;
  for (int i = 0; i < 64; ++i) {
    int64_t o = s.alloc(1000 + i * 37);
    CHECK(o >= 0 && o % 256 == 0);
    offs.push_back(o);
  }
  for (size_t i = 0; i < offs.size(); i += 2) s.free(offs[i]);
  for (size_t i = 1; i < offs.size(); i += 2) s.free(offs[i]);
  CHECK(s.used() == 0 && s.num_allocations() == 0);
  CHECK(s.largest_free() == (1u << 20));   // everything coalesced back
  CHECK(s.alloc(2u << 20) == -1);
}

static void test_pagefile(const std::string& dir) {
  PageFile f(dir + "/pf.dat", 4096);
  std::vector<uint8_t> a(3000, 7), b(4096, 9), out(4096);
  f.write_page(3, a.data(), a.size());
  f.write_page(0, b.data(), b.size());
  CHECK(f.has_page(3) && f.has_page(0) && !f.has_page(1));
  CHECK(f.read_page(3, out.data(), out.size()) == 3000 && out[2999] == 7);
  CHECK(f.read_page(0, out.data(), out.size()) == 4096 && out[4095] == 9);
  f.sync();
}

static void test_buffer_manager_concurrent(const std::string& dir) {
  const uint64_t page = 4096;
  BufferManager bm(page, 8, dir);
  const int sets = 4, pages = 24;
  // create pages (more than the pool holds: eviction to the page files happens while writing)
  for (int s = 0; s < sets; ++s)
    for (int p = 0; p < pages; ++p) {
      int64_t slot = bm.pin(s, p, true);
      std::memset(bm.slot_ptr(slot), (s * 31 + p) & 0xff, page);
      bm.unpin(s, p, true, page);
    }
  CHECK(bm.evictions() > 0);
  WorkerQueue q(3);
  std::atomic<int> errors{0};
  // readers pin/verify/unpin while the workers prefetch and flush the same sets
  std::vector<std::thread> readers;
  for (int t = 0; t < 4; ++t)
    readers.emplace_back([&, t] {
      for (int it = 0; it < 200; ++it) {
        const int s = (t + it) % sets, p = (it * 7 + t) % pages;
        int64_t slot = bm.pin(s, p, false);
        const uint8_t v = bm.slot_ptr(slot)[page - 1];
        if (v != ((s * 31 + p) & 0xff)) errors.fetch_add(1);
        bm.unpin(s, p, false, 0);
      }
    });
  std::vector<std::shared_ptr<Buzzer>> buzz;
  for (int i = 0; i < 40; ++i) {
    const int s = i % sets;
    if (i % 3 == 0) {
      buzz.push_back(q.submit([&bm, s] { bm.flush_set(s); }));
    } else {
      buzz.push_back(q.submit([&bm, s, i] {
        for (int p = i % 5; p < pages; p += 5) bm.prefetch(s, p);
      }));
    }
  }
  for (auto& r : readers) r.join();
  for (auto& b : buzz) CHECK(b->wait(60.0) && b->error().empty());
  q.drain();
  CHECK(q.pending() == 0 && q.completed() == 40);
  CHECK(errors.load() == 0);
  // a failing work item reports through its buzzer instead of killing the worker
  auto bad = q.submit([] { throw std::runtime_error("boom"); });
  CHECK(bad->wait(10.0) && bad->error() == "boom");
  auto ok = q.submit([] {});
  CHECK(ok->wait(10.0) && ok->error().empty());
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_tcap();
  test_slab();
  test_pagefile(dir);
  test_buffer_manager_concurrent(dir);
  std::printf("runtime selftest ok\n");
  return 0;
}
