// Host-side stress test of the native runtime, built with sanitizers by
// tools/sanitize.sh (ASan+UBSan and TSan builds; GPU sanitizers are not available):
//   * MPMC IndexRing: P producers / C consumers move every index exactly once
//     (the reference's free/full queue pair, microbeast.py:169-175);
//   * seqlock: a writer republishes a buffer while readers copy it; every successful
//     read must be internally consistent (no torn weights, libs/utils.py:337);
//   * VecEnv: packed-action stepping (plain and self-play) over many episodes, with
//     worker threads stepping disjoint env ranges concurrently (GpuEngine's pattern).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <random>
#include <thread>
#include <vector>

#include "../runtime/shm_ring.h"
#include "../runtime/vec_env.h"

using namespace mb;

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

static void ring_test() {
  const size_t cap = 64;
  std::vector<uint64_t> mem((IndexRing::bytes_needed(cap) + 7) / 8);
  IndexRing ring(mem.data(), cap, true);
  const int P = 3, C = 3, per = 20000;
  std::vector<std::atomic<int>> seen(P * per);
  for (auto& s : seen) s.store(0);
  std::vector<std::thread> th;
  for (int p = 0; p < P; ++p)
    th.emplace_back([&, p] {
      for (int i = 0; i < per; ++i) CHECK(ring.push(p * per + i, 10.0));
    });
  std::atomic<int> got{0};
  for (int c = 0; c < C; ++c)
    th.emplace_back([&] {
      int64_t v;
      while (got.load() < P * per) {
        if (ring.pop(&v, 0.01)) {
          CHECK(v >= 0 && v < P * per);
          seen[v].fetch_add(1);
          got.fetch_add(1);
        }
      }
    });
  for (auto& t : th) t.join();
  for (auto& s : seen) CHECK(s.load() == 1);
  ring.close();
  int64_t v;
  CHECK(!ring.pop(&v, 0.0));
  std::printf("ring ok (%d items, %d producers, %d consumers)\n", P * per, P, C);
}

static void seqlock_test() {
  const size_t n = 4096;
  std::vector<uint64_t> buf(n, 0);
  std::atomic<uint64_t> ver{0};
  std::atomic<bool> stop{false};
  std::thread writer([&] {
    std::vector<uint64_t> src(n);
    for (uint64_t k = 1; k <= 3000; ++k) {
      std::fill(src.begin(), src.end(), k);
      seqlock_write(&ver, src.data(), buf.data(), n * 8);
    }
    stop.store(true);
  });
  std::vector<std::thread> readers;
  std::atomic<int> good{0};
  for (int r = 0; r < 2; ++r)
    readers.emplace_back([&] {
      std::vector<uint64_t> dst(n);
      while (!stop.load()) {
        if (seqlock_read(&ver, buf.data(), dst.data(), n * 8, 64)) {
          for (size_t i = 1; i < n; ++i) CHECK(dst[i] == dst[0]);  // never torn
          good.fetch_add(1);
        }
      }
    });
  writer.join();
  for (auto& t : readers) t.join();
  std::printf("seqlock ok (%d consistent reads)\n", good.load());
}

static void env_test() {
  const int s = 10, n = 64, S = s * s, threads = 4;
  VecEnv env(s, n, 120, 3, {0, 1, 2, 3, 5}, nullptr, 0);
  env.set_validate(false);
  env.set_external_opponent(n / 2, n, true);
  std::vector<uint16_t> codes((size_t)n * S), codes1((size_t)n * S), act((size_t)n * S),
      opp((size_t)n * S);
  std::vector<int32_t> res(n), res1(n);
  std::vector<float> rew(n);
  std::vector<uint8_t> done(n);
  env.reset_codes(codes.data(), res.data());
  env.reset_codes_p1(codes1.data(), res1.data());
  EpisodeLog log;
  std::mt19937 rng(7);
  for (int step = 0; step < 400; ++step) {
    for (auto& a : act) a = (uint16_t)(rng() & 0x3FFF);
    for (auto& a : opp) a = (uint16_t)(rng() & 0x3FFF);
    std::vector<std::thread> th;
    for (int w = 0; w < threads; ++w)
      th.emplace_back([&, w] {
        const int e0 = w * n / threads, e1 = (w + 1) * n / threads;
        env.step_range_codes_sp(e0, e1, act.data(), opp.data(), codes.data(), res.data(),
                                codes1.data(), res1.data(), rew.data(), done.data(), &log, 5);
      });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; ++i) CHECK(res[i] >= 0);
  }
  auto eps = log.drain();
  CHECK(!eps.empty());
  for (auto& e : eps) {
    CHECK(e.ep_step > 0 && e.ep_step <= 120);
    CHECK(e.env_index >= n / 2 ? e.opponent == 5 : e.opponent < 0);
  }
  std::printf("env ok (%zu episodes)\n", eps.size());
}

int main() {
  ring_test();
  seqlock_test();
  env_test();
  std::printf("host stress: all ok\n");
  return 0;
}
