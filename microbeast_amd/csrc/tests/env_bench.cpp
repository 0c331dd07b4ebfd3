// Per-env-step CPU cost of the simulator on the engine's fast path (packed actions in, sparse
// code rows out, no CPU mask), under two agent policies:
//   uniform  -- every component uniform over its legal choices (the random-init policy)
//   producer -- a trained-like policy: bases / barracks produce, workers harvest and return,
//               everyone attacks what is in range, else a random legal action
// Masks for the agent's choice come from a separate validating copy of each sim's rules
// (write_mask), outside the timed region.
//   g++ -O3 -std=c++17 -I.. env_bench.cpp ../env/microrts_sim.cpp -o /tmp/env_bench
//   /tmp/env_bench [size=16] [envs=2048] [steps=400] [policy=producer|uniform] [bot=-1 (mix)]
// The last line's hash (FNV-1a over every step's code rows, done flags and rewards) pins the
// games: a simulator optimisation must leave it unchanged.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../env/microrts_sim.h"
#include "../include/microrts_rules.h"

using namespace mb;

static bool bit(const uint32_t* w, int j) { return (w[j >> 5] >> (j & 31)) & 1u; }

static int pick(const uint32_t* m, int k, std::mt19937_64& rng) {
  int cand[49], n = 0;
  for (int j = 0; j < kNvec[k]; ++j)
    if (bit(m, kNvecOff[k] + j)) cand[n++] = j;
  return n ? cand[rng() % n] : 0;
}

int main(int argc, char** argv) {
  const int s = argc > 1 ? std::atoi(argv[1]) : 16;
  const int E = argc > 2 ? std::atoi(argv[2]) : 2048;
  const int T = argc > 3 ? std::atoi(argv[3]) : 400;
  const bool producer = !(argc > 4 && std::strcmp(argv[4], "uniform") == 0);
  const int S = s * s;
  const int only = argc > 5 ? std::atoi(argv[5]) : -1;
  const int bots[6] = {BOT_COAC, BOT_COAC, BOT_COAC, BOT_RANDOM_BIASED, BOT_LIGHT_RUSH,
                       BOT_WORKER_RUSH};
  std::vector<MicroRTSSim*> sims;
  for (int i = 0; i < E; ++i) {
    sims.push_back(new MicroRTSSim(s, 2000, only >= 0 ? only : bots[i % 6], 1000 + i, nullptr));
    sims.back()->set_validate(true);  // masks for the agent's choice (not the engine's path)
  }
  std::mt19937_64 rng(3);
  std::vector<uint32_t> mask(S * 3), rows((size_t)E * (S + 1));
  std::vector<uint16_t> act((size_t)E * S);
  std::vector<float> rew(E);
  std::vector<uint8_t> dn(E);
  double t_loop = 0;
  long long n_steps = 0, units = 0, idle = 0;
  uint64_t hash = 1469598103934665603ull;
  auto mix = [&](uint32_t v) { hash = (hash ^ v) * 1099511628211ull; };
  for (int t = 0; t < T; ++t) {
    for (int i = 0; i < E; ++i) {  // the agent's choices (untimed)
      MicroRTSSim& sim = *sims[i];
      sim.write_mask(mask.data());
      uint16_t* ar = &act[(size_t)i * S];
      std::fill(ar, ar + S, (uint16_t)0);
      for (int c = 0; c < S; ++c) {
        const uint32_t* m = &mask[c * 3];
        if (!(m[0] | m[1] | m[2])) continue;
        uint8_t a[7] = {0, 0, 0, 0, 0, 0, 0};
        for (int k = 1; k < 7; ++k) a[k] = (uint8_t)pick(m, k, rng);
        a[0] = (uint8_t)pick(m, 0, rng);
        if (producer) {
          if (bit(m, kNvecOff[0] + mbr::A_ATTACK)) a[0] = mbr::A_ATTACK;
          else if (bit(m, kNvecOff[0] + mbr::A_RETURN)) a[0] = mbr::A_RETURN;
          else if (bit(m, kNvecOff[0] + mbr::A_HARVEST)) a[0] = mbr::A_HARVEST;
          else if (bit(m, kNvecOff[0] + mbr::A_PRODUCE) && (rng() & 1)) a[0] = mbr::A_PRODUCE;
        }
        ar[c] = mbr::pack_env_action(a);
      }
      sim.set_validate(false);  // the engine's path: no CPU mask in the timed step
    }
    // timed: the engine worker's loop (VecEnv::step_range_lists): prefetch the next env's
    // state, step on the packed actions, write the sparse code row
    int id = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < E; ++i) {
      if (i + 2 < E) __builtin_prefetch(sims[i + 2]);
      if (i + 1 < E) sims[i + 1]->prefetch();
      bool d = false;
      uint32_t* row = &rows[(size_t)i * (S + 1)];
      int n = 0;
      rew[i] = sims[i]->step_packed_list(&act[(size_t)i * S], &d, row + 1, &n, &id);
      dn[i] = d;
      row[0] = (uint32_t)n;
    }
    const auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < E; ++i) {
      const uint32_t* row = &rows[(size_t)i * (S + 1)];
      for (uint32_t k = 0; k < row[0]; ++k) mix(row[1 + k]);
      mix((uint32_t)dn[i]);
      uint32_t rb;
      std::memcpy(&rb, &rew[i], 4);
      mix(rb);
      sims[i]->set_validate(true);
      if (t >= T / 4) units += row[0];
    }
    if (t >= T / 4) {  // past the opening: units spread, bases producing
      t_loop += std::chrono::duration<double, std::nano>(t1 - t0).count();
      n_steps += E;
      idle += id;
    }
  }
  std::printf("size %d envs %d steps %d policy %s: step + row %.0f ns per env step; "
              "%.1f occupied cells, %.2f idle own units per env\n",
              s, E, T, producer ? "producer" : "uniform", t_loop / n_steps,
              (double)units / n_steps, (double)idle / n_steps);
  std::printf("hash %016llx\n", (unsigned long long)hash);
  return 0;
}
