// Per-env-step CPU cost of the simulator on the engine's fast path (packed actions in, sparse
// code rows out, no CPU mask), under two agent policies:
//   uniform  -- every component uniform over its legal choices (the random-init policy)
//   producer -- a trained-like policy: bases / barracks produce, workers harvest and return,
//               everyone attacks what is in range, else a random legal action
// Masks for the agent's choice come from a separate validating copy of each sim's rules
// (write_mask), outside the timed region.
//   g++ -O3 -std=c++17 -I.. env_bench.cpp ../env/microrts_sim.cpp -o /tmp/env_bench
//   /tmp/env_bench [size=16] [envs=2048] [steps=400] [policy=producer|uniform]
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
  const int bots[6] = {BOT_COAC, BOT_COAC, BOT_COAC, BOT_RANDOM_BIASED, BOT_LIGHT_RUSH,
                       BOT_WORKER_RUSH};
  std::vector<MicroRTSSim*> sims;
  for (int i = 0; i < E; ++i) {
    sims.push_back(new MicroRTSSim(s, 2000, bots[i % 6], 1000 + i, nullptr));
    sims.back()->set_validate(true);  // masks for the agent's choice (not the engine's path)
  }
  std::mt19937_64 rng(3);
  std::vector<uint32_t> mask(S * 3), rows(S + 1);
  std::vector<uint16_t> act(S);
  double t_step = 0, t_rows = 0;
  long long n_steps = 0, units = 0, idle = 0;
  for (int t = 0; t < T; ++t) {
    for (int i = 0; i < E; ++i) {
      MicroRTSSim& sim = *sims[i];
      sim.write_mask(mask.data());
      std::fill(act.begin(), act.end(), (uint16_t)0);
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
        act[c] = mbr::pack_env_action(a);
      }
      sim.set_validate(false);  // the engine's path: no CPU mask in the timed step
      bool d = false;
      const auto t0 = std::chrono::steady_clock::now();
      sim.step_packed(act.data(), &d);
      const auto t1 = std::chrono::steady_clock::now();
      int id = 0;
      const int n = sim.write_obs_code_list(rows.data() + 1, &id);
      const auto t2 = std::chrono::steady_clock::now();
      sim.set_validate(true);
      if (t >= T / 4) {  // past the opening: units spread, bases producing
        t_step += std::chrono::duration<double, std::nano>(t1 - t0).count();
        t_rows += std::chrono::duration<double, std::nano>(t2 - t1).count();
        ++n_steps;
        units += n;
        idle += id;
      }
    }
  }
  std::printf("size %d envs %d steps %d policy %s: step %.0f ns + rows %.0f ns per env step; "
              "%.1f occupied cells, %.2f idle own units per env\n",
              s, E, T, producer ? "producer" : "uniform", t_step / n_steps, t_rows / n_steps,
              (double)units / n_steps, (double)idle / n_steps);
  return 0;
}
