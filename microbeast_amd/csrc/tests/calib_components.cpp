// Where a uniform-random agent's episode return comes from in the stand-in, per scripted bot:
// plays the reference's initial policy (every component uniform over its legal choices, as
// tools/calibrate_env.py) and sums the six raw reward components per episode.
//   g++ -O2 -std=c++17 -I.. calib_components.cpp ../env/microrts_sim.cpp -o /tmp/calib
//   /tmp/calib [size=8] [episodes per bot=300] [max_steps=2000]
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../env/microrts_sim.h"

using namespace mb;

static bool bit(const uint32_t* w, int j) { return (w[j >> 5] >> (j & 31)) & 1u; }

int main(int argc, char** argv) {
  const int s = argc > 1 ? std::atoi(argv[1]) : 8;
  const int want = argc > 2 ? std::atoi(argv[2]) : 300;
  const float rw[6] = {10, 1, 1, 0.2f, 1, 4};
  const char* names[4] = {"coac", "random_biased", "light_rush", "worker_rush"};
  std::mt19937_64 rng(7);
  for (int bot = 0; bot < 4; ++bot) {
    MicroRTSSim sim(s, argc > 3 ? std::atoi(argv[3]) : 2000, bot, 1234 + bot, rw);
    sim.reset();
    const int S = s * s;
    std::vector<uint32_t> mask(S * 3);
    std::vector<uint8_t> act(S * 7);
    double comp[6] = {0, 0, 0, 0, 0, 0}, ep_comp[6] = {0, 0, 0, 0, 0, 0};
    double ret = 0, ep_ret = 0, len = 0, ge10 = 0, wins = 0;
    int ep = 0, t = 0, base_dead = -1;
    double base_t = 0, tail = 0;
    while (ep < want) {
      sim.write_mask(mask.data());
      for (int c = 0; c < S; ++c) {
        const uint32_t* m = &mask[c * 3];
        for (int k = 0; k < 7; ++k) {
          int cand[49], n = 0;
          for (int j = 0; j < kNvec[k]; ++j)
            if (bit(m, kNvecOff[k] + j)) cand[n++] = j;
          act[c * 7 + k] = n ? (uint8_t)cand[rng() % n] : 0;
        }
      }
      bool done = false;
      float raw[6];
      const float r = sim.step(act.data(), &done, raw);
      ep_ret += r;
      for (int i = 0; i < 6; ++i) ep_comp[i] += raw[i];
      ++t;
      if (base_dead < 0 && !done && sim.count_units(0, BASE) == 0) base_dead = t;
      if (done) {
        const int bd = base_dead < 0 ? t : base_dead;
        base_t += bd;
        tail += t - bd;
        base_dead = -1;
        ret += ep_ret;
        len += t;
        ge10 += ep_ret >= 10.f;
        wins += ep_comp[0] > 0;
        for (int i = 0; i < 6; ++i) comp[i] += ep_comp[i];
        ep_ret = 0;
        t = 0;
        for (double& v : ep_comp) v = 0;
        ++ep;
      }
    }
    std::printf("%-14s len %6.1f return %6.2f ge10 %5.1f%% win %4.1f%% | per episode: win/loss %.2f "
                "res %.2f worker %.2f build %.2f attack %.2f combat %.2f | base dies %.0f, then %.0f\n",
                names[bot], len / ep, ret / ep, 100 * ge10 / ep, 100 * wins / ep, comp[0] / ep,
                comp[1] / ep, comp[2] / ep, comp[3] / ep, comp[4] / ep, comp[5] / ep, base_t / ep,
                tail / ep);
  }
  return 0;
}
