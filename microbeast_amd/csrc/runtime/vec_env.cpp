#include "vec_env.h"

#include <algorithm>
#include <atomic>
#include <random>
#include <thread>

namespace mb {

VecEnv::VecEnv(int size, int n_envs, int max_steps, uint64_t seed, const std::vector<int>& bots,
               const float* rw, int env_index_base)
    : size_(size), base_(env_index_base) {
  for (int i = 0; i < n_envs; ++i) {
    int bot = bots.empty() ? (int)BOT_COAC : bots[i % bots.size()];
    sims_.emplace_back(new MicroRTSSim(size, max_steps, bot,
                                       seed * 1000003ull + (uint64_t)(env_index_base + i), rw));
  }
  ep_ret_.assign(n_envs, 0.f);
  ep_len_.assign(n_envs, 0);
}

void VecEnv::reset(uint32_t* obs, uint32_t* mask) {
  const size_t S = (size_t)size_ * size_;
  for (size_t i = 0; i < sims_.size(); ++i) {
    sims_[i]->reset();
    ep_ret_[i] = 0.f;
    ep_len_[i] = 0;
    if (obs) sims_[i]->write_obs(obs + i * S);
    if (mask) sims_[i]->write_mask(mask + i * S * kMaskWords);
  }
}

void VecEnv::step_range(int e0, int e1, int base, const uint8_t* actions, uint32_t* obs,
                        uint32_t* mask, float* reward, uint8_t* done, float* ep_return,
                        int32_t* ep_step, EpisodeLog* log) {
  const size_t S = (size_t)size_ * size_;
  for (int i = e0; i < e1; ++i) {
    const size_t j = (size_t)(i - base);
    bool d = false;
    float r = sims_[i]->step(actions + j * S * kActComps, &d, nullptr);
    ep_ret_[i] += r;
    ep_len_[i] += 1;
    if (ep_return) ep_return[j] = ep_ret_[i];
    if (ep_step) ep_step[j] = ep_len_[i];
    if (d) {
      if (log) log->push({ep_ret_[i], ep_len_[i], base_ + i, sims_[i]->winner(), -1 - sims_[i]->bot()});
      ep_ret_[i] = 0.f;
      ep_len_[i] = 0;
    }
    if (reward) reward[j] = r;
    if (done) done[j] = d ? 1 : 0;
    if (obs) sims_[i]->write_obs(obs + j * S);
    if (mask) sims_[i]->write_mask(mask + j * S * kMaskWords);
  }
}

void VecEnv::set_validate(bool on) {
  for (auto& s : sims_) s->set_validate(on);
}

void VecEnv::reset_codes(uint16_t* codes, int32_t* res) {
  const size_t S = (size_t)size_ * size_;
  for (size_t i = 0; i < sims_.size(); ++i) {
    sims_[i]->reset();
    ep_ret_[i] = 0.f;
    ep_len_[i] = 0;
    if (codes) sims_[i]->write_obs_codes(codes + i * S);
    if (res) res[i] = sims_[i]->resources(0);
  }
}

void VecEnv::write_codes(uint16_t* codes, int32_t* res) const {
  const size_t S = (size_t)size_ * size_;
  for (size_t i = 0; i < sims_.size(); ++i) {
    sims_[i]->write_obs_codes(codes + i * S);
    res[i] = sims_[i]->resources(0);
  }
}

namespace {
// one draw per action component, uniform over the legal choices of the cell's 78-bit mask
void uniform_legal(const uint32_t* mask, int S, std::mt19937_64& rng, uint8_t* act) {
  for (int c = 0; c < S; ++c) {
    const uint32_t* m = mask + (size_t)c * kMaskWords;
    uint8_t* a = act + (size_t)c * kActComps;
    if ((m[0] | m[1] | m[2]) == 0) {  // no own idle unit here (almost every cell)
      for (int k = 0; k < kActComps; ++k) a[k] = 0;
      continue;
    }
    for (int k = 0; k < kActComps; ++k) {
      int cand[49], n = 0;
      for (int j = 0; j < kNvec[k]; ++j) {
        const int b = kNvecOff[k] + j;
        if ((m[b >> 5] >> (b & 31)) & 1u) cand[n++] = j;
      }
      a[k] = n ? (uint8_t)cand[rng() % (uint64_t)n] : 0;
    }
  }
}
}  // namespace

int64_t VecEnv::preroll(int max_pre, uint64_t seed, int n_threads) {
  if (max_pre <= 1 || sims_.empty()) return 0;
  const int n = (int)sims_.size(), S = size_ * size_;
  std::atomic<int> next{0};
  std::atomic<int64_t> played{0};
  auto work = [&]() {
    std::vector<uint32_t> m(S * kMaskWords), m1(S * kMaskWords);
    std::vector<uint8_t> a(S * kActComps), a1(S * kActComps);
    for (int i; (i = next.fetch_add(1)) < n;) {
      std::mt19937_64 rng(seed * 0x9E3779B97F4A7C15ull + (uint64_t)(base_ + i));
      const int r = (int)(rng() % (uint64_t)max_pre);
      MicroRTSSim& sim = *sims_[i];
      for (int t = 0; t < r; ++t) {
        sim.write_mask(m.data());
        uniform_legal(m.data(), S, rng, a.data());
        if (sim.external_opponent()) {
          sim.write_mask_p1(m1.data());
          uniform_legal(m1.data(), S, rng, a1.data());
          sim.set_opponent_actions(a1.data());
        }
        bool d = false;
        sim.step(a.data(), &d, nullptr);
      }
      // the preroll's uniform-policy play is not the policy's: the first logged episode of a
      // prerolled env counts reward and steps from the hand-off on only
      ep_ret_[i] = 0.f;
      ep_len_[i] = 0;
      played.fetch_add(r);
    }
  };
  const int nt = std::max(1, std::min(n_threads, n));
  std::vector<std::thread> th;
  for (int k = 1; k < nt; ++k) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return played.load();
}

void VecEnv::reset_codes_p1(uint16_t* codes_p1, int32_t* res_p1) const {
  const size_t S = (size_t)size_ * size_;
  for (size_t i = 0; i < sims_.size(); ++i) {
    if (!sims_[i]->external_opponent()) continue;
    sims_[i]->write_obs_codes_as(1, codes_p1 + i * S);
    res_p1[i] = sims_[i]->resources(1);
  }
}

void VecEnv::step_range_codes(int e0, int e1, const uint16_t* actions, uint16_t* codes,
                              int32_t* res, float* reward, uint8_t* done, EpisodeLog* log,
                              float* ep_return, int32_t* ep_step) {
  const size_t S = (size_t)size_ * size_;
  for (int i = e0; i < e1; ++i) {
    // two envs ahead: the sim object; one ahead: its unit list and grid
    if (i + 2 < e1) __builtin_prefetch(sims_[i + 2].get());
    if (i + 1 < e1) {
      sims_[i + 1]->prefetch();
      for (size_t o = 0; o < S * 2; o += 64) {  // next env's action row + codes row (write)
        __builtin_prefetch((const char*)(actions + (i + 1) * S) + o);
        __builtin_prefetch((char*)(codes + (i + 1) * S) + o, 1);
      }
    }
    bool d = false;
    const float r = sims_[i]->step_packed(actions + (size_t)i * S, &d);
    ep_ret_[i] += r;
    ep_len_[i] += 1;
    if (ep_return) ep_return[i] = ep_ret_[i];
    if (ep_step) ep_step[i] = ep_len_[i];
    if (d) {
      if (log) log->push({ep_ret_[i], ep_len_[i], base_ + i, sims_[i]->winner(), -1 - sims_[i]->bot()});
      ep_ret_[i] = 0.f;
      ep_len_[i] = 0;
    }
    reward[i] = r;
    done[i] = d ? 1 : 0;
    sims_[i]->write_obs_codes(codes + (size_t)i * S);
    res[i] = sims_[i]->resources(0);
  }
}

void VecEnv::write_code_lists(uint32_t* lists, int stride, int player) const {
  for (size_t i = 0; i < sims_.size(); ++i) {
    if (player != 0 && !sims_[i]->external_opponent()) continue;
    uint32_t* row = lists + i * (size_t)stride;
    const int n = sims_[i]->write_obs_code_list(row + 1, nullptr, player);
    row[0] = (uint32_t)n | ((uint32_t)sims_[i]->resources(player) << 16);
  }
}

int VecEnv::step_range_lists_sp(int e0, int e1, const uint32_t* act_lists,
                                const uint32_t* opp_lists, uint32_t* code_lists,
                                uint32_t* code_lists_p1, int stride, float* reward, uint8_t* done,
                                EpisodeLog* log, int opponent) {
  const size_t S = (size_t)size_ * size_;
  thread_local std::vector<uint16_t> dense, dense_opp;  // listed actions as cell rows
  dense.assign(S, 0);
  dense_opp.assign(S, 0);
  auto expand = [&](const uint32_t* row, std::vector<uint16_t>& out, uint16_t keep) {
    const uint32_t na = std::min<uint32_t>(row[0] & 0xFFFFu, (uint32_t)S);
    for (uint32_t k = 1; k <= na; ++k) {
      const uint32_t c = row[k] & 0xFFFFu;
      if (c < S) out[c] = keep ? (uint16_t)(row[k] >> 16) : 0;
    }
  };
  int idle = 0;
  for (int i = e0; i < e1; ++i) {
    if (i + 1 < e1) sims_[i + 1]->prefetch();
    MicroRTSSim& sim = *sims_[i];
    const bool sp = sim.external_opponent();
    const uint32_t* arow = act_lists + (size_t)i * stride;
    const uint32_t* orow = opp_lists + (size_t)i * stride;
    expand(arow, dense, 1);
    if (sp) expand(orow, dense_opp, 1);
    bool d = false;
    uint32_t* crow = code_lists + (size_t)i * stride;
    int n = 0;
    const float r = sp ? sim.step_packed2_list(dense.data(), dense_opp.data(), &d, crow + 1, &n, &idle)
                       : sim.step_packed_list(dense.data(), &d, crow + 1, &n, &idle);
    expand(arow, dense, 0);  // back to all-noop for the next env
    if (sp) expand(orow, dense_opp, 0);
    ep_ret_[i] += r;
    ep_len_[i] += 1;
    if (d) {
      if (log) log->push({ep_ret_[i], ep_len_[i], base_ + i, sim.winner(),
                          sp ? opponent : -1 - sim.bot()});
      ep_ret_[i] = 0.f;
      ep_len_[i] = 0;
    }
    reward[i] = r;
    done[i] = d ? 1 : 0;
    crow[0] = (uint32_t)n | ((uint32_t)sim.resources(0) << 16);
    if (sp) {
      uint32_t* prow = code_lists_p1 + (size_t)i * stride;
      const int n1 = sim.write_obs_code_list(prow + 1, nullptr, 1);
      prow[0] = (uint32_t)n1 | ((uint32_t)sim.resources(1) << 16);
    }
  }
  return idle;
}

int VecEnv::step_range_lists(int e0, int e1, const uint32_t* act_lists, uint32_t* code_lists,
                             int stride, float* reward, uint8_t* done, EpisodeLog* log) {
  const size_t S = (size_t)size_ * size_;
  int idle = 0;
  thread_local std::vector<uint16_t> dense;  // the listed actions expanded to a cell row
  dense.assign(S, 0);
  for (int i = e0; i < e1; ++i) {
    if (i + 2 < e1) __builtin_prefetch(sims_[i + 2].get());
    if (i + 1 < e1) {
      sims_[i + 1]->prefetch();
      __builtin_prefetch(act_lists + (size_t)(i + 1) * stride);
    }
    const uint32_t* arow = act_lists + (size_t)i * stride;
    const uint32_t na = std::min<uint32_t>(arow[0] & 0xFFFFu, (uint32_t)S);
    for (uint32_t k = 1; k <= na; ++k) {
      const uint32_t c = arow[k] & 0xFFFFu;
      if (c < S) dense[c] = (uint16_t)(arow[k] >> 16);
    }
    bool d = false;
    uint32_t* crow = code_lists + (size_t)i * stride;
    int n = 0;
    const float r = sims_[i]->step_packed_list(dense.data(), &d, crow + 1, &n, &idle);
    for (uint32_t k = 1; k <= na; ++k) {  // back to all-noop for the next env
      const uint32_t c = arow[k] & 0xFFFFu;
      if (c < S) dense[c] = 0;
    }
    ep_ret_[i] += r;
    ep_len_[i] += 1;
    if (d) {
      if (log) log->push({ep_ret_[i], ep_len_[i], base_ + i, sims_[i]->winner(), -1 - sims_[i]->bot()});
      ep_ret_[i] = 0.f;
      ep_len_[i] = 0;
    }
    reward[i] = r;
    done[i] = d ? 1 : 0;
    crow[0] = (uint32_t)n | ((uint32_t)sims_[i]->resources(0) << 16);
  }
  return idle;
}

void VecEnv::step_range_codes_sp(int e0, int e1, const uint16_t* actions,
                                 const uint16_t* opp_actions, uint16_t* codes, int32_t* res,
                                 uint16_t* codes_p1, int32_t* res_p1, float* reward,
                                 uint8_t* done, EpisodeLog* log, int opponent,
                                 float* ep_return, int32_t* ep_step) {
  const size_t S = (size_t)size_ * size_;
  for (int i = e0; i < e1; ++i) {
    if (i + 2 < e1) __builtin_prefetch(sims_[i + 2].get());
    if (i + 1 < e1) sims_[i + 1]->prefetch();
    MicroRTSSim& sim = *sims_[i];
    const bool sp = sim.external_opponent();
    bool d = false;
    const float r = sp ? sim.step_packed2(actions + (size_t)i * S, opp_actions + (size_t)i * S, &d)
                       : sim.step_packed(actions + (size_t)i * S, &d);
    ep_ret_[i] += r;
    ep_len_[i] += 1;
    if (ep_return) ep_return[i] = ep_ret_[i];
    if (ep_step) ep_step[i] = ep_len_[i];
    if (d) {
      if (log) log->push({ep_ret_[i], ep_len_[i], base_ + i, sim.winner(), sp ? opponent : -1 - sim.bot()});
      ep_ret_[i] = 0.f;
      ep_len_[i] = 0;
    }
    reward[i] = r;
    done[i] = d ? 1 : 0;
    sim.write_obs_codes(codes + (size_t)i * S);
    res[i] = sim.resources(0);
    if (sp) {
      sim.write_obs_codes_as(1, codes_p1 + (size_t)i * S);
      res_p1[i] = sim.resources(1);
    }
  }
}

void VecEnv::set_external_opponent(int e0, int e1, bool on) {
  for (int i = e0; i < e1; ++i) sims_[i]->set_external_opponent(on);
}

void VecEnv::dense_obs(float* out) const {
  const size_t S = (size_t)size_ * size_;
  for (size_t i = 0; i < sims_.size(); ++i) sims_[i]->write_obs_dense(out + i * S * kPlanes);
}

void VecEnv::dense_mask(uint8_t* out) const {
  const size_t S = (size_t)size_ * size_;
  for (size_t i = 0; i < sims_.size(); ++i) sims_[i]->write_mask_dense(out + i * S * kMaskBits);
}

}  // namespace mb
