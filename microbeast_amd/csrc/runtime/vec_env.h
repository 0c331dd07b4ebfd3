// Vectorised synthetic microRTS env: n independent simulators stepped in one
// call (the analogue of one MicroRTSGridModeVecEnv instance,
// reference libs/utils.py:64-75), with episode accounting that the reference
// did in Python (env_packer.py:55-100) done natively and with correct dtypes
// (float return, int32 length — fixes the uint8 wrap of env_packer.py:35-37).
#pragma once
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>
#include "../env/microrts_sim.h"

namespace mb {

struct EpisodeRecord {
  float ep_return;
  int32_t ep_step;
  int32_t env_index;
  int32_t winner;
  int32_t opponent;  // league opponent id (self-play env) or -1 - bot id (scripted bot)
};

class EpisodeLog {
 public:
  void push(const EpisodeRecord& r) {
    std::lock_guard<std::mutex> g(m_);
    recs_.push_back(r);
    ++total_;
  }
  std::vector<EpisodeRecord> drain() {
    std::lock_guard<std::mutex> g(m_);
    std::vector<EpisodeRecord> out;
    out.swap(recs_);
    return out;
  }
  int64_t total() const { return total_; }

 private:
  std::mutex m_;
  std::vector<EpisodeRecord> recs_;
  int64_t total_ = 0;
};

class VecEnv {
 public:
  VecEnv(int size, int n_envs, int max_steps, uint64_t seed, const std::vector<int>& bots,
         const float* reward_weight, int env_index_base = 0);
  int num_envs() const { return (int)sims_.size(); }
  int size() const { return size_; }
  // Compact I/O (see microrts_sim.h). Pointers cover all envs, env-major.
  void reset(uint32_t* obs, uint32_t* mask);
  // Steps envs [e0, e1). All I/O pointers address env `base` at offset 0, so
  // callers can pass either whole-vector buffers (base = 0) or group-local
  // staging (base = first env of the group).
  void step_range(int e0, int e1, int base, const uint8_t* actions, uint32_t* obs,
                  uint32_t* mask, float* reward, uint8_t* done, float* ep_return,
                  int32_t* ep_step, EpisodeLog* log);
  // GPU-engine fast path (16-bit cell codes + per-env resources out, packed 16-bit env
  // actions in, no CPU mask): 0.5 KB H2D + 0.5 KB D2H per 16x16 env step.
  void set_validate(bool on);
  void reset_codes(uint16_t* codes, int32_t* res);
  // current player-1 codes / resources of the self-play envs (after reset_codes)
  void reset_codes_p1(uint16_t* codes_p1, int32_t* res_p1) const;
  // ep_return / ep_step (optional, per env): running episode return / length after the step
  // (before the reset of a finished episode), the reference's Env_Packer keys
  void step_range_codes(int e0, int e1, const uint16_t* actions, uint16_t* codes, int32_t* res,
                        float* reward, uint8_t* done, EpisodeLog* log,
                        float* ep_return = nullptr, int32_t* ep_step = nullptr);
  // Sparse PCIe form (fused acting step, zero-copy): per env a row of `stride` uint32 words,
  // word 0 = n | resources << 16, then n entries cell | value << 16. Codes out: the occupied
  // cells; actions in: the cells with a non-noop action (a cell not listed no-ops).
  // player 1: the self-play envs' opponent rows (mirrored frame; other envs untouched)
  void write_code_lists(uint32_t* lists, int stride, int player = 0) const;
  // Returns the agent's idle units over the range (the cells the next policy step samples).
  int step_range_lists(int e0, int e1, const uint32_t* act_lists, uint32_t* code_lists,
                       int stride, float* reward, uint8_t* done, EpisodeLog* log);
  // Self-play form: envs with an external opponent also take its sparse action rows
  // (opp_lists, its mirrored frame) and emit its code rows (code_lists_p1); their finished
  // episodes are tagged with `opponent`.
  int step_range_lists_sp(int e0, int e1, const uint32_t* act_lists, const uint32_t* opp_lists,
                          uint32_t* code_lists, uint32_t* code_lists_p1, int stride,
                          float* reward, uint8_t* done, EpisodeLog* log, int opponent);
  // Self-play variant: envs with an external opponent also take its packed actions
  // (opp_actions, its mirrored frame) and emit its codes / resources; their finished
  // episodes are tagged with `opponent` (the league snapshot that was playing).
  void step_range_codes_sp(int e0, int e1, const uint16_t* actions, const uint16_t* opp_actions,
                           uint16_t* codes, int32_t* res, uint16_t* codes_p1, int32_t* res_p1,
                           float* reward, uint8_t* done, EpisodeLog* log, int opponent,
                           float* ep_return = nullptr, int32_t* ep_step = nullptr);
  void set_external_opponent(int e0, int e1, bool on);
  // Desynchronise the envs (bench.py / --preroll): env i plays r_i ~ U[0, max_pre) steps of
  // the random-init agent's policy -- every action component uniform over its legal choices
  // (actor gain 0, reference model.py:136) -- and of the same policy for a self-play opponent,
  // with auto-reset, so a measurement starts from a spread of game phases instead of every env
  // at its first frame. Needs the CPU masks (set_validate(true)); finished episodes are not
  // logged, running returns / lengths carry over. Returns the env steps played.
  int64_t preroll(int max_pre, uint64_t seed, int n_threads);
  // current codes / resources of every env (no reset)
  void write_codes(uint16_t* codes, int32_t* res) const;
  // Dense reference layout for parity tools: obs f32 (n,s,s,27), mask u8 (n,s*s*78)
  void dense_obs(float* out) const;
  void dense_mask(uint8_t* out) const;
  MicroRTSSim& sim(int i) { return *sims_[i]; }
  const std::vector<float>& ep_return() const { return ep_ret_; }
  const std::vector<int32_t>& ep_step() const { return ep_len_; }

 private:
  int size_;
  int base_;
  std::vector<std::unique_ptr<MicroRTSSim>> sims_;
  std::vector<float> ep_ret_;
  std::vector<int32_t> ep_len_;
};

}  // namespace mb
