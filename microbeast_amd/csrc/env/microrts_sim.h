// Synthetic gym-microRTS (GridMode) simulator — native C++.
//
// The reference drives the Java microRTS engine through JPype
// (reference: libs/utils.py:59-76 create_env, env_packer.py:17-111 Env_Packer).
// That engine is not available offline, so this file re-creates the *tensor
// contract* of MicroRTSGridModeVecEnv as used by the reference:
//   obs    (n, s, s, 27) one-hot planes  hp(5) res(5) owner(3) type(8) action(6)
//   mask   (n, s*s, 78)  per cell: type(6) move(4) harvest(4) return(4)
//                        produce-dir(4) produce-type(7) attack-target(49)
//   action (n, s*s, 7)   per cell component indices, nvec=[6,4,4,4,4,7,49]
//   reward weighted by [win/loss, resource, worker, building, attack, combat]
//   (libs/utils.py:74 reward_weight = [10,1,1,0.2,1,4])
// with scripted opponents standing in for coacAI / randomBiasedAI /
// lightRushAI / workerRushAI (libs/utils.py:69-72).
//
// Compact layouts (what the GPU path ships over PCIe):
//   obs  : uint32 per cell, bit p set <=> plane p is hot   (4 B/cell)
//   mask : 3 x uint32 per cell, bit j of the 96-bit word = mask[j] (12 B/cell)
//   action: uint8 per component (7 B/cell)
#pragma once
#include <cstdint>
#include <vector>
#include <string>

namespace mb {

constexpr int kPlanes = 27;
constexpr int kMaskBits = 78;
constexpr int kMaskWords = 3;
constexpr int kActComps = 7;
constexpr int kNvec[kActComps] = {6, 4, 4, 4, 4, 7, 49};
constexpr int kNvecOff[kActComps + 1] = {0, 6, 10, 14, 18, 22, 29, 78};
constexpr int kNumRewards = 6;

enum UnitType : int8_t { NONE = 0, RESOURCE = 1, BASE = 2, BARRACKS = 3, WORKER = 4,
                         LIGHT = 5, HEAVY = 6, RANGED = 7 };
enum ActType : int8_t { A_NOOP = 0, A_MOVE = 1, A_HARVEST = 2, A_RETURN = 3,
                        A_PRODUCE = 4, A_ATTACK = 5 };
enum Bot : int8_t { BOT_COAC = 0, BOT_RANDOM_BIASED = 1, BOT_LIGHT_RUSH = 2,
                    BOT_WORKER_RUSH = 3, BOT_PASSIVE = 4, BOT_RANDOM = 5 };

struct Unit {
  int16_t x, y;
  int8_t type;
  int8_t owner;     // -1 resource, 0 agent, 1 opponent
  int16_t hp;
  int16_t res;      // resource amount (resource unit) or carried amount (worker)
  int16_t busy;     // remaining ticks of current action
  int8_t act;       // current action type (ActType)
  int8_t alive;
};

struct SimStats {  // accumulated per episode, read by the packer
  float ep_return = 0.f;
  int32_t ep_step = 0;
};

class MicroRTSSim {
 public:
  MicroRTSSim(int size, int max_steps, int bot, uint64_t seed,
              const float* reward_weight /*6 or null*/);
  void reset();
  // actions: s*s*7 uint8 (cell-major). Returns weighted reward; sets done.
  // Auto-resets on done (vec-env semantics): the observation written next is
  // the first frame of the new episode.
  float step(const uint8_t* actions, bool* done, float* raw_rewards /*6 or null*/);
  void write_obs(uint32_t* out) const;      // s*s words
  void write_mask(uint32_t* out) const;     // s*s*3 words (valid after reset/step)
  // Dense reference-compatible outputs.
  void write_obs_dense(float* out) const;   // s*s*27
  void write_mask_dense(uint8_t* out) const;// s*s*78
  int size() const { return s_; }
  // Software prefetch of the per-step working set (unit list + occupancy grid): the
  // vec-env steps thousands of sims whose state is cold in cache, and the step is a
  // chain of dependent misses otherwise
  void prefetch() const {
    const char* u = (const char*)units_.data();
    for (size_t o = 0; o < units_.size() * sizeof(Unit); o += 64) __builtin_prefetch(u + o);
    const char* g = (const char*)grid_.data();
    for (size_t o = 0; o < grid_.size() * sizeof(int16_t); o += 64) __builtin_prefetch(g + o);
  }
  int bot() const { return bot_; }
  void set_bot(int b) { bot_ = b; }
  int winner() const { return last_winner_; }
  int ticks() const { return tick_; }
  // Self-play: opponent actions supplied externally (player-1 perspective,
  // coordinates mirrored so the same network can drive either side).
  void set_external_opponent(bool on) {
    external_opp_ = on;
    if (on && validate_) compute_mask(1, mask_p1_);
  }
  void write_obs_p1(uint32_t* out) const;
  void write_mask_p1(uint32_t* out) const;
  void set_opponent_actions(const uint8_t* actions_p1);
  // GPU-engine fast path: 16-bit cell codes out, 16-bit packed env actions in, and no
  // CPU-side mask (the GPU derives it from the codes + resources, see
  // include/microrts_rules.h); exec() still validates every action's feasibility.
  void set_validate(bool on) {
    validate_ = on;
    if (on) {
      compute_mask(0, mask_);
      if (external_opp_) compute_mask(1, mask_p1_);
    }
  }
  float step_packed(const uint16_t* env_actions, bool* done);
  // step_packed + write_obs_code_list(entries, idle_own) (player 0) in the step's last pass over
  // the units; *n = the entries written
  float step_packed_list(const uint16_t* env_actions, bool* done, uint32_t* entries, int* n,
                         int* idle_own);
  float step_packed2_list(const uint16_t* env_actions, const uint16_t* opp_actions, bool* done,
                          uint32_t* entries, int* n, int* idle_own);
  // self-play fast path: both players' packed actions, each in its own frame
  float step_packed2(const uint16_t* env_actions, const uint16_t* opp_actions, bool* done);
  void write_obs_codes(uint16_t* out) const { write_obs_codes_as(0, out); }
  // sparse form of write_obs_codes for the fused acting step's PCIe-light input: the occupied
  // cells only, entry = cell | code << 16, into entries[0 .. n); returns n (<= cells).
  // *idle_own (optional) += the agent's idle units: the cells the sparse head samples.
  // player 1: its mirrored frame (write_obs_codes_as), for the self-play opponent's policy
  int write_obs_code_list(uint32_t* entries, int* idle_own = nullptr, int player = 0) const;
  // codes from `player`'s perspective (player 1: mirrored frame, owner 1 = itself)
  void write_obs_codes_as(int player, uint16_t* out) const;
  bool external_opponent() const { return external_opp_; }
  int resources(int player) const { return resources_[player]; }
  int count_units(int owner, int type) const {  // alive units of owner (0/1), type (< 0: all)
    if (owner < 0 || owner > 1) {
      int n = 0;
      for (const Unit& u : units_) n += u.alive && u.owner == owner && (type < 0 || u.type == type);
      return n;
    }
    if (type >= 0) return cnt_[owner][type];
    int n = 0;
    for (int t = 0; t < 8; ++t) n += cnt_[owner][t];
    return n;
  }

 private:
  int s_, max_steps_, bot_;
  uint64_t rng_;
  float rw_[kNumRewards];
  int tick_ = 0;
  int resources_[2] = {0, 0};
  int last_winner_ = -1;
  bool external_opp_ = false;
  bool validate_ = true;
  std::vector<uint8_t> act_buf_;
  std::vector<Unit> units_;
  std::vector<int16_t> grid_;     // unit index per cell, -1 empty
  std::vector<uint32_t> mask_;    // cached agent mask (s*s*3)
  std::vector<uint32_t> mask_p1_; // cached opponent mask (for self-play / validation)
  std::vector<uint8_t> opp_actions_;
  int cnt_[2][8] = {};            // alive units per owner (0 / 1) and type, kept by add / kill
  const uint16_t* p16_ = nullptr;    // step_packed: agent actions decoded lazily per cell
  const uint16_t* opp16_ = nullptr;  // step_packed2: opponent's packed actions
  uint32_t* rows_out_ = nullptr;     // step_packed_list: the sparse row's entries
  int rows_n_ = 0, rows_idle_ = 0;   // ... and its length / the agent's idle units
  int last_add_ = -1;                // slot of the last add_unit (bot_act's worker index)

  uint32_t rand_u32();
  float rand_unit();
  int cell(int x, int y) const { return y * s_ + x; }
  // sparse-row entry of a unit from `player`'s side: cell | code << 16 (player 1: mirrored;
  // the code is include/microrts_rules.h cell_code)
  uint32_t row_entry(const Unit& u, int player) const {
    const int px = player ? s_ - 1 - u.x : u.x, py = player ? s_ - 1 - u.y : u.y;
    const int own = u.owner < 0 ? 0 : (u.owner == player ? 1 : 2);
    const int hp = u.hp < 0 ? 0 : (u.hp > 4 ? 4 : u.hp);
    const int res = u.res < 0 ? 0 : (u.res > 4 ? 4 : u.res);
    return (uint32_t)cell(px, py) |
           ((uint32_t)(hp | (res << 3) | (own << 6) | (u.type << 8) | (u.act << 11)) << 16);
  }
  bool in_bounds(int x, int y) const { return x >= 0 && y >= 0 && x < s_ && y < s_; }
  bool empty(int x, int y) const { return in_bounds(x, y) && grid_[cell(x, y)] < 0; }
  int add_unit(int type, int owner, int x, int y, int res = 0);
  void kill(int uid);
  void compute_mask(int player, std::vector<uint32_t>& out) const;
  void unit_mask(const Unit& u, int player, uint32_t* w) const;
  // Returns true if the action was valid and executed.
  bool exec(int uid, const uint8_t* a, float* rw);
  void bot_act(int player, float* rw_opp);
  void bot_unit(int uid, int player, float* rw_opp, int n_workers, int n_barracks, int widx);
  int nearest(int uid, int owner_filter, int type_filter, int* dist) const;
  int dir_toward(const Unit& u, int tx, int ty) const;
  void map_xy(int player, int x, int y, int* ox, int* oy) const;
};

// Unit parameters (ticks are env steps).
struct UnitSpec { int16_t hp, cost, damage, range, move_t, attack_t, produce_t; };
extern const UnitSpec kSpec[8];

}  // namespace mb
