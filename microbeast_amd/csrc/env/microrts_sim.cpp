// Synthetic gym-microRTS simulator. See microrts_sim.h for the contract.
#include "microrts_sim.h"
#include "../include/microrts_rules.h"
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <stdexcept>

namespace mb {

// single source of truth shared with the GPU mask kernel (include/microrts_rules.h)
#define MB_SPEC(t)                                                                          \
  {(int16_t)mbr::spec_hp(t), (int16_t)mbr::spec_cost(t), (int16_t)mbr::spec_damage(t),      \
   (int16_t)mbr::spec_range(t), (int16_t)mbr::spec_move_t(t), (int16_t)mbr::spec_attack_t(t), \
   (int16_t)mbr::spec_produce_t(t)}
const UnitSpec kSpec[8] = {MB_SPEC(0), MB_SPEC(1), MB_SPEC(2), MB_SPEC(3),
                           MB_SPEC(4), MB_SPEC(5), MB_SPEC(6), MB_SPEC(7)};
#undef MB_SPEC
static constexpr int kHarvestT = mbr::kHarvestT, kReturnT = mbr::kReturnT;
static constexpr int kDX[4] = {0, 1, 0, -1};
static constexpr int kDY[4] = {-1, 0, 1, 0};

// reward component indices (libs/utils.py:74 order)
enum { R_WIN = 0, R_RES = 1, R_WORKER = 2, R_BUILD = 3, R_ATTACK = 4, R_COMBAT = 5 };

static inline void setbit(uint32_t* w, int j) { w[j >> 5] |= 1u << (j & 31); }
static inline bool getbit(const uint32_t* w, int j) { return (w[j >> 5] >> (j & 31)) & 1u; }

MicroRTSSim::MicroRTSSim(int size, int max_steps, int bot, uint64_t seed, const float* rw)
    : s_(size), max_steps_(max_steps), bot_(bot) {
  // maps up to 32x32: step()'s idle list and dir_toward's BFS live on the stack, and a cell
  // index fits the 16-bit fields of the sparse rows
  if (size < 1 || size > 32) throw std::invalid_argument("MicroRTSSim: map size must be 1..32");
  static const float def[kNumRewards] = {10.f, 1.f, 1.f, 0.2f, 1.f, 4.f};
  for (int i = 0; i < kNumRewards; ++i) rw_[i] = rw ? rw[i] : def[i];
  // splitmix64 seeding so neighbouring seeds give unrelated streams
  uint64_t z = seed + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  rng_ = (z ^ (z >> 31)) | 1ull;
  grid_.assign(s_ * s_, -1);
  act_buf_.assign((size_t)s_ * s_ * kActComps, 0);
  mask_.assign(s_ * s_ * kMaskWords, 0u);
  mask_p1_.assign(s_ * s_ * kMaskWords, 0u);
  opp_actions_.assign(s_ * s_ * kActComps, 0);
  reset();
}

uint32_t MicroRTSSim::rand_u32() {
  rng_ ^= rng_ << 13; rng_ ^= rng_ >> 7; rng_ ^= rng_ << 17;
  return (uint32_t)(rng_ >> 16);
}
float MicroRTSSim::rand_unit() { return (rand_u32() & 0xFFFFFF) * (1.f / 16777216.f); }

int MicroRTSSim::add_unit(int type, int owner, int x, int y, int res) {
  Unit u{};
  u.x = x; u.y = y; u.type = type; u.owner = owner;
  u.hp = kSpec[type].hp; u.res = res; u.busy = 0; u.act = A_NOOP; u.alive = 1;
  // reuse a dead slot when possible
  int uid = -1;
  for (size_t i = 0; i < units_.size(); ++i)
    if (!units_[i].alive) { uid = (int)i; break; }
  if (uid < 0) { uid = (int)units_.size(); units_.push_back(u); }
  else units_[uid] = u;
  grid_[cell(x, y)] = (int16_t)uid;
  if (owner >= 0) ++cnt_[owner][type];
  last_add_ = uid;
  return uid;
}

void MicroRTSSim::kill(int uid) {
  Unit& u = units_[uid];
  if (!u.alive) return;
  grid_[cell(u.x, u.y)] = -1;
  u.alive = 0;
  if (u.owner >= 0) --cnt_[u.owner][u.type];
}

// "maps/{s}x{s}/basesWorkers{s}x{s}.xml" stand-in (libs/utils.py:73): each
// player owns a base and a worker next to a resource field in opposite corners.
void MicroRTSSim::reset() {
  units_.clear();
  units_.reserve((size_t)s_ * s_ + 4);  // units never outnumber cells: no reallocation
  std::memset(cnt_, 0, sizeof(cnt_));
  std::fill(grid_.begin(), grid_.end(), (int16_t)-1);
  tick_ = 0;
  resources_[0] = resources_[1] = 5;
  const int o = s_ >= 8 ? 1 : 0;
  const int b = s_ >= 8 ? 2 : 1;
  // player 0 top-left, player 1 bottom-right (180 degree rotation)
  for (int p = 0; p < 2; ++p) {
    auto X = [&](int x) { return p == 0 ? x : s_ - 1 - x; };
    auto Y = [&](int y) { return p == 0 ? y : s_ - 1 - y; };
    add_unit(RESOURCE, -1, X(0), Y(0), s_ >= 8 ? 20 : 10);
    if (s_ >= 8) add_unit(RESOURCE, -1, X(0), Y(1), 20);
    add_unit(BASE, p, X(b), Y(b));
    add_unit(WORKER, p, X(o), Y(b == 1 ? 0 : o), 0);
    if (s_ >= 12) add_unit(WORKER, p, X(b + 1), Y(b), 0);
  }
  if (validate_) compute_mask(0, mask_);
  if (external_opp_ && validate_) compute_mask(1, mask_p1_);
}

// ---------------------------------------------------------------- masks
void MicroRTSSim::unit_mask(const Unit& u, int player, uint32_t* w) const {
  // w: 3 words, real-frame bits; caller mirrors for player 1 perspective.
  w[0] = w[1] = w[2] = 0;
  if (!u.alive || u.owner != player || u.busy > 0 || u.type == RESOURCE) return;
  const UnitSpec& sp = kSpec[u.type];
  setbit(w, kNvecOff[0] + A_NOOP);
  bool any_move = false, any_harv = false, any_ret = false, any_prod = false, any_att = false;
  const bool mobile = u.type >= WORKER;
  for (int d = 0; d < 4; ++d) {
    int nx = u.x + kDX[d], ny = u.y + kDY[d];
    if (!in_bounds(nx, ny)) continue;
    int g = grid_[cell(nx, ny)];
    if (g < 0) {
      if (mobile) { setbit(w, kNvecOff[1] + d); any_move = true; }
      // produce direction: any empty neighbour when something is affordable
      bool can_prod = false;
      if (u.type == BASE && resources_[player] >= kSpec[WORKER].cost) can_prod = true;
      if (u.type == BARRACKS && resources_[player] >= kSpec[LIGHT].cost) can_prod = true;
      if (u.type == WORKER && resources_[player] >= kSpec[BARRACKS].cost) can_prod = true;
      if (can_prod) { setbit(w, kNvecOff[4] + d); any_prod = true; }
    } else {
      const Unit& t = units_[g];
      if (u.type == WORKER && t.type == RESOURCE && u.res == 0 && t.res > 0) {
        setbit(w, kNvecOff[2] + d); any_harv = true;
      }
      if (u.type == WORKER && t.type == BASE && t.owner == player && u.res > 0) {
        setbit(w, kNvecOff[3] + d); any_ret = true;
      }
    }
  }
  if (any_prod) {
    const int r = resources_[player];
    if (u.type == BASE) setbit(w, kNvecOff[5] + (WORKER - 1));
    if (u.type == BARRACKS) {
      if (r >= kSpec[LIGHT].cost) setbit(w, kNvecOff[5] + (LIGHT - 1));
      if (r >= kSpec[HEAVY].cost) setbit(w, kNvecOff[5] + (HEAVY - 1));
      if (r >= kSpec[RANGED].cost) setbit(w, kNvecOff[5] + (RANGED - 1));
    }
    if (u.type == WORKER) {
      if (r >= kSpec[BASE].cost) setbit(w, kNvecOff[5] + (BASE - 1));
      if (r >= kSpec[BARRACKS].cost) setbit(w, kNvecOff[5] + (BARRACKS - 1));
    }
  }
  if (sp.damage > 0) {
    const int R = sp.range, Rs = std::min(R, 3);
    for (int ay = -Rs; ay <= Rs; ++ay)
      for (int ax = -Rs; ax <= Rs; ++ax) {
        if (ax * ax + ay * ay > R * R || (ax == 0 && ay == 0)) continue;
        int tx = u.x + ax, ty = u.y + ay;
        if (!in_bounds(tx, ty)) continue;
        int g = grid_[cell(tx, ty)];
        if (g >= 0 && units_[g].owner == 1 - player) {
          setbit(w, kNvecOff[6] + (ay + 3) * 7 + (ax + 3)); any_att = true;
        }
      }
  }
  if (any_move) setbit(w, kNvecOff[0] + A_MOVE);
  if (any_harv) setbit(w, kNvecOff[0] + A_HARVEST);
  if (any_ret) setbit(w, kNvecOff[0] + A_RETURN);
  if (any_prod) setbit(w, kNvecOff[0] + A_PRODUCE);
  if (any_att) setbit(w, kNvecOff[0] + A_ATTACK);
}

static void mirror_mask_bits(const uint32_t* in, uint32_t* out) {
  out[0] = out[1] = out[2] = 0;
  for (int j = 0; j < kMaskBits; ++j) {
    if (!getbit(in, j)) continue;
    int k = j;
    if (j >= kNvecOff[1] && j < kNvecOff[5]) {  // the four direction groups
      int g = (j - kNvecOff[1]) / 4, d = (j - kNvecOff[1]) % 4;
      k = kNvecOff[1] + g * 4 + (d + 2) % 4;
    } else if (j >= kNvecOff[6]) {
      int a = j - kNvecOff[6];
      k = kNvecOff[6] + (6 - a / 7) * 7 + (6 - a % 7);
    }
    setbit(out, k);
  }
}

void MicroRTSSim::map_xy(int player, int x, int y, int* ox, int* oy) const {
  if (player == 0) { *ox = x; *oy = y; }
  else { *ox = s_ - 1 - x; *oy = s_ - 1 - y; }
}

void MicroRTSSim::compute_mask(int player, std::vector<uint32_t>& out) const {
  std::fill(out.begin(), out.end(), 0u);
  for (const Unit& u : units_) {
    if (!u.alive || u.owner != player || u.busy > 0) continue;
    uint32_t w[3];
    unit_mask(u, player, w);
    int px, py;
    map_xy(player, u.x, u.y, &px, &py);
    uint32_t* dst = &out[(size_t)cell(px, py) * kMaskWords];
    if (player == 0) { dst[0] = w[0]; dst[1] = w[1]; dst[2] = w[2]; }
    else mirror_mask_bits(w, dst);
  }
}

// ---------------------------------------------------------------- actions
bool MicroRTSSim::exec(int uid, const uint8_t* a, float* rw) {
  Unit& u = units_[uid];
  if (!u.alive || u.busy > 0) return false;
  const int player = u.owner;
  const UnitSpec& sp = kSpec[u.type];
  switch (a[0]) {
    case A_NOOP: return true;
    case A_MOVE: {
      if (u.type < WORKER) return false;
      int d = a[1] & 3, nx = u.x + kDX[d], ny = u.y + kDY[d];
      if (!empty(nx, ny)) return false;
      grid_[cell(u.x, u.y)] = -1;
      u.x = nx; u.y = ny;
      grid_[cell(nx, ny)] = (int16_t)uid;
      u.busy = sp.move_t; u.act = A_MOVE;
      return true;
    }
    case A_HARVEST: {
      int d = a[2] & 3, nx = u.x + kDX[d], ny = u.y + kDY[d];
      if (u.type != WORKER || u.res > 0 || !in_bounds(nx, ny)) return false;
      int g = grid_[cell(nx, ny)];
      if (g < 0 || units_[g].type != RESOURCE || units_[g].res <= 0) return false;
      units_[g].res -= 1; u.res = 1;
      if (units_[g].res <= 0) kill(g);
      u.busy = kHarvestT; u.act = A_HARVEST;
      if (rw) rw[R_RES] += 1.f;
      return true;
    }
    case A_RETURN: {
      int d = a[3] & 3, nx = u.x + kDX[d], ny = u.y + kDY[d];
      if (u.type != WORKER || u.res <= 0 || !in_bounds(nx, ny)) return false;
      int g = grid_[cell(nx, ny)];
      if (g < 0 || units_[g].type != BASE || units_[g].owner != player) return false;
      resources_[player] += u.res; u.res = 0;
      u.busy = kReturnT; u.act = A_RETURN;
      if (rw) rw[R_RES] += 1.f;
      return true;
    }
    case A_PRODUCE: {
      int d = a[4] & 3, nx = u.x + kDX[d], ny = u.y + kDY[d];
      int t = (int)a[5] + 1;
      if (t < 1 || t > 7 || !empty(nx, ny)) return false;
      bool ok = (u.type == BASE && t == WORKER) ||
                (u.type == BARRACKS && (t == LIGHT || t == HEAVY || t == RANGED)) ||
                (u.type == WORKER && (t == BASE || t == BARRACKS));
      if (!ok || resources_[player] < kSpec[t].cost) return false;
      resources_[player] -= kSpec[t].cost;
      int nu = add_unit(t, player, nx, ny);
      Unit& uu = units_[uid];  // add_unit may reallocate
      units_[nu].busy = kSpec[t].produce_t;  // under construction: shown as "produce"
      units_[nu].act = A_PRODUCE;            // so busy > 0 <=> act != noop (GPU mask relies on it)
      uu.busy = kSpec[t].produce_t; uu.act = A_PRODUCE;
      if (rw) {
        if (t == WORKER) rw[R_WORKER] += 1.f;
        else if (t == BASE || t == BARRACKS) rw[R_BUILD] += 1.f;
        else rw[R_COMBAT] += 1.f;
      }
      return true;
    }
    case A_ATTACK: {
      if (sp.damage <= 0) return false;
      int ax = (int)(a[6] % 7) - 3, ay = (int)(a[6] / 7) - 3;
      if (ax * ax + ay * ay > sp.range * sp.range) return false;
      int tx = u.x + ax, ty = u.y + ay;
      if (!in_bounds(tx, ty)) return false;
      int g = grid_[cell(tx, ty)];
      if (g < 0 || units_[g].owner != 1 - player) return false;
      units_[g].hp -= sp.damage;
      if (units_[g].hp <= 0) kill(g);
      u.busy = sp.attack_t; u.act = A_ATTACK;
      if (rw) rw[R_ATTACK] += 1.f;
      return true;
    }
  }
  return false;
}

int MicroRTSSim::nearest(int uid, int owner_filter, int type_filter, int* dist) const {
  const Unit& u = units_[uid];
  int best = -1, bd = 1 << 30;
  for (size_t i = 0; i < units_.size(); ++i) {
    const Unit& t = units_[i];
    if (!t.alive || (int)i == uid) continue;
    if (owner_filter != -2 && t.owner != owner_filter) continue;
    if (type_filter > 0 && t.type != type_filter) continue;
    int d = std::abs(t.x - u.x) + std::abs(t.y - u.y);
    if (d < bd) { bd = d; best = (int)i; }
  }
  if (dist) *dist = bd;
  return best;
}

// Bots move one step toward (tx, ty): the free neighbour that shortens the Manhattan distance
// (most steps on an open map), else the first step of a shortest path around the units in the
// way (BFS over free cells from the target; the greedy step alone left bots oscillating behind
// a blocker, which made the stand-in's games far longer than microRTS's pathfinding bots')
int MicroRTSSim::dir_toward(const Unit& u, int tx, int ty) const {
  int best = -1, bd = 1 << 30;
  const int d0 = std::abs(tx - u.x) + std::abs(ty - u.y);
  for (int d = 0; d < 4; ++d) {
    int nx = u.x + kDX[d], ny = u.y + kDY[d];
    if (!empty(nx, ny)) continue;
    int dd = std::abs(tx - nx) + std::abs(ty - ny);
    if (dd < bd) { bd = dd; best = d; }
  }
  if (best < 0 || bd < d0) return best;
  const int S = s_ * s_;
  int16_t dist[32 * 32];
  int16_t q[32 * 32];
  if (S > 32 * 32) return best;
  std::fill(dist, dist + S, (int16_t)-1);
  int qh = 0, qt = 0;
  const int tc = cell(tx, ty);
  dist[tc] = 0;
  q[qt++] = (int16_t)tc;
  while (qh < qt) {
    const int c = q[qh++], cx = c % s_, cy = c / s_;
    for (int d = 0; d < 4; ++d) {
      const int nx = cx + kDX[d], ny = cy + kDY[d];
      if (!in_bounds(nx, ny)) continue;
      const int nc = cell(nx, ny);
      if (dist[nc] >= 0) continue;
      if (nx == u.x && ny == u.y) {  // reached the mover: step to the neighbour it came from
        for (int k = 0; k < 4; ++k)
          if (u.x + kDX[k] == cx && u.y + kDY[k] == cy) return empty(cx, cy) ? k : best;
      }
      if (grid_[nc] >= 0) continue;
      dist[nc] = (int16_t)(dist[c] + 1);
      q[qt++] = (int16_t)nc;
    }
  }
  return best;  // no path: keep the greedy step
}

// Bot tuning (compile-time; docs/DESIGN.md 9a, csrc/tests/calib_components.cpp):
// coac build order: workers kept by the base, and how many of them harvest (the rest rush)
static constexpr int kCoacWorkers = 8, kCoacHarvesters = 1;
static constexpr int kLightWorkers = 3;  // light rush: workers kept, all but one harvest
static constexpr bool kChaseBaseFirst = true;
static constexpr int kChaseBaseSlack = 3;
// random-biased: a move toward the nearest enemy unit weighs kRBToward (microRTS's
// RandomBiasedAI moves uniformly; its games against the uniform agent end by step ~500 in the
// reference's logs, the stand-in's random walk needed ~860), and once the enemy base is down
// its mobile units hunt what is left (kHuntNoBase); the same hunt for the scripted rushes'
// harvesters (kHuntAll) measured longer games and is off
static constexpr int kRBToward = 8;
static constexpr bool kHuntNoBase = true;
static constexpr bool kHuntAll = false;

// Scripted opponents (stand-ins for coacAI, randomBiasedAI, lightRushAI,
// workerRushAI — libs/utils.py:69-72). They act through exec() with the same
// validity rules as the learning agent.
void MicroRTSSim::bot_unit(int uid, int player, float* rwo, int n_workers, int n_barracks,
                           int widx) {
  Unit& u = units_[uid];
  uint8_t a[7] = {0, 0, 0, 0, 0, 0, 0};
  const int enemy = 1 - player;
  // attack in range, units that fight back first (lowest hp among them), buildings last --
  // the target choice of microRTS's rush AIs
  auto try_attack = [&]() -> bool {
    const UnitSpec& sp = kSpec[u.type];
    if (sp.damage <= 0) return false;
    int best = -1, bkey = 1 << 30;
    const int Rs = std::min<int>(sp.range, 3);  // the cells in range, in the same order
    for (int ay = -Rs; ay <= Rs; ++ay)
      for (int ax = -Rs; ax <= Rs; ++ax) {
        if (ax * ax + ay * ay > sp.range * sp.range || (ax == 0 && ay == 0)) continue;
        int tx = u.x + ax, ty = u.y + ay;
        if (!in_bounds(tx, ty)) continue;
        int g = grid_[cell(tx, ty)];
        if (g >= 0 && units_[g].owner == enemy) {
          const Unit& t = units_[g];
          const int key = (kSpec[t.type].damage > 0 ? 0 : 64) + t.hp;
          if (key < bkey) { bkey = key; best = (ay + 3) * 7 + (ax + 3); }
        }
      }
    if (best < 0) return false;
    a[0] = A_ATTACK; a[6] = (uint8_t)best;
    return exec(uid, a, rwo);
  };
  auto move_to = [&](int tx, int ty) -> bool {
    int d = dir_toward(u, tx, ty);
    if (d < 0) return false;
    a[0] = A_MOVE; a[1] = (uint8_t)d;
    return exec(uid, a, rwo);
  };
  auto produce = [&](int type) -> bool {
    for (int k = 0; k < 4; ++k) {
      int d = (int)((rand_u32() + k) & 3);
      if (!empty(u.x + kDX[d], u.y + kDY[d])) continue;
      a[0] = A_PRODUCE; a[4] = (uint8_t)d; a[5] = (uint8_t)(type - 1);
      return exec(uid, a, rwo);
    }
    return false;
  };
  auto harvest_cycle = [&]() -> bool {
    if (u.res > 0) {
      int dist, b = nearest(uid, player, BASE, &dist);
      if (b < 0) return false;
      if (dist == 1) {
        for (int d = 0; d < 4; ++d)
          if (u.x + kDX[d] == units_[b].x && u.y + kDY[d] == units_[b].y) {
            a[0] = A_RETURN; a[3] = (uint8_t)d; return exec(uid, a, rwo);
          }
      }
      return move_to(units_[b].x, units_[b].y);
    }
    int dist, r = nearest(uid, -1, RESOURCE, &dist);
    if (r < 0) return false;
    if (dist == 1) {
      for (int d = 0; d < 4; ++d)
        if (u.x + kDX[d] == units_[r].x && u.y + kDY[d] == units_[r].y) {
          a[0] = A_HARVEST; a[2] = (uint8_t)d; return exec(uid, a, rwo);
        }
    }
    return move_to(units_[r].x, units_[r].y);
  };
  // attack-move: the nearest enemy unit that can fight back or produce (mobile units, bases,
  // barracks), the rest (e.g. nothing) only when none is left
  auto chase = [&]() -> bool {
    // nearest(uid, enemy, -1) and nearest(uid, enemy, BASE) in one pass (same tie order)
    int e = -1, dist = 1 << 30, b = -1, db = 1 << 30;
    for (size_t i = 0; i < units_.size(); ++i) {
      const Unit& t = units_[i];
      if (!t.alive || t.owner != enemy) continue;
      const int d = std::abs(t.x - u.x) + std::abs(t.y - u.y);
      if (d < dist) { dist = d; e = (int)i; }
      if (t.type == BASE && d < db) { db = d; b = (int)i; }
    }
    if (e < 0) return false;
    if (kChaseBaseFirst && b >= 0 && db <= dist + kChaseBaseSlack) e = b;
    return move_to(units_[e].x, units_[e].y);
  };

  switch (bot_) {
    case BOT_PASSIVE: return;
    case BOT_RANDOM_BIASED: {
      // stand-in calibration: once the enemy base is down, mobile units hunt what is left
      if (kHuntNoBase && u.type >= WORKER && count_units(enemy, BASE) == 0) {
        if (try_attack()) return;
        if (chase()) return;
      }
      // microRTS RandomBiasedAI: one of the unit's concrete actions (each move direction, each
      // harvest / return direction, each produce direction x type, each attack target, and
      // none) at random, attack / harvest / return weighted 5x the others
      uint32_t w[3];
      unit_mask(u, player, w);
      struct Cand { uint8_t t, p0, p1; };
      Cand cand[4 + 4 + 4 + 4 * 7 + 49 + 1];
      int wt[sizeof(cand) / sizeof(cand[0])], n = 0, tot = 0;
      auto add = [&](uint8_t t, uint8_t p0, uint8_t p1, int weight) {
        cand[n] = {t, p0, p1};
        wt[n++] = weight;
        tot += weight;
      };
      add(A_NOOP, 0, 0, 1);
      // stand-in calibration (docs/DESIGN.md 9a): a move that closes in on the nearest enemy
      // unit weighs kRBToward (1 = microRTS's uniform moves)
      int ed = -1, ex = 0, ey = 0;
      if (kRBToward > 1 && u.type >= WORKER) {
        const int e = nearest(uid, 1 - player, -1, &ed);
        if (e >= 0) { ex = units_[e].x; ey = units_[e].y; } else { ed = -1; }
      }
      for (int d = 0; d < 4; ++d) {
        if (getbit(w, kNvecOff[1] + d)) {
          const int nd = std::abs(ex - (u.x + kDX[d])) + std::abs(ey - (u.y + kDY[d]));
          add(A_MOVE, (uint8_t)d, 0, ed >= 0 && nd < ed ? kRBToward : 1);
        }
        if (getbit(w, kNvecOff[2] + d)) add(A_HARVEST, (uint8_t)d, 0, 5);
        if (getbit(w, kNvecOff[3] + d)) add(A_RETURN, (uint8_t)d, 0, 5);
        if (getbit(w, kNvecOff[4] + d))
          for (int k = 0; k < 7; ++k)
            if (getbit(w, kNvecOff[5] + k)) add(A_PRODUCE, (uint8_t)d, (uint8_t)k, 1);
      }
      if (getbit(w, kNvecOff[0] + A_ATTACK))
        for (int j = 0; j < 49; ++j)
          if (getbit(w, kNvecOff[6] + j)) add(A_ATTACK, (uint8_t)j, 0, 5);
      int r = (int)(rand_u32() % (uint32_t)tot), k = 0;
      while (r >= wt[k]) r -= wt[k++];
      const Cand c = cand[k];
      if (c.t == A_NOOP) return;
      a[0] = c.t;
      switch (c.t) {
        case A_MOVE: a[1] = c.p0; break;
        case A_HARVEST: a[2] = c.p0; break;
        case A_RETURN: a[3] = c.p0; break;
        case A_PRODUCE: a[4] = c.p0; a[5] = c.p1; break;
        case A_ATTACK: a[6] = c.p0; break;
        default: break;
      }
      exec(uid, a, rwo);
      return;
    }
    case BOT_RANDOM: {
      uint32_t w[3];
      unit_mask(u, player, w);
      // biased: prefer attack > harvest/return > produce > move (randomBiasedAI)
      int at = A_NOOP;
      {
        int c[6], n = 0;
        for (int k = 0; k < 6; ++k) if (getbit(w, k)) c[n++] = k;
        at = n ? c[rand_u32() % n] : A_NOOP;
      }
      a[0] = (uint8_t)at;
      // draw only the parameters the chosen type reads (exec ignores the others): the
      // 49-bit attack component was scanned for every unit every tick (random_biased cost
      // ~1.6 us per env step vs ~0.8 for the scripted bots)
      int comps[2] = {0, 0}, nc = 0;
      switch (at) {
        case A_MOVE: comps[nc++] = 1; break;
        case A_HARVEST: comps[nc++] = 2; break;
        case A_RETURN: comps[nc++] = 3; break;
        case A_PRODUCE: comps[nc++] = 4; comps[nc++] = 5; break;
        case A_ATTACK: comps[nc++] = 6; break;
        default: break;
      }
      for (int k = 0; k < nc; ++k) {
        const int comp = comps[k];
        int cand[49], n = 0;
        for (int j = 0; j < kNvec[comp]; ++j)
          if (getbit(w, kNvecOff[comp] + j)) cand[n++] = j;
        a[comp] = n ? (uint8_t)cand[rand_u32() % n] : 0;
      }
      if (at != A_NOOP) exec(uid, a, rwo);
      return;
    }
    case BOT_WORKER_RUSH: {
      if (u.type == BASE) { produce(WORKER); return; }
      if (u.type == WORKER) {
        if (try_attack()) return;
        if (widx == 0 && !(kHuntAll && count_units(enemy, BASE) == 0) && harvest_cycle()) return;
        chase();
      }
      return;
    }
    case BOT_LIGHT_RUSH: {
      // the first worker puts the barracks down with the starting resources, two harvest for
      // the light units, any further worker joins the attack
      if (u.type == BASE) { if (n_workers < kLightWorkers) produce(WORKER); return; }
      if (u.type == BARRACKS) { produce(LIGHT); return; }
      if (u.type == WORKER) {
        if (try_attack()) return;
        if (n_barracks == 0 && resources_[player] >= kSpec[BARRACKS].cost && widx == 0) {
          if (produce(BARRACKS)) return;
        }
        if (widx < kLightWorkers - 1 && harvest_cycle()) return;
        chase();
        return;
      }
      if (try_attack()) return;
      chase();
      return;
    }
    case BOT_COAC:
    default: {
      // economy + mixed army (a small "coacAI"-like build order)
      if (u.type == BASE) { if (n_workers < kCoacWorkers) produce(WORKER); return; }
      if (u.type == BARRACKS) {
        const int r = resources_[player];
        int t = (r >= kSpec[HEAVY].cost && rand_unit() < 0.3f) ? HEAVY
              : (rand_unit() < 0.5f ? RANGED : LIGHT);
        produce(t);
        return;
      }
      if (u.type == WORKER) {
        if (try_attack()) return;
        // barracks only once the worker rush is under way (the rush comes first on small maps)
        if (n_barracks == 0 && n_workers >= kCoacWorkers / 2 &&
            resources_[player] >= kSpec[BARRACKS].cost && widx == 1) {
          if (produce(BARRACKS)) return;
        }
        if (widx < kCoacHarvesters && !(kHuntAll && count_units(enemy, BASE) == 0) &&
            harvest_cycle())
          return;
        chase();
        return;
      }
      if (try_attack()) return;
      chase();
      return;
    }
  }
}

void MicroRTSSim::bot_act(int player, float* rwo) {
  // own worker / barracks counts for the build orders (taken once per tick), and each
  // worker's index among own workers in unit order (the first ones harvest)
  const int n_workers = cnt_[player][WORKER], n_barracks = cnt_[player][BARRACKS];
  // the idle own units in unit order, each with its index among the own workers before it
  // (branch-free: owners and idleness are mixed along the list). Equivalent to one loop that
  // acts as it goes: a bot's action never kills or busies another own unit, and a unit it
  // creates is busy; the one thing the sequential loop sees is a produced WORKER landing in a
  // dead slot k between the producer and the list's end, which moves the worker index of the
  // units after k (added[] below)
  const int n = (int)units_.size();
  uint16_t cand[32 * 32 + 4], cw[32 * 32 + 4], added[32 * 32 + 4];
  int nc = 0, w = 0, na = 0;
  for (int i = 0; i < n; ++i) {
    const Unit& u = units_[i];
    const int own = (u.alive != 0) & (u.owner == player);
    cand[nc] = (uint16_t)i;
    cw[nc] = (uint16_t)w;
    nc += own & (u.busy == 0);
    w += own & (u.type == WORKER);
  }
  for (int q = 0; q < nc; ++q) {
    const int i = cand[q];
    int widx = cw[q];
    for (int t = 0; t < na; ++t) widx += added[t] < i;
    last_add_ = -1;
    bot_unit(i, player, rwo, n_workers, n_barracks, widx);
    const int k = last_add_;
    if (k > i && k < n && units_[k].type == WORKER && units_[k].owner == player)
      added[na++] = (uint16_t)k;
  }
}

void MicroRTSSim::set_opponent_actions(const uint8_t* a) {
  std::memcpy(opp_actions_.data(), a, opp_actions_.size());
}

float MicroRTSSim::step(const uint8_t* actions, bool* done, float* raw) {
  float rw[kNumRewards] = {0, 0, 0, 0, 0, 0};
  // 1) agent actions for idle units, validated against the mask it observed. Applied in
  // cell (row-major) order like the per-cell action array, but found from the unit list
  // (~10-30 units) instead of a scan of every cell: units an action creates are busy and
  // own units cannot be removed by own actions, so the set is fixed at this point and
  // exec() re-checks idleness. Same semantics as the scan, a fraction of the memory traffic.
  const int nc = s_ * s_;
  uint32_t idle[32 * 32 + 4];  // units never outnumber cells (maps up to 32x32)
  int n_idle = 0;
  for (size_t i = 0; i < units_.size(); ++i) {  // branch-free collection, then sort by cell
    const Unit& u = units_[i];
    idle[n_idle] = ((uint32_t)cell(u.x, u.y) << 16) | (uint32_t)i;
    n_idle += (u.alive != 0) & (u.owner == 0) & (u.busy == 0);
  }
  for (int q = 1; q < n_idle; ++q) {
    const uint32_t key = idle[q];
    int j = q;
    for (; j > 0 && idle[j - 1] > key; --j) idle[j] = idle[j - 1];
    idle[j] = key;
  }
  for (int q = 0; q < n_idle; ++q) {
    const uint32_t key = idle[q];
    const int c = (int)(key >> 16), g = (int)(key & 0xFFFFu);
    uint8_t tmp[kActComps];
    const uint8_t* a = actions + (size_t)c * kActComps;
    if (p16_) {  // packed fast path: decode only cells that hold an idle own unit
      mbr::unpack_env_action(p16_[c], tmp);
      a = tmp;
    }
    if (!validate_) {  // the mask lives on the GPU; exec() re-checks feasibility itself
      if (a[0] < 6) exec(g, a, rw);
      continue;
    }
    const uint32_t* m = &mask_[(size_t)c * kMaskWords];
    if (a[0] >= 6 || !getbit(m, a[0])) continue;
    // the chosen type's parameter must be legal too
    int comp = 0;
    switch (a[0]) {
      case A_MOVE: comp = 1; break; case A_HARVEST: comp = 2; break;
      case A_RETURN: comp = 3; break; case A_PRODUCE: comp = 4; break;
      case A_ATTACK: comp = 6; break; default: comp = 0;
    }
    if (comp && (a[comp] >= kNvec[comp] || !getbit(m, kNvecOff[comp] + a[comp]))) continue;
    if (a[0] == A_PRODUCE && (a[5] >= 7 || !getbit(m, kNvecOff[5] + a[5]))) continue;
    exec(g, a, rw);
  }
  // 2) opponent
  if (external_opp_) {
    for (int c = 0; c < nc; ++c) {
      // opponent actions are given in its own (mirrored) frame
      int rx, ry;
      map_xy(1, c % s_, c / s_, &rx, &ry);
      const int g = grid_[cell(rx, ry)];
      if (g < 0) continue;
      const Unit& u = units_[g];
      if (u.owner != 1 || u.busy > 0) continue;
      uint8_t otmp[kActComps];
      const uint8_t* ap = &opp_actions_[(size_t)c * kActComps];
      if (opp16_) {
        mbr::unpack_env_action(opp16_[c], otmp);
        ap = otmp;
      }
      if (ap[0] >= 6) continue;
      // fast path: the opponent's mask lives on the GPU; exec() re-checks feasibility
      if (validate_ && !getbit(&mask_p1_[(size_t)c * kMaskWords], ap[0])) continue;
      uint8_t a[7];
      for (int k = 0; k < 7; ++k) a[k] = ap[k];
      for (int k = 1; k <= 4; ++k) a[k] = (uint8_t)((ap[k] + 2) & 3);
      a[6] = (uint8_t)((6 - ap[6] / 7) * 7 + (6 - ap[6] % 7));
      exec(g, a, nullptr);
    }
  } else {
    bot_act(1, nullptr);
  }
  // 3) terminal check (advancing time below changes nobody's life: it can come first)
  ++tick_;
  int alive[2] = {0, 0};
  for (int t = 0; t < 8; ++t) {
    alive[0] += cnt_[0][t];
    alive[1] += cnt_[1][t];
  }
  bool d = false;
  if (alive[1] == 0 || alive[0] == 0) {
    d = true;
    last_winner_ = alive[1] == 0 ? (alive[0] == 0 ? -1 : 0) : 1;
    rw[R_WIN] = last_winner_ == 0 ? 1.f : (last_winner_ == 1 ? -1.f : 0.f);
  } else if (tick_ >= max_steps_) {
    d = true;
    last_winner_ = -1;
  }
  // 4) advance time (skipped on a terminal step: reset() follows), branch-free since the busy
  // flips are data-dependent; step_packed_list writes the sparse row in the same pass
  int rows_n = 0, rows_idle = 0;
  if (!d && rows_out_) {
    uint32_t spill;
    for (Unit& u : units_) {
      const int16_t b = u.busy, nb = (int16_t)(b - (u.alive && b > 0));
      u.act = (b > 0 && nb == 0 && u.alive) ? (int8_t)A_NOOP : u.act;
      u.busy = nb;
      const int live = u.alive != 0;
      rows_idle += live & (u.owner == 0) & (u.act == A_NOOP);
      *(rows_n < nc ? rows_out_ + rows_n : &spill) = row_entry(u, 0);
      rows_n += live;
    }
  } else if (!d) {
    for (Unit& u : units_) {
      const int16_t b = u.busy, nb = (int16_t)(b - (u.alive && b > 0));
      u.act = (b > 0 && nb == 0 && u.alive) ? (int8_t)A_NOOP : u.act;
      u.busy = nb;
    }
  }
  float r = 0.f;
  for (int i = 0; i < kNumRewards; ++i) r += rw_[i] * rw[i];
  if (raw) for (int i = 0; i < kNumRewards; ++i) raw[i] = rw[i];
  *done = d;
  if (d) {
    reset();
    if (rows_out_) rows_n = write_obs_code_list(rows_out_, &rows_idle);
  }
  rows_n_ = rows_n;
  rows_idle_ = rows_idle;
  if (!d) {
    if (validate_) compute_mask(0, mask_);
    if (external_opp_ && validate_) compute_mask(1, mask_p1_);
  }
  return r;
}

float MicroRTSSim::step_packed_list(const uint16_t* env_actions, bool* done, uint32_t* entries,
                                    int* n, int* idle_own) {
  rows_out_ = entries;
  const float r = step_packed(env_actions, done);
  rows_out_ = nullptr;
  *n = rows_n_;
  if (idle_own) *idle_own += rows_idle_;
  return r;
}

float MicroRTSSim::step_packed2_list(const uint16_t* env_actions, const uint16_t* opp_actions,
                                     bool* done, uint32_t* entries, int* n, int* idle_own) {
  rows_out_ = entries;
  const float r = step_packed2(env_actions, opp_actions, done);
  rows_out_ = nullptr;
  *n = rows_n_;
  if (idle_own) *idle_own += rows_idle_;
  return r;
}

float MicroRTSSim::step_packed(const uint16_t* env_actions, bool* done) {
  p16_ = env_actions;
  const float r = step(nullptr, done, nullptr);
  p16_ = nullptr;
  return r;
}

float MicroRTSSim::step_packed2(const uint16_t* env_actions, const uint16_t* opp_actions,
                                bool* done) {
  // the opponent's packed actions are in its own (mirrored) frame, as set_opponent_actions
  opp16_ = opp_actions;
  const float r = step_packed(env_actions, done);
  opp16_ = nullptr;
  return r;
}

void MicroRTSSim::write_obs_codes_as(int player, uint16_t* out) const {
  // empty cells are code 0: clear, then overlay the live units
  const int nc = s_ * s_;
  std::memset(out, 0, (size_t)nc * sizeof(uint16_t));
  for (const Unit& u : units_) {
    if (!u.alive) continue;
    int px, py;
    map_xy(player, u.x, u.y, &px, &py);
    const int own = u.owner < 0 ? 0 : (u.owner == player ? 1 : 2);
    out[cell(px, py)] = mbr::cell_code(std::min<int>(std::max<int>(u.hp, 0), 4),
                                       std::min<int>(std::max<int>(u.res, 0), 4), own, u.type,
                                       u.act);
  }
}

int MicroRTSSim::write_obs_code_list(uint32_t* entries, int* idle_own, int player) const {
  // branch-free over the unit list (dead slots sit between live ones): every unit's entry is
  // written at n, and n advances past the live ones only (a write past the S cells' entries,
  // only possible on a full board, goes to a scratch word)
  const int S = s_ * s_;
  uint32_t spill;
  int n = 0, idle = 0;
  for (const Unit& u : units_) {
    const int live = u.alive != 0;
    idle += live & (u.owner == player) & (u.act == A_NOOP);
    *(n < S ? entries + n : &spill) = row_entry(u, player);
    n += live;
  }
  if (idle_own) *idle_own += idle;
  return n;
}

// ---------------------------------------------------------------- observations
static inline uint32_t unit_bits(const Unit* u, int player) {
  // empty cell: hp0, res0, owner none, type none, action noop
  if (!u) return (1u << 0) | (1u << 5) | (1u << 10) | (1u << 13) | (1u << 21);
  uint32_t b = 0;
  b |= 1u << (0 + std::min<int>(std::max<int>(u->hp, 0), 4));
  b |= 1u << (5 + std::min<int>(std::max<int>(u->res, 0), 4));
  int own = u->owner < 0 ? 0 : (u->owner == player ? 1 : 2);
  b |= 1u << (10 + own);
  b |= 1u << (13 + u->type);
  b |= 1u << (21 + u->act);
  return b;
}

void MicroRTSSim::write_obs(uint32_t* out) const {
  const int nc = s_ * s_;
  for (int c = 0; c < nc; ++c) {
    int g = grid_[c];
    out[c] = unit_bits(g >= 0 ? &units_[g] : nullptr, 0);
  }
}

void MicroRTSSim::write_obs_p1(uint32_t* out) const {
  const int nc = s_ * s_;
  for (int c = 0; c < nc; ++c) {
    int rx, ry;
    map_xy(1, c % s_, c / s_, &rx, &ry);
    int g = grid_[cell(rx, ry)];
    out[c] = unit_bits(g >= 0 ? &units_[g] : nullptr, 1);
  }
}

void MicroRTSSim::write_mask(uint32_t* out) const {
  std::memcpy(out, mask_.data(), mask_.size() * sizeof(uint32_t));
}
void MicroRTSSim::write_mask_p1(uint32_t* out) const {
  std::memcpy(out, mask_p1_.data(), mask_p1_.size() * sizeof(uint32_t));
}

void MicroRTSSim::write_obs_dense(float* out) const {
  const int nc = s_ * s_;
  for (int c = 0; c < nc; ++c) {
    int g = grid_[c];
    uint32_t b = unit_bits(g >= 0 ? &units_[g] : nullptr, 0);
    for (int p = 0; p < kPlanes; ++p) out[(size_t)c * kPlanes + p] = (float)((b >> p) & 1u);
  }
}

void MicroRTSSim::write_mask_dense(uint8_t* out) const {
  const int nc = s_ * s_;
  for (int c = 0; c < nc; ++c)
    for (int j = 0; j < kMaskBits; ++j)
      out[(size_t)c * kMaskBits + j] = getbit(&mask_[(size_t)c * kMaskWords], j) ? 1 : 0;
}

}  // namespace mb
