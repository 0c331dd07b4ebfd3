// Rules of the synthetic microRTS shared by the C++ simulator (host) and the
// GPU mask kernel (device), so the action mask computed on the GPU from the
// observation is bit-identical to the simulator's own mask.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MB_HD __host__ __device__
#else
#define MB_HD
#endif

namespace mbr {

enum : int { NONE = 0, RESOURCE = 1, BASE = 2, BARRACKS = 3, WORKER = 4, LIGHT = 5, HEAVY = 6,
             RANGED = 7 };
enum : int { A_NOOP = 0, A_MOVE = 1, A_HARVEST = 2, A_RETURN = 3, A_PRODUCE = 4, A_ATTACK = 5 };

// per unit type: hp, cost, damage, attack range, move / attack / produce ticks -- the values of
// microRTS's UnitTypeTable (the Java engine gym-microrts wraps; one env step = one game tick),
// so a uniform-random agent's episodes against the reference bot mix have the length, return and
// win share of the reference's logged runs (tools/calibrate_env.py, docs/DESIGN.md section 9a)
MB_HD constexpr int spec_hp(int t) {
  return t == RESOURCE ? 1 : t == BASE ? 10 : t == BARRACKS ? 4 : t == WORKER ? 1 : t == LIGHT ? 4
       : t == HEAVY ? 4 : t == RANGED ? 1 : 0;
}
MB_HD constexpr int spec_cost(int t) {
  return t == BASE ? 10 : t == BARRACKS ? 5 : t == WORKER ? 1 : t == LIGHT ? 2 : t == HEAVY ? 3
       : t == RANGED ? 2 : 0;
}
MB_HD constexpr int spec_damage(int t) {
  return t == WORKER ? 1 : t == LIGHT ? 2 : t == HEAVY ? 4 : t == RANGED ? 1 : 0;
}
MB_HD constexpr int spec_range(int t) { return t == RANGED ? 3 : (t >= WORKER ? 1 : 0); }
MB_HD constexpr int spec_move_t(int t) {
  return t == WORKER ? 10 : t == LIGHT ? 8 : t == HEAVY ? 12 : t == RANGED ? 10 : 0;
}
MB_HD constexpr int spec_attack_t(int t) { return t >= WORKER ? 5 : 0; }
MB_HD constexpr int spec_produce_t(int t) {
  return t == BASE ? 250 : t == BARRACKS ? 200 : t == WORKER ? 50 : t == LIGHT ? 80 : t == HEAVY ? 120
       : t == RANGED ? 100 : 0;
}
constexpr int kHarvestT = 20, kReturnT = 10;

// 16-bit cell code: hp(3) | res(3) << 3 | owner(2) << 6 | type(3) << 8 | act(3) << 11
// owner: 0 none, 1 = the observing player, 2 = the opponent. hp / res capped at 4.
MB_HD inline uint16_t cell_code(int hp, int res, int owner, int type, int act) {
  return (uint16_t)(hp | (res << 3) | (owner << 6) | (type << 8) | (act << 11));
}
MB_HD inline int code_hp(uint16_t c) { return c & 7; }
MB_HD inline int code_res(uint16_t c) { return (c >> 3) & 7; }
MB_HD inline int code_owner(uint16_t c) { return (c >> 6) & 3; }
MB_HD inline int code_type(uint16_t c) { return (c >> 8) & 7; }
MB_HD inline int code_act(uint16_t c) { return (c >> 11) & 7; }
// the 27-plane one-hot bits of a code (plane p <=> bit p)
MB_HD inline uint32_t code_bits(uint16_t c) {
  return (1u << code_hp(c)) | (1u << (5 + code_res(c))) | (1u << (10 + code_owner(c))) |
         (1u << (13 + code_type(c))) | (1u << (21 + code_act(c)));
}

// 16-bit env action per cell: type(3) | dir(2) << 3 | produce type(3) << 5 | attack(6) << 8
// (only the chosen type's parameter travels; the rollout keeps all 7 components)
MB_HD inline uint16_t pack_env_action(const uint8_t* a) {
  const int t = a[0] < 6 ? a[0] : 0;
  const int dir = t == A_MOVE ? a[1] : t == A_HARVEST ? a[2] : t == A_RETURN ? a[3]
                : t == A_PRODUCE ? a[4] : 0;
  return (uint16_t)(t | ((dir & 3) << 3) | ((a[5] & 7) << 5) | ((a[6] & 63) << 8));
}
MB_HD inline void unpack_env_action(uint16_t v, uint8_t* a) {
  const uint8_t dir = (v >> 3) & 3;
  a[0] = v & 7;
  a[1] = a[2] = a[3] = a[4] = dir;
  a[5] = (v >> 5) & 7;
  a[6] = (v >> 8) & 63;
}

constexpr int kSegOff[8] = {0, 6, 10, 14, 18, 22, 29, 78};
constexpr int kDX[4] = {0, 1, 0, -1};
constexpr int kDY[4] = {-1, 0, 1, 0};

}  // namespace mbr
