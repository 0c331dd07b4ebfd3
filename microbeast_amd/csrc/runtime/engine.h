// GPU actor engine: native replacement for the reference's actor processes
// (reference microbeast.py:30-105 act(), :179-191 spawn loop) re-designed for
// one MI355X per learner process:
//
//   * env worker threads (C++, no GIL) step the synthetic microRTS sims and
//     write compact obs / mask / reward / done into PINNED host staging;
//   * a driver thread pipelines env groups through the GPU on `n_lanes` HIP
//     streams (group g on lane g % n_lanes; each lane has its own policy graph,
//     I/O buffers and inference-weight copy, so policy steps of different
//     groups run concurrently instead of queueing behind each other and behind
//     the learner's kernels): H2D staging -> hipGraphLaunch(policy graph) ->
//     one multi-segment copy kernel that scatters the step into an
//     HBM-resident rollout slot -> D2H actions -> event;
//   * rollout slots live in HBM (288 GB/GPU: thousands of slots fit), so the
//     learner reads them in place — no stack/reshape/copy (reference
//     libs/utils.py:197-205 get_batch);
//   * free/full slot hand-off with HIP events instead of pickled queue ints;
//   * weight publish is a D2D copy applied between inference steps, ordered by
//     events (no torn reads; reference libs/utils.py:337 had none);
//   * self-play league (BASELINE config 5): the last `selfplay_groups` groups play
//     against an external opponent. Their envs also ship player-1 codes (mirrored
//     frame), a second captured graph runs the opponent policy (a league snapshot,
//     swapped in through a second publish channel) and both players' packed actions
//     come back; finished episodes are tagged with the opponent's league id.
//
// Slot layout (time-major [T+1, E]): index t holds obs_t, mask_t, the action
// a_t sampled at obs_t with its behaviour log-prob and value, and r_t/done_t
// produced by stepping a_t. Index T holds obs_T/mask_T for the bootstrap and is
// also index 0 of the group's next slot (TorchBeast overlap), fixing the
// reference's obs/action off-by-one.
#pragma once
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "vec_env.h"
#include "../include/mbk_api.h"

namespace mb {

struct EngineConfig {
  int size = 16;
  int n_groups = 2;
  int envs_per_group = 256;
  int unroll = 64;  // T
  int n_slots = 8;
  int n_threads = 8;
  int max_steps = 2000;
  uint64_t seed = 1;
  std::vector<int> bots;
  std::vector<float> reward_weight;
  int env_index_base = 0;
  int device = 0;
  int selfplay_groups = 0;  // groups [n_groups - selfplay_groups, n_groups) are self-play
  int n_lanes = 1;          // concurrent policy streams (each with its own graph + I/O)
  // >1: before the first policy step every env plays r ~ U[0, preroll) uniform-policy steps on
  // the CPU (VecEnv::preroll), so the envs start spread over the game's phases, not all at
  // their first frame (bench.py: the timed window then measures the steady state)
  int preroll = 0;
};

// Fixed-address I/O of one lane's captured policy graph (and opponent graph). The graph
// decodes in_codes/in_res into in_obs / in_mask (GPU-side mask) and packs out_action
// into out_act16.
struct LaneIO {
  uintptr_t in_obs = 0, in_mask = 0, out_action = 0, out_logp = 0, out_value = 0;
  uintptr_t in_codes = 0, in_res = 0, out_act16 = 0;
  // opponent graph I/O (self-play groups only)
  uintptr_t in_codes_p1 = 0, in_res_p1 = 0, out_act16_p1 = 0;
  uintptr_t out_logits = 0;  // dense policy logits [E][78*S] f32 (reference keys only)
};

// Per-lane graphs (raw hipGraphExec_t). opp: opponent policy (self-play only); pack /
// opp_pack (optional): replayed right after a publish lands on that lane, rebuilding the
// derived inference weights so the policy graph itself never re-packs.
struct LaneGraphs {
  uintptr_t policy = 0, opp = 0, pack = 0, opp_pack = 0;
};

// Device buffers owned by Python (torch tensors); raw addresses.
struct EngineBuffers {
  // rollout storage, all [n_slots, T+1, E, ...]
  uintptr_t obs = 0;      // u32 [.., S]
  uintptr_t mask = 0;     // u32 [.., S, 3]
  uintptr_t action = 0;   // u8  [.., S, 7]
  uintptr_t logp = 0;     // f32
  uintptr_t value = 0;    // f32
  uintptr_t reward = 0;   // f32
  uintptr_t done = 0;     // u8
  // optional reference buffer keys (libs/utils.py:34-46); 0 = not emitted
  uintptr_t ep_return = 0;     // f32 [.., E]   running episode return after the step
  uintptr_t ep_step = 0;       // i32 [.., E]   running episode length after the step
  uintptr_t last_action0 = 0;  // u8 [n_slots, E, S, 7]: the action before row 0 of a slot
  uintptr_t logits = 0;        // f32 [.., E, 78*S] dense policy logits
  // optional active-cell bitmap [.., E, S/32] u32 (fused acting steps write it; the learner's
  // head compaction reads it instead of the masks)
  uintptr_t abits = 0;
  std::vector<LaneIO> lanes;  // one per policy lane
};

struct EngineStats {
  int64_t frames = 0;          // env steps taken (all envs)
  int64_t gpu_steps = 0;       // inference graph launches
  int64_t slots_full = 0;      // rollout slots filled so far
  int full_depth = 0;          // full slots waiting for the learner right now
  double driver_idle_s = 0.0;  // driver found nothing to do
  double slot_wait_s = 0.0;    // groups stalled for a free slot (learner-bound)
  double env_s = 0.0;          // summed worker time inside env step
  // pipeline phases, summed over group steps: enqueue -> the driver sees the step's event
  // complete (GPU latency incl. queueing behind other groups / learner contention), and
  // dispatch to env workers -> the group's last env stepped (CPU phase)
  double gpu_phase_s = 0.0;
  double env_phase_s = 0.0;
  double enqueue_s = 0.0;       // driver thread time inside enqueue (HIP API calls)
  double graph_launch_s = 0.0;  // of which hipGraphLaunch of the policy graph(s)
  // MBK_STEP_TIMING=1: GPU-side split of each policy step's own stream time (timing events):
  // H2D of codes/resources, policy graph(s), rollout scatter + D2H of actions
  double step_h2d_s = 0.0, step_graph_s = 0.0, step_out_s = 0.0;
  int64_t timed_steps = 0;
  int64_t publishes = 0;
  int64_t opp_publishes = 0;
  int opp_version = -1;
  // fused acting steps (act models set) and the agent's idle units (active cells: the cells
  // the sparse head samples) summed over them
  int64_t act_steps = 0, act_active_cells = 0;
  int64_t preroll_steps = 0;  // env steps played by EngineConfig::preroll before the start
};

class GpuEngine {
 public:
  GpuEngine(const EngineConfig& cfg, const EngineBuffers& buf);
  ~GpuEngine();
  // one LaneGraphs per lane; the opponent graph is required iff selfplay_groups > 0
  void start(const std::vector<LaneGraphs>& graphs);
  void stop();
  // Blocks until n full slots are available (or timeout). Returns slot ids.
  std::vector<int> get_full(int n, double timeout_s);
  void stream_wait_full(uintptr_t stream, int slot);
  void release(const std::vector<int>& slots, uintptr_t stream);
  // Copy src (device, on `stream`) into every lane's inference weights dsts[lane], each
  // applied between two of that lane's policy steps. Returns false (skipped) if the
  // previous publish has not landed on every lane yet.
  // version: the learner update these weights come from (tags the rollout slots that
  // act with them, so the learner can measure its policy lag); -1 = untagged
  bool publish(uintptr_t src, const std::vector<uintptr_t>& dsts, size_t nbytes,
               uintptr_t stream, int version = -1) {
    return publish_chan(0, src, dsts, nbytes, stream, version);
  }
  // Version of the behaviour weights a slot's FIRST step acted with (the oldest in it).
  int slot_version(int slot) const { return slot_version_.at(slot); }
  // Learner update of the weights the lanes start with (a restarted engine acts with the
  // learner's current weights, not version 0); before start().
  void set_policy_version(int version) {
    for (auto& L : lanes_) L.policy_version = version;
  }
  // League id of the opponent weights in place at start (before any publish_opponent).
  void set_initial_opponent(int version) {
    for (auto& L : lanes_) L.opp_version = version;
    opp_version_pub_.store(version);
  }
  // League: swap the opponent policy's weights to snapshot `version` (same ordering).
  bool publish_opponent(uintptr_t src, const std::vector<uintptr_t>& dsts, size_t nbytes,
                        uintptr_t stream, int version) {
    return publish_chan(1, src, dsts, nbytes, stream, version);
  }
  std::vector<EpisodeRecord> drain_episodes() { return log_.drain(); }
  EngineStats stats() const;
  uintptr_t stream(int lane = 0) const { return (uintptr_t)lanes_.at(lane).stream; }
  // pinned host staging (all envs contiguous): 16-bit cell codes [n_envs][S], resources
  // [n_envs], packed actions [n_envs][S] -- device-addressable (coherent hipHostMalloc)
  uintptr_t host_codes() const { return (uintptr_t)h_codes_; }
  uintptr_t host_res() const { return (uintptr_t)h_res_; }
  uintptr_t host_act16() const { return (uintptr_t)h_act16_; }
  // sparse fused-step staging (0 unless set_act_models(.., copy=false)) and its row stride
  uintptr_t host_code_list() const { return (uintptr_t)h_code_list_; }
  uintptr_t host_act_list() const { return (uintptr_t)h_act_list_; }
  int list_stride() const { return list_stride_; }
  // fused acting steps (mbk_act_step: two kernel launches per step, writing the rollout row
  // directly -- no policy graph, no scatter copy -- from / to the env workers' pinned sparse
  // rows): one model / workspace block per lane, set before start(). opp_models: one block per
  // lane of the self-play opponent's inference weights (required iff self-play groups exist):
  // its step reads the opponent's mirrored code rows and writes its action rows, its
  // rollout-shaped outputs go to lane scratch.
  void set_act_models(const std::vector<MbkActModel>& models,
                      const std::vector<MbkActModel>& opp_models = {});
  bool act_mode() const { return !act_models_.empty(); }
  // captured-graph steps with sparse-row I/O (before start(); not with reference keys): env
  // workers write occupied-cell rows, one small launch
  // expands them into the graph's device codes and another compacts its packed actions into
  // the workers' action rows -- no H2D / D2H blit copies of dense [S] code rows
  void set_sparse_io(bool on);
  bool sparse_io() const { return sparse_; }
  const EngineConfig& config() const { return cfg_; }
  VecEnv& env() { return *env_; }
  bool failed() const { return failed_.load(); }
  // Fault injection (tests / --fault_inject_every): the next env step of some worker throws.
  void inject_fault() { inject_fault_.store(1); }
  std::string error() const;

 private:
  enum Phase : int { ENV_BUSY = 0, READY = 1, ON_GPU = 2 };
  struct Group {
    std::atomic<int> phase{ENV_BUSY};
    std::atomic<int> next_env{0};
    std::atomic<int> remaining{0};
    std::atomic<int> idle{0};  // sparse env workers: the agent's idle units after this step
    int cur = -1, prev = -1, t = 0;
    bool first = true;
    bool selfplay = false;
    int opp_version = -1;  // league id of the opponent that chose this step's p1 actions
    int lane = 0;
    hipEvent_t ev = nullptr;
    hipEvent_t tev[4] = {nullptr, nullptr, nullptr, nullptr};  // MBK_STEP_TIMING events
    bool timed = false;                                         // tev recorded this step
    std::chrono::steady_clock::time_point t_phase;  // start of the current phase
    std::atomic<int64_t> t_ready_ns{0};              // worker: when the env phase ended
  };
  struct PubChan {  // event-ordered D2D weight publish, applied between policy steps
    std::vector<bool> pending;          // per lane: staging not yet copied out
    std::vector<uintptr_t> dst;         // per lane inference weights
    size_t n = 0;
    int version = -1;
    hipEvent_t ready = nullptr;         // publisher stream: staging filled
    std::vector<hipEvent_t> consumed;   // per lane stream: staging copied out
    uint8_t* staging = nullptr;
    size_t staging_n = 0;
  };
  struct Lane {
    hipStream_t stream = nullptr;
    hipGraphExec_t graph = nullptr, opp_graph = nullptr;
    hipGraphExec_t pack_graph[2] = {nullptr, nullptr};
    LaneIO io;
    int opp_version = -1;     // driver thread only
    int policy_version = 0;   // learner update of the weights landed on this lane
    uint64_t act_step = 0;    // fused steps: Philox step of the lane's next policy step
    // self-play opponent steps: HBM rows + scratch for the outputs the rollout does not keep
    // (obs [E][S] u32, mask [E][S][3] u32, action [E][S][7] u8, logp / value [E] f32)
    uint8_t* opp_scratch = nullptr;
    uint64_t opp_act_step = 0;
  };

  EngineConfig cfg_;
  EngineBuffers buf_;
  int S_;
  size_t slot_stride_obs_, slot_stride_mask_, slot_stride_act_, slot_stride_scalar_;
  std::unique_ptr<VecEnv> env_;
  EpisodeLog log_;
  std::vector<Lane> lanes_;
  std::vector<std::unique_ptr<Group>> groups_;
  // pinned staging, all envs contiguous
  uint16_t* h_codes_ = nullptr;  // 16-bit cell codes
  int32_t* h_res_ = nullptr;     // player resources (GPU mask input)
  float* h_reward_ = nullptr;
  uint8_t* h_done_ = nullptr;
  uint16_t* h_act16_ = nullptr;  // packed env actions
  uint16_t* h_codes_p1_ = nullptr;  // self-play: opponent-perspective codes
  int32_t* h_res_p1_ = nullptr;
  uint16_t* h_act16_p1_ = nullptr;  // opponent's packed actions (its frame)
  float* h_ep_return_ = nullptr;     // reference keys: per-env episode return / length
  int32_t* h_ep_step_ = nullptr;

  // slots
  mutable std::mutex slot_m_;
  std::condition_variable full_cv_;
  std::deque<int> free_slots_, full_slots_;
  std::vector<hipEvent_t> full_ev_, release_ev_;
  int64_t preroll_steps_ = 0;
  std::vector<uint8_t> release_pending_;  // per slot; guarded by slot_m_ (bytes, not bits)
  std::vector<int> slot_version_;  // written when a group takes the slot (driver thread)
  std::deque<int> slot_wait_q_;  // driver thread only: groups waiting for a free slot

  // publish channels: 0 = learner policy, 1 = league opponent
  std::mutex pub_m_;
  PubChan pub_[2];
  bool publish_chan(int chan, uintptr_t src, const std::vector<uintptr_t>& dsts, size_t nbytes,
                    uintptr_t stream, int version);

  // workers
  std::vector<std::thread> workers_;
  std::thread driver_;
  std::mutex work_m_;
  std::condition_variable work_cv_;
  std::atomic<uint64_t> work_epoch_{0};
  std::atomic<bool> running_{false};
  std::atomic<bool> failed_{false};
  std::atomic<int> inject_fault_{0};
  mutable std::mutex err_m_;
  std::string err_;

  // stats
  std::atomic<int64_t> frames_{0}, gpu_steps_{0}, slots_full_{0}, publishes_{0}, opp_publishes_{0};
  std::atomic<int> opp_version_pub_{-1};
  std::atomic<int64_t> env_ns_{0};
  std::atomic<int64_t> gpu_phase_ns_{0}, env_phase_ns_{0}, enqueue_ns_{0}, launch_ns_{0};
  bool step_timing_ = false;
  std::atomic<int64_t> step_h2d_ns_{0}, step_graph_ns_{0}, step_out_ns_{0}, timed_steps_{0};
  std::atomic<int64_t> act_steps_{0}, act_active_cells_{0};
  double driver_idle_s_ = 0.0, slot_wait_s_ = 0.0;
  mutable std::mutex stats_m_;

  void worker_loop(int wid);
  void driver_loop();
  bool enqueue_gpu(int g);
  void dispatch_env(int g);
  void fail(const std::string& msg);
  void alloc_rows();
  int chunk_;
  std::vector<MbkActModel> act_models_;      // fused acting steps per lane (may be empty)
  std::vector<MbkActModel> opp_act_models_;  // ... and the self-play opponent's
  // sparse PCIe rows (VecEnv::step_range_lists): pinned rows of list_stride_ uint32 per env,
  // occupied-cell codes in, non-noop actions out (the fused step and the graph path's
  // set_sparse_io)
  bool sparse_ = false;
  int list_stride_ = 0;
  uint32_t* h_code_list_ = nullptr;
  uint32_t* h_act_list_ = nullptr;
  uint32_t* h_code_list_p1_ = nullptr;  // self-play: the opponent's rows (its own frame)
  uint32_t* h_act_list_p1_ = nullptr;
};

}  // namespace mb
