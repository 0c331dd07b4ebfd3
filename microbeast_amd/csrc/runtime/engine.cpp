#include "engine.h"


#include <chrono>
#include <cstdlib>

#include <pthread.h>
#include <sched.h>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../include/mbk_api.h"

namespace mb {

#define ENG_CHECK(expr)                                                              \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      fail(std::string(#expr) + " failed: " + hipGetErrorString(_e));                \
      return false;                                                                  \
    }                                                                                \
  } while (0)

#define CTOR_CHECK(expr)                                                             \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess)                                                            \
      throw std::runtime_error(std::string(#expr) + " failed: " + hipGetErrorString(_e)); \
  } while (0)

GpuEngine::GpuEngine(const EngineConfig& cfg, const EngineBuffers& buf) : cfg_(cfg), buf_(buf) {
  if (cfg_.n_groups < 1 || cfg_.envs_per_group < 1 || cfg_.unroll < 1)
    throw std::runtime_error("GpuEngine: bad config");
  if (cfg_.n_slots < cfg_.n_groups + 1)
    throw std::runtime_error("GpuEngine: need n_slots >= n_groups + 1");
  S_ = cfg_.size * cfg_.size;
  const size_t E = cfg_.envs_per_group, T1 = cfg_.unroll + 1;
  slot_stride_obs_ = T1 * E * S_ * 4;
  slot_stride_mask_ = T1 * E * S_ * 4 * kMaskWords;
  slot_stride_act_ = T1 * E * S_ * kActComps;
  slot_stride_scalar_ = T1 * E;  // elements
  const int total = cfg_.n_groups * cfg_.envs_per_group;
  env_.reset(new VecEnv(cfg_.size, total, cfg_.max_steps, cfg_.seed, cfg_.bots,
                        cfg_.reward_weight.empty() ? nullptr : cfg_.reward_weight.data(),
                        cfg_.env_index_base));
  CTOR_CHECK(hipSetDevice(cfg_.device));
  if (cfg_.n_lanes < 1 || (int)buf_.lanes.size() != cfg_.n_lanes)
    throw std::runtime_error("GpuEngine: need one LaneIO per lane");
  // highest priority: a policy step is latency-critical (env workers wait on it) and
  // must not queue behind the learner's long kernels on the other stream
  int prio_least = 0, prio_greatest = 0;
  CTOR_CHECK(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
  lanes_.resize(cfg_.n_lanes);
  for (int l = 0; l < cfg_.n_lanes; ++l) {
    Lane& L = lanes_[l];
    L.io = buf_.lanes[l];
    if (!L.io.in_codes || !L.io.in_res || !L.io.out_act16)
      throw std::runtime_error("GpuEngine: in_codes / in_res / out_act16 buffers required");
    CTOR_CHECK(hipStreamCreateWithPriority(&L.stream, hipStreamNonBlocking, prio_greatest));
  }
  CTOR_CHECK(hipHostMalloc((void**)&h_codes_, (size_t)total * S_ * 2, hipHostMallocDefault));
  CTOR_CHECK(hipHostMalloc((void**)&h_res_, (size_t)total * 4, hipHostMallocDefault));
  CTOR_CHECK(hipHostMalloc((void**)&h_act16_, (size_t)total * S_ * 2, hipHostMallocDefault));
  CTOR_CHECK(hipHostMalloc((void**)&h_reward_, (size_t)total * 4, hipHostMallocDefault));
  CTOR_CHECK(hipHostMalloc((void**)&h_done_, (size_t)total, hipHostMallocDefault));
  std::memset(h_reward_, 0, (size_t)total * 4);
  std::memset(h_done_, 0, (size_t)total);
  if (buf_.ep_return || buf_.ep_step) {
    CTOR_CHECK(hipHostMalloc((void**)&h_ep_return_, (size_t)total * 4, hipHostMallocDefault));
    CTOR_CHECK(hipHostMalloc((void**)&h_ep_step_, (size_t)total * 4, hipHostMallocDefault));
    std::memset(h_ep_return_, 0, (size_t)total * 4);
    std::memset(h_ep_step_, 0, (size_t)total * 4);
  }
  if (cfg_.selfplay_groups < 0 || cfg_.selfplay_groups > cfg_.n_groups)
    throw std::runtime_error("GpuEngine: bad selfplay_groups");
  const int sp0 = cfg_.n_groups - cfg_.selfplay_groups;  // first self-play group
  if (cfg_.selfplay_groups > 0) {
    for (const Lane& L : lanes_)
      if (!L.io.in_codes_p1 || !L.io.in_res_p1 || !L.io.out_act16_p1)
        throw std::runtime_error(
            "GpuEngine: self-play needs in_codes_p1 / in_res_p1 / out_act16_p1");
    CTOR_CHECK(hipHostMalloc((void**)&h_codes_p1_, (size_t)total * S_ * 2, hipHostMallocDefault));
    CTOR_CHECK(hipHostMalloc((void**)&h_res_p1_, (size_t)total * 4, hipHostMallocDefault));
    CTOR_CHECK(hipHostMalloc((void**)&h_act16_p1_, (size_t)total * S_ * 2, hipHostMallocDefault));
    std::memset(h_act16_p1_, 0, (size_t)total * S_ * 2);
    env_->set_external_opponent(sp0 * cfg_.envs_per_group, total, true);
  }
  if (cfg_.preroll > 1) {
    // desynchronised start (bench.py): each env first plays a random number of uniform-policy
    // steps on the CPU (with CPU masks), then the GPU takes over from those states
    env_->reset_codes(nullptr, nullptr);
    preroll_steps_ = env_->preroll(cfg_.preroll, cfg_.seed, std::max(1, cfg_.n_threads));
    env_->set_validate(false);  // masks are derived on the GPU from the codes
    env_->write_codes(h_codes_, h_res_);
  } else {
    env_->set_validate(false);  // masks are derived on the GPU from the codes
    env_->reset_codes(h_codes_, h_res_);
  }
  if (cfg_.selfplay_groups > 0) env_->reset_codes_p1(h_codes_p1_, h_res_p1_);
  {
    const char* st = std::getenv("MBK_STEP_TIMING");
    step_timing_ = st && st[0] == '1';
  }
  for (int g = 0; g < cfg_.n_groups; ++g) {
    groups_.emplace_back(new Group());
    CTOR_CHECK(hipEventCreateWithFlags(&groups_[g]->ev, hipEventDisableTiming));
    if (step_timing_)
      for (auto& e : groups_[g]->tev) CTOR_CHECK(hipEventCreate(&e));
    groups_[g]->selfplay = g >= sp0;
    groups_[g]->lane = g % cfg_.n_lanes;
    groups_[g]->phase.store(READY);  // reset observations are ready
  }
  full_ev_.resize(cfg_.n_slots);
  release_ev_.resize(cfg_.n_slots);
  release_pending_.assign(cfg_.n_slots, 0);
  slot_version_.assign(cfg_.n_slots, 0);
  for (int s = 0; s < cfg_.n_slots; ++s) {
    CTOR_CHECK(hipEventCreateWithFlags(&full_ev_[s], hipEventDisableTiming));
    CTOR_CHECK(hipEventCreateWithFlags(&release_ev_[s], hipEventDisableTiming));
    free_slots_.push_back(s);
  }
  for (PubChan& c : pub_) {
    CTOR_CHECK(hipEventCreateWithFlags(&c.ready, hipEventDisableTiming));
    c.pending.assign(cfg_.n_lanes, false);
    c.dst.assign(cfg_.n_lanes, 0);
    c.consumed.assign(cfg_.n_lanes, nullptr);
    for (auto& ev : c.consumed) CTOR_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  }
  // work chunk: enough chunks for every worker, at least 2 envs each (16 envs per item
  // measured level with 8, 24, 32 and faster than 8: profile 36)
  chunk_ = std::max(1, std::min(16, cfg_.envs_per_group / std::max(1, 2 * cfg_.n_threads)));
}

GpuEngine::~GpuEngine() {
  stop();
  for (Lane& L : lanes_)
    if (L.stream) hipStreamSynchronize(L.stream);
  for (auto& g : groups_) {
    if (g->ev) hipEventDestroy(g->ev);
    for (auto e : g->tev)
      if (e) hipEventDestroy(e);
  }
  for (auto e : full_ev_) hipEventDestroy(e);
  for (auto e : release_ev_) hipEventDestroy(e);
  for (PubChan& c : pub_) {
    if (c.ready) hipEventDestroy(c.ready);
    for (auto ev : c.consumed)
      if (ev) hipEventDestroy(ev);
    if (c.staging) hipFree(c.staging);
  }
  if (h_codes_p1_) hipHostFree(h_codes_p1_);
  if (h_res_p1_) hipHostFree(h_res_p1_);
  if (h_act16_p1_) hipHostFree(h_act16_p1_);
  if (h_codes_) hipHostFree(h_codes_);
  if (h_res_) hipHostFree(h_res_);
  if (h_act16_) hipHostFree(h_act16_);
  if (h_reward_) hipHostFree(h_reward_);
  if (h_ep_return_) hipHostFree(h_ep_return_);
  if (h_ep_step_) hipHostFree(h_ep_step_);
  if (h_done_) hipHostFree(h_done_);
  if (h_code_list_) hipHostFree(h_code_list_);
  if (h_act_list_) hipHostFree(h_act_list_);
  if (h_code_list_p1_) hipHostFree(h_code_list_p1_);
  if (h_act_list_p1_) hipHostFree(h_act_list_p1_);
  for (Lane& L : lanes_) {
    if (L.opp_scratch) hipFree(L.opp_scratch);
    if (L.stream) hipStreamDestroy(L.stream);
  }
}

void GpuEngine::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> g(err_m_);
    if (err_.empty()) err_ = msg;
  }
  failed_.store(true);
  running_.store(false);
  work_cv_.notify_all();
  full_cv_.notify_all();
}

std::string GpuEngine::error() const {
  std::lock_guard<std::mutex> g(err_m_);
  return err_;
}

void GpuEngine::start(const std::vector<LaneGraphs>& graphs) {
  if (running_.load()) return;
  if ((int)graphs.size() != cfg_.n_lanes)
    throw std::runtime_error("GpuEngine::start: need one LaneGraphs per lane");
  for (int l = 0; l < cfg_.n_lanes; ++l) {
    const LaneGraphs& g = graphs[l];
    if (!g.policy) throw std::runtime_error("GpuEngine::start: missing policy graph");
    if (cfg_.selfplay_groups > 0 && !g.opp)
      throw std::runtime_error("GpuEngine::start: self-play groups need the opponent graph");
    Lane& L = lanes_[l];
    L.graph = (hipGraphExec_t)g.policy;
    L.opp_graph = (hipGraphExec_t)g.opp;
    L.pack_graph[0] = (hipGraphExec_t)g.pack;
    L.pack_graph[1] = (hipGraphExec_t)g.opp_pack;
  }
  running_.store(true);
  for (int w = 0; w < cfg_.n_threads; ++w) workers_.emplace_back(&GpuEngine::worker_loop, this, w);
  driver_ = std::thread(&GpuEngine::driver_loop, this);
}

// pinned sparse rows for every env (both players' for self-play envs), filled with the reset
// state; shared by the fused acting step and the graph path's sparse I/O
void GpuEngine::alloc_rows() {
  if (h_code_list_) return;
  const size_t total = (size_t)cfg_.n_groups * cfg_.envs_per_group;
  list_stride_ = (S_ + 1 + 3) & ~3;  // word 0 + up to S entries, 16-byte rows
  const size_t bytes = total * list_stride_ * 4;
  if (hipHostMalloc((void**)&h_code_list_, bytes, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&h_act_list_, bytes, hipHostMallocDefault) != hipSuccess)
    throw std::runtime_error("GpuEngine: hipHostMalloc of the sparse rows failed");
  std::memset(h_act_list_, 0, bytes);
  env_->write_code_lists(h_code_list_, list_stride_);  // the reset state, as lists
  if (cfg_.selfplay_groups > 0) {
    if (hipHostMalloc((void**)&h_code_list_p1_, bytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&h_act_list_p1_, bytes, hipHostMallocDefault) != hipSuccess)
      throw std::runtime_error("GpuEngine: hipHostMalloc of the opponent rows failed");
    std::memset(h_act_list_p1_, 0, bytes);
    std::memset(h_code_list_p1_, 0, bytes);
    env_->write_code_lists(h_code_list_p1_, list_stride_, 1);
  }
}

void GpuEngine::set_sparse_io(bool on) {
  if (running_.load()) throw std::runtime_error("set_sparse_io: engine running");
  if (!on) { sparse_ = false; return; }
  if (act_mode()) return;  // the fused step always runs on the sparse rows
  if (buf_.ep_return || buf_.ep_step)
    throw std::runtime_error("set_sparse_io: not with the reference buffer keys");
  alloc_rows();
  sparse_ = true;
}

void GpuEngine::set_act_models(const std::vector<MbkActModel>& models,
                               const std::vector<MbkActModel>& opp_models) {
  if (running_.load()) throw std::runtime_error("set_act_models: engine running");
  if (!models.empty() && (int)models.size() != cfg_.n_lanes)
    throw std::runtime_error("set_act_models: need one model per lane");
  if (!models.empty() && (buf_.ep_return || buf_.ep_step || buf_.last_action0 || buf_.logits))
    throw std::runtime_error("set_act_models: not with reference buffer keys");
  const bool sp_needed = !models.empty() && cfg_.selfplay_groups > 0;
  if (sp_needed && (int)opp_models.size() != cfg_.n_lanes)
    throw std::runtime_error("set_act_models: self-play needs one opponent block per lane");
  if (!sp_needed && !opp_models.empty())
    throw std::runtime_error("set_act_models: opponent blocks without self-play groups");
  for (const std::vector<MbkActModel>* v : {&models, &opp_models})
    for (const MbkActModel& m : *v)
      if (m.E != cfg_.envs_per_group || m.H != cfg_.size || m.W != cfg_.size)
        throw std::runtime_error("set_act_models: model block shape mismatch");
  act_models_ = models;
  opp_act_models_ = opp_models;
  // sparse rows in / out of pinned host memory, read / written by the kernels themselves
  // (dense codes / actions cost 4 + 4 MB of PCIe per 8192-env step instead of ~0.5-1 MB)
  sparse_ = !models.empty();
  if (sparse_) alloc_rows();
  if (sp_needed) {
    const size_t E = cfg_.envs_per_group, sc = E * S_ * (4 + 12 + 8) + 2 * E * 4 + 256;
    for (Lane& L : lanes_)
      if (!L.opp_scratch && hipMalloc((void**)&L.opp_scratch, sc) != hipSuccess)
        throw std::runtime_error("set_act_models: hipMalloc of the opponent scratch failed");
  }
}

void GpuEngine::stop() {
  running_.store(false);
  work_cv_.notify_all();
  full_cv_.notify_all();
  if (driver_.joinable()) driver_.join();
  for (auto& t : workers_) if (t.joinable()) t.join();
  workers_.clear();
  for (Lane& L : lanes_)
    if (L.stream) hipStreamSynchronize(L.stream);
}

void GpuEngine::dispatch_env(int g) {
  Group& G = *groups_[g];
  const auto now = std::chrono::steady_clock::now();
  gpu_phase_ns_.fetch_add(
      std::chrono::duration_cast<std::chrono::nanoseconds>(now - G.t_phase).count(),
      std::memory_order_relaxed);
  G.t_phase = now;
  if (G.timed) {  // the step's events are complete (G.ev, recorded after them, is)
    float ms[3] = {0.f, 0.f, 0.f};
    bool ok = true;
    for (int i = 0; i < 3; ++i)
      ok = ok && hipEventElapsedTime(&ms[i], G.tev[i], G.tev[i + 1]) == hipSuccess;
    if (ok) {
      step_h2d_ns_.fetch_add((int64_t)(ms[0] * 1e6), std::memory_order_relaxed);
      step_graph_ns_.fetch_add((int64_t)(ms[1] * 1e6), std::memory_order_relaxed);
      step_out_ns_.fetch_add((int64_t)(ms[2] * 1e6), std::memory_order_relaxed);
      timed_steps_.fetch_add(1, std::memory_order_relaxed);
    }
    G.timed = false;
  }
  G.idle.store(0, std::memory_order_relaxed);
  G.phase.store(ENV_BUSY, std::memory_order_release);
  G.remaining.store(cfg_.envs_per_group, std::memory_order_release);
  G.next_env.store(0, std::memory_order_release);
  {
    std::lock_guard<std::mutex> l(work_m_);
    work_epoch_.fetch_add(1);
  }
  work_cv_.notify_all();
}

void GpuEngine::worker_loop(int wid) {
  const int E = cfg_.envs_per_group, NG = cfg_.n_groups;
  while (running_.load(std::memory_order_relaxed)) {
    const uint64_t epoch = work_epoch_.load();
    bool did = false;
    for (int k = 0; k < NG; ++k) {
      const int g = (wid + k) % NG;
      Group& G = *groups_[g];
      if (G.phase.load(std::memory_order_acquire) != ENV_BUSY) continue;
      for (;;) {
        int e = G.next_env.fetch_add(chunk_);
        if (e >= E) break;
        int e1 = std::min(e + chunk_, E);
        const int a0 = g * E;
        auto t0 = std::chrono::steady_clock::now();
        try {
          if (inject_fault_.exchange(0) != 0)
            throw std::runtime_error("injected env-worker fault (--fault_inject_every)");
          if (sparse_ && G.selfplay)
            G.idle.fetch_add(env_->step_range_lists_sp(a0 + e, a0 + e1, h_act_list_,
                                                       h_act_list_p1_, h_code_list_,
                                                       h_code_list_p1_, list_stride_, h_reward_,
                                                       h_done_, &log_, G.opp_version),
                             std::memory_order_relaxed);
          else if (sparse_)
            G.idle.fetch_add(env_->step_range_lists(a0 + e, a0 + e1, h_act_list_, h_code_list_,
                                                    list_stride_, h_reward_, h_done_, &log_),
                             std::memory_order_relaxed);
          else if (G.selfplay)
            env_->step_range_codes_sp(a0 + e, a0 + e1, h_act16_, h_act16_p1_, h_codes_, h_res_,
                                      h_codes_p1_, h_res_p1_, h_reward_, h_done_, &log_,
                                      G.opp_version, h_ep_return_, h_ep_step_);
          else
            env_->step_range_codes(a0 + e, a0 + e1, h_act16_, h_codes_, h_res_, h_reward_,
                                   h_done_, &log_, h_ep_return_, h_ep_step_);
        } catch (const std::exception& ex) {
          // a failing env worker must not std::terminate the learner process: the engine
          // stops, get_full() wakes up, and Python (GpuActorRuntime.check) raises with this
          // message so the trainer can rebuild the actor side (train.py recovery)
          fail("env worker " + std::to_string(wid) + ": " + ex.what());
          return;
        }
        env_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now() - t0).count(),
                          std::memory_order_relaxed);
        frames_.fetch_add(e1 - e, std::memory_order_relaxed);
        did = true;
        if (G.remaining.fetch_sub(e1 - e) == e1 - e) {
          G.t_ready_ns.store(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                 std::chrono::steady_clock::now().time_since_epoch()).count(),
                             std::memory_order_relaxed);
          G.phase.store(READY, std::memory_order_release);
        }
      }
    }
    if (!did) {
      std::unique_lock<std::mutex> l(work_m_);
      work_cv_.wait_for(l, std::chrono::milliseconds(2),
                        [&] { return work_epoch_.load() != epoch || !running_.load(); });
    }
  }
}

bool GpuEngine::enqueue_gpu(int g) {
  const auto t_enq = std::chrono::steady_clock::now();
  struct Timer {  // adds the enqueue's duration on every exit path
    std::atomic<int64_t>& acc;
    std::chrono::steady_clock::time_point t0;
    ~Timer() {
      acc.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now() - t0).count(),
                    std::memory_order_relaxed);
    }
  } timer{enqueue_ns_, t_enq};
  Group& G = *groups_[g];
  Lane& L = lanes_[G.lane];
  hipStream_t st = L.stream;
  const LaneIO& io = L.io;
  const size_t E = cfg_.envs_per_group, T = cfg_.unroll;
  {  // apply pending weight publishes to this lane between two of its inference steps
    std::lock_guard<std::mutex> l(pub_m_);
    const int ln = G.lane;
    for (int c = 0; c < 2; ++c) {
      PubChan& P = pub_[c];
      if (!P.pending[ln]) continue;
      // not before the staging copy has executed: the learner's thread publishes as soon as
      // it has queued an update, and a stream wait here would hold this lane's policy steps
      // (every group on it) until that whole update is done; a later step applies it
      if (hipEventQuery(P.ready) == hipErrorNotReady) continue;
      ENG_CHECK(hipStreamWaitEvent(st, P.ready, 0));
      ENG_CHECK(hipMemcpyAsync((void*)P.dst[ln], P.staging, P.n, hipMemcpyDeviceToDevice,
                               st));
      ENG_CHECK(hipEventRecord(P.consumed[ln], st));
      if (L.pack_graph[c]) ENG_CHECK(hipGraphLaunch(L.pack_graph[c], st));
      P.pending[ln] = false;
      if (c == 1) L.opp_version = P.version;
      else if (P.version >= 0) L.policy_version = P.version;
      bool all = true;
      for (bool pl : P.pending) all = all && !pl;
      if (all) {  // landed on every lane
        if (c == 0) publishes_.fetch_add(1);
        else {
          opp_version_pub_.store(P.version);
          opp_publishes_.fetch_add(1);
        }
      }
    }
  }
  if (G.t == 0) {
    // free slots go to waiting groups in FIFO order: without it the group scanned first
    // would take every released slot and starve the others when the learner is the
    // bottleneck (and a starved lane would never apply weight publishes)
    auto waiting = [&] {
      for (int w : slot_wait_q_) if (w == g) return true;
      return false;
    };
    if (!slot_wait_q_.empty() && slot_wait_q_.front() != g) {
      if (!waiting()) slot_wait_q_.push_back(g);
      return false;
    }
    int slot = -1;
    bool pending = false;  // read under slot_m_: release() updates the flags from another thread
    {
      std::lock_guard<std::mutex> l(slot_m_);
      // the first free slot whose release has executed on the GPU: a slot the learner
      // released right after queueing its update would make this lane's stream wait for the
      // whole update (the learner's thread no longer blocks mid-update); the group waits
      // on the host instead while the lane's other groups keep acting
      for (auto it = free_slots_.begin(); it != free_slots_.end(); ++it) {
        const int s = *it;
        if (release_pending_[s]) {
          const hipError_t q = hipEventQuery(release_ev_[s]);
          if (q == hipErrorNotReady) continue;
          if (q == hipSuccess) release_pending_[s] = 0;
        }
        slot = s;
        pending = release_pending_[s] != 0;
        free_slots_.erase(it);
        break;
      }
    }
    if (slot < 0) {  // learner-bound: wait for a released slot
      if (!waiting()) slot_wait_q_.push_back(g);
      return false;
    }
    if (!slot_wait_q_.empty() && slot_wait_q_.front() == g) slot_wait_q_.pop_front();
    if (pending) ENG_CHECK(hipStreamWaitEvent(st, release_ev_[slot], 0));
    G.cur = slot;
    slot_version_[slot] = L.policy_version;
  }
  const size_t e0 = (size_t)g * E;
  G.timed = step_timing_;
  const size_t t = G.t;
  auto obs_at = [&](int slot, size_t i) {
    return (char*)buf_.obs + slot * slot_stride_obs_ + i * E * S_ * 4;
  };
  auto mask_at = [&](int slot, size_t i) {
    return (char*)buf_.mask + slot * slot_stride_mask_ + i * E * S_ * 4 * kMaskWords;
  };
  auto act_at = [&](int slot, size_t i) {
    return (char*)buf_.action + slot * slot_stride_act_ + i * E * S_ * kActComps;
  };
  auto f32_at = [&](uintptr_t base, int slot, size_t i) {
    return (char*)base + (slot * slot_stride_scalar_ + i * E) * 4;
  };
  auto u8_at = [&](uintptr_t base, int slot, size_t i) {
    return (char*)base + (slot * slot_stride_scalar_ + i * E);
  };
  const bool close_prev = (t == 0 && G.prev >= 0);
  // the step that just finished (its reward / done rows): the last row of this slot, or of the
  // previous slot at t == 0
  const int rs = t > 0 ? G.cur : G.prev;
  const size_t ri = t > 0 ? t - 1 : T - 1;
  if (act_mode()) {
    // fused acting step: 2 launches decode the codes, run the trunk, sample, and write the
    // rollout row (obs, mask, action, log-prob, value, previous reward / done) in place
    const MbkActModel& M = act_models_[G.lane];
    if (G.timed) ENG_CHECK(hipEventRecord(G.tev[0], st));
    if (G.timed) ENG_CHECK(hipEventRecord(G.tev[1], st));
    MbkActStep a{};
    a.code_list = h_code_list_ + e0 * list_stride_;
    a.act_list = h_act_list_ + e0 * list_stride_;
    a.list_stride = list_stride_;
    a.obs = (uint32_t*)obs_at(G.cur, t);
    a.mask = (uint32_t*)mask_at(G.cur, t);
    if (close_prev) {  // this row is also the previous slot's bootstrap row T
      a.obs2 = (uint32_t*)obs_at(G.prev, T);
      a.mask2 = (uint32_t*)mask_at(G.prev, T);
    }
    a.action = (uint8_t*)act_at(G.cur, t);
    if (buf_.abits) {  // [slot][T+1][E][S/32]
      const size_t sw = (size_t)(S_ + 31) / 32;
      auto ab_at = [&](int slot, size_t i) {
        return (uint32_t*)buf_.abits + (slot * slot_stride_scalar_ + i * E) * sw;
      };
      a.abits = ab_at(G.cur, t);
      if (close_prev) a.abits2 = ab_at(G.prev, T);
    }
    a.logp = (float*)f32_at(buf_.logp, G.cur, t);
    a.value = (float*)f32_at(buf_.value, G.cur, t);
    if (!G.first) {
      a.reward_src = h_reward_ + e0;
      a.done_src = h_done_ + e0;
      a.reward_dst = (float*)f32_at(buf_.reward, rs, ri);
      a.done_dst = (uint8_t*)u8_at(buf_.done, rs, ri);
    }
    a.step = L.act_step++;
    act_active_cells_.fetch_add(G.idle.load(std::memory_order_relaxed), std::memory_order_relaxed);
    act_steps_.fetch_add(1, std::memory_order_relaxed);
    {
      const auto t0 = std::chrono::steady_clock::now();
      ENG_CHECK((hipError_t)mbk_act_step(&M, &a, st));
      if (G.selfplay) {  // the opponent acts on its own (mirrored) rows with its own weights
        const size_t ES = E * S_;
        uint8_t* sc = L.opp_scratch;
        MbkActStep o{};
        o.code_list = h_code_list_p1_ + e0 * list_stride_;
        o.act_list = h_act_list_p1_ + e0 * list_stride_;
        o.list_stride = list_stride_;
        o.obs = (uint32_t*)sc;
        o.mask = (uint32_t*)(sc + ES * 4);
        o.action = sc + ES * 16;
        o.logp = (float*)(sc + ES * 24);
        o.value = (float*)(sc + ES * 24 + E * 4);
        o.step = L.opp_act_step++;
        ENG_CHECK((hipError_t)mbk_act_step(&opp_act_models_[G.lane], &o, st));
        G.opp_version = L.opp_version;
      }
      launch_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now() - t0).count(),
                           std::memory_order_relaxed);
    }
    if (G.timed) ENG_CHECK(hipEventRecord(G.tev[2], st));
    if (close_prev) {
      ENG_CHECK(hipEventRecord(full_ev_[G.prev], st));
      {
        std::lock_guard<std::mutex> l(slot_m_);
        full_slots_.push_back(G.prev);
      }
      slots_full_.fetch_add(1);
      full_cv_.notify_all();
      G.prev = -1;
    }
    if (G.timed) ENG_CHECK(hipEventRecord(G.tev[3], st));
    ENG_CHECK(hipEventRecord(G.ev, st));
  } else {
    // captured-graph step (other map sizes / agents, fp8 acting, the reference buffer keys)
    const uintptr_t in_codes = io.in_codes, in_res = io.in_res, out_act16 = io.out_act16;
    if (G.timed) ENG_CHECK(hipEventRecord(G.tev[0], st));
    if (sparse_) {  // occupied-cell rows -> the graph's dense codes (no blit copy)
      ENG_CHECK((hipError_t)mbk_rows_to_codes(h_code_list_ + e0 * list_stride_, list_stride_,
                                              (int)E, S_, (void*)in_codes, (int32_t*)in_res,
                                              st));
    } else {
      ENG_CHECK(hipMemcpyAsync((void*)in_codes, h_codes_ + e0 * S_, E * S_ * 2,
                               hipMemcpyHostToDevice, st));
      ENG_CHECK(hipMemcpyAsync((void*)in_res, h_res_ + e0, E * 4, hipMemcpyHostToDevice, st));
    }
    if (G.timed) ENG_CHECK(hipEventRecord(G.tev[1], st));
    {
      const auto t0 = std::chrono::steady_clock::now();
      ENG_CHECK(hipGraphLaunch(L.graph, st));
      launch_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now() - t0).count(),
                           std::memory_order_relaxed);
    }
    if (G.selfplay) {  // the opponent acts on its own (mirrored) view with its own weights
      if (sparse_) {
        ENG_CHECK((hipError_t)mbk_rows_to_codes(h_code_list_p1_ + e0 * list_stride_,
                                                list_stride_, (int)E, S_, (void*)io.in_codes_p1,
                                                (int32_t*)io.in_res_p1, st));
      } else {
        ENG_CHECK(hipMemcpyAsync((void*)io.in_codes_p1, h_codes_p1_ + e0 * S_, E * S_ * 2,
                                 hipMemcpyHostToDevice, st));
        ENG_CHECK(hipMemcpyAsync((void*)io.in_res_p1, h_res_p1_ + e0, E * 4,
                                 hipMemcpyHostToDevice, st));
      }
      ENG_CHECK(hipGraphLaunch(L.opp_graph, st));
      G.opp_version = L.opp_version;
    }

    if (G.timed) ENG_CHECK(hipEventRecord(G.tev[2], st));
    // scatter this step into the HBM rollout slot(s)
    MbkCopySeg seg[MBK_MAX_COPY_SEGS];
    int n = 0;
    seg[n++] = {(const void*)io.in_obs, obs_at(G.cur, t), E * S_ * 4};
    seg[n++] = {(const void*)io.in_mask, mask_at(G.cur, t), E * S_ * 4 * kMaskWords};
    seg[n++] = {(const void*)io.out_action, act_at(G.cur, t), E * S_ * kActComps};
    seg[n++] = {(const void*)io.out_logp, f32_at(buf_.logp, G.cur, t), E * 4};
    seg[n++] = {(const void*)io.out_value, f32_at(buf_.value, G.cur, t), E * 4};
    if (!G.first) {
      // reward / done of the env step that just finished, read by the scatter kernel straight
      // from pinned host memory (two fewer blit launches per step); the group's envs do not
      // write them again before G.ev, which is recorded after this kernel
      seg[n++] = {(const void*)(h_reward_ + e0), f32_at(buf_.reward, rs, ri), E * 4};
      seg[n++] = {(const void*)(h_done_ + e0), u8_at(buf_.done, rs, ri), E};
      if (buf_.ep_return)
        seg[n++] = {(const void*)(h_ep_return_ + e0), f32_at(buf_.ep_return, rs, ri), E * 4};
      if (buf_.ep_step)
        seg[n++] = {(const void*)(h_ep_step_ + e0), f32_at(buf_.ep_step, rs, ri), E * 4};
    }
    if (buf_.logits && io.out_logits)
      seg[n++] = {(const void*)io.out_logits,
                  (char*)buf_.logits + (G.cur * slot_stride_scalar_ + t * E) * (size_t)S_ * 78 * 4,
                  E * (size_t)S_ * 78 * 4};
    if (close_prev && buf_.last_action0)  // the action taken just before this slot's row 0
      seg[n++] = {(const void*)act_at(G.prev, T - 1),
                  (char*)buf_.last_action0 + (size_t)G.cur * E * S_ * kActComps,
                  E * S_ * kActComps};
    if (close_prev) {
      seg[n++] = {(const void*)io.in_obs, obs_at(G.prev, T), E * S_ * 4};
      seg[n++] = {(const void*)io.in_mask, mask_at(G.prev, T), E * S_ * 4 * kMaskWords};
    }
    ENG_CHECK((hipError_t)mbk_multi_copy(seg, n, st));
    if (close_prev) {
      ENG_CHECK(hipEventRecord(full_ev_[G.prev], st));
      {
        std::lock_guard<std::mutex> l(slot_m_);
        full_slots_.push_back(G.prev);
      }
      slots_full_.fetch_add(1);
      full_cv_.notify_all();
      G.prev = -1;
    }
    if (sparse_) {  // packed actions -> the env workers' non-noop action rows
      ENG_CHECK((hipError_t)mbk_codes_to_rows((const void*)out_act16, (int)E, S_,
                                              h_act_list_ + e0 * list_stride_, list_stride_,
                                              st));
      if (G.selfplay)
        ENG_CHECK((hipError_t)mbk_codes_to_rows((const void*)io.out_act16_p1, (int)E, S_,
                                                h_act_list_p1_ + e0 * list_stride_,
                                                list_stride_, st));
    } else {
      ENG_CHECK(hipMemcpyAsync(h_act16_ + e0 * S_, (const void*)out_act16, E * S_ * 2,
                               hipMemcpyDeviceToHost, st));
      if (G.selfplay)
        ENG_CHECK(hipMemcpyAsync(h_act16_p1_ + e0 * S_, (const void*)io.out_act16_p1,
                                 E * S_ * 2, hipMemcpyDeviceToHost, st));
    }
    if (G.timed) ENG_CHECK(hipEventRecord(G.tev[3], st));
    ENG_CHECK(hipEventRecord(G.ev, st));
  }
  gpu_steps_.fetch_add(1);
  G.t += 1;
  if (G.t == (int)T) {
    G.t = 0;
    G.prev = G.cur;
    G.cur = -1;
  }
  G.first = false;
  {
    const auto now = std::chrono::steady_clock::now();
    const int64_t rdy = G.t_ready_ns.exchange(0, std::memory_order_relaxed);
    if (rdy > 0)  // env phase: dispatch -> last env of the group stepped
      env_phase_ns_.fetch_add(
          rdy - std::chrono::duration_cast<std::chrono::nanoseconds>(
                    G.t_phase.time_since_epoch()).count(),
          std::memory_order_relaxed);
    G.t_phase = now;
  }
  G.phase.store(ON_GPU, std::memory_order_release);
  return true;
}

void GpuEngine::driver_loop() {
  hipSetDevice(cfg_.device);
  const int NG = cfg_.n_groups;
  int idle_spins = 0;
  auto idle_t0 = std::chrono::steady_clock::now();
  bool idle = false;
  double stall_s = 0.0;
  while (running_.load(std::memory_order_relaxed)) {
    bool progressed = false, stalled = false;
    for (int g = 0; g < NG && running_.load(std::memory_order_relaxed); ++g) {
      Group& G = *groups_[g];
      int ph = G.phase.load(std::memory_order_acquire);
      if (ph == READY) {
        if (enqueue_gpu(g)) progressed = true;
        else if (failed_.load()) return;
        else stalled = true;
      } else if (ph == ON_GPU) {
        hipError_t q = hipEventQuery(G.ev);
        if (q == hipSuccess) {
          dispatch_env(g);
          progressed = true;
        } else if (q != hipErrorNotReady) {
          fail(std::string("hipEventQuery: ") + hipGetErrorString(q));
          return;
        }
      }
    }
    if (progressed) {
      if (idle) {
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - idle_t0).count();
        std::lock_guard<std::mutex> l(stats_m_);
        driver_idle_s_ += dt;
        if (stall_s > 0) slot_wait_s_ += dt;
      }
      idle = false;
      idle_spins = 0;
      stall_s = 0.0;
    } else {
      if (!idle) { idle = true; idle_t0 = std::chrono::steady_clock::now(); }
      if (stalled) stall_s = 1.0;
      if (++idle_spins < 256) {
        __builtin_ia32_pause();
      } else if (idle_spins < 2048) {
        std::this_thread::yield();
      } else {
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
  }
}

std::vector<int> GpuEngine::get_full(int n, double timeout_s) {
  std::unique_lock<std::mutex> l(slot_m_);
  auto pred = [&] { return (int)full_slots_.size() >= n || !running_.load() || failed_.load(); };
  if (timeout_s < 0) full_cv_.wait(l, pred);
  else full_cv_.wait_for(l, std::chrono::duration<double>(timeout_s), pred);
  std::vector<int> out;
  if ((int)full_slots_.size() < n) return out;
  for (int i = 0; i < n; ++i) { out.push_back(full_slots_.front()); full_slots_.pop_front(); }
  return out;
}

void GpuEngine::stream_wait_full(uintptr_t stream, int slot) {
  hipError_t e = hipStreamWaitEvent((hipStream_t)stream, full_ev_[slot], 0);
  if (e != hipSuccess) throw std::runtime_error(std::string("stream_wait_full: ") + hipGetErrorString(e));
}

void GpuEngine::release(const std::vector<int>& slots, uintptr_t stream) {
  for (int s : slots) {
    hipError_t e = hipEventRecord(release_ev_[s], (hipStream_t)stream);
    if (e != hipSuccess) throw std::runtime_error(std::string("release: ") + hipGetErrorString(e));
  }
  std::lock_guard<std::mutex> l(slot_m_);
  for (int s : slots) {
    release_pending_[s] = 1;
    free_slots_.push_back(s);
  }
}

bool GpuEngine::publish_chan(int chan, uintptr_t src, const std::vector<uintptr_t>& dsts,
                             size_t nbytes, uintptr_t stream, int version) {
  std::lock_guard<std::mutex> l(pub_m_);
  PubChan& P = pub_[chan];
  if ((int)dsts.size() != cfg_.n_lanes)
    throw std::runtime_error("publish: need one destination per lane");
  for (bool pl : P.pending)
    if (pl) return false;  // previous version not applied on every lane yet: skip this one
  hipStream_t s = (hipStream_t)stream;
  if (nbytes > P.staging_n) {
    // first publish (or growth): synchronous realloc is fine outside the hot loop
    if (P.staging) {
      for (Lane& L : lanes_) hipStreamSynchronize(L.stream);
      hipFree(P.staging);
    }
    if (hipMalloc((void**)&P.staging, nbytes) != hipSuccess)
      throw std::runtime_error("publish: hipMalloc staging failed");
    P.staging_n = nbytes;
  }
  // staging is reused only after every lane's previous copy-out has executed
  for (hipEvent_t ev : P.consumed) hipStreamWaitEvent(s, ev, 0);
  hipMemcpyAsync(P.staging, (const void*)src, nbytes, hipMemcpyDeviceToDevice, s);
  hipEventRecord(P.ready, s);
  P.dst = dsts;
  P.n = nbytes;
  P.version = version;
  P.pending.assign(cfg_.n_lanes, true);
  return true;
}

EngineStats GpuEngine::stats() const {
  EngineStats s;
  s.frames = frames_.load();
  s.gpu_steps = gpu_steps_.load();
  s.slots_full = slots_full_.load();
  s.env_s = env_ns_.load() * 1e-9;
  s.gpu_phase_s = gpu_phase_ns_.load() * 1e-9;
  s.step_h2d_s = step_h2d_ns_.load() * 1e-9;
  s.step_graph_s = step_graph_ns_.load() * 1e-9;
  s.step_out_s = step_out_ns_.load() * 1e-9;
  s.timed_steps = timed_steps_.load();
  s.preroll_steps = preroll_steps_;
  s.env_phase_s = env_phase_ns_.load() * 1e-9;
  s.enqueue_s = enqueue_ns_.load() * 1e-9;
  s.graph_launch_s = launch_ns_.load() * 1e-9;
  s.publishes = publishes_.load();
  s.opp_publishes = opp_publishes_.load();
  s.opp_version = opp_version_pub_.load();
  s.act_steps = act_steps_.load();
  s.act_active_cells = act_active_cells_.load();
  {
    std::lock_guard<std::mutex> q(slot_m_);
    s.full_depth = (int)full_slots_.size();
  }
  std::lock_guard<std::mutex> l(stats_m_);
  s.driver_idle_s = driver_idle_s_;
  s.slot_wait_s = slot_wait_s_;
  return s;
}

}  // namespace mb
