// pybind11 bindings of the native runtime (_mbrt). Buffers cross the boundary
// as raw addresses (torch tensor .data_ptr()), so the same calls work on
// pinned host tensors, shared-memory tensors and numpy arrays; every
// potentially long call releases the GIL.
#include <cstring>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>

#include <hip/hip_runtime_api.h>

#include "engine.h"
#include "shm_ring.h"
#include "vec_env.h"

namespace py = pybind11;
using namespace mb;

namespace {

template <typename T>
T* P(uintptr_t a) { return reinterpret_cast<T*>(a); }

struct PyVecEnv {
  std::unique_ptr<VecEnv> env;
  EpisodeLog log;
  PyVecEnv(int size, int n, int max_steps, uint64_t seed, std::vector<int> bots,
           std::vector<float> rw, int base)
      : env(new VecEnv(size, n, max_steps, seed, bots, rw.empty() ? nullptr : rw.data(), base)) {}
};

py::list records_to_list(const std::vector<EpisodeRecord>& recs) {
  py::list out;
  for (const auto& r : recs) out.append(py::make_tuple(r.ep_return, r.ep_step, r.env_index, r.winner, r.opponent));
  return out;
}

}  // namespace

PYBIND11_MODULE(_mbrt, m) {
  m.doc() = "microbeast_amd native runtime";
  m.attr("PLANES") = kPlanes;
  m.attr("MASK_BITS") = kMaskBits;
  m.attr("MASK_WORDS") = kMaskWords;
  m.attr("ACT_COMPS") = kActComps;
  m.attr("NVEC") = std::vector<int>(kNvec, kNvec + kActComps);
  py::dict bots;
  bots["coac"] = (int)BOT_COAC;
  bots["random_biased"] = (int)BOT_RANDOM_BIASED;
  bots["light_rush"] = (int)BOT_LIGHT_RUSH;
  bots["worker_rush"] = (int)BOT_WORKER_RUSH;
  bots["passive"] = (int)BOT_PASSIVE;
  bots["random"] = (int)BOT_RANDOM;
  m.attr("BOTS") = bots;

  py::class_<PyVecEnv>(m, "VecEnv")
      .def(py::init<int, int, int, uint64_t, std::vector<int>, std::vector<float>, int>(),
           py::arg("size"), py::arg("n_envs"), py::arg("max_steps"), py::arg("seed"),
           py::arg("bots") = std::vector<int>{}, py::arg("reward_weight") = std::vector<float>{},
           py::arg("env_index_base") = 0)
      .def_property_readonly("num_envs", [](PyVecEnv& e) { return e.env->num_envs(); })
      .def_property_readonly("size", [](PyVecEnv& e) { return e.env->size(); })
      .def("reset",
           [](PyVecEnv& e, uintptr_t obs, uintptr_t mask) {
             py::gil_scoped_release g;
             e.env->reset(P<uint32_t>(obs), P<uint32_t>(mask));
           })
      .def("step",
           [](PyVecEnv& e, uintptr_t act, uintptr_t obs, uintptr_t mask, uintptr_t rew,
              uintptr_t done, uintptr_t ep_ret, uintptr_t ep_step) {
             py::gil_scoped_release g;
             e.env->step_range(0, e.env->num_envs(), 0, P<uint8_t>(act), P<uint32_t>(obs),
                               P<uint32_t>(mask), P<float>(rew), P<uint8_t>(done),
                               P<float>(ep_ret), P<int32_t>(ep_step), &e.log);
           },
           py::arg("actions"), py::arg("obs"), py::arg("mask"), py::arg("reward"),
           py::arg("done"), py::arg("ep_return") = 0, py::arg("ep_step") = 0)
      .def("dense_obs", [](PyVecEnv& e, uintptr_t out) { e.env->dense_obs(P<float>(out)); })
      .def("dense_mask", [](PyVecEnv& e, uintptr_t out) { e.env->dense_mask(P<uint8_t>(out)); })
      .def("drain_episodes", [](PyVecEnv& e) { return records_to_list(e.log.drain()); })
      .def("set_bot", [](PyVecEnv& e, int i, int bot) { e.env->sim(i).set_bot(bot); })
      .def("bot", [](PyVecEnv& e, int i) { return e.env->sim(i).bot(); })
      .def("preroll",
           [](PyVecEnv& e, int max_pre, uint64_t seed, int n_threads) {
             py::gil_scoped_release g;
             return e.env->preroll(max_pre, seed, n_threads);
           },
           py::arg("max_pre"), py::arg("seed"), py::arg("n_threads") = 1)
      .def("set_external_opponent",
           [](PyVecEnv& e, bool on) {
             for (int i = 0; i < e.env->num_envs(); ++i) e.env->sim(i).set_external_opponent(on);
           })
      .def("obs_p1",
           [](PyVecEnv& e, uintptr_t out) {
             const size_t S = (size_t)e.env->size() * e.env->size();
             for (int i = 0; i < e.env->num_envs(); ++i)
               e.env->sim(i).write_obs_p1(P<uint32_t>(out) + i * S);
           })
      .def("mask_p1",
           [](PyVecEnv& e, uintptr_t out) {
             const size_t S = (size_t)e.env->size() * e.env->size();
             for (int i = 0; i < e.env->num_envs(); ++i)
               e.env->sim(i).write_mask_p1(P<uint32_t>(out) + i * S * kMaskWords);
           })
      .def("set_opponent_actions",
           [](PyVecEnv& e, uintptr_t act) {
             const size_t S = (size_t)e.env->size() * e.env->size();
             for (int i = 0; i < e.env->num_envs(); ++i)
               e.env->sim(i).set_opponent_actions(P<uint8_t>(act) + i * S * kActComps);
           })
      .def("ticks", [](PyVecEnv& e, int i) { return e.env->sim(i).ticks(); })
      .def("set_validate", [](PyVecEnv& e, bool on) { e.env->set_validate(on); })
      .def("obs_codes",
           [](PyVecEnv& e, uintptr_t codes, uintptr_t res) {
             const size_t S = (size_t)e.env->size() * e.env->size();
             for (int i = 0; i < e.env->num_envs(); ++i) {
               e.env->sim(i).write_obs_codes(P<uint16_t>(codes) + i * S);
               P<int32_t>(res)[i] = e.env->sim(i).resources(0);
             }
           })
      .def("set_external_opponent_range",
           [](PyVecEnv& e, int e0, int e1, bool on) { e.env->set_external_opponent(e0, e1, on); })
      .def("obs_codes_p1",
           [](PyVecEnv& e, uintptr_t codes, uintptr_t res) {
             const size_t S = (size_t)e.env->size() * e.env->size();
             for (int i = 0; i < e.env->num_envs(); ++i) {
               e.env->sim(i).write_obs_codes_as(1, P<uint16_t>(codes) + i * S);
               P<int32_t>(res)[i] = e.env->sim(i).resources(1);
             }
           })
      .def("step_codes_sp",
           [](PyVecEnv& e, uintptr_t act16, uintptr_t opp16, uintptr_t codes, uintptr_t res,
              uintptr_t codes_p1, uintptr_t res_p1, uintptr_t rew, uintptr_t done, int opponent) {
             py::gil_scoped_release g;
             e.env->step_range_codes_sp(0, e.env->num_envs(), P<uint16_t>(act16),
                                        P<uint16_t>(opp16), P<uint16_t>(codes), P<int32_t>(res),
                                        P<uint16_t>(codes_p1), P<int32_t>(res_p1), P<float>(rew),
                                        P<uint8_t>(done), &e.log, opponent);
           })
      .def("step_codes",
           [](PyVecEnv& e, uintptr_t act16, uintptr_t codes, uintptr_t res, uintptr_t rew,
              uintptr_t done) {
             py::gil_scoped_release g;
             e.env->step_range_codes(0, e.env->num_envs(), P<uint16_t>(act16), P<uint16_t>(codes),
                                     P<int32_t>(res), P<float>(rew), P<uint8_t>(done), &e.log);
           })
      // sparse rows (the engine's fused-step form): code_lists(player) and the self-play step
      .def("code_lists",
           [](PyVecEnv& e, uintptr_t lists, int stride, int player) {
             e.env->write_code_lists(P<uint32_t>(lists), stride, player);
           },
           py::arg("lists"), py::arg("stride"), py::arg("player") = 0)
      .def("step_lists_sp",
           [](PyVecEnv& e, uintptr_t acts, uintptr_t opp_acts, uintptr_t lists,
              uintptr_t lists_p1, int stride, uintptr_t rew, uintptr_t done, int opponent) {
             py::gil_scoped_release g;
             return e.env->step_range_lists_sp(0, e.env->num_envs(), P<uint32_t>(acts),
                                               P<uint32_t>(opp_acts), P<uint32_t>(lists),
                                               P<uint32_t>(lists_p1), stride, P<float>(rew),
                                               P<uint8_t>(done), &e.log, opponent);
           });

  py::class_<IndexRing>(m, "IndexRing")
      .def(py::init([](uintptr_t addr, size_t cap, bool init) {
             return new IndexRing(P<void>(addr), cap, init);
           }),
           py::arg("addr"), py::arg("capacity"), py::arg("init"))
      .def_static("bytes_needed", &IndexRing::bytes_needed)
      .def("try_push", &IndexRing::try_push)
      .def("try_pop",
           [](IndexRing& r) -> py::object {
             int64_t v;
             if (r.try_pop(&v)) return py::int_(v);
             return py::none();
           })
      .def("push",
           [](IndexRing& r, int64_t v, double timeout) {
             py::gil_scoped_release g;
             return r.push(v, timeout);
           },
           py::arg("value"), py::arg("timeout") = -1.0)
      .def("pop",
           [](IndexRing& r, double timeout) -> py::object {
             int64_t v;
             bool ok;
             {
               py::gil_scoped_release g;
               ok = r.pop(&v, timeout);
             }
             if (ok) return py::int_(v);
             return py::none();
           },
           py::arg("timeout") = -1.0)
      .def("size", &IndexRing::size)
      .def("capacity", &IndexRing::capacity)
      .def("close", &IndexRing::close)
      .def("closed", &IndexRing::closed);

  m.def("seqlock_write_begin",
        [](uintptr_t ver) { return seqlock_write_begin(P<std::atomic<uint64_t>>(ver)); });
  m.def("seqlock_write_end", [](uintptr_t ver) { seqlock_write_end(P<std::atomic<uint64_t>>(ver)); });
  m.def("seqlock_write",
        [](uintptr_t ver, uintptr_t src, uintptr_t dst, size_t n) {
          py::gil_scoped_release g;
          seqlock_write(P<std::atomic<uint64_t>>(ver), P<const void>(src), P<void>(dst), n);
        },
        py::arg("ver"), py::arg("src"), py::arg("dst"), py::arg("nbytes"));
  m.def("seqlock_read",
        [](uintptr_t ver, uintptr_t src, uintptr_t dst, size_t n, int tries) {
          py::gil_scoped_release g;
          return seqlock_read(P<const std::atomic<uint64_t>>(ver), P<const void>(src), P<void>(dst),
                              n, tries);
        },
        py::arg("ver"), py::arg("src"), py::arg("dst"), py::arg("nbytes"),
        py::arg("max_tries") = 1000);

  // Page-lock an existing host range (e.g. a POSIX shared-memory rollout slot written by
  // CPU actor processes) so hipMemcpyAsync moves it by DMA instead of staging through a
  // driver bounce buffer. Returns the hipError_t (0 = registered).
  m.def("host_register", [](uintptr_t addr, size_t nbytes) -> int {
    return (int)hipHostRegister(P<void>(addr), nbytes, hipHostRegisterDefault);
  });
  m.def("host_unregister", [](uintptr_t addr) -> int {
    return (int)hipHostUnregister(P<void>(addr));
  });
  // Strided DMA (hipMemcpy2DAsync): `height` rows of `width` bytes, e.g. one actor slot's
  // [T+1][row] rollout into column j of a time-major [T+1][B][row] learner batch, so the
  // batch lands in its final layout with no device-side transpose copy.
  m.def("memcpy2d_async", [](uintptr_t dst, size_t dpitch, uintptr_t src, size_t spitch,
                             size_t width, size_t height, uintptr_t stream) -> int {
    return (int)hipMemcpy2DAsync(P<void>(dst), dpitch, P<const void>(src), spitch, width, height,
                                 hipMemcpyDefault, (hipStream_t)stream);
  });

  py::class_<GpuEngine>(m, "GpuEngine")
      .def(py::init([](py::dict c, py::dict b) {
        EngineConfig cfg;
        cfg.size = c["size"].cast<int>();
        cfg.n_groups = c["n_groups"].cast<int>();
        cfg.envs_per_group = c["envs_per_group"].cast<int>();
        cfg.unroll = c["unroll"].cast<int>();
        cfg.n_slots = c["n_slots"].cast<int>();
        cfg.n_threads = c["n_threads"].cast<int>();
        cfg.max_steps = c["max_steps"].cast<int>();
        cfg.seed = c["seed"].cast<uint64_t>();
        cfg.bots = c["bots"].cast<std::vector<int>>();
        cfg.reward_weight = c["reward_weight"].cast<std::vector<float>>();
        cfg.env_index_base = c["env_index_base"].cast<int>();
        cfg.device = c["device"].cast<int>();
        if (c.contains("selfplay_groups")) cfg.selfplay_groups = c["selfplay_groups"].cast<int>();
        if (c.contains("n_lanes")) cfg.n_lanes = c["n_lanes"].cast<int>();
        if (c.contains("preroll")) cfg.preroll = c["preroll"].cast<int>();
        EngineBuffers buf;
        buf.obs = b["obs"].cast<uintptr_t>();
        buf.mask = b["mask"].cast<uintptr_t>();
        buf.action = b["action"].cast<uintptr_t>();
        buf.logp = b["logp"].cast<uintptr_t>();
        buf.value = b["value"].cast<uintptr_t>();
        buf.reward = b["reward"].cast<uintptr_t>();
        buf.done = b["done"].cast<uintptr_t>();
        auto opt = [&](const char* k) {
          return b.contains(k) ? b[k].cast<uintptr_t>() : (uintptr_t)0;
        };
        buf.ep_return = opt("ep_return");
        buf.ep_step = opt("ep_step");
        buf.last_action0 = opt("last_action0");
        buf.logits = opt("policy_logits");
        buf.abits = opt("abits");
        auto get = [](py::dict d, const char* k) {
          return d.contains(k) ? d[k].cast<uintptr_t>() : (uintptr_t)0;
        };
        for (auto item : b["lanes"].cast<py::list>()) {
          py::dict d = item.cast<py::dict>();
          LaneIO io;
          io.in_obs = get(d, "in_obs");
          io.in_mask = get(d, "in_mask");
          io.out_action = get(d, "out_action");
          io.out_logp = get(d, "out_logp");
          io.out_value = get(d, "out_value");
          io.in_codes = get(d, "in_codes");
          io.in_res = get(d, "in_res");
          io.out_act16 = get(d, "out_act16");
          io.in_codes_p1 = get(d, "in_codes_p1");
          io.in_res_p1 = get(d, "in_res_p1");
          io.out_act16_p1 = get(d, "out_act16_p1");
          io.out_logits = get(d, "out_logits");
          buf.lanes.push_back(io);
        }
        return new GpuEngine(cfg, buf);
      }))
      // graphs: one (policy, opp, pack, opp_pack) tuple of raw hipGraphExec_t per lane
      .def("start",
           [](GpuEngine& e, std::vector<std::vector<uintptr_t>> graphs) {
             std::vector<LaneGraphs> lg;
             for (const auto& t : graphs) {
               if (t.size() != 4)
                 throw std::runtime_error("start: need 4 graph handles per lane");
               lg.push_back(LaneGraphs{t[0], t[1], t[2], t[3]});
             }
             e.start(lg);
           })
      .def("stop", [](GpuEngine& e) { py::gil_scoped_release g; e.stop(); })
      .def("get_full",
           [](GpuEngine& e, int n, double timeout) {
             py::gil_scoped_release g;
             return e.get_full(n, timeout);
           },
           py::arg("n"), py::arg("timeout") = -1.0)
      .def("stream_wait_full", &GpuEngine::stream_wait_full)
      .def("release", &GpuEngine::release)
      .def("publish", &GpuEngine::publish, py::arg("src"), py::arg("dsts"), py::arg("nbytes"),
           py::arg("stream"), py::arg("version") = -1)
      .def("slot_version", &GpuEngine::slot_version)
      .def("set_policy_version", &GpuEngine::set_policy_version)
      .def("publish_opponent", &GpuEngine::publish_opponent)
      .def("set_initial_opponent", &GpuEngine::set_initial_opponent)
      .def("drain_episodes", [](GpuEngine& e) { return records_to_list(e.drain_episodes()); })
      .def("stream", &GpuEngine::stream, py::arg("lane") = 0)
      .def("failed", &GpuEngine::failed)
      .def("host_codes", &GpuEngine::host_codes)
      .def("host_res", &GpuEngine::host_res)
      .def("host_act16", &GpuEngine::host_act16)
      // fused acting steps: one packed MbkActModel (mbk_api.h, built by ops/act.py) per lane
      .def("set_act_models",
           [](GpuEngine& e, std::vector<py::bytes> blocks, std::vector<py::bytes> opp_blocks) {
             auto unpack = [](const std::vector<py::bytes>& bs) {
               std::vector<MbkActModel> ms;
               for (const py::bytes& b : bs) {
                 const std::string raw = b;
                 if (raw.size() != sizeof(MbkActModel))
                   throw std::runtime_error("set_act_models: block size " +
                                            std::to_string(raw.size()) +
                                            " != sizeof(MbkActModel) " +
                                            std::to_string(sizeof(MbkActModel)));
                 MbkActModel m;
                 std::memcpy(&m, raw.data(), sizeof(m));
                 ms.push_back(m);
               }
               return ms;
             };
             e.set_act_models(unpack(blocks), unpack(opp_blocks));
           },
           py::arg("blocks"),
           py::arg("opp_blocks") = std::vector<py::bytes>{})
      .def("act_mode", &GpuEngine::act_mode)
      .def("set_sparse_io", &GpuEngine::set_sparse_io)
      .def("sparse_io", &GpuEngine::sparse_io)
      .def_static("act_model_size", [] { return (int)sizeof(MbkActModel); })
      .def("inject_fault", &GpuEngine::inject_fault)
      // the pinned sparse code rows (word 0 = occupied cells | resources << 16): diagnostics
      .def("code_rows", [](GpuEngine& e) {
        return py::make_tuple((uintptr_t)e.host_code_list(), e.list_stride());
      })
      .def("error", &GpuEngine::error)
      .def("stats", [](GpuEngine& e) {
        EngineStats s = e.stats();
        py::dict d;
        d["frames"] = s.frames;
        d["gpu_steps"] = s.gpu_steps;
        d["slots_full"] = s.slots_full;
        d["full_depth"] = s.full_depth;
        d["driver_idle_s"] = s.driver_idle_s;
        d["gpu_phase_s"] = s.gpu_phase_s;
        d["step_h2d_s"] = s.step_h2d_s;
        d["step_graph_s"] = s.step_graph_s;
        d["step_out_s"] = s.step_out_s;
        d["timed_steps"] = s.timed_steps;
        d["env_phase_s"] = s.env_phase_s;
        d["enqueue_s"] = s.enqueue_s;
        d["graph_launch_s"] = s.graph_launch_s;
        d["act_steps"] = s.act_steps;
        d["act_active_cells"] = s.act_active_cells;
        d["slot_wait_s"] = s.slot_wait_s;
        d["env_s"] = s.env_s;
        d["publishes"] = s.publishes;
        d["opp_publishes"] = s.opp_publishes;
        d["opp_version"] = s.opp_version;
        d["preroll_steps"] = s.preroll_steps;
        return d;
      });
}
