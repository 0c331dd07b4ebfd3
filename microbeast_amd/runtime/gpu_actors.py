"""GPU actor runtime: native env workers + batched on-GPU policy inference.

Python side of ``csrc/runtime/engine.cpp``. Replaces the reference's actor
processes (microbeast.py:30-105, 179-191) and get_batch (libs/utils.py:166-218):

* rollout slots are allocated once in HBM, time-major ``[n_slots, T+1, E, ...]``
  with compact dtypes (obs uint32 bit planes, mask 3 x uint32 bits, actions
  uint8) — ~6 KB per 16x16 frame instead of ~170 KB in the reference layout;
* PCIe carries only 16-bit cell codes + the resource count in and one packed
  16-bit action per cell out (~1 KB per env step); the observation planes and
  the 78-bit action masks are derived on the GPU (``obs_mask.hip``);
* the policy step (encoder + head + masked sampling) for one env group is
  captured once into a hipGraph; the C++ driver thread replays it, so acting
  costs no Python and no GIL;
* the inference model is a separate parameter copy refreshed by an
  event-ordered D2D publish after each update (bounded policy lag);
* self-play (``selfplay_groups``): those groups' envs play an external opponent;
  a second captured graph runs the opponent policy (its own parameter copy, fed
  from the league's snapshot pool, ``runtime/league.py``) on the opponent's
  mirrored codes.
"""
from __future__ import annotations

import os

import torch

from .. import _native as N
from ..ops import act as act_ops
from ..ops.pixconv import pbc_to_cell_major
from ..ops import cell_head
from ..ops.copy import zeros
from ..ops.optim import FlatParams

BOT_IDS = {"coac": 0, "random_biased": 1, "light_rush": 2, "worker_rush": 3, "passive": 4,
           "random": 5}
# reference libs/utils.py:69-72: 3x coacAI, randomBiasedAI, lightRushAI, workerRushAI
DEFAULT_BOTS = ("coac", "coac", "coac", "random_biased", "light_rush", "worker_rush")


def available_cpus() -> int:
    """CPUs this process may use (affinity and cgroup quota aware)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            if q != "max":
                n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


class EngineFailure(RuntimeError):
    """The native engine stopped (an env worker raised, or a HIP call failed); the learner
    process is intact and may rebuild the actor side (train.py)."""


def graph_policy_step(io: dict, m, rng: torch.Tensor, E: int, size: int, device) -> None:
    """The captured graph's policy step (6 launches for the flat agent: decode + bucket, stage-0
    conv, trunk, network.5 + critic, head, finale) on fixed-address I/O ``io`` (``make_io``).
    The fused two-launch step (ops/act.py) is pinned bit-identical to it."""
    k = N.kernels()
    st = N.stream_ptr()
    # sparse-head models (flat IMPALA head) bucket their active pairs in the decode pass;
    # dense-head models (GridNet) sample with the masked-cell kernel
    hip = hasattr(m, "_head") and m._use_hip(io["in_obs"])
    packed = False
    if hip:
        # decode + bucket the sparse head's active pairs by cell in the same pass
        head = m._head(device)
        head.ensure_buckets(E)
        N.check(k.mbk_decode_obs_mask_bucket(
            io["in_codes"].data_ptr(), io["in_res"].data_ptr(), E, size, size,
            io["in_obs"].data_ptr(), io["in_mask"].data_ptr(), head.bucket_cnt.data_ptr(),
            head.bucket.data_ptr(), head.cell_lp.data_ptr(), io["out_action"].data_ptr(),
            st), "decode_obs_mask_bucket")
        # the head's last launch also packs the env action codes (row_sum_pack)
        _, _, value = m.act(io["in_obs"], io["in_mask"], rng, action_out=io["out_action"],
                            logp_out=io["out_logp"], bucketed=True,
                            logits_out=io.get("out_logits"), value_out=io["out_value"],
                            act16_out=io["out_act16"])
        packed = True
    else:
        N.check(k.mbk_decode_obs_mask(io["in_codes"].data_ptr(), io["in_res"].data_ptr(),
                                      E, size, size, io["in_obs"].data_ptr(),
                                      io["in_mask"].data_ptr(), st), "decode_obs_mask")
        if hasattr(m, "policy_value_pbc") and m._use_hip(io["in_obs"]):
            if "out_logits" in io:   # dense logits requested: pixel-major path
                logits, value = m.policy_value_pbc(io["in_obs"])
                io["out_logits"].copy_(pbc_to_cell_major(logits).reshape(io["out_logits"].shape))
                cell_head.sample_pbc(logits, io["in_mask"], rng, action_out=io["out_action"],
                                     cell_logp=io["cell_logp"], logp_out=io["out_logp"])
            else:                    # GridNet: active-cell logits straight into the sampler
                _, _, value = m.act(io["in_obs"], io["in_mask"], rng, action_out=io["out_action"],
                                    cell_logp=io["cell_logp"], logp_out=io["out_logp"])
        else:
            logits, value = m.policy_value(io["in_obs"])
            if "out_logits" in io:
                io["out_logits"].copy_(logits.reshape(io["out_logits"].shape))
            cell_head.sample_gpu(logits, io["in_mask"], rng, action_out=io["out_action"],
                                 cell_logp=io["cell_logp"], logp_out=io["out_logp"])
    if value.data_ptr() != io["out_value"].data_ptr():  # (written in place when fused)
        io["out_value"].copy_(value.view(-1))
    if not packed:
        N.check(k.mbk_pack_env_actions(io["out_action"].data_ptr(), E * size * size,
                                       io["out_act16"].data_ptr(), N.stream_ptr()),
                "pack_env_actions")


def make_io(E: int, S: int, device, logits: bool = False) -> dict:
    """Fixed-address I/O of one policy lane's captured graph."""
    return {
        # what crosses PCIe: 16-bit cell codes + resources in, packed actions out
        "in_codes": zeros(E, S, dtype=torch.int16, device=device),
        "in_res": zeros(E, dtype=torch.int32, device=device),
        "out_act16": zeros(E, S, dtype=torch.int16, device=device),
        # decoded on the GPU inside the policy graph
        "in_obs": zeros(E, S, dtype=torch.int32, device=device),
        "in_mask": zeros(E, S, 3, dtype=torch.int32, device=device),
        "out_action": zeros(E, S, 7, dtype=torch.uint8, device=device),
        "out_logp": zeros(E, dtype=torch.float32, device=device),
        "out_value": zeros(E, dtype=torch.float32, device=device),
        # dense-head (GridNet) sampling workspace, per lane
        "cell_logp": zeros(E * S, dtype=torch.float32, device=device),
    } | ({"out_logits": zeros(E, S * 78, dtype=torch.float32, device=device)} if logits else {})


class GpuActorRuntime:
    def __init__(self, make_model, size: int, n_groups: int, envs_per_group: int, unroll: int,
                 batch_slots: int, device: torch.device, n_threads: int | None = None,
                 n_slots: int | None = None, max_steps: int = 2000, seed: int = 1,
                 bots=DEFAULT_BOTS, reward_weight=(10.0, 1.0, 1.0, 0.2, 1.0, 4.0),
                 env_index_base: int = 0, selfplay_groups: int = 0, fp8_policy: bool = False,
                 n_lanes: int | None = None,
                 reference_keys: bool = False, policy_logits: bool = False,
                 preroll: int = 0, fused_act: bool | None = None):
        """preroll > 1: every env first plays r ~ U[0, preroll) steps of the uniform
        random-init policy on the CPU (engine.h EngineConfig::preroll), so the run starts from
        envs spread over the game's phases rather than all at their first frame.
        reference_keys: also emit the reference buffer keys ep_return / ep_step /
        last_action (libs/utils.py:34-46) into the slots; policy_logits: plus the dense
        78*h*w policy logits of every step (the sparse acting head never needs them, so
        this adds one dense head GEMM per policy step and 312*h*w bytes per frame).
        fused_act: None picks the fused acting step whenever ops/act.py supports the model
        shape; False forces the captured-graph step (the tests compare the two)."""
        rt = N.runtime()
        self.device = device
        self.size, self.S = size, size * size
        self.G, self.E, self.T = n_groups, envs_per_group, unroll
        self.batch_slots = batch_slots
        self.n_slots = n_slots or (2 * n_groups + batch_slots + 1)
        S, E, T1, NS = self.S, self.E, self.T + 1, self.n_slots
        dev = device
        self.rb = {
            "obs": zeros(NS, T1, E, S, dtype=torch.int32, device=dev),
            "mask": zeros(NS, T1, E, S, 3, dtype=torch.int32, device=dev),
            "action": zeros(NS, T1, E, S, 7, dtype=torch.uint8, device=dev),
            "logp": zeros(NS, T1, E, dtype=torch.float32, device=dev),
            "value": zeros(NS, T1, E, dtype=torch.float32, device=dev),
            "reward": zeros(NS, T1, E, dtype=torch.float32, device=dev),
            "done": zeros(NS, T1, E, dtype=torch.uint8, device=dev),
        }
        # active-cell bitmap rows (32 B per 16x16 frame), written by the fused acting step:
        # the learner's head compaction reads them instead of the [S, 3] masks (dropped from
        # the batch below when the graph path acts)
        if S % 32 == 0:
            self.rb["abits"] = zeros(NS, T1, E, S // 32, dtype=torch.int32, device=dev)
        self.reference_keys = reference_keys or policy_logits
        self.emit_logits = policy_logits
        if self.reference_keys:
            self.rb["ep_return"] = zeros(NS, T1, E, dtype=torch.float32, device=dev)
            self.rb["ep_step"] = zeros(NS, T1, E, dtype=torch.int32, device=dev)
            self.rb["last_action0"] = zeros(NS, E, S, 7, dtype=torch.uint8, device=dev)
        if policy_logits:
            self.rb["policy_logits"] = zeros(NS, T1, E, S * 78, dtype=torch.float32,
                                                   device=dev)
        # policy lanes: group g steps on lane g % n_lanes; every lane has its own stream,
        # captured graph, I/O buffers, RNG stream and inference-weight copy, so policy steps
        # of different groups can run concurrently. Measured on one MI355X (4 x 4096 envs,
        # same box, back to back): 1 lane 6.22 M frames/s, 2 lanes 5.78 M, 4 lanes 5.68 M:
        # the GPU, not the single stream, is the limit there, so the default is one lane
        self.n_lanes = max(1, min(n_groups, n_lanes if n_lanes is not None else 1))
        self.fp8_policy = fp8_policy
        self.selfplay_groups = int(selfplay_groups)
        self.lanes = []
        for ln in range(self.n_lanes):
            lane = {"io": self._make_io(),
                    "rng": torch.tensor([seed * 7919 + env_index_base + 15485863 * ln, 0],
                                        dtype=torch.int64, device=dev),
                    "model": make_model().to(dev)}
            lane["model"].eval()
            if fp8_policy:  # acting trunk on fp8 MFMA; V-trace corrects the behaviour gap
                lane["model"].fp8_inference = True
            lane["flat"] = FlatParams(lane["model"], dev)
            lane["pack_graph"] = self._capture_pack(lane["model"])
            lane["graph"] = self._capture(lane["io"], lane["model"], lane["rng"])
            if self.selfplay_groups > 0:
                lane["io_p1"] = self._make_io()
                lane["rng_p1"] = torch.tensor(
                    [seed * 7919 + env_index_base + 104729 + 15485863 * ln, 0],
                    dtype=torch.int64, device=dev)
                lane["opp_model"] = make_model().to(dev)
                lane["opp_model"].eval()
                lane["opp_model"].fp8_inference = fp8_policy
                lane["opp_flat"] = FlatParams(lane["opp_model"], dev)
                lane["opp_pack_graph"] = self._capture_pack(lane["opp_model"])
                lane["opp_graph"] = self._capture(lane["io_p1"], lane["opp_model"],
                                                  lane["rng_p1"])
            self.lanes.append(lane)
        # lane-0 aliases (tests / tools)
        l0 = self.lanes[0]
        self.io, self.rng, self.infer_model = l0["io"], l0["rng"], l0["model"]
        self.infer_flat, self.pack_graph, self.graph = l0["flat"], l0["pack_graph"], l0["graph"]
        self.opp_graph = l0.get("opp_graph")
        if self.selfplay_groups > 0:
            self.opp_flat, self.opp_model = l0["opp_flat"], l0["opp_model"]
        if n_threads is None:
            n_threads = max(1, min(32, available_cpus() - 1))
        self.n_threads = n_threads
        cfg = dict(size=size, n_groups=n_groups, envs_per_group=E, unroll=self.T, n_slots=NS,
                   n_threads=n_threads, max_steps=max_steps, seed=seed,
                   bots=[BOT_IDS[b] if isinstance(b, str) else int(b) for b in bots],
                   reward_weight=list(reward_weight), env_index_base=env_index_base,
                   device=dev.index if dev.index is not None else torch.cuda.current_device(),
                   selfplay_groups=self.selfplay_groups, n_lanes=self.n_lanes,
                   preroll=int(preroll))
        bufs = {k: v.data_ptr() for k, v in self.rb.items()}
        bufs["lanes"] = []
        for lane in self.lanes:
            d = {k: v.data_ptr() for k, v in lane["io"].items()}
            if self.selfplay_groups > 0:
                d.update({"in_codes_p1": lane["io_p1"]["in_codes"].data_ptr(),
                          "in_res_p1": lane["io_p1"]["in_res"].data_ptr(),
                          "out_act16_p1": lane["io_p1"]["out_act16"].data_ptr()})
            bufs["lanes"].append(d)
        torch.cuda.synchronize()
        self.engine = rt.GpuEngine(cfg, bufs)
        # fused acting steps (ops/act.py): 2 launches per policy step that write the rollout
        # row in place, instead of the captured 6-launch graph + scatter copy. Headline agent
        # shape (16x16, bf16 trunk), self-play groups included (the opponent's step runs the
        # same launches on its mirrored rows with its own weights). The kernels read the
        # occupied-cell rows from / write the action rows to the engine's pinned host staging
        self.fused_act = (fused_act is not False and not self.reference_keys
                          and all(act_ops.supported(ln["model"], size, fp8_policy)
                                  for ln in self.lanes))
        if fused_act and not self.fused_act:
            raise ValueError("fused_act=True: the fused acting step does not cover this model "
                             "/ map size / dtype or the reference buffer keys")
        if self.fused_act:
            for lane in self.lanes:
                lane["act"] = act_ops.ActWorkspace(lane["model"], E, lane["rng"], dev)
                if self.selfplay_groups > 0:  # (packed by its captured pack graph)
                    lane["opp_act"] = act_ops.ActWorkspace(lane["opp_model"], E,
                                                           lane["rng_p1"], dev)
            torch.cuda.synchronize()
            self.engine.set_act_models([ln["act"].block() for ln in self.lanes],
                                       [ln["opp_act"].block() for ln in self.lanes
                                        if "opp_act" in ln])
        # captured-graph steps (shapes the fused step does not cover, fp8 acting, GridNet):
        # sparse occupied-cell rows in / non-noop action rows out through two small launches
        # instead of H2D / D2H blit copies of dense code rows (the reference buffer keys keep
        # the dense copies: their last_action / logits rows are dense)
        self.sparse_io = not self.fused_act and not self.reference_keys
        if self.sparse_io:
            self.engine.set_sparse_io(True)
        if not self.fused_act and "abits" in self.rb:
            self._abits_unwritten = self.rb.pop("abits")  # (the engine holds its address)
        self.started = False
        self.frames_per_slot = E * self.T

    # ------------------------------------------------------------ inference graph
    def _make_io(self):
        return make_io(self.E, self.S, self.device, getattr(self, "emit_logits", False))

    def _policy_step(self, io, m, rng):
        graph_policy_step(io, m, rng, self.E, self.size, self.device)

    def _capture_pack(self, model):
        """Graph of ``model.pack_inference`` (derived weight buffers), replayed by the engine
        after each publish; the policy graph then never re-packs (None: model has none)."""
        if not hasattr(model, "pack_inference"):
            return None
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            model.pack_inference(self.device)  # allocates the persistent buffers
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            model.pack_inference(self.device)
        torch.cuda.synchronize()
        return g

    def _capture(self, io, model, rng):
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):  # warm up allocator / kernels outside capture
                self._policy_step(io, model, rng)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            self._policy_step(io, model, rng)
        torch.cuda.synchronize()
        rng[1] = 0
        return g

    # ------------------------------------------------------------ control
    def start(self, learner_flat: FlatParams | None = None, opponent_version: int = -1,
              version: int = 0):
        """opponent_version: league id of the starting opponent weights (self-play groups
        start against a copy of ``learner_flat``; tag their episodes with this id).
        version: learner update count of ``learner_flat`` (a restarted engine's slots are
        tagged with it, so policy_lag stays the true lag)."""
        self.engine.set_policy_version(int(version))
        if self.selfplay_groups > 0:
            self.engine.set_initial_opponent(int(opponent_version))
        for lane in self.lanes:
            if learner_flat is not None:
                lane["flat"].data.copy_(learner_flat.data)
                if self.selfplay_groups > 0:  # until the league picks one
                    lane["opp_flat"].data.copy_(learner_flat.data)
            for pg in (lane["pack_graph"], lane.get("opp_pack_graph")):
                if pg is not None:
                    pg.replay()
        torch.cuda.synchronize()
        ex = lambda g: int(g.raw_cuda_graph_exec()) if g is not None else 0  # noqa: E731
        self.engine.start([[ex(ln["graph"]), ex(ln.get("opp_graph")), ex(ln["pack_graph"]),
                            ex(ln.get("opp_pack_graph"))]
                           for ln in self.lanes])
        self.started = True

    def stop(self):
        if self.started:
            self.engine.stop()
            self.started = False

    def close(self):
        """Stop, then drop the engine and every device buffer / captured graph this runtime
        owns, so its HBM goes back to the allocator even while a caller still holds the (now
        empty) object (train.restart_runtime)."""
        self.stop()
        self.engine = None  # the native engine first: it points into the buffers below
        self.lanes = []
        self.rb = {}
        for k in ("io", "rng", "infer_model", "infer_flat", "pack_graph", "graph", "opp_graph",
                  "opp_flat", "opp_model"):
            if hasattr(self, k):
                setattr(self, k, None)

    def check(self):
        if self.engine.failed():
            raise EngineFailure(f"GPU actor engine failed: {self.engine.error()}")

    def inject_fault(self):
        """Make the next env step of some worker throw (fault-injection tests)."""
        self.engine.inject_fault()

    def get_batch(self, n_slots: int | None = None, timeout: float = 600.0):
        """Block until n full rollout slots exist; return (batch dict, slot ids).

        The learner's current stream is made to wait on the slots' completion
        events; no host synchronisation with the GPU happens here.
        """
        n = n_slots or self.batch_slots
        self.check()
        slots = self.engine.get_full(n, timeout)
        self.check()
        if len(slots) < n:
            raise TimeoutError(f"no full rollout slot within {timeout}s (engine stats "
                               f"{self.engine.stats()})")
        sp = N.stream_ptr()
        for s in slots:
            self.engine.stream_wait_full(sp, s)
        keys = [k for k in self.rb if k != "last_action0"]
        if n == 1:
            s = slots[0]
            batch = {k: self.rb[k][s] for k in keys}
        else:
            batch = {k: torch.cat([self.rb[k][s] for s in slots], dim=1) for k in keys}
        if self.reference_keys:
            # last_action[t] = the action taken before obs_t: a_{t-1}, row 0 from the group's
            # previous slot (reference Env_Packer 'last_action'); materialised on request only
            la = [torch.cat([self.rb["last_action0"][s][None], self.rb["action"][s][:-1]])
                  for s in slots]
            batch["last_action"] = la[0] if n == 1 else torch.cat(la, dim=1)
        return batch, slots

    def release(self, slots):
        self.engine.release(list(slots), N.stream_ptr())

    def publish(self, learner_flat: FlatParams, version: int = -1) -> bool:
        """Event-ordered copy of the learner weights into every lane's inference copy.
        version: learner update count of these weights (tags the slots that act with them,
        see ``policy_lag``)."""
        return self.engine.publish(learner_flat.data.data_ptr(),
                                   [ln["flat"].data.data_ptr() for ln in self.lanes],
                                   learner_flat.numel * 4, N.stream_ptr(), int(version))

    def policy_lag(self, slots, learner_version: int) -> int:
        """Learner updates between the oldest behaviour weights in ``slots`` and
        ``learner_version`` (the update about to consume them); IMPALA's off-policy gap."""
        return int(learner_version) - min(self.engine.slot_version(int(s)) for s in slots)

    def set_opponent(self, flat: torch.Tensor, version: int) -> bool:
        """Swap the self-play opponent to league snapshot ``version`` (a flat fp32 buffer).
        Returns False (and changes nothing) if the previous swap is still pending."""
        if self.selfplay_groups <= 0:
            raise RuntimeError("set_opponent: runtime has no self-play groups")
        assert flat.numel() == self.opp_flat.numel and flat.dtype == torch.float32
        return self.engine.publish_opponent(flat.data_ptr(),
                                            [ln["opp_flat"].data.data_ptr() for ln in self.lanes],
                                            self.opp_flat.numel * 4, N.stream_ptr(), int(version))

    def drain_episodes(self):
        return self.engine.drain_episodes()

    def stats(self):
        return self.engine.stats()
