"""Training orchestration (reference ``train()`` + ``batch_and_learn``,
microbeast.py:109-264), one process per GPU.

Runtimes:
* ``gpu``  — native env workers + on-GPU batched policy inference + HBM
  rollout slots (runtime/gpu_actors.py); the flagship throughput path;
* ``mono`` — CPU actor processes with shared-memory buffers
  (runtime/mono.py); the reference shape, CPU-only capable (config 1).

Data parallelism: launch with torchrun; each rank owns its actors, the
learners all-reduce gradients (parallel/dist.py); rank 0 writes the CSVs and
checkpoints. The reference's learner loop never terminated (while-True spin,
microbeast.py:262-263); this one stops at ``total_steps`` / ``max_updates``,
checkpoints and shuts its actors down.
"""
from __future__ import annotations

import dataclasses
import gc
import os
import time
import warnings

import torch

from .config import Flags, bwd_occupancy
from .learner import Learner, LearnerHParams
from .models.factory import make_model
from .parallel import dist as D
from .utils.checkpoint import (load_checkpoint, load_league_shard, restore, save_checkpoint,
                               save_league_shard)
from .utils.metrics import CsvLogger


def scaled_lr(flags: Flags, frames_per_update: int) -> float:
    """--lr_scaling: the base --lr is tuned for --lr_base_batch frames per update (the reference
    2.5e-4 at one GPU's 524,288); weak-scaled DP multiplies the global batch by the world size
    (and --batch_size by its value), so the step size can follow it: sqrt (Adam's usual rule,
    the default) or linear in the batch ratio, or stay (none). Only batches LARGER than the
    base are scaled: smaller configs keep the reference lr. Measured on 16x16 at 1.68 B frames
    (experiments/README.md): 4.2 M frames per update reaches a 0.80 win rate with sqrt vs 0.47
    unscaled (0.56 at 524 K frames per update)."""
    r = max(1.0, frames_per_update / max(1, flags.lr_base_batch))
    k = {"none": 0.0, "sqrt": 0.5, "linear": 1.0}[flags.lr_scaling]
    return flags.lr * (r ** k)


def update_frames(flags: Flags, runtime: str, world_size: int = 1) -> int:
    """Env frames consumed per learner update over all ranks: batch slots x envs per slot x T x
    world (gpu runtime: a slot is one env group's unroll; mono: one actor's n_envs)."""
    per_slot = flags.envs_per_group if runtime == "gpu" else flags.n_envs
    return flags.resolved_batch_size(runtime) * per_slot * flags.unroll_length * world_size


def _hparams(flags: Flags, lr: float | None = None) -> LearnerHParams:
    return LearnerHParams(lr=flags.lr if lr is None else lr, adam_eps=flags.adam_eps, gamma=flags.gamma,
                          baseline_cost=flags.baseline_cost, entropy_cost=flags.entropy_cost,
                          rho_bar=flags.rho_bar, c_bar=flags.c_bar, pg_rho_bar=flags.pg_rho_bar,
                          reward_clip=flags.reward_clip, max_grad_norm=flags.max_grad_norm,
                          bucket_mb=flags.bucket_mb, allreduce_dtype=flags.allreduce_dtype)


def checkpoint_path(flags: Flags) -> str:
    return flags.checkpoint or os.path.join(flags.savedir, f"{flags.exp_name}.ckpt")


def _gather_episodes(recs, info):
    """Every rank's finished episodes to rank 0 (gloo host group: no GPU-stream sync)."""
    parts = D.gather_objects(recs, info)
    return [r for part in parts for r in (part or [])]


class _LossReadout:
    """Loss values reach the host one update late: an async D2H copy into pinned memory
    plus an event, polled with ``query()``. The learner loop therefore never waits for the
    GPU to finish an update before enqueueing the next one (the reference read floats
    synchronously every update, libs/utils.py:340)."""

    def __init__(self, cuda: bool):
        self.cuda = cuda
        self.q = []

    def push(self, vals: torch.Tensor, meta: dict):
        if self.cuda:
            host = torch.empty(vals.numel(), dtype=vals.dtype, pin_memory=True)
            host.copy_(vals, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = vals.clone(), None
        self.q.append((host, ev, meta))

    def pop(self, wait: bool = False):
        out = []
        while self.q and (wait or self.q[0][1] is None or self.q[0][1].query()):
            host, ev, meta = self.q.pop(0)
            if ev is not None:
                ev.synchronize()
            out.append((host.tolist(), meta))
        return out


_PROFILE_START = 3  # skip the first updates (graph capture, allocator warm-up)


def _profile_tick(prof, n_update: int, flags: Flags, cuda: bool):
    """Start the torch.profiler at update _PROFILE_START, stop after profile_updates updates
    (or at shutdown: n_update = -1) and write {exp}_trace.json + {exp}_profile.txt."""
    from torch.profiler import ProfilerActivity, profile
    end = _PROFILE_START + flags.profile_updates
    if prof is None and n_update == _PROFILE_START:
        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if cuda else [])
        prof = profile(activities=acts, record_shapes=False)
        prof.__enter__()
        return prof
    if prof is not None and (n_update == end or n_update < 0):
        if cuda:
            torch.cuda.synchronize()
        prof.__exit__(None, None, None)
        base = os.path.join(flags.savedir, flags.exp_name)
        prof.export_chrome_trace(base + "_trace.json")
        sort = "self_cuda_time_total" if cuda else "self_cpu_time_total"
        with open(base + "_profile.txt", "w") as f:
            f.write(prof.key_averages().table(sort_by=sort, row_limit=40))
        return None
    return prof


def restart_runtime(rt, make, learner_flat, n_update: int, league=None):
    """Replace a failed GPU actor runtime: stop it and drop every reference to it, collect,
    return its cached HBM to the allocator, THEN build and start the new one (acting with
    the learner's current weights, tagged with update ``n_update``). ``rt.close()`` drops the
    old runtime's buffers even though the caller's own variable still references it; the caller
    must not hold other references into it (e.g. a batch that views its rollout slots)."""
    rt.close()
    rt = None
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    new = make()
    new.start(learner_flat, opponent_version=league.current if league is not None else -1,
              version=n_update)
    if league is not None and league.current in league.snaps:
        new.set_opponent(league.snapshot(league.current), league.current)
    return new


def _league_extra(league):
    return {"league": league.state_dict()} if league is not None else None


def resolve_runtime(flags: Flags, want_cuda: bool) -> str:
    """The actor runtime a run uses. The GPU engine's env workers step the native stand-in
    only (C++ MicroRTSSim, sparse code rows); the real gym-microrts adapter (envs/microrts.py,
    reference libs/utils.py:59-76) runs in the mono runtime's CPU actor processes, so
    ``--env microrts`` picks that runtime under ``--runtime auto`` and is refused on ``gpu``."""
    if flags.env not in ("synthetic", "microrts"):
        raise ValueError(f"--env {flags.env!r}: expected synthetic | microrts")
    runtime = flags.runtime if flags.runtime != "auto" else (
        "gpu" if want_cuda and flags.env == "synthetic" else "mono")
    if runtime == "gpu" and flags.env != "synthetic":
        raise ValueError(f"--env {flags.env} is not available on the gpu runtime (its env workers "
                         "step the native microRTS stand-in only); use --runtime mono (CPU actor "
                         "processes over the gym-microrts adapter) or --env synthetic")
    return runtime


def train(flags: Flags) -> dict:
    want_cuda = flags.device == "cuda" or (flags.device == "auto" and torch.cuda.is_available())
    info = D.init_distributed(use_cuda=want_cuda, high_priority=flags.rccl_high_priority)
    dev = torch.device("cuda", info.local_rank) if want_cuda else torch.device("cpu")
    runtime = resolve_runtime(flags, want_cuda)
    if runtime == "gpu" and flags.dtype == "fp32":
        # the engine's policy step and the learner are the bf16 MFMA kernels: refuse rather
        # than run bf16 under an fp32 flag
        raise ValueError("--dtype fp32 is not available on the gpu runtime (bf16 / fp8 MFMA "
                         "kernels); use --dtype bf16, or --runtime mono for fp32 PyTorch ops")
    if runtime == "gpu" and not want_cuda:
        raise RuntimeError("--runtime gpu needs a GPU")
    if flags.batch_size <= 0:  # auto: 2 slots on mono (reference B), 1 on gpu (524,288 frames)
        flags = dataclasses.replace(flags, batch_size=flags.resolved_batch_size(runtime))
    actor_threads = flags.actor_threads
    if runtime == "gpu":
        from .parallel.launch import pin_rank, rank_cpu_budget

        # NUMA/core placement before the engine starts its env worker / driver threads
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(info.world_size)))
        pin_rank(info.local_rank, local_world, dev.index)
        # the rank's CPU budget less one for the spinning engine driver (bench.py: 15 env
        # threads on a 16-CPU share halve the env phase vs 13, profile 23)
        actor_threads = actor_threads or max(1, min(32, rank_cpu_budget(local_world) - 1))
    torch.manual_seed(flags.seed + info.rank)
    log = (lambda *a: None) if (flags.quiet or not info.is_main) else (lambda *a: print(*a, flush=True))
    log(f"[microbeast_amd] exp={flags.exp_name} runtime={runtime} device={dev} "
        f"world={info.world_size} map={flags.env_size}x{flags.env_size} arch={flags.arch}")

    if runtime == "gpu":  # before the learner sizes its partial buffers
        from . import _native
        if _native.kernels().mbk_set_learner_occupancy(flags.learner_fwd_occupancy,
                                                     bwd_occupancy(flags.learner_bwd_occupancy,
                                                                   flags.arch)) != 0:
            # a learner of this process already sized its grids (tests run several trainings
            # in one process): the caps stay as they were
            warnings.warn("--learner_fwd/bwd_occupancy ignored: learner grids already sized in "
                          "this process")
    model = make_model(flags, dev)
    lr = scaled_lr(flags, update_frames(flags, runtime, info.world_size))
    if lr != flags.lr:
        log(f"[microbeast_amd] lr {flags.lr:g} -> {lr:g} (--lr_scaling {flags.lr_scaling})")
    learner = Learner(model, _hparams(flags, lr), dev, info)
    step = n_update = 0
    ck_path = checkpoint_path(flags)
    ck = None
    if flags.resume and os.path.exists(ck_path):
        ck = load_checkpoint(ck_path)
        step, n_update = restore(ck, learner.model, learner.opt)
        learner.n_updates = n_update
        log(f"[microbeast_amd] resumed {ck_path} at step={step} update={n_update}")
    logger = CsvLogger(flags.savedir, flags.exp_name, enabled=info.is_main, append=flags.resume)

    league = None
    if flags.self_play and runtime != "gpu":
        raise RuntimeError("--self_play needs the gpu runtime (the league plays on the GPU engine)")
    if runtime == "gpu":
        from .runtime.gpu_actors import EngineFailure, GpuActorRuntime

        envs_total = flags.groups * flags.envs_per_group
        sp_groups = min(flags.selfplay_groups, flags.groups) if flags.self_play else 0

        def make_gpu_runtime(restart: int):
            """(Re)build the actor side: env workers, policy graphs, HBM slots. A restart
            gets fresh env seeds; the learner (weights, Adam, league) is untouched."""
            return GpuActorRuntime(lambda: make_model(flags, "cpu"), flags.env_size,
                                   flags.groups, flags.envs_per_group, flags.unroll_length,
                                   flags.batch_size, dev, n_threads=actor_threads,
                                   max_steps=flags.max_episode_steps,
                                   seed=flags.seed + 1000 * info.rank + 7777 * restart,
                                   bots=flags.opponent_list(), reward_weight=flags.reward_weights(),
                                   env_index_base=info.rank * envs_total, selfplay_groups=sp_groups,
                                   fp8_policy=flags.fp8_policy or flags.dtype == "fp8",
                                   n_lanes=max(1, min(flags.policy_lanes, flags.groups)))

        rt = make_gpu_runtime(0)
        if sp_groups:
            from .runtime.league import League

            league = League(capacity=flags.league_size, snapshot_every=flags.league_update_every,
                            pfsp_power=flags.pfsp_power, eps=flags.league_eps,
                            seed=flags.seed + info.rank)
            shard = (load_league_shard(ck_path, info.rank, ck.get("n_update"))
                     if ck is not None else None)
            if shard is not None:  # this rank's own league (DP runs save one per rank)
                league.load_state_dict(shard, dev)
            elif ck is not None and ck.get("league"):
                league.load_state_dict(ck["league"], dev)
            else:
                league.add_snapshot(learner.flat.data)
            league.current = league.next_id - 1
        rt.start(learner.flat, opponent_version=league.current if league is not None else -1,
                 version=n_update)
        if league is not None and ck is not None and ck.get("league"):
            # resumed: play the restored snapshot instead of the learner copy
            rt.set_opponent(league.snapshot(league.current), league.current)
    else:
        from .runtime.mono import MonoRuntime

        rt = MonoRuntime(flags, learner.flat.numel, device=dev,
                         make_model=lambda: make_model(flags, "cpu"))
        rt.publish(learner.flat.data)
        rt.start()
        if want_cuda:  # pinned DMA of full slots into HBM, one batch ahead of the learner
            rt.enable_prefetch(dev)
    frames_per_update = update_frames(flags, runtime, info.world_size)

    def save_all(step_, n_update_):
        """Rank 0 writes the checkpoint; every rank with a league writes its own league shard
        (snapshots + PFSP results: each DP rank matches against its own league)."""
        if info.is_main:
            save_checkpoint(ck_path, learner.model, learner.opt, step_, n_update_, flags,
                            extra=_league_extra(league))
        if league is not None:  # every run with a league, so a shard is never stale
            save_league_shard(ck_path, info.rank, league.state_dict(), n_update_)

    engine_restarts = 0
    prof = None  # --profile_updates: torch.profiler timeline of a few steady-state updates
    t_start = time.perf_counter()
    t_prev = t_start
    last = {}
    readout = _LossReadout(want_cuda)

    def flush(wait=False):
        for lv, m in readout.pop(wait):
            logger.losses(m["update"], lv[0], lv[1], lv[2], lv[3], m["period"], m["step"],
                          m["fps"], m["wait_s"], m["learn_s"], lv[4], phase_ms=m["phase"],
                          policy_lag=m["lag"])
            last.update(update=m["update"], step=m["step"], pg_loss=lv[0], value_loss=lv[1],
                        entropy=lv[2], total_loss=lv[3], fps=m["fps"])
            log(f"update {m['update']} step {m['step']} total_loss {lv[3]:.4f} pg {lv[0]:.4f} "
                f"v {lv[1]:.4f} ent {lv[2]:.3f} fps {m['fps']:,.0f} lag {m['lag']}"
                + (f" league {m['league']}" if m.get("league") else ""))

    held = None  # gpu runtime: a batch kept over a round in which a DP peer restarted
    pending_eps = []  # finished episodes since the last rank-0 gather (DP: batched exchange)

    def sync_episodes(force=False):
        # rank 0 writes every rank's episodes; under DP they travel every
        # --episode_sync_every updates in one gloo gather instead of one per update
        if not info.enabled or force or n_update % max(1, flags.episode_sync_every) == 0:
            logger.episodes(_gather_episodes(list(pending_eps), info))
            pending_eps.clear()

    try:
        while step < flags.total_steps and (flags.max_updates <= 0 or n_update < flags.max_updates):
            if flags.profile_updates > 0 and info.is_main:
                prof = _profile_tick(prof, n_update, flags, want_cuda)
            t0 = time.perf_counter()
            failure = None
            if runtime == "gpu":
                if held is not None:  # fetched in a round a peer spent restarting
                    (batch, slots), held = held, None
                else:
                    try:
                        batch, slots = rt.get_batch(timeout=flags.batch_timeout)
                    except EngineFailure as ex:
                        failure = str(ex)  # (the exception's frames hold the old runtime: drop it)
            state = (D.OK if failure is None
                     else D.RESTARTING if engine_restarts < flags.actor_restarts else D.FAILED)
            # every rank agrees on the update before its gradient collectives: one that cannot
            # go on (restarts exhausted) stops all of them now, not at the PG timeout, and one
            # that restarts its engine makes all of them skip the round together
            agreed = D.agree(state, info)
            if agreed == D.FAILED:
                if failure is not None:
                    raise EngineFailure(failure)
                raise RuntimeError("another data-parallel rank stopped (engine failure)")
            if agreed == D.RESTARTING:
                if failure is None:
                    held = (batch, slots)
                    continue
                # a dead env worker stops the native engine; rebuild the
                # actor side and keep training (bounded by --actor_restarts). The old
                # runtime (HBM slots, pinned staging, graphs) is freed BEFORE the new one
                # is allocated, so a restart never needs two runtimes' memory
                engine_restarts += 1
                log(f"[microbeast_amd] {failure}; restarting the actor engine "
                    f"({engine_restarts}/{flags.actor_restarts})")
                batch = slots = None  # (views of the old runtime's rollout slots)
                try:
                    rt = restart_runtime(rt, lambda: make_gpu_runtime(engine_restarts),
                                         learner.flat, n_update, league)
                except Exception:
                    # the peers skipped this round and now wait in the next agree(): tell them
                    # to stop instead of leaving them blocked until the host-group timeout
                    # (ADVICE r4); the old runtime is already closed, stop() is a no-op
                    D.agree(D.FAILED, info)
                    raise
                continue
            if runtime == "gpu":
                lag = rt.policy_lag(slots, n_update)
            else:
                batch, slots = rt.get_batch(flags.batch_timeout)
                lag = -1
                if not want_cuda:
                    batch = {k: v.to(dev) for k, v in batch.items()}
            t1 = time.perf_counter()
            losses = learner.learn(batch)
            if runtime == "gpu":
                rt.release(slots)
                rt.publish(learner.flat, version=n_update + 1)
            else:
                rt.publish(learner.flat.data)
            learner.phases.mark("publish")
            step += frames_per_update
            n_update += 1
            if league is not None:
                # freeze a snapshot now and then; re-draw the opponent (PFSP) every update
                league.maybe_snapshot(n_update, learner.flat.data)
                sid = league.sample()
                if sid != league.current and rt.set_opponent(league.snapshot(sid), sid):
                    league.current = sid
            if flags.fault_inject_every and n_update % flags.fault_inject_every == 0:
                if runtime == "mono":
                    rt.kill_random_actor()
                else:
                    rt.inject_fault()
            if n_update % flags.log_every == 0:
                t2 = time.perf_counter()
                period = (t2 - t_prev) / flags.log_every  # loop period, as the reference timed it
                t_prev = t2
                readout.push(D.all_reduce_mean(losses.detach().clone(), info), {
                    "update": n_update, "step": step, "period": period,
                    "fps": frames_per_update / max(period, 1e-9), "wait_s": t1 - t0,
                    "learn_s": t2 - t1, "phase": learner.phases.read(), "lag": lag,
                    "league": (f"{len(league)} vs #{league.current}" if league is not None
                               else None)})
                eps = rt.drain_episodes()
                if league is not None:
                    league.record(eps)  # each rank matches against its own league
                pending_eps.extend(eps)
                sync_episodes()
            flush()
            if flags.checkpoint_every and n_update % flags.checkpoint_every == 0:
                save_all(step, n_update)
                D.barrier(info)
        sync_episodes(force=True)
    finally:
        if prof is not None:
            _profile_tick(prof, -1, flags, want_cuda)
        flush(wait=True)
        rt.stop()
        save_all(step, n_update)
        logger.close()
    wall = time.perf_counter() - t_start
    out = dict(last, updates=n_update, steps=step, wall_s=wall, checkpoint=ck_path,
               mean_fps=step / max(wall, 1e-9), engine_restarts=engine_restarts,
               # gpu runtime: the policy step ran the fused two-launch kernels (ops/act.py)
               fused_act=bool(getattr(rt, "fused_act", False)))
    log(f"[microbeast_amd] done: {out}")
    D.destroy(info)
    return out
