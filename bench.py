#!/usr/bin/env python
"""Headline benchmark: env frames/sec (whole node) on 16x16 microRTS.

Metric and config from BASELINE.json: "env frames/sec (whole node) on 16x16
microRTS at 1/2/4/8 MI355X learners". One process per GPU (torchrun), each
with its own native env workers + on-GPU batched inference (GpuActorRuntime)
and a data-parallel learner (RCCL all-reduce). A timed step = one learner
update (forward, V-trace, backward, bucketed all-reduce, Adam, weight
publish) consuming ``batch_slots * envs_per_group * unroll`` fresh env frames
per rank that the actors produced concurrently; value = frames consumed by all
learners / wall time. Weak scaling (default): per-GPU work fixed, the global batch grows
with N. ``--scaling strong``: the 1-GPU problem (envs and frames per update) split over N.

Synthetic environment (native microRTS stand-in; gym-microrts/Java is not
available offline) and the reference architecture (IMPALA-CNN 16/32/32 + 256 FC +
flat 78*16*16 head, 5.27 M params), random-init and then trained for ``--settle``
untimed updates (default 500) so the timed window measures a training run's steady
state; the JSON ``data`` field names the settle count.

    python bench.py --gpus N --steps K --warmup W

With ``--gpus N > 1`` and no torchrun environment, bench.py launches N ranks
itself (``torch.distributed.run`` as a child process, parallel/launch.py) and
fails if fewer than N GPUs are visible. Each rank pins itself (and its env
worker / driver threads) to its share of the physical cores on its GPU's NUMA
node before starting them.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_FPS = 38.9  # best reference run (5_ener), frames/s whole node
CPU_BOUND_BUSY = 0.85  # env-worker busy fraction from which a rank counts as CPU-bound


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--size", type=int, default=16)
    p.add_argument("--arch", type=str, default="impala_flat",
                   help="impala_flat (headline) | gridnet (BASELINE config 2) | impala_deep")
    p.add_argument("--groups", type=int, default=4,
                   help="env groups pipelined through the policy lanes (profile 42 same-box "
                        "A/Bs at the round-5 learner speed, 2 lanes: 4 x 8192 16.4-17.8M vs "
                        "3 x 8192 14.5-15.3M frames/s at a mean policy lag of ~4.5 vs ~3.6 "
                        "updates; profile 36 measured them level with the round-4 learner)")
    p.add_argument("--lanes", type=int, default=0,
                   help="concurrent policy streams, each with its own graph + I/O (0 = auto: "
                        "2; strong scaling at N > 1: min(groups, N), at least 2)")
    p.add_argument("--envs_per_group", type=int, default=8192)
    p.add_argument("--unroll", type=int, default=64)
    p.add_argument("--batch_slots", type=int, default=1)
    p.add_argument("--threads", type=int, default=0, help="env worker threads per rank (0=auto)")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--verbose", action="store_true", help="per-step progress on stderr")
    p.add_argument("--selfplay_groups", type=int, default=0,
                   help="BASELINE config 5: env groups playing a self-play league (opponent "
                        "policy graph + PFSP over HBM snapshots) instead of scripted bots")
    p.add_argument("--fp8_policy", action="store_true",
                   help="acting trunk on the fp8 (e4m3) MFMA conv kernels (config 5)")
    p.add_argument("--profile_phases", action="store_true",
                   help="also report per-phase learner timings (adds syncs; not for the headline)")
    p.add_argument("--oversubscribe", action="store_true",
                   help="rehearsal only: allow more ranks than GPUs (ranks share a GPU over gloo)")
    p.add_argument("--allreduce_dtype", type=str, default="fp32", help="fp32 | bf16 payload")
    p.add_argument("--bucket_mb", type=float, default=8.0)
    p.add_argument("--learner_bwd_occupancy", type=int, default=-1,
                   help="learner backward workgroups per CU (0 = as many as fit; 1 leaves the "
                        "acting kernels a slot beside them: +4-7 %% on the headline, profile 45; "
                        "-1 = auto: 1 for impala_flat, 0 for the learner-heavy gridnet / "
                        "impala_deep, where the cap measured -2 / -7 %%)")
    p.add_argument("--learner_fwd_occupancy", type=int, default=0,
                   help="learner forward workgroups per CU (0 = as many as fit)")
    p.add_argument("--comm_rehearsal", action="store_true",
                   help="1 GPU only: every gradient bucket fires a stand-in collective kernel "
                        "on a 4th high-priority stream from the same hooks (the stream set of an "
                        "N > 1 rank; parallel/dist.py). Diagnostics, not the headline")
    p.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                   help="weak: every rank runs --groups x --envs_per_group envs and consumes "
                        "one slot per update (global batch grows with N); strong: the global "
                        "problem of 1 GPU (the same groups x envs_per_group envs, one update "
                        "of envs_per_group x unroll frames) is split over the N ranks")
    p.add_argument("--settle", type=int, default=500,
                   help="untimed training updates before the warm-up, so the timed window measures "
                        "a training run's steady state: from random init the policy learns to "
                        "produce units, the agent's idle units (active cells) per env rise from "
                        "~1.1 to ~9 by update ~120 (the acting step, the sparse head and the env "
                        "side slow down: ~13 M frames/s) and settle at 4-5 from update ~450 on "
                        "(profile 38; the 4-group training run r5d1L logs 17.0-18.8 M from "
                        "update 650 on, 17.2 M whole-run). 0 = time the early-game transient "
                        "(and drop the warm-up's queued rollouts before the window)")
    p.add_argument("--preroll", type=int, default=0,
                   help="before the first policy step every env plays r ~ U[0, preroll) steps of "
                        "the uniform random-init policy on the CPU (untimed), so the timed window "
                        "starts from envs spread over the game's phases, not all at reset "
                        "(0 = off)")
    p.add_argument("--report_every", type=int, default=0,
                   help="diagnostics: every k timed steps print the window's frames/s and active "
                        "cells per env to stderr (host clock; 0 = off)")
    return p.parse_args(argv)


def _occupancy(rt):
    """Occupied cells per env in the engine's sparse code rows (None without them)."""
    import ctypes

    import numpy as np
    try:
        ptr, stride = rt.engine.code_rows()
    except AttributeError:
        return None
    if not ptr or not stride:
        return None
    n_envs = rt.E * rt.G
    buf = (ctypes.c_uint32 * (n_envs * stride)).from_address(ptr)
    n = np.frombuffer(buf, dtype=np.uint32).reshape(n_envs, stride)[:, 0] & 0xFFFF
    return {"mean": round(float(n.mean()), 2), "p90": int(np.percentile(n, 90)),
            "max": int(n.max()), "frac_over_31": round(float((n > 31).mean()), 4)}


def main(argv=None):
    args = parse(argv)
    from microbeast_amd.parallel import launch

    if args.oversubscribe:
        os.environ.setdefault("MBK_DIST_BACKEND", "gloo")  # RCCL refuses 2 ranks per GPU
    rc = launch.relaunch(args.gpus, sys.argv[1:] if argv is None else list(argv),
                         script=os.path.abspath(__file__), shared_gpu=args.oversubscribe)
    if rc is not None:
        return rc
    import torch

    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent, num_params
    from microbeast_amd.parallel import dist as D
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    info = D.init_distributed(use_cuda=True)
    if args.scaling == "strong" and info.world_size > 1:
        # fixed global problem: each rank steps 1/N of the envs and its update consumes 1/N of
        # the global batch (the all-reduced gradient is the full batch's)
        if args.envs_per_group % info.world_size:
            print(f"--scaling strong: --envs_per_group {args.envs_per_group} is not divisible "
                  f"by {info.world_size} ranks", file=sys.stderr)
            return 2
        args.envs_per_group //= info.world_size
        # the per-rank group shrinks with N (8192 -> 1024 at N = 8): a lone 1024-env policy
        # step leaves most of the GPU idle (latency-bound), so strong scaling runs the groups'
        # steps on concurrent policy lanes -- the GPU then sees ~groups x envs_per_group envs
        # of acting work at a time, as at N = 1 (--lanes overrides)
        if args.lanes == 0:
            args.lanes = max(2, min(args.groups, info.world_size))
    if args.lanes == 0:
        args.lanes = min(2, args.groups)
    if info.world_size != args.gpus and info.is_main:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {info.world_size}; reporting "
              f"{info.world_size}", file=sys.stderr)
    dev = torch.device("cuda", info.local_rank)
    torch.set_num_threads(2)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(info.world_size)))
    # NUMA/core placement BEFORE any native thread exists (they inherit the affinity)
    cpus = launch.pin_rank(int(os.environ.get("LOCAL_RANK", "0")), local_world, dev.index)
    budget = launch.rank_cpu_budget(local_world)
    # env workers: the rank's CPU budget less one (the engine driver thread spins between
    # policy steps); profile 23 sweep on a 16-CPU share: 15 threads halve the env phase vs 13
    threads = args.threads or max(2, min(24, budget - 1))
    s = args.size

    def make_model():
        if args.arch == "gridnet":
            from microbeast_amd.models.gridnet import GridNetAgent
            return GridNetAgent((s, s, 27))
        if args.arch == "impala_deep":
            return Agent((s, s, 27), channels=(16, 32, 32, 32))
        return Agent((s, s, 27))

    torch.manual_seed(args.seed)
    from microbeast_amd import _native  # before the learner sizes its partial buffers
    from microbeast_amd.config import bwd_occupancy
    _native.check(_native.kernels().mbk_set_learner_occupancy(
        args.learner_fwd_occupancy, bwd_occupancy(args.learner_bwd_occupancy, args.arch)),
        "set_learner_occupancy")
    model = make_model()
    learner = Learner(model, LearnerHParams(bucket_mb=args.bucket_mb,
                                            allreduce_dtype=args.allreduce_dtype,
                                            comm_rehearsal=args.comm_rehearsal), dev, info)
    envs_total = args.groups * args.envs_per_group
    rt = GpuActorRuntime(make_model, s, args.groups, args.envs_per_group, args.unroll,
                         args.batch_slots, dev, n_threads=threads, seed=args.seed + 1000 * info.rank,
                         env_index_base=info.rank * envs_total,
                         selfplay_groups=args.selfplay_groups, fp8_policy=args.fp8_policy,
                         n_lanes=args.lanes, preroll=args.preroll)
    league = None
    if args.selfplay_groups > 0:
        from microbeast_amd.runtime.league import League
        league = League(capacity=16, snapshot_every=5, seed=args.seed + info.rank)
        league.current = league.add_snapshot(learner.flat.data)
    rt.start(learner.flat, opponent_version=league.current if league is not None else -1)
    frames_per_step = args.batch_slots * args.envs_per_group * args.unroll

    nstep = [0]
    lags = []

    def step():
        batch, slots = rt.get_batch(timeout=120.0)
        nstep[0] += 1
        if args.verbose:
            print(f"[rank {info.rank}] step {nstep[0]} slots {slots} {rt.stats()}",
                  file=sys.stderr, flush=True)
        lags.append(rt.policy_lag(slots, learner.n_updates))
        losses = learner.learn(batch)
        rt.release(slots)
        rt.publish(learner.flat, version=learner.n_updates)
        learner.phases.mark("publish")
        if league is not None:  # the full league loop is inside the timed step
            league.maybe_snapshot(nstep[0], learner.flat.data)
            league.record(rt.drain_episodes())
            sid = league.sample()
            if sid != league.current and rt.set_opponent(league.snapshot(sid), sid):
                league.current = sid
        return losses

    for _ in range(args.settle + args.warmup):
        losses = step()
    # --settle 0 (early-game transient): drop rollouts that piled up during the short warm-up
    # (graph capture, first-call setup) so the window does not consume a pre-filled backlog.
    # After a settle the queue of full rollouts is at its steady-state depth, which the window
    # also leaves behind at its end; draining it there would open the window on an empty
    # pipeline (the learner idles ~one step while acting refills it) and, at 20 steps, read
    # ~5 % below the same config's 150-step window (profile 42, r8h)
    # after a settle, open the window in the pipeline's median steady state -- exactly one full
    # rollout queued (starts with 0 or 2 moved a 20-step window by about -/+5 %; the window's
    # start and end depths are reported) -- running at most 8 more untimed updates to get there
    for _ in range(8 if args.settle > 0 else 0):
        if rt.stats().get("full_depth") == 1:
            break
        step()
    torch.cuda.synchronize()
    while args.settle == 0:
        slots = rt.engine.get_full(1, 0.0)
        if not slots:
            break
        rt.engine.release(slots, torch.cuda.current_stream().cuda_stream)
    D.barrier(info)
    st0 = rt.stats()
    lags.clear()
    t0 = time.perf_counter()
    win = (time.perf_counter(), st0)
    for i in range(args.steps):
        losses = step()
        if args.report_every > 0 and (i + 1) % args.report_every == 0 and info.is_main:
            now, st = time.perf_counter(), rt.stats()
            nst = max(1, st["act_steps"] - win[1]["act_steps"])
            print(f"[window] steps {i + 1 - args.report_every}-{i + 1}: "
                  f"{args.report_every * frames_per_step / (now - win[0]) / 1e6:.2f} M frames/s, "
                  f"active cells/env {(st['act_active_cells'] - win[1]['act_active_cells']) / (nst * rt.E):.3f}",
                  file=sys.stderr, flush=True)
            win = (now, st)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    D.barrier(info)
    st1 = rt.stats()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if info.enabled:
        torch.distributed.all_reduce(elapsed, op=torch.distributed.ReduceOp.MAX)
    el = float(elapsed.item())
    total_frames = frames_per_step * args.steps * info.world_size
    fps = total_frames / el
    loss_vals = [float(x) for x in losses.tolist()]
    phase_ms = learner.phases.read()  # HIP-event split of the last timed update (no sync)
    occ = _occupancy(rt)
    phase = None
    if args.profile_phases:
        learner.learn(rt.get_batch()[0], sync_timing=True)
        phase = learner.timing
    rt.stop()
    # every rank's actor side, so a weak-scaled N-GPU run shows which rank (if any) is
    # CPU-bound: env workers busy ~100 % of the time means the rank's CPU share, not the
    # GPU, sets its frame rate (each rank steps its own envs)
    steps_done = max(1, st1["gpu_steps"] - st0["gpu_steps"])
    busy = (st1["env_s"] - st0["env_s"]) / (el * threads)
    mine = {"rank": info.rank, "cpus_per_rank": budget, "env_threads": threads,
            "env_worker_busy_frac": round(busy, 3),
            "env_cores_busy": round(busy * threads, 2),
            "frames_stepped_per_s": round((st1["frames"] - st0["frames"]) / el, 1),
            "gpu_phase_ms": round(1e3 * (st1["gpu_phase_s"] - st0["gpu_phase_s"]) / steps_done, 3),
            "env_phase_ms": round(1e3 * (st1["env_phase_s"] - st0["env_phase_s"]) / steps_done, 3)}
    na = st1.get("act_steps", 0) - st0.get("act_steps", 0)
    if na:  # fused acting steps: the agent's idle units per env and step (the game phase)
        mine["active_cells_per_env"] = round(
            (st1["act_active_cells"] - st0["act_active_cells"]) / (na * rt.E), 3)
    ranks = D.gather_objects(mine, info)
    cpu_bound = [r["rank"] for r in ranks if r["env_worker_busy_frac"] >= CPU_BOUND_BUSY]
    if cpu_bound and info.is_main:
        print(f"warning: env workers of rank(s) {cpu_bound} are >= {CPU_BOUND_BUSY:.0%} busy: "
              f"those ranks are CPU-bound on their {budget}-CPU share (give each rank more CPUs "
              f"or fewer envs)", file=sys.stderr)
    if info.is_main:
        out = {
            "metric": f"env frames/sec (whole node) on {s}x{s} microRTS",
            "value": round(fps, 1),
            "unit": "frames/s",
            # game phase the window measured: the agent's idle units (cells the sparse head
            # samples) per env and policy step, rank 0; the head's and the env's work grow with it
            "active_cells_per_env": mine.get("active_cells_per_env"),
            "n_gpus": info.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * el / args.steps, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            # BASELINE.md's 38.9 fps is quoted on the 16x16 IMPALA config only
            "vs_baseline": (round(fps / BASELINE_FPS, 1)
                            if args.arch == "impala_flat" and s == 16 else None),
            "dtype": "bf16" + (" (fp8 e4m3 acting trunk)" if args.fp8_policy else ""),
            "data": ("synthetic (native microRTS stand-in env, "
                     + (f"random-init weights after {args.settle} untimed training updates)"
                        if args.settle else "random-init weights)")),
            "config": {
                "model": (f"impala_flat IMPALA-CNN 16/32/32 + FC256 + flat 78x{s}x{s} head "
                          f"({num_params(model) / 1e6:.2f}M params)" if args.arch == "impala_flat"
                          else f"{args.arch} ({num_params(model) / 1e6:.2f}M params)"),
                "map": f"{s}x{s}",
                "global_batch": frames_per_step * info.world_size,
                "seq_len": args.unroll,
                "parallelism": f"dp{info.world_size}",
                "opponents": (f"self-play league on {args.selfplay_groups}/{args.groups} groups"
                              if args.selfplay_groups else "scripted bots"),
                "envs_per_gpu": envs_total,
                "env_groups": f"{args.groups} x {args.envs_per_group}",
                "env_threads_per_gpu": threads,
                "cpus_per_rank": budget,  # the rank's quota-limited CPU budget
                "cpu_affinity_per_rank": len(cpus),
                "policy_lanes": rt.n_lanes,
                "allreduce": f"{args.allreduce_dtype} {args.bucket_mb:g}MB buckets",
                "settle_updates": args.settle,
                "comm_rehearsal": args.comm_rehearsal,
                "preroll": args.preroll,
            },
            "actor_stats": {
                "env_frames_stepped_per_s_rank0": round((st1["frames"] - st0["frames"]) / el, 1),
                "env_worker_busy_frac": round((st1["env_s"] - st0["env_s"]) / (el * threads), 3),
                "gpu_policy_steps_per_s": round((st1["gpu_steps"] - st0["gpu_steps"]) / el, 1),
                "publishes": st1["publishes"] - st0["publishes"],
                # rollouts queued for the learner when the window opened / closed: the window
                # starts and ends in the same pipeline state (no pre-filled backlog consumed)
                "full_slots_waiting": {"start": st0.get("full_depth"),
                                       "end": st1.get("full_depth")},
                "slot_wait_s": round(st1["slot_wait_s"] - st0["slot_wait_s"], 3),
                "driver_idle_s": round(st1["driver_idle_s"] - st0["driver_idle_s"], 3),
                # per group step: GPU latency (enqueue -> done seen) and CPU env phase
                "gpu_phase_ms": round(1e3 * (st1["gpu_phase_s"] - st0["gpu_phase_s"])
                                      / max(1, st1["gpu_steps"] - st0["gpu_steps"]), 3),
                "env_phase_ms": round(1e3 * (st1["env_phase_s"] - st0["env_phase_s"])
                                      / max(1, st1["gpu_steps"] - st0["gpu_steps"]), 3),
                "enqueue_ms": round(1e3 * (st1["enqueue_s"] - st0["enqueue_s"])
                                    / max(1, st1["gpu_steps"] - st0["gpu_steps"]), 3),
                "graph_launch_ms": round(1e3 * (st1["graph_launch_s"] - st0["graph_launch_s"])
                                         / max(1, st1["gpu_steps"] - st0["gpu_steps"]), 3),
            },
            # occupied cells per env in the rows launch A read at the window's end (its first
            # access reads 32 words: rows of more than 31 cells cost a second PCIe round trip)
            "occupied_cells_per_env": occ,
            "actor_stats_per_rank": ranks,
            "cpu_bound_ranks": cpu_bound,
            "learner_phase_ms_rank0": {k: round(v, 3) for k, v in phase_ms.items()},
            "policy_lag_updates": ({"mean": round(sum(lags) / len(lags), 2), "max": max(lags)}
                                   if lags else None),
            "last_losses": {"pg": loss_vals[0], "value": loss_vals[1], "entropy": loss_vals[2],
                            "total": loss_vals[3]},
        }
        if phase:
            out["learner_phase_s"] = phase
        nt = st1.get("timed_steps", 0) - st0.get("timed_steps", 0)
        if nt > 0:  # MBK_STEP_TIMING=1: GPU-side split of a policy step's own stream time
            out["policy_step_gpu_ms"] = {
                k: round(1e3 * (st1[f"step_{k}_s"] - st0[f"step_{k}_s"]) / nt, 3)
                for k in ("h2d", "graph", "out")}
        print(json.dumps(out), flush=True)
    D.destroy(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
