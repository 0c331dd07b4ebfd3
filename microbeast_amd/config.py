"""Configuration + CLI.

Reference CLI (parser.py:1-15): ``--test`` (flag, or ``--test true/false``)
and ``--exp_name`` (default "No_name", interactive prompt when omitted,
microbeast.py:123-124). Everything the reference hard-codes in ``train()``
(microbeast.py:113-121), ``create_env`` (libs/utils.py:64-75) and
``PPO_learn`` (libs/utils.py:277-329) is a flag here, defaulting to the
reference value. ``strtobool`` is implemented (the reference used it without
importing it, so ``--test true`` crashed there).
"""
from __future__ import annotations

import argparse
import dataclasses
import sys
from dataclasses import dataclass, field


def strtobool(v: str) -> bool:
    s = str(v).strip().lower()
    if s in ("y", "yes", "t", "true", "on", "1"):
        return True
    if s in ("n", "no", "f", "false", "off", "0"):
        return False
    raise argparse.ArgumentTypeError(f"invalid truth value {v!r}")


@dataclass
class Flags:
    # --- reference CLI
    exp_name: str = "No_name"
    test: bool = False
    # --- run shape (reference microbeast.py:113-121)
    n_actors: int = 10
    n_envs: int = 6
    env_size: int = 8
    unroll_length: int = 64
    batch_size: int = 0           # rollout slots per update; 0 = auto: 2 on the mono runtime
                                  # (the reference's B = 2, microbeast.py:117), 1 on the gpu
                                  # runtime (one 8192-env x 64-step slot = 524,288 frames: the
                                  # benched update, and --lr_base_batch, so the lr stays 2.5e-4)
    n_buffers: int = 0            # 0 -> max(2 * n_actors, batch_size)
    total_steps: int = 100_000_000
    max_episode_steps: int = 2000
    # --- algorithm (libs/utils.py:277-329, microbeast.py:200)
    gamma: float = 0.99
    lr: float = 2.5e-4
    adam_eps: float = 1e-5
    baseline_cost: float = 0.5
    entropy_cost: float = 0.01
    rho_bar: float = 1.0
    c_bar: float = 1.0
    pg_rho_bar: float = 1.0
    reward_clip: float = 0.0
    max_grad_norm: float = 0.0
    # --- environment
    env: str = "synthetic"        # synthetic | microrts (gym-microrts adapter, if installed)
    opponents: str = "coac,coac,coac,random_biased,light_rush,worker_rush"
    reward_weight: str = "10,1,1,0.2,1,4"
    self_play: bool = False       # gpu runtime: self-play league (past snapshots as opponents)
    selfplay_groups: int = 1      # with --self_play: env groups playing the league (rest: bots)
    league_size: int = 16         # snapshots kept in HBM
    league_update_every: int = 50  # updates between snapshots
    pfsp_power: float = 2.0       # opponent weight (1 - win rate)^p
    league_eps: float = 0.1       # uniform mixing of the matchmaking distribution
    # --- model
    arch: str = "impala_flat"     # impala_flat | gridnet | impala_deep
    channels: str = "16,32,32"
    hidden: int = 256
    dtype: str = "bf16"           # fp32 | bf16 | fp8 (= bf16 learner + fp8 acting trunk)
    fp8_policy: bool = False      # gpu runtime: acting trunk on fp8 (e4m3) MFMA convs
    # --- runtime
    runtime: str = "auto"         # auto | gpu (native engine) | mono (CPU actor processes)
    device: str = "auto"          # auto | cpu | cuda
    groups: int = 4               # gpu runtime: env groups pipelined through the GPU
    envs_per_group: int = 8192    # (4 x 8192 on 2 lanes = the benched headline config, bench.py)
    actor_threads: int = 0        # gpu runtime: native env worker threads (0 = auto)
    policy_lanes: int = 2         # gpu runtime: concurrent policy streams (own graph + I/O each)
    actor_inference: str = "auto"  # mono runtime: server (batched policy in the learner
                                   # process) | local (CPU policy per actor) | auto
    inference_wait_ms: float = 2.0  # mono runtime server: dynamic-batching window
    seed: int = 1
    nproc_per_node: int = 1       # >1: launch that many DP ranks (one per GPU) over RCCL
    bucket_mb: float = 8.0
    allreduce_dtype: str = "fp32"  # fp32 | bf16 gradient all-reduce payload (fp32 master grads)
    rccl_high_priority: bool = True  # RCCL collectives on a high-priority stream
    learner_bwd_occupancy: int = -1  # gpu runtime: learner backward workgroups per CU (-1 = auto; 0 = as
                                    # many as fit; 1 leaves the acting kernels a slot, profile 45)
    learner_fwd_occupancy: int = 0  # gpu runtime: learner forward workgroups per CU (0 = as many as fit)
    lr_scaling: str = "sqrt"      # none | sqrt | linear: lr *= max(1, frames per update / lr_base_batch)^k
    lr_base_batch: int = 524288   # frames per update the base lr is tuned for (1 GPU, 4 x 8192 x 64 / 4)
    episode_sync_every: int = 10  # DP: gather finished episodes to rank 0 every N updates
    profile_updates: int = 0      # >0: torch.profiler trace of that many updates -> savedir
    # --- io / robustness
    savedir: str = "."
    checkpoint_every: int = 100   # updates
    resume: bool = False
    checkpoint: str = ""          # path for --test / --resume (default <savedir>/<exp>.ckpt)
    eval_episodes: int = 10
    allow_random_init: bool = False  # --test without a checkpoint: evaluate random weights
                                     # instead of failing
    batch_timeout: float = 600.0
    actor_restarts: int = 3       # watchdog: respawn a dead actor at most this often
    fault_inject_every: int = 0   # kill an actor every N updates (tests the watchdog)
    log_every: int = 1
    quiet: bool = False
    max_updates: int = 0          # stop after N updates (0 = until total_steps)

    def resolved_batch_size(self, runtime: str) -> int:
        """--batch_size 0 (the default) picks the per-runtime value (see the field)."""
        if self.batch_size > 0:
            return self.batch_size
        return 1 if runtime == "gpu" else 2

    def resolved_n_buffers(self) -> int:
        return self.n_buffers or max(2 * self.n_actors, self.resolved_batch_size("mono"))

    def opponent_list(self) -> list[str]:
        return [s.strip() for s in self.opponents.split(",") if s.strip()]

    def reward_weights(self) -> list[float]:
        return [float(x) for x in self.reward_weight.split(",")]

    def channel_list(self) -> tuple[int, ...]:
        return tuple(int(x) for x in self.channels.split(","))


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        prog="microbeast",
        description="microbeast_amd: MI355X-native IMPALA for (synthetic) gym-microRTS")
    p.add_argument("--test", type=strtobool, default=False, nargs="?", const=True,
                   help="evaluate a saved model instead of training")
    p.add_argument("--exp_name", type=str, default="No_name", nargs="?",
                   help="name of the result tables of this experiment")
    for f in dataclasses.fields(Flags):
        if f.name in ("test", "exp_name"):
            continue
        flag = "--" + f.name
        if f.type in ("bool", bool):
            p.add_argument(flag, type=strtobool, default=f.default, nargs="?", const=True)
        elif f.type in ("int", int):
            p.add_argument(flag, type=int, default=f.default)
        elif f.type in ("float", float):
            p.add_argument(flag, type=float, default=f.default)
        else:
            p.add_argument(flag, type=str, default=f.default)
    return p


def parse_flags(argv=None, interactive: bool | None = None) -> Flags:
    ns = build_parser().parse_args(argv)
    flags = Flags(**vars(ns))
    if interactive is None:
        interactive = sys.stdin is not None and sys.stdin.isatty()
    if flags.exp_name in (None, "No_name") and interactive and not flags.test:
        name = input("Nombre del experimento:").strip()  # reference microbeast.py:124
        if name:
            flags.exp_name = name
    if flags.exp_name is None:
        flags.exp_name = "No_name"
    return flags


__all__ = ["Flags", "build_parser", "parse_flags", "strtobool", "field"]


def bwd_occupancy(requested: int, arch: str) -> int:
    """The learner's backward workgroups per CU under the GPU actor runtime (-1 = auto): one
    for the headline IMPALA-flat model, whose acting kernels need a slot beside the learner
    (+4-7 %), none for the learner-heavy GridNet / deep IMPALA configs (the cap measured -7 /
    -2 % there, profile 45)."""
    if requested >= 0:
        return requested
    return 1 if arch == "impala_flat" else 0
