"""CPU actor processes + learner ("MonoBeast" shape of the reference).

Reference: ``act()`` (microbeast.py:30-105), the spawn loop
(microbeast.py:179-191), ``get_batch`` (libs/utils.py:166-218) and the
in-place weight sync (libs/utils.py:337). Kept as the parity / CPU-only
runtime (BASELINE config 1: 4x4, 2 CPU actors + CPU learner) and as the
reference for the native GPU engine. Fixed on the way:

* every actor steps the configured map size (reference hard-coded 8, D5);
* weights are published into a shared flat buffer under a seqlock and
  actors copy a consistent version at rollout boundaries (no torn reads);
* the index hand-off is the native shm ring (no pickling / busy spin);
* a watchdog respawns dead actors and recycles the slot they held; an
  optional fault injector kills actors to exercise it;
* clean shutdown: rings are closed, actors exit, processes are joined;
* with a GPU learner (BASELINE config 2) actors send observations to a
  dynamic-batching policy server in the learner process instead of running a CPU
  policy each (``runtime/inference.py``), and full slots reach HBM through pinned
  DMA on a copy stream one batch ahead of the learner (``runtime/staging.py``).
"""
from __future__ import annotations

import os
import random
import signal
import time

import torch
import torch.multiprocessing as mp

from .. import _native as N
from ..utils.buffers import ShmRing, create_buffers, get_batch


def _actor_main(actor_id: int, flags_dict: dict, buffers, free_ring: ShmRing, full_ring: ShmRing,
                weights: torch.Tensor, version: torch.Tensor, cur_slot: torch.Tensor,
                episode_q, seed: int, client=None):
    """Child process: step a vec-env, fill slots. Actions come from a CPU copy of the
    policy, or from the learner process's inference server when ``client`` is given."""
    os.environ["OMP_NUM_THREADS"] = "1"
    torch.set_num_threads(1)
    if not (free_ring.alive and full_ring.alive):
        return  # the runtime stopped before this actor finished spawning
    from ..config import Flags
    from ..envs.synthetic import create_env
    from ..models.factory import make_model
    from ..ops.optim import FlatParams

    flags = Flags(**flags_dict)
    rt = N.runtime()
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed)
    s, n, T = flags.env_size, flags.n_envs, flags.unroll_length
    rank = int(os.environ.get("RANK", "0"))  # DP: every rank owns its own actor pool
    env = create_env(s, n, flags.max_episode_steps, seed=seed, opponents=flags.opponent_list(),
                     reward_weight=flags.reward_weights(),
                     env_index_base=(rank * flags.n_actors + actor_id) * n,
                     env=flags.env)
    model = flat = None
    if client is None:
        model = make_model(flags, torch.device("cpu"))
        model.eval()
        flat = FlatParams(model, "cpu")
    my_version = -1

    def refresh():
        nonlocal my_version
        if flat is None:
            return  # the server applies weight publishes itself
        v = int(version[0].item())
        if v == my_version:
            return
        got = rt.seqlock_read(version.data_ptr(), weights.data_ptr(), flat.data.data_ptr(),
                              flat.numel * 4, 100000)
        if got:
            my_version = got - 1

    S = s * s
    if client is not None:  # the env writes straight into this actor's request rows
        obs, mask = client.obs, client.mask
    else:
        obs = torch.zeros(n, S, dtype=torch.int32)
        mask = torch.zeros(n, S, 3, dtype=torch.int32)
    rew = torch.zeros(n)
    done = torch.zeros(n, dtype=torch.uint8)
    env.reset_compact(obs, mask)
    last_action = torch.zeros(n, S, 7, dtype=torch.uint8)
    ep_ret = torch.zeros(n)
    ep_len = torch.zeros(n, dtype=torch.int32)
    while True:
        idx = free_ring.pop(-1.0)
        if idx is None or idx < 0:
            break
        cur_slot[actor_id] = idx
        refresh()
        with torch.no_grad():
            for t in range(T + 1):
                buffers["obs"][idx][t].copy_(obs)
                buffers["action_mask"][idx][t].copy_(mask)
                buffers["last_action"][idx][t].copy_(last_action)
                if client is None:
                    a, lp, v = model.act(obs, mask, generator=gen)
                else:
                    got = client.act()
                    if got is None:  # server shut down
                        return
                    a, lp, v = got
                buffers["action"][idx][t].copy_(a)
                buffers["logprobs"][idx][t].copy_(lp)
                buffers["baseline"][idx][t].copy_(v)
                if t == T:
                    break  # obs_T / mask_T are the bootstrap row; a_T is re-sampled next slot
                env.step_compact(a, obs, mask, rew, done)
                ep_ret += rew
                ep_len += 1
                buffers["reward"][idx][t].copy_(rew)
                buffers["done"][idx][t].copy_(done)
                buffers["ep_return"][idx][t].copy_(ep_ret)
                buffers["ep_step"][idx][t].copy_(ep_len)
                d = done.bool()
                ep_ret[d] = 0
                ep_len[d] = 0
                last_action.copy_(a)
        eps = env.drain_episodes()
        if eps:
            episode_q.put(eps)
        cur_slot[actor_id] = -1
        if not full_ring.push(idx, -1.0):
            break


class MonoRuntime:
    """Owns buffers, rings, actor processes and the watchdog."""

    def __init__(self, flags, model_numel: int, device=None, make_model=None):
        self.flags = flags
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        n_buf = flags.resolved_n_buffers()
        self.buffers = create_buffers(n_buf, flags.n_envs, flags.unroll_length, flags.env_size)
        self.free = ShmRing(n_buf + 1)
        self.full = ShmRing(n_buf + 1)
        for i in range(n_buf):
            self.free.push(i)
        self.weights = torch.zeros(model_numel, dtype=torch.float32).share_memory_()
        self.version = torch.zeros(1, dtype=torch.int64).share_memory_()
        self.cur_slot = torch.full((flags.n_actors,), -1, dtype=torch.int64).share_memory_()
        self.ctx = mp.get_context("spawn")
        self.episode_q = self.ctx.SimpleQueue()
        self.procs: list = [None] * flags.n_actors
        self.restarts = 0
        self.frames_per_slot = flags.n_envs * flags.unroll_length
        mode = getattr(flags, "actor_inference", "auto")
        if mode == "auto":
            mode = "server" if self.device.type == "cuda" else "local"
        if mode not in ("server", "local"):
            raise ValueError(f"--actor_inference must be auto|server|local, got {mode!r}")
        self.server = None
        if mode == "server":
            from .inference import InferenceServer
            if make_model is None:
                raise ValueError("the inference server needs make_model")
            self.server = InferenceServer(make_model, flags.n_actors, flags.n_envs,
                                          flags.env_size, self.device,
                                          max_wait_ms=getattr(flags, "inference_wait_ms", 2.0),
                                          seed=flags.seed)
        self.prefetcher = None

    def enable_prefetch(self, device, depth: int = 2):
        """GPU learner: pinned-DMA slot uploads one batch ahead (runtime/staging.py)."""
        from .staging import PinnedPrefetcher
        self.prefetcher = PinnedPrefetcher(self, device, depth, self.flags.batch_timeout)

    def publish(self, flat_data: torch.Tensor) -> None:
        if self.server is not None:
            self.server.publish(flat_data)
            return
        rt = N.runtime()
        src = flat_data.detach()
        if src.is_cuda:
            src = src.cpu()
        src = src.contiguous()
        assert src.numel() == self.weights.numel() and src.dtype == self.weights.dtype
        rt.seqlock_write(self.version.data_ptr(), src.data_ptr(), self.weights.data_ptr(),
                         src.numel() * src.element_size())

    def _spawn(self, i: int):
        fd = {k: getattr(self.flags, k) for k in self.flags.__dataclass_fields__}
        p = self.ctx.Process(target=_actor_main,
                             args=(i, fd, self.buffers, self.free, self.full, self.weights,
                                   self.version, self.cur_slot, self.episode_q,
                                   self.flags.seed * 1009 + i + 97 * self.restarts
                                   + 7919 * int(os.environ.get("RANK", "0")),
                                   self.server.client(i) if self.server is not None else None),
                             daemon=True)
        p.start()
        self.procs[i] = p

    def start(self):
        if self.server is not None:
            self.server.start()
        for i in range(self.flags.n_actors):
            self._spawn(i)

    def watchdog(self):
        """Respawn dead actors; give their in-flight slot back to the free ring."""
        for i, p in enumerate(self.procs):
            if p is not None and not p.is_alive():
                held = int(self.cur_slot[i].item())
                if held >= 0:
                    self.cur_slot[i] = -1
                    self.free.push(held)
                if self.restarts >= self.flags.actor_restarts:
                    raise RuntimeError(f"actor {i} died (exit {p.exitcode}) and the restart "
                                       f"budget ({self.flags.actor_restarts}) is spent")
                self.restarts += 1
                print(f"[watchdog] actor {i} died (exit {p.exitcode}); respawning", flush=True)
                self._spawn(i)

    def kill_random_actor(self):
        i = random.randrange(len(self.procs))
        p = self.procs[i]
        if p is not None and p.is_alive():
            os.kill(p.pid, signal.SIGKILL)
            p.join(5)

    def get_batch(self, timeout: float):
        if self.server is not None:
            self.server.check()
        if self.prefetcher is not None:
            return self.prefetcher.get_batch(timeout)
        return get_batch(self.flags.resolved_batch_size("mono"), self.free, self.full, self.buffers,
                         timeout=timeout, on_wait=self.watchdog)

    def drain_episodes(self):
        out = []
        while not self.episode_q.empty():
            out.extend(self.episode_q.get())
        return out

    def stop(self):
        if self.prefetcher is not None:
            self.prefetcher.stop()
        self.free.close()
        self.full.close()
        if self.server is not None:
            self.server.stop()
        for p in self.procs:
            if p is not None:
                p.join(5)
                if p.is_alive():
                    p.terminate()
                    p.join(2)
        time.sleep(0.05)
        self.free.unlink()
        self.full.unlink()
