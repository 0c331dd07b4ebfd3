"""Shared-memory rollout buffers + index rings for the CPU-actor runtime.

Reference: ``create_buffers`` / ``get_batch`` (libs/utils.py:29-55, 166-218)
and the free/full ``multiprocessing.Queue`` pair (microbeast.py:169-175).

Same key names as the reference; compact dtypes (obs uint32 bit planes,
masks 3 x uint32 bits per cell, actions uint8) so a 16x16 slot is ~6 KB per
env-step instead of ~170 KB; time-major ``[T+1, n, ...]`` per slot. Row t holds
obs_t / action_mask_t, the action a_t sampled there with its log-prob and
baseline, and reward_t / done_t obtained by stepping a_t (SURVEY §8 D3 fix);
``last_action`` is a_{t-1}. ``get_batch`` concatenates slots along the env
axis — time stays the leading axis (§8 D2 fix).

The index hand-off uses the native lock-free ``IndexRing`` living in POSIX
shared memory (futex sleep instead of busy-polling ``qsize()``).
"""
from __future__ import annotations

import time
from multiprocessing import shared_memory

import torch

from .. import _native as N

Buffers = dict  # str -> list[Tensor], like the reference's typing alias


def buffer_specs(n_envs: int, T: int, size: int, store_logits: bool = False) -> dict:
    S = size * size
    specs = dict(
        obs=((T + 1, n_envs, S), torch.int32),
        reward=((T + 1, n_envs), torch.float32),
        done=((T + 1, n_envs), torch.uint8),
        ep_return=((T + 1, n_envs), torch.float32),
        ep_step=((T + 1, n_envs), torch.int32),
        baseline=((T + 1, n_envs), torch.float32),
        last_action=((T + 1, n_envs, S, 7), torch.uint8),
        action=((T + 1, n_envs, S, 7), torch.uint8),
        action_mask=((T + 1, n_envs, S, 3), torch.int32),
        logprobs=((T + 1, n_envs), torch.float32),
    )
    if store_logits:
        specs["policy_logits"] = ((T + 1, n_envs, 78 * S), torch.float32)
    return specs


def create_buffers(n_buffers: int, n_envs: int, T: int, size: int,
                   store_logits: bool = False) -> Buffers:
    """n_buffers slots of shared-memory tensors (reference libs/utils.py:29-55)."""
    specs = buffer_specs(n_envs, T, size, store_logits)
    bufs: Buffers = {k: [] for k in specs}
    for _ in range(n_buffers):
        for k, (shape, dt) in specs.items():
            bufs[k].append(torch.zeros(shape, dtype=dt).share_memory_())
    return bufs


class ShmRing:
    """Picklable handle to a native IndexRing in POSIX shared memory."""

    def __init__(self, capacity: int, name: str | None = None, create: bool = True):
        rt = N.runtime()
        self.capacity = capacity
        nbytes = rt.IndexRing.bytes_needed(capacity)
        if create:
            self.shm = shared_memory.SharedMemory(create=True, size=nbytes)
        else:
            self.shm = shared_memory.SharedMemory(name=name)
        self.name = self.shm.name
        self._owner = create
        import ctypes

        self._addr = ctypes.addressof(ctypes.c_char.from_buffer(self.shm.buf))
        self.ring = rt.IndexRing(self._addr, capacity, create)

    def __getstate__(self):
        return {"capacity": self.capacity, "name": self.name}

    def __setstate__(self, st):
        try:
            self.__init__(st["capacity"], st["name"], create=False)
        except FileNotFoundError:
            # the owner already shut down and unlinked the ring while this (slow-spawning)
            # child was still starting: come up as a dead handle, the child then exits quietly
            self.capacity, self.name, self._owner = st["capacity"], st["name"], False
            self.shm = self.ring = None

    @property
    def alive(self) -> bool:
        return self.ring is not None

    def push(self, v: int, timeout: float = -1.0) -> bool:
        return self.ring.push(int(v), timeout)

    def pop(self, timeout: float = -1.0):
        return self.ring.pop(timeout)

    def size(self) -> int:
        return self.ring.size()

    def close(self):
        self.ring.close()

    def unlink(self):
        self.ring = None
        if self.shm is None:
            return
        try:
            self.shm.close()
        except BufferError:
            pass
        if self._owner:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass


LEARNER_KEYS = {"obs": "obs", "action_mask": "mask", "action": "action", "logprobs": "logp",
                "reward": "reward", "done": "done", "baseline": "baseline"}


def pop_full(batch_size: int, full_ring: ShmRing, timeout: float = 600.0, on_wait=None,
             stop=None) -> list[int]:
    """Pop ``batch_size`` full slot indices (``on_wait`` about once a second while waiting;
    ``stop()`` true or a closed ring -> return what was popped so far)."""
    idx = []
    t0 = time.perf_counter()
    while len(idx) < batch_size:
        v = full_ring.pop(1.0)
        if v is None:
            if on_wait is not None:
                on_wait()
            if (stop is not None and stop()) or full_ring.ring.closed():
                return idx
            if time.perf_counter() - t0 > timeout:
                raise TimeoutError(f"get_batch: no full slot within {timeout}s")
            continue
        idx.append(int(v))
    return idx


def get_batch(batch_size: int, free_ring: ShmRing, full_ring: ShmRing, buffers: Buffers,
              timeout: float = 600.0, on_wait=None, release: bool = True):
    """Pop ``batch_size`` full slots, return (time-major batch, indices).

    Keys are renamed to what the learner consumes: obs, mask, action, logp,
    reward, done (+ baseline). ``on_wait`` is called about once a second while
    waiting (watchdog hook). With ``release`` the slots go straight back to the
    free ring after the copy (CPU learner); otherwise the caller releases them.
    """
    idx = pop_full(batch_size, full_ring, timeout, on_wait)
    if len(idx) < batch_size:
        raise RuntimeError("get_batch: rollout ring closed")
    batch = {dst: torch.cat([buffers[src][m] for m in idx], dim=1)
             for src, dst in LEARNER_KEYS.items()}
    if release:
        for m in idx:
            free_ring.push(m)
    return batch, idx
