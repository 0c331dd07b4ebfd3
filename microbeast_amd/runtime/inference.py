"""Dynamic-batching policy server for CPU actor processes (MonoRuntime).

Reference: every actor process ran its own CPU copy of the policy, one call per env
step (``agent.get_action`` at microbeast.py:86-87, 6 envs per call), reading weights
from a shared nn.Module. With a GPU learner that wastes the GPU and puts the 7*h*w
Python categoricals on every actor's single CPU thread (238 ms per 16x16
step). Here the actors keep stepping their environments on the CPU (the only option
for the JVM gym-microRTS env, which cannot share a process) and send observations to
ONE server in the learner process:

* request area: per-actor rows of obs bits / mask bits in POSIX shared memory,
  page-locked in the server process (``host_register``) so the upload is one DMA;
* request ring (native lock-free ``IndexRing``, futex wait): actors push their id;
* the server takes the first id, then keeps draining until ``max_wait_ms`` passes or
  every actor is in the batch (timeout-based dynamic batching);
* one H2D of the request area, a device-side row gather, one policy call on the
  high-priority inference stream (HIP conv trunk + sparse sampled head), one D2H
  into pinned staging, a CPU scatter into the actors' response rows, and a push on
  each actor's response ring;
* weights: the learner's ``publish`` copies its flat buffer into a device staging
  copy on the learner stream and records an event; the server applies it between
  two batches once that event has executed (D2D), so a batch never mixes weight versions
  and the inference stream never waits for the learner's queued update.

The server also runs on a CPU device (same protocol; used by the CPU test suite).
"""
from __future__ import annotations

import threading
import time

import torch

from .. import _native as N
from ..ops.copy import row_gather
from ..ops.optim import FlatParams
from ..utils.buffers import ShmRing


class InferenceClient:
    """Actor-side handle (picklable: shared-memory tensors + ring names)."""

    def __init__(self, actor_id: int, req_obs, req_mask, resp_action, resp_logp, resp_value,
                 requests: ShmRing, response: ShmRing):
        self.actor_id = actor_id
        self.obs = req_obs[actor_id]
        self.mask = req_mask[actor_id]
        self.action = resp_action[actor_id]
        self.logp = resp_logp[actor_id]
        self.value = resp_value[actor_id]
        self.requests, self.response = requests, response
        self.seq = None

    def act(self, timeout: float = 600.0):
        """Ask for actions on ``self.obs`` / ``self.mask`` (already written by the env).
        Returns (action [n,S,7] u8, logp [n], value [n]) views of the response rows, or
        None if the server shut down.

        Requests carry a sequence number (``seq << 16 | actor_id``) that the server
        echoes, so an actor respawned by the watchdog ignores replies addressed to the
        process it replaced."""
        if self.seq is None:  # first call in this process: start from a fresh number
            import os
            self.seq = (os.getpid() << 8) & ((1 << 40) - 1)
        self.seq = (self.seq + 1) & ((1 << 40) - 1)
        if not self.requests.push((self.seq << 16) | self.actor_id, timeout):
            return None
        t0 = time.perf_counter()
        while True:
            v = self.response.pop(1.0)
            if v == self.seq:
                return self.action, self.logp, self.value
            if v is None and (self.response.ring.closed() or time.perf_counter() - t0 > timeout):
                return None


class InferenceServer:
    def __init__(self, make_model, n_actors: int, n_envs: int, size: int, device,
                 max_wait_ms: float = 2.0, seed: int = 1):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.n_actors, self.n_envs, self.S = n_actors, n_envs, size * size
        A, n, S = n_actors, n_envs, self.S
        self.req_obs = torch.zeros(A, n, S, dtype=torch.int32).share_memory_()
        self.req_mask = torch.zeros(A, n, S, 3, dtype=torch.int32).share_memory_()
        self.resp_action = torch.zeros(A, n, S, 7, dtype=torch.uint8).share_memory_()
        self.resp_logp = torch.zeros(A, n, dtype=torch.float32).share_memory_()
        self.resp_value = torch.zeros(A, n, dtype=torch.float32).share_memory_()
        self.requests = ShmRing(A + 1)
        self.responses = [ShmRing(4) for _ in range(A)]
        self.max_wait_s = max_wait_ms * 1e-3
        self.model = make_model().to(self.device)
        self.model.eval()
        self.flat = FlatParams(self.model, self.device)
        self._registered = []
        self.batches = 0
        self.requests_served = 0
        self._lock = threading.Lock()
        self._pending = None  # (staging, event) of a publish not applied yet
        self._stop = threading.Event()
        self._thread = None
        self._error = None
        if self.cuda:
            self._pin(self.req_obs, self.req_mask)
            self.stream = torch.cuda.Stream(self.device, priority=-1)
            self.d_obs = torch.empty(A, n, S, dtype=torch.int32, device=self.device)
            self.d_mask = torch.empty(A, n, S, 3, dtype=torch.int32, device=self.device)
            self.h_ids = torch.empty(A, dtype=torch.int64).pin_memory()
            self.h_action = torch.empty(A * n, S, 7, dtype=torch.uint8).pin_memory()
            self.h_logp = torch.empty(A * n, dtype=torch.float32).pin_memory()
            self.h_value = torch.empty(A * n, dtype=torch.float32).pin_memory()
            self.rng = torch.tensor([seed * 7919 + 17, 0], dtype=torch.int64, device=self.device)
            self._staging = torch.empty_like(self.flat.data)
            self._consumed = torch.cuda.Event()
            self._consumed.record(self.stream)
        else:
            self.gen = torch.Generator().manual_seed(seed * 7919 + 17)

    def _pin(self, *tensors):
        rt = N.runtime()
        for t in tensors:
            err = rt.host_register(t.data_ptr(), t.numel() * t.element_size())
            if err != 0:
                raise RuntimeError(f"hipHostRegister of the shared request area failed ({err})")
            self._registered.append(t)

    def client(self, actor_id: int) -> InferenceClient:
        return InferenceClient(actor_id, self.req_obs, self.req_mask, self.resp_action,
                               self.resp_logp, self.resp_value, self.requests,
                               self.responses[actor_id])

    # ------------------------------------------------------------ weights
    def publish(self, learner_flat: torch.Tensor) -> None:
        """Hand the learner's current weights to the server (applied before its next
        batch). Called on the learner's stream; never blocks on the server."""
        src = learner_flat.detach()
        if not self.cuda:
            with self._lock:
                self.flat.data.copy_(src.to(self.device))
            return
        with self._lock:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(self._consumed)  # the previous staging copy-out has executed
            self._staging.copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cur)
            self._pending = ev

    def _apply_pending(self):
        with self._lock:
            ev, self._pending = self._pending, None
            if ev is None:
                return
            if not ev.query():
                # the learner's thread publishes once it has queued an update: waiting on the
                # staging copy here would hold the inference stream until that whole update
                # ran; a later batch applies it (a newer publish supersedes it meanwhile)
                self._pending = ev
                return
            self.stream.wait_event(ev)
            with torch.cuda.stream(self.stream):
                self.flat.data.copy_(self._staging, non_blocking=True)
            self._consumed.record(self.stream)

    # ------------------------------------------------------------ serving
    def start(self):
        self._thread = threading.Thread(target=self._loop, name="inference-server", daemon=True)
        self._thread.start()

    def _collect(self) -> dict[int, int]:
        """{actor id: request seq} of one dynamic batch."""
        first = self.requests.pop(0.2)
        if first is None:
            return {}
        reqs = {int(first) & 0xFFFF: int(first) >> 16}
        deadline = time.perf_counter() + self.max_wait_s
        while len(reqs) < self.n_actors:
            left = deadline - time.perf_counter()
            if left <= 0:
                break
            v = self.requests.pop(left)
            if v is None:
                break
            reqs[int(v) & 0xFFFF] = int(v) >> 16
        return reqs

    def _serve(self, reqs: dict[int, int]):
        ids = sorted(reqs)
        k, n, S = len(ids), self.n_envs, self.S
        if not self.cuda:
            idx = torch.tensor(ids, dtype=torch.int64)
            with torch.no_grad(), self._lock:
                a, lp, v = self.model.act(self.req_obs.index_select(0, idx).view(k * n, S),
                                          self.req_mask.index_select(0, idx).view(k * n, S, 3),
                                          generator=self.gen)
            self.resp_action.index_copy_(0, idx, a.view(k, n, S, 7))
            self.resp_logp.index_copy_(0, idx, lp.view(k, n).float())
            self.resp_value.index_copy_(0, idx, v.view(k, n).float())
        else:
            self._apply_pending()
            self.h_ids[:k] = torch.tensor(ids, dtype=torch.int64)
            with torch.cuda.stream(self.stream), torch.no_grad():
                # one DMA of the whole (pinned) request area, gather on the device
                self.d_obs.copy_(self.req_obs, non_blocking=True)
                self.d_mask.copy_(self.req_mask, non_blocking=True)
                idx = self.h_ids[:k].to(self.device, non_blocking=True)
                obs = row_gather(self.d_obs, idx, k).view(k * n, S)
                mask = row_gather(self.d_mask, idx, k).view(k * n, S, 3)
                a, lp, v = self.model.act(obs, mask, rng_state=self.rng)
                self.h_action[:k * n].copy_(a.view(k * n, S, 7), non_blocking=True)
                self.h_logp[:k * n].copy_(lp.view(-1), non_blocking=True)
                self.h_value[:k * n].copy_(v.view(-1), non_blocking=True)
            self.stream.synchronize()
            idx = self.h_ids[:k]
            self.resp_action.index_copy_(0, idx, self.h_action[:k * n].view(k, n, S, 7))
            self.resp_logp.index_copy_(0, idx, self.h_logp[:k * n].view(k, n))
            self.resp_value.index_copy_(0, idx, self.h_value[:k * n].view(k, n))
        for i in ids:
            self.responses[i].push(reqs[i], 1.0)
        self.batches += 1
        self.requests_served += k

    def _loop(self):
        if self.cuda:
            torch.cuda.set_device(self.device)
        try:
            while not self._stop.is_set():
                reqs = self._collect()
                if reqs:
                    self._serve(reqs)
        except BaseException as e:  # surfaced through check()
            self._error = e
            for r in self.responses:
                r.close()

    def check(self):
        if self._error is not None:
            raise RuntimeError(f"inference server failed: {self._error!r}") from self._error

    def stats(self) -> dict:
        return {"batches": self.batches, "requests": self.requests_served,
                "mean_batch_actors": self.requests_served / max(1, self.batches)}

    def stop(self):
        self._stop.set()
        self.requests.close()
        for r in self.responses:
            r.close()
        if self._thread is not None:
            self._thread.join(10)
        if self.cuda:
            torch.cuda.synchronize(self.device)
            rt = N.runtime()
            for t in self._registered:
                rt.host_unregister(t.data_ptr())
            self._registered = []
        self.requests.unlink()
        for r in self.responses:
            r.unlink()
