"""Rollout slots from CPU actor processes to HBM, one batch ahead of the learner.

Reference: ``get_batch`` (libs/utils.py:166-218) busy-waited on ``qsize()``, then
``torch.stack``-ed the B slots on the CPU and never moved the batch to a device
(the ``.to(device)`` was commented out, :216). For a GPU learner fed by CPU actor
processes (MonoRuntime, BASELINE config 2) this module:

* page-locks every shared-memory slot tensor once (``hipHostRegister`` via the native
  runtime), so slot uploads are DMA transfers straight out of the actors' pages;
* runs a prefetch thread that pops the next B full slots, issues their H2D copies on a
  dedicated copy stream into a fresh ``[B, T+1, n, ...]`` HBM batch, waits for the
  copies and only then returns the slots to the actors (no torn reads);
* hands finished batches to the learner through a bounded queue (``depth`` batches in
  flight: batch k+1 uploads while the learner computes on batch k); the learner's
  stream waits on the batch's copy event, and the time-major ``[T+1, B*n, ...]`` view
  is built on the device.
"""
from __future__ import annotations

import queue
import threading

import torch

from .. import _native as N
from ..utils.buffers import LEARNER_KEYS, pop_full


class PinnedPrefetcher:
    def __init__(self, runtime, device, depth: int = 2, timeout: float = 600.0):
        self.rt = runtime
        self.device = torch.device(device)
        self.B = runtime.flags.resolved_batch_size("mono")
        self.timeout = timeout
        self.copy_stream = torch.cuda.Stream(self.device)
        self.q: queue.Queue = queue.Queue(maxsize=max(1, depth))
        self._stop = threading.Event()
        self._error = None
        self._registered = []
        rtn = N.runtime()
        for src in LEARNER_KEYS:
            for t in runtime.buffers[src]:
                err = rtn.host_register(t.data_ptr(), t.numel() * t.element_size())
                if err != 0:
                    self._unpin()
                    raise RuntimeError(f"hipHostRegister of rollout buffer '{src}' failed ({err})")
                self._registered.append(t)
        self.h2d_bytes = 0
        self._thread = threading.Thread(target=self._loop, name="rollout-prefetch", daemon=True)
        self._thread.start()

    def _unpin(self):
        rtn = N.runtime()
        for t in self._registered:
            rtn.host_unregister(t.data_ptr())
        self._registered = []

    def _loop(self):
        torch.cuda.set_device(self.device)
        bufs = self.rt.buffers
        try:
            while not self._stop.is_set():
                idx = pop_full(self.B, self.rt.full, self.timeout, self.rt.watchdog,
                               stop=self._stop.is_set)
                if len(idx) < self.B:
                    for m in idx:  # shutting down: hand back what was taken
                        self.rt.free.push(m, 0.0)
                    return
                out = {}
                rtn = N.runtime()
                st = self.copy_stream.cuda_stream
                with torch.cuda.stream(self.copy_stream):
                    for src, dst in LEARNER_KEYS.items():
                        s0 = bufs[src][idx[0]]            # [T+1, n, ...] of one slot
                        T1 = s0.shape[0]
                        row = s0[0].numel() * s0.element_size()
                        # time-major [T+1, B, n, ...]: slot j is a strided column block
                        d = torch.empty((T1, self.B) + tuple(s0.shape[1:]), dtype=s0.dtype,
                                        device=self.device)
                        for j, m in enumerate(idx):
                            err = rtn.memcpy2d_async(d.data_ptr() + j * row, self.B * row,
                                                     bufs[src][m].data_ptr(), row, row, T1, st)
                            if err != 0:
                                raise RuntimeError(f"hipMemcpy2DAsync of '{src}' failed ({err})")
                            self.h2d_bytes += s0.numel() * s0.element_size()
                        out[dst] = d
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                ev.synchronize()  # the DMA has read the slots: actors may refill them
                for m in idx:
                    self.rt.free.push(m)
                while not self._stop.is_set():
                    try:
                        self.q.put((out, ev), timeout=0.5)
                        break
                    except queue.Full:
                        continue
        except BaseException as e:  # surfaced in get_batch
            self._error = e

    def get_batch(self, timeout: float):
        """Next device batch, time-major ``[T+1, B*n, ...]``; the current stream is ordered
        after its upload. Returns (batch, []) (slots were already recycled)."""
        waited = 0.0
        while True:
            if self._error is not None:
                raise RuntimeError(f"rollout prefetch failed: {self._error!r}") from self._error
            try:
                out, ev = self.q.get(timeout=1.0)
                break
            except queue.Empty:
                waited += 1.0
                if waited > timeout:
                    raise TimeoutError(f"no rollout batch within {timeout}s")
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        batch = {}
        for k, d in out.items():
            d.record_stream(cur)
            batch[k] = d.view((d.shape[0], d.shape[1] * d.shape[2]) + tuple(d.shape[3:]))
        return batch, []

    def stop(self):
        self._stop.set()
        self._thread.join(10)
        torch.cuda.synchronize(self.device)
        self._unpin()
