"""Data-parallel learners over torch.distributed (RCCL on ROCm, gloo on CPU).

The reference has no distributed code at all; BASELINE
configs 3/5 need 1 learner process per MI355X. Design for xGMI (7
point-to-point links per GPU, ring collectives per-link bound):

* one process per GPU, ``backend="nccl"`` (= librccl on ROCm);
* parameters live in ONE flat fp32 buffer (ops/optim.FlatParams), so the
  gradient all-reduce runs over a handful of large contiguous buckets
  (default >= 8 MB) — fewer, larger collectives amortise RCCL launch latency
  over the small (21 MB at 16x16) gradient;
* buckets are cut from the END of the flat buffer (head parameters first)
  and launched from post-accumulate-grad hooks as soon as their last
  gradient lands, so the 20 MB actor-head bucket's all-reduce overlaps the
  encoder backward;
* ``finish()`` waits on the async work (stream-ordered, no host sync); the
  1/world average is folded into the Adam kernel (``grad_scale``), not a
  separate pass over the gradient buffer;
* host-side objects (episode rows for the rank-0 CSV) travel over a separate
  gloo group, so gathering them never enqueues anything on a GPU stream or
  waits for the learner's kernels.

``MBK_FORCE_PG=1`` (or ``init_distributed(force_pg=True)``) creates a real
process group even at world size 1, so the RCCL path — broadcast, hook-fired
bucketed all-reduce, barrier, object gather — runs on a single-GPU box
(tests/test_gpu_dist_rccl.py).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from ..ops.optim import FlatParams


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    pg: bool = False          # a process group exists (world > 1, or forced at world 1)
    host_group: object = None  # gloo group for host objects (None: the default group is gloo)

    @property
    def enabled(self) -> bool:
        return self.world_size > 1 or self.pg

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(use_cuda: bool, timeout_s: float = 600.0,
                     force_pg: bool | None = None, high_priority: bool | None = None) -> DistInfo:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*).

    high_priority (default: MBK_RCCL_HIGH_PRIORITY, on): RCCL runs its collectives on a
    high-priority internal stream, so hook-fired all-reduce kernels do not queue behind the
    learner's long persistent backward kernels on the default-priority queues."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if force_pg is None:
        force_pg = os.environ.get("MBK_FORCE_PG", "0") == "1"
    if world <= 1 and not force_pg:
        if use_cuda:
            torch.cuda.set_device(local)
        return DistInfo(rank, world, local, "none")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # nccl == RCCL on ROCm; MBK_DIST_BACKEND=gloo lets several ranks share one GPU in tests
    backend = os.environ.get("MBK_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    if use_cuda:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if use_cuda and backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
            if high_priority is None:
                high_priority = os.environ.get("MBK_RCCL_HIGH_PRIORITY", "1") == "1"
            if high_priority:
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kw["pg_options"] = opts
        if "MASTER_PORT" not in os.environ:  # forced single-rank group outside torchrun
            from .launch import free_port
            kw.update(init_method=f"tcp://127.0.0.1:{free_port()}", rank=rank, world_size=world)
        dist.init_process_group(**kw)
    # the host group's timeout also bounds how long healthy ranks wait in agree() while a
    # peer rebuilds its actor engine (graph capture, HBM slots: seconds, up to --actor_restarts
    # times): give it room beyond the RCCL group's
    host = (dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=max(timeout_s, 1800)))
            if backend != "gloo" else None)
    return DistInfo(rank, world, local, backend, pg=True, host_group=host)


def broadcast_flat(flat: FlatParams, info: DistInfo) -> None:
    if info.enabled:
        dist.broadcast(flat.data, src=0)


# world-1 rehearsal of the hook-fired collectives (bench.py --comm_rehearsal): per bucket a
# stand-in kernel on a separate high-priority stream, RCCL-like grid (one workgroup per
# channel) and roughly a ring all-reduce's HBM bytes (2 read-modify-write sweeps of the bucket)
REHEARSAL_CHANNELS = 32
REHEARSAL_PASSES = 2


class GradAllReducer:
    """Bucketed, backward-overlapped gradient all-reduce over a FlatParams grad."""

    def __init__(self, flat: FlatParams, info: DistInfo, bucket_mb: float = 8.0,
                 comm_dtype: torch.dtype = torch.float32, rehearse: bool = False):
        """comm_dtype=bfloat16 all-reduces a bf16 copy of each bucket (half the xGMI bytes);
        the result is written back into the fp32 gradient buffer (fp32 master grads).
        rehearse (world size 1, no process group, GPU): the same buckets fire from the same
        hooks, but each launches ``mbk_comm_standin`` on a 4th, high-priority stream in place
        of RCCL's all-reduce, and ``finish`` makes the learner's stream wait for it as it
        waits for RCCL -- so a 1-GPU kernel trace shows whether the policy lanes or the
        learner serialize behind a collective's stream (docs/DESIGN.md §6). The gradient
        itself is never written."""
        self.flat, self.info = flat, info
        self.rehearse = bool(rehearse) and not info.enabled and flat.grad.is_cuda
        self.side = None      # rehearsal stream
        self.scratch = None   # rehearsal payload (the stand-in's accumulator)
        self.comm_dtype = comm_dtype
        self.grad_scale = 1.0 / max(1, info.world_size)  # applied inside Adam
        self.comm = None  # persistent low-precision payload (comm_dtype != fp32)
        self.buckets: list[tuple[int, int]] = []
        self.param_bucket: dict[int, int] = {}
        self.works = []
        self.pending: list[int] = []
        self.fired: list[bool] = []
        if not info.enabled and not self.rehearse:
            return
        if self.rehearse:
            self.side = torch.cuda.Stream(flat.grad.device, priority=-1)
            self.scratch = torch.zeros(flat.numel, dtype=torch.float32, device=flat.grad.device)
        limit = int(bucket_mb * 1e6 / 4)
        # walk parameters from last to first (backward order), cutting buckets
        cur_end, cur_start, members, groups = None, None, [], []
        for i in range(len(flat.slices) - 1, -1, -1):
            _, o, n, _ = flat.slices[i]
            end = flat.slices[i + 1][1] if i + 1 < len(flat.slices) else flat.numel
            if cur_end is None:
                cur_end = end
            cur_start = o
            members.append(i)
            if cur_end - cur_start >= limit:
                groups.append((cur_start, cur_end, members))
                cur_end, members = None, []
        if members:
            groups.append((0, cur_end, members))
        for b, (s, e, mem) in enumerate(groups):
            self.buckets.append((s, e))
            for i in mem:
                self.param_bucket[i] = b
        self.need = [sum(1 for i in self.param_bucket if self.param_bucket[i] == b)
                     for b in range(len(self.buckets))]
        self.count = [0] * len(self.buckets)
        self.fired = [False] * len(self.buckets)
        if comm_dtype != torch.float32:
            self.comm = torch.empty(flat.numel, dtype=comm_dtype, device=flat.grad.device)
        for i, p in enumerate(flat.params):
            p.register_post_accumulate_grad_hook(self._make_hook(i))

    def _make_hook(self, i: int):
        def hook(_p):
            b = self.param_bucket[i]
            self.count[b] += 1
            if self.count[b] == self.need[b] and not self.fired[b]:
                self._launch(b)
        return hook

    def _launch(self, b: int):
        s, e = self.buckets[b]
        self.fired[b] = True
        g = self.flat.grad[s:e]
        if self.rehearse:
            from .. import _native as N
            self.side.wait_stream(torch.cuda.current_stream())
            # (bucket starts are multiples of 4 floats: FlatParams pads every slice)
            N.check(N.kernels().mbk_comm_standin(g.data_ptr(), self.scratch[s:e].data_ptr(),
                                                 e - s, REHEARSAL_PASSES, REHEARSAL_CHANNELS,
                                                 self.side.cuda_stream), "comm_standin")
            return
        if self.comm is not None:
            c = self.comm[s:e]
            if g.is_cuda and c.dtype == torch.bfloat16:  # native narrowing copy (no ATen)
                from .. import _native as N
                N.check(N.kernels().mbk_to_bf16(g.data_ptr(), e - s, c.data_ptr(),
                                                N.stream_ptr()), "to_bf16")
            else:
                c.copy_(g)
            g = c
        self.works.append(dist.all_reduce(g, op=dist.ReduceOp.SUM, async_op=True))

    def start_step(self):
        if self.info.enabled or self.rehearse:
            self.count = [0] * len(self.buckets)
            self.fired = [False] * len(self.buckets)
            self.works = []

    def finish(self):
        """Launch any bucket whose params got no gradient and make the current stream wait
        for all of them (no host sync). The gradient is left as the SUM over ranks: the
        optimizer applies ``grad_scale`` (1/world) in its own pass."""
        if not self.info.enabled and not self.rehearse:
            return
        for b in range(len(self.buckets)):
            if not self.fired[b]:
                self._launch(b)
        if self.rehearse:
            torch.cuda.current_stream().wait_stream(self.side)
            return
        for w in self.works:
            w.wait()
        self.works = []
        if self.comm is not None:
            if self.comm.is_cuda and self.comm.dtype == torch.bfloat16:
                from .. import _native as N
                N.check(N.kernels().mbk_from_bf16(self.comm.data_ptr(), self.flat.numel,
                                                  self.flat.grad.data_ptr(), N.stream_ptr()),
                        "from_bf16")
            else:
                self.flat.grad.copy_(self.comm)


def all_reduce_mean(t: torch.Tensor, info: DistInfo) -> torch.Tensor:
    if info.enabled:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(info.world_size)
    return t


def gather_objects(obj, info: DistInfo) -> list:
    """Rank 0 receives every rank's ``obj`` (others get []), over the gloo host group: a
    CPU-only exchange that never waits on a GPU stream (RCCL's object collectives would
    stage through device memory and synchronise)."""
    if not info.enabled:
        return [obj]
    out = [None] * info.world_size if info.is_main else None
    dist.gather_object(obj, out, dst=0, group=info.host_group)
    return out if info.is_main else []


def all_ok(ok: bool, info: DistInfo) -> bool:
    """True iff every rank passes ``ok`` (a MIN all-reduce of one int over the gloo host
    group: CPU only, never waits on a GPU stream). Called once per update before the
    gradient collectives, so a rank that cannot continue (engine restarts exhausted) makes
    every rank stop at the same point instead of leaving its peers blocked in an RCCL
    all-reduce until the process-group timeout."""
    if not info.enabled:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=info.host_group)
    return bool(t.item())


# per-update rank states for agree(): the MIN over ranks decides what every rank does
FAILED, RESTARTING, OK = 0, 1, 2


def agree(state: int, info: DistInfo) -> int:
    """MIN of every rank's update state (FAILED < RESTARTING < OK) over the gloo host group.
    A rank whose engine failed but may restart reports RESTARTING: every rank then skips the
    update together (healthy ranks keep the batch they fetched) and meets again in the next
    round, so no rank sits in a gradient collective while a peer rebuilds its actors."""
    if not info.enabled:
        return int(state)
    t = torch.tensor([int(state)], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=info.host_group)
    return int(t.item())


def barrier(info: DistInfo) -> None:
    if info.enabled:
        dist.barrier()


def destroy(info: DistInfo) -> None:
    if info.enabled and dist.is_initialized():
        dist.destroy_process_group()
