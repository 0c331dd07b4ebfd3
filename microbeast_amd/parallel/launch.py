"""One process per GPU: self-launch and CPU/NUMA placement of each rank.

The reference never leaves one CPU node (10 actor processes + 1 learner,
microbeast.py:169-191; SURVEY §2.2 P5 has no DP). Here every MI355X gets one
learner process that owns its env workers, policy graphs and rollout slots, and
the learners all-reduce gradients over RCCL/xGMI (parallel/dist.py). Two
pieces make that launchable by hand and fast on an 8-GPU node:

* ``relaunch`` — ``python bench.py --gpus 8`` (or ``microbeast.py
  --nproc_per_node 8``) with no ``WORLD_SIZE`` in the environment starts
  ``torch.distributed.run`` with N ranks as a CHILD process and returns its
  exit code. It runs before anything touches the GPU (counting devices does
  not initialise HIP on this image) and never ``exec``s.
* ``pin_rank`` — restricts a rank (every thread it already runs -- HIP runtime,
  RCCL / gloo, torch's pools -- and every thread it starts afterwards: the
  native env workers, the engine's driver thread, the pinned-staging first
  touch) to whole physical cores on the NUMA node its GPU hangs off. Ranks that
  share a node split its cores into disjoint sets, so env workers of two GPUs
  never contend for a core or cross the socket interconnect for their pinned
  staging buffers.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def relaunch(nproc: int, argv: list[str], script: str | None = None, module: str | None = None,
             shared_gpu: bool = False) -> int | None:
    """Launch ``nproc`` ranks of ``script`` (or ``-m module``) with ``argv`` when this
    process is not already a rank. Returns the launcher's exit code, or None when the
    caller should run in-process (nproc <= 1 or already under torchrun).

    shared_gpu: allow more ranks than devices (rehearsal on a 1-GPU box; the ranks
    then share cuda:0 and must use the gloo backend, MBK_DIST_BACKEND=gloo)."""
    if nproc <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import torch

    ndev = torch.cuda.device_count()
    if ndev < nproc and not shared_gpu:
        print(f"--gpus/--nproc_per_node {nproc} needs {nproc} visible GPUs, found {ndev}",
              file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}"]
    cmd += ["-m", module] if module else [script]
    cmd += list(argv)
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL on this driver)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------ CPU placement
def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def parse_cpulist(s: str) -> list[int]:
    out: list[int] = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_pci_path(device_index: int) -> str | None:
    import torch

    try:
        p = torch.cuda.get_device_properties(device_index)
        return (f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:"
                f"{p.pci_device_id:02x}.0")
    except Exception:  # noqa: BLE001 - no device / old torch: no placement
        return None


def gpu_numa_node(device_index: int) -> int:
    path = gpu_pci_path(device_index)
    v = _read(path + "/numa_node") if path else None
    try:
        return int(v) if v is not None else -1
    except ValueError:
        return -1


def gpu_local_cpus(device_index: int) -> list[int]:
    path = gpu_pci_path(device_index)
    v = _read(path + "/local_cpulist") if path else None
    return parse_cpulist(v) if v else []


def physical_cores(cpus: list[int]) -> list[list[int]]:
    """Group logical CPUs into physical cores (SMT siblings together), in core order."""
    seen, cores = set(), []
    allowed = set(cpus)
    for c in sorted(cpus):
        if c in seen:
            continue
        sib = _read(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list")
        group = [x for x in (parse_cpulist(sib) if sib else [c]) if x in allowed] or [c]
        seen.update(group)
        cores.append(sorted(group))
    return cores


def split_cores(cores: list[list[int]], n: int, i: int) -> list[int]:
    """Core-granular contiguous split of ``cores`` into ``n`` parts; part ``i``'s CPUs."""
    n = max(1, n)
    lo = len(cores) * i // n
    hi = len(cores) * (i + 1) // n
    part = cores[lo:hi] or cores[min(lo, len(cores) - 1):min(lo, len(cores) - 1) + 1]
    return [c for core in part for c in core]


def plan_affinity(local_rank: int, local_world: int, allowed: list[int],
                  node_of_rank: list[int], cpus_of_node: dict[int, list[int]],
                  min_cpus: int = 1) -> list[int]:
    """Pure placement rule (unit-tested): rank r gets a disjoint share of the physical cores
    of its GPU's NUMA node (∩ ``allowed``), split among the local ranks on that node. Falls
    back to splitting ``allowed`` among all local ranks when topology is unknown or the
    node share would hold fewer than ``min_cpus`` CPUs (the rank's CPU-quota share):
    locality is not worth idling granted CPU time."""
    fallback = split_cores(physical_cores(allowed), local_world, local_rank)
    node = node_of_rank[local_rank]
    allowed_set = set(allowed)
    local = [c for c in cpus_of_node.get(node, []) if c in allowed_set]
    if node < 0 or not local:
        return fallback
    peers = [r for r in range(local_world) if node_of_rank[r] == node]
    mine = split_cores(physical_cores(local), len(peers), peers.index(local_rank))
    return mine if len(mine) >= min(min_cpus, len(fallback)) else fallback


def set_process_affinity(cpus: list[int]) -> None:
    """sched_setaffinity on EVERY thread of this process (``os.sched_setaffinity(0)`` only
    moves the calling thread and the threads it creates later; the HIP runtime, RCCL / gloo
    and torch's intra-op pool may already be running)."""
    os.sched_setaffinity(0, cpus)
    try:
        tids = os.listdir("/proc/self/task")
    except OSError:
        return
    for t in tids:
        try:
            os.sched_setaffinity(int(t), cpus)
        except (OSError, ValueError):
            pass  # a thread that exited meanwhile


def pin_rank(local_rank: int, local_world: int, device_index: int | None = None) -> list[int]:
    """Pin every thread of this process (and threads it starts later) to this rank's CPU
    share. Returns the CPU list (unchanged affinity if pinning is disabled or impossible)."""
    allowed = sorted(os.sched_getaffinity(0))
    if os.environ.get("MBK_NUMA_PIN", "1") == "0":
        return allowed
    import torch

    ndev = max(1, torch.cuda.device_count())
    devs = [(device_index if r == local_rank and device_index is not None else r) % ndev
            for r in range(local_world)]
    node_of_rank = [gpu_numa_node(d) for d in devs]
    cpus_of_node = {}
    for r, node in enumerate(node_of_rank):
        if node >= 0 and node not in cpus_of_node:
            cpus_of_node[node] = gpu_local_cpus(devs[r])
    q = cpu_quota()
    share = int(q / max(1, local_world)) if q is not None else 1
    mine = plan_affinity(local_rank, local_world, allowed, node_of_rank, cpus_of_node,
                         min_cpus=share)
    if mine:
        try:
            set_process_affinity(mine)
        except OSError:
            return allowed
    return mine or allowed


def cpu_quota() -> float | None:
    """CPUs granted by the cgroup quota (cpu.max), or None if unlimited."""
    v = _read("/sys/fs/cgroup/cpu.max")
    try:
        q, p = v.split()
        return None if q == "max" else int(q) / int(p)
    except (AttributeError, ValueError):
        return None


def rank_cpu_budget(local_world: int) -> int:
    """CPUs this rank may keep busy: its affinity set, capped by its share of the quota."""
    n = len(os.sched_getaffinity(0))
    q = cpu_quota()
    if q is not None:
        n = min(n, max(1, int(q / max(1, local_world))))
    return max(1, n)
