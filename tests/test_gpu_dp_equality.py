"""Data parallelism is RIGHT on the HIP learner path, not only runnable:
two DP ranks (gloo, both on cuda:0 -- RCCL refuses two ranks on one device) each take one
real engine rollout batch; after one update both ranks' parameters must equal a single-rank
HIP update on the two batches concatenated along the env axis, within the bf16 floor.

This covers what the CPU gloo test (test_dist_gloo.py) cannot: the HIP backward's direct
gradient slots (ops/optim.py grad_out) interacting with the bucketed all-reduce hooks, the
1/world average folded into adam.hip, and the per-rank V-trace / loss means on the GPU."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

S = 16  # the headline map: the fused tail node + sparse head + 16-channel residual kernels


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mk():
    from microbeast_amd.models.agent import Agent
    return Agent((S, S, 27))


def _rank(rank, world, port, d, comm):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), MBK_DIST_BACKEND="gloo")
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.parallel.dist import destroy, init_distributed
    info = init_distributed(use_cuda=True)
    dev = torch.device("cuda", 0)
    torch.manual_seed(1000 + rank)  # different init per rank: the broadcast must fix it
    L = Learner(_mk(), LearnerHParams(bucket_mb=2.0, allreduce_dtype=comm), dev, info)
    assert len(L.reducer.buckets) >= 2
    L.flat.data.copy_(torch.load(os.path.join(d, "init.pt")).to(dev))  # same start as the ref
    b = {k: v.to(dev) for k, v in torch.load(os.path.join(d, f"batch{rank}.pt")).items()}
    L.learn(b)
    torch.cuda.synchronize()
    torch.save(L.flat.data.cpu(), os.path.join(d, f"after{rank}.pt"))
    destroy(info)


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_two_rank_hip_update_equals_concatenated_batch(cuda, tmp_path, comm):
    from helpers import engine_batches

    from microbeast_amd.learner import Learner, LearnerHParams
    bs = engine_batches(cuda, S, 2, groups=2, envs=64, T=16, seed=3, learn=False)
    torch.manual_seed(7)
    ref = Learner(_mk(), LearnerHParams(), cuda)
    init = ref.flat.data.clone()
    torch.save(init.cpu(), tmp_path / "init.pt")
    for r in range(2):
        torch.save({k: v.cpu() for k, v in bs[r].items()}, tmp_path / f"batch{r}.pt")
    mp.start_processes(_rank, args=(2, _free_port(), str(tmp_path), comm), nprocs=2, join=True,
                       start_method="spawn")
    a0 = torch.load(tmp_path / "after0.pt")
    a1 = torch.load(tmp_path / "after1.pt")
    assert torch.equal(a0, a1)  # every rank applied the same averaged update
    cat = {k: torch.cat([bs[0][k], bs[1][k]], dim=1) for k in bs[0]}  # [T+1, 2E, ...]
    if comm == "bf16":  # the payload is rounded to bf16 before the sum
        ref.reducer.finish = lambda: ref.flat.grad.copy_(ref.flat.grad.bfloat16().float())
    ref.learn(cat)
    torch.cuda.synchronize()
    want = ref.flat.data.cpu()
    moved = (want - init.cpu()).abs()
    assert float(moved.max()) > 1e-5  # the update did something
    d = (want - a0).abs()
    # Adam's first step is ~lr * sign(g): gradients summed in a different order (per-rank
    # partial sums vs one pass over 2E envs) may only move near-zero entries, by <= ~2 lr
    lr = LearnerHParams().lr
    print(f"{comm}: max {float(d.max()):.3g} mean {float(d.mean()):.3g} "
          f"frac>1e-6 {float((d > 1e-6).float().mean()):.4f}")
    assert float(d.max()) <= 2.5 * lr
    assert float((d > 1e-6).float().mean()) < 0.02
    assert float(d.mean()) < 2e-6
