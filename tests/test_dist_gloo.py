"""Data-parallel learners over torch.distributed (gloo, world_size 2, CPU): bucketed,
hook-launched all-reduce gives exactly the single-process update on the concatenated batch."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, comm="fp32"):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from helpers import synthetic_batch
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.parallel.dist import destroy, init_distributed
    info = init_distributed(use_cuda=False)
    torch.manual_seed(1234 + rank)  # different init per rank: broadcast must fix it
    m = Agent((4, 4, 27))
    L = Learner(m, LearnerHParams(bucket_mb=0.5, allreduce_dtype=comm), torch.device("cpu"), info)
    assert len(L.reducer.buckets) >= 2  # several buckets, launched from hooks
    torch.manual_seed(0)
    ref = Agent((4, 4, 27))
    torch.save(L.flat.data.clone(), os.path.join(outdir, f"init{rank}.pt"))
    b = synthetic_batch(m, 6, 3, 16, seed=100 + rank)
    torch.save(b, os.path.join(outdir, f"batch{rank}.pt"))
    L.learn(b)
    torch.save(L.flat.data.clone(), os.path.join(outdir, f"after{rank}.pt"))
    destroy(info)
    del ref


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_dp_allreduce_equals_single_process(tmp_path, comm):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), comm), nprocs=world,
                       join=True, start_method="spawn")
    init0 = torch.load(tmp_path / "init0.pt")
    init1 = torch.load(tmp_path / "init1.pt")
    assert torch.equal(init0, init1)  # broadcast from rank 0
    a0 = torch.load(tmp_path / "after0.pt")
    a1 = torch.load(tmp_path / "after1.pt")
    assert torch.equal(a0, a1)
    # single process on the concatenated batch from the same init
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    m = Agent((4, 4, 27))
    L = Learner(m, LearnerHParams(), torch.device("cpu"))
    L.flat.data.copy_(init0)
    b0 = torch.load(tmp_path / "batch0.pt")
    b1 = torch.load(tmp_path / "batch1.pt")
    b = {k: torch.cat([b0[k], b1[k]], dim=1) for k in b0}
    L.learn(b)
    if comm == "fp32":
        torch.testing.assert_close(L.flat.data, a0, rtol=1e-5, atol=1e-6)
    else:
        # bf16 payload: gradients rounded to bf16 before the sum (fp32 master grads). Adam's
        # first step is ~lr * sign(g): only near-zero gradients (sign / zero flips) may move
        # by up to ~lr; everything else matches
        d = (L.flat.data - a0).abs()
        assert float(d.max()) <= 2 * 2.5e-4
        assert float((d > 1e-6).float().mean()) < 0.02
        assert float(d.mean()) < 1e-6


def _worker_ok_league(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from microbeast_amd.parallel import dist as D
    from microbeast_amd.parallel.dist import all_ok, barrier, destroy, init_distributed
    from microbeast_amd.runtime.league import League
    from microbeast_amd.utils.checkpoint import load_league_shard, save_league_shard
    info = init_distributed(use_cuda=False)
    res = [all_ok(True, info), all_ok(rank != 1, info), all_ok(True, info)]
    # tri-state per-update agreement: a restarting rank makes every rank skip the round
    res += [D.agree(D.OK, info), D.agree(D.RESTARTING if rank == 1 else D.OK, info),
            D.agree(D.FAILED if rank == 0 else D.RESTARTING, info)]
    # every rank checkpoints its own league (snapshots + PFSP results) next to the main file
    lg = League(capacity=4, snapshot_every=1, seed=rank)
    for k in range(3):
        lg.add_snapshot(torch.full((8,), float(10 * rank + k)))
    lg.record([(1.0, 10, 0, 0, 1), (0.0, 10, 0, 1, 1 + rank)])
    ck = os.path.join(outdir, "run.ckpt")
    save_league_shard(ck, info.rank, lg.state_dict())
    barrier(info)
    back = League()
    back.load_state_dict(load_league_shard(ck, info.rank))
    torch.save({"ok": res, "games": back.games, "snap2": back.snapshot(2)},
               os.path.join(outdir, f"ok{rank}.pt"))
    destroy(info)


def test_fail_fast_flag_and_per_rank_league_shards(tmp_path):
    """all_ok: one rank that cannot continue stops every rank at the same update (gloo host
    group); each rank's league is checkpointed and restored from its own shard."""
    world = 2
    mp.start_processes(_worker_ok_league, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        d = torch.load(tmp_path / f"ok{r}.pt")
        assert d["ok"] == [True, False, True, 2, 1, 0]
        assert torch.equal(d["snap2"], torch.full((8,), float(10 * r + 2)))
        assert d["games"][1] == (2.0 if r == 0 else 1.0)
