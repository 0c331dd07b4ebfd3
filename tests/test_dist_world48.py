"""Data parallelism at the world sizes an 8-GPU node runs (4 and 8 ranks), on gloo / CPU.

The driver's N = 2/4/8 scaling bench is the first place these sizes meet RCCL; everything the
DP path does besides the collective kernel itself is pinned here first:

* bucket cuts + grad scale: after two updates every rank holds the parameters (and Adam state)
  that ONE process computes on the concatenation of all ranks' batches -- the hook-fired
  bucketed all-reduce sums in fp32 and the 1/world factor is folded into Adam
  (parallel/dist.py, learner.py);
* fail-fast: one rank reporting FAILED / RESTARTING / not-ok makes every rank see it in the
  same round (agree / all_ok over the gloo host group);
* the batched episode gather: every rank's finished episodes reach rank 0's CSV, nobody else
  writes one (train._gather_episodes + CsvLogger);
* the rank-0 checkpoint behind a barrier restores the same model on every rank.

Reference: the reference has no DP (/root/reference/microbeast.py:119,254-260 leaves its two
Hogwild learner threads commented out); SURVEY section 2.2 P5 and section 4 ("gloo ... world_size
2-4"). Each case spawns its ranks once (a few seconds per rank to import torch).
"""
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


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    torch.set_num_threads(1)


def _worker_update(rank, world, port, outdir):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    _env(rank, world, port)
    from helpers import synthetic_batch
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.parallel.dist import destroy, init_distributed
    info = init_distributed(use_cuda=False)
    assert info.world_size == world and info.rank == rank
    torch.manual_seed(99 + rank)  # a different init per rank: the broadcast must fix it
    m = Agent((4, 4, 27))
    L = Learner(m, LearnerHParams(bucket_mb=0.25), torch.device("cpu"), info)
    # several hook-fired buckets, cut over the flat parameter buffer
    assert len(L.reducer.buckets) >= 3
    torch.save(L.flat.data.clone(), os.path.join(outdir, f"init{rank}.pt"))
    for k in range(2):  # two updates: the second one runs on Adam state built from the first
        b = synthetic_batch(m, 4, 2, 16, seed=1000 * k + rank)
        torch.save(b, os.path.join(outdir, f"batch{rank}_{k}.pt"))
        L.learn(b)
    torch.save(L.flat.data.clone(), os.path.join(outdir, f"after{rank}.pt"))
    destroy(info)


@pytest.mark.parametrize("world", [4, 8])
def test_dp_update_equals_single_process_on_concatenated_batch(tmp_path, world):
    mp.start_processes(_worker_update, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    inits = [torch.load(tmp_path / f"init{r}.pt") for r in range(world)]
    afters = [torch.load(tmp_path / f"after{r}.pt") for r in range(world)]
    for r in range(1, world):
        assert torch.equal(inits[r], inits[0]), f"rank {r}: broadcast from rank 0 missing"
        assert torch.equal(afters[r], afters[0]), f"rank {r} diverged from rank 0"
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    L = Learner(Agent((4, 4, 27)), LearnerHParams(), torch.device("cpu"))
    L.flat.data.copy_(inits[0])
    for k in range(2):
        bs = [torch.load(tmp_path / f"batch{r}_{k}.pt") for r in range(world)]
        L.learn({key: torch.cat([b[key] for b in bs], dim=1) for key in bs[0]})
    torch.testing.assert_close(L.flat.data, afters[0], rtol=1e-5, atol=1e-6)


def _worker_control(rank, world, port, outdir):
    _env(rank, world, port)
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.parallel import dist as D
    from microbeast_amd.train import _gather_episodes
    from microbeast_amd.utils.checkpoint import load_checkpoint, restore, save_checkpoint
    from microbeast_amd.utils.metrics import CsvLogger
    info = D.init_distributed(use_cuda=False)
    last = world - 1
    # fail-fast: the one rank that cannot continue is seen by all in the same round
    res = [D.all_ok(True, info), D.all_ok(rank != last, info), D.all_ok(True, info),
           D.agree(D.OK, info), D.agree(D.RESTARTING if rank == last else D.OK, info),
           D.agree(D.FAILED if rank == last else D.OK, info),
           D.agree(D.RESTARTING if rank == 1 else (D.FAILED if rank == last else D.OK), info)]
    # batched episode gather: (return, length, env index, winner, opponent) rows, rank r
    # finished r + 1 episodes; only rank 0 opens the CSV
    logger = CsvLogger(outdir, "dp", enabled=info.is_main)
    eps = [(float(10 * rank + k), 100 + k, 1000 * rank + k, k % 2, -1) for k in range(rank + 1)]
    logger.episodes(_gather_episodes(eps, info))
    logger.episodes(_gather_episodes([], info))  # a round in which nobody finished one
    logger.close()
    # rank-0 checkpoint, barrier, every rank restores it
    torch.manual_seed(7 + rank)
    L = Learner(Agent((4, 4, 27)), LearnerHParams(), torch.device("cpu"), info)
    with torch.no_grad():
        for q in L.model.parameters():  # ranks disagree until the restore
            q.add_(float(rank))
    ck = os.path.join(outdir, "dp.ckpt")
    if info.is_main:
        save_checkpoint(ck, L.model, L.opt, step=123, n_update=4)
    D.barrier(info)
    step, n_update = restore(load_checkpoint(ck), L.model, L.opt)
    params = torch.cat([q.detach().flatten() for q in L.model.parameters()])
    torch.save({"res": res, "flat": params, "step": step, "n_update": n_update},
               os.path.join(outdir, f"ctl{rank}.pt"))
    D.destroy(info)


@pytest.mark.parametrize("world", [4, 8])
def test_dp_fail_fast_episode_gather_and_rank0_checkpoint(tmp_path, world):
    mp.start_processes(_worker_control, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    from microbeast_amd.parallel import dist as D
    from microbeast_amd.utils.metrics import read_episodes
    outs = [torch.load(tmp_path / f"ctl{r}.pt") for r in range(world)]
    for r, o in enumerate(outs):
        assert o["res"] == [True, False, True, D.OK, D.RESTARTING, D.FAILED, D.FAILED], r
        assert (o["step"], o["n_update"]) == (123, 4)
        assert torch.equal(o["flat"], outs[0]["flat"]), f"rank {r} restored other weights"
    _, rows = read_episodes(str(tmp_path / "dp.csv"))
    got = sorted((int(r[2]), r[0]) for r in rows)
    want = sorted((1000 * r + k, float(10 * r + k)) for r in range(world) for k in range(r + 1))
    assert got == want  # every rank's episodes, exactly once, in rank 0's file
