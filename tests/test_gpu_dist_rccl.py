"""The RCCL data-parallel path, executed for real on one MI355X (world size 1, forced
process group, backend "nccl" = librccl): broadcast, bucketed all-reduce fired from the
post-accumulate-grad hooks during backward (fp32 and bf16 payloads), the 1/world average
folded into Adam, barrier and the gloo host-group episode gather, inside real
``Learner.learn`` calls on a rollout batch produced by the GPU engine. The updates must be
BIT-identical to the non-distributed learner (bf16: to the non-distributed learner with the
gradient rounded to bf16). Also the policy-lag tagging of rollout slots.
(SURVEY §2.2 P5, §4 "the RCCL path is validated on 1 GPU".)"""
import pytest
import torch

pytestmark = pytest.mark.gpu

S = 8


def _mk():
    from microbeast_amd.models.agent import Agent
    return Agent((S, S, 27))


@pytest.fixture(scope="module")
def batch(cuda):
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime
    torch.manual_seed(0)
    learner = Learner(_mk(), LearnerHParams(), cuda)
    rt = GpuActorRuntime(_mk, S, n_groups=2, envs_per_group=32, unroll=8, batch_slots=1,
                         device=cuda, n_threads=2)
    rt.start(learner.flat)
    try:
        out = []
        lags = []
        for it in range(4):
            b, slots = rt.get_batch(timeout=120)
            lags.append(rt.policy_lag(slots, learner.n_updates))
            out.append({k: v.clone() for k, v in b.items()})
            learner.learn(b)
            rt.release(slots)
            rt.publish(learner.flat, version=learner.n_updates)
        torch.cuda.synchronize()
    finally:
        rt.stop()
    assert lags[0] == 0 and all(0 <= x <= 4 for x in lags)
    return out


def _run(dev, batches, info=None, hp=None, round_bf16=False):
    from microbeast_amd.learner import Learner, LearnerHParams
    torch.manual_seed(123)
    L = Learner(_mk(), hp or LearnerHParams(), dev, info)
    if round_bf16:  # emulate a bf16 payload on the non-distributed learner
        L.reducer.finish = lambda: L.flat.grad.copy_(L.flat.grad.bfloat16().float())
    for b in batches[:2]:
        L.learn(b)
    torch.cuda.synchronize()
    return L


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_rccl_world1_bit_identical(cuda, batch, comm):
    from microbeast_amd.learner import LearnerHParams
    from microbeast_amd.parallel import dist as D
    from microbeast_amd.train import _gather_episodes

    ref = _run(cuda, batch, round_bf16=comm == "bf16")
    info = D.init_distributed(use_cuda=True, force_pg=True)
    try:
        assert info.enabled and info.backend == "nccl" and info.world_size == 1
        assert torch.distributed.get_backend() == "nccl"
        hp = LearnerHParams(bucket_mb=0.25, allreduce_dtype=comm)
        from microbeast_amd.learner import Learner
        torch.manual_seed(123)
        L = Learner(_mk(), hp, cuda, info)  # broadcast_flat over RCCL
        red = L.reducer
        assert len(red.buckets) >= 3 and red.buckets[0][1] == L.flat.numel
        fired_before_finish = []
        orig = red.finish

        def finish():
            fired_before_finish.append(list(red.fired))
            orig()
        red.finish = finish
        for b in batch[:2]:
            L.learn(b)
        D.barrier(info)
        torch.cuda.synchronize()
        # every bucket was launched by a grad hook while backward ran, none by finish()
        assert all(all(f) for f in fired_before_finish)
        assert torch.equal(L.flat.data, ref.flat.data)
        assert torch.equal(L.opt.m, ref.opt.m) and torch.equal(L.opt.v, ref.opt.v)
        recs = [(1.0, 10, 3, 1, -1), (0.5, 20, 4, 0, -1)]
        assert _gather_episodes(recs, info) == recs  # gloo host group
    finally:
        D.destroy(info)


def test_comm_rehearsal_fires_from_hooks_and_leaves_update_identical(cuda, batch):
    """bench.py --comm_rehearsal (world 1, no process group): every bucket's stand-in
    collective launches from a grad hook on the 4th (high-priority) stream while backward
    runs, the learner's stream waits for it, and the update stays bit-identical (the stand-in
    never writes the gradient)."""
    from microbeast_amd.learner import Learner, LearnerHParams
    ref = _run(cuda, batch)
    torch.manual_seed(123)
    L = Learner(_mk(), LearnerHParams(bucket_mb=0.25, comm_rehearsal=True), cuda)
    red = L.reducer
    assert red.rehearse and red.side is not None and len(red.buckets) >= 3
    assert red.side.priority < torch.cuda.current_stream().priority
    fired_before_finish = []
    orig = red.finish

    def finish():
        fired_before_finish.append(list(red.fired))
        orig()
    red.finish = finish
    for b in batch[:2]:
        L.learn(b)
    torch.cuda.synchronize()
    assert all(all(f) for f in fired_before_finish)
    assert float(red.scratch.abs().sum()) > 0  # the stand-in ran over the gradient
    assert torch.equal(L.flat.data, ref.flat.data)
    assert torch.equal(L.opt.m, ref.opt.m) and torch.equal(L.opt.v, ref.opt.v)
