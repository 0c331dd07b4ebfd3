"""Fused two-launch acting step (ops/act.py, mbk_act_step) == the captured 6-launch graph step.

Same codes, same weights, same Philox state: obs planes, masks, sampled actions, behaviour
log-probs, values and the packed env actions must match bit for bit, and the sampler's step
counter must advance identically (reference act path: model.py:165-216)."""
import pytest
import torch

from microbeast_amd import _native as N

pytestmark = pytest.mark.gpu


def _codes_stream(E, steps, seed):
    """Codes of E real 16x16 simulator envs over `steps` steps of random legal play."""
    from microbeast_amd.ops.cell_head import OFFS, unpack_mask
    rt = N.runtime()
    S = 256
    env = rt.VecEnv(16, E, 300, seed, [0, 1, 2, 3, 5])
    obs = torch.zeros(E, S, dtype=torch.int32)
    mask = torch.zeros(E, S, 3, dtype=torch.int32)
    env.reset(obs.data_ptr(), mask.data_ptr())
    codes = torch.zeros(E, S, dtype=torch.int16)
    res = torch.zeros(E, dtype=torch.int32)
    rew, done = torch.zeros(E), torch.zeros(E, dtype=torch.uint8)
    gen = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(steps):
        env.obs_codes(codes.data_ptr(), res.data_ptr())
        out.append((codes.clone(), res.clone()))
        mb = unpack_mask(mask)
        a = torch.zeros(E, S, 7, dtype=torch.uint8)
        for k in range(7):
            seg = mb[..., OFFS[k]:OFFS[k + 1]].float() + 1e-6
            a[..., k] = torch.multinomial(seg.view(-1, seg.shape[-1]), 1,
                                          generator=gen).view(E, S)
        env.step(a.data_ptr(), obs.data_ptr(), mask.data_ptr(), rew.data_ptr(), done.data_ptr())
    return out


def _pad_rows(cl, codes, k):
    """cl with k extra (empty cell, code 0) entries appended to every other env's row."""
    cl = cl.clone()
    E, S = codes.shape
    for e in range(0, E, 2):
        n = int(cl[e, 0]) & 0xFFFF
        empty = torch.nonzero(codes[e] == 0).view(-1)[:k]
        cl[e, 1 + n:1 + n + len(empty)] = empty.to(torch.int32)
        cl[e, 0] = (int(cl[e, 0]) & ~0xFFFF) | (n + len(empty))
    return cl


def _model(cuda, seed):
    from microbeast_amd.models.agent import Agent
    torch.manual_seed(seed)
    m = Agent((16, 16, 27))
    torch.nn.init.normal_(m.actor.weight, std=0.05)  # a non-uniform policy
    torch.nn.init.normal_(m.actor.bias, std=0.5)
    m = m.to(cuda).eval()
    m.pack_inference(cuda)
    return m


@pytest.mark.parametrize("E,sparse", [(96, False), (520, False), (200, True), (200, "pad")])
def test_fused_act_step_bit_identical(cuda, E, sparse):
    """The fused step (launch A: decode + trunk + critic, launch B: sparse head) is
    bit-identical to the captured-graph step. sparse: the PCIe-light form the engine uses
    (occupied-cell code rows in, non-noop action rows out) must give the same step as the
    dense codes / dense packed actions; "pad": every other env's row longer than launch A's
    first 32-word access (the rest of the row is read in a second pass)."""
    from microbeast_amd.ops.act import ActWorkspace, code_lists, dense_actions
    from microbeast_amd.runtime.gpu_actors import graph_policy_step, make_io

    S = 256
    m = _model(cuda, 3)
    rng_a = torch.tensor([12345, 7], dtype=torch.int64, device=cuda)
    rng_b = rng_a.clone()
    io = make_io(E, S, cuda)
    ws = ActWorkspace(m, E, rng_b, cuda)
    obs = torch.empty(E, S, dtype=torch.int32, device=cuda)
    mask = torch.empty(E, S, 3, dtype=torch.int32, device=cuda)
    obs2, mask2 = torch.empty_like(obs), torch.empty_like(mask)
    action = torch.full((E, S, 7), 0xAB, dtype=torch.uint8, device=cuda)
    logp = torch.full((E,), float("nan"), device=cuda)
    value = torch.full((E,), float("nan"), device=cuda)
    act16 = torch.full((E, S), -1, dtype=torch.int16, device=cuda)
    stride = S + 4
    act_list = torch.full((E, stride), -1, dtype=torch.int32, device=cuda)
    reward = torch.randn(E, device=cuda)
    done = (torch.rand(E, device=cuda) < 0.3).to(torch.uint8)
    rdst, ddst = torch.zeros_like(reward), torch.zeros_like(done)
    n_active = 0
    abits = torch.full((E, S // 32), -1, dtype=torch.int32, device=cuda)
    abits2 = torch.full_like(abits, -1)
    for i, (codes, res) in enumerate(_codes_stream(E, 24, seed=E)):
        io["in_codes"].copy_(codes)
        io["in_res"].copy_(res)
        graph_policy_step(io, m, rng_a, E, 16, cuda)
        second = i % 3 == 0
        if sparse:
            # odd steps: rows in pinned host memory, read by launch A over PCIe (the engine's
            # form); even steps: rows already in HBM
            cl = code_lists(codes, res, stride)
            if sparse == "pad":  # rows longer than launch A's first access (32 words)
                cl = _pad_rows(cl, codes, 40)
                assert int((cl[:, 0] & 0xFFFF).max()) >= 32
            cl = cl.pin_memory() if i % 2 == 1 else cl.to(cuda)
            ws.step(None, None, obs, mask, action, logp, value, None,
                    obs2=obs2 if second else None, mask2=mask2 if second else None,
                    reward=reward, done=done, reward_dst=rdst, done_dst=ddst, code_list=cl,
                    act_list=act_list, abits=abits, abits2=abits2 if second else None)
            torch.cuda.synchronize()
            act16 = dense_actions(act_list, S).to(cuda)
            al = act_list.cpu().to(torch.int64) & 0xFFFFFFFF
            listed = torch.arange(stride - 1)[None, :] < al[:, :1]
            assert int(al[:, 0].max()) <= S and bool(((al[:, 1:] >> 16) != 0)[listed].all())
        else:
            ws.step(io["in_codes"], io["in_res"], obs, mask, action, logp, value, act16,
                    obs2=obs2 if second else None, mask2=mask2 if second else None,
                    reward=reward, done=done, reward_dst=rdst, done_dst=ddst,
                    abits=abits, abits2=abits2 if second else None)
        torch.cuda.synchronize()
        assert torch.equal(obs, io["in_obs"]), f"obs planes differ at step {i}"
        assert torch.equal(mask, io["in_mask"]), f"masks differ at step {i}"
        if second:
            assert torch.equal(obs2, obs) and torch.equal(mask2, mask)
            assert torch.equal(abits2, abits)
        # the active-cell bitmap row = the masks' non-zero cells, bit c & 31 of word c >> 5
        live = (mask != 0).any(-1).view(E, S // 32, 32).to(torch.int64)
        ref = (live << torch.arange(32, device=cuda)).sum(-1)
        assert torch.equal(abits.to(torch.int64) & 0xFFFFFFFF, ref), f"abits differ at step {i}"
        assert torch.equal(action, io["out_action"]), f"actions differ at step {i}"
        assert torch.equal(act16, io["out_act16"]), f"packed actions differ at step {i}"
        assert torch.equal(logp.view(torch.int32), io["out_logp"].view(torch.int32)), \
            f"log-probs differ at step {i}: {(logp - io['out_logp']).abs().max().item()}"
        assert torch.equal(value.view(torch.int32), io["out_value"].view(torch.int32)), \
            f"values differ at step {i}"
        assert torch.equal(rng_a, rng_b), f"sampler state differs after step {i}"
        assert torch.equal(rdst, reward) and torch.equal(ddst, done)
        # between steps the previous step's bucket counters are back at zero (double buffer)
        par = (7 + i) % 2  # this step's Philox step is 7 + i
        assert int(ws.bucket_cnt[par * 256:(par + 1) * 256].abs().sum()) > 0
        if i > 0:
            assert int(ws.bucket_cnt[(1 - par) * 256:(2 - par) * 256].abs().sum()) == 0
        assert int(ws.pending[:E].abs().sum()) == 0
        n_active += int((mask != 0).any(-1).sum())
    assert n_active > 50 * 24  # the head actually sampled
    assert int(rng_b[1]) == 7 + 24


def _fast_codes_stream(E, steps, seed):
    """Codes of E simulator envs over `steps` steps of random packed actions (the engine's
    step_codes path with validation off: infeasible actions are dropped by the simulator)."""
    rt = N.runtime()
    S = 256
    env = rt.VecEnv(16, E, 300, seed, [0, 1, 2, 3, 5])
    env.set_validate(False)
    env.reset(0, 0)
    codes = torch.zeros(E, S, dtype=torch.int16)
    res = torch.zeros(E, dtype=torch.int32)
    rew, done = torch.zeros(E), torch.zeros(E, dtype=torch.uint8)
    g = torch.Generator().manual_seed(seed)
    out = []
    for t in range(steps):
        a16 = torch.randint(0, 1 << 14, (E, S), generator=g, dtype=torch.int32).to(torch.int16)
        env.step_codes(a16.data_ptr(), codes.data_ptr(), res.data_ptr(), rew.data_ptr(),
                       done.data_ptr())
        if t >= steps - 4:
            out.append((codes.clone(), res.clone()))
    return out


def test_fused_act_step_bit_identical_full_grid(cuda):
    """The headline's 8192-env group: launch A runs 2 tiles per workgroup (the next tile's rows
    prefetched during the current one, the tile lists / counters double-buffered by parity)
    and launch B deals ~hundreds of 64-pair jobs -- paths a small E never reaches. The fused
    step must still equal the captured-graph step bit for bit, with the rows read over PCIe
    from pinned memory and every other env's row longer than launch A's first access."""
    from microbeast_amd.ops.act import ActWorkspace, code_lists, dense_actions
    from microbeast_amd.runtime.gpu_actors import graph_policy_step, make_io

    E, S = 8192, 256
    m = _model(cuda, 5)
    rng_a = torch.tensor([777, 3], dtype=torch.int64, device=cuda)
    rng_b = rng_a.clone()
    io = make_io(E, S, cuda)
    ws = ActWorkspace(m, E, rng_b, cuda)
    obs = torch.empty(E, S, dtype=torch.int32, device=cuda)
    mask = torch.empty(E, S, 3, dtype=torch.int32, device=cuda)
    action = torch.full((E, S, 7), 0xAB, dtype=torch.uint8, device=cuda)
    logp = torch.full((E,), float("nan"), device=cuda)
    value = torch.full((E,), float("nan"), device=cuda)
    stride = S + 4
    act_list = torch.full((E, stride), -1, dtype=torch.int32).pin_memory()
    for i, (codes, res) in enumerate(_fast_codes_stream(E, 40, seed=11)):
        io["in_codes"].copy_(codes)
        io["in_res"].copy_(res)
        graph_policy_step(io, m, rng_a, E, 16, cuda)
        cl = _pad_rows(code_lists(codes, res, stride), codes, 40).pin_memory()
        ws.step(None, None, obs, mask, action, logp, value, None, code_list=cl,
                act_list=act_list)
        torch.cuda.synchronize()
        assert torch.equal(obs, io["in_obs"]), f"obs planes differ at step {i}"
        assert torch.equal(mask, io["in_mask"]), f"masks differ at step {i}"
        assert torch.equal(action, io["out_action"]), f"actions differ at step {i}"
        assert torch.equal(dense_actions(act_list, S).to(cuda), io["out_act16"]), \
            f"packed actions differ at step {i}"
        assert torch.equal(logp.view(torch.int32), io["out_logp"].view(torch.int32)), \
            f"log-probs differ at step {i}"
        assert torch.equal(value.view(torch.int32), io["out_value"].view(torch.int32)), \
            f"values differ at step {i}"
        assert torch.equal(rng_a, rng_b)
        assert int(ws.pending[:E].abs().sum()) == 0
    assert int((mask != 0).any(-1).sum()) > E  # the head sampled


def test_engine_fused_act_learns(cuda):
    """The engine's fused step form on a 16x16 map: rollout rows written in place are aligned
    (legal actions under the mask of the same row), learn / publish work, two lanes."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.cell_head import OFFS, unpack_mask
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    s, T, E = 16, 8, 64

    def mk():
        return Agent((s, s, 27))

    torch.manual_seed(0)
    learner = Learner(mk(), LearnerHParams(), cuda)
    rt = GpuActorRuntime(mk, s, n_groups=3, envs_per_group=E, unroll=T, batch_slots=1,
                         device=cuda, n_threads=2, n_lanes=2)
    assert rt.fused_act and rt.engine.act_mode()
    rt.start(learner.flat)
    try:
        for it in range(5):
            batch, slots = rt.get_batch()
            torch.cuda.synchronize()
            obs, mask, act = batch["obs"], batch["mask"], batch["action"]
            bits = obs.cpu().view(-1).numpy().view("uint32")
            assert set(int(bin(int(x)).count("1")) for x in bits[:5000]) == {5}
            mb = unpack_mask(mask[:T].cpu())
            a = act[:T].cpu().long()
            for k in range(7):
                seg = mb[..., OFFS[k]:OFFS[k + 1]]
                has = seg.any(-1)
                ok = seg.gather(-1, a[..., k:k + 1]).squeeze(-1) | ~has
                assert bool(ok.all()), f"illegal action component {k}"
            # inactive cells carry action 0; active ones at least one legal choice
            assert int(a[~mb.any(-1)].abs().sum()) == 0
            assert torch.isfinite(batch["logp"][:T]).all() and (batch["logp"][:T] <= 0).all()
            losses = learner.learn(batch)
            rt.release(slots)
            rt.publish(learner.flat, version=it + 1)
            assert torch.isfinite(losses).all()
        st = rt.stats()
        assert st["frames"] > 0 and st["gpu_steps"] > 0 and st["publishes"] >= 1
        assert st["act_steps"] > 0
        assert st["act_active_cells"] > 0
    finally:
        rt.stop()


@pytest.mark.parametrize("size", [8, 10, 24])
def test_graph_sparse_row_io(cuda, size):
    """The captured-graph step's sparse I/O (copy.hip): pinned occupied-cell rows -> dense
    device codes + resources, and dense packed actions -> pinned non-noop action rows, equal to
    the host-side helpers (ops/act.py code_lists / dense_actions) on real simulator codes."""
    from microbeast_amd.ops.act import code_lists, dense_actions
    k = N.kernels()
    S, E = size * size, 37
    stride = (S + 1 + 3) & ~3
    rt = N.runtime()
    env = rt.VecEnv(size, E, 300, 4, [0, 1, 2, 3])
    env.reset(0, 0)
    rows = torch.full((E, stride), -7, dtype=torch.int32).pin_memory()
    env.code_lists(rows.data_ptr(), stride, 0)
    codes = torch.empty(E, S, dtype=torch.int16, device=cuda)
    res = torch.empty(E, dtype=torch.int32, device=cuda)
    N.check(k.mbk_rows_to_codes(rows.data_ptr(), stride, E, S, codes.data_ptr(), res.data_ptr(),
                                N.stream_ptr()), "rows_to_codes")
    c_ref = torch.zeros(E, S, dtype=torch.int16)
    r_ref = torch.zeros(E, dtype=torch.int32)
    env.obs_codes(c_ref.data_ptr(), r_ref.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(codes.cpu(), c_ref) and torch.equal(res.cpu(), r_ref)
    g = torch.Generator().manual_seed(size)
    act16 = torch.randint(1, 30000, (E, S), generator=g, dtype=torch.int16)
    act16[torch.rand(E, S, generator=g) < 0.97] = 0
    act16[0] = 0  # an env with no action at all
    out = torch.full((E, stride), -1, dtype=torch.int32).pin_memory()
    N.check(k.mbk_codes_to_rows(act16.to(cuda).data_ptr(), E, S, out.data_ptr(), stride,
                                N.stream_ptr()), "codes_to_rows")
    torch.cuda.synchronize()
    assert int(out[0, 0]) == 0
    assert torch.equal(dense_actions(out, S), act16)
    ref = code_lists(act16, torch.zeros(E, dtype=torch.int32), stride)
    n = ref[:, 0]
    for e in range(E):  # entries ascending by cell, exactly the non-noop cells
        assert torch.equal(out[e, :1 + int(n[e])], ref[e, :1 + int(n[e])])


def test_engine_fused_act_logp_tracks_published_weights(cuda):
    """After publishes, a rollout acted with the fused step under version v carries behaviour
    log-probs equal to what the learner scores with the weights of version v (the step reads
    packed weights through pointers captured once; a publish that missed a buffer would leave
    the actors on stale weights)."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    s, T, E = 16, 8, 64

    def mk():
        return Agent((s, s, 27))

    torch.manual_seed(0)
    learner = Learner(mk(), LearnerHParams(), cuda)
    with torch.no_grad():  # a non-uniform policy (params are views of the flat buffer)
        learner.model.actor.weight.normal_(0, 0.05)
    rt = GpuActorRuntime(mk, s, n_groups=2, envs_per_group=E, unroll=T, batch_slots=1,
                         device=cuda, n_threads=2)
    assert rt.fused_act and rt.engine.act_mode()
    rt.start(learner.flat)
    version, batch = 0, None
    try:
        for _ in range(24):
            b, slots = rt.get_batch()
            vers = [rt.engine.slot_version(int(x)) for x in slots]
            if version >= 2:  # weights frozen at the last publish: wait for its rollouts
                if min(vers) == version:
                    torch.cuda.synchronize()
                    batch = {k: v.clone() for k, v in b.items()}
                    rt.release(slots)
                    break
                rt.release(slots)
                continue
            learner.learn(b)
            rt.release(slots)
            version += 1
            rt.publish(learner.flat, version=version)
    finally:
        rt.stop()
    assert batch is not None, "no rollout acted under the latest published weights"
    m = learner.model
    obs = batch["obs"].reshape((T + 1) * E, -1)
    mask = batch["mask"][:T].reshape(T * E, s * s, 3)
    act = batch["action"][:T].reshape(T * E, s * s, 7)
    with torch.no_grad():
        lp, _, _ = m.evaluate(obs, mask, act, n_score=T * E)
    assert (mask != 0).any(-1).sum().item() > 0
    torch.testing.assert_close(lp, batch["logp"][:T].reshape(-1), rtol=2e-2, atol=5e-2)



def test_learner_update_with_acting_bitmap_is_identical(cuda):
    """A real engine rollout carries the fused step's active-cell bitmap rows; the learner's
    head compaction then skips its pass over the masks. The update (losses and every updated
    parameter) is bit-identical to the one that builds the bitmap from the masks itself."""
    import sys
    sys.path.insert(0, __import__("os").path.dirname(__file__))
    from helpers import engine_batches

    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    (batch,) = engine_batches(cuda, 16, 1, groups=2, envs=64, T=8, seed=3, learn=False)
    assert "abits" in batch
    mask = batch["mask"]
    T1, B, S, _ = mask.shape
    live = (mask != 0).any(-1).view(T1, B, S // 32, 32).to(torch.int64)
    ref = (live << torch.arange(32, device=cuda)).sum(-1)
    assert torch.equal(batch["abits"].to(torch.int64) & 0xFFFFFFFF, ref)
    outs = []
    for with_bits in (True, False):
        torch.manual_seed(11)
        learner = Learner(Agent((16, 16, 27)), LearnerHParams(), cuda)
        b = dict(batch) if with_bits else {k: v for k, v in batch.items() if k != "abits"}
        losses = learner.learn(b)
        torch.cuda.synchronize()
        outs.append((losses.clone(), learner.flat.data.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
