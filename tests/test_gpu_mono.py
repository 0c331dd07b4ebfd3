"""CPU actor processes -> one MI355X learner (BASELINE config 2 shape): actors step their
envs on the CPU and get actions from the learner process's batched GPU policy server;
full slots reach HBM by pinned DMA on a copy stream one batch ahead of the learner."""
import pytest
import torch

from microbeast_amd.config import parse_flags

pytestmark = pytest.mark.gpu


def test_mono_runtime_gpu_server_and_prefetch(tmp_path):
    from microbeast_amd.train import train
    flags = parse_flags(["--exp_name", "mono_gpu", "--runtime", "mono", "--device", "cuda",
                         "--env_size", "10", "--n_actors", "4", "--n_envs", "6",
                         "--unroll_length", "16", "--batch_size", "2", "--savedir", str(tmp_path),
                         "--quiet", "--max_updates", "5", "--checkpoint_every", "0",
                         "--batch_timeout", "90"], interactive=False)
    out = train(flags)
    assert out["updates"] == 5 and out["steps"] == 5 * 2 * 6 * 16
    rows = open(tmp_path / "mono_gpuLosses.csv").read().splitlines()[1:]
    assert len(rows) == 5
    for r in rows:
        vals = [float(x) for x in r.split(",")[1:5]]
        assert all(v == v for v in vals)  # no NaN losses


def test_prefetched_batch_matches_cpu_concat(tmp_path):
    """The pinned-DMA device batch equals the CPU get_batch concatenation of the same slots."""
    from microbeast_amd.runtime.staging import PinnedPrefetcher
    from microbeast_amd.utils.buffers import LEARNER_KEYS, ShmRing, create_buffers

    class _RT:  # the slice of MonoRuntime the prefetcher uses
        pass

    rt = _RT()
    rt.flags = parse_flags(["--batch_size", "3", "--quiet"], interactive=False)
    rt.buffers = create_buffers(5, 4, 6, 4)
    torch.manual_seed(0)
    for k, lst in rt.buffers.items():
        for t in lst:
            t.copy_(torch.randint(0, 100, t.shape).to(t.dtype))
    rt.free, rt.full = ShmRing(8), ShmRing(8)
    rt.watchdog = lambda: None
    for m in (3, 0, 4):
        rt.full.push(m)
    dev = torch.device("cuda", 0)
    pf = PinnedPrefetcher(rt, dev)
    try:
        batch, _ = pf.get_batch(30)
        torch.cuda.synchronize()
        for src, dst in LEARNER_KEYS.items():
            ref = torch.cat([rt.buffers[src][m] for m in (3, 0, 4)], dim=1)
            assert torch.equal(batch[dst].cpu(), ref), dst
        freed = sorted(rt.free.pop(1.0) for _ in range(3))
        assert freed == [0, 3, 4]
    finally:
        pf.stop()
        rt.free.unlink()
        rt.full.unlink()
