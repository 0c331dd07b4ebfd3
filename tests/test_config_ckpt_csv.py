"""CLI flags, checkpoint format, CSV formats, offline processing."""
import os

import pytest
import torch

from microbeast_amd.config import parse_flags, strtobool
from microbeast_amd.models.agent import Agent
from microbeast_amd.ops.optim import FlatAdam, FlatParams
from microbeast_amd.utils.checkpoint import load_checkpoint, restore, save_checkpoint
from microbeast_amd.utils.metrics import EPISODE_HEADER, LOSS_HEADER, CsvLogger


def test_cli_reference_flags():
    f = parse_flags(["--exp_name", "x"], interactive=False)
    assert f.exp_name == "x" and f.test is False
    assert parse_flags(["--test"], interactive=False).test is True
    assert parse_flags(["--test", "true"], interactive=False).test is True  # crashed in reference
    assert parse_flags(["--test", "false"], interactive=False).test is False
    f = parse_flags(["--env_size", "16", "--lr", "1e-3", "--self_play"], interactive=False)
    assert f.env_size == 16 and f.lr == 1e-3 and f.self_play is True
    d = parse_flags([], interactive=False)
    assert (d.n_actors, d.n_envs, d.env_size, d.unroll_length) == (10, 6, 8, 64)
    assert d.resolved_batch_size("mono") == 2 and d.resolved_batch_size("gpu") == 1
    assert parse_flags(["--batch_size", "3"], interactive=False).resolved_batch_size("gpu") == 3
    assert d.resolved_n_buffers() == 20 and d.gamma == 0.99 and d.adam_eps == 1e-5
    with pytest.raises(Exception):
        strtobool("maybe")


def test_default_lr_is_reference_on_one_rank():
    """the default flags on one GPU must train at the reference lr 2.5e-4
    (microbeast.py:200); only a larger (DP / --batch_size) update scales it."""
    from microbeast_amd.train import scaled_lr, update_frames

    d = parse_flags([], interactive=False)
    assert update_frames(d, "gpu", 1) == 524288
    assert scaled_lr(d, update_frames(d, "gpu", 1)) == pytest.approx(2.5e-4)
    assert scaled_lr(d, update_frames(d, "mono", 1)) == pytest.approx(2.5e-4)
    assert scaled_lr(d, update_frames(d, "gpu", 4)) == pytest.approx(5e-4)  # sqrt(4)


def test_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = Agent((4, 4, 27))
    flat = FlatParams(m, "cpu")
    opt = FlatAdam(flat)
    for q in m.parameters():
        q.grad.normal_()  # through the views: alignment padding stays zero
    opt.step()
    p = save_checkpoint(str(tmp_path / "a.ckpt"), m, opt, step=123, n_update=7,
                        flags={"exp_name": "a"})
    ck = load_checkpoint(p)  # weights_only=True inside
    assert ck["step"] == 123 and ck["n_update"] == 7
    assert "network.0.conv.weight" in ck["model_state_dict"]
    m2 = Agent((4, 4, 27))
    flat2 = FlatParams(m2, "cpu")
    opt2 = FlatAdam(flat2)
    step, nu = restore(ck, m2, opt2)
    assert (step, nu) == (123, 7) and opt2.step_count == 1
    assert torch.equal(flat.data, flat2.data) and torch.equal(opt.m, opt2.m)
    # a bare reference-style state_dict also loads
    torch.save(m.state_dict(), str(tmp_path / "ref.pt"))
    ck = load_checkpoint(str(tmp_path / "ref.pt"))
    Agent((4, 4, 27)).load_state_dict(ck["model_state_dict"])


def test_csv_logger_and_process(tmp_path):
    lg = CsvLogger(str(tmp_path), "e")
    lg.episodes([(1.5, 20, 0, 0), (-10.0, 300, 1, 1)] * 6)
    lg.losses(0, 0.1, 0.2, 0.3, 0.4, 1.0, 768, 768.0, 0.5, 0.5, 1.0)
    lg.close()
    rows = open(tmp_path / "e.csv").read().splitlines()
    assert rows[0] == ",".join(EPISODE_HEADER) and len(rows) == 13
    assert rows[2].split(",")[1] == "300"  # episode lengths are ints > 255 (reference wrapped)
    lrows = open(tmp_path / "eLosses.csv").read().splitlines()
    assert lrows[0].startswith("update,pg_loss,value_loss,entropy_loss,total_loss,update time")
    assert lrows[0] == ",".join(LOSS_HEADER)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    from process_csv import process
    out = process(str(tmp_path / "e"), 10)
    prow = open(out).read().splitlines()
    assert prow[0] == "Return,steps" and len(prow) == 3
    assert prow[2].split(",")[0] == "1"  # remainder row keeps its window index


def test_lr_scaling_only_scales_batches_above_the_base():
    """--lr_scaling (train.scaled_lr): sqrt by default; only global batches above
    --lr_base_batch are scaled (the DP weak-scaling case), smaller configs keep --lr."""
    from microbeast_amd.config import parse_flags
    from microbeast_amd.train import scaled_lr

    f = parse_flags(["--quiet"], interactive=False)
    assert f.lr_scaling == "sqrt"
    base = f.lr_base_batch
    assert scaled_lr(f, base) == f.lr
    assert scaled_lr(f, base // 32) == f.lr
    assert abs(scaled_lr(f, 8 * base) - f.lr * 8 ** 0.5) < 1e-12
    f.lr_scaling = "linear"
    assert abs(scaled_lr(f, 4 * base) - 4 * f.lr) < 1e-12
    f.lr_scaling = "none"
    assert scaled_lr(f, 8 * base) == f.lr


def test_stale_league_shard_is_ignored(tmp_path):
    """a shard from an earlier DP run must not override a newer checkpoint's
    league: shards carry their update number and load only when it matches."""
    from microbeast_amd.utils.checkpoint import load_league_shard, save_league_shard

    ck = str(tmp_path / "x.ckpt")
    save_league_shard(ck, 0, {"results": {1: [2, 3]}, "next_id": 4}, n_update=5)
    assert load_league_shard(ck, 0, 5)["next_id"] == 4
    assert load_league_shard(ck, 0, 7) is None
    assert load_league_shard(ck, 0) is not None  # no update given: no check
    assert load_league_shard(ck, 1, 5) is None
