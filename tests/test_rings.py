"""Shared-memory index rings + seqlock (replace the reference's mp.Queue pair)."""
import multiprocessing as mp

import torch

from microbeast_amd import _native as N
from microbeast_amd.utils.buffers import ShmRing


def _producer(ring, start, n):
    for i in range(start, start + n):
        assert ring.push(i, 10.0)


def test_ring_semantics():
    r = ShmRing(4)
    try:
        for i in range(4):
            assert r.push(i, 0.0)
        assert not r.push(99, 0.01)  # full
        assert r.size() == 4
        assert [r.pop(0.0) for _ in range(4)] == [0, 1, 2, 3]
        assert r.pop(0.01) is None  # empty -> timeout
        r.close()
        assert r.pop(1.0) is None  # closed
    finally:
        r.unlink()


def test_ring_multiprocess_spawn():
    ctx = mp.get_context("spawn")
    r = ShmRing(8)
    try:
        ps = [ctx.Process(target=_producer, args=(r, k * 1000, 200)) for k in range(2)]
        for p in ps:
            p.start()
        got = [r.pop(20.0) for _ in range(400)]
        for p in ps:
            p.join(20)
            assert p.exitcode == 0
        assert sorted(got) == sorted(list(range(200)) + list(range(1000, 1200)))
        # per-producer FIFO order is preserved
        a = [g for g in got if g < 1000]
        assert a == sorted(a)
    finally:
        r.unlink()


def test_seqlock_roundtrip():
    rt = N.runtime()
    ver = torch.zeros(1, dtype=torch.int64)
    src = torch.arange(1000, dtype=torch.float32)
    dst = torch.zeros(1000)
    rt.seqlock_write_begin(ver.data_ptr())
    assert int(ver.item()) % 2 == 1
    assert rt.seqlock_read(ver.data_ptr(), src.data_ptr(), dst.data_ptr(), 4000, 10) == 0
    rt.seqlock_write_end(ver.data_ptr())
    got = rt.seqlock_read(ver.data_ptr(), src.data_ptr(), dst.data_ptr(), 4000, 10)
    assert got == int(ver.item()) + 1
    assert torch.equal(src, dst)
