"""League bookkeeping: snapshots, PFSP weighting, result attribution, checkpoint state."""
import io

import torch

from microbeast_amd.runtime.league import League


def test_pfsp_prefers_opponents_the_learner_loses_to():
    lg = League(capacity=8, pfsp_power=2.0, eps=0.0, seed=0)
    a = lg.add_snapshot(torch.zeros(10))
    b = lg.add_snapshot(torch.ones(10))
    # learner beats a 9/10, loses to b 9/10; bot episodes (opponent < 0) are ignored
    eps = [(1.0, 100, 0, 0, a)] * 9 + [(1.0, 100, 0, 1, a)] + \
          [(1.0, 100, 0, 1, b)] * 9 + [(1.0, 100, 0, 0, b)] + [(1.0, 100, 0, 0, -1)] * 50
    lg.record(eps)
    assert lg.games[a] == 10 and lg.games[b] == 10
    assert lg.win_rate(a) > 0.8 and lg.win_rate(b) < 0.2
    w = lg.weights()
    assert w[b] > 10 * w[a]
    picks = [lg.sample() for _ in range(500)]
    assert picks.count(b) > 400


def test_draws_count_half_and_capacity_evicts_easiest():
    lg = League(capacity=2, eps=0.0)
    a = lg.add_snapshot(torch.zeros(3))
    lg.record([(0.0, 10, 0, -1, a)] * 4)
    assert abs(lg.win_rate(a) - 0.5) < 1e-9
    b = lg.add_snapshot(torch.zeros(3))
    lg.record([(0.0, 10, 0, 0, b)] * 20)  # b is easy
    c = lg.add_snapshot(torch.zeros(3))
    assert len(lg) == 2 and b not in lg.snaps and c in lg.snaps and a in lg.snaps


def test_state_dict_roundtrip_is_weights_only_loadable():
    lg = League(capacity=4)
    for i in range(3):
        lg.add_snapshot(torch.full((5,), float(i)))
    lg.record([(1.0, 5, 0, 0, 1), (1.0, 5, 0, 1, 2)])
    lg.current = 2
    buf = io.BytesIO()
    torch.save({"league": lg.state_dict()}, buf)
    buf.seek(0)
    d = torch.load(buf, weights_only=True)["league"]
    lg2 = League(capacity=4)
    lg2.load_state_dict(d)
    assert lg2.next_id == 3 and lg2.current == 2
    assert lg2.win_rate(1) == lg.win_rate(1) and lg2.win_rate(2) == lg.win_rate(2)
    assert torch.equal(lg2.snapshot(2), torch.full((5,), 2.0))
