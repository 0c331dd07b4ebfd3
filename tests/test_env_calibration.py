"""The stand-in env, played by the reference's initial (uniform over legal actions) policy
against the reference bot mix on 8x8, stays in the statistical regime of the reference's
logged runs (which logged exactly that policy: its optimizer never updated the
acting model). Pinned so that a rules / bot change that moves the env away from the game the
reference ran is noticed (tools/calibrate_env.py prints the full comparison; the residual
deviation is recorded in docs/DESIGN.md section 9a)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools"))


def test_uniform_policy_episode_statistics():
    from calibrate_env import run
    out = run(size=8, envs=48, steps=1500, seed=5, max_steps=2000)
    print(out)
    assert out["episodes"] >= 100
    # reference logs: ~300-step episodes, 221..512 (stand-in: ~340, median ~270)
    assert 250 <= out["mean_len"] <= 400
    # reference: mean return -2.26 .. -1.85 (a loss is -10 plus ~8 of shaping rewards)
    assert -3.0 <= out["mean_return"] <= 0.0
    # reference: 3.4-4.2 % of episodes reach return 10. The stand-in's share is 10.8 % over
    # 973 episodes (tools/calibrate_env.py, 120 envs x 3000 steps) and 10.3 % in this seed-5
    # run (deterministic). Per bot and reward component (csrc/tests/calib_components.cpp, 300
    # episodes each, docs/DESIGN.md section 9a): coac 4.7 %, worker rush 8.0 %, random-biased
    # 26.7 % (the uniform agent WINS 21 % of those games) and light rush 30.0 % (a 520-step
    # loss collects 5.2 harvest + 4.6 worker + 5.3 attack = ~15 of shaping reward, because the
    # rush's first light unit needs the 200-tick barracks and arrives ~step 370: microRTS's own
    # unit timings). Band = the measured value + 1 point
    assert out["win_share_return_ge_10"] <= 0.118
    # the logged episodes all end by step 512: no bot family may average longer than that
    # (random_biased averaged ~785-860 steps before its moves leaned toward the enemy)
    for bot, st in out["per_bot"].items():
        assert st["mean_len"] <= 520, (bot, st)
    assert out["win_share_engine"] <= 0.06
    # the sparse head's work: ~1 % of cells hold an idle own unit
    assert 0.004 <= out["active_cell_fraction"] <= 0.03
