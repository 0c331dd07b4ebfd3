"""Offline CSV post-processor against the reference's own fixture.

The reference ships an episode log and the file its ``data_processor.py`` produced from it
(``experiments/5_ener/5_enero.csv`` -> ``5_enero_processed.csv``). ``tools/process_csv.py``
must reproduce every full 10-episode window of that fixture; the remainder row differs on
purpose (the reference dropped its window index, data_processor.py:37-39).
"""
from __future__ import annotations

import csv
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/experiments/5_ener"
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _rows(path):
    with open(path) as f:
        return [r for r in csv.reader(f) if r]


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "5_enero_processed.csv")),
                    reason="reference fixture not mounted")
def test_matches_reference_processed_fixture(tmp_path):
    import process_csv

    shutil.copy(os.path.join(REF, "5_enero.csv"), tmp_path / "5_enero.csv")
    out = process_csv.process(str(tmp_path / "5_enero"))
    got, want = _rows(out), _rows(os.path.join(REF, "5_enero_processed.csv"))
    assert got[0] == want[0] == ["Return", "steps"]
    full_want = [r for r in want[1:] if len(r) == 3]
    assert len(full_want) > 300
    for g, w in zip(got[1:], full_want):
        assert int(g[0]) == int(w[0])
        assert float(g[1]) == pytest.approx(float(w[1]), abs=1e-9)
        assert float(g[2]) == pytest.approx(float(w[2]), abs=1e-9)
    n_body = len(_rows(os.path.join(REF, "5_enero.csv"))) - 1
    assert len(got) - 1 == (n_body + 9) // 10


def test_remainder_window_keeps_index(tmp_path):
    import process_csv

    p = tmp_path / "x.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Return", "steps"])
        for i in range(13):
            w.writerow([float(i), 100 + i])
    got = _rows(process_csv.process(str(tmp_path / "x")))
    assert got[1] == ["0", str(4.5), str(104.5)]
    assert got[2][0] == "1" and float(got[2][1]) == pytest.approx(11.0)
