"""BATguess_uniques (gdk/gdk_join.c:3572, guess_uniques :3519): the join cost
model's distinct-value estimate -- the candidate count for a key column, the
cached tunique_est of a full column, else the two-point extrapolation
B = cnt1 - n1 A + A ncand, A = (cnt2 - cnt1) / (n2 - n1), over a 1000-row
sample whose first half has cnt1 and whole cnt2 distinct values.  The
reference samples at random (BATsample); the oracle and the device take 1000
evenly spaced rows, so the estimate is checked against the oracle's and
against a numpy model of the formula (parity unpinned beyond the model)."""
import numpy as np
import pytest

from helpers import rng


def _model(v, cand):
    """the formula over evenly spaced sample positions of the candidates"""
    c = np.asarray(cand)
    m = len(c)
    pos = np.arange(m) if m <= 1000 else np.array([(i * m) // 1000 for i in range(1000)])
    s = v[c[pos]]
    n2 = len(s)
    n1 = n2 // 2
    cnt1, cnt2 = len(np.unique(s[:n1])), len(np.unique(s))
    a = (cnt2 - cnt1) / (n2 - n1)
    return int(cnt1 - n1 * a + a * m)


@pytest.mark.parametrize("ndistinct", [7, 300, 50_000])
def test_oracle_guess_uniques_model(ora, ndistinct):
    r = rng(2621)
    n = 200_000
    v = r.integers(0, ndistinct, n).astype(np.int32)
    b = ora.Bat.from_array(ora.TYPE_int, v)
    assert ora.BATguess_uniques(b) == _model(v, np.arange(n))
    c = np.sort(r.choice(n, 77_777, replace=False)).astype(np.uint64)
    s = ora.Bat.from_array(ora.TYPE_oid, c, sorted_=True, key=True, nonil=True)
    assert ora.BATguess_uniques(ora.Bat.from_array(ora.TYPE_int, v), s) == _model(v, c.astype(np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("ndistinct", [1, 7, 300, 50_000, 10_000_000])
@pytest.mark.parametrize("form", ["none", "dense", "oids"])
def test_gpu_guess_uniques(gdk, ora, ndistinct, form):
    r = rng(2622 + ndistinct)
    n = 1_000_003
    v = r.integers(0, ndistinct, n).astype(np.int64)
    B = gdk.BAT.from_numpy(gdk.TYPE_lng, v, sorted_=False, revsorted=False, key=False, nonil=True)
    O = ora.Bat.from_array(ora.TYPE_lng, v)
    gs = os_ = None
    if form == "dense":
        gs, os_ = gdk.BAT.dense(1000, 500_000), ora.Bat.dense(1000, 500_000)
    elif form == "oids":
        c = np.sort(r.choice(n, 300_000, replace=False)).astype(np.uint64)
        gs = gdk.BAT.from_numpy(gdk.TYPE_oid, c, sorted_=True, key=True, nonil=True)
        os_ = ora.Bat.from_array(ora.TYPE_oid, c, sorted_=True, key=True, nonil=True)
    assert gdk.BATguess_uniques(B, gs) == ora.BATguess_uniques(O, os_)
    if form == "none":
        # a full column's estimate is cached in tunique_est, as the reference does
        assert B.s.tunique_est == pytest.approx(O.s.unique_est)


@pytest.mark.gpu
def test_gpu_guess_uniques_key(gdk):
    v = np.arange(5000, dtype=np.int32)
    B = gdk.BAT.from_numpy(gdk.TYPE_int, v, sorted_=True, revsorted=False, key=True, nonil=True)
    assert gdk.BATguess_uniques(B) == 5000
    s = gdk.BAT.from_numpy(gdk.TYPE_oid, np.array([1, 5, 9], np.uint64), sorted_=True, key=True, nonil=True)
    assert gdk.BATguess_uniques(B, s) == 3
