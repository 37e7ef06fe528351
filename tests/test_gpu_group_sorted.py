"""BATgroup of ordered columns on the device (GRP_compare_consecutive_values,
gdk/gdk_group.c:103-175, taken at :940-975 when b is sorted or reverse
sorted and g is ordered) against the oracle: ids, extents, histogram and
properties, with nils, -0.0 / NaN, candidate lists and ordered prior groups."""
import numpy as np
import pytest

from helpers import rng
from test_gpu_props import dprops, oprops

pytestmark = pytest.mark.gpu


def _pair(gdk, ora, tname, v, **fl):
    kw = dict(sorted_=fl.get("sorted", False), revsorted=fl.get("revsorted", False), key=False,
              nonil=fl.get("nonil", False))
    d = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tname), v, hseqbase=5, **kw)
    o = ora.Bat.from_array(getattr(ora, "TYPE_" + tname), v, hseqbase=5, **kw)
    return d, o


def _same(d, o, extra=False):
    assert np.array_equal(np.asarray(d.values()), np.asarray(o.values()))
    assert dprops(d, extra) == oprops(o, extra)


@pytest.mark.parametrize("tname,dt", [("int", np.int32), ("lng", np.int64), ("dbl", np.float64)])
@pytest.mark.parametrize("rev", [False, True])
def test_group_ordered(gdk, ora, tname, dt, rev):
    r = rng(700)
    n = 300_000
    v = np.sort(r.integers(-5000, 5000, n)).astype(dt)
    if dt == np.float64:
        v = v / 8
        v[:50] = np.nan            # nil sorts first
        v[v == 0] = -0.0
    else:
        v[:50] = np.iinfo(dt).min
    if rev:
        v = v[::-1].copy()
    D, O = _pair(gdk, ora, tname, v, sorted=not rev, revsorted=rev)
    g, e, h = gdk.BATgroup(D)
    og, oe, oh = ora.BATgroup(O)
    _same(g, og, extra=True)
    _same(e, oe)
    _same(h, oh)
    # candidate list and an ordered prior grouping
    cand = np.sort(r.choice(n, 100_000, replace=False)).astype(np.uint64) + 5
    S = (gdk.BAT.from_numpy(gdk.TYPE_oid, cand, sorted_=True, key=True, nonil=True, revsorted=False),
         ora.Bat.from_array(ora.TYPE_oid, cand, sorted_=True, key=True, nonil=True))
    g, e, h = gdk.BATgroup(D, S[0])
    og, oe, oh = ora.BATgroup(O, S[1])
    _same(g, og, extra=True)
    _same(e, oe)
    _same(h, oh)
    # a dense candidate slice (extents = its seqbase + start rows, stored by
    # the write pass itself) and no histogram wanted: BATgroup(&g, &e, NULL, ...)
    for want_h in (True, False):
        g, e, h = gdk.BATgroup(D, gdk.BAT.dense(1005, 150_000), want_histo=want_h)
        og, oe, oh = ora.BATgroup(O, ora.Bat.dense(1005, 150_000))
        _same(g, og, extra=True)
        _same(e, oe)
        if want_h:
            _same(h, oh)
        else:
            assert h is None
    prior = (np.arange(n) // 7000).astype(np.uint64)
    G = (gdk.BAT.from_numpy(gdk.TYPE_oid, prior, sorted_=True, revsorted=False, key=False, nonil=True),
         ora.Bat.from_array(ora.TYPE_oid, prior, sorted_=True, nonil=True))
    g, e, h = gdk.BATgroup(D, None, G[0])
    og, oe, oh = ora.BATgroup(O, None, G[1])
    _same(g, og, extra=True)
    _same(e, oe)
    _same(h, oh)


def test_group_establishes_order(gdk, ora):
    """BATgroup computes b's order first (gdk_group.c:764-765): a sorted
    column without the property set groups like the oracle and comes back
    with tsorted known"""
    r = np.random.default_rng(77)
    vals = np.sort(r.integers(-10**6, 10**6, 300_001)).astype(np.int64)
    b = gdk.BAT.from_numpy(gdk.TYPE_lng, vals, sorted_=False, revsorted=False, key=False, nonil=True)
    g, e, h = gdk.BATgroup(b)
    og, oe, oh = ora.BATgroup(ora.Bat.from_array(ora.TYPE_lng, vals))
    assert np.array_equal(g.to_numpy(), og.values())
    assert np.array_equal(e.to_numpy(), oe.values())
    assert np.array_equal(h.to_numpy(), oh.values())
    assert b.s.tsorted == 1
