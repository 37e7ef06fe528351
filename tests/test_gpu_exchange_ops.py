"""Device pieces of the multi-GPU exchange steps: hash partitioning, (key,
position) lower bounds, BATappend, device-to-device BAT copies."""
import numpy as np
import pytest

from helpers import rng

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tname,dt", [("int", np.int32), ("lng", np.int64), ("sht", np.int16)])
@pytest.mark.parametrize("nparts", [1, 2, 7, 8])
def test_hashpartition(gdk, tname, dt, nparts):
    r = rng(201)
    tp = getattr(gdk, "TYPE_" + tname)
    v = r.integers(-3000, 3000, 100_003).astype(dt)
    b = gdk.BAT.from_numpy(tp, v, hseqbase=11)
    o, counts = gdk.BAThashpartition(b, nparts)
    pos = o.to_numpy().astype(np.int64) - 11
    assert sorted(pos.tolist()) == list(range(len(v)))            # a permutation
    assert sum(counts) == len(v)
    edges = np.concatenate([[0], np.cumsum(counts)])
    owner = {}
    for d in range(nparts):
        seg = pos[edges[d]:edges[d + 1]]
        assert np.all(np.diff(seg) > 0)                             # stable inside a part
        for x in np.unique(v[seg]):
            assert owner.setdefault(int(x), d) == d                 # a value meets one part
    # the same value hashes to the same part whatever its storage width
    w = gdk.BAT.from_numpy(gdk.TYPE_lng, v.astype(np.int64))
    o2, c2 = gdk.BAThashpartition(w, nparts)
    assert c2 == counts


def test_lowerbound2(gdk):
    r = rng(202)
    k = np.sort(r.integers(0, 50, 10_000)).astype(np.int64)
    p = np.arange(10_000, dtype=np.uint64) * 3
    kb = gdk.BAT.from_numpy(gdk.TYPE_lng, k)
    pb = gdk.BAT.from_numpy(gdk.TYPE_oid, p)
    qk = [-1, 0, 7, 7, 49, 60]
    qp = [0, 0, 0, int(p[np.searchsorted(k, 7) + 3]), 10**9, 0]
    got = gdk.BATlowerbound2(kb, pb, qk, qp)
    want = [int(np.count_nonzero((k < a) | ((k == a) & (p < b)))) for a, b in zip(qk, qp)]
    assert got == want
    f7 = int(np.searchsorted(k, 7))           # positions are the row numbers when pos is NULL
    assert gdk.BATlowerbound2(kb, None, [7, 7], [5, f7 + 5]) == [f7, f7 + 5]


@pytest.mark.parametrize("tname,dt", [("bte", np.int8), ("int", np.int32), ("lng", np.int64)])
def test_append(gdk, tname, dt):
    r = rng(203)
    tp = getattr(gdk, "TYPE_" + tname)
    a = r.integers(-100, 100, 1000).astype(dt)
    b = gdk.BAT.from_numpy(tp, a)
    parts = [a]
    for n in (1, 5000, 0, 70_000):
        x = r.integers(-100, 100, n).astype(dt)
        gdk.BATappend(b, gdk.BAT.from_numpy(tp, x))
        parts.append(x)
    assert np.array_equal(b.to_numpy(), np.concatenate(parts))
    # with a candidate list
    x = r.integers(-100, 100, 500).astype(dt)
    s = np.sort(r.choice(500, 100, replace=False)).astype(np.uint64)
    gdk.BATappend(b, gdk.BAT.from_numpy(tp, x), gdk.BAT.from_numpy(gdk.TYPE_oid, s))
    assert np.array_equal(b.to_numpy()[-100:], x[s.astype(np.int64)])
    with pytest.raises(gdk.GDKError):
        gdk.BATappend(b, gdk.BAT.from_numpy(gdk.TYPE_dbl, np.zeros(3)))


def test_append_keeps_extreme_positions(gdk, ora):
    """BATappend maintains tmaxpos / tminpos / tunique_est
    (gdk_batop.c:762-792).  BATgroup reads g's tmaxpos for the largest prior
    group id: a group-id column that grew larger ids by an append must be
    regrouped with those ids, exactly as the oracle does."""
    r = rng(204)
    v = r.integers(0, 4, 20_000).astype(np.int32)
    g, _, _ = gdk.BATgroup(gdk.BAT.from_numpy(gdk.TYPE_int, v))
    assert g.s.tmaxpos != (1 << 63) - 1
    more = r.integers(4, 60, 5_000).astype(np.uint64)          # larger ids
    gdk.BATappend(g, gdk.BAT.from_numpy(gdk.TYPE_oid, more))
    gids = g.to_numpy()
    mp = g.s.tmaxpos
    assert mp == (1 << 63) - 1 or gids[mp] == gids.max()
    assert g.s.tunique_est == 0
    w = r.integers(0, 3, len(gids)).astype(np.int8)
    gd, ed, hd = gdk.BATgroup(gdk.BAT.from_numpy(gdk.TYPE_bte, w), None, g)
    og, oe, oh = ora.BATgroup(ora.Bat.from_array(ora.TYPE_bte, w),
                              None, ora.Bat.from_array(ora.TYPE_oid, gids))
    assert np.array_equal(gd.to_numpy(), og.values())
    assert np.array_equal(ed.to_numpy(), oe.values())
    assert np.array_equal(hd.to_numpy(), oh.values())
    # a value known to be the maximum: its position moves with the append
    b = gdk.BAT.from_numpy(gdk.TYPE_lng, np.array([5, 9, 1], np.int64))
    b.s.tmaxpos, b.s.tminpos = 1, 2
    n = gdk.BAT.from_numpy(gdk.TYPE_lng, np.array([3, 12, 0, 2], np.int64))
    n.s.tmaxpos, n.s.tminpos = 1, 2
    gdk.BATappend(b, n)
    assert (b.s.tmaxpos, b.s.tminpos) == (4, 5)
    n2 = gdk.BAT.from_numpy(gdk.TYPE_lng, np.array([4], np.int64))   # extremes unknown
    gdk.BATappend(b, n2)
    assert b.s.tmaxpos == b.s.tminpos == (1 << 63) - 1


def test_append_void(gdk):
    v = gdk.BAT.dense(10, 5)
    gdk.BATappend(v, gdk.BAT.dense(15, 3))                          # continues: stays dense
    assert v.ttype == gdk.TYPE_void and v.count() == 8
    gdk.BATappend(v, gdk.BAT.dense(100, 2))                         # breaks: materialised
    assert list(v.to_numpy()) == list(range(10, 18)) + [100, 101]


def test_device_copies(gdk):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no torch device")
    x = np.arange(1000, dtype=np.int64) * 7
    b = gdk.BAT.from_numpy(gdk.TYPE_lng, x)
    t = torch.empty(1000, dtype=torch.int64, device="cuda:0")
    gdk.BATdownload_device(b, t.data_ptr())
    assert np.array_equal(t.cpu().numpy(), x)
    c = gdk.BAT(gdk.lib().mgdk_COLnew(0, gdk.TYPE_lng, 1))
    gdk.BATupload_device(c, (t * 2).contiguous().data_ptr(), 1000)
    torch.cuda.synchronize()
    assert np.array_equal(c.to_numpy(), x * 2)
