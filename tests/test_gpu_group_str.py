"""BATgroup / BATunique of str columns on the device against the oracle and
against groups computed in Python from the strings: heaps of at least
GDK_ELIMLIMIT (64 KiB) hold equal strings at different offsets and are
grouped by content (gdk/gdk_group.c:897-919, :1118-1282); 2-, 4- and 8-byte
offsets, prior groups, candidate lists, many offset groups per string (the
device's hash + compare of the offset groups' strings), properties."""
import numpy as np
import pytest

from helpers import rng
from strheap import ELIMLIMIT, build_heap, content_groups, sample, tail, WORDS
from test_gpu_props import dprops, oprops

pytestmark = pytest.mark.gpu


def _pair(gdk, ora, t, heap, hseq=0):
    d = gdk.BAT.from_numpy(gdk.TYPE_str, t, vheap=heap, hseqbase=hseq, sorted_=False, revsorted=False,
                           key=False, nonil=False)
    o = ora.Bat.from_array(ora.TYPE_str, t, vheap=heap, hseqbase=hseq)
    return d, o


def _same(d, o, want=None, extra=False):
    dv = np.asarray(d.values())
    assert np.array_equal(dv, np.asarray(o.values()))
    if want is not None:
        assert np.array_equal(dv.astype(np.int64), np.asarray(want).astype(np.int64))
    assert dprops(d, extra) == oprops(o, extra)


@pytest.mark.parametrize("width", [2, 4, 8])
def test_group_str_content(gdk, ora, width):
    r = rng(920 + width)
    n = 100_000
    t, heap, wi = sample(r, n, width)
    assert len(heap) >= ELIMLIMIT
    D, O = _pair(gdk, ora, t, heap)
    gd, ed, hd = gdk.BATgroup(D)
    go, eo, ho = ora.BATgroup(O)
    ids, ext, cnt = content_groups([WORDS[i] for i in wi])
    _same(gd, go, ids, extra=True)
    _same(ed, eo, ext)
    _same(hd, ho, cnt)
    assert D.s.tunique_est == O.s.unique_est == len(ext)
    u = gdk.BATunique(D)
    assert np.array_equal(u.to_numpy() if u.s.ttype else u.values(), ext)


@pytest.mark.parametrize("width", [2, 8])
def test_group_str_subgroup_cands(gdk, ora, width):
    r = rng(930 + width)
    n = 60_000
    t, heap, wi = sample(r, n, width)
    words = [WORDS[i] for i in wi]
    D, O = _pair(gdk, ora, t, heap, hseq=11)
    prior = r.integers(0, 5, n).astype(np.int32)
    g0d, _, _ = gdk.BATgroup(gdk.BAT.from_numpy(gdk.TYPE_int, prior, hseqbase=11))
    g0o, _, _ = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, prior, hseqbase=11))
    gd, ed, hd = gdk.BATgroup(D, None, g0d)
    go, eo, ho = ora.BATgroup(O, None, g0o)
    ids, ext, cnt = content_groups(words, g0o.values())
    _same(gd, go, ids, extra=True)
    _same(ed, eo, ext + 11)
    _same(hd, ho, cnt)
    cand = np.sort(r.choice(n, 25_000, replace=False)).astype(np.uint64) + 11
    SD = gdk.BAT.from_numpy(gdk.TYPE_oid, cand, sorted_=True, key=True, nonil=True, revsorted=False)
    SO = ora.Bat.from_array(ora.TYPE_oid, cand, sorted_=True, key=True, nonil=True)
    gd, ed, hd = gdk.BATgroup(D, SD)
    go, eo, ho = ora.BATgroup(O, SO)
    ids, ext, cnt = content_groups([words[int(i) - 11] for i in cand])
    _same(gd, go, ids, extra=True)
    _same(ed, eo, cand[ext])
    _same(hd, ho, cnt)


def test_group_str_many_offset_groups(gdk, ora):
    """thousands of distinct strings, each stored 3 times: > 3072 offset
    groups (the device's general hash path), rows grouped per string; and
    a sorted column (every equal string still one group)"""
    r = rng(940)
    words = [b"w%05d" % k for k in range(5000)] + [b"", b"\x80"]
    heap, offs = build_heap(words, 3, rng=r)
    assert len(heap) >= ELIMLIMIT
    n = 300_000
    wi = r.integers(0, len(words), n)
    ci = r.integers(0, 3, n)
    t = tail([offs[w][c] for w, c in zip(wi, ci)], 4)
    D, O = _pair(gdk, ora, t, heap)
    gd, ed, hd = gdk.BATgroup(D)
    go, eo, ho = ora.BATgroup(O)
    ids, ext, cnt = content_groups([words[i] for i in wi])
    _same(gd, go, ids, extra=True)
    _same(ed, eo, ext)
    _same(hd, ho, cnt)
    # contiguous runs of equal strings (ids ascending: tsorted)
    wi2 = np.sort(wi)
    t2 = tail([offs[w][c] for w, c in zip(wi2, ci)], 4)
    D2, O2 = _pair(gdk, ora, t2, heap)
    gd, ed, hd = gdk.BATgroup(D2)
    go, eo, ho = ora.BATgroup(O2)
    _same(gd, go, content_groups([words[i] for i in wi2])[0], extra=True)
    assert gd.s.tsorted
    _same(hd, ho)


def test_group_str_small_heap_by_offset(gdk, ora):
    heap, offs = build_heap([b"x", b"y"], 2)
    rel = [offs[0][0], offs[0][1], offs[1][0], offs[0][0]] * 1000
    D, O = _pair(gdk, ora, tail(rel, 2), heap)
    gd, ed, hd = gdk.BATgroup(D)
    go, eo, ho = ora.BATgroup(O)
    _same(gd, go, [0, 1, 2, 0] * 1000, extra=True)
    _same(hd, ho, [2000, 1000, 1000])
