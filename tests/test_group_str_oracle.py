"""BATgroup of str columns in the oracle (CPU): a heap of at least GDK_ELIMLIMIT
(64 KiB) is not duplicate eliminated, so equal strings at different offsets
form ONE group (gdk/gdk_group.c:897-919 keeps the str type and compares with
strCmp; the hash path :1118-1282); a smaller heap is grouped by offset.
Expected values are computed in Python from the strings themselves."""
import numpy as np
import pytest

from helpers import rng
from strheap import ELIMLIMIT, build_heap, content_groups, sample, tail, WORDS


def _bat(ora, t, heap, **kw):
    return ora.Bat.from_array(ora.TYPE_str, t, vheap=heap, **kw)


@pytest.mark.parametrize("width", [2, 4, 8])
def test_group_str_by_content(ora, width):
    r = rng(900 + width)
    t, heap, wi = sample(r, 5000, width)
    assert len(heap) >= ELIMLIMIT
    g, e, h = ora.BATgroup(_bat(ora, t, heap))
    words = [WORDS[i] for i in wi]
    ids, ext, cnt = content_groups(words)
    assert np.array_equal(g.values(), ids)
    assert np.array_equal(e.values(), ext)
    assert np.array_equal(h.values(), cnt)
    assert len(ext) == len(set(words))


def test_group_str_subgroup_and_cands(ora):
    r = rng(911)
    n = 4000
    t, heap, wi = sample(r, n, 4)
    words = [WORDS[i] for i in wi]
    b = _bat(ora, t, heap)
    prior = r.integers(0, 3, n).astype(np.int32)
    g0, _, _ = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, prior))
    g, e, h = ora.BATgroup(b, None, g0)
    ids, ext, cnt = content_groups(words, g0.values())
    assert np.array_equal(g.values(), ids) and np.array_equal(e.values(), ext)
    assert np.array_equal(h.values(), cnt)
    cand = np.sort(r.choice(n, 1500, replace=False)).astype(np.uint64)
    s = ora.Bat.from_array(ora.TYPE_oid, cand, sorted_=True, key=True, nonil=True)
    g, e, h = ora.BATgroup(b, s)
    ids, ext, cnt = content_groups([words[i] for i in cand])
    assert np.array_equal(g.values(), ids)
    assert np.array_equal(e.values(), cand[ext])
    assert np.array_equal(h.values(), cnt)


def test_group_str_small_heap_by_offset(ora):
    """below 64 KiB the reference trusts the heap's duplicate elimination and
    groups offsets (gdk_group.c:900): two copies of one string stay apart"""
    heap, offs = build_heap([b"x", b"y"], 2)
    assert len(heap) < ELIMLIMIT
    rel = [offs[0][0], offs[0][1], offs[1][0], offs[0][0]]
    g, e, h = ora.BATgroup(_bat(ora, tail(rel, 2), heap))
    assert list(g.values()) == [0, 1, 2, 0]
    assert list(h.values()) == [2, 1, 1]
