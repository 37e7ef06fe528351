"""BATsort's radix scatter must make progress whatever the dispatcher keeps
resident (VERDICT r04 "do this" 1).

The scatter's tiles are claimed per XCD in groups of `MGDK_SORT_XCDG` tiles
(sort.hip `claim_tile`), so a tile can wait in its look-back on a
predecessor that no workgroup has claimed yet.  Round 4 relied on one
group fitting in one XCD's resident workgroups; `xg` = 256 never completed.
Now a waiting tile counts an unpublished predecessor's digits itself after
a bounded wait.  These cases break the round-4 assumption on purpose: two
sorts running at once on two threads (each one's workgroups take CUs from
the other), and groups far larger than an XCD runs at once.  Results are
compared with the oracle's BATsort (gdk/gdk_batop.c:2342, GDKrsort
gdk/gdk_rsort.c:21): sorted values, order oids and group ids."""
import os
import threading

import numpy as np
import pytest

from helpers import rng

N = 30_000_000


def _check(gdk, ora, vals, tp_name, got):
    s, o, g = got
    ob = ora.Bat.from_array(getattr(ora, "TYPE_" + tp_name), vals)
    os_, oo, og = ora.BATsort_full(ob)
    assert np.array_equal(s.to_numpy(), os_.values())
    assert np.array_equal(o.to_numpy(), oo.values())
    assert np.array_equal(g.to_numpy(), og.values())


def _sort(gdk, tp_name, vals):
    b = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tp_name), vals, sorted_=False, revsorted=False, key=False)
    return gdk.BATsort(b)


@pytest.mark.gpu
def test_two_sorts_at_once(gdk, ora):
    r = rng(501)
    inputs = [r.integers(-2**31 + 1, 2**31 - 1, N).astype(np.int32),
              r.integers(-1_000_000, 1_000_000, N).astype(np.int32)]
    out, errors = [None, None], []

    def run(k):
        try:
            for _ in range(3):
                out[k] = _sort(gdk, "int", inputs[k])
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    for k in range(2):
        _check(gdk, ora, inputs[k], "int", out[k])


@pytest.mark.gpu
@pytest.mark.parametrize("xg", ["256", "4096"])
def test_sort_large_xcd_groups(gdk, ora, xg, monkeypatch):
    r = rng(502)
    vals = r.integers(-2**31 + 1, 2**31 - 1, N).astype(np.int32)
    monkeypatch.setenv("MGDK_SORT_XCDG", xg)
    got = _sort(gdk, "int", vals)
    monkeypatch.delenv("MGDK_SORT_XCDG")
    _check(gdk, ora, vals, "int", got)


@pytest.mark.gpu
def test_sort_large_xcd_groups_lng(gdk, ora, monkeypatch):
    r = rng(503)
    vals = r.integers(-2**62, 2**62, N // 3).astype(np.int64)
    monkeypatch.setenv("MGDK_SORT_XCDG", "512")
    got = _sort(gdk, "lng", vals)
    monkeypatch.delenv("MGDK_SORT_XCDG")
    _check(gdk, ora, vals, "lng", got)
