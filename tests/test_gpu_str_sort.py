"""BATsort of str columns on the device (gdk_batop.c BATsort with strCmp,
gdk_atoms.h:414: nil first, then strcmp's unsigned byte order): chunk-key
sorts checked against the same order computed in Python, incl. strings
longer than one chunk, shared prefixes, empty strings, nil, reverse, and a
sub-sort under a prior order / groups (the Q1 ORDER BY)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORDS = [b"", b"A", b"N", b"R", b"abcdefg", b"abcdefgh", b"abcdefga", b"abcdefgh\xc3\xa9z",
         b"abcdefghijklmnopq", b"abcdefghijklmnopr", b"\xff", b"\x7f", b"zz"]
NIL = b"\x80"


def _heap(words):
    heap = bytearray(8192)
    offs = []
    for wd in words:
        offs.append(len(heap) - 8192)
        heap += wd + b"\0"
        while len(heap) % 8:
            heap += b"\0"
    assert offs[-1] < 256
    return bytes(heap), offs


def _col(gdk, idx, words):
    heap, offs = _heap(words)
    return gdk.BAT.from_numpy(gdk.TYPE_str, np.asarray([offs[i] for i in idx], np.uint8), vheap=heap,
                              sorted_=False, revsorted=False, key=False, nonil=NIL not in [words[i] for i in idx])


def _rank(words):
    # strCmp order: nil smallest, then bytes (unsigned) order
    order = sorted(range(len(words)), key=lambda i: (words[i] != NIL, words[i] if words[i] != NIL else b""))
    r = np.empty(len(words), np.int64)
    for k, i in enumerate(order):
        r[i] = k
    return r


@pytest.mark.parametrize("reverse", [False, True])
def test_str_sort(gdk, reverse):
    words = WORDS + [NIL]
    rng = np.random.default_rng(5)
    idx = rng.integers(0, len(words), 20_000)
    b = _col(gdk, idx, words)
    s, o, g = gdk.BATsort(b, reverse=reverse, nilslast=reverse)
    key = _rank(words)[idx]
    want = np.argsort(-key if reverse else key, kind="stable")
    assert np.array_equal(o.to_numpy().astype(np.int64), want)
    assert np.array_equal(s.to_numpy(), b.to_numpy()[want])
    ks = key[want]
    wg = np.concatenate([[0], np.cumsum(ks[1:] != ks[:-1])])
    assert np.array_equal(g.to_numpy().astype(np.int64), wg)
    assert s.s.tsorted == (not reverse) and s.s.trevsorted == reverse


def test_str_subsort_q1_order(gdk):
    """ORDER BY a, b with b a str column: sort a, then sub-sort b."""
    rng = np.random.default_rng(9)
    n = 5_000
    a = rng.integers(0, 4, n).astype(np.int32)
    words = WORDS + [NIL]
    idx = rng.integers(0, len(words), n)
    A = gdk.BAT.from_numpy(gdk.TYPE_int, a)
    B = _col(gdk, idx, words)
    _, o1, g1 = gdk.BATsort(A)
    _, o2, g2 = gdk.BATsort(B, o1, g1)
    want = np.lexsort((_rank(words)[idx], a))     # stable: a, then the string order
    assert np.array_equal(o2.to_numpy().astype(np.int64), want)


def test_str_sort_empty(gdk):
    b = _col(gdk, [], WORDS)
    s, o, g = gdk.BATsort(b)
    assert s.count() == 0 and o.count() == 0 and g.count() == 0
