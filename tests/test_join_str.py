"""BATjoin on str keys (gdk/gdk_join.c:4451-4623 with strCmp / strHash:
nil "\\200" before every string, then strcmp's unsigned bytes).  The
algorithm choice, the scans for order and the result order only see that
order and equality, so both the oracle and the device join the strings as
lng ranks among the distinct strings of both sides (nil -> lng nil); the
oracle ranks with a qsort, the device with BATgroup + the chunked str
BATsort.  The CPU tests pin the oracle's pairs against a brute-force model
and its algorithm choice for ordered inputs; the -m gpu tests compare the
device with the oracle (pairs, their order, the cached order flags) over
1- / 2- / 4- / 8-byte offsets, two different heaps, duplicate copies of a
string in one heap, candidate lists and the ordered paths."""
import numpy as np
import pytest

from helpers import rng
from strheap import ELIMLIMIT, NIL, WORDS, build_heap, tail

VOCAB = WORDS + [b"key%05d" % i for i in range(0, 300, 7)] + \
    [b"a_rather_long_shared_prefix_%03d" % i for i in range(40)] + [b"a_rather_long_shared_prefix_"]


def _key(w):
    return (w != NIL, w)


def _side(r, n, width, words, order=None):
    """(tail, heap, row words): n rows over `words`, each row a random copy
    of its word; order 'asc' / 'desc' sorts the rows by content."""
    copies = 1 if width == 1 else 3     # 1-byte offsets reach 255 bytes
    heap, offs = build_heap(words, copies, pad_to=ELIMLIMIT + 512 if width > 2 else 0, rng=r)
    wi = r.integers(0, len(words), n)
    if order:
        wi = np.array(sorted(wi, key=lambda i: _key(words[i]), reverse=order == "desc"))
    ci = r.integers(0, copies, n)
    return tail([offs[w][c] for w, c in zip(wi, ci)], width), heap, [words[i] for i in wi]


CASES = {
    "shuffled_w2_w8": dict(nl=3000, nr=800, wl=2, wr=8),
    "shuffled_w4_w1": dict(nl=2500, nr=90, wl=4, wr=1, rwords=WORDS),
    "sorted_both": dict(nl=2000, nr=600, wl=4, wr=8, lo="asc", ro="asc"),
    "sorted_desc_l": dict(nl=2000, nr=700, wl=8, wr=4, lo="desc"),
    "unique_build": dict(nl=4000, nr=0, wl=8, wr=8, unique_r=True),
    "single_l": dict(nl=1, nr=900, wl=8, wr=2),
}


def _make(M, tp_str, case, seed):
    c = CASES[case]
    r = rng(seed)
    lw = c.get("lwords", VOCAB)
    rw = c.get("rwords", VOCAB[::-1])
    lt, lh, lv = _side(r, c["nl"], c["wl"], lw, c.get("lo"))
    if c.get("unique_r"):
        rw = [VOCAB[i] for i in r.permutation(len(VOCAB))]
        heap, offs = build_heap(rw, 1, pad_to=ELIMLIMIT + 512)
        rt, rh, rv = tail([offs[i][0] for i in range(len(rw))], c["wr"]), heap, rw
    else:
        rt, rh, rv = _side(r, c["nr"], c["wr"], rw, c.get("ro"))
    mk = (lambda t, h, s: M.BAT.from_numpy(tp_str, t, vheap=h, hseqbase=s, sorted_=False, revsorted=False,
                                           key=False, nonil=False)) if hasattr(M, "BAT") else \
        (lambda t, h, s: M.Bat.from_array(tp_str, t, vheap=h, hseqbase=s))
    return mk(lt, lh, 3), mk(rt, rh, 11), lv, rv


def _model(lv, rv, nil_matches):
    return sorted((i + 3, j + 11) for i, x in enumerate(lv) for j, y in enumerate(rv)
                  if x == y and (x != NIL or nil_matches))


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("nil_matches", [False, True])
def test_oracle_str_join_pairs(ora, case, nil_matches):
    L, R, lv, rv = _make(ora, ora.TYPE_str, case, 5)
    a, b = ora.BATjoin(L, R, nil_matches=nil_matches)
    got = sorted(zip(np.asarray(a.values()).tolist(), np.asarray(b.values()).tolist()))
    assert got == _model(lv, rv, nil_matches)


def test_oracle_str_join_algorithm(ora):
    """ordered inputs take the merge path (and cache the order they found);
    a single-row left side a selectjoin; shuffled sides a hash join"""
    L, R, _, _ = _make(ora, ora.TYPE_str, "sorted_both", 5)
    assert ora.join_algo(L, R) == "mergejoin_sorted"
    assert L.s.sorted and R.s.sorted
    L, R, _, _ = _make(ora, ora.TYPE_str, "single_l", 5)
    assert ora.join_algo(L, R) == "selectjoin"
    L, R, _, _ = _make(ora, ora.TYPE_str, "shuffled_w2_w8", 5)
    assert ora.join_algo(L, R) in ("hashjoin", "hashjoin_swapped")


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("nil_matches", [False, True])
def test_gpu_str_join(gdk, ora, case, nil_matches):
    dl, dr, _, _ = _make(gdk, gdk.TYPE_str, case, 5)
    ol, orr, _, _ = _make(ora, ora.TYPE_str, case, 5)
    a, b = gdk.BATjoin(dl, dr, nil_matches=nil_matches)
    oa, ob = ora.BATjoin(ol, orr, nil_matches=nil_matches)
    assert np.array_equal(a.to_numpy(), oa.values()), case
    assert np.array_equal(b.to_numpy(), ob.values()), case
    for d, o in ((dl, ol), (dr, orr)):
        assert (d.s.tsorted, d.s.trevsorted, d.s.tkey) == (o.s.sorted, o.s.revsorted, o.s.key), case


@pytest.mark.gpu
def test_gpu_str_join_cands(gdk, ora):
    dl, dr, lv, rv = _make(gdk, gdk.TYPE_str, "shuffled_w2_w8", 9)
    ol, orr, _, _ = _make(ora, ora.TYPE_str, "shuffled_w2_w8", 9)
    r = rng(3)
    cl = np.sort(r.choice(len(lv), len(lv) // 3, replace=False)).astype(np.uint64) + 3
    bits = r.random(len(rv)) < 0.5
    DS = gdk.BAT.from_numpy(gdk.TYPE_oid, cl, sorted_=True, key=True, nonil=True)
    OS = ora.Bat.from_array(ora.TYPE_oid, cl, sorted_=True, key=True, nonil=True)
    a, b = gdk.BATjoin(dl, dr, DS, gdk.BAT.msk(bits, hseqbase=11))
    oa, ob = ora.BATjoin(ol, orr, OS, ora.Bat.msk(bits, hseqbase=11))
    assert np.array_equal(a.to_numpy(), oa.values())
    assert np.array_equal(b.to_numpy(), ob.values())
