"""String heaps in GDK's layout for the tests (gdk/gdk_atoms.h:356-436): a
GDK_VAROFFSET = 8192-byte hash header, then NUL-terminated strings at 8-byte
aligned positions; 1- and 2-byte tail offsets are relative to the header,
4- and 8-byte offsets are absolute.  A heap below GDK_ELIMLIMIT (64 KiB) is
duplicate eliminated, so BATgroup compares offsets there; a larger one may
hold the same string at several offsets and BATgroup compares contents
(gdk/gdk_group.c:897-919)."""
import numpy as np

VAROFFSET = 8192
ELIMLIMIT = 1 << 16
NIL = b"\x80"


def build_heap(words, copies, pad_to=0, rng=None):
    """Heap holding `copies` copies of every word (a nonduplicate-eliminated
    heap), interleaved so equal strings sit far apart, padded with filler
    strings up to pad_to bytes.  Returns (heap bytes, list of offset lists per
    word, relative to the header)."""
    heap = bytearray(VAROFFSET)
    offs = [[] for _ in words]
    order = [(c, i) for c in range(copies) for i in range(len(words))]
    if rng is not None:
        rng.shuffle(order)
    for _, i in order:
        offs[i].append(len(heap) - VAROFFSET)
        heap += words[i] + b"\0"
        while len(heap) % 8:
            heap += b"\0"
    k = 0
    while len(heap) < pad_to:
        heap += b"filler%06d\0" % k
        while len(heap) % 8:
            heap += b"\0"
        k += 1
    return bytes(heap), offs


def tail(offs_rel, width):
    """Tail offsets of the given width from header-relative offsets."""
    a = np.asarray(offs_rel, np.uint64)
    if width >= 4:
        a = a + VAROFFSET
    dt = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[width]
    assert a.max(initial=0) <= np.iinfo(dt).max
    return a.astype(dt)


def content_groups(words_of_rows, g=None):
    """Expected BATgroup by content: first-occurrence ids of (g, string),
    extents (row positions) and histogram."""
    ids, ext, cnt, seen = [], [], [], {}
    for i, w in enumerate(words_of_rows):
        k = (None if g is None else int(g[i]), w)
        if k not in seen:
            seen[k] = len(ext)
            ext.append(i)
            cnt.append(0)
        ids.append(seen[k])
        cnt[seen[k]] += 1
    return np.asarray(ids, np.uint64), np.asarray(ext, np.uint64), np.asarray(cnt, np.int64)


WORDS = [b"", b"A", b"N", b"R", b"F", b"O", b"abcdefgh", b"abcdefgi", b"zz", b"\xc3\xa9t\xc3\xa9", NIL]


def sample(rng, n, width, copies=6, words=WORDS):
    """n rows drawing a random word and a random copy of it; a heap of at least
    64 KiB.  Returns (tail, heap, word index per row)."""
    heap, offs = build_heap(words, copies, pad_to=ELIMLIMIT + 512 if width != 1 else 0, rng=rng)
    wi = rng.integers(0, len(words), n)
    ci = rng.integers(0, copies, n)
    rel = [offs[w][c] for w, c in zip(wi, ci)]
    return tail(rel, width), heap, wi
