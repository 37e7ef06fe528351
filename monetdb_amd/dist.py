"""Multi-GPU plumbing: row-range shards and the exchange steps of SURVEY.md §8(e).

One process per GPU (torchrun); rank r owns a row range of every input in its
own HBM -- the mitosis partitioning of opt_mitosis.c:150-230 -- and partial
results are combined the way mergetable re-aggregates packed partials
(opt_mergetable.c:1496-1885):

  * select / calc / sum / Q6 / Q1: no data exchange; exact 128-bit partial
    sums, counts and group keys all-gathered (combine_hge, combine_q1);
  * group + aggregates: local BATgroup + BATgroupsum per rank, the partial
    (key, first row, count, sums) rows hash-partitioned by key and shuffled
    with ONE all_to_all, merged by a second BATgroup on the owner, and group
    ids renumbered in global first-occurrence order (dist_group_aggr); when
    the shards' keys are ordered and their ranges meet only at the shard
    edges (an ordered column cut into row ranges) only the groups shared
    across an edge are merged, from two small all_gathers (_ordered_merge);
  * join: both sides hash-partitioned by key and shuffled, joined on the
    owner, the (l, r) pairs shuffled back to the home rank of their driving
    row and put in the order of the algorithm single-node BATjoin would take
    (join_plan: the same tests and cost model over all-gathered order facts
    and a 1000-value sample) by two stable sorts (dist_join);
  * sort: local stable sort, (key, position) splitters from an all-gathered
    sample, one all_to_all of the runs, stable merge sort per rank
    (dist_sort);
  * RANGE window bounds: shards re-cut at partition starts -- the rows before
    a rank's first partition start move to the rank where that partition
    began -- then bounds are local (dist_window_bounds).

The algorithms are written once against a small backend interface: GdkBackend
runs the local operators through libmgdk on this rank's GPU and exchanges
device buffers with RCCL (torch.distributed backend "nccl"); the tests run the
same code with an oracle backend over gloo on the CPU.  Exchanged columns are
packed into one (rows, k) int64 tensor per shuffle (hge = two words), so each
shuffle is a count exchange plus a single all_to_all_single.
"""

MASK64 = (1 << 64) - 1


def _words(v):
    v &= (1 << 128) - 1
    return [v & MASK64, v >> 64]


def _from_words(lo, hi):
    v = ((hi & MASK64) << 64) | (lo & MASK64)
    return v - (1 << 128) if v >= (1 << 127) else v


def _s64(v):
    v &= MASK64
    return v - (1 << 64) if v >= (1 << 63) else v


def shard(rows_per_rank, rank):
    """Row range [row0, row0 + n) of `rank` under weak scaling."""
    return rank * rows_per_rank, rows_per_rank


def _world(dist):
    if dist is None or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(), dist.get_rank()


def _gather_int64(dist, device, vals):
    import torch
    t = torch.tensor([_s64(v) for v in vals], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[int(x) & MASK64 for x in o.cpu().tolist()] for o in out]


def _gather_var(dist, device, vals):
    """all_gather of a variable-length list of int64 per rank."""
    n = len(vals)
    counts = [c[0] for c in _gather_int64(dist, device, [n])]
    m = max(counts) if counts else 0
    parts = _gather_int64(dist, device, list(vals) + [0] * (m - n))
    return [[_s64(x) for x in p[:c]] for p, c in zip(parts, counts)]


def combine_hge(value, dist=None, device="cpu"):
    """Exact sum of one 128-bit integer per rank."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    parts = _gather_int64(dist, device, _words(value))
    return sum(_from_words(lo, hi) for lo, hi in parts)


Q1_SUMS = ("sum_qty", "sum_base_price", "sum_disc_price", "sum_charge", "sum_disc")
Q1_MAXG = 16


def combine_q1(rows, dist=None, device="cpu", rows_per_rank=0, rank=0):
    """Merge per-rank Q1 group rows: key (returnflag, linestatus), exact sums
    and counts added, first_row = global minimum (first-occurrence order)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return sorted(rows, key=lambda r: r["first_row"])
    flat = [len(rows)]
    for i in range(Q1_MAXG):
        if i < len(rows):
            r = rows[i]
            # first rows are rank-local; the global row is rank * rows_per_rank + local
            flat += [r["returnflag"], r["linestatus"], r["first_row"] + rank * rows_per_rank, r["count_order"]]
            for k in Q1_SUMS:
                flat += _words(r[k])
        else:
            flat += [0] * (4 + 2 * len(Q1_SUMS))
    merged = {}
    for part in _gather_int64(dist, device, flat):
        n = part[0]
        for i in range(n):
            base = 1 + i * (4 + 2 * len(Q1_SUMS))
            key = (part[base], part[base + 1])
            first = part[base + 2]
            m = merged.setdefault(key, {"returnflag": key[0], "linestatus": key[1],
                                        "first_row": first, "count_order": 0,
                                        **{k: 0 for k in Q1_SUMS}})
            m["first_row"] = min(m["first_row"], first)
            m["count_order"] += part[base + 3]
            for j, k in enumerate(Q1_SUMS):
                m[k] += _from_words(part[base + 4 + 2 * j], part[base + 5 + 2 * j])
    return sorted(merged.values(), key=lambda r: r["first_row"])


def avg3(total, count):
    """BATgroupavg3 rounding of an exact sum (gdk/gdk_aggr.c:2070-2095):
    floor average, then half away from zero; returns (avg, remainder)."""
    q, r = divmod(total, count)
    if r > 0:
        if q < 0:
            if 2 * r > count:
                q, r = q + 1, r - count
        elif 2 * r >= count:
            q, r = q + 1, r - count
    return q, r


# ---------------------------------------------------------------------------
# backend: libmgdk on this rank's GPU, RCCL on torch device buffers
# ---------------------------------------------------------------------------

class GdkBackend:
    """Local operators of one rank through libmgdk (device BATs); packing
    into / out of torch tensors on the same GPU for the collectives."""

    def __init__(self, device):
        from monetdb_amd import gdk
        self.gdk = gdk
        self.device = device
        # (event on torch's stream after an exchange's collectives, the source
        # tensors and BATs they read): held until the event has completed
        self._pending = []

    def drain(self, wait=False):
        """release the sources of finished exchanges (all of them, after
        waiting, with wait=True)"""
        left = []
        for ev, keep in self._pending:
            if wait:
                ev.synchronize()
            elif not ev.query():
                left.append((ev, keep))
        self._pending = left

    # -- columns -------------------------------------------------------------
    def n(self, c):
        return c.count()

    def column(self, tp, values, hseq=0):
        import numpy as np
        return self.gdk.BAT.from_numpy(tp, np.asarray(values), hseqbase=hseq)

    def values(self, c):
        return c.values()          # numpy; hge as Python ints

    def widen(self, c):
        g = self.gdk
        if c.ttype in (g.TYPE_lng, g.TYPE_oid):
            return c
        return g.BATcalcaddcst(c, 0, g.TYPE_lng, g.TYPE_lng)

    def zeros_bit(self, n):
        return self.gdk.BATconstant(self.gdk.TYPE_bit, 0, n)

    def append(self, b, n):
        return self.gdk.BATappend(b, n)

    def copy(self, c):
        g = self.gdk
        return g.BATappend(g.BAT(g.lib().mgdk_COLnew(c.hseqbase, c.ttype, max(1, c.count()))), c)

    def slice(self, c, lo, hi):
        return self.gdk.BATslice(c, lo, hi)

    def dense(self, tseq, n):
        return self.gdk.BAT.dense(tseq, n)

    def addcst(self, c, v):
        """c + v as lng (bounds oids to global row numbers).  An oid column
        of row numbers (< 2^63, no nils) has the bits of the same lng values:
        it is relabelled through a view of its heap, not converted, and v == 0
        needs no pass at all."""
        g = self.gdk
        if c.ttype == g.TYPE_oid and c.s.tnonil:
            c = g.BATslice(c, 0, c.count())
            c.s.ttype = g.TYPE_lng
        elif c.ttype != g.TYPE_lng:      # batcalc refuses oid arithmetic: convert first
            c = g.BATconvert(c, None, g.TYPE_lng)
        if v == 0:
            return c
        return g.BATcalcaddcst(c, v, g.TYPE_lng, g.TYPE_lng)

    # -- operators -----------------------------------------------------------
    def hashpartition(self, c, nparts):
        return self.gdk.BAThashpartition(c, nparts)

    def project(self, order, c):
        return self.gdk.BATproject(order, c)

    def group(self, c, histo=True):
        return self.gdk.BATgroup(c, want_histo=histo)

    def groupsum(self, c, g, e, tp):
        return self.gdk.BATgroupsum(c, g, e, tp)

    def group_sums(self, keys, vals, tp):
        """(extents, histo, keys widened to lng, [sums]) of GROUP BY keys
        with exact sums: ONE fused pass when the keys are ordered and the
        sums are hge (mgdk_group_sums_ordered), else BATgroup + BATgroupsum
        + BATproject -- the same columns either way."""
        g = self.gdk
        if tp == g.TYPE_hge and 1 <= len(vals) <= 4:
            r = g.group_sums_ordered(keys, vals)
            if r is not None:
                return r
        gi, e, h = self.group(keys)
        return e, h, self.widen(self.project(e, keys)), [self.groupsum(v, gi, e, tp) for v in vals]

    def groupmin(self, c, g, e):
        # MAL aggr.min: the positions of BATgroupmin projected (aggr.c:321-333)
        return self.gdk.BATproject(self.gdk.BATgroupmin(c, g, e), c)

    def groupavg3(self, c, g, e):
        return self.gdk.BATgroupavg3(c, g, e, True)

    def groupavg3combine(self, a, r, c, g, e):
        return self.gdk.BATgroupavg3combine(a, r, c, g, e, True)

    def join(self, l, r):
        return self.gdk.BATjoin(l, r)

    def sort(self, c, reverse=False):
        # an ordered column is found out first (one read; BATordered records
        # it) so BATsort takes its trivial path (gdk_batop.c:2422-2472):
        # the exchange steps often sort what is sorted already
        if reverse:
            self.gdk.BATordered_rev(c)
        else:
            self.gdk.BATordered(c)
        s, o, _ = self.gdk.BATsort(c, reverse=reverse, nilslast=reverse, groups=False)
        return s, o

    def order_info(self, c):
        """(sorted, revsorted, key-if-sorted, first, last) of a widened column"""
        g = self.gdk
        srt, rev = g.BATordered(c), g.BATordered_rev(c)
        n = c.count()
        first = int(g.BATslice(c, 0, 1).to_numpy()[0])
        last = int(g.BATslice(c, n - 1, n).to_numpy()[0])
        return srt, rev, bool(c.s.tkey) and srt, first, last

    def values_at(self, c, positions):
        import numpy as np
        g = self.gdk
        if len(positions) == 0:
            return []
        o = g.BAT.from_numpy(g.TYPE_oid, np.asarray(positions, np.uint64) + c.hseqbase, sorted_=True, key=True)
        return [int(v) for v in g.BATproject(o, c).to_numpy()]

    def lowerbound2(self, keys, pos, qk, qp):
        return self.gdk.BATlowerbound2(keys, pos, qk, qp)

    def rangebounds(self, vals, parts, limit, preceding):
        return self.gdk.GDKanalyticalwindowbounds(vals, parts, limit, preceding)

    def first_start(self, parts):
        """first position with a partition start bit, or None"""
        s = self.gdk.BATthetaselect(parts, None, 1, "==")
        if s.count() == 0:
            return None
        return int(self.gdk.BATslice(s, 0, 1).to_numpy()[0]) - parts.hseqbase

    # -- zero-copy exchange (RCCL) ---------------------------------------------
    def tensor(self, c):
        """c's tail as a torch tensor on the rank's GPU WITHOUT a copy (the
        CUDA array interface over the BAT's heap); hge as (n, 2) int64.  A
        dense (void) column is materialised first."""
        import torch
        g = self.gdk
        if c.ttype == g.TYPE_void:
            m = g.BAT(g.lib().mgdk_COLnew(c.hseqbase, g.TYPE_oid, max(1, c.count())))
            g.BATappend(m, c)
            c = m
        return torch.as_tensor(_HeapView(c, g), device=self.device)

    def exchange_cols(self, dist, cols, types, send_counts):
        """all_to_all of columns whose rows are grouped by destination rank
        (send_counts[d] rows for rank d): ONE collective per column straight
        from the BAT heaps into the new BATs' heaps (no packing, no host
        staging).  Returns (received columns in rank order, recv counts)."""
        import torch
        g = self.gdk
        sc = torch.tensor(send_counts, dtype=torch.int64, device=self.device)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc)
        recv = [int(x) for x in rc.cpu().tolist()]
        tot = sum(recv)
        # stream order instead of host waits: torch's stream (on which the
        # collectives are ordered) waits for the library stream that wrote
        # the sources, and the library stream -- where every later operator
        # on the received BATs runs -- waits for the collectives
        cur = torch.cuda.current_stream(torch.device(self.device))
        lib = torch.cuda.ExternalStream(g.lib().mgdk_stream(), device=torch.device(self.device))
        cur.wait_stream(lib)
        out, keep = [], []
        for c, tp in zip(cols, types):
            b = g.BAT(g.lib().mgdk_COLnew(0, tp, max(1, tot)))
            b.s.count = tot
            b.s.tsorted = b.s.trevsorted = b.s.tkey = int(tot <= 1)
            b.s.tnonil = int(tot == 0)
            b.s.tnil = 0
            src = self.tensor(c)
            dst = self.tensor(b)
            keep += [src, c]
            dist.all_to_all_single(dst, src, recv, list(send_counts))
            out.append(b)
        lib.wait_stream(cur)
        # the collectives may still be reading the sources on torch's stream.
        # This thread's later operators run on the library stream, ordered
        # after them, but a heap the caller releases goes back to the shared
        # caching allocator, whose next user may be another thread's stream
        # (MAL dataflow workers): the sources are held until an event
        # recorded after the collectives has completed
        ev = torch.cuda.Event()
        ev.record(cur)
        self._pending.append((ev, keep))
        self.drain()
        return out, recv

    # -- packing -------------------------------------------------------------
    def pack(self, cols):
        """(rows, k) int64 tensor of 8-byte and hge (2 words) columns, on the
        GPU (RCCL) or staged through the host for a gloo rehearsal"""
        import torch
        g = self.gdk
        n = cols[0].count() if cols else 0
        if self.device == "cpu":
            parts = []
            for c in cols:
                a = c.to_numpy()
                parts.append(a.view("int64").reshape(n, 2) if c.ttype == g.TYPE_hge
                             else a.astype("int64", copy=False).reshape(n, 1))
            import numpy as np
            return torch.from_numpy(np.ascontiguousarray(np.concatenate(parts, axis=1)))
        width = sum(2 if c.ttype == g.TYPE_hge else 1 for c in cols)
        out = torch.empty((width, n), dtype=torch.int64, device=self.device)
        j = 0
        for c in cols:
            if c.ttype == g.TYPE_hge:
                t = torch.empty((n, 2), dtype=torch.int64, device=self.device)
                if n:
                    g.BATdownload_device(c, t.data_ptr())
                out[j:j + 2] = t.t()
                j += 2
            else:
                if n:
                    g.BATdownload_device(c, out[j].data_ptr())
                j += 1
        return out.t().contiguous()

    def unpack(self, t, types, hseq=0):
        import torch
        g = self.gdk
        n = t.shape[0]
        cols, j = [], 0
        if self.device == "cpu":
            a = t.numpy()
            for tp in types:
                if tp == g.TYPE_hge:
                    cols.append(g.BAT.from_numpy(tp, a[:, j:j + 2].view("uint64"), hseqbase=hseq))
                    j += 2
                else:
                    cols.append(g.BAT.from_numpy(tp, a[:, j].astype(g.NP[tp]), hseqbase=hseq))
                    j += 1
            return cols
        torch.cuda.current_stream(t.device).synchronize()   # collectives ran on torch's stream
        for tp in types:
            if tp == g.TYPE_hge:
                src = t[:, j:j + 2].contiguous()
                j += 2
            else:
                src = t[:, j].contiguous()
                j += 1
            b = g.BAT(g.lib().mgdk_COLnew(hseq, tp, max(n, 1)))
            g.BATupload_device(b, src.data_ptr() if n else 0, n)
            cols.append(b)
        return cols


class _HeapView:
    """A BAT tail under the CUDA array interface (torch.as_tensor wraps it
    without copying); keeps the BAT alive as long as the tensor."""

    def __init__(self, b, g):
        self.b = b
        n = b.count()
        w = b.s.twidth
        shape = (n, 2) if b.ttype == g.TYPE_hge else (n,)
        typestr = "<i8" if b.ttype == g.TYPE_hge else {1: "|i1", 2: "<i2", 4: "<i4", 8: "<i8"}[w]
        ptr = b.s.theap or 0
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False),
                                         "version": 2, "strides": None}


# time spent in the shuffles (exchange below), for the bench's split of a
# step into local operators and exchange
STATS = {"exchange_s": 0.0}


def exchange(be, dist, cols, types, send_counts):
    """Columns shuffled by destination: per-column RCCL all_to_all from the
    heaps when the backend lives on a GPU, else packed rows over gloo."""
    import time
    t = time.perf_counter()
    if getattr(be, "device", "cpu") != "cpu" and hasattr(be, "exchange_cols"):
        out = be.exchange_cols(dist, cols, types, send_counts)[0]
    else:
        recv, _ = _exchange(dist, be.device, be.pack(cols), send_counts)
        out = be.unpack(recv, types)
    STATS["exchange_s"] += time.perf_counter() - t
    return out


def _exchange(dist, device, packed, send_counts):
    """all_to_all of a (rows, k) int64 tensor whose rows are grouped by
    destination rank (send_counts[d] rows for rank d)."""
    import torch
    sc = torch.tensor(send_counts, dtype=torch.int64, device=device)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc)
    recv = [int(x) for x in rc.cpu().tolist()]
    out = torch.empty((sum(recv), packed.shape[1]), dtype=torch.int64, device=device)
    dist.all_to_all_single(out, packed, recv, list(send_counts))
    return out, recv


def _types(be):
    g = getattr(be, "gdk", None) or be
    return g.TYPE_lng, g.TYPE_oid, g.TYPE_hge


# ---------------------------------------------------------------------------
# group + aggregates
# ---------------------------------------------------------------------------

def _allgather_col(be, dist, c, tp):
    """Concatenation over ranks (rank order) of one column, as a column of
    this rank's backend (device BATs for GdkBackend): a size exchange and ONE
    all_gather of the packed rows padded to the largest rank.  Returns
    (column, this rank's offset in it)."""
    import torch
    world, rank = _world(dist)
    if world == 1:
        return c, 0
    n = be.n(c)
    sizes = [int(x[0]) for x in _gather_int64(dist, be.device, [n])]
    width = 2 if tp == _types(be)[2] else 1
    pad = torch.zeros((max(sizes), width), dtype=torch.int64, device=be.device)
    if n:
        pad[:n] = be.pack([c])
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    (col,) = be.unpack(torch.cat([o[:k] for o, k in zip(outs, sizes)]), [tp])
    return col, sum(sizes[:rank])


def _row0s(be, dist, keys):
    """Every rank's first global row (its shard's hseqbase).  The home-rank
    numbering (_home_ids) needs the shards to be contiguous row ranges in rank
    order -- mitosis slices, opt_mitosis.c:150-230 -- so that the row ranges
    cut the ascending first rows; anything else is refused loudly."""
    row0s = [_s64(x[0]) for x in _gather_int64(dist, be.device, [keys.hseqbase])]
    if any(a > b for a, b in zip(row0s, row0s[1:])):
        raise ValueError("dist_group: shards must be row ranges in rank order (hseqbase per rank %s)"
                         % row0s)
    return row0s


def _global_ids(be, dist, firsts):
    """Group ids in global first-occurrence order (what BATgroup over all
    rows numbers them): the rank of each owned group's first row among the
    first rows of every rank.  All on the backend's columns: the all-gathered
    first rows sorted, the sort order sorted again (its inverse permutation),
    this rank's slice of it."""
    TL, TO, TH = _types(be)
    allf, off = _allgather_col(be, dist, firsts, TO)
    _, o = be.sort(allf)
    _, inv = be.sort(o)
    return be.project(be.dense(off, be.n(firsts)), inv)


def _by_gid(be, gid, cols):
    """The owned groups' columns put in ascending gid order."""
    _, og = be.sort(gid)
    return be.project(og, gid), [be.project(og, c) for c in cols]


def _home_ids(be, dist, firsts, row0s, cols):
    """World > 1: the owned groups in ascending gid order, numbered in
    global first-occurrence order without gathering every rank's first rows.
    A group's gid is the number of groups whose first row comes before its
    own.  The ranks' shards are contiguous row ranges in rank order, so the
    owner sorts its first rows and sends each to its HOME rank (the one whose
    range holds it); a home rank ranks the first rows it receives (a sort and
    its inverse) and adds the count of first rows homed at the ranks before
    it; the ranks travel back to the owners in the order they were sent --
    ascending first row, which is ascending gid.  Three sorts of one rank's
    groups instead of two sorts of every rank's (the all-gathered path)."""
    TL, TO, _ = _types(be)
    world, rank = _world(dist)
    n = be.n(firsts)
    s, o = be.sort(firsts)
    cuts = be.lowerbound2(s, None, row0s[1:], [0] * (world - 1)) if n else [0] * (world - 1)
    edges = [0] + [int(c) for c in cuts] + [n]
    counts = [edges[k + 1] - edges[k] for k in range(world)]
    fh = exchange(be, dist, [s], [TO], counts)[0]
    _, oh = be.sort(fh)
    _, inv = be.sort(oh)                     # inv[i] = rank of the i-th received first row
    homed = [int(x[0]) for x in _gather_int64(dist, be.device, [be.n(fh)])]
    gid_h = be.addcst(inv, sum(homed[:rank]))
    sent = _gather_int64(dist, be.device, counts)
    gid = exchange(be, dist, [gid_h], [TL], [sent[q][rank] for q in range(world)])[0]
    return gid, [be.project(o, c) for c in cols]


def _hge_column(be, vals):
    import numpy as np
    TL, TO, TH = _types(be)
    return be.column(TH, np.array([_words(int(v)) for v in vals], dtype=np.uint64).reshape(-1, 2))


def _ordered_merge(be, dist, keys, e, h, gk, gs):
    """dist_group_aggr when every rank's keys are in ascending order and the
    ranks' key ranges follow each other in rank order (max of rank r <= min
    of the next non-empty rank), as an ordered column cut into row ranges
    (mitosis over l_orderkey) is: a group then lives on ONE rank, except a
    key shared across a shard boundary, which is the first group of the
    later rank(s) and the last group of the earlier one.  The earliest rank
    holding a key owns its group (its first row is the group's first row);
    a later rank's first group is folded into it -- count and exact sums
    added -- and dropped there.  Group ids in global first-occurrence order
    are then the owned groups numbered rank by rank.  The exchange is two
    all_gathers of a few words per rank instead of the hash all_to_all of
    every partial group.  Returns None (caller takes the hash path) when the
    shards are not ordered that way."""
    TL, TO, TH = _types(be)
    world, rank = _world(dist)
    n, ng = be.n(keys), be.n(e)
    srt, first, last = 1, 0, 0
    if n:
        s_, _, _, first, last = be.order_info(be.widen(keys))
        srt = int(bool(s_))
    info = _gather_int64(dist, be.device, [srt, ng, first, last])
    info = [[int(q[0]), int(q[1]), _s64(q[2]), _s64(q[3])] for q in info]
    live = [q for q in range(world) if info[q][1]]
    if not all(info[q][0] for q in live) or any(info[a][3] > info[b][2] for a, b in zip(live, live[1:])):
        return None
    STATS["ordered_merge"] = STATS.get("ordered_merge", 0) + 1
    # the first group's partial (count, sums) of every rank, for its owner
    nv = len(gs)
    mine = [0] * (1 + 2 * nv)
    if ng:
        mine[0] = int(be.values(be.slice(h, 0, 1))[0])
        for j, c in enumerate(gs):
            mine[1 + 2 * j:3 + 2 * j] = _words(int(be.values(be.slice(c, 0, 1))[0]))
    parts = _gather_int64(dist, be.device, mine)
    # owner of each live rank's first group: the earliest live rank holding its key
    owner = {}
    for q in live:
        o = q
        for p in live:
            if p < q and info[p][3] == info[q][2]:
                o = p
                break
        owner[q] = o
    kept = {q: info[q][1] - (1 if owner[q] != q else 0) for q in live}
    off = sum(kept.get(q, 0) for q in range(rank))
    if rank not in kept:
        return {"gid": be.dense(off, 0), "key": gk, "first_row": e, "count": h, "sums": gs}
    lo = 1 if owner[rank] != rank else 0
    add = [q for q in live if q != rank and owner[q] == rank and info[q][2] == info[rank][3]]
    cols = [gk, e, h] + list(gs)
    if lo:
        cols = [be.slice(c, 1, ng) for c in cols]
    if add:
        m = be.n(cols[0])
        cnt = int(be.values(be.slice(cols[2], m - 1, m))[0]) + sum(_s64(parts[q][0]) for q in add)
        sums = []
        for j in range(nv):
            c = cols[3 + j]
            v = int(be.values(be.slice(c, m - 1, m))[0])
            v += sum(_from_words(parts[q][1 + 2 * j], parts[q][2 + 2 * j]) for q in add)
            sums.append(v)
        head = [be.copy(be.slice(c, 0, m - 1)) for c in cols]
        cols[2] = be.append(head[2], be.column(TL, [cnt]))
        for j in range(nv):
            cols[3 + j] = be.append(head[3 + j], _hge_column(be, [sums[j]]))
    return {"gid": be.dense(off, kept[rank]), "key": cols[0], "first_row": cols[1], "count": cols[2],
            "sums": cols[3:]}


def dist_group_aggr(be, dist, keys, vals):
    """GROUP BY keys with exact sums of `vals` (lng columns) and counts.

    keys/vals: this rank's shard, hseqbase = the shard's first global row.
    Returns the groups OWNED by this rank as columns of the backend (device
    BATs with GdkBackend), in ascending gid order.  Ownership: by the hash of
    the key when the shards' key ranges overlap (one all_to_all of the
    partial rows); when the ranges meet only at neighbours (ordered input,
    `_ordered_merge`, `STATS["ordered_merge"]`) a group belongs to the
    earliest rank holding its key instead -- a consumer that co-partitions
    other data by `hashpartition` must not assume hash placement then:
    {"gid", "key" (lng), "first_row" (oid), "count" (lng), "sums" [hge]},
    gid = the group's number in global first-occurrence order (what BATgroup
    over all rows would give).  No per-group host objects: the merge, the
    numbering and the ordering run as backend operators and collectives.
    """
    TL, TO, TH = _types(be)
    world, rank = _world(dist)
    # the piece's BATgroup + BATgroupsum (+ the group keys): fused into one
    # pass over the values when the keys are ordered (be.group_sums)
    e, h, gk, gs = be.group_sums(keys, vals, TH)
    if world == 1:
        # one piece: mergetable leaves the plan's BATgroup + BATgroupsum as
        # they are (opt_mergetable.c:1496-1670); their ids are already the
        # first-occurrence numbering, extents the first rows, histo the counts
        return {"gid": be.dense(0, be.n(e)), "key": gk, "first_row": e, "count": h, "sums": gs}
    row0s = _row0s(be, dist, keys)
    got = _ordered_merge(be, dist, keys, e, h, gk, gs)
    if got is not None:
        return got
    parts = [gk, e, h] + gs
    order, counts = be.hashpartition(parts[0], world)
    parts = [be.project(order, c) for c in parts]
    parts = exchange(be, dist, parts, [TL, TO, TL] + [TH] * len(vals), counts)
    rk, rfirst, rcount, rsums = parts[0], parts[1], parts[2], parts[3:]
    if be.n(rk) == 0:
        mk, mf, mc, ms = rk, rfirst, rcount, list(rsums)
    else:
        g2, e2, _ = be.group(rk, histo=False)
        mk = be.project(e2, rk)
        mf = be.groupmin(rfirst, g2, e2)
        mc = be.groupsum(rcount, g2, e2, TL)
        ms = [be.groupsum(s, g2, e2, TH) for s in rsums]
    gid, cols = _home_ids(be, dist, mf, row0s, [mk, mf, mc] + ms)
    return {"gid": gid, "key": cols[0], "first_row": cols[1], "count": cols[2], "sums": cols[3:]}


# ---------------------------------------------------------------------------
# group + exact average (the mergetable plan of AVG: opt_mergetable.c
# mat_group_aggr turns avg into per-shard BATgroupavg3 and one
# BATgroupavg3combine over the partials, gdk_aggr.c:1996 / :2634)
# ---------------------------------------------------------------------------

def dist_group_avg(be, dist, keys, vals):
    """GROUP BY keys, AVG(vals) (lng), as BATgroupavg3 over all rows would
    round it.  Each rank groups its shard and computes (avg, rem, cnt)
    partials; the partial rows are hash-partitioned by key (ONE all_to_all)
    and each owner combines its groups' partials with BATgroupavg3combine.
    Returns this rank's owned groups as backend columns in ascending gid
    order: {"gid", "key", "first_row", "avg"}."""
    TL, TO, TH = _types(be)
    world, rank = _world(dist)
    row0s = _row0s(be, dist, keys) if world > 1 else [0]
    g, e, _ = be.group(keys, histo=False)
    a, r, c = be.groupavg3(vals, g, e)
    parts = [be.widen(be.project(e, keys)), e, a, r, c]
    if world > 1:
        order, counts = be.hashpartition(parts[0], world)
        parts = [be.project(order, x) for x in parts]
        parts = exchange(be, dist, parts, [TL, TO, TL, TL, TL], counts)
    rk, rfirst, ra, rr, rc = parts
    if be.n(rk) == 0:
        mk, mf, ma = rk, rfirst, ra
    else:
        g2, e2, _ = be.group(rk, histo=False)
        mk = be.project(e2, rk)
        mf = be.groupmin(rfirst, g2, e2)
        ma = be.groupavg3combine(ra, rr, rc, g2, e2)
    if world > 1:
        gid, cols = _home_ids(be, dist, mf, row0s, [mk, mf, ma])
    else:
        gid, cols = _by_gid(be, _global_ids(be, dist, mf), [mk, mf, ma])
    return {"gid": gid, "key": cols[0], "first_row": cols[1], "avg": cols[2]}


# ---------------------------------------------------------------------------
# hash join
# ---------------------------------------------------------------------------

def _side_stats(be, dist, c, row0):
    """What BATjoin's tests see of a sharded side (gdk_join.c:4542-4618):
    global count, BATordered / BATordered_rev / the key BATordered records,
    and the values at the positions BATsample(b, 1000) stands for (all rows
    up to 1000, else floor(i * n / 1000)) in row order."""
    n = be.n(c)
    srt, rev, key, first, last = be.order_info(c) if n else (True, True, True, 0, 0)
    parts = _gather_var(dist, be.device, [n, int(srt), int(rev), int(key), _s64(first), _s64(last)])
    N = sum(p[0] for p in parts)
    gs = gr = gk = True
    prev = None
    for p in parts:
        if p[0] == 0:
            continue
        gs &= bool(p[1])
        gr &= bool(p[2])
        gk &= bool(p[3])
        if prev is not None:
            gs &= prev <= p[4]
            gr &= prev >= p[4]
            gk &= prev < p[4]
        prev = p[5]
    gk &= gs
    pos = list(range(N)) if N <= 1000 else [i * N // 1000 for i in range(1000)]
    mine = [q - row0 for q in pos if row0 <= q < row0 + n]
    vals = be.values_at(c, mine) if mine else []
    sample = [v for p in _gather_var(dist, be.device, [_s64(int(v)) for v in vals]) for v in p]
    return dict(n=N, sorted=gs or N <= 1, revsorted=gr or N <= 1, key=gk or N <= 1, sample=sample)


def _guess_uniques(st):
    """guess_uniques / count_unique (gdk_join.c:3337-3576) over the sample."""
    n = st["n"]
    if st["key"]:
        return float(n)
    smp = st["sample"]
    n2 = len(smp)
    n1 = n2 // 2
    if n2 <= 1:
        c1, c2 = n1, n2
    elif st["sorted"] and st["revsorted"]:
        c1 = c2 = 1
    else:
        c1, c2 = len(set(smp[:n1])), len(set(smp))
    A = (c2 - c1) / (n2 - n1)
    B = c1 - n1 * A
    return B + A * n


def join_plan(be, dist, lkeys, rkeys, lrow0, rrow0):
    """The algorithm single-node BATjoin takes on the whole (unsharded) sides
    (gdk_join.c:4542-4618, no candidate lists, value columns) as (driving
    side, matches descending): ("l", False) selectjoin / mergejoin, ("r",
    False) their swapped forms, ("l", True) hashjoin, ("r", True) swapped
    hashjoin; None when a side is empty.

    The estimate is always taken from the 1000-value sample (guess_uniques):
    single-node BATjoin uses a side's tunique_est instead when one is set
    (e.g. by an earlier BATgroup on that column, joinalgo.hip / gdk_join.c
    :3600-3620) and mergejoin_void for a dense side; the pairs' order then
    equals the single-node result only for sides without those properties."""
    import math
    L = _side_stats(be, dist, be.widen(lkeys), lrow0)
    R = _side_stats(be, dist, be.widen(rkeys), rrow0)
    if L["n"] == 0 or R["n"] == 0:
        return None
    if L["n"] == 1 or (L["sorted"] and L["revsorted"]):
        return ("l", False)
    if R["n"] == 1 or (R["sorted"] and R["revsorted"]):
        return ("r", False)
    lord = L["sorted"] or L["revsorted"]
    rord = R["sorted"] or R["revsorted"]
    if lord and rord:
        return ("l", False)

    def cost(b, other_n):          # joincost (gdk_join.c:3586-3689)
        return other_n * 1.1 * (b["n"] / _guess_uniques(b)) + b["n"] * 2.0

    lcost, rcost = cost(L, R["n"]), cost(R, L["n"])
    swap = lcost < rcost
    best = lcost if swap else rcost
    if rord and L["n"] * (math.log2(R["n"]) + 1) < best:
        return ("l", False)
    if lord and R["n"] * (math.log2(L["n"]) + 1) < best:
        return ("r", False)
    return ("r", True) if swap else ("l", True)


def dist_join(be, dist, lkeys, rkeys, lrows_per_rank, rrows_per_rank=None):
    """BATjoin(l, r) over sharded sides.  lkeys/rkeys have hseqbase = their
    shard's first global row.  Returns (r1, r2, driving): this rank's share of
    the global result in the reference's order -- the pairs whose driving row
    (l, or r for the swapped algorithms, `driving`) this rank owns; the
    concatenation over ranks is the single-node BATjoin result."""
    TL, TO, _ = _types(be)
    world, rank = _world(dist)
    if rrows_per_rank is None:
        rrows_per_rank = lrows_per_rank
    if world == 1:
        a, b = be.join(lkeys, rkeys)
        return a, b, None
    plan = join_plan(be, dist, lkeys, rkeys, lkeys.hseqbase, rkeys.hseqbase)
    sides = []
    for c in (lkeys, rkeys):
        w = be.widen(c)
        order, counts = be.hashpartition(w, world)
        sides.append(exchange(be, dist, [be.project(order, w), order], [TL, TO], counts))
    (lk, lo), (rk, ro) = sides
    j1, j2 = be.join(lk, rk)
    r1, r2 = be.project(j1, lo), be.project(j2, ro)
    driving, desc = plan if plan is not None else ("l", False)
    d, o = (r1, r2) if driving == "l" else (r2, r1)
    per = lrows_per_rank if driving == "l" else rrows_per_rank
    # to the driving row's home rank: sort by the driving oid, split by bounds
    _, ordd = be.sort(d)
    d, o = be.project(ordd, d), be.project(ordd, o)
    cuts = be.lowerbound2(d, None, [k * per for k in range(1, world)], [0] * (world - 1))
    edges = [0] + list(cuts) + [be.n(d)]
    counts = [edges[k + 1] - edges[k] for k in range(world)]
    d, o = exchange(be, dist, [d, o], [TO, TO], counts)
    # the reference order: driving rows ascending, their matches ascending
    # (select / merge joins) or descending (hash chains): two stable sorts
    _, oo = be.sort(o, reverse=desc)
    d, o = be.project(oo, d), be.project(oo, o)
    _, od = be.sort(d)
    d, o = be.project(od, d), be.project(od, o)
    return (d, o, driving) if driving == "l" else (o, d, driving)


# ---------------------------------------------------------------------------
# sort
# ---------------------------------------------------------------------------

def dist_sort(be, dist, keys, sample=64):
    """Stable ascending sort of a sharded column (hseqbase = the shard's first
    global row).  Returns this rank's slice of the global result: (sorted
    keys widened to lng, order oids = global positions)."""
    TL, TO, _ = _types(be)
    world, rank = _world(dist)
    w = be.widen(keys)
    s, o = be.sort(w)
    if world == 1:
        return s, o
    n = be.n(s)
    idx = [(i * n) // sample for i in range(sample)] if n else []
    samp = []
    for k, p in zip(be.values_at(s, idx), be.values_at(o, idx)):
        samp += [int(k), int(p)]
    allp = _gather_var(dist, be.device, samp)
    pairs = sorted((p[i], p[i + 1]) for p in allp for i in range(0, len(p), 2))
    spl = [pairs[(d * len(pairs)) // world] for d in range(1, world)] if pairs else []
    cuts = be.lowerbound2(s, o, [k for k, _ in spl], [p for _, p in spl]) if spl else [n] * (world - 1)
    edges = [0] + list(cuts) + [n]
    counts = [edges[d + 1] - edges[d] for d in range(world)]
    k2, p2 = exchange(be, dist, [s, o], [TL, TO], counts)
    if be.n(k2) == 0:
        return k2, p2
    # runs arrive in rank order = ascending positions among equal keys, so
    # a stable sort by key alone gives the global stable order
    s3, o3 = be.sort(k2)
    return s3, be.project(o3, p2)


# ---------------------------------------------------------------------------
# RANGE window bounds
# ---------------------------------------------------------------------------

def dist_window_bounds(be, dist, vals, parts, limit, preceding):
    """GDKanalyticalwindowbounds over row-range shards.  The rows before a
    rank's first partition start belong to a partition that began on an
    earlier rank: they move to that rank (one all_to_all), so every rank
    holds whole partitions and computes its bounds locally.  Returns
    (first global row held, bounds as global row numbers -- a lng column of
    the backend) for the rows this rank holds after the move."""
    TL, TO, _ = _types(be)
    world, rank = _world(dist)
    row0 = vals.hseqbase
    n = be.n(vals)
    if world == 1:
        return row0, be.addcst(be.rangebounds(vals, parts, limit, preceding), row0)
    fs = be.first_start(parts)
    starts = [_s64(x[0]) for x in _gather_int64(dist, be.device, [fs if fs is not None else -1])]
    lead = 0 if rank == 0 else (n if fs is None else fs)
    owner = rank
    if rank > 0:
        owner = rank - 1
        while owner > 0 and starts[owner] < 0:
            owner -= 1
    counts = [0] * world
    counts[owner] = lead
    w = be.widen(vals)
    (rv,) = exchange(be, dist, [be.slice(w, 0, lead)], [TL], counts)
    # kept rows [lead, n), then the leading rows of later ranks (they
    # arrive in rank order and carry no partition start)
    v2 = be.copy(be.slice(w, lead, n))
    p2 = be.copy(be.slice(parts, lead, n))
    if be.n(rv):
        be.append(v2, rv)
        be.append(p2, be.zeros_bit(be.n(rv)))
    kept_first = row0 + lead
    if be.n(v2) == 0:
        # no rows left: an empty lng column (widen's type), the type every
        # other rank's bounds have
        return kept_first, be.copy(be.slice(w, 0, 0))
    return kept_first, be.addcst(be.rangebounds(v2, p2, limit, preceding), kept_first)
