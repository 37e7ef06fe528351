"""Per-operator times of dist_group_aggr on one GPU (world 1): where a
high-cardinality GROUP BY (l_orderkey-shaped, 4 rows per group) spends its
time.  python tools/prof_dist_group.py [rows]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from monetdb_amd import dist as D  # noqa: E402
from monetdb_amd import gdk  # noqa: E402


class TimedBackend(D.GdkBackend):
    """GdkBackend with wall time per method."""

    def __init__(self, device):
        super().__init__(device)
        self.t = {}

    def __getattribute__(self, name):
        attr = super().__getattribute__(name)
        if name.startswith("_") or name in ("t", "gdk", "device") or not callable(attr):
            return attr

        def wrap(*a, **k):
            t0 = time.perf_counter()
            r = attr(*a, **k)
            gdk.sync()
            d = self.t.setdefault(name, [0.0, 0])
            d[0] += time.perf_counter() - t0
            d[1] += 1
            return r
        return wrap


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 6_000_000
    gdk.init(0)
    cols = gdk.tpch_lineitem(7, 0, rows, max(1, rows // 30))
    okey = gdk.BATconvert(gdk.BAT.dense(0, rows), None, gdk.TYPE_lng)
    okey = gdk.BATcalcdivmod("/", okey, None, gdk.TYPE_lng, c2=4, t2=gdk.TYPE_lng)
    okey.s.tsorted, okey.s.trevsorted, okey.s.tkey, okey.s.tnonil = 1, 0, 0, 1
    vals = [cols["quantity"], cols["extendedprice"]]
    be = TimedBackend("cuda:0")
    D.dist_group_aggr(be, None, okey, vals)
    be.t.clear()
    gdk.prof_reset()
    gdk.prof_enable(True)
    t0 = time.perf_counter()
    D.dist_group_aggr(be, None, okey, vals)
    tot = time.perf_counter() - t0
    ops = {}
    for k in ("group_sums_ordered", "group", "groupsum", "groupcount", "project", "sort", "calc", "convert", "BATsort", "groupmin"):
        ms, n = gdk.prof_get(k)
        if n:
            ops[k] = [round(ms, 3), n]
    print(json.dumps({"rows": rows, "total_ms": round(tot * 1e3, 2),
                      "backend_ms": {k: [round(v[0] * 1e3, 2), v[1]] for k, v in be.t.items()},
                      "lib_prof_ms": ops}, indent=1))


if __name__ == "__main__":
    main()
