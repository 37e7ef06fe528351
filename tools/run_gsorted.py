"""BATgroupsum over sorted group ids (config 4's shape: l_orderkey-like
runs of 4 rows) for profiling runs: python tools/run_gsorted.py [n] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monetdb_amd import gdk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 600_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
gdk.init(0)
cols = gdk.tpch_lineitem(1, 0, n, 20_000)
okey = gdk.BATconvert(gdk.BAT.dense(0, n), None, gdk.TYPE_lng)
okey = gdk.BATcalcdivmod("/", okey, None, gdk.TYPE_lng, c2=4, t2=gdk.TYPE_lng)
okey.s.tsorted, okey.s.trevsorted, okey.s.tkey, okey.s.tnonil = 1, 0, 0, 1
g, e, h = gdk.BATgroup(okey)
for _ in range(reps):
    s = gdk.BATgroupsum(cols["quantity"], g, e, gdk.TYPE_lng, True)
    del s
    s = gdk.BATgroupsum(cols["extendedprice"], g, e, gdk.TYPE_hge, True)
    del s
gdk.sync()
print("ok")
