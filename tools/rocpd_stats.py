"""Kernel statistics from a rocprofv3 SQLite result (rocpd schema).

    python tools/rocpd_stats.py RESULTS_DB OUT_CSV

Writes the same columns as rocprofv3's `--stats` kernel_stats.csv
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev),
so runs recorded without `--output-format csv` can be summarised under
profiles/ like the others.
"""
import csv
import math
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        rows.setdefault(name, []).append(float(dur))
    total = sum(sum(v) for v in rows.values()) or 1.0
    stats = []
    for name, v in rows.items():
        n = len(v)
        mean = sum(v) / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        stats.append((name, n, sum(v), mean, 100.0 * sum(v) / total, min(v), max(v), sd))
    stats.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage",
                    "MinNs", "MaxNs", "StdDev"])
        for r in stats:
            w.writerow([r[0], r[1], int(r[2]), round(r[3], 3), round(r[4], 4),
                        int(r[5]), int(r[6]), round(r[7], 3)])


if __name__ == "__main__":
    main()
