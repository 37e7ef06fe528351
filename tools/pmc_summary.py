"""Summarise rocprofv3 PMC passes into profiles/pmc_traffic.json.

    python tools/pmc_summary.py [--src KERNEL_SOURCE] FETCH_CSV WRITE_CSV ROWS_PER_LAUNCH [KERNEL ...]

--src names the .hip file holding the kernels; its sha256 is recorded, and
bench.py reports `traffic` only while that file is unchanged.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  On gfx950 FETCH_SIZE counts
exactly half of the bytes of a wide (16 B/lane) coalesced streaming read
(MI355X_MICROARCH.md, HBM section), so it is doubled here; WRITE_SIZE is
exact for 16-B stores and atomics.
"""
import collections
import csv
import hashlib
import json
import os
import re
import sys


def short(name):
    """k_xxx of a demangled kernel name (template arguments dropped)"""
    m = re.search(r"\bk_\w+", name)
    return m.group(0) if m else name


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    argv = sys.argv[1:]
    src = None
    if argv and argv[0] == "--src":
        src, argv = argv[1], argv[2:]
    fetch, write, rows = argv[0], argv[1], int(argv[2])
    kernels = argv[3:] or None
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = per_kernel(fetch, "FETCH_SIZE")
    w = per_kernel(write, "WRITE_SIZE")
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "profiles", "pmc_traffic.json")
    out = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for k in f:
        if kernels and k not in kernels:
            continue
        fb = f[k] * 1024 * 2
        wb = w.get(k, 0.0) * 1024
        out[k] = {"fetch_size_kib": round(f[k], 1), "write_size_kib": round(w.get(k, 0.0), 1),
                  "hbm_bytes_per_launch": int(fb + wb), "rows_per_launch": rows,
                  "hbm_bytes_per_row": (fb + wb) / rows,
                  "source": [os.path.relpath(fetch), os.path.relpath(write)]}
        if src:
            out[k]["kernel_source"] = os.path.relpath(os.path.abspath(src), root)
            out[k]["kernel_source_sha16"] = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
