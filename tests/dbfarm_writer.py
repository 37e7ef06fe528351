"""Writes a small MonetDB-layout bat directory (BBP.dir + heap files) in the
format the reference writes it (gdk/gdk_bbp.c:2154-2199 new_bbpentry,
heap_entry, vheap_entry, BBPdir_header; file names BBPgetfilename :363-396,
settailname gdk_bat.c:194).  Test infrastructure for the loader: there is no
dbfarm in the reference tree to read."""
import os

import numpy as np

GDKLIBRARY = 0o61050
TYPES = {"bte": 1, "sht": 2, "int": 4, "oid": 8, "lng": 8, "dbl": 8, "date": 4, "hge": 16}


def physical(batid):
    if batid < 0o100:
        return "%o" % batid
    dirs = []
    v = batid >> 6
    while True:
        dirs.append("%02o" % (v & 0o77))
        if v < 0o100:
            break
        v >>= 6
    return "/".join(reversed(dirs)) + "/%o" % batid


def props(sorted_=False, revsorted=False, key=False, dense=False, nonil=False, nil=False):
    return (int(sorted_) | int(revsorted) << 7 | int(key) << 8 | int(dense) << 9 | int(nonil) << 10
            | int(nil) << 11)


def write_dbfarm(bat_dir, bats, version=GDKLIBRARY):
    """bats: list of dicts {id, name, type, values (numpy) | strings (list),
    hseqbase, props}"""
    os.makedirs(bat_dir, exist_ok=True)
    lines = ["BBP.dir, GDKversion %d" % version, "8 8 16", "BBPsize=%d" % (max(b["id"] for b in bats) + 1),
             "BBPinfo=0"]
    for b in bats:
        phys = physical(b["id"])
        os.makedirs(os.path.dirname(os.path.join(bat_dir, phys)) or bat_dir, exist_ok=True)
        tp = b["type"]
        if tp == "str":
            # duplicate-eliminated heap with GDK_VAROFFSET-based offsets
            heap = bytearray(8192)
            offs = {}
            codes = []
            for sv in b["strings"]:
                if sv not in offs:
                    offs[sv] = len(heap)
                    heap += sv.encode() + b"\0"
                    while len(heap) % 8:
                        heap += b"\0"
                codes.append(offs[sv] - 8192)
            w = 1 if max(codes) < 256 else 2
            tail = np.array(codes, dtype=np.uint8 if w == 1 else np.uint16)
            ext = ".tail1" if w == 1 else ".tail2"
            with open(os.path.join(bat_dir, phys + ext), "wb") as f:
                f.write(tail.tobytes())
            with open(os.path.join(bat_dir, phys + ".theap"), "wb") as f:
                f.write(bytes(heap))
            n = len(codes)
            lines.append("%d %s %d %d %d str %d 1 %d 0 0 0 0 %d %d %d %d %d" % (
                b["id"], b["name"], 0, n, b.get("hseqbase", 0), w, b.get("props", 0), 1 << 63, n * w,
                1 << 63, 1 << 63, len(heap)))
        elif tp == "void":
            n = b["count"]
            lines.append("%d %s %d %d %d void 0 1 %d 0 0 0 0 %d 0 %d %d" % (
                b["id"], b["name"], 0, n, b.get("hseqbase", 0), props(True, n <= 1, True, True, True),
                b["tseqbase"], 1 << 63, 1 << 63))
        else:
            v = np.ascontiguousarray(b["values"])
            w = TYPES[tp]
            if len(v):      # HEAPsave writes no file for an empty heap (gdk_heap.c:871-884)
                with open(os.path.join(bat_dir, phys + ".tail"), "wb") as f:
                    f.write(v.tobytes())
            n = len(v)
            lines.append("%d %s %d %d %d %s %d 0 %d 0 0 0 0 %d %d %d %d" % (
                b["id"], b["name"], 0, n, b.get("hseqbase", 0), tp, w, b.get("props", 0), 1 << 63, n * w,
                1 << 63, 1 << 63))
    with open(os.path.join(bat_dir, "BBP.dir"), "w") as f:
        f.write("\n".join(lines) + "\n")
