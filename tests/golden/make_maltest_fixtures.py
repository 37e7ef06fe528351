#!/usr/bin/env python3
"""Extract golden vectors from the reference's own MAL known-answer tests.

Run in the build container (where /root/reference exists); the output JSON
files are committed and are what the tests read (the GPU box has no
/root/reference).  Only inputs and expected outputs are kept -- no text of the
reference test files.

Sources (reference paths, relative to /root/reference):
  monetdb5/modules/kernel/Tests/select.maltest  -- algebra.select over an int
      BAT with a nil, on unsorted / sorted / reverse-sorted copies, every
      li/hi/anti combination; expected = projected values of the selection
      (ALGselect2 -> BATselect, monetdb5/modules/kernel/algebra.c:260-326)
  monetdb5/mal/Tests/tst1500.maltest, tst1503.maltest -- group.group on a bte
      BAT: groups / extents / histo (GRPsubgroup5 -> BATgroup)
  monetdb5/modules/mal/Tests/bigsum.maltest -- aggr.sum of 10^16 followed by
      10^7 ones into dbl (BATsum exactness)
  monetdb5/modules/mal/Tests/pqueue.maltest, pqueue2.maltest, pqueue3.maltest
      -- algebra.firstn (ALGfirstn -> BATfirstn, algebra.c:937-990) on int
      BATs: plain top-n (which of the tied rows the heap keeps), top-n with
      group ids, and the two-column cascade (s, g from the previous step);
      str columns are skipped (not on the device path)
  sql/test/analytics/Tests/analytics03.test -- windowed SUM / COUNT over
      RANGE / GROUPS frames that end at the current row's peers (frame
      "unbounded preceding .. current row" and whole-partition frames); only
      columns whose values are the same for every order among peers are
      kept, so they pin GDKanalyticalsum / GDKanalyticalcount
      (gdk_analytic_func.c:1626, :1959) independently of sort stability
  monetdb5/modules/mal/Tests/orderidx00.maltest, orderidx04.maltest --
      algebra.sort (ALGsort -> BATsort, algebra.c:1754-1831) of an int BAT:
      sorted values, and the order oids of the stable variant
  monetdb5/mal/Tests/tst033.maltest, tst034.maltest,
  monetdb5/modules/mal/Tests/orderidx02.maltest -- algebra.projection of
      algebra.select results (every li/hi/anti combination, nil bounds, a
      slice view): the printed (head, value) / (head, oid, value) rows; and
      orderidx02's bat.orderidx order (a stable sort's order oids)
  sql/test/quantiles/Tests/quantiles.test, sql/test/Tests/median_stdev.test,
  sql/test/BugTracker-2013/Tests/stddev-group.Bug-3257.test,
  median-null.Bug-3280.test -- quantile / median / stddev_pop / var_pop
      data and expected printed results (stats_fixtures.json)
"""
import json
import os
import re
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def parse_blocks(text):
    """Yield (kind, header, body_lines, expected_lines) records."""
    lines = text.split("\n")
    i = 0
    while i < len(lines):
        ln = lines[i].strip()
        if ln.startswith("statement") or ln.startswith("query"):
            kind = ln
            body = []
            i += 1
            while i < len(lines) and lines[i].strip() not in ("", "----"):
                body.append(lines[i].strip())
                i += 1
            exp = []
            if i < len(lines) and lines[i].strip() == "----":
                i += 1
                while i < len(lines) and lines[i].strip() != "":
                    exp.append(lines[i].strip())
                    i += 1
            yield kind, body, exp
        else:
            i += 1


def val(tok):
    tok = tok.strip()
    if tok.startswith("nil"):
        return None
    return int(tok.split(":")[0])


def select_fixture():
    path = os.path.join(REF, "monetdb5/modules/kernel/Tests/select.maltest")
    text = open(path).read()
    values = []
    cases = []
    pending = None
    for kind, body, exp in parse_blocks(text):
        stmt = " ".join(body)
        m = re.match(r"bat\.append\(b,\s*(.*)\)$", stmt)
        if m:
            values.append(val(m.group(1)))
            continue
        m = re.match(r"x := algebra\.select\((\w), nil:bat\[:oid\], ([^,]+), ([^,]+), "
                     r"(true|false), (true|false), (true|false)\)$", stmt)
        if m:
            pending = dict(bat=m.group(1), low=val(m.group(2)), high=val(m.group(3)),
                           li=m.group(4) == "true", hi=m.group(5) == "true",
                           anti=m.group(6) == "true")
            continue
        if kind.startswith("query II") and stmt == "io.print(z)" and pending is not None:
            # rows are (head, value) pairs, flattened
            vals = exp[1::2]
            pending["expected"] = sorted(None if v == "NULL" else int(v) for v in vals
                                         if True) if "NULL" not in vals else \
                [None] * vals.count("NULL") + sorted(int(v) for v in vals if v != "NULL")
            cases.append(pending)
            pending = None
    return {"source": "monetdb5/modules/kernel/Tests/select.maltest",
            "type": "int", "values": values,
            "note": "s = algebra.sort(b) ascending nils first; r = descending nils last",
            "cases": cases}


def group_fixture(rel):
    text = open(os.path.join(REF, rel)).read()
    x = []
    outs = {}
    label = None
    for kind, body, exp in parse_blocks(text):
        stmt = " ".join(body)
        m = re.match(r"\w+ := bat\.append\(x,\s*(\d+):bte\)$", stmt)
        if m:
            x.append(int(m.group(1)))
            continue
        if kind.startswith("query II") and re.match(r"io\.print\((g1|e1|h1)\)$", stmt):
            name = stmt[9:11]
            if exp:
                outs[name] = [int(v) for v in exp[1::2]]
    return {"source": rel, "type": "bte", "values": x, "expected": outs}


def bigsum_fixture():
    rel = "monetdb5/modules/mal/Tests/bigsum.maltest"
    text = open(os.path.join(REF, rel)).read()
    first = int(re.search(r"bat\.append\(b,(\d+):lng\)", text).group(1))
    m = re.search(r"iterator\.next\((\d+):lng,(\d+):lng\)", text)
    step, upto = int(m.group(1)), int(m.group(2))
    ones = re.search(r"bat\.append\(b,(\d+):lng\)\s*\n\s*\nstatement ok\s*\n\s*redo", text)
    expected = re.search(r"io\.print\(s\)\s*\n----\s*\n(\S+)", text).group(1)
    return {"source": rel, "first": first, "repeat_value": 1,
            "repeat_count": upto // step, "result_type": "dbl", "expected": expected}


def firstn_fixture(rel):
    """Replay the bat.new / bat.append / algebra.firstn statements; every
    io.print of a result gives the expected (head, tail) rows."""
    text = open(os.path.join(REF, rel)).read()
    bats, types = {}, {}
    results = {}          # name -> expected tail values (from io.print)
    cases = []
    pending = []
    for kind, body, exp in parse_blocks(text):
        stmt = " ".join(body)
        m = re.match(r"(\w+):= bat\.new\(:(\w+)\)$", stmt)
        if m:
            bats[m.group(1)] = []
            types[m.group(1)] = m.group(2)
            continue
        m = re.match(r"bat\.append\((\w+),(.*)\)$", stmt)
        if m:
            bats[m.group(1)].append(m.group(2))
            continue
        m = re.match(r"(?:\((\w+),(\w+)\)|(\w+)):= algebra\.firstn\((\w+),(\w+(?::bat)?),(\w+(?::bat)?),"
                     r"(\d+):lng,(true|false),(true|false),(true|false)\)$", stmt)
        if m:
            topn = m.group(1) or m.group(3)
            gids = m.group(2)
            b, sname, gname = m.group(4), m.group(5), m.group(6)
            case = dict(b=b, type=types[b], values=None if types[b] != "int" else [int(v) for v in bats[b]],
                        s=None if sname.startswith("nil") else sname,
                        g=None if gname.startswith("nil") else gname,
                        n=int(m.group(7)), asc=m.group(8) == "true", nilslast=m.group(9) == "true",
                        distinct=m.group(10) == "true", topn=topn, gids=gids, expected={})
            # s / g are the previous step's results, as the reference printed them
            case["s_values"] = results.get(case["s"]) if case["s"] else None
            case["g_values"] = results.get(case["g"]) if case["g"] else None
            cases.append(case)
            pending = [case]
            continue
        m = re.match(r"io\.print\((\w+)\)$", stmt)
        if m and kind.startswith("query II"):
            rows = sorted((int(exp[i]), int(exp[i + 1])) for i in range(0, len(exp), 2))
            tail = [t for _, t in rows]
            results[m.group(1)] = tail
            for c in pending:
                if m.group(1) in (c["topn"], c["gids"]):
                    c["expected"]["gids" if m.group(1) == c["gids"] else "topn"] = tail
    return {"source": rel, "cases": [c for c in cases if c["type"] == "int"]}


def sort_fixture(rel):
    text = open(os.path.join(REF, rel)).read()
    vals = []
    cases = []
    pending = None
    for kind, body, exp in parse_blocks(text):
        stmt = " ".join(body)
        m = re.match(r"bat\.append\(bv,\s*(-?\d+)\s*\)$", stmt)
        if m:
            vals.append(int(m.group(1)))
            continue
        m = re.match(r"(?:\((\w+),(\w+)\)|(\w+)):= algebra\.sort\(bv,(\S+?),(\S+?),(\S+?)\)$", stmt)
        if m:
            flag = lambda t: t.startswith("1") or t == "true"
            pending = dict(reverse=flag(m.group(4)), nilslast=flag(m.group(5)), stable=flag(m.group(6)),
                           order=m.group(2) is not None, values=list(vals))
            continue
        if pending and kind.startswith("query I") and stmt.startswith("io.print("):
            width = len(kind.split()[1])
            rows = sorted(tuple(int(exp[i + k]) for k in range(width)) for i in range(0, len(exp), width))
            pending["sorted"] = [r[1] for r in rows]
            if width == 3:
                pending["order_oids"] = [r[2] for r in rows]
            cases.append(pending)
            pending = None
    return {"source": rel, "cases": cases}


def project_fixture(rel):
    """algebra.select + algebra.projection (ALGprojection -> BATproject,
    algebra.c:1040-1060) over int BATs built with bat.append (optionally
    algebra.slice views), expected = the printed (head, [oid,] value) rows;
    the order index of bat.orderidx / bat.getorderidx becomes a sort case"""
    text = open(os.path.join(REF, rel)).read()
    bats, sels, projs = {}, {}, {}
    cases, sorts = [], []
    pending = None
    for kind, body, exp in parse_blocks(text):
        stmt = " ".join(body)
        m = re.match(r"(\w+)\s*:=\s*bat\.new\(:int\)$", stmt)
        if m:
            bats[m.group(1)] = []
            continue
        m = re.match(r"bat\.append\((\w+),\s*(-?\d+)\s*\)$", stmt)
        if m and m.group(1) in bats:
            bats[m.group(1)].append(int(m.group(2)))
            continue
        m = re.match(r"(\w+)\s*:=\s*algebra\.slice\((\w+),(\d+),(\d+)\)$", stmt)
        if m:
            bats[m.group(1)] = bats[m.group(2)][int(m.group(3)):int(m.group(4)) + 1]
            continue
        m = re.match(r"(\w+)\s*:=\s*algebra\.select\((\w+),nil:bat\[:oid\],([^,]+),([^,]+),"
                     r"(true|false),(true|false),(true|false)\)$", stmt)
        if m:
            sels[m.group(1)] = dict(bat=m.group(2), low=val(m.group(3)), high=val(m.group(4)),
                                    li=m.group(5) == "true", hi=m.group(6) == "true", anti=m.group(7) == "true")
            continue
        m = re.match(r"(\w+)\s*:=\s*algebra\.projection\((\w+),(\w+)\)$", stmt)
        if m:
            projs[m.group(1)] = (m.group(2), m.group(3))
            continue
        m = re.match(r"(\w+)\s*:=\s*bat\.getorderidx\((\w+)\)$", stmt)
        if m:
            pending = ("orderidx", m.group(2))
            continue
        m = re.match(r"io\.print\((\w+)(?:,(\w+))?\)$", stmt)
        if m and kind.startswith("query I"):
            width = len(kind.split()[1])
            rows = sorted(tuple(int(exp[i + k]) for k in range(width)) for i in range(0, len(exp), width))
            a, b = m.group(1), m.group(2)
            if pending and pending[0] == "orderidx" and b == pending[1]:
                sorts.append(dict(reverse=False, nilslast=False, stable=True, order=True,
                                  values=list(bats[b]), sorted=sorted(bats[b]),
                                  order_oids=[r[1] for r in rows]))
                pending = None
                continue
            if b is None and a in projs:
                sname, bname = projs[a]
                sel = sels[sname]
                if sel["bat"] != bname:
                    continue
                cases.append(dict(sel, values=list(bats[bname]), expected_rows=[list(r) for r in rows]))
            elif b is not None and a in sels and b in projs:
                sel = sels[a]
                cases.append(dict(sel, values=list(bats[sel["bat"]]), expected_rows=[list(r) for r in rows]))
    return {"source": rel, "cases": cases}, sorts


def analytics03_fixture():
    rel = "sql/test/analytics/Tests/analytics03.test"
    text = open(os.path.join(REF, rel)).read()
    m = re.search(r"insert into rowsvsrangevsgroups values (.*)\n", text)
    rows = [tuple(int(float(x)) for x in t.split(",")) for t in re.findall(r"\(([^)]*)\)", m.group(1))]
    blocks = list(parse_blocks(text))
    out = []
    # (query prefix, columns kept: index -> (aggregate, partition col, order col, frame))
    specs = [
        ("select cast(sum(aa) over (rows unbounded preceding)",
         {1: ("sum", None, None, "all"), 3: ("sum", None, "aa", "upto"), 4: ("sum", None, "aa", "upto"),
          6: ("sum", "bb", "bb", "upto"), 7: ("sum", "bb", "bb", "upto")}, 8),
        ("select cast(sum(aa) over (order by aa range between unbounded preceding and current row)",
         {0: ("sum", None, "aa", "upto"), 2: ("count*", None, "aa", "upto"), 3: ("count", None, "aa", "upto")}, 8),
    ]
    deleted = False
    for kind, body, exp in blocks:
        stmt = " ".join(body)
        if stmt.startswith("delete from rowsvsrangevsgroups where aa = 2"):
            deleted = True
            continue
        for prefix, cols, width in specs:
            if stmt.startswith(prefix) and kind.startswith("query"):
                data = [r for r in rows if not (deleted and r[0] == 2)]
                nrow = len(exp) // width
                for ci, (agg, part, order, frame) in cols.items():
                    out.append(dict(aa=[r[0] for r in data], bb=[r[1] for r in data], agg=agg, part=part,
                                    order=order, frame=frame,
                                    # query 1 prints its rows ordered by (bb, aa) -- the
                                    # running sum of its first column is aa in that order
                                    output_order="bb,aa" if "rows unbounded preceding)" in prefix else "sorted",
                                    expected=[int(exp[i * width + ci]) for i in range(nrow)]))
    return {"source": rel, "cases": out}


def analytics03_avg_fixture():
    """Windowed AVG cases of analytics03.test (GDKanalyticalavg,
    gdk/gdk_analytic_statistics.c:364): avg(aa) / avg(cc) (cc real, equal to
    aa in that table) over RANGE unbounded preceding .. current row, and the
    overflowme table's int averages past the int range (floor printed)."""
    rel = "sql/test/analytics/Tests/analytics03.test"
    text = open(os.path.join(REF, rel)).read()
    m = re.search(r"insert into rowsvsrangevsgroups values (.*)\n", text)
    rows = [tuple(int(float(x)) for x in t.split(",")) for t in re.findall(r"\(([^)]*)\)", m.group(1))]
    m = re.search(r"insert into overflowme values (.*)\n", text)
    ovf = [tuple(int(x) for x in t.split(",")) for t in re.findall(r"\(([^)]*)\)", m.group(1))]
    out = []
    deleted = False
    for kind, body, exp in parse_blocks(text):
        stmt = " ".join(body)
        if stmt.startswith("delete from rowsvsrangevsgroups where aa = 2"):
            deleted = True
            continue
        if not kind.startswith("query"):
            continue
        if stmt.startswith("select cast(sum(aa) over (order by aa range between unbounded preceding and current row)"):
            data = [r for r in rows if not (deleted and r[0] == 2)]
            nrow = len(exp) // 8
            for ci, agg in ((6, "avg"), (7, "avgf")):
                out.append(dict(aa=[r[0] for r in data], bb=[r[1] for r in data], agg=agg, part=None,
                                order="aa", frame="upto", floor=False,
                                expected=[float(exp[i * 8 + ci]) for i in range(nrow)]))
        elif stmt.startswith("select floor(avg(aa) over (rows between current row and unbounded following))"):
            nrow = len(exp) // 6
            # 1: range .. unbounded following, no order (one peer group);
            # 3: order by bb range current row .. unbounded following;
            # 5: partition by bb order by bb range unbounded preceding
            for ci, part, order, frame in ((1, None, None, "from"), (3, None, "bb", "from"), (5, "bb", "bb", "upto")):
                out.append(dict(aa=[r[0] for r in ovf], bb=[r[1] for r in ovf], agg="avg", part=part,
                                order=order, frame=frame, floor=True,
                                expected=[float(exp[i * 6 + ci]) for i in range(nrow)]))
    return {"source": rel, "cases": out}


# ---- window frame bounds (GDKanalyticalwindowbounds) ---------------------
def frame_spec(sql):
    """(unit, start, end) of an OVER clause's frame text; a bound is
    [kind, amount, unit_word] with kind PRECEDING / FOLLOWING / CURRENT /
    UNBOUNDED and amount / unit_word as written (e.g. 100.0, None or 1,
    'month').  `range unbounded preceding` abbreviates `range between
    unbounded preceding and current row`."""
    m = re.search(r"\b(rows|range|groups)\s+(between\s+(.*?)\s+and\s+(.*?)|unbounded preceding)\s*\)",
                  sql, re.I | re.S)
    unit = {"rows": 0, "range": 1, "groups": 2}[m.group(1).lower()]

    def bound(t):
        t = t.strip().lower()
        if t == "current row":
            return ["CURRENT", None, None]
        if t.startswith("unbounded"):
            return ["UNBOUNDED", None, None]
        mm = re.match(r"interval\s+'(-?\d+)'\s+(\w+)\s+(preceding|following)", t)
        if mm:
            return [mm.group(3).upper(), int(mm.group(1)), mm.group(2)]
        mm = re.match(r"(-?[\d.]+)\s+(preceding|following)", t)
        return [mm.group(2).upper(), mm.group(1), None]
    if m.group(3) is None:
        return unit, ["UNBOUNDED", None, None], ["CURRENT", None, None]
    return unit, bound(m.group(3)), bound(m.group(4))


def window_functions_fixture():
    """sql/test/Tests/window_functions.test: SUM(salary) over ROWS / GROUPS /
    RANGE frames of the employee table (salary DECIMAL(7,2) = int at scale
    2, PARTITION BY dep_name ORDER BY salary); expected sums per row in the
    printed (partition, order) order."""
    rel = "sql/test/Tests/window_functions.test"
    text = open(os.path.join(REF, rel)).read()
    emp = []
    for m in re.finditer(r"INSERT INTO employee VALUES \(\s*(\d+),\s*'(\w+)',\s*'(\w+)',\s*(\d+),\s*(\d+)\)", text):
        emp.append([int(m.group(1)), m.group(3), int(m.group(4)) * 100])
    cases = []
    for kind, body, exp in parse_blocks(text):
        stmt = " ".join(body)
        if not kind.startswith("query") or "SUM(salary)" not in stmt or "PARTITION BY dep_name ORDER BY salary" \
                not in stmt:
            continue
        overs = re.findall(r"OVER\s*\((.*?\))\s*as", stmt, re.I)
        width = 3 + len(overs)
        nrow = len(exp) // width
        if nrow * width != len(exp) or nrow != len(emp):
            continue
        for ci, over in enumerate(overs):
            unit, st, en = frame_spec(over)
            cases.append(dict(unit=unit, start=st, end=en,
                              ids=[int(float(exp[i * width])) for i in range(nrow)],
                              expected=[int(round(float(exp[i * width + 3 + ci]) * 100)) for i in range(nrow)]))
    return {"source": rel, "employee": emp, "scale": 2, "cases": cases}


def analytics07_fixture():
    """sql/test/analytics/Tests/analytics07.test: count(*) over RANGE frames
    with month / second intervals on date, timestamp and time columns, asc
    and desc; count = frame end - frame start.  Values are kept as their
    calendar / clock components; expected counts in printed order."""
    rel = "sql/test/analytics/Tests/analytics07.test"
    text = open(os.path.join(REF, rel)).read()
    tables = {}
    for m in re.finditer(r"insert into (testintervals\d?) values (.*?)\n\n", text, re.S):
        vals = []
        for t in re.findall(r"\((\w+) '([^']*)', (-?\d+)\)", m.group(2)):
            vals.append([t[0], t[1]])
        tables[m.group(1)] = vals
    cases, errors = [], []
    blocks = list(parse_blocks(text))
    for kind, body, exp in blocks:
        stmt = " ".join(body)
        mt = re.search(r"from (testintervals\d?)\s*$", stmt)
        if not mt or "count(*) over" not in stmt:
            continue
        overs = re.findall(r"over \((.*?\))", stmt)
        if kind.startswith("statement error"):
            for over in overs:
                unit, st, en = frame_spec(over)
                errors.append(dict(table=mt.group(1), desc=" desc " in over, unit=unit, start=st, end=en))
            continue
        width = len(overs)
        nrow = len(exp) // width
        for ci, over in enumerate(overs):
            unit, st, en = frame_spec(over)
            cases.append(dict(table=mt.group(1), desc=" desc " in over, unit=unit, start=st, end=en,
                              expected=[int(exp[i * width + ci]) for i in range(nrow)]))
    return {"source": rel, "tables": tables, "cases": cases, "errors": errors}


# ---- window functions of analytics00 / 01 / 02.test ------------------------
WIN_FUNCS = ("ntile", "first_value", "last_value", "nth_value", "lag", "lead", "min", "max", "sum", "count",
             "avg", "prod", "stddev_samp", "stddev_pop", "var_samp", "var_pop", "covar_samp", "covar_pop", "corr")
SQL_TYPES = {"int": "int", "bigint": "lng", "real": "flt", "double": "dbl"}


def _split_top(s, sep=","):
    """split s at top-level separators (outside parentheses / quotes)"""
    out, depth, cur, q = [], 0, "", False
    for ch in s:
        if ch == "'":
            q = not q
        if not q and ch == "(":
            depth += 1
        elif not q and ch == ")":
            depth -= 1
        if ch == sep and depth == 0 and not q:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    out.append(cur.strip())
    return out


def _sql_literal(t):
    t = t.strip()
    if t == "null":
        return None
    if t.startswith("'"):
        return t.strip("'")
    try:
        return float(t) if "." in t else int(t)
    except ValueError:
        return t                  # e.g. a date literal: the table is not replayed


def _frame_bound(t):
    t = t.strip()
    if t == "current row":
        return ["CURRENT", 0]
    if t.startswith("unbounded"):
        return ["UNBOUNDED", None]
    n, kind = t.split()
    return [kind.upper(), int(n)]


def _window_spec(spec):
    """partition / order column, direction and ROWS frame of an OVER clause
    (None when outside what the replay models)"""
    m = re.fullmatch(r"\s*(?:partition by (\w+))?\s*(?:order by (\w+)(?:\s+(asc|desc))?)?\s*(rows .*)?\s*", spec)
    if not m:
        return None
    part, order, direction, rows = m.groups()
    frame = None
    if rows:
        fm = re.fullmatch(r"rows between (.*) and (.*)", rows.strip())
        if fm:
            frame = [_frame_bound(fm.group(1)), _frame_bound(fm.group(2))]
        else:
            frame = [_frame_bound(rows[5:]), ["CURRENT", 0]]
    return dict(part=part, order=order, desc=direction == "desc", rows=frame)


def _window_item(item, cols):
    """a select-list item: a table column, or FUNC(args) OVER (spec) with an
    optional cast(... as bigint) / floor(...) around it"""
    wrap = None
    m = re.fullmatch(r"cast\((.*) as bigint\)", item)
    if m:
        item, wrap = m.group(1), "cast"
    m = re.fullmatch(r"floor\((.*)\)", item)
    if m:
        item, wrap = m.group(1), "floor"
    if item in cols:
        return dict(kind="col", col=item)
    m = re.fullmatch(r"(\w+)\((.*?)\) over \((.*)\)", item)
    if not m or m.group(1) not in WIN_FUNCS:
        return None
    func, args, spec = m.group(1), _split_top(m.group(2)) if m.group(2) else [], _window_spec(m.group(3))
    if spec is None:
        return None
    for c in (spec["part"], spec["order"]):
        if c is not None and c not in cols:
            return None
    val = args[0] if args else None
    rest = []
    if func == "ntile":
        if val in cols:
            rest = [dict(col=val)]
        else:
            rest = [dict(lit=_sql_literal(val))]
        val = None
    elif func == "count" and val == "*":
        val = None
    else:
        if val not in cols or cols[val] not in SQL_TYPES.values():
            return None               # literal / str values: not GDK window calls on the device
        for a in args[1:]:
            rest.append(dict(col=a) if a in cols else dict(lit=_sql_literal(a)))
    if func in ("first_value", "last_value", "nth_value", "ntile", "lag", "lead") and spec["rows"]:
        return None
    return dict(kind="win", func=func, val=val, args=rest, spec=spec, wrap=wrap)


def analytics_window_fixture():
    """sql/test/analytics/Tests/analytics00 / 01 / 02 / 14 / 15 / 16.test:
    window functions (ntile, first_value, last_value, nth_value, lag, lead,
    min, max, sum, count, avg, prod, stddev_samp / _pop, var_samp / _pop,
    covar_samp / _pop, corr) over PARTITION BY / ORDER BY / ROWS frames of
    small tables with NULLs; a query may mix OVER clauses (spec None: each
    item is evaluated in its own order and the rows compare as a multiset,
    whatever the sort mode).  Each case keeps the tables as inserted (the SQL front end's
    window sort is stable, so rows keep their insertion order among peers)
    and the expected rows as printed (rowsort: compared as multisets)."""
    out = []
    for name in ("analytics00", "analytics01", "analytics02", "analytics14", "analytics15", "analytics16"):
        rel = "sql/test/analytics/Tests/%s.test" % name
        text = open(os.path.join(REF, rel)).read()
        tables, cases = {}, []
        for kind, body, exp in parse_blocks(text):
            stmt = " ".join(body).strip()
            low = stmt.lower()
            m = re.match(r"create table (\w+) \((.*)\)$", low)
            if m:
                cols = {}
                for cd in _split_top(m.group(2)):
                    cn, ct = cd.split()[:2]
                    cols[cn] = SQL_TYPES.get(ct, "str" if ct.startswith("varchar") else None)
                tables[m.group(1)] = dict(cols=cols, names=list(cols), rows=[])
                continue
            m = re.match(r"insert into (\w+) values (.*)$", low)
            if m and m.group(1) in tables:
                for t in re.findall(r"\(([^()]*)\)", stmt[stmt.lower().index(" values ") + 8:]):
                    tables[m.group(1)]["rows"].append([_sql_literal(x.lower() if "'" not in x else x)
                                                       for x in _split_top(t)])
                continue
            if not kind.startswith("query"):
                continue
            m = re.fullmatch(r"select (.*) from (\w+)", low)
            if not m or m.group(2) not in tables:
                continue
            tb = tables[m.group(2)]
            items = [_window_item(it, tb["cols"]) for it in _split_top(m.group(1))]
            wins = [it for it in items if it and it["kind"] == "win"]
            if not wins or any(it is None for it in items):
                continue
            types, sortmode = kind.split()[1], kind.split()[2]
            mixed = any(w["spec"] != wins[0]["spec"] for w in wins)
            if "T" in types:
                continue
            width = len(types)
            if len(exp) % width:
                continue
            rows = [[None if x == "NULL" else (float(x) if t == "R" else int(x))
                     for x, t in zip(exp[i:i + width], types)] for i in range(0, len(exp), width)]
            cases.append(dict(table=m.group(2), items=items, spec=None if mixed else wins[0]["spec"], types=types,
                              sortmode=sortmode, expected=rows))
        out.append(dict(source=rel, tables={k: dict(cols=v["cols"], names=v["names"], rows=v["rows"])
                                            for k, v in tables.items()}, cases=cases))
    return out


# ---- batcalc (tst901 / tst906 / tst908) -------------------------------------
def batcalc_fixture():
    """monetdb5/mal/Tests/tst901.maltest, tst906.maltest: io.print of the BATs
    of a batcalc +, +cst, (/cst,) *, ==, not sequence over 0..9, expected
    as sqllogictest's rowsort md5 of the (oid, value) rows; tst908.maltest:
    batcalc./(b, 1:lng) printed in full."""
    out = {}
    for name in ("tst901", "tst906"):
        rel = "monetdb5/mal/Tests/%s.maltest" % name
        text = open(os.path.join(REF, rel)).read()
        m = re.search(r"bat\.new\(:(\w+)\)", text)
        ops = re.findall(r"(\w) ?:= ?batcalc\.(\+|\*|/|==|not)\((\w+),\s*([\w:]+)", text)
        h = re.search(r"(\d+) values hashing to ([0-9a-f]{32})", text)
        out[name] = {"source": rel, "type": m.group(1), "n": 10,
                     "ops": [list(o) for o in ops], "nvalues": int(h.group(1)), "md5": h.group(2)}
    rel = "monetdb5/mal/Tests/tst908.maltest"
    text = open(os.path.join(REF, rel)).read()
    exp = [e for k, b, e in parse_blocks(text) if k.startswith("query")][0]
    out["tst908"] = {"source": rel, "type": "lng", "divisor": 1,
                     "expected": [[int(exp[i]), int(exp[i + 1])] for i in range(0, len(exp), 2)]}
    return out


# ---- statistics (median / quantile / stddev / var SQL tests) ----------------
def _copy_rows(text):
    """the data rows of the first COPY ... FROM stdin block"""
    i = text.index("<COPY_INTO_DATA>")
    rows = []
    for ln in text[i:].split("\n")[1:]:
        if not ln.strip():
            break
        rows.append(ln)
    return rows


def _inserts(text):
    return [tuple(int(x) for x in m.group(1).split(","))
            for m in re.finditer(r"INSERT INTO \w+ VALUES \(([-\d, ]+)\)", text)] + \
        [tuple(int(x) for x in t.split(","))
         for m in re.finditer(r"insert into \w+ values ((?:\([-\d, ]+\),? ?)+)", text)
         for t in re.findall(r"\(([-\d, ]+)\)", m.group(1))]


def stats_fixture():
    """sql/test/quantiles/Tests/quantiles.test (quantile / median of a
    DECIMAL(15,2) column over 10000 rows, whole and per l_returnflag, p out of
    [0,1] an error), sql/test/Tests/median_stdev.test (median of int columns,
    whole and grouped), sql/test/BugTracker-2013/Tests/stddev-group.Bug-3257.test
    (stddev_pop / var_pop, whole and grouped), median-null.Bug-3280.test
    (median of a DOUBLE column with NULLs).  Kept: the data and the queries'
    (function, p, grouped) with their expected printed results."""
    out = {}
    rel = "sql/test/quantiles/Tests/quantiles.test"
    text = open(os.path.join(REF, rel)).read()
    price, flag = [], []
    for ln in _copy_rows(text):
        a, b = ln.split("\t")
        whole, frac = a.split(".")
        price.append(int(whole) * 100 + int(frac.ljust(2, "0")))
        flag.append(b.strip('"'))
    queries = []
    for kind, body, exp in parse_blocks(text):
        sql = " ".join(body)
        if "l_extendedprice" not in sql or not sql.lower().startswith("select"):
            continue
        items = []
        for m in re.finditer(r"(quantile|median)\(l_extendedprice(?:,\s*([-\d.]+))?\)", sql):
            items.append([m.group(1), float(m.group(2)) if m.group(2) else 0.5])
        queries.append({"items": items, "grouped": "group by" in sql.lower(),
                        "error": kind.startswith("statement error"), "rowsort": "rowsort" in kind,
                        "expected": exp})
    out["quantiles"] = {"source": rel, "price_cents": price, "flag": flag, "queries": queries}
    rel = "sql/test/Tests/median_stdev.test"
    text = open(os.path.join(REF, rel)).read()
    rows = _inserts(text)
    qs = []
    for kind, body, exp in parse_blocks(text):
        sql = " ".join(body)
        m = re.match(r"SELECT (groupID, )?median\((\w+)\) FROM sampleData( GROUP BY groupID)?", sql)
        if m:
            qs.append({"column": m.group(2), "grouped": bool(m.group(3)), "expected": exp})
    out["median_stdev"] = {"source": rel, "groupID": [r[0] for r in rows], "numValue": [r[1] for r in rows],
                           "queries": qs}
    rel = "sql/test/BugTracker-2013/Tests/stddev-group.Bug-3257.test"
    text = open(os.path.join(REF, rel)).read()
    rows = _inserts(text)
    qs = []
    for kind, body, exp in parse_blocks(text):
        sql = " ".join(body)
        m = re.match(r"select (stddev_pop|var_pop)\(i\) from t3257( group by j)?", sql)
        if m:
            qs.append({"func": m.group(1), "grouped": bool(m.group(2)), "expected": exp})
    out["stddev_group"] = {"source": rel, "i": [r[0] for r in rows], "j": [r[1] for r in rows], "queries": qs}
    rel = "sql/test/BugTracker-2013/Tests/median-null.Bug-3280.test"
    text = open(os.path.join(REF, rel)).read()
    rows = [ln.split(",") for ln in _copy_rows(text)[1:]]
    # UPDATE mtcars SET mpg = NULL WHERE cyl = 6
    assert "UPDATE mtcars SET mpg = NULL WHERE cyl = 6" in text
    mpg = [None if float(r[2]) == 6 else float(r[1]) for r in rows]
    exp = [e for k, b, e in parse_blocks(text) if k.startswith("query") and "median" in " ".join(b)][0]
    out["median_null"] = {"source": rel, "mpg": mpg, "expected": exp}
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present; fixtures are already committed")
    fx = {"select": select_fixture(),
          "group_tst1500": group_fixture("monetdb5/mal/Tests/tst1500.maltest"),
          "group_tst1503": group_fixture("monetdb5/mal/Tests/tst1503.maltest"),
          "bigsum": bigsum_fixture(),
          "firstn": [firstn_fixture("monetdb5/modules/mal/Tests/%s.maltest" % f)
                     for f in ("pqueue", "pqueue2", "pqueue3")],
          "window_frames": analytics03_fixture(),
          "window_avg": analytics03_avg_fixture(),
          "sort": [sort_fixture("monetdb5/modules/mal/Tests/%s.maltest" % f)
                   for f in ("orderidx00", "orderidx04")],
          "window_bounds_employee": window_functions_fixture(),
          "window_bounds_intervals": analytics07_fixture(),
          "batcalc": batcalc_fixture(),
          "window_sqltests": analytics_window_fixture()}
    fx["project"] = []
    for rel in ("monetdb5/mal/Tests/tst033.maltest", "monetdb5/mal/Tests/tst034.maltest",
                "monetdb5/modules/mal/Tests/orderidx02.maltest"):
        proj, sorts = project_fixture(rel)
        fx["project"].append(proj)
        if sorts:
            fx["sort"].append({"source": rel, "cases": sorts})
    with open(os.path.join(OUT, "maltest_fixtures.json"), "w") as f:
        json.dump(fx, f, indent=1)
    with open(os.path.join(OUT, "stats_fixtures.json"), "w") as f:
        json.dump(stats_fixture(), f, indent=0)
    print("select cases:", len(fx["select"]["cases"]))
    print("firstn cases:", [len(f["cases"]) for f in fx["firstn"]])
    print("window sqltest cases:", [(f["source"], len(f["cases"])) for f in fx["window_sqltests"]])


if __name__ == "__main__":
    main()
