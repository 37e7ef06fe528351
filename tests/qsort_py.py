"""A second, independent restatement of GDKqsort (gdk/gdk_qsort_impl.h:61-204,
Bentley & McIlroy's three-way quicksort with MonetDB's INSERTSORT = 60 and
the "no swap: insertion sort below 1024" shortcut) in Python, used to
cross-check the C oracle's restatement (oracle/gdk_oracle_sort.c) on small
inputs.  Values are Python numbers / bytes with None as nil; the result is
the permutation of positions (which of the equal values ends where)."""


def _order(reverse, nilslast):
    def lt(x, y):
        if x is None or y is None:
            if x is None and y is None:
                return False
            return (y is None) if nilslast else (x is None)
        return x > y if reverse else x < y

    def eq(x, y):
        if x is None or y is None:
            return x is None and y is None
        return x == y
    return lt, eq


def gdk_qsort(vals, reverse=False, nilslast=False):
    lt, eq = _order(reverse, nilslast)
    v = list(vals)
    pos = list(range(len(v)))

    def swap(i, j):
        v[i], v[j] = v[j], v[i]
        pos[i], pos[j] = pos[j], pos[i]

    def ins(o, n):
        for b in range(1, n):
            a = b
            while a > 0 and lt(v[o + a], v[o + a - 1]):
                swap(o + a, o + a - 1)
                a -= 1

    def med3(o, a, b, c):
        A, B, C = v[o + a], v[o + b], v[o + c]
        if lt(A, B):
            return b if lt(B, C) else (c if lt(A, C) else a)
        return b if lt(C, B) else (a if lt(A, C) else c)

    def sort(o, n):
        while True:
            if n < 60:
                ins(o, n)
                return
            d = n >> 3
            a = med3(o, 0, d, 2 * d)
            b = med3(o, (n >> 1) - d, n >> 1, (n >> 1) + d)
            c = med3(o, n - 1 - 2 * d, n - 1 - d, n - 1)
            b = med3(o, a, b, c)
            if b:
                swap(o, o + b)
            a = b = 1
            c = dd = n - 1
            moved = False
            while True:
                while b <= c and not lt(v[o], v[o + b]):
                    if eq(v[o + b], v[o]):
                        moved = True
                        swap(o + a, o + b)
                        a += 1
                    b += 1
                while b <= c and not lt(v[o + c], v[o]):
                    if eq(v[o], v[o + c]):
                        moved = True
                        swap(o + c, o + dd)
                        dd -= 1
                    c -= 1
                if b > c:
                    break
                swap(o + b, o + c)
                moved = True
                b += 1
                c -= 1
            if not moved and n < 1024:
                ins(o, n)
                return
            r = min(a, b - a)
            for k in range(r):
                swap(o + k, o + b - r + k)
            r = min(dd - c, n - dd - 1)
            for k in range(r):
                swap(o + b + k, o + n - r + k)
            nl, ng = b - a, dd - c
            if nl < ng:
                if nl > 1:
                    sort(o, nl)
                if ng <= 1:
                    return
                o, n = o + n - ng, ng
            else:
                if ng > 1:
                    sort(o + n - ng, ng)
                if nl <= 1:
                    return
                n = nl

    sort(0, len(v))
    return pos
