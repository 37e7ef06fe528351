"""Host-side mirror of the MAL bindings that sit above the GDK operators.

The reference keeps these bindings unchanged (monetdb5/modules/kernel/
algebra.c, aggr.c, group.c, monetdb5/modules/mal/batcalc.c); they only
normalise arguments and call the BAT* functions.  This module restates the
argument normalisation so that MAL-level known-answer fixtures can be
replayed against any GDK implementation (the HIP product or the oracle):
`gdk` is a module exposing BATselect / BATthetaselect / BATproject / ...
"""


def alg_select_args(low, high, li, hi, anti, unknown, is_nil):
    """ALGselect2nil argument rewrite (monetdb5/modules/kernel/algebra.c:260-316).

    Returns (low, high, li, hi, anti) to pass to BATselect with
    nil_matches=False.  `high` None means "th == NULL" (point select);
    `is_nil(v)` tells whether a value is the type's nil.
    """
    nanti, nli, nhi = anti, li, hi
    if not nanti and unknown:
        if nli and is_nil(low):
            low = high
            nli = False
        if nhi and is_nil(high):
            high = low
            nhi = False
        if low == high and is_nil(high):
            nanti = True
        return low, high, nli, nhi, nanti, False
    if not unknown:
        if nli and nhi and is_nil(low) and is_nil(high):
            # special case: equi-select for NIL
            return low, None, nli, nhi, nanti, True
    return low, high, nli, nhi, nanti, False


def ALGselect2(gdk, b, s, low, high, li, hi, anti, unknown=False, nil=None):
    """algebra.select(b, s, low, high, li, hi, anti[, unknown])."""
    is_nil = (lambda v: v is None or v == nil)
    lo, hg, li2, hi2, anti2, point = alg_select_args(low, high, li, hi, anti, unknown, is_nil)
    lo = nil if lo is None else lo
    if point:
        hg = None
    else:
        hg = nil if hg is None else hg
    return gdk.BATselect(b, s, lo, hg, li2, hi2, anti2, False)


def ALGthetaselect2(gdk, b, s, val, op):
    """algebra.thetaselect(b, s, val, op) (algebra.c:340-363)."""
    return gdk.BATthetaselect(b, s, val, op)
