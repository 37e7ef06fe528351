"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker / CPU comparator, never as the product path.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

TYPE_void, TYPE_bit, TYPE_bte, TYPE_sht, TYPE_int, TYPE_oid = 0, 2, 3, 4, 5, 6
TYPE_flt, TYPE_dbl, TYPE_lng, TYPE_hge, TYPE_date, TYPE_str = 8, 9, 10, 11, 12, 16
TYPE_daytime, TYPE_timestamp = 13, 14
TYPE_msk = 1
OID_NIL = 1 << 63

NP = {TYPE_bit: np.int8, TYPE_bte: np.int8, TYPE_sht: np.int16, TYPE_int: np.int32,
      TYPE_date: np.int32, TYPE_oid: np.uint64, TYPE_lng: np.int64, TYPE_flt: np.float32,
      TYPE_dbl: np.float64, TYPE_str: np.uint8, TYPE_daytime: np.int64, TYPE_timestamp: np.int64}
CT = {TYPE_bit: C.c_int8, TYPE_bte: C.c_int8, TYPE_sht: C.c_int16, TYPE_int: C.c_int32,
      TYPE_date: C.c_int32, TYPE_oid: C.c_uint64, TYPE_lng: C.c_int64, TYPE_flt: C.c_float,
      TYPE_dbl: C.c_double, TYPE_daytime: C.c_int64, TYPE_timestamp: C.c_int64}
NIL = {TYPE_bit: -128, TYPE_bte: -128, TYPE_sht: -(1 << 15), TYPE_int: -(1 << 31),
       TYPE_date: -(1 << 31), TYPE_lng: -(1 << 63), TYPE_hge: -(1 << 127), TYPE_oid: OID_NIL}


class OraBat(C.Structure):
    _fields_ = [("type", C.c_int32), ("width", C.c_int32), ("count", C.c_uint64),
                ("hseqbase", C.c_uint64), ("tseqbase", C.c_uint64), ("base", C.c_void_p),
                ("vheap", C.c_void_p), ("vheapsize", C.c_uint64),
                ("sorted", C.c_uint8), ("revsorted", C.c_uint8), ("key", C.c_uint8),
                ("nonil", C.c_uint8), ("nil", C.c_uint8), ("owned", C.c_uint8),
                ("_pad", C.c_uint8 * 2), ("unique_est", C.c_double),
                ("minpos", C.c_uint64), ("maxpos", C.c_uint64)]


class OraLineitem(C.Structure):
    _fields_ = [("n", C.c_uint64), ("shipdate", C.c_void_p), ("quantity", C.c_void_p),
                ("extendedprice", C.c_void_p), ("discount", C.c_void_p), ("tax", C.c_void_p),
                ("returnflag", C.c_void_p), ("linestatus", C.c_void_p)]


class OraQ1Row(C.Structure):
    # ora_hge members are 16-byte aligned in the C struct
    _fields_ = [("returnflag", C.c_uint8), ("linestatus", C.c_uint8), ("_pad", C.c_uint8 * 14),
                ("sum_qty", C.c_uint64 * 2), ("sum_base_price", C.c_uint64 * 2),
                ("sum_disc_price", C.c_uint64 * 2), ("sum_charge", C.c_uint64 * 2),
                ("avg_qty", C.c_int64), ("avg_price", C.c_int64), ("avg_disc", C.c_int64),
                ("rem_qty", C.c_int64), ("rem_price", C.c_int64), ("rem_disc", C.c_int64),
                ("count_order", C.c_int64), ("_tail", C.c_uint8 * 8)]   # sizeof = 144


P = C.POINTER(OraBat)
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle/liboracle.so not built (run make -C oracle)")
        L = C.CDLL(LIB_PATH)
        L.ora_new.restype = P
        L.ora_new.argtypes = [C.c_int, C.c_uint64, C.c_uint64]
        L.ora_free.argtypes = [P]
        L.ora_errbuf.restype = C.c_char_p
        L.ora_select.restype = P
        L.ora_select.argtypes = [P, P, C.c_void_p, C.c_void_p, C.c_bool, C.c_bool, C.c_bool, C.c_bool]
        L.ora_thetaselect.restype = P
        L.ora_thetaselect.argtypes = [P, P, C.c_void_p, C.c_char_p]
        L.ora_project.restype = P
        L.ora_unmask.restype = P
        L.ora_unmask.argtypes = [P]
        L.ora_maskedcands.restype = P
        L.ora_maskedcands.argtypes = [C.c_uint64, C.c_uint64, P, C.c_bool]
        for f in ("ora_mergecand", "ora_intersectcand", "ora_diffcand"):
            getattr(L, f).restype = P
            getattr(L, f).argtypes = [P, P]
        L.ora_negcands.restype = P
        L.ora_negcands.argtypes = [C.c_uint64, C.c_uint64, P]
        L.ora_project.argtypes = [P, P]
        L.ora_calc.restype = P
        L.ora_calc.argtypes = [C.c_char, P, C.c_void_p, C.c_int, P, C.c_void_p, C.c_int, P, C.c_int]
        L.ora_calccmp.restype = P
        L.ora_calccmp.argtypes = [C.c_int, P, C.c_void_p, C.c_int, P, C.c_void_p, C.c_int, P, P, C.c_bool]
        L.ora_calcbetween.restype = P
        L.ora_calcbetween.argtypes = [P, P, C.c_void_p, P, C.c_void_p, C.c_int, P, P, P] + [C.c_bool] * 5
        L.ora_convert.restype = P
        L.ora_convert.argtypes = [P, P, C.c_int, C.c_int, C.c_int, C.c_int]
        L.ora_calcnot.restype = P
        L.ora_calcunary.restype = P
        L.ora_calcunary.argtypes = [C.c_int, P, P]
        L.ora_calcminmax.restype = P
        L.ora_calcminmax.argtypes = [C.c_int, P, P, C.c_void_p, C.c_int, P, P]
        L.ora_calcbits.restype = P
        L.ora_calcbits.argtypes = [C.c_int, C.c_char_p, P, C.c_void_p, C.c_int, P, C.c_void_p, C.c_int, P, P]
        L.ora_calcifthenelse.restype = P
        L.ora_calcifthenelse.argtypes = [P, P, C.c_void_p, P, C.c_void_p, C.c_int]
        L.ora_calcnot.argtypes = [P, P]
        L.ora_calcdivmod.restype = P
        L.ora_calcdivmod.argtypes = [C.c_char, P, C.c_void_p, C.c_int, P, C.c_void_p, C.c_int, P, P, C.c_int]
        L.ora_sum.argtypes = [C.c_void_p, C.c_int, P, P, C.c_bool, C.c_bool]
        L.ora_group.argtypes = [C.POINTER(P), C.POINTER(P), C.POINTER(P), P, P, P]
        for f in ("ora_groupsum",):
            getattr(L, f).restype = P
            getattr(L, f).argtypes = [P, P, P, P, C.c_int, C.c_bool]
        L.ora_groupcount.restype = P
        L.ora_groupcount.argtypes = [P, P, P, P, C.c_bool]
        L.ora_groupminmax.restype = P
        L.ora_groupminmax.argtypes = [P, P, P, P, C.c_bool, C.c_bool]
        L.ora_groupavg.argtypes = [C.POINTER(P), C.POINTER(P), P, P, P, P, C.c_bool, C.c_int]
        L.ora_groupavg3combine.restype = P
        L.ora_groupavg3combine.argtypes = [P, P, P, P, P, C.c_bool]
        L.ora_groupavg3.argtypes = [C.POINTER(P), C.POINTER(P), C.POINTER(P), P, P, P, P, C.c_bool]
        L.ora_join.argtypes = [C.POINTER(P), C.POINTER(P), P, P, P, P, C.c_bool]
        L.ora_groupmoments.restype = P
        L.ora_groupmoments.argtypes = [C.c_int, P, P, P, P, P, C.c_bool, C.c_bool, C.c_bool]
        L.ora_calcmoments.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int, P, P, C.c_bool,
                                      C.c_bool]
        L.ora_groupquantile.restype = P
        L.ora_groupquantile.argtypes = [P, P, P, P, C.c_double, C.c_bool, C.c_bool]
        L.ora_thetajoin.argtypes = [C.POINTER(P), C.POINTER(P), P, P, P, P, C.c_int, C.c_bool]
        L.ora_bandjoin.argtypes = [C.POINTER(P), C.POINTER(P), P, P, P, P, C.c_void_p, C.c_void_p, C.c_bool,
                                   C.c_bool]
        L.ora_rangejoin.argtypes = [C.POINTER(P), C.POINTER(P), P, P, P, P, P, C.c_bool, C.c_bool, C.c_bool,
                                    C.c_bool]
        L.ora_semijoin_cands.restype = P
        L.ora_semijoin_cands.argtypes = [P, P, P, P, C.c_bool, C.c_bool, C.c_bool, C.c_bool]
        L.ora_leftjoin.argtypes = [C.POINTER(P), C.POINTER(P), P, P, P, P, C.c_bool, C.c_bool, C.c_bool]
        L.ora_markjoin.argtypes = [C.POINTER(P), C.POINTER(P), C.POINTER(P), P, P, P, P]
        L.ora_count_no_nil.argtypes = [P, P]
        L.ora_guess_uniques.argtypes = [P, P]
        L.ora_guess_uniques.restype = C.c_uint64
        L.ora_count_no_nil.restype = C.c_uint64
        L.ora_crossproduct.argtypes = [C.POINTER(P), C.POINTER(P), P, P, P, P, C.c_bool, C.c_bool]
        L.ora_minmax.argtypes = [P, C.c_bool, C.c_bool, C.c_void_p, C.POINTER(C.c_char_p)]
        L.ora_prod.argtypes = [C.c_void_p, C.c_int, P, P, C.c_bool, C.c_bool]
        L.ora_groupprod.restype = P
        L.ora_groupprod.argtypes = [P, P, P, P, C.c_int, C.c_bool]
        L.ora_calcavg.argtypes = [P, P, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_int]
        L.ora_leftjoin_ex.argtypes = [C.POINTER(P), C.POINTER(P), C.POINTER(P), P, P, P, P, C.c_bool, C.c_bool,
                                      C.c_bool, C.c_bool, C.c_bool, C.POINTER(C.c_int)]
        L.ora_join_algo.argtypes = [P, P, P, P]
        L.ora_BATsort.argtypes = [C.POINTER(P), C.POINTER(P), C.POINTER(P), P, P, P, C.c_bool, C.c_bool,
                                  C.c_bool]
        L.ora_GDKqsort.argtypes = [P, C.c_void_p, C.c_void_p, C.c_uint64, C.c_bool, C.c_bool]
        L.ora_firstn.restype = P
        L.ora_firstn.argtypes = [P, P, P, C.c_uint64, C.c_bool, C.c_bool]
        L.ora_windowbounds.argtypes = [P, P, P, P, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_bool,
                                       C.c_uint64]
        L.ora_analyticalsum.argtypes = [P, P, P, P, P, P, C.c_int, C.c_int, C.c_int]
        L.ora_analyticalavg.argtypes = [P, P, P, P, P, P, C.c_int, C.c_int]
        L.ora_analyticalavginteger.argtypes = [P, P, P, P, P, P, C.c_int, C.c_int]
        L.ora_analyticalstat.argtypes = [P, P, P, P, P, P, P, C.c_int, C.c_int, C.c_int]
        L.ora_analyticalprod.argtypes = [P, P, P, P, P, P, C.c_int, C.c_int]
        L.ora_analyticalcount.argtypes = [P, P, P, P, P, P, C.c_bool, C.c_int]
        L.ora_analyticalntile.argtypes = [P, P, P, P, C.c_int, C.c_void_p]
        L.ora_analyticalfirst.argtypes = [P, P, P, P, C.c_int]
        L.ora_analyticallast.argtypes = [P, P, P, P, C.c_int]
        L.ora_analyticalnthvalue.argtypes = [P, P, P, P, P, C.c_void_p, C.c_int]
        L.ora_analyticallag.argtypes = [P, P, P, C.c_uint64, C.c_void_p, C.c_int]
        L.ora_analyticallead.argtypes = [P, P, P, C.c_uint64, C.c_void_p, C.c_int]
        L.ora_analyticalmin.argtypes = [P, P, P, P, P, P, C.c_int, C.c_int]
        L.ora_analyticaldiff.argtypes = [P, P, P, C.c_void_p, C.c_int]
        L.ora_analyticalmax.argtypes = [P, P, P, P, P, P, C.c_int, C.c_int]
        L.ora_tpch_lineitem.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64] + [C.c_void_p] * 7
        L.ora_mkdate.restype = C.c_int32
        L.ora_mkdate.argtypes = [C.c_int, C.c_int, C.c_int]
        L.ora_q6.argtypes = [C.POINTER(OraLineitem), C.c_int, C.c_void_p]
        L.ora_q1.argtypes = [C.POINTER(OraLineitem), C.c_int, C.POINTER(OraQ1Row), C.POINTER(C.c_int)]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    pass


def _err():
    return OracleError(lib().ora_errbuf().decode())


def hge_to_int(words):
    lo, hi = int(words[0]), int(words[1])
    v = (hi << 64) | lo
    return v - (1 << 128) if v >= (1 << 127) else v


def int_to_hge_words(v):
    v &= (1 << 128) - 1
    return v & ((1 << 64) - 1), v >> 64


class Bat:
    """Python-side holder of an ora_bat; keeps numpy buffers alive."""

    def __init__(self, ptr=None, keep=None):
        self.ptr = ptr
        self.keep = keep or []
        self.owned = ptr is not None and keep is None

    @classmethod
    def from_array(cls, tp, arr, hseqbase=0, sorted_=False, revsorted=False, key=False,
                   nonil=False, vheap=None, tseqbase=OID_NIL, unique_est=0.0):
        if tp == TYPE_hge:
            a = np.ascontiguousarray(arr, dtype=np.uint64).reshape(-1, 2)
        elif tp == TYPE_str:
            # heap offsets of 1, 2, 4 or 8 bytes (the width follows the array)
            a = np.ascontiguousarray(arr)
            if a.dtype not in (np.uint8, np.uint16, np.uint32, np.uint64):
                a = a.astype(np.uint8)
        else:
            a = np.ascontiguousarray(arr, dtype=NP[tp])
        n = a.shape[0]
        b = OraBat()
        b.type = tp
        b.width = 16 if tp == TYPE_hge else a.dtype.itemsize
        b.count = n
        b.hseqbase = hseqbase
        b.tseqbase = tseqbase
        b.unique_est = unique_est
        b.minpos = b.maxpos = (1 << 63) - 1
        b.base = a.ctypes.data if n else a.ctypes.data
        keep = [a, b]
        if vheap is not None:
            vh = np.frombuffer(vheap, dtype=np.uint8).copy()
            b.vheap = vh.ctypes.data
            b.vheapsize = vh.size
            keep.append(vh)
        b.sorted, b.revsorted, b.key, b.nonil = sorted_, revsorted, key, nonil
        return cls(C.pointer(b), keep)

    @classmethod
    def msk(cls, bits, hseqbase=0):
        """A msk BAT: one bit per row in 32-bit words, count = len(bits)."""
        bits = np.asarray(bits, bool)
        n = bits.size
        a = np.packbits(np.concatenate([bits, np.zeros((-n) % 32 + 32, bool)]),
                        bitorder="little").view(np.uint32).copy()
        b = OraBat()
        b.type = TYPE_msk
        b.width = 4
        b.count = n
        b.hseqbase = hseqbase
        b.tseqbase = OID_NIL
        b.base = a.ctypes.data
        b.minpos = b.maxpos = (1 << 63) - 1
        return cls(C.pointer(b), [a, b])

    @classmethod
    def dense(cls, tseq, n, hseqbase=0):
        b = OraBat()
        b.type = TYPE_void
        b.count = n
        b.hseqbase = hseqbase
        b.tseqbase = tseq
        b.sorted = b.key = b.nonil = 1
        b.revsorted = n <= 1
        b.minpos = b.maxpos = (1 << 63) - 1
        return cls(C.pointer(b), [b])

    @property
    def s(self):
        return self.ptr.contents

    def count(self):
        return self.s.count

    def values(self):
        b = self.s
        if b.type == TYPE_void:
            return np.arange(b.tseqbase, b.tseqbase + b.count, dtype=np.uint64)
        if b.type == TYPE_hge:
            raw = np.ctypeslib.as_array(C.cast(b.base, C.POINTER(C.c_uint64)), (b.count * 2,)) \
                if b.count else np.zeros(0, np.uint64)
            return [hge_to_int(raw[2 * i:2 * i + 2]) for i in range(b.count)]
        if b.count == 0:
            return np.zeros(0, NP[b.type])
        ct = CT.get(b.type, C.c_uint8)
        return np.ctypeslib.as_array(C.cast(b.base, C.POINTER(ct)), (b.count,)).copy()

    def __del__(self):
        if self.owned and self.ptr is not None:
            lib().ora_free(self.ptr)
            self.ptr = None


def _valptr(tp, v, keep):
    if v is None:
        return None
    if tp == TYPE_str:
        # a C string (bytes or str); b"\x80" is str nil
        buf = C.create_string_buffer(v if isinstance(v, bytes) else v.encode())
        keep.append(buf)
        return C.cast(buf, C.c_void_p)
    if tp == TYPE_hge:
        buf = (C.c_uint64 * 2)(*int_to_hge_words(v))
    elif tp == TYPE_void:
        buf = C.c_uint64(v)
    else:
        buf = CT[tp](v)
    keep.append(buf)
    return C.cast(C.pointer(buf), C.c_void_p)


def _ret(p):
    if not p:
        raise _err()
    return Bat(p)


def BATselect(b, s, tl, th, li, hi, anti, nil_matches=False):
    keep = []
    tp = b.s.type
    return _ret(lib().ora_select(b.ptr, s.ptr if s else None, _valptr(tp, tl, keep),
                                 _valptr(tp, th, keep), li, hi, anti, nil_matches))


def unmask(b):
    return _ret(lib().ora_unmask(b.ptr))


def maskedcands(hseq, nr, masked, selected=True):
    return _ret(lib().ora_maskedcands(hseq, nr, masked.ptr, selected))


def mergecand(a, b):
    return _ret(lib().ora_mergecand(a.ptr, b.ptr))


def intersectcand(a, b):
    return _ret(lib().ora_intersectcand(a.ptr, b.ptr))


def diffcand(a, b):
    return _ret(lib().ora_diffcand(a.ptr, b.ptr))


def negcands(tseq, nr, odels):
    return _ret(lib().ora_negcands(tseq, nr, odels.ptr))


def BATthetaselect(b, s, val, op):
    keep = []
    return _ret(lib().ora_thetaselect(b.ptr, s.ptr if s else None,
                                      _valptr(b.s.type, val, keep), op.encode()))


def BATproject(l, r):
    return _ret(lib().ora_project(l.ptr, r.ptr))


def BATcalc(op, b1, b2, tp, s=None, c1=None, t1=0, c2=None, t2=0):
    keep = []
    return _ret(lib().ora_calc(op.encode(), b1.ptr if b1 else None, _valptr(t1, c1, keep), t1,
                               b2.ptr if b2 else None, _valptr(t2, c2, keep), t2,
                               s.ptr if s else None, tp))


CMP_OPS = {"<": 0, "<=": 1, ">": 2, ">=": 3, "==": 4, "!=": 5, "cmp": 6}


def _pp(b):
    return b.ptr if b is not None else None


def BATcalccmp(op, b1, b2, s1=None, s2=None, c1=None, t1=0, c2=None, t2=0, nil_matches=False):
    """op in CMP_OPS; b1 / b2 None: the constant c1 / c2 of type t1 / t2"""
    keep = []
    return _ret(lib().ora_calccmp(CMP_OPS[op], _pp(b1), _valptr(t1, c1, keep), t1, _pp(b2),
                                  _valptr(t2, c2, keep), t2, _pp(s1), _pp(s2), nil_matches))


XOPS = {"negate": 0, "absolute": 1, "iszero": 2, "sign": 3, "isnil": 4, "isnotnil": 5, "min": 6, "max": 7,
        "min_no_nil": 8, "max_no_nil": 9, "and": 10, "or": 11, "xor": 12, "lsh": 13, "rsh": 14}


def BATcalcunary(name, b, s=None):
    """gdk_calc.c:233-920 (ora_calcunary)"""
    return _ret(lib().ora_calcunary(XOPS[name], b.ptr, _pp(s)))


def BATcalcminmax(name, b1, b2=None, s1=None, s2=None, c=None, ct=0):
    """gdk_calc.c:976-2436 min / max / _no_nil; b2 None: the constant c"""
    keep = []
    return _ret(lib().ora_calcminmax(XOPS[name], b1.ptr, _pp(b2), _valptr(ct, c, keep), ct, _pp(s1), _pp(s2)))


def BATcalcbits(name, fname, b1=None, b2=None, s1=None, s2=None, c1=None, t1=0, c2=None, t2=0):
    """gdk_calc.c:2439-3760 and / or / xor / lsh / rsh; None BAT: the constant"""
    keep = []
    return _ret(lib().ora_calcbits(XOPS[name], fname.encode(), _pp(b1), _valptr(t1, c1, keep), t1, _pp(b2),
                                   _valptr(t2, c2, keep), t2, _pp(s1), _pp(s2)))


def BATcalcifthenelse(b, b1=None, b2=None, c1=None, c2=None, ct=0):
    """gdk_calc.c:4376 ifthenelse; None BAT: the constant of type ct"""
    keep = []
    return _ret(lib().ora_calcifthenelse(b.ptr, _pp(b1), _valptr(ct, c1, keep), _pp(b2), _valptr(ct, c2, keep), ct))


def BATcalcbetween(b, lo, hi, s=None, slo=None, shi=None, clo=None, chi=None, ct=0,
                   symmetric=False, linc=True, hinc=True, nils_false=False, anti=False):
    keep = []
    return _ret(lib().ora_calcbetween(b.ptr, _pp(lo), _valptr(ct, clo, keep), _pp(hi),
                                      _valptr(ct, chi, keep), ct, _pp(s), _pp(slo), _pp(shi),
                                      symmetric, linc, hinc, nils_false, anti))


def BATconvert(b, s, tp, scale1=0, scale2=0, precision=0):
    return _ret(lib().ora_convert(b.ptr, _pp(s), tp, scale1, scale2, precision))


def BATcalcnot(b, s=None):
    return _ret(lib().ora_calcnot(b.ptr, _pp(s)))


def BATcalcdivmod(op, b1, b2, tp, s1=None, s2=None, c1=None, t1=0, c2=None, t2=0):
    keep = []
    return _ret(lib().ora_calcdivmod(op.encode(), _pp(b1), _valptr(t1, c1, keep), t1, _pp(b2),
                                     _valptr(t2, c2, keep), t2, _pp(s1), _pp(s2), tp))


def BATsum(tp, b, s=None, skip_nils=True, nil_if_empty=True):
    buf = (C.c_uint64 * 2)()
    if lib().ora_sum(C.cast(buf, C.c_void_p), tp, b.ptr, s.ptr if s else None,
                     skip_nils, nil_if_empty) < 0:
        raise _err()
    if tp == TYPE_hge:
        return hge_to_int(buf)
    if tp == TYPE_dbl:
        return C.cast(buf, C.POINTER(C.c_double))[0]
    return C.cast(buf, C.POINTER(CT[tp]))[0]


def _scalar(tp, buf):
    if tp == TYPE_hge:
        return hge_to_int(buf)
    return C.cast(buf, C.POINTER(CT[TYPE_oid if tp == TYPE_void else tp]))[0]


def BATminmax(b, skipnil=True, domax=False):
    """BATmin_skipnil / BATmax_skipnil (gdk_aggr.c:3570, :3727); str as bytes"""
    buf = (C.c_uint64 * 2)()
    sp = C.c_char_p()
    if lib().ora_minmax(b.ptr, skipnil, domax, C.cast(buf, C.c_void_p), C.byref(sp)) < 0:
        raise _err()
    if b.s.type == TYPE_str:
        return sp.value
    return _scalar(b.s.type, buf)


def BATprod(tp, b, s=None, skip_nils=True, nil_if_empty=True):
    """BATprod (gdk_aggr.c:1650)"""
    buf = (C.c_uint64 * 2)()
    if lib().ora_prod(C.cast(buf, C.c_void_p), tp, b.ptr, s.ptr if s else None, skip_nils, nil_if_empty) < 0:
        raise _err()
    return _scalar(tp, buf)


def BATgroupprod(b, g, e, tp, skip_nils=True, s=None):
    """BATgroupprod (gdk_aggr.c:1575)"""
    return _ret(lib().ora_groupprod(b.ptr, g.ptr, e.ptr if e else None, s.ptr if s else None, tp, skip_nils))


def BATgroup(b, s=None, g=None):
    gp, ep, hp = P(), P(), P()
    if lib().ora_group(C.byref(gp), C.byref(ep), C.byref(hp), b.ptr, s.ptr if s else None,
                       g.ptr if g else None) < 0:
        raise _err()
    return Bat(gp), Bat(ep), Bat(hp)


def BATgroupsum(b, g, e, tp, skip_nils=True, s=None):
    return _ret(lib().ora_groupsum(b.ptr, g.ptr, e.ptr if e else None, s.ptr if s else None,
                                   tp, skip_nils))


def BATgroupcount(b, g, e, skip_nils=True, s=None):
    return _ret(lib().ora_groupcount(b.ptr, g.ptr, e.ptr if e else None, s.ptr if s else None,
                                     skip_nils))


def BATgroupminmax(b, g, e, domax, skip_nils=True, s=None):
    return _ret(lib().ora_groupminmax(b.ptr, g.ptr, e.ptr if e else None,
                                      s.ptr if s else None, skip_nils, domax))


_ST = {"stdev": 0, "variance": 0, "covariance": 1, "correlation": 2}


def BATgroupstat(name, b1, b2, g, e, skip_nils=True, s=None, sample=True):
    """the grouped statistics of gdk_aggr.c:4612-5202: name one of stdev,
    variance, covariance, correlation (b2 for the two-column ones)"""
    return _ret(lib().ora_groupmoments(_ST[name], b1.ptr, b2.ptr if b2 else None, g.ptr if g else None,
                                       e.ptr if e else None, s.ptr if s else None, skip_nils,
                                       sample and name != "correlation", name == "variance"))


def BATcalcstat(name, b1, b2=None, sample=True):
    """calcvariance / calccovariance / BATcalccorrelation (gdk_aggr.c:4276-4559):
    (value, average) -- NaN is nil"""
    r, a = C.c_double(), C.c_double()
    if lib().ora_calcmoments(C.byref(r), C.byref(a), _ST[name], b1.ptr, b2.ptr if b2 else None,
                             sample and name != "correlation", name == "variance") < 0:
        raise _err()
    return r.value, a.value


def BATgroupquantile(b, g, e, quantile, skip_nils=True, s=None, average=False):
    """doBATgroupquantile (gdk_aggr.c:3881); g may be None"""
    return _ret(lib().ora_groupquantile(b.ptr, g.ptr if g else None, e.ptr if e else None,
                                        s.ptr if s else None, quantile, skip_nils, average))


def BATcalcavg(b, s=None, scale=0):
    """gdk_aggr.c:2987: (average or NaN, number of non-nil values)"""
    a, n = C.c_double(), C.c_uint64()
    if lib().ora_calcavg(b.ptr, s.ptr if s else None, C.byref(a), C.byref(n), scale) < 0:
        raise _err()
    return a.value, n.value


def BATgroupavg(b, g, e, skip_nils=True, s=None, scale=0, want_counts=True):
    a, c = P(), P()
    if lib().ora_groupavg(C.byref(a), C.byref(c) if want_counts else None, b.ptr, g.ptr,
                          e.ptr if e else None, s.ptr if s else None, skip_nils, scale) < 0:
        raise _err()
    return Bat(a), (Bat(c) if want_counts else None)


def BATgroupavg3combine(avg, rem, cnt, g, e, skip_nils=True):
    return _ret(lib().ora_groupavg3combine(avg.ptr, rem.ptr, cnt.ptr, g.ptr if g else None,
                                           e.ptr if e else None, skip_nils))


def BATgroupavg3(b, g, e, skip_nils=True, s=None):
    a, r, c = P(), P(), P()
    if lib().ora_groupavg3(C.byref(a), C.byref(r), C.byref(c), b.ptr, g.ptr,
                           e.ptr if e else None, s.ptr if s else None, skip_nils) < 0:
        raise _err()
    return Bat(a), Bat(r), Bat(c)


def BATjoin(l, r, sl=None, sr=None, nil_matches=False):
    a, b = P(), P()
    if lib().ora_join(C.byref(a), C.byref(b), l.ptr, r.ptr, sl.ptr if sl else None,
                      sr.ptr if sr else None, nil_matches) < 0:
        raise _err()
    return Bat(a), Bat(b)


def BATguess_uniques(b, s=None):
    """gdk_join.c:3572 (records tunique_est on b for a full column)"""
    return int(lib().ora_guess_uniques(b.ptr, s.ptr if s else None))


def BATcount_no_nil(b, s=None):
    """gdk_batop.c:3078"""
    return int(lib().ora_count_no_nil(b.ptr, s.ptr if s else None))


def crossproduct(l, r, sl=None, sr=None, max_one=False, outer=False, want_r2=True):
    """BATsubcross (gdk_cross.c:138) / BAToutercross (:153)"""
    a, b = P(), P()
    if lib().ora_crossproduct(C.byref(a), C.byref(b) if want_r2 else None, l.ptr, r.ptr,
                              sl.ptr if sl else None, sr.ptr if sr else None, max_one, outer) < 0:
        raise _err()
    return (Bat(a), Bat(b)) if want_r2 else Bat(a)


def BATmarkjoin(l, r, sl=None, sr=None, want_r2=True):
    """BATmarkjoin (gdk_join.c:4367): (r1, r2, r3) or, without r2 (semi),
    (r1, r3); None when r2 is wanted and a left candidate matches twice"""
    a, b, c = P(), P(), P()
    rc = lib().ora_markjoin(C.byref(a), C.byref(b) if want_r2 else None, C.byref(c), l.ptr, r.ptr,
                            sl.ptr if sl else None, sr.ptr if sr else None)
    if rc == -2:
        return None
    if rc < 0:
        raise _err()
    return (Bat(a), Bat(b), Bat(c)) if want_r2 else (Bat(a), Bat(c))


_THETA_MASK = {-1: 2, -2: 3, 1: 4, 2: 5, -3: 6}


def BATthetajoin(l, r, sl=None, sr=None, op=-1, nil_matches=False):
    """gdk_join.c:4409 / thetajoin :3699 (op as JOIN_LT -1 ... JOIN_NE -3)"""
    a, b = P(), P()
    if lib().ora_thetajoin(C.byref(a), C.byref(b), l.ptr, r.ptr, sl.ptr if sl else None, sr.ptr if sr else None,
                           _THETA_MASK[op], nil_matches) < 0:
        raise _err()
    return Bat(a), Bat(b)


def BATbandjoin(l, r, c1, c2, sl=None, sr=None, linc=True, hinc=True):
    """gdk_join.c:4626"""
    ct = CT[l.s.type]
    v1, v2 = ct(c1), ct(c2)
    a, b = P(), P()
    if lib().ora_bandjoin(C.byref(a), C.byref(b), l.ptr, r.ptr, sl.ptr if sl else None, sr.ptr if sr else None,
                          C.cast(C.pointer(v1), C.c_void_p), C.cast(C.pointer(v2), C.c_void_p), linc, hinc) < 0:
        raise _err()
    return Bat(a), Bat(b)


def BATrangejoin(l, rl, rh, sl=None, sr=None, linc=True, hinc=True, anti=False, symmetric=False):
    """gdk_join.c:5422 / rangejoin :5067"""
    a, b = P(), P()
    if lib().ora_rangejoin(C.byref(a), C.byref(b), l.ptr, rl.ptr, rh.ptr, sl.ptr if sl else None,
                           sr.ptr if sr else None, linc, hinc, anti, symmetric) < 0:
        raise _err()
    return Bat(a), Bat(b)


def BATintersect(l, r, sl=None, sr=None, nil_matches=False, max_one=False):
    """gdk_join.c:4366: the left candidates whose value occurs on the right"""
    return _ret(lib().ora_semijoin_cands(l.ptr, r.ptr, sl.ptr if sl else None, sr.ptr if sr else None,
                                         nil_matches, max_one, False, False))


def BATdiff(l, r, sl=None, sr=None, nil_matches=False, not_in=False):
    """gdk_join.c:4388: the left candidates whose value does not occur on the right"""
    return _ret(lib().ora_semijoin_cands(l.ptr, r.ptr, sl.ptr if sl else None, sr.ptr if sr else None,
                                         nil_matches, False, True, not_in))


def BATleftjoin(l, r, sl=None, sr=None, nil_matches=False, outer=False, match_one=False):
    """BATleftjoin / BATouterjoin (gdk_join.c:4320, :4334) with at most one
    match per left candidate; None when a candidate matches twice"""
    a, b = P(), P()
    rc = lib().ora_leftjoin(C.byref(a), C.byref(b), l.ptr, r.ptr, sl.ptr if sl else None,
                            sr.ptr if sr else None, nil_matches, outer, match_one)
    if rc == -2:
        return None
    if rc < 0:
        raise _err()
    return Bat(a), Bat(b)


LJ_ALGOS = ["nomatch", "selectjoin", "mergejoin_void", "fetchjoin", "bitmaskjoin", "mergejoin",
            "hashjoin_swapped", "hashjoin"]


def leftjoin_ex(l, r, sl=None, sr=None, nil_matches=False, nil_on_miss=False, semi=False, max_one=False,
                min_one=False, want_r2=True, want_r3=False):
    """leftjoin (gdk_join.c:4049) with the reference's algorithm choice and
    the order of several matches per left candidate (gdk_oracle_join.c):
    (r1, r2 or None, r3 or None, algorithm name)"""
    a, b, c = P(), P(), P()
    al = C.c_int(-1)
    if lib().ora_leftjoin_ex(C.byref(a), C.byref(b) if want_r2 else None, C.byref(c) if want_r3 else None,
                             l.ptr, r.ptr, sl.ptr if sl else None, sr.ptr if sr else None, nil_matches,
                             nil_on_miss, semi, max_one, min_one, C.byref(al)) < 0:
        raise _err()
    return Bat(a), (Bat(b) if want_r2 else None), (Bat(c) if want_r3 else None), LJ_ALGOS[al.value]


JOIN_ALGOS = ["nomatch", "selectjoin", "selectjoin_swapped", "mergejoin_void", "mergejoin_void_swapped",
              "mergejoin_sorted", "mergejoin", "mergejoin_swapped", "hashjoin_swapped", "hashjoin"]


def join_algo(l, r, sl=None, sr=None):
    """Name of the algorithm BATjoin(l, r, sl, sr) takes (gdk_join.c:4542-4618)."""
    k = lib().ora_join_algo(l.ptr, r.ptr, sl.ptr if sl else None, sr.ptr if sr else None)
    if k < 0:
        raise _err()
    return JOIN_ALGOS[k]


def props(b):
    """The result properties a parity test compares (gdk/gdk.h:712-740)."""
    s = b.s
    return dict(type="void" if s.type == TYPE_void else "oid" if s.type == TYPE_oid else s.type,
                count=s.count, tseqbase=s.tseqbase, sorted=bool(s.sorted), revsorted=bool(s.revsorted),
                key=bool(s.key), nonil=bool(s.nonil), nil=bool(s.nil))


def BATsort(b, reverse=False, nilslast=False, stable=None):
    """(sorted, order) of BATsort without o / g; stable unless the nil
    placement asks for an unstable sort (reverse != nilslast)"""
    s, o, _ = BATsort_full(b, reverse=reverse, nilslast=nilslast,
                           stable=(reverse == nilslast) if stable is None else stable, want_groups=False)
    return s, o


def BATsort_full(b, o=None, g=None, reverse=False, nilslast=False, stable=True, want_groups=True):
    """BATsort(&sorted, &order, &groups, b, o, g, reverse, nilslast, stable)
    (gdk/gdk_batop.c:2342) with do_sort's choice per run, GDKqsort included
    (gdk_oracle_sort.c).  Returns (sorted, order, groups or None)."""
    a, od, gp = P(), P(), P()
    if lib().ora_BATsort(C.byref(a), C.byref(od), C.byref(gp) if want_groups else None, b.ptr,
                         o.ptr if o else None, g.ptr if g else None, reverse, nilslast, stable) < 0:
        raise _err()
    return Bat(a), Bat(od), (Bat(gp) if want_groups else None)


def GDKqsort(b, reverse=False, nilslast=False):
    """GDKqsort (gdk/gdk_qsort.c:358) of b's values with positions as payload:
    returns the permutation (positions in sorted order)."""
    n = b.s.count
    h = np.arange(n, dtype=np.uint64)
    t = np.arange(n, dtype=np.uint64)
    lib().ora_GDKqsort(b.ptr, h.ctypes.data, t.ctypes.data, n, reverse, nilslast)
    assert np.array_equal(h, t)
    return h


def BATfirstn(b, n, s=None, g=None, asc=True, nilslast=False):
    """BATfirstn(&topn, NULL, b, s, g, n, asc, nilslast, false)"""
    return _ret(lib().ora_firstn(b.ptr, s.ptr if s else None, g.ptr if g else None, n, asc, nilslast))


def windowbounds(b, p, l, bound, tp1, tp2, unit, preceding, second_half=0):
    """GDKanalyticalwindowbounds(r, b, p, l, bound, tp1, tp2, unit, preceding,
    second_half) (gdk/gdk_analytic_bounds.c:1440); `bound` is the static
    limit as a Python value of type tp2 (None when the per-row BAT l is
    given).  Returns the bounds BAT (with the nonil / nil properties the
    reference sets)."""
    n = b.count()
    r = lib().ora_new(TYPE_oid, n, 0)
    keep = []
    bp = _valptr(tp2, bound, keep) if l is None else None
    if lib().ora_windowbounds(r, b.ptr, p.ptr if p else None, l.ptr if l else None, bp, tp1, tp2, unit,
                              preceding, second_half) < 0:
        lib().ora_free(r)
        raise _err()
    return Bat(r)


def rangebounds(b, p, limit, preceding):
    return windowbounds(b, p, None, limit, b.s.type, TYPE_lng, 1, preceding)


def analyticalsum(b, p, o, s, e, tp2, frame_type):
    n = b.count()
    r = lib().ora_new(tp2, n, 0)
    if lib().ora_analyticalsum(r, p.ptr if p else None, o.ptr if o else None, b.ptr,
                               s.ptr if s else None, e.ptr if e else None, b.s.type, tp2,
                               frame_type) < 0:
        lib().ora_free(r)
        raise _err()
    return Bat(r)


def analyticalavg(b, p, o, s, e, frame_type):
    r = lib().ora_new(TYPE_dbl, b.count(), 0)
    if lib().ora_analyticalavg(r, p.ptr if p else None, o.ptr if o else None, b.ptr,
                               s.ptr if s else None, e.ptr if e else None, b.s.type,
                               frame_type) < 0:
        lib().ora_free(r)
        raise _err()
    return Bat(r)


# GDKanalytical_<name> (gdk_analytic_statistics.c:962-1443): (kind, op)
WIN_STATS = {"stddev_samp": (0, 0), "stddev_pop": (0, 1), "variance_samp": (0, 2), "variance_pop": (0, 3),
             "covariance_samp": (1, 0), "covariance_pop": (1, 1), "correlation": (2, 0)}


def analyticalstat(name, b1, b2, p, o, s, e, frame_type):
    kind, op = WIN_STATS[name]
    r = lib().ora_new(TYPE_dbl, b1.count(), 0)
    if lib().ora_analyticalstat(r, p.ptr if p else None, o.ptr if o else None, b1.ptr, b2.ptr if b2 else None,
                                s.ptr if s else None, e.ptr if e else None, kind, op, frame_type) < 0:
        lib().ora_free(r)
        raise _err()
    return Bat(r)


def analyticalprod(b, p, o, s, e, tp2, frame_type):
    r = lib().ora_new(tp2, b.count(), 0)
    if lib().ora_analyticalprod(r, p.ptr if p else None, o.ptr if o else None, b.ptr,
                                s.ptr if s else None, e.ptr if e else None, tp2, frame_type) < 0:
        lib().ora_free(r)
        raise _err()
    return Bat(r)


def analyticalavginteger(b, p, o, s, e, frame_type):
    r = lib().ora_new(b.s.type, b.count(), 0)
    if lib().ora_analyticalavginteger(r, p.ptr if p else None, o.ptr if o else None, b.ptr,
                                      s.ptr if s else None, e.ptr if e else None, b.s.type,
                                      frame_type) < 0:
        lib().ora_free(r)
        raise _err()
    return Bat(r)


def analyticalcount(b, p, o, s, e, ignore_nils, frame_type):
    n = b.count()
    r = lib().ora_new(TYPE_lng, n, 0)
    if lib().ora_analyticalcount(r, p.ptr if p else None, o.ptr if o else None, b.ptr,
                                 s.ptr if s else None, e.ptr if e else None, ignore_nils,
                                 frame_type) < 0:
        lib().ora_free(r)
        raise _err()
    return Bat(r)


def mkdate(y, m, d):
    return lib().ora_mkdate(y, m, d)


def tpch_lineitem(seed, row0, n, sf_parts):
    cols = dict(shipdate=np.empty(n, np.int32), quantity=np.empty(n, np.int64),
                extendedprice=np.empty(n, np.int64), discount=np.empty(n, np.int64),
                tax=np.empty(n, np.int64), returnflag=np.empty(n, np.uint8),
                linestatus=np.empty(n, np.uint8))
    lib().ora_tpch_lineitem(seed, row0, n, sf_parts,
                            *[cols[k].ctypes.data for k in ("shipdate", "quantity",
                                                            "extendedprice", "discount", "tax",
                                                            "returnflag", "linestatus")])
    return cols


def _li(cols):
    li = OraLineitem()
    li.n = cols["shipdate"].shape[0]
    for k in ("shipdate", "quantity", "extendedprice", "discount", "tax", "returnflag",
              "linestatus"):
        setattr(li, k, cols[k].ctypes.data)
    return li


def q6(cols, nthreads=1):
    out = (C.c_uint64 * 2)()
    li = _li(cols)
    if lib().ora_q6(C.byref(li), nthreads, C.cast(out, C.c_void_p)) < 0:
        raise _err()
    return hge_to_int(out)


def q1(cols, nthreads=1):
    rows = (OraQ1Row * 16)()
    n = C.c_int()
    li = _li(cols)
    if lib().ora_q1(C.byref(li), nthreads, rows, C.byref(n)) < 0:
        raise _err()
    res = []
    for i in range(n.value):
        r = rows[i]
        res.append(dict(returnflag=r.returnflag, linestatus=r.linestatus,
                        sum_qty=hge_to_int(r.sum_qty), sum_base_price=hge_to_int(r.sum_base_price),
                        sum_disc_price=hge_to_int(r.sum_disc_price),
                        sum_charge=hge_to_int(r.sum_charge),
                        avg_qty=r.avg_qty, avg_price=r.avg_price, avg_disc=r.avg_disc,
                        rem_qty=r.rem_qty, rem_price=r.rem_price, rem_disc=r.rem_disc,
                        count_order=r.count_order))
    return res


# ---- window functions (gdk_oracle_window.c) --------------------------------
BUN_NONE = (1 << 63) - 1


def _wrun(tp, n, fn, *args):
    r = lib().ora_new(tp, n, 0)
    if fn(r, *args) < 0:
        lib().ora_free(r)
        raise _err()
    return Bat(r)


def _pp(b):
    return b.ptr if b is not None else None


def analyticalntile(b, p, n=None, ntile=None, tpe=None):
    """GDKanalyticalntile: n a BAT of per-row tile counts, or ntile a scalar of tpe."""
    keep = []
    tpe = tpe if tpe is not None else n.s.type
    return _wrun(tpe, b.count(), lib().ora_analyticalntile, b.ptr, _pp(p), _pp(n), tpe,
                 _valptr(tpe, ntile, keep) if n is None else None)


def analyticalfirst(b, s, e):
    return _wrun(b.s.type, b.count(), lib().ora_analyticalfirst, b.ptr, s.ptr, e.ptr, b.s.type)


def analyticallast(b, s, e):
    return _wrun(b.s.type, b.count(), lib().ora_analyticallast, b.ptr, s.ptr, e.ptr, b.s.type)


def analyticalnthvalue(b, s, e, t=None, nth=None):
    ref = C.c_int64(nth) if t is None else None
    return _wrun(b.s.type, b.count(), lib().ora_analyticalnthvalue, b.ptr, s.ptr, e.ptr, _pp(t),
                 C.cast(C.pointer(ref), C.c_void_p) if ref is not None else None, b.s.type)


def analyticallag(b, p, lag, default):
    keep = []
    return _wrun(b.s.type, b.count(), lib().ora_analyticallag, b.ptr, _pp(p), lag,
                 _valptr(b.s.type, default, keep), b.s.type)


def analyticallead(b, p, lead, default):
    keep = []
    return _wrun(b.s.type, b.count(), lib().ora_analyticallead, b.ptr, _pp(p), lead,
                 _valptr(b.s.type, default, keep), b.s.type)


def analyticalmin(b, p, o, s, e, frame_type):
    return _wrun(b.s.type, b.count(), lib().ora_analyticalmin, _pp(p), _pp(o), b.ptr, _pp(s), _pp(e),
                 b.s.type, frame_type)


def analyticalmax(b, p, o, s, e, frame_type):
    return _wrun(b.s.type, b.count(), lib().ora_analyticalmax, _pp(p), _pp(o), b.ptr, _pp(s), _pp(e),
                 b.s.type, frame_type)


def analyticaldiff(b, p=None, npbit=None):
    ref = C.c_int8(npbit) if npbit is not None else None
    return _wrun(TYPE_bit, b.count(), lib().ora_analyticaldiff, b.ptr, _pp(p),
                 C.cast(C.pointer(ref), C.c_void_p) if ref is not None else None, b.s.type)
