"""Host-side mirror of the GDK operator interface over libmgdk.so.

Same names and argument meaning as the reference's C functions
(gdk/gdk.h:1447,1526,2245-2275, gdk/gdk_calc.h, gdk/gdk_analytic.h); errors
raise GDKError carrying the reference's SQLSTATE-prefixed message (the
C functions return NULL/GDK_FAIL and set GDKerrbuf).  There is no CPU
fallback: if libmgdk.so is missing or no GPU is present, calls fail loudly.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MGDK_LIB") or os.path.join(HERE, "libmgdk.so")

TYPE_void, TYPE_msk, TYPE_bit, TYPE_bte, TYPE_sht, TYPE_int, TYPE_oid = 0, 1, 2, 3, 4, 5, 6
TYPE_flt, TYPE_dbl, TYPE_lng, TYPE_hge, TYPE_date, TYPE_str = 8, 9, 10, 11, 12, 16
TYPE_daytime, TYPE_timestamp = 13, 14
OID_NIL = 1 << 63

NP = {TYPE_bit: np.int8, TYPE_bte: np.int8, TYPE_sht: np.int16, TYPE_int: np.int32,
      TYPE_date: np.int32, TYPE_oid: np.uint64, TYPE_lng: np.int64, TYPE_flt: np.float32,
      TYPE_dbl: np.float64, TYPE_str: np.uint8, TYPE_daytime: np.int64, TYPE_timestamp: np.int64}
CT = {TYPE_bit: C.c_int8, TYPE_bte: C.c_int8, TYPE_sht: C.c_int16, TYPE_int: C.c_int32,
      TYPE_date: C.c_int32, TYPE_oid: C.c_uint64, TYPE_void: C.c_uint64, TYPE_lng: C.c_int64,
      TYPE_flt: C.c_float, TYPE_dbl: C.c_double, TYPE_daytime: C.c_int64, TYPE_timestamp: C.c_int64}
NIL = {TYPE_bit: -128, TYPE_bte: -128, TYPE_sht: -(1 << 15), TYPE_int: -(1 << 31),
       TYPE_date: -(1 << 31), TYPE_lng: -(1 << 63), TYPE_hge: -(1 << 127), TYPE_oid: OID_NIL,
       TYPE_void: OID_NIL, TYPE_flt: float("nan"), TYPE_dbl: float("nan"), TYPE_daytime: -(1 << 63),
       TYPE_timestamp: -(1 << 63)}
WIDTH = {TYPE_void: 0, TYPE_bit: 1, TYPE_bte: 1, TYPE_sht: 2, TYPE_int: 4, TYPE_date: 4,
         TYPE_flt: 4, TYPE_oid: 8, TYPE_lng: 8, TYPE_dbl: 8, TYPE_hge: 16, TYPE_str: 1, TYPE_daytime: 8,
         TYPE_timestamp: 8}


class MgdkBat(C.Structure):
    _fields_ = [("ttype", C.c_int32), ("twidth", C.c_int32), ("count", C.c_uint64),
                ("hseqbase", C.c_uint64), ("tseqbase", C.c_uint64), ("theap", C.c_void_p),
                ("tvheap", C.c_void_p), ("tvheapsize", C.c_uint64),
                ("tsorted", C.c_uint8), ("trevsorted", C.c_uint8), ("tkey", C.c_uint8),
                ("tnonil", C.c_uint8), ("tnil", C.c_uint8), ("_pad", C.c_uint8 * 3),
                ("priv", C.c_void_p), ("tnosorted", C.c_uint64), ("tnorevsorted", C.c_uint64),
                ("tminpos", C.c_uint64), ("tmaxpos", C.c_uint64), ("tunique_est", C.c_double)]


class Q1Row(C.Structure):
    _fields_ = [("returnflag", C.c_uint8), ("linestatus", C.c_uint8), ("_pad", C.c_uint8 * 6),
                ("sum_qty", C.c_uint64 * 2), ("sum_base_price", C.c_uint64 * 2),
                ("sum_disc_price", C.c_uint64 * 2), ("sum_charge", C.c_uint64 * 2),
                ("sum_disc", C.c_uint64 * 2), ("count_order", C.c_int64),
                ("first_row", C.c_uint64),
                ("avg_qty", C.c_int64), ("avg_price", C.c_int64), ("avg_disc", C.c_int64),
                ("rem_qty", C.c_int64), ("rem_price", C.c_int64), ("rem_disc", C.c_int64)]


P = C.POINTER(MgdkBat)
PP = C.POINTER(P)


class GDKError(RuntimeError):
    pass


_lib = None
_inited = False

# name -> (restype, argtypes)
_SIGS = {
    "mgdk_init": (C.c_int, [C.c_int]),
    "mgdk_GDKerrbuf": (C.c_char_p, []),
    "mgdk_GDKclrerr": (None, []),
    "mgdk_sync": (C.c_int, []),
    "mgdk_stream": (C.c_void_p, []),
    "mgdk_mem_cursize": (C.c_uint64, []),
    "mgdk_mem_release_cache": (None, []),
    "mgdk_thread_set_qry_ctx": (None, [C.c_void_p]),
    "mgdk_thread_get_qry_ctx": (C.c_void_p, []),
    "mgdk_usec": (C.c_int64, []),
    "mgdk_prof_enable": (None, [C.c_int]),
    "mgdk_prof_get": (C.c_int, [C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "mgdk_prof_reset": (None, []),
    "mgdk_COLnew": (P, [C.c_uint64, C.c_int, C.c_uint64]),
    "mgdk_BATdense": (P, [C.c_uint64, C.c_uint64, C.c_uint64]),
    "mgdk_BATconstant": (P, [C.c_uint64, C.c_int, C.c_void_p, C.c_uint64]),
    "mgdk_BATslice": (P, [P, C.c_uint64, C.c_uint64]),
    "mgdk_BBPunfix": (None, [P]),
    "mgdk_BATupload": (C.c_int, [P, C.c_void_p, C.c_uint64]),
    "mgdk_BATdownload": (C.c_int, [P, C.c_void_p]),
    "mgdk_BATsetvheap": (C.c_int, [P, C.c_void_p, C.c_uint64]),
    "mgdk_BATdownload_vheap": (C.c_int, [P, C.c_void_p]),
    "mgdk_BATmaskedcands": (P, [C.c_uint64, C.c_uint64, P, C.c_bool]),
    "mgdk_BATmergecand": (P, [P, P]),
    "mgdk_BATintersectcand": (P, [P, P]),
    "mgdk_BATdiffcand": (P, [P, P]),
    "mgdk_BATnegcands": (P, [C.c_uint64, C.c_uint64, P]),
    "mgdk_BATselect": (P, [P, P, C.c_void_p, C.c_void_p, C.c_bool, C.c_bool, C.c_bool, C.c_bool]),
    "mgdk_BATthetaselect": (P, [P, P, C.c_void_p, C.c_char_p]),
    "mgdk_BATproject": (P, [P, P]),
    "mgdk_BATproject2": (P, [P, P, P]),
    "mgdk_BATprojectchain": (P, [C.c_void_p]),
    "mgdk_BATcalcadd": (P, [P, P, P, P, C.c_int]),
    "mgdk_BATcalcsub": (P, [P, P, P, P, C.c_int]),
    "mgdk_BATcalcmul": (P, [P, P, P, P, C.c_int]),
    "mgdk_BATcalcaddcst": (P, [P, C.c_void_p, C.c_int, P, C.c_int]),
    "mgdk_BATcalcsubcst": (P, [P, C.c_void_p, C.c_int, P, C.c_int]),
    "mgdk_BATcalcmulcst": (P, [P, C.c_void_p, C.c_int, P, C.c_int]),
    "mgdk_BATcalccstadd": (P, [C.c_void_p, C.c_int, P, P, C.c_int]),
    "mgdk_BATcalccstsub": (P, [C.c_void_p, C.c_int, P, P, C.c_int]),
    "mgdk_BATcalccstmul": (P, [C.c_void_p, C.c_int, P, P, C.c_int]),
    "mgdk_BATcalccmp_op": (P, [C.c_int, P, C.c_void_p, C.c_int, P, C.c_void_p, C.c_int, P, P, C.c_bool]),
    "mgdk_BATcalcbetween": (P, [P, P, P, P, P, P] + [C.c_bool] * 5),
    "mgdk_BATcalcbetweencstcst": (P, [P, C.c_void_p, C.c_void_p, C.c_int, P] + [C.c_bool] * 5),
    "mgdk_BATcalcbetweenbatcst": (P, [P, P, C.c_void_p, C.c_int, P, P] + [C.c_bool] * 5),
    "mgdk_BATcalcbetweencstbat": (P, [P, C.c_void_p, P, C.c_int, P, P] + [C.c_bool] * 5),
    "mgdk_BATconvert": (P, [P, P, C.c_int, C.c_uint8, C.c_uint8, C.c_uint8]),
    "mgdk_BATcalcnot": (P, [P, P]),
    "mgdk_BATcalcnegate": (P, [P, P]),
    "mgdk_BATcalcabsolute": (P, [P, P]),
    "mgdk_BATcalciszero": (P, [P, P]),
    "mgdk_BATcalcsign": (P, [P, P]),
    "mgdk_BATcalcisnil": (P, [P, P]),
    "mgdk_BATcalcisnotnil": (P, [P, P]),
    "mgdk_BATcalcincr": (P, [P, P]),
    "mgdk_BATcalcdecr": (P, [P, P]),
    "mgdk_BATcalcmin": (P, [P, P, P, P]),
    "mgdk_BATcalcmax": (P, [P, P, P, P]),
    "mgdk_BATcalcmin_no_nil": (P, [P, P, P, P]),
    "mgdk_BATcalcmax_no_nil": (P, [P, P, P, P]),
    "mgdk_BATcalcand": (P, [P, P, P, P]),
    "mgdk_BATcalcor": (P, [P, P, P, P]),
    "mgdk_BATcalcxor": (P, [P, P, P, P]),
    "mgdk_BATcalclsh": (P, [P, P, P, P]),
    "mgdk_BATcalcrsh": (P, [P, P, P, P]),
    "mgdk_BATcalcmincst": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalcmaxcst": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalcmincst_no_nil": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalcmaxcst_no_nil": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalcandcst": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalcorcst": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalcxorcst": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalclshcst": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalcrshcst": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalccstmin": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalccstmax": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalccstmin_no_nil": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalccstmax_no_nil": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalccstand": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalccstor": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalccstxor": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalccstlsh": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalccstrsh": (P, [C.c_void_p, C.c_int, P, P]),
    "mgdk_BATcalcifthenelse": (P, [P, P, P]),
    "mgdk_BATcalcifthenelsecst": (P, [P, P, C.c_void_p, C.c_int]),
    "mgdk_BATcalcifthencstelse": (P, [P, C.c_void_p, C.c_int, P]),
    "mgdk_BATcalcifthencstelsecst": (P, [P, C.c_void_p, C.c_void_p, C.c_int]),
    "mgdk_BATcalcdiv": (P, [P, P, P, P, C.c_int]),
    "mgdk_BATcalcdivcst": (P, [P, C.c_void_p, C.c_int, P, C.c_int]),
    "mgdk_BATcalccstdiv": (P, [C.c_void_p, C.c_int, P, P, C.c_int]),
    "mgdk_BATcalcmod": (P, [P, P, P, P, C.c_int]),
    "mgdk_BATcalcmodcst": (P, [P, C.c_void_p, C.c_int, P, C.c_int]),
    "mgdk_BATcalccstmod": (P, [C.c_void_p, C.c_int, P, P, C.c_int]),
    "mgdk_BATsum": (C.c_int, [C.c_void_p, C.c_int, P, P, C.c_bool, C.c_bool]),
    "mgdk_BATgroupsum": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupcount": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupavg": (C.c_int, [PP, PP, P, P, P, P, C.c_int, C.c_bool, C.c_int]),
    "mgdk_BATgroupavg3combine": (P, [P, P, P, P, P, C.c_bool]),
    "mgdk_BATgroupavg3": (C.c_int, [PP, PP, PP, P, P, P, P, C.c_bool]),
    "mgdk_BATgroupmin": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATmin_skipnil": (C.c_void_p, [P, C.c_void_p, C.c_bool]),
    "mgdk_BATmax_skipnil": (C.c_void_p, [P, C.c_void_p, C.c_bool]),
    "mgdk_BATmin": (C.c_void_p, [P, C.c_void_p]),
    "mgdk_BATmax": (C.c_void_p, [P, C.c_void_p]),
    "mgdk_free": (None, [C.c_void_p]),
    "mgdk_BATprod": (C.c_int, [C.c_void_p, C.c_int, P, P, C.c_bool, C.c_bool]),
    "mgdk_BATgroupprod": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATunmask": (P, [P]),
    "mgdk_BATorderidx": (C.c_int, [P, C.c_bool]),
    "mgdk_set_fp_parallel_min": (C.c_uint64, [C.c_uint64]),
    "mgdk_BATcalcavg": (C.c_int, [P, P, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_int]),
    "mgdk_BATcheckorderidx": (C.c_bool, [P]),
    "mgdk_OIDXdestroy": (None, [P]),
    "mgdk_BATorderidx_get": (P, [P, C.POINTER(C.c_bool)]),
    "mgdk_BATgroupstdev_sample": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupstdev_population": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupvariance_sample": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupvariance_population": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupmedian": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupmedian_avg": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupcovariance_sample": (P, [P, P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupcovariance_population": (P, [P, P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupcorrelation": (P, [P, P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroupquantile": (P, [P, P, P, P, C.c_int, C.c_double, C.c_bool]),
    "mgdk_BATgroupquantile_avg": (P, [P, P, P, P, C.c_int, C.c_double, C.c_bool]),
    "mgdk_BATcalcstdev_population": (C.c_double, [C.POINTER(C.c_double), P]),
    "mgdk_BATcalcstdev_sample": (C.c_double, [C.POINTER(C.c_double), P]),
    "mgdk_BATcalcvariance_population": (C.c_double, [C.POINTER(C.c_double), P]),
    "mgdk_BATcalcvariance_sample": (C.c_double, [C.POINTER(C.c_double), P]),
    "mgdk_BATcalccovariance_population": (C.c_double, [P, P]),
    "mgdk_BATcalccovariance_sample": (C.c_double, [P, P]),
    "mgdk_BATcalccorrelation": (C.c_double, [P, P]),
    "mgdk_BATgroupmax": (P, [P, P, P, P, C.c_int, C.c_bool]),
    "mgdk_BATgroup": (C.c_int, [PP, PP, PP, P, P, P, P, P]),
    "mgdk_BATjoin": (C.c_int, [PP, PP, P, P, P, P, C.c_bool, C.c_uint64]),
    "mgdk_BATintersect": (P, [P, P, P, P, C.c_bool, C.c_bool, C.c_uint64]),
    "mgdk_BATdiff": (P, [P, P, P, P, C.c_bool, C.c_bool, C.c_uint64]),
    "mgdk_BATsemijoin": (C.c_int, [PP, PP, P, P, P, P, C.c_bool, C.c_bool, C.c_uint64]),
    "mgdk_BATleftjoin": (C.c_int, [PP, PP, P, P, P, P, C.c_bool, C.c_uint64]),
    "mgdk_BATthetajoin": (C.c_int, [PP, PP, P, P, P, P, C.c_int, C.c_bool, C.c_uint64]),
    "mgdk_BATsubcross": (C.c_int, [PP, PP, P, P, P, P, C.c_bool]),
    "mgdk_BATcount_no_nil": (C.c_uint64, [P, P]),
    "mgdk_BATguess_uniques": (C.c_uint64, [P, P]),
    "mgdk_BAToutercross": (C.c_int, [PP, PP, P, P, P, P, C.c_bool]),
    "mgdk_BATbandjoin": (C.c_int, [PP, PP, P, P, P, P, C.c_void_p, C.c_void_p, C.c_bool, C.c_bool, C.c_uint64]),
    "mgdk_BATrangejoin": (C.c_int, [PP, PP, P, P, P, P, P, C.c_bool, C.c_bool, C.c_bool, C.c_bool, C.c_uint64]),
    "mgdk_BATouterjoin": (C.c_int, [PP, PP, P, P, P, P, C.c_bool, C.c_bool, C.c_uint64]),
    "mgdk_BATmarkjoin": (C.c_int, [PP, PP, PP, P, P, P, P, C.c_uint64]),
    "mgdk_BATordered": (C.c_bool, [P]),
    "mgdk_BATordered_rev": (C.c_bool, [P]),
    "mgdk_BATsort": (C.c_int, [PP, PP, PP, P, P, P, C.c_bool, C.c_bool, C.c_bool]),
    "mgdk_GDKanalyticalwindowbounds": (C.c_int, [P, P, P, P, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                                 C.c_bool, C.c_uint64]),
    "mgdk_group_sums_ordered": (C.c_int, [C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P), P,
                                           C.POINTER(P), C.c_int]),
    "mgdk_q6_fused": (C.c_int, [P, P, P, P, C.c_int32, C.c_int32, C.c_int64, C.c_int64, C.c_int64,
                                C.c_void_p]),
    "mgdk_q1_fused": (C.c_int, [P, P, P, P, P, P, P, C.c_int32, C.POINTER(Q1Row), C.c_int,
                                C.POINTER(C.c_int)]),
    "mgdk_q6_opatatime": (C.c_int, [P, P, P, P, C.c_int32, C.c_int32, C.c_int64, C.c_int64,
                                    C.c_int64, C.c_void_p]),
    "mgdk_q1_opatatime": (C.c_int, [P, P, P, P, P, P, P, C.c_int32, C.POINTER(Q1Row), C.c_int,
                                    C.POINTER(C.c_int)]),
    "mgdk_tpch_lineitem": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, PP]),
    "mgdk_gen_window_column": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, PP, PP]),
    "mgdk_BAThashpartition": (C.c_int, [PP, C.c_void_p, C.c_int, C.c_void_p]),
    "mgdk_BATunique": (P, [C.c_void_p, C.c_void_p]),
    "mgdk_BBPreaddir": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "mgdk_BATload": (P, [C.c_char_p, C.c_void_p]),
    "mgdk_DICTcompress": (C.c_int, [PP, PP, C.c_void_p, C.c_bool, C.c_bool]),
    "mgdk_DICTdecompress": (P, [C.c_void_p, C.c_void_p]),
    "mgdk_DICTselect": (P, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_bool, C.c_bool,
                            C.c_bool]),
    "mgdk_DICTthetaselect": (P, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p]),
    "mgdk_FORcompress": (P, [C.c_void_p, C.c_void_p]),
    "mgdk_FORdecompress": (P, [C.c_void_p, C.c_int64, C.c_int]),
    "mgdk_BATfirstn": (C.c_int, [PP, PP, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_bool, C.c_bool,
                                 C.c_bool]),
    "mgdk_GDKanalyticalsum": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int, C.c_int]),
    "mgdk_GDKanalyticalcount": (C.c_int, [C.c_void_p] * 6 + [C.c_bool, C.c_int, C.c_int]),
    "mgdk_GDKanalyticalavg": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int]),
    "mgdk_GDKanalyticalntile": (C.c_int, [C.c_void_p] * 4 + [C.c_int, C.c_void_p]),
    "mgdk_GDKanalyticaldiff": (C.c_int, [C.c_void_p] * 4 + [C.c_int]),
    "mgdk_GDKanalyticalfirst": (C.c_int, [C.c_void_p] * 4 + [C.c_int]),
    "mgdk_GDKanalyticallast": (C.c_int, [C.c_void_p] * 4 + [C.c_int]),
    "mgdk_GDKanalyticalnthvalue": (C.c_int, [C.c_void_p] * 6 + [C.c_int]),
    "mgdk_GDKanalyticallag": (C.c_int, [C.c_void_p] * 3 + [C.c_uint64, C.c_void_p, C.c_int]),
    "mgdk_GDKanalyticallead": (C.c_int, [C.c_void_p] * 3 + [C.c_uint64, C.c_void_p, C.c_int]),
    "mgdk_GDKanalyticalmin": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int]),
    "mgdk_GDKanalyticalmax": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int]),
    "mgdk_GDKanalyticalavginteger": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int]),
    "mgdk_GDKanalytical_stddev_samp": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int]),
    "mgdk_GDKanalytical_stddev_pop": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int]),
    "mgdk_GDKanalytical_variance_samp": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int]),
    "mgdk_GDKanalytical_variance_pop": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int]),
    "mgdk_GDKanalytical_covariance_samp": (C.c_int, [C.c_void_p] * 7 + [C.c_int, C.c_int]),
    "mgdk_GDKanalytical_covariance_pop": (C.c_int, [C.c_void_p] * 7 + [C.c_int, C.c_int]),
    "mgdk_GDKanalytical_correlation": (C.c_int, [C.c_void_p] * 7 + [C.c_int, C.c_int]),
    "mgdk_GDKanalyticalprod": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_int, C.c_int]),
    "mgdk_BATlowerbound2": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                      C.c_void_p]),
    "mgdk_BATupload_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "mgdk_BATappend": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_bool]),
    "mgdk_BATdownload_device": (C.c_int, [C.c_void_p, C.c_void_p]),
}


def lib():
    """Load libmgdk.so (in-tree build).  Raises if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run python -m monetdb_amd.build")
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7
        # (same soname as /opt/rocm's).  Whichever loads first is shared by
        # both; if ours came first torch's device discovery fails, so let
        # torch (the plumbing for collectives and device tensors) load first.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def init(device=0):
    global _inited
    if not _inited:
        if lib().mgdk_init(device) != 0:
            raise GDKError(lib().mgdk_GDKerrbuf().decode())
        _inited = True


def _err():
    return GDKError(lib().mgdk_GDKerrbuf().decode())


def _chk(rc):
    if rc != 0:
        raise _err()


def hge_to_int(words):
    lo, hi = int(words[0]) & ((1 << 64) - 1), int(words[1]) & ((1 << 64) - 1)
    v = (hi << 64) | lo
    return v - (1 << 128) if v >= (1 << 127) else v


def int_to_hge_words(v):
    v &= (1 << 128) - 1
    return v & ((1 << 64) - 1), v >> 64


class BBPEntry(C.Structure):
    _fields_ = [("batid", C.c_int64), ("name", C.c_char * 129), ("type", C.c_char * 33), ("tt", C.c_int32),
                ("width", C.c_int32), ("var", C.c_int32), ("props", C.c_uint32), ("count", C.c_uint64),
                ("hseqbase", C.c_uint64), ("tseqbase", C.c_uint64), ("free", C.c_uint64),
                ("vfree", C.c_uint64), ("tail", C.c_char * 256), ("theap", C.c_char * 256)]


class BAT:
    """Owning handle of one mgdk_bat (heap in HBM)."""

    __slots__ = ("ptr",)

    def __init__(self, ptr):
        if not ptr:
            raise _err()
        self.ptr = ptr

    # -- construction --
    @classmethod
    def from_numpy(cls, tp, arr, hseqbase=0, sorted_=None, revsorted=None, key=None,
                   nonil=None, vheap=None):
        init()
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
        ctp = {1: TYPE_bte, 2: TYPE_sht, 4: TYPE_int, 8: TYPE_lng}[a.dtype.itemsize] if tp == TYPE_str else tp
        b = BAT(lib().mgdk_COLnew(hseqbase, ctp, n))
        _chk(lib().mgdk_BATupload(b.ptr, a.ctypes.data, n))
        s = b.ptr.contents
        if tp == TYPE_str:
            s.ttype = TYPE_str
            s.twidth = a.dtype.itemsize
        if tp != TYPE_hge and tp != TYPE_str and n:
            flat = a
            isn = np.isnan(flat) if flat.dtype.kind == "f" else (flat == NIL[tp]) if tp in NIL else \
                np.zeros(n, bool)
            s.tnonil = int(not isn.any()) if nonil is None else int(nonil)
            s.tnil = int(isn.any())
            cmpv = flat.astype(np.float64) if flat.dtype.kind == "f" else flat
            # compare neighbours (np.diff wraps for unsigned oids)
            s.tsorted = int(bool((cmpv[1:] >= cmpv[:-1]).all())) if sorted_ is None else int(sorted_)
            s.trevsorted = int(bool((cmpv[1:] <= cmpv[:-1]).all())) if revsorted is None else int(revsorted)
            s.tkey = int(len(np.unique(flat)) == n) if key is None else int(key)
        else:
            s.tnonil = 1 if nonil is None else int(nonil)
            s.tsorted = int(n <= 1) if sorted_ is None else int(sorted_)
            s.trevsorted = int(n <= 1) if revsorted is None else int(revsorted)
            s.tkey = int(n <= 1) if key is None else int(key)
        if vheap is not None:
            vh = np.frombuffer(bytes(vheap), dtype=np.uint8)
            _chk(lib().mgdk_BATsetvheap(b.ptr, vh.ctypes.data, vh.size))
        return b

    @classmethod
    def dense(cls, tseq, n, hseqbase=0):
        init()
        return BAT(lib().mgdk_BATdense(hseqbase, tseq, n))

    @classmethod
    def negoid_cand(cls, tseq, count, exceptions):
        """A cand_except candidate list (gdk/gdk_cand.h:23-38): the dense
        range [tseq, tseq + count + len(exceptions)) minus the sorted
        exception oids, as a void BAT whose vheap holds ccand_t
        {type = CAND_NEGOID} + the exceptions."""
        b = cls.dense(tseq, count)
        exc = np.asarray(exceptions, np.uint64)
        buf = np.concatenate([np.zeros(1, np.uint64), exc]).tobytes()
        _chk(lib().mgdk_BATsetvheap(b.ptr, buf, len(buf)))
        return b

    @classmethod
    def mask_cand(cls, seq, bits):
        """A cand_mask candidate list: candidate seq + i for every set bit i
        of `bits` (bool array); ccand_t {type = CAND_MSK, firstbit} + 32-bit
        words, tseqbase = the first candidate."""
        bits = np.asarray(bits, bool)
        nz = np.flatnonzero(bits)
        first = int(nz[0]) if nz.size else 0
        words = np.packbits(np.concatenate([bits, np.zeros((-len(bits)) % 32, bool)]),
                            bitorder="little").view(np.uint32)
        b = cls.dense(seq + first, int(nz.size))
        hdr = np.array([1 | (first << 1)], np.uint64)
        buf = hdr.tobytes() + words.tobytes()
        _chk(lib().mgdk_BATsetvheap(b.ptr, buf, len(buf)))
        return b

    @classmethod
    def msk(cls, bits, hseqbase=0):
        """A msk BAT (TYPE_msk): one bit per row packed into 32-bit words,
        count = len(bits)."""
        init()
        bits = np.asarray(bits, bool)
        n = bits.size
        words = np.packbits(np.concatenate([bits, np.zeros((-n) % 32, bool)]),
                            bitorder="little").view(np.uint32)
        b = BAT(lib().mgdk_COLnew(hseqbase, TYPE_msk, max(1, n)))
        _chk(lib().mgdk_BATupload(b.ptr, words.ctypes.data, n))
        b.ptr.contents.count = n
        return b

    # -- properties --
    @property
    def s(self):
        return self.ptr.contents

    @property
    def ttype(self):
        return self.s.ttype

    def count(self):
        return self.s.count

    def __len__(self):
        return self.s.count

    @property
    def hseqbase(self):
        return self.s.hseqbase

    def is_dense(self):
        return self.s.ttype == TYPE_void

    def to_numpy(self):
        s = self.s
        n = s.count
        if s.ttype == TYPE_void:
            if s.tseqbase == OID_NIL:
                return np.full(n, OID_NIL, np.uint64)
            return np.arange(s.tseqbase, s.tseqbase + n, dtype=np.uint64)
        if s.ttype == TYPE_hge:
            out = np.empty((n, 2), np.uint64)
        elif s.ttype == TYPE_str:
            out = np.empty(n, {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[s.twidth])
        else:
            out = np.empty(n, NP[s.ttype])
        if n:
            _chk(lib().mgdk_BATdownload(self.ptr, out.ctypes.data))
        return out

    def values(self):
        """Python values (hge as int)."""
        a = self.to_numpy()
        if self.s.ttype == TYPE_hge:
            return [hge_to_int(r) for r in a]
        return a

    def __del__(self):
        p = getattr(self, "ptr", None)
        if p and _lib is not None:
            _lib.mgdk_BBPunfix(p)
            self.ptr = None


def _p(b):
    return b.ptr if b is not None else None


def _valptr(tp, v, keep):
    if v is None:
        return None
    if tp == TYPE_str:
        # a C string (bytes or str); b"\x80" is str nil
        buf = C.create_string_buffer(v if isinstance(v, bytes) else v.encode())
        keep.append(buf)
        return C.cast(buf, C.c_void_p)
    if tp == TYPE_hge:
        buf = (C.c_uint64 * 2)(*int_to_hge_words(int(v)))
    else:
        buf = CT[tp](v)
    keep.append(buf)
    return C.cast(C.pointer(buf), C.c_void_p)


# ---- operators (same names as GDK) ------------------------------------------

def BATmaskedcands(hseq, nr, masked, selected=True):
    """gdk/gdk_cand.c:1366: a cand_mask candidate list from a msk BAT."""
    return BAT(lib().mgdk_BATmaskedcands(hseq, nr, masked.ptr, selected))


def BATmergecand(a, b):
    """gdk/gdk_cand.c:46: the union of two candidate lists."""
    return BAT(lib().mgdk_BATmergecand(a.ptr, b.ptr))


def BATintersectcand(a, b):
    """gdk/gdk_cand.c:184: the intersection of two candidate lists."""
    return BAT(lib().mgdk_BATintersectcand(a.ptr, b.ptr))


def BATdiffcand(a, b):
    """gdk/gdk_cand.c:259: the candidates of a that are not in b."""
    return BAT(lib().mgdk_BATdiffcand(a.ptr, b.ptr))


def BATnegcands(tseq, nr, odels):
    """gdk/gdk_cand.c:1296: [tseq, tseq + nr) minus the sorted deletions odels
    (a cand_except list when a deletion falls inside)."""
    return BAT(lib().mgdk_BATnegcands(tseq, nr, odels.ptr))


def cand_oids(c):
    """The oids a candidate list of any form stands for (numpy uint64), read
    back through BATmergecand with an empty list (canditer_slice)."""
    return BATmergecand(c, BAT.dense(0, 0)).to_numpy().astype(np.uint64)


def BATselect(b, s, tl, th, li, hi, anti, nil_matches=False):
    keep = []
    tp = b.ttype
    return BAT(lib().mgdk_BATselect(b.ptr, _p(s), _valptr(tp, tl, keep), _valptr(tp, th, keep),
                                    li, hi, anti, nil_matches))


def BATthetaselect(b, s, val, op):
    keep = []
    return BAT(lib().mgdk_BATthetaselect(b.ptr, _p(s), _valptr(b.ttype, val, keep), op.encode()))


def BATproject2(l, r1, r2):
    """BATproject2(l, r1, r2) (gdk/gdk_project.c:590): l over r1 ++ r2."""
    return BAT(lib().mgdk_BATproject2(l.ptr, r1.ptr, _p(r2)))


def BATprojectchain(bats):
    """BATprojectchain (gdk/gdk_project.c:879): bats[0] . bats[1] . ... in one pass."""
    arr = (P * (len(bats) + 1))(*[b.ptr for b in bats], None)
    return BAT(lib().mgdk_BATprojectchain(C.cast(arr, C.c_void_p)))


def BATproject(l, r):
    return BAT(lib().mgdk_BATproject(l.ptr, r.ptr))


def BATcalcadd(b1, b2, tp, s1=None, s2=None):
    return BAT(lib().mgdk_BATcalcadd(b1.ptr, b2.ptr, _p(s1), _p(s2), tp))


def BATcalcsub(b1, b2, tp, s1=None, s2=None):
    return BAT(lib().mgdk_BATcalcsub(b1.ptr, b2.ptr, _p(s1), _p(s2), tp))


def BATcalcmul(b1, b2, tp, s1=None, s2=None):
    return BAT(lib().mgdk_BATcalcmul(b1.ptr, b2.ptr, _p(s1), _p(s2), tp))


CMP_OPS = {"<": 0, "<=": 1, ">": 2, ">=": 3, "==": 4, "!=": 5, "cmp": 6}


def BATcalccmp(op, b1, b2, s1=None, s2=None, c1=None, t1=0, c2=None, t2=0, nil_matches=False):
    """BATcalc{lt,le,gt,ge,eq,ne,cmp} and their cst forms (gdk/gdk_calc.h:66-84):
    op in CMP_OPS; b1 / b2 None takes the constant c1 / c2 of type t1 / t2."""
    keep = []
    return BAT(lib().mgdk_BATcalccmp_op(CMP_OPS[op], _p(b1), _valptr(t1, c1, keep), t1, _p(b2),
                                        _valptr(t2, c2, keep), t2, _p(s1), _p(s2), nil_matches))


def BATcalcbetween(b, lo, hi, s=None, slo=None, shi=None, clo=None, chi=None, ct=0, symmetric=False,
                   linc=True, hinc=True, nils_false=False, anti=False):
    """BATcalcbetween / -cstcst / -batcst / -cstbat (gdk/gdk_calc.c:3968-4206);
    lo / hi None take the constants clo / chi of type ct."""
    keep = []
    f = (symmetric, linc, hinc, nils_false, anti)
    L = lib()
    if lo is not None and hi is not None:
        return BAT(L.mgdk_BATcalcbetween(b.ptr, lo.ptr, hi.ptr, _p(s), _p(slo), _p(shi), *f))
    if lo is None and hi is None:
        return BAT(L.mgdk_BATcalcbetweencstcst(b.ptr, _valptr(ct, clo, keep), _valptr(ct, chi, keep), ct,
                                               _p(s), *f))
    if hi is None:
        return BAT(L.mgdk_BATcalcbetweenbatcst(b.ptr, lo.ptr, _valptr(ct, chi, keep), ct, _p(s), _p(slo), *f))
    return BAT(L.mgdk_BATcalcbetweencstbat(b.ptr, _valptr(ct, clo, keep), hi.ptr, ct, _p(s), _p(shi), *f))


def BATconvert(b, s, tp, scale1=0, scale2=0, precision=0):
    """BATconvert (gdk/gdk_calc_convert.c:1415)"""
    return BAT(lib().mgdk_BATconvert(b.ptr, _p(s), tp, scale1, scale2, precision))


def BATcalcnot(b, s=None):
    return BAT(lib().mgdk_BATcalcnot(b.ptr, _p(s)))


def BATcalcdivmod(op, b1, b2, tp, s1=None, s2=None, c1=None, t1=0, c2=None, t2=0):
    """BATcalcdiv / BATcalcmod and their cst forms; op '/' or '%'"""
    keep = []
    nm = "div" if op == "/" else "mod"
    L = lib()
    if b1 is not None and b2 is not None:
        return BAT(getattr(L, "mgdk_BATcalc" + nm)(b1.ptr, b2.ptr, _p(s1), _p(s2), tp))
    if b2 is None:
        return BAT(getattr(L, "mgdk_BATcalc%scst" % nm)(b1.ptr, _valptr(t2, c2, keep), t2, _p(s1), tp))
    return BAT(getattr(L, "mgdk_BATcalccst" + nm)(_valptr(t1, c1, keep), t1, b2.ptr, _p(s1), tp))


def _cst(fn, b, v, vt, s, tp):
    keep = []
    return BAT(getattr(lib(), fn)(b.ptr, _valptr(vt, v, keep), vt, _p(s), tp))


def _cstb(fn, v, vt, b, s, tp):
    keep = []
    return BAT(getattr(lib(), fn)(_valptr(vt, v, keep), vt, b.ptr, _p(s), tp))


def BATcalcaddcst(b, v, vt, tp, s=None):
    return _cst("mgdk_BATcalcaddcst", b, v, vt, s, tp)


def BATcalcsubcst(b, v, vt, tp, s=None):
    return _cst("mgdk_BATcalcsubcst", b, v, vt, s, tp)


def BATcalcmulcst(b, v, vt, tp, s=None):
    return _cst("mgdk_BATcalcmulcst", b, v, vt, s, tp)


def BATcalccstadd(v, vt, b, tp, s=None):
    return _cstb("mgdk_BATcalccstadd", v, vt, b, s, tp)


def BATcalccstsub(v, vt, b, tp, s=None):
    return _cstb("mgdk_BATcalccstsub", v, vt, b, s, tp)


def BATcalccstmul(v, vt, b, tp, s=None):
    return _cstb("mgdk_BATcalccstmul", v, vt, b, s, tp)


def BATsum(tp, b, s=None, skip_nils=True, nil_if_empty=True):
    buf = (C.c_uint64 * 2)()
    _chk(lib().mgdk_BATsum(C.cast(buf, C.c_void_p), tp, b.ptr, _p(s), skip_nils, nil_if_empty))
    if tp == TYPE_hge:
        return hge_to_int(buf)
    if tp == TYPE_dbl:
        return C.cast(buf, C.POINTER(C.c_double))[0]
    return C.cast(buf, C.POINTER(CT[tp]))[0]


def BATgroupsum(b, g, e, tp, skip_nils=True, s=None):
    return BAT(lib().mgdk_BATgroupsum(b.ptr, g.ptr, _p(e), _p(s), tp, skip_nils))


def BATgroupcount(b, g, e, skip_nils=True, s=None):
    return BAT(lib().mgdk_BATgroupcount(b.ptr, g.ptr, _p(e), _p(s), TYPE_lng, skip_nils))


def _scalar(tp, buf):
    """a value of type tp from a raw buffer (hge as an int)"""
    if tp == TYPE_hge:
        return hge_to_int(C.cast(buf, C.POINTER(C.c_uint64 * 2))[0])
    return C.cast(buf, C.POINTER(CT[tp]))[0]


def _minmax(fn, b, skipnil):
    if b.ttype == TYPE_str:
        p = fn(b.ptr, None, skipnil)
        if not p:
            _chk(-1)
        try:
            return C.string_at(p)
        finally:
            lib().mgdk_free(p)
    buf = (C.c_uint64 * 2)()
    if not fn(b.ptr, C.cast(buf, C.c_void_p), skipnil):
        _chk(-1)
    return _scalar(TYPE_oid if b.ttype == TYPE_void else b.ttype, buf)


def BATmin(b, skipnil=True):
    """BATmin_skipnil (gdk_aggr.c:3570): the smallest value (nil when none;
    str as bytes)"""
    return _minmax(lib().mgdk_BATmin_skipnil, b, skipnil)


def BATmax(b, skipnil=True):
    """BATmax_skipnil (gdk_aggr.c:3727)"""
    return _minmax(lib().mgdk_BATmax_skipnil, b, skipnil)


def BATprod(tp, b, s=None, skip_nils=True, nil_if_empty=True):
    """BATprod (gdk_aggr.c:1650)"""
    buf = (C.c_uint64 * 2)()
    _chk(lib().mgdk_BATprod(C.cast(buf, C.c_void_p), tp, b.ptr, _p(s), skip_nils, nil_if_empty))
    return _scalar(tp, buf)


def BATgroupprod(b, g, e, tp, skip_nils=True, s=None):
    """BATgroupprod (gdk_aggr.c:1575)"""
    return BAT(lib().mgdk_BATgroupprod(b.ptr, g.ptr, _p(e), _p(s), tp, skip_nils))


def BATunmask(b):
    """BATunmask (gdk_cand.c:1464)"""
    return BAT(lib().mgdk_BATunmask(b.ptr))


def set_fp_parallel_min(rows):
    """rows from which one group / partition of an order-dependent float fold
    takes the parallel form (None: never); returns the previous value"""
    init()
    return int(lib().mgdk_set_fp_parallel_min(BUN_NONE if rows is None else int(rows)))


def BATorderidx(b, stable=False):
    """BATorderidx (gdk_orderidx.c:184): keep b's sort order with b"""
    _chk(lib().mgdk_BATorderidx(b.ptr, stable))


def BATcheckorderidx(b):
    """BATcheckorderidx (gdk_orderidx.c:74)"""
    return bool(lib().mgdk_BATcheckorderidx(b.ptr))


def OIDXdestroy(b):
    """OIDXdestroy (gdk_orderidx.c:534)"""
    lib().mgdk_OIDXdestroy(b.ptr)


def BATorderidx_get(b):
    """(index as an oid BAT, stable flag) of b's order index, or None"""
    st = C.c_bool(False)
    p = lib().mgdk_BATorderidx_get(b.ptr, C.byref(st))
    if not p:
        return None
    return BAT(p), bool(st.value)


def BATcalcunary(name, b, s=None):
    """BATcalc{negate,absolute,iszero,sign,isnil,isnotnil,incr,decr}(b, s)"""
    return BAT(getattr(lib(), "mgdk_BATcalc" + name)(b.ptr, _p(s)))


def BATcalcbin(name, b1, b2, s1=None, s2=None):
    """BATcalc{min,max,min_no_nil,max_no_nil,and,or,xor,lsh,rsh}(b1, b2, s1, s2)"""
    return BAT(getattr(lib(), "mgdk_BATcalc" + name)(b1.ptr, b2.ptr, _p(s1), _p(s2)))


def BATcalcbincst(name, b, v, vt, s=None, cst_first=False):
    """BATcalc<name>cst(b, v, s) or, cst_first, BATcalccst<name>(v, b, s)"""
    keep = []
    vp = _valptr(vt, v, keep)
    if cst_first:
        return BAT(getattr(lib(), "mgdk_BATcalccst" + name)(vp, vt, b.ptr, _p(s)))
    n = name.replace("_no_nil", "cst_no_nil") if name.endswith("_no_nil") else name + "cst"
    return BAT(getattr(lib(), "mgdk_BATcalc" + n)(b.ptr, vp, vt, _p(s)))


def BATcalcifthenelse(b, then, else_, ct=None):
    """BATcalcifthenelse (gdk_calc.c:4661) and its constant forms: then /
    else are BATs or Python values of type ct"""
    keep = []
    t_bat, e_bat = isinstance(then, BAT), isinstance(else_, BAT)
    if t_bat and e_bat:
        return BAT(lib().mgdk_BATcalcifthenelse(b.ptr, then.ptr, else_.ptr))
    if t_bat:
        return BAT(lib().mgdk_BATcalcifthenelsecst(b.ptr, then.ptr, _valptr(ct, else_, keep), ct))
    if e_bat:
        return BAT(lib().mgdk_BATcalcifthencstelse(b.ptr, _valptr(ct, then, keep), ct, else_.ptr))
    return BAT(lib().mgdk_BATcalcifthencstelsecst(b.ptr, _valptr(ct, then, keep), _valptr(ct, else_, keep), ct))


def BATgroupmin(b, g, e, skip_nils=True, s=None):
    return BAT(lib().mgdk_BATgroupmin(b.ptr, g.ptr, _p(e), _p(s), b.ttype, skip_nils))


def BATgroupmax(b, g, e, skip_nils=True, s=None):
    return BAT(lib().mgdk_BATgroupmax(b.ptr, g.ptr, _p(e), _p(s), b.ttype, skip_nils))


def _stat1(name, b, g, e, skip_nils, s):
    return BAT(getattr(lib(), "mgdk_BATgroup" + name)(b.ptr, _p(g), _p(e), _p(s), TYPE_dbl, skip_nils))


def _stat2(name, b1, b2, g, e, skip_nils, s):
    return BAT(getattr(lib(), "mgdk_BATgroup" + name)(b1.ptr, b2.ptr, _p(g), _p(e), _p(s), TYPE_dbl, skip_nils))


def BATgroupstdev_sample(b, g, e, skip_nils=True, s=None):
    """gdk_aggr.c:4778 (dogroupstdev :4612): Welford per group, dbl"""
    return _stat1("stdev_sample", b, g, e, skip_nils, s)


def BATgroupstdev_population(b, g, e, skip_nils=True, s=None):
    """gdk_aggr.c:4785"""
    return _stat1("stdev_population", b, g, e, skip_nils, s)


def BATgroupvariance_sample(b, g, e, skip_nils=True, s=None):
    """gdk_aggr.c:4793"""
    return _stat1("variance_sample", b, g, e, skip_nils, s)


def BATgroupvariance_population(b, g, e, skip_nils=True, s=None):
    """gdk_aggr.c:4801"""
    return _stat1("variance_population", b, g, e, skip_nils, s)


def BATgroupcovariance_sample(b1, b2, g, e, skip_nils=True, s=None):
    """gdk_aggr.c:5000 (dogroupcovariance :4851)"""
    return _stat2("covariance_sample", b1, b2, g, e, skip_nils, s)


def BATgroupcovariance_population(b1, b2, g, e, skip_nils=True, s=None):
    """gdk_aggr.c:5007"""
    return _stat2("covariance_population", b1, b2, g, e, skip_nils, s)


def BATgroupcorrelation(b1, b2, g, e, skip_nils=True, s=None):
    """gdk_aggr.c:5057"""
    return _stat2("correlation", b1, b2, g, e, skip_nils, s)


def _calc(fn, *args):
    lib().mgdk_GDKclrerr()
    v = fn(*args)
    msg = lib().mgdk_GDKerrbuf().decode()
    if msg:
        raise GDKError(msg)
    return v


def BATcalcvariance(b, sample, stdev=False):
    """BATcalc{stdev,variance}_{sample,population}(&avg, b) (gdk_aggr.c:4327-4380):
    returns (value, average); nil is NaN"""
    avg = C.c_double()
    name = "mgdk_BATcalc%s_%s" % ("stdev" if stdev else "variance", "sample" if sample else "population")
    v = _calc(getattr(lib(), name), C.byref(avg), b.ptr)
    return v, avg.value


def BATcalccovariance(b1, b2, sample):
    """BATcalccovariance_{sample,population} (gdk_aggr.c:4449-4476)"""
    name = "mgdk_BATcalccovariance_%s" % ("sample" if sample else "population")
    return _calc(getattr(lib(), name), b1.ptr, b2.ptr)


def BATcalccorrelation(b1, b2):
    """gdk_aggr.c:4503"""
    return _calc(lib().mgdk_BATcalccorrelation, b1.ptr, b2.ptr)


def BATgroupquantile(b, g, e, quantile, skip_nils=True, s=None, average=False):
    """doBATgroupquantile (gdk_aggr.c:3881) through BATgroupquantile (:4233) or
    BATgroupquantile_avg (:4247); g may be None"""
    f = lib().mgdk_BATgroupquantile_avg if average else lib().mgdk_BATgroupquantile
    return BAT(f(b.ptr, _p(g), _p(e), _p(s), b.ttype, quantile, skip_nils))


def BATgroupmedian(b, g, e, skip_nils=True, s=None, average=False):
    """BATgroupmedian (gdk_aggr.c:4225) / BATgroupmedian_avg (:4241)"""
    f = lib().mgdk_BATgroupmedian_avg if average else lib().mgdk_BATgroupmedian
    return BAT(f(b.ptr, _p(g), _p(e), _p(s), b.ttype, skip_nils))


def BATcalcavg(b, s=None, scale=0):
    """BATcalcavg (gdk_aggr.c:2987): (average, number of non-nil values); nil is NaN"""
    a, n = C.c_double(), C.c_uint64()
    _chk(lib().mgdk_BATcalcavg(b.ptr, _p(s), C.byref(a), C.byref(n), scale))
    return a.value, n.value


def BATgroupavg(b, g, e, skip_nils=True, s=None, scale=0, want_counts=True):
    """BATgroupavg(&bn, &cnts, b, g, e, s, TYPE_dbl, skip_nils, scale)
    (gdk/gdk_aggr.c:1801); returns (averages, counts or None)."""
    a, c = P(), P()
    _chk(lib().mgdk_BATgroupavg(C.byref(a), C.byref(c) if want_counts else None, b.ptr, g.ptr, _p(e),
                                _p(s), TYPE_dbl, skip_nils, scale))
    return BAT(a), (BAT(c) if want_counts else None)


def BATgroupavg3combine(avg, rem, cnt, g, e, skip_nils=True):
    """BATgroupavg3combine (gdk/gdk_aggr.c:2634): rounded group averages of
    partial (avg, rem, cnt) rows."""
    return BAT(lib().mgdk_BATgroupavg3combine(avg.ptr, rem.ptr, cnt.ptr, _p(g), _p(e), skip_nils))


def BATgroupavg3(b, g, e, skip_nils=True, s=None):
    a, r, c = P(), P(), P()
    _chk(lib().mgdk_BATgroupavg3(C.byref(a), C.byref(r), C.byref(c), b.ptr, g.ptr, _p(e), _p(s),
                                 skip_nils))
    return BAT(a), BAT(r), BAT(c)


def BATgroup(b, s=None, g=None, e=None, h=None, want_histo=True):
    """(groups, extents, histo) -- gdk_group.c:1359; histo is None (and not
    computed) when want_histo is False, as BATgroup(&g, &e, NULL, ...)."""
    gp, ep, hp = P(), P(), P()
    _chk(lib().mgdk_BATgroup(C.byref(gp), C.byref(ep), C.byref(hp) if want_histo else None, b.ptr, _p(s),
                             _p(g), _p(e), _p(h)))
    return BAT(gp), BAT(ep), (BAT(hp) if want_histo else None)


def BATjoin(l, r, sl=None, sr=None, nil_matches=False, estimate=0):
    a, b = P(), P()
    _chk(lib().mgdk_BATjoin(C.byref(a), C.byref(b), l.ptr, r.ptr, _p(sl), _p(sr), nil_matches,
                            estimate))
    return BAT(a), BAT(b)


def BATintersect(l, r, sl=None, sr=None, nil_matches=False, max_one=False, estimate=0):
    """gdk_join.c:4366: the left candidates whose value occurs on the right."""
    return BAT(lib().mgdk_BATintersect(l.ptr, r.ptr, _p(sl), _p(sr), nil_matches, max_one, estimate))


def BATdiff(l, r, sl=None, sr=None, nil_matches=False, not_in=False, estimate=0):
    """gdk_join.c:4388: the left candidates whose value does not occur on the right."""
    return BAT(lib().mgdk_BATdiff(l.ptr, r.ptr, _p(sl), _p(sr), nil_matches, not_in, estimate))


def BATsemijoin(l, r, sl=None, sr=None, nil_matches=False, max_one=False, estimate=0, want_r2=False):
    """gdk_join.c:4346: the left output (a candidate list); with want_r2 also
    the right output, one match per kept left candidate (algebra.semijoin,
    algebra.c:1792), as (r1, r2)."""
    a, b = P(), P()
    _chk(lib().mgdk_BATsemijoin(C.byref(a), C.byref(b) if want_r2 else None, l.ptr, r.ptr, _p(sl), _p(sr),
                                nil_matches, max_one, estimate))
    return (BAT(a), BAT(b)) if want_r2 else BAT(a)


def BATleftjoin(l, r, sl=None, sr=None, nil_matches=False, estimate=0):
    """gdk_join.c:4320: (left, match) pairs in left order."""
    a, b = P(), P()
    _chk(lib().mgdk_BATleftjoin(C.byref(a), C.byref(b), l.ptr, r.ptr, _p(sl), _p(sr), nil_matches, estimate))
    return BAT(a), BAT(b)


JOIN_EQ, JOIN_LT, JOIN_LE, JOIN_GT, JOIN_GE, JOIN_NE = 0, -1, -2, 1, 2, -3


def BATthetajoin(l, r, sl=None, sr=None, op=JOIN_LT, nil_matches=False, estimate=0):
    """BATthetajoin (gdk_join.c:4409): (r1, r2) pairs with l op r"""
    a, b = P(), P()
    _chk(lib().mgdk_BATthetajoin(C.byref(a), C.byref(b), l.ptr, r.ptr, _p(sl), _p(sr), op, nil_matches,
                                 estimate))
    return BAT(a), BAT(b)


def BATguess_uniques(b, s=None):
    """BATguess_uniques (gdk_join.c:3572): distinct-value estimate"""
    n = lib().mgdk_BATguess_uniques(b.ptr, _p(s))
    if n == BUN_NONE:
        _chk(-1)
    return n


def BATcount_no_nil(b, s=None):
    """BATcount_no_nil (gdk_batop.c:3078): candidates with a non-nil value"""
    n = lib().mgdk_BATcount_no_nil(b.ptr, _p(s))
    if n == BUN_NONE:
        _chk(-1)
    return n


def BATsubcross(l, r, sl=None, sr=None, max_one=False, want_r2=True):
    """BATsubcross (gdk_cross.c:138): every (left, right) candidate pair,
    left-major; (r1, r2) or, without want_r2, r1"""
    a, b = P(), P()
    _chk(lib().mgdk_BATsubcross(C.byref(a), C.byref(b) if want_r2 else None, l.ptr, r.ptr, _p(sl), _p(sr),
                                max_one))
    return (BAT(a), BAT(b)) if want_r2 else BAT(a)


def BAToutercross(l, r, sl=None, sr=None, max_one=False, want_r2=True):
    """BAToutercross (gdk_cross.c:153): as BATsubcross; no right candidate
    pairs every left one with nil"""
    a, b = P(), P()
    _chk(lib().mgdk_BAToutercross(C.byref(a), C.byref(b) if want_r2 else None, l.ptr, r.ptr, _p(sl), _p(sr),
                                  max_one))
    return (BAT(a), BAT(b)) if want_r2 else BAT(a)


def BATbandjoin(l, r, c1, c2, sl=None, sr=None, linc=True, hinc=True, estimate=0):
    """BATbandjoin (gdk_join.c:4626): r - c1 <= l <= r + c2"""
    keep = []
    a, b = P(), P()
    _chk(lib().mgdk_BATbandjoin(C.byref(a), C.byref(b), l.ptr, r.ptr, _p(sl), _p(sr), _valptr(l.ttype, c1, keep),
                                _valptr(l.ttype, c2, keep), linc, hinc, estimate))
    return BAT(a), BAT(b)


def BATrangejoin(l, rl, rh, sl=None, sr=None, linc=True, hinc=True, anti=False, symmetric=False, estimate=0):
    """BATrangejoin (gdk_join.c:5422): rl <= l <= rh per right candidate"""
    a, b = P(), P()
    _chk(lib().mgdk_BATrangejoin(C.byref(a), C.byref(b), l.ptr, rl.ptr, rh.ptr, _p(sl), _p(sr), linc, hinc, anti,
                                 symmetric, estimate))
    return BAT(a), BAT(b)


def BATouterjoin(l, r, sl=None, sr=None, nil_matches=False, match_one=False, estimate=0):
    """gdk_join.c:4334: (left, match or nil) pairs in left order."""
    a, b = P(), P()
    _chk(lib().mgdk_BATouterjoin(C.byref(a), C.byref(b), l.ptr, r.ptr, _p(sl), _p(sr), nil_matches, match_one,
                                 estimate))
    return BAT(a), BAT(b)


def BATmarkjoin(l, r, sl=None, sr=None, want_r2=True, estimate=0):
    """gdk_join.c:4367: (r1, r2, r3) -- every left candidate, its match or
    nil, the mark (TRUE / FALSE / nil); without r2 (semi) (r1, r3)."""
    a, b, c = P(), P(), P()
    _chk(lib().mgdk_BATmarkjoin(C.byref(a), C.byref(b) if want_r2 else None, C.byref(c), l.ptr, r.ptr, _p(sl), _p(sr),
                                estimate))
    return (BAT(a), BAT(b), BAT(c)) if want_r2 else (BAT(a), BAT(c))


def BATordered(b):
    """gdk_batop.c:2002: b sorted ascending (the finding is cached in b)."""
    return bool(lib().mgdk_BATordered(b.ptr))


def BATordered_rev(b):
    """gdk_batop.c:2181: b sorted descending (cached in b)."""
    return bool(lib().mgdk_BATordered_rev(b.ptr))


def BATsort(b, o=None, g=None, reverse=False, nilslast=False, stable=True, groups=True):
    sp, op, gp = P(), P(), P()
    _chk(lib().mgdk_BATsort(C.byref(sp), C.byref(op), C.byref(gp) if groups else None, b.ptr, _p(o), _p(g),
                            reverse, nilslast, stable))
    return BAT(sp), BAT(op), (BAT(gp) if gp else None)


def BATunique(b, s=None):
    """Candidate list of the first occurrence of each distinct value (gdk_unique.c:30)."""
    return BAT(lib().mgdk_BATunique(b.ptr, _p(s)))


def BATfirstn(b, n, s=None, g=None, asc=True, nilslast=False, distinct=False, want_gids=False):
    """(topn candidate list, gids or None) -- gdk_firstn.c:1280."""
    t, gi = P(), P()
    _chk(lib().mgdk_BATfirstn(C.byref(t), C.byref(gi) if want_gids else None, b.ptr, _p(s), _p(g), n,
                              asc, nilslast, distinct))
    return BAT(t), (BAT(gi) if want_gids else None)


def BBPreaddir(path):
    """Entries of a dbfarm's bat/BBP.dir (gdk_bbp.c:595-714)."""
    n = C.c_int()
    _chk(lib().mgdk_BBPreaddir(path.encode(), None, 0, C.byref(n)))
    arr = (BBPEntry * max(1, n.value))()
    _chk(lib().mgdk_BBPreaddir(path.encode(), C.cast(arr, C.c_void_p), n.value, C.byref(n)))
    return list(arr[:n.value])


def BATload(bat_dir, entry):
    """Stream one persistent BAT's heaps into HBM (gdk_heap.c:729 HEAPload)."""
    return BAT(lib().mgdk_BATload(bat_dir.encode(), C.cast(C.pointer(entry), C.c_void_p)))


def DICTcompress(b, ordered=True, smallest_type=True):
    """(codes, dictionary) -- dict.c:110."""
    o, u = P(), P()
    _chk(lib().mgdk_DICTcompress(C.byref(o), C.byref(u), b.ptr, ordered, smallest_type))
    return BAT(o), BAT(u)


def DICTdecompress(o, u):
    return BAT(lib().mgdk_DICTdecompress(o.ptr, u.ptr))


def DICTselect(lo, lc, lv, low, high, li, hi, anti):
    keep = []
    return BAT(lib().mgdk_DICTselect(lo.ptr, _p(lc), lv.ptr, _valptr(lv.ttype, low, keep),
                                     _valptr(lv.ttype, high, keep), li, hi, anti))


def DICTthetaselect(lo, lc, lv, val, op):
    keep = []
    return BAT(lib().mgdk_DICTthetaselect(lo.ptr, _p(lc), lv.ptr, _valptr(lv.ttype, val, keep), op.encode()))


def FORcompress(b):
    """(offsets, minval) -- for.c:148."""
    mn = C.c_int64()
    o = BAT(lib().mgdk_FORcompress(b.ptr, C.byref(mn)))
    return o, mn.value


def FORdecompress(o, minval, tp):
    return BAT(lib().mgdk_FORdecompress(o.ptr, minval, tp))


def GDKanalyticalwindowbounds(b, p, limit, preceding, tp1=None, tp2=TYPE_lng, unit=1, l=None, second_half=0):
    """GDKanalyticalwindowbounds(r, b, p, l, bound, tp1, tp2, unit,
    preceding, second_half) (gdk/gdk_analytic_bounds.c:1440) into a new
    oid BAT r; `limit` is the static bound (a value of type tp2) unless the
    per-row limit BAT l is given."""
    n = b.count()
    r = BAT(lib().mgdk_COLnew(0, TYPE_oid, n))
    keep = []
    bp = _valptr(tp2, limit, keep) if l is None else None
    _chk(lib().mgdk_GDKanalyticalwindowbounds(r.ptr, b.ptr, _p(p), _p(l), bp, b.ttype if tp1 is None else tp1,
                                              tp2, unit, preceding, second_half))
    return r


def GDKanalyticalsum(b, p, o, s, e, tp2, frame_type):
    """Windowed sum per row over its frame (gdk_analytic_func.c:1959)."""
    r = BAT(lib().mgdk_COLnew(0, tp2, max(1, b.count())))
    _chk(lib().mgdk_GDKanalyticalsum(r.ptr, _p(p), _p(o), b.ptr, _p(s), _p(e), b.ttype, tp2, frame_type))
    return r


BUN_NONE = (1 << 63) - 1


def _wres(tp, n):
    return BAT(lib().mgdk_COLnew(0, tp, max(1, n)))


def GDKanalyticaldiff(b, p=None, npbit=None):
    """gdk_analytic_bounds.c:95: bit column of the rows whose value differs
    from the row before (else p[i] / npbit / 0)."""
    r = _wres(TYPE_bit, b.count())
    ref = C.c_int8(npbit) if npbit is not None else None
    _chk(lib().mgdk_GDKanalyticaldiff(r.ptr, b.ptr, _p(p), C.cast(C.pointer(ref), C.c_void_p) if ref is not None
                                      else None, b.ttype))
    return r


def GDKanalyticalntile(b, p, n=None, ntile=None, tpe=None):
    """gdk_analytic_func.c:124: the tile number of every row in its
    partition; n a BAT of per-row tile counts or ntile one value of tpe."""
    keep = []
    tpe = tpe if tpe is not None else n.ttype
    r = _wres(tpe, b.count())
    _chk(lib().mgdk_GDKanalyticalntile(r.ptr, b.ptr, _p(p), _p(n), tpe,
                                       _valptr(tpe, ntile, keep) if n is None else None))
    return r


def GDKanalyticalfirst(b, s, e):
    """gdk_analytic_func.c:230: the first value of every row's frame."""
    r = _wres(b.ttype, b.count())
    _chk(lib().mgdk_GDKanalyticalfirst(r.ptr, b.ptr, s.ptr, e.ptr, b.ttype))
    return r


def GDKanalyticallast(b, s, e):
    """gdk_analytic_func.c:312: the last value of every row's frame."""
    r = _wres(b.ttype, b.count())
    _chk(lib().mgdk_GDKanalyticallast(r.ptr, b.ptr, s.ptr, e.ptr, b.ttype))
    return r


def GDKanalyticalnthvalue(b, s, e, t=None, nth=None):
    """gdk_analytic_func.c:421: the nth value of every row's frame (t: lng
    BAT of per-row n, or nth one value)."""
    r = _wres(b.ttype, b.count())
    ref = C.c_int64(nth) if t is None else None
    _chk(lib().mgdk_GDKanalyticalnthvalue(r.ptr, b.ptr, s.ptr, e.ptr, _p(t),
                                          C.cast(C.pointer(ref), C.c_void_p) if ref is not None else None,
                                          b.ttype))
    return r


def GDKanalyticallag(b, p, lag, default):
    """gdk_analytic_func.c:671: the value `lag` rows back in the partition."""
    keep = []
    r = _wres(b.ttype, b.count())
    _chk(lib().mgdk_GDKanalyticallag(r.ptr, b.ptr, _p(p), lag, _valptr(b.ttype, default, keep), b.ttype))
    return r


def GDKanalyticallead(b, p, lead, default):
    """gdk_analytic_func.c:823: the value `lead` rows ahead in the partition."""
    keep = []
    r = _wres(b.ttype, b.count())
    _chk(lib().mgdk_GDKanalyticallead(r.ptr, b.ptr, _p(p), lead, _valptr(b.ttype, default, keep), b.ttype))
    return r


def GDKanalyticalmin(b, p, o, s, e, frame_type):
    """gdk_analytic_func.c:1264: windowed min per row over its frame."""
    r = _wres(b.ttype, b.count())
    _chk(lib().mgdk_GDKanalyticalmin(r.ptr, _p(p), _p(o), b.ptr, _p(s), _p(e), b.ttype, frame_type))
    return r


def GDKanalyticalmax(b, p, o, s, e, frame_type):
    """gdk_analytic_func.c:1264: windowed max per row over its frame."""
    r = _wres(b.ttype, b.count())
    _chk(lib().mgdk_GDKanalyticalmax(r.ptr, _p(p), _p(o), b.ptr, _p(s), _p(e), b.ttype, frame_type))
    return r


def GDKanalyticalcount(b, p, o, s, e, ignore_nils, frame_type):
    """Windowed count per row over its frame (gdk_analytic_func.c:1626)."""
    r = BAT(lib().mgdk_COLnew(0, TYPE_lng, max(1, b.count())))
    _chk(lib().mgdk_GDKanalyticalcount(r.ptr, _p(p), _p(o), b.ptr, _p(s), _p(e), ignore_nils, b.ttype,
                                       frame_type))
    return r


def GDKanalyticalavg(b, p, o, s, e, frame_type):
    """Windowed dbl average per row over its frame
    (gdk/gdk_analytic_statistics.c:364)."""
    r = BAT(lib().mgdk_COLnew(0, TYPE_dbl, max(1, b.count())))
    _chk(lib().mgdk_GDKanalyticalavg(r.ptr, _p(p), _p(o), b.ptr, _p(s), _p(e), b.ttype, frame_type))
    return r


def GDKanalytical_stat(name, b1, b2, p, o, s, e, frame_type):
    """GDKanalytical_<name> (gdk_analytic_statistics.c:962-1443): name one of
    stddev_samp, stddev_pop, variance_samp, variance_pop (b2 None),
    covariance_samp, covariance_pop, correlation; dbl per row"""
    r = BAT(lib().mgdk_COLnew(0, TYPE_dbl, max(1, b1.count())))
    f = getattr(lib(), "mgdk_GDKanalytical_" + name)
    if b2 is None:
        _chk(f(r.ptr, _p(p), _p(o), b1.ptr, _p(s), _p(e), b1.ttype, frame_type))
    else:
        _chk(f(r.ptr, _p(p), _p(o), b1.ptr, b2.ptr, _p(s), _p(e), b1.ttype, frame_type))
    return r


def GDKanalyticalprod(b, p, o, s, e, tp2, frame_type):
    """Windowed product per row over its frame (gdk_analytic_func.c:2479)."""
    r = BAT(lib().mgdk_COLnew(0, tp2, max(1, b.count())))
    _chk(lib().mgdk_GDKanalyticalprod(r.ptr, _p(p), _p(o), b.ptr, _p(s), _p(e), b.ttype, tp2, frame_type))
    return r


def GDKanalyticalavginteger(b, p, o, s, e, frame_type):
    """Windowed average in b's integer type (gdk/gdk_analytic_statistics.c:631)."""
    r = BAT(lib().mgdk_COLnew(0, b.ttype, max(1, b.count())))
    _chk(lib().mgdk_GDKanalyticalavginteger(r.ptr, _p(p), _p(o), b.ptr, _p(s), _p(e), b.ttype, frame_type))
    return r


def group_sums_ordered(b, vals):
    """(extents, histo, keys-as-lng, [hge sums]) of GROUP BY an ordered b with
    exact sums of vals (mgdk_group_sums_ordered), or None when b's order or
    the types do not allow it (the caller runs BATgroup + BATgroupsum)."""
    e, h, k = P(), P(), P()
    nv = len(vals)
    sums = (P * nv)()
    vv = (P * nv)(*[v.ptr for v in vals])
    rc = lib().mgdk_group_sums_ordered(C.byref(e), C.byref(h), C.byref(k), sums, b.ptr, vv, nv)
    if rc < 0:
        raise _err()
    if rc > 0:
        return None
    return BAT(e), BAT(h), BAT(k), [BAT(sums[i]) for i in range(nv)]


def q6_fused(shipdate, discount, quantity, price, d0, d1, dlo, dhi, qmax):
    out = (C.c_uint64 * 2)()
    _chk(lib().mgdk_q6_fused(shipdate.ptr, discount.ptr, quantity.ptr, price.ptr, d0, d1, dlo, dhi,
                             qmax, C.cast(out, C.c_void_p)))
    return hge_to_int(out)


def q6_last_lines():
    """128-B column lines the last q6_fused on this thread read beyond shipdate
    (0 for a full-read variant)."""
    f = lib().mgdk_q6_last_sectors
    f.restype = C.c_ulonglong
    return int(f())


def q6_set_variant(variant, blocks_per_cu):
    """Launch variant of the fused Q6 (tuning / tests): 14 = full read (k_q6c),
    16 / 17 / 18 = predicate cascade (k_q6s) with 4 / 2 / 1 chunks in flight, 19 / 20 = the
    cascade with buffer loads (2 / 4 chunks; the default is 19 at 16 workgroups per CU)."""
    lib().mgdk_q6_set_variant(C.c_int(variant), C.c_int(blocks_per_cu))


def q6_opatatime(shipdate, discount, quantity, price, d0, d1, dlo, dhi, qmax):
    out = (C.c_uint64 * 2)()
    _chk(lib().mgdk_q6_opatatime(shipdate.ptr, discount.ptr, quantity.ptr, price.ptr, d0, d1, dlo,
                                 dhi, qmax, C.cast(out, C.c_void_p)))
    return hge_to_int(out)


def q1_fused(cols, dmax, maxgroups=64, fused=True):
    rows = (Q1Row * maxgroups)()
    n = C.c_int()
    fn = lib().mgdk_q1_fused if fused else lib().mgdk_q1_opatatime
    _chk(fn(cols["shipdate"].ptr, cols["returnflag"].ptr,
            cols["linestatus"].ptr, cols["quantity"].ptr,
            cols["extendedprice"].ptr, cols["discount"].ptr, cols["tax"].ptr,
            dmax, rows, maxgroups, C.byref(n)))
    res = []
    for i in range(n.value):
        r = rows[i]
        res.append(dict(returnflag=r.returnflag, linestatus=r.linestatus,
                        sum_qty=hge_to_int(r.sum_qty), sum_base_price=hge_to_int(r.sum_base_price),
                        sum_disc_price=hge_to_int(r.sum_disc_price),
                        sum_charge=hge_to_int(r.sum_charge), sum_disc=hge_to_int(r.sum_disc),
                        count_order=r.count_order, first_row=r.first_row,
                        avg_qty=r.avg_qty, avg_price=r.avg_price, avg_disc=r.avg_disc,
                        rem_qty=r.rem_qty, rem_price=r.rem_price, rem_disc=r.rem_disc))
    return res


LINEITEM_COLS = ("shipdate", "quantity", "extendedprice", "discount", "tax", "returnflag",
                 "linestatus")


def tpch_lineitem(seed, row0, n, sf_parts):
    """Generate the synthetic lineitem columns directly in HBM."""
    init()
    arr = (P * 7)()
    _chk(lib().mgdk_tpch_lineitem(seed, row0, n, sf_parts, arr))
    return {k: BAT(arr[i]) for i, k in enumerate(LINEITEM_COLS)}


def gen_window_column(seed, n, plen):
    """Ascending lng column + partition bits generated in HBM (config 5)."""
    init()
    v, p = P(), P()
    _chk(lib().mgdk_gen_window_column(seed, n, plen, C.byref(v), C.byref(p)))
    return BAT(v), BAT(p)


def sync():
    _chk(lib().mgdk_sync())


class QryCtx(C.Structure):
    """gdk/gdk_system.h:187 QryCtx (starttime, endtime in microseconds)."""
    _fields_ = [("starttime", C.c_int64), ("endtime", C.c_int64)]


QRY_TIMEOUT, QRY_INTERRUPT, QRY_DISCONNECT = -1, -2, -3


def set_qry_ctx(ctx):
    """MT_thread_set_qry_ctx for the calling thread (None clears it); the
    caller keeps ctx alive while it is set."""
    lib().mgdk_thread_set_qry_ctx(C.cast(C.pointer(ctx), C.c_void_p) if ctx is not None else None)


def usec():
    return lib().mgdk_usec()


def prof_enable(on=True):
    lib().mgdk_prof_enable(1 if on else 0)


def prof_get(kernel):
    ms, n = C.c_double(), C.c_uint64()
    lib().mgdk_prof_get(kernel.encode(), C.byref(ms), C.byref(n))
    return ms.value, n.value


def prof_reset():
    lib().mgdk_prof_reset()


# ---- multi-GPU exchange helpers ------------------------------------------------

def BAThashpartition(b, nparts):
    """(order BAT, counts list): positions of b grouped by destination part."""
    o = P()
    cnt = (C.c_uint64 * nparts)()
    _chk(lib().mgdk_BAThashpartition(C.byref(o), b.ptr, nparts, C.cast(cnt, C.c_void_p)))
    return BAT(o), [int(c) for c in cnt]


def BATlowerbound2(keys, pos, qk, qp):
    nq = len(qk)
    k = (C.c_int64 * max(1, nq))(*[int(x) for x in qk])
    p = (C.c_uint64 * max(1, nq))(*[int(x) for x in qp])
    out = (C.c_uint64 * max(1, nq))()
    _chk(lib().mgdk_BATlowerbound2(keys.ptr, _p(pos), C.cast(k, C.c_void_p), C.cast(p, C.c_void_p), nq,
                                   C.cast(out, C.c_void_p)))
    return [int(x) for x in out[:nq]]


def BATslice(b, lo, hi):
    """View of rows [lo, hi) sharing b's heap (gdk_batop.c BATslice)."""
    return BAT(lib().mgdk_BATslice(b.ptr, lo, hi))


def BATconstant(tp, val, n, hseqbase=0):
    keep = []
    return BAT(lib().mgdk_BATconstant(hseqbase, tp, _valptr(tp, val, keep), n))


def BATappend(b, n, s=None, force=False):
    """Append (the candidates s of) n to b in place (gdk_batop.c:1011)."""
    _chk(lib().mgdk_BATappend(b.ptr, n.ptr, _p(s), force))
    return b


def BATupload_device(b, dev_ptr, n):
    _chk(lib().mgdk_BATupload_device(b.ptr, C.c_void_p(dev_ptr), n))


def BATdownload_device(b, dev_ptr):
    _chk(lib().mgdk_BATdownload_device(b.ptr, C.c_void_p(dev_ptr)))
