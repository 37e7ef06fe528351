/*
 * mgdk.h -- C ABI of the MI355X-native GDK column-operator kernel
 * (libmgdk.so).
 *
 * Each entry point replaces one GDK function of the reference MonetDB
 * v11.52.0 and keeps its argument meaning, result properties, ownership and
 * error behaviour; the BAT descriptor is a flat struct whose heaps live in HBM.
 * A GDK maintainer binds these from the existing BAT* wrappers (see
 * INTEGRATION.md): marshal BAT -> mgdk_bat (device heap), call, wrap the
 * result.  No torch types, no C++ in the signatures.
 *
 * Conventions (gdk/gdk.h:1710,1947; gdk/gdk_bbp.c:3149-3183):
 *   - functions returning a BAT return a NEW transient BAT with one reference
 *     (release with mgdk_BBPunfix) or NULL after setting the thread-local
 *     error buffer (mgdk_GDKerrbuf), with the reference's SQLSTATE-prefixed
 *     messages ("22003!overflow in calculation ...");
 *   - functions returning int return 0 (GDK_SUCCEED) or -1 (GDK_FAIL);
 *   - inputs are borrowed; the library is thread safe, every calling thread
 *     gets its own HIP stream; results are complete when a call returns.
 */
#ifndef MGDK_H
#define MGDK_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uint64_t mgdk_oid;          /* gdk/gdk.h oid (SIZEOF_OID 8) */
typedef uint64_t mgdk_BUN;

/* GDK type ids, gdk/gdk.h:428-451 (HAVE_HGE build) */
enum {
	MGDK_void = 0, MGDK_msk = 1, MGDK_bit = 2, MGDK_bte = 3, MGDK_sht = 4,
	MGDK_int = 5, MGDK_oid = 6, MGDK_flt = 8, MGDK_dbl = 9, MGDK_lng = 10,
	MGDK_hge = 11, MGDK_date = 12, MGDK_daytime = 13, MGDK_timestamp = 14, MGDK_str = 16,
};

#define MGDK_OID_NIL ((mgdk_oid) 1 << 63)   /* oid_nil */
#define MGDK_BUN_NONE ((mgdk_BUN) INT64_MAX)  /* BUN_NONE, gdk/gdk.h:518 */

/* BAT descriptor: the column-side fields of gdk/gdk.h:712-804 (COLrec, BAT)
 * that the operators read or set.  theap/tvheap are HBM pointers. */
typedef struct mgdk_bat {
	int32_t ttype;          /* tail type (MGDK_*) */
	int32_t twidth;         /* bytes per tail value; str: offset width 1/2/4/8 */
	mgdk_BUN count;         /* BATcount */
	mgdk_oid hseqbase;      /* head sequence base */
	mgdk_oid tseqbase;      /* void: first oid; oid/other: MGDK_OID_NIL */
	void *theap;            /* tail values in HBM (NULL for void) */
	void *tvheap;           /* str: string heap in HBM (offsets are into it) */
	uint64_t tvheapsize;
	uint8_t tsorted, trevsorted, tkey, tnonil, tnil;
	uint8_t _pad[3];
	void *priv;             /* runtime-owned */
	/* knowledge kept with the column (gdk/gdk.h:721-726): positions proving
	 * the column is not sorted / not reverse sorted (0: unknown), the
	 * positions of its minimum / maximum (MGDK_BUN_NONE: unknown) and the
	 * estimated number of distinct values (0: unknown).  Operators set them
	 * on their results as the reference does and read them from inputs
	 * (BATgroup's maximum group id, BATjoin's cost model). */
	mgdk_BUN tnosorted, tnorevsorted;
	mgdk_BUN tminpos, tmaxpos;
	double tunique_est;
} mgdk_bat;

/* ---- runtime ---------------------------------------------------------- */
int mgdk_init(int device);                       /* select HIP device */
/* Order-dependent floating-point folds (Welford moments, the running mean of
 * a flt/dbl average, a running flt/dbl SUM) are replayed in the reference's
 * order, bit for bit, one lane per group or partition.  A single group or
 * partition of at least `rows` rows (default 2^20; MGDK_BUN_NONE: never)
 * takes the parallel form instead -- blocked folds combined pairwise (Chan
 * et al. for the moments) -- whose results differ from the sequential ones
 * by rounding only, within the bounds DESIGN.md states (a few n ulp).
 * Process-wide; returns the previous value. */
mgdk_BUN mgdk_set_fp_parallel_min(mgdk_BUN rows);
const char *mgdk_GDKerrbuf(void);                /* gdk.h:1947 GDKerrbuf */
void mgdk_GDKclrerr(void);
int mgdk_sync(void);                             /* drain calling thread's stream */
void *mgdk_stream(void);                         /* calling thread's hipStream_t */
uint64_t mgdk_mem_cursize(void);                 /* gdk_utils.c:1636 GDKmem_cursize */
void mgdk_mem_release_cache(void);

/* query context (gdk/gdk_system.h:187-210 QryCtx, MT_thread_set_qry_ctx):
 * endtime in microseconds of mgdk_usec() (0: none), or one of the negative
 * codes a client sets (gdk/gdk.h:2325-2327).  Every operator of the calling
 * thread tests it whenever it waits for its stream -- between its kernel
 * launches -- and fails with the reference's message ("Timeout was
 * reached!", "Query interrupted!", "Client is disconnected!"). */
typedef struct mgdk_qryctx {
	int64_t starttime;
	int64_t endtime;
} mgdk_qryctx;
#define MGDK_QRY_TIMEOUT (-1)
#define MGDK_QRY_INTERRUPT (-2)
#define MGDK_QRY_DISCONNECT (-3)
void mgdk_thread_set_qry_ctx(mgdk_qryctx *ctx);   /* NULL: no context */
mgdk_qryctx *mgdk_thread_get_qry_ctx(void);
int64_t mgdk_usec(void);                           /* GDKusec */

/* per-kernel timing with hipEvents on the library stream (ALGO tracing,
 * gdk/gdk_private.h:331): enable, then read totals per kernel name */
void mgdk_prof_enable(int on);
int mgdk_prof_get(const char *kernel, double *total_ms, uint64_t *launches);
void mgdk_prof_reset(void);

/* ---- BAT lifecycle (gdk/gdk_bat.c:292 COLnew, :298 BATdense,
 *      gdk/gdk_bbp.c:3149 BBPunfix, gdk/gdk_batop.c:1825 BATslice) ---- */
mgdk_bat *mgdk_COLnew(mgdk_oid hseq, int tt, mgdk_BUN cap);
mgdk_bat *mgdk_BATdense(mgdk_oid hseq, mgdk_oid tseq, mgdk_BUN cnt);
mgdk_bat *mgdk_BATconstant(mgdk_oid hseq, int tt, const void *val, mgdk_BUN cnt);
mgdk_bat *mgdk_BATslice(mgdk_bat *b, mgdk_BUN lo, mgdk_BUN hi);
void mgdk_BBPunfix(mgdk_bat *b);
/* host <-> HBM staging (the heap upload a GDK adaptor does once per BAT) */
int mgdk_BATupload(mgdk_bat *b, const void *host, mgdk_BUN n);
int mgdk_BATdownload(const mgdk_bat *b, void *host);
int mgdk_BATsetvheap(mgdk_bat *b, const void *host, uint64_t size);
int mgdk_BATdownload_vheap(const mgdk_bat *b, void *host);
/* BATmaskedcands (gdk/gdk_cand.h:232; gdk/gdk_cand.c:1366): a cand_mask
 * candidate list over [hseq, hseq + nr) from a msk BAT's bits (selected) or
 * their complement; rows past masked's end are candidates.  msk BATs (tail
 * = 32-bit words of bits, count = bits) are accepted wherever a candidate
 * list is: they stand for the oid list BATunmask makes of them */
mgdk_bat *mgdk_BATmaskedcands(mgdk_oid hseq, mgdk_BUN nr, mgdk_bat *masked, bool selected);
/* candidate-list algebra (gdk/gdk_cand.h:160-170): BATmergecand
 * (gdk/gdk_cand.c:46) the union, BATintersectcand (:184) the intersection,
 * BATdiffcand (:259) a minus b, of two candidate lists in any form; the
 * result is a new list (void when dense), hseqbase 0.  BATnegcands (:1296):
 * [tseq, tseq + nr) minus the sorted deletions odels, as a cand_except list
 * (void BAT + ccand_t {CAND_NEGOID} vheap) when a deletion falls inside */
mgdk_bat *mgdk_BATmergecand(mgdk_bat *a, mgdk_bat *b);
mgdk_bat *mgdk_BATintersectcand(mgdk_bat *a, mgdk_bat *b);
mgdk_bat *mgdk_BATdiffcand(mgdk_bat *a, mgdk_bat *b);
mgdk_bat *mgdk_BATnegcands(mgdk_oid tseq, mgdk_BUN nr, mgdk_bat *odels);
/* BATunmask (gdk/gdk_cand.h; gdk_cand.c:1464): a msk BAT or a cand_mask list
 * as the candidate list of its set bits -- a sorted oid list (virtualized
 * when dense), or for a mask list with more than half its bits set the
 * negative (cand_except) list of the unset ones, as the reference returns */
mgdk_bat *mgdk_BATunmask(mgdk_bat *b);

/* ---- select (gdk/gdk.h:2245-2246; gdk/gdk_select.c:1342, :2103) ------- */
mgdk_bat *mgdk_BATselect(mgdk_bat *b, mgdk_bat *s, const void *tl, const void *th,
			 bool li, bool hi, bool anti, bool nil_matches);
mgdk_bat *mgdk_BATthetaselect(mgdk_bat *b, mgdk_bat *s, const void *val, const char *op);

/* ---- project (gdk/gdk.h:2273; gdk/gdk_project.c:857) ------------------ */
mgdk_bat *mgdk_BATproject(mgdk_bat *l, mgdk_bat *r);
/* BATproject2 (gdk.h:2274, gdk_project.c:590): l projected over r1 ++ r2
 * (r2's head oids follow r1's); BATprojectchain (gdk.h:2275,
 * gdk_project.c:879): NULL-terminated chain bats[0] . bats[1] . ... */
mgdk_bat *mgdk_BATproject2(mgdk_bat *l, mgdk_bat *r1, mgdk_bat *r2);
mgdk_bat *mgdk_BATprojectchain(mgdk_bat **bats);

/* ---- calc (gdk/gdk_calc.h:36-44; gdk_calc_addsub.c:1480,1549,3166,3225,3280;
 *      gdk_calc_mul.c:2085,2092).  Constants are given as (pointer, type). */
mgdk_bat *mgdk_BATcalcadd(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp);
mgdk_bat *mgdk_BATcalcsub(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp);
mgdk_bat *mgdk_BATcalcmul(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp);
mgdk_bat *mgdk_BATcalcaddcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp);
mgdk_bat *mgdk_BATcalcsubcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp);
mgdk_bat *mgdk_BATcalcmulcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp);
mgdk_bat *mgdk_BATcalccstadd(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp);
mgdk_bat *mgdk_BATcalccstsub(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp);
mgdk_bat *mgdk_BATcalccstmul(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp);

/* comparisons (gdk/gdk_calc.h:66-84; gdk/gdk_calc_compare.h:827-964): bit
 * results (bte for cmp: -1/0/1), nil unless nil_matches (eq / ne) */
mgdk_bat *mgdk_BATcalclt(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcltcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstlt(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcle(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalclecst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstle(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcgt(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcgtcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstgt(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcge(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcgecst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstge(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalceq(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, bool nil_matches);
mgdk_bat *mgdk_BATcalceqcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, bool nil_matches);
mgdk_bat *mgdk_BATcalccsteq(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, bool nil_matches);
mgdk_bat *mgdk_BATcalcne(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, bool nil_matches);
mgdk_bat *mgdk_BATcalcnecst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, bool nil_matches);
mgdk_bat *mgdk_BATcalccstne(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, bool nil_matches);
mgdk_bat *mgdk_BATcalccmp(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalccmpcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstcmp(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
/* the same, op 0..6 = lt le gt ge eq ne cmp; b1 / b2 NULL take v1 / v2 */
mgdk_bat *mgdk_BATcalccmp_op(int op, mgdk_bat *b1, const void *v1, int t1, mgdk_bat *b2, const void *v2,
			     int t2, mgdk_bat *s1, mgdk_bat *s2, bool nil_matches);
/* between (gdk/gdk_calc.h:85-88; gdk/gdk_calc.c:3968-4206); constants of type vt */
mgdk_bat *mgdk_BATcalcbetween(mgdk_bat *b, mgdk_bat *lo, mgdk_bat *hi, mgdk_bat *s, mgdk_bat *slo, mgdk_bat *shi,
			      bool symmetric, bool linc, bool hinc, bool nils_false, bool anti);
mgdk_bat *mgdk_BATcalcbetweencstcst(mgdk_bat *b, const void *lo, const void *hi, int vt, mgdk_bat *s,
				    bool symmetric, bool linc, bool hinc, bool nils_false, bool anti);
mgdk_bat *mgdk_BATcalcbetweenbatcst(mgdk_bat *b, mgdk_bat *lo, const void *hi, int vt, mgdk_bat *s, mgdk_bat *slo,
				    bool symmetric, bool linc, bool hinc, bool nils_false, bool anti);
mgdk_bat *mgdk_BATcalcbetweencstbat(mgdk_bat *b, const void *lo, mgdk_bat *hi, int vt, mgdk_bat *s, mgdk_bat *shi,
				    bool symmetric, bool linc, bool hinc, bool nils_false, bool anti);
/* BATconvert (gdk/gdk_calc.h:118; gdk_calc_convert.c:1415): numeric, bit and
 * oid types, DECIMAL rescaling (scale1 -> scale2) with the precision check */
mgdk_bat *mgdk_BATconvert(mgdk_bat *b, mgdk_bat *s, int tp, uint8_t scale1, uint8_t scale2, uint8_t precision);
/* BATcalcnot (gdk/gdk_calc.h:23; gdk_calc.c:41) */
mgdk_bat *mgdk_BATcalcnot(mgdk_bat *b, mgdk_bat *s);
/* the rest of gdk_calc.c's element-wise operators (gdk/gdk_calc.h:15-93):
 * negate / absolute (b's type), iszero (bit), sign (bte), isnil / isnotnil
 * (bit, never nil), incr / decr (b's type, overflow checked), min / max and
 * their _no_nil forms (ATOMtype of the inputs; a constant v of type vt in
 * the cst forms), and / or / xor (bit: three-valued; integers bitwise, a
 * result equal to nil an overflow), lsh / rsh ("shift operand too large"),
 * ifthenelse (b of type bit; a nil condition takes the else branch; then /
 * else BATs or constants c of type ct).  Messages and result properties as
 * the reference's. */
mgdk_bat *mgdk_BATcalcnegate(mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcabsolute(mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalciszero(mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcsign(mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcisnil(mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcisnotnil(mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcincr(mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcdecr(mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcmin(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcmax(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcmin_no_nil(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcmax_no_nil(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcmincst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcmaxcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcmincst_no_nil(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcmaxcst_no_nil(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstmin(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstmax(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstmin_no_nil(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstmax_no_nil(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcand(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcandcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstand(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcor(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcorcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstor(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcxor(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcxorcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstxor(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalclsh(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalclshcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstlsh(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcrsh(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2);
mgdk_bat *mgdk_BATcalcrshcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s);
mgdk_bat *mgdk_BATcalccstrsh(const void *v, int vt, mgdk_bat *b, mgdk_bat *s);
mgdk_bat *mgdk_BATcalcifthenelse(mgdk_bat *b, mgdk_bat *b1, mgdk_bat *b2);
mgdk_bat *mgdk_BATcalcifthenelsecst(mgdk_bat *b, mgdk_bat *b1, const void *c2, int ct);
mgdk_bat *mgdk_BATcalcifthencstelse(mgdk_bat *b, const void *c1, int ct, mgdk_bat *b2);
mgdk_bat *mgdk_BATcalcifthencstelsecst(mgdk_bat *b, const void *c1, const void *c2, int ct);
/* division / modulo (gdk/gdk_calc.h:45-50; gdk_calc_div.c:1945, gdk_calc_mod.c:1179) */
mgdk_bat *mgdk_BATcalcdiv(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp);
mgdk_bat *mgdk_BATcalcdivcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp);
mgdk_bat *mgdk_BATcalccstdiv(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp);
mgdk_bat *mgdk_BATcalcmod(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp);
mgdk_bat *mgdk_BATcalcmodcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp);
mgdk_bat *mgdk_BATcalccstmod(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp);

/* ---- aggregates (gdk/gdk_calc.h:127-147; gdk/gdk_aggr.c:900,1018,1996,3069,
 *      3487-3844) --------------------------------------------------------- */
int mgdk_BATsum(void *res, int tp, mgdk_bat *b, mgdk_bat *s, bool skip_nils, bool nil_if_empty);
mgdk_bat *mgdk_BATgroupsum(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);
mgdk_bat *mgdk_BATgroupcount(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);
/* BATgroupavg (gdk_calc.h:129, gdk_aggr.c:1801): dbl averages; tp must be
 * MGDK_dbl; cntsp may be NULL; scale divides by 10^scale */
/* BATcalcavg (gdk_calc.h; gdk_aggr.c:2987): average of b[s] without nils into
 * *avg (nil: NaN when there is none) and their number into *vals (may be
 * NULL); integers (dbl) exact sum / n, flt / dbl the running mean in
 * candidate order; divided by 10^scale.  An hge column whose sum leaves 128
 * bits is refused (the reference continues with a remainder recurrence) */
int mgdk_BATcalcavg(mgdk_bat *b, mgdk_bat *s, double *avg, mgdk_BUN *vals, int scale);
int mgdk_BATgroupavg(mgdk_bat **bnp, mgdk_bat **cntsp, mgdk_bat *b, mgdk_bat *g, mgdk_bat *e,
		     mgdk_bat *s, int tp, bool skip_nils, int scale);
/* BATgroupavg3combine (gdk_calc.h, gdk_aggr.c:2634): combine per-row partial
 * (avg, rem, cnt) triples of BATgroupavg3 into the rounded group averages */
mgdk_bat *mgdk_BATgroupavg3combine(mgdk_bat *avg, mgdk_bat *rem, mgdk_bat *cnt, mgdk_bat *g, mgdk_bat *e,
				   bool skip_nils);
int mgdk_BATgroupavg3(mgdk_bat **avgp, mgdk_bat **remp, mgdk_bat **cntp,
		      mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, bool skip_nils);
/* grouped statistics (gdk_calc.h:156-167): Welford moments per group in
 * candidate order (dogroupstdev gdk_aggr.c:4612, BATgroupstdev_sample :4778,
 * _population :4785, BATgroupvariance_sample :4793, _population :4801;
 * dogroupcovariance :4851, BATgroupcovariance_sample :5000, _population
 * :5007; BATgroupcorrelation :5057); dbl results, tp is not read */
mgdk_bat *mgdk_BATgroupstdev_sample(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);
mgdk_bat *mgdk_BATgroupstdev_population(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp,
					bool skip_nils);
mgdk_bat *mgdk_BATgroupvariance_sample(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);
mgdk_bat *mgdk_BATgroupvariance_population(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp,
					   bool skip_nils);
mgdk_bat *mgdk_BATgroupcovariance_sample(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp,
					 bool skip_nils);
mgdk_bat *mgdk_BATgroupcovariance_population(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s,
					     int tp, bool skip_nils);
mgdk_bat *mgdk_BATgroupcorrelation(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp,
				   bool skip_nils);
/* whole-column forms (gdk_calc.h:154-164; calcvariance gdk_aggr.c:4276,
 * BATcalcstdev_population :4327, _sample :4341, BATcalcvariance_population
 * :4355, _sample :4369; calccovariance :4404, BATcalccovariance_population
 * :4449, _sample :4464; BATcalccorrelation :4503): nil (NaN) results when
 * undefined; errors (overflow, type) leave a message in mgdk_GDKerrbuf */
double mgdk_BATcalcstdev_population(double *avgp, mgdk_bat *b);
double mgdk_BATcalcstdev_sample(double *avgp, mgdk_bat *b);
double mgdk_BATcalcvariance_population(double *avgp, mgdk_bat *b);
double mgdk_BATcalcvariance_sample(double *avgp, mgdk_bat *b);
double mgdk_BATcalccovariance_population(mgdk_bat *b1, mgdk_bat *b2);
double mgdk_BATcalccovariance_sample(mgdk_bat *b1, mgdk_bat *b2);
double mgdk_BATcalccorrelation(mgdk_bat *b1, mgdk_bat *b2);
/* quantiles (gdk_calc.h:135-138; doBATgroupquantile gdk_aggr.c:3881,
 * BATgroupmedian :4225, BATgroupquantile :4233, BATgroupmedian_avg :4241,
 * BATgroupquantile_avg :4247): g may be NULL (one result); _avg
 * interpolates and returns dbl */
mgdk_bat *mgdk_BATgroupmedian(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);
mgdk_bat *mgdk_BATgroupquantile(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, double quantile,
				bool skip_nils);
mgdk_bat *mgdk_BATgroupmedian_avg(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);
mgdk_bat *mgdk_BATgroupquantile_avg(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, double quantile,
				    bool skip_nils);
mgdk_bat *mgdk_BATgroupmin(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);
mgdk_bat *mgdk_BATgroupmax(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);
/* BATmin / BATmax / BATmin_skipnil / BATmax_skipnil (gdk/gdk.h;
 * gdk_aggr.c:3570-3844): the column's smallest / largest value as the
 * reference finds it -- a cached tminpos / tmaxpos, an ordered column's end,
 * else the first row holding the extreme (without skipnil the first nil) --
 * nil for an empty or all-nil column; the position found is cached in b.
 * aggr: a buffer of the value's width, or NULL for a copy from malloc (str:
 * the NUL-terminated string; release it with mgdk_free).  NULL on error
 * ("non-linear type" for msk). */
void *mgdk_BATmin(mgdk_bat *b, void *aggr);
void *mgdk_BATmax(mgdk_bat *b, void *aggr);
void *mgdk_BATmin_skipnil(mgdk_bat *b, void *aggr, bool skipnil);
void *mgdk_BATmax_skipnil(mgdk_bat *b, void *aggr, bool skipnil);
void mgdk_free(void *p);
/* BATprod (gdk/gdk.h; gdk_aggr.c:1650): the product of b's candidates into
 * *res of type tp (bte..hge, flt, dbl; doprod's type table), "22003!overflow
 * in product aggregate." as the reference raises it; BATgroupprod (:1575)
 * the product per group (nil for an empty group) */
int mgdk_BATprod(void *res, int tp, mgdk_bat *b, mgdk_bat *s, bool skip_nils, bool nil_if_empty);
mgdk_bat *mgdk_BATgroupprod(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils);

/* BATguess_uniques (gdk/gdk.h:2268; gdk_join.c:3572): the join cost model's
 * estimate of distinct values among b's candidates s (NULL: all of b; the
 * reference takes a struct canditer); a full column's estimate is cached in
 * b->tunique_est.  The 1000-row sample is evenly spaced (the reference's
 * BATsample is random).  MGDK_BUN_NONE on an error */
mgdk_BUN mgdk_BATguess_uniques(mgdk_bat *b, mgdk_bat *s);
/* BATcount_no_nil (gdk/gdk.h; gdk_batop.c:3078): b's candidates whose
 * value is not nil (tnonil / msk: every candidate; void: none when the
 * sequence is nil); a count of every row sets b's tnonil.  0 for a NULL b;
 * MGDK_BUN_NONE (message set) on a device error, which the reference has no
 * way to report */
mgdk_BUN mgdk_BATcount_no_nil(mgdk_bat *b, mgdk_bat *s);

/* ---- group (gdk/gdk.h:1447; gdk/gdk_group.c:1347) --------------------- */
int mgdk_BATgroup(mgdk_bat **groups, mgdk_bat **extents, mgdk_bat **histo,
		  mgdk_bat *b, mgdk_bat *s, mgdk_bat *g, mgdk_bat *e, mgdk_bat *h);

/* ---- join (gdk/gdk.h:2266; gdk/gdk_join.c:4451): the reference's choice
 * of selectjoin / mergejoin_void / mergejoin / hashjoin (and swapped),
 * which fixes the result order and properties ---------------------------- */
int mgdk_BATjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r,
		 mgdk_bat *sl, mgdk_bat *sr, bool nil_matches, mgdk_BUN estimate);
/* the left-output join family (gdk/gdk.h:2264-2272; gdk_join.c:4320-4407,
 * through leftjoin :4049): BATintersect / BATsemijoin the left candidates
 * with a match (BATsemijoin's r2p, as algebra.semijoin binds it,
 * algebra.c:1792: the match kept for each, the one leftjoin's algorithm
 * keeps), BATdiff those without (not_in: SQL NOT IN), as candidate lists;
 * BATleftjoin / BATouterjoin the (left, match) pairs in left order (outer: a
 * miss pairs with nil), a left candidate's several matches in the order
 * leftjoin's algorithm choice gives them (joinkinds.hip; match_one raises
 * "more than one match").  Keys of every join type: integers, oid, temporal,
 * flt / dbl and str (as BATjoin's order-preserving images) */
mgdk_bat *mgdk_BATintersect(mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, bool nil_matches,
			    bool max_one, mgdk_BUN estimate);
mgdk_bat *mgdk_BATdiff(mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, bool nil_matches, bool not_in,
		       mgdk_BUN estimate);
int mgdk_BATsemijoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		     bool nil_matches, bool max_one, mgdk_BUN estimate);
int mgdk_BATleftjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		     bool nil_matches, mgdk_BUN estimate);
int mgdk_BATouterjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		      bool nil_matches, bool match_one, mgdk_BUN estimate);
/* BATmarkjoin (gdk/gdk.h; gdk_join.c:4367, leftjoin with nil_on_miss): every
 * left candidate once (r2p NULL: semi) or with its match (nil on a miss), and
 * the mark column r3 (bit): TRUE on a match; on a miss nil when the left value
 * is nil or a right candidate is nil, else FALSE; no right candidates: FALSE.
 * With r2p, one row per match in leftjoin's order, as BATouterjoin */
int mgdk_BATmarkjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat **r3p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl,
		     mgdk_bat *sr, mgdk_BUN estimate);
/* BATthetajoin (gdk/gdk.h; gdk_join.c:4409, nested loop thetajoin :3699):
 * op JOIN_EQ 0 (= BATjoin), JOIN_LT -1, JOIN_LE -2, JOIN_GT 1, JOIN_GE 2,
 * JOIN_NE -3 (gdk.h:2237-2243); the pairs in left-candidate order, each left
 * candidate's matches in right-candidate order.  BATbandjoin (gdk_join.c:
 * 4626): r - c1 <= l <= r + c2 (linc / hinc: the ends included), c1 / c2
 * point at values of the columns' type */
int mgdk_BATthetajoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, int op,
		      bool nil_matches, mgdk_BUN estimate);
int mgdk_BATbandjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		     const void *c1, const void *c2, bool linc, bool hinc, mgdk_BUN estimate);
/* BATrangejoin (gdk_join.c:5422, rangejoin :5067): l within [rl, rh] of each
 * right candidate (rl, rh aligned); not anti / symmetric and l ordered:
 * right-major pairs by binary search, otherwise the nested loop's
 * left-major pairs with BETWEEN's three-valued logic */
int mgdk_BATrangejoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *rl, mgdk_bat *rh, mgdk_bat *sl,
		      mgdk_bat *sr, bool linc, bool hinc, bool anti, bool symmetric, mgdk_BUN estimate);
/* BATsubcross (gdk/gdk.h; gdk_cross.c:138, BATcrossci :22): every (left,
 * right) candidate pair, left-major (r1 the left oid, r2 the right one); one
 * candidate on a side gives a candidate slice and a constant column, none two
 * empty dense columns.  BAToutercross (gdk_cross.c:153): no right candidate
 * pairs each left candidate with nil (a void column of nil oids).  max_one:
 * "more than one match" when a left candidate meets several right ones */
int mgdk_BATsubcross(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		     bool max_one);
int mgdk_BAToutercross(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		       bool max_one);
/* gdk/gdk.h:1524-1525 (gdk_batop.c:2002, :2181): whether b is sorted /
 * reverse sorted; what is found is recorded in b (tsorted, trevsorted,
 * tkey, tnosorted, tnorevsorted) as the reference does */
bool mgdk_BATordered(mgdk_bat *b);
bool mgdk_BATordered_rev(mgdk_bat *b);

/* ---- sort (gdk/gdk.h:1526; gdk/gdk_batop.c:2342) ---------------------- */
int mgdk_BATsort(mgdk_bat **sorted, mgdk_bat **order, mgdk_bat **groups,
		 mgdk_bat *b, mgdk_bat *o, mgdk_bat *g, bool reverse, bool nilslast, bool stable);
/* order index (gdk/gdk.h:1590-1592; gdk_orderidx.c:184 BATorderidx, :74
 * BATcheckorderidx, :534 OIDXdestroy): the oids of b in sorted order kept
 * with b (stable: ties in oid order).  As in the reference, BATsort uses it
 * (unstable sorts, and stable ones when it was built stable) and builds one
 * when it returns an order of a column that is not a view; BATrangejoin
 * probes an unsorted l through it (right-major pairs, the index's order per
 * right candidate); a written tail drops it.  mgdk_BATorderidx_get: a copy
 * of the index as an oid BAT (NULL without an error when b has none) */
int mgdk_BATorderidx(mgdk_bat *b, bool stable);
bool mgdk_BATcheckorderidx(mgdk_bat *b);
void mgdk_OIDXdestroy(mgdk_bat *b);
mgdk_bat *mgdk_BATorderidx_get(mgdk_bat *b, bool *stable);
/* gdk_unique.c:30 BATunique: candidate list of the first occurrence of
 * every distinct value of b[s] */
mgdk_bat *mgdk_BATunique(mgdk_bat *b, mgdk_bat *s);
/* gdk_firstn.c:1280 BATfirstn: candidate list of the n first rows of b[s]
 * in (g, b) order (asc / nilslast); gids != NULL or distinct: every row
 * tied with the last one is included (as the reference); otherwise the
 * first tied rows in candidate order (the reference: whichever its heap
 * kept) */
int mgdk_BATfirstn(mgdk_bat **topn, mgdk_bat **gids, mgdk_bat *b, mgdk_bat *s, mgdk_bat *g, mgdk_BUN n,
		   bool asc, bool nilslast, bool distinct);

/* ---- window bounds (gdk/gdk_analytic.h:27-30;
 *      gdk/gdk_analytic_bounds.c:1440) ------------------------------------- */
int mgdk_GDKanalyticalwindowbounds(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_bat *l,
				   const void *bound, int tp1, int tp2, int unit,
				   bool preceding, mgdk_oid first_half);

/* ---- fused MAL pipelines (one pass over the lineitem columns; same
 *      results as the op-at-a-time plans of SURVEY.md §3.2/§3.3) --------- */
/* GROUP BY an ordered key with exact sums: the results of
 * BATgroup(&g, &e, &h, b, NULL, NULL, NULL, NULL) (gdk/gdk_group.c:940-975),
 * BATgroupsum(vals[v], g, e, NULL, TYPE_hge, true) for each value column
 * (gdk/gdk_aggr.c:1009) and BATproject(e, b) widened to lng, without the
 * group-id column: *extents (oid), *histo (lng), *keys (lng), sums[v] (hge).
 * b: int / lng / oid / date / timestamp keys, sorted or reverse sorted (its
 * order is looked up as BATordered does); vals: 1..4 int or lng columns of
 * one width aligned with b.  Returns 0, 1 when not applicable (the caller
 * runs the GDK operators), -1 on error.  The local step of the mergetable
 * GROUP BY plan (opt_mergetable.c:1496-1670) in dist_group_aggr. */
int mgdk_group_sums_ordered(mgdk_bat **extents, mgdk_bat **histo, mgdk_bat **keys, mgdk_bat **sums, mgdk_bat *b,
			    mgdk_bat **vals, int nvals);
/* Q6: sum(price*disc) over rows with d0 <= shipdate < d1, dlo <= disc <= dhi,
 * qty < qmax; result hge written to *revenue (16 bytes). */
int mgdk_q6_fused(mgdk_bat *shipdate, mgdk_bat *discount, mgdk_bat *quantity,
		  mgdk_bat *extendedprice, int32_t d0, int32_t d1, int64_t dlo,
		  int64_t dhi, int64_t qmax, void *revenue);
/* 128-byte lines of discount / quantity / extendedprice the calling thread's
 * last mgdk_q6_fused read (its predicate cascade reads a column's line only
 * when one of the line's rows passed the earlier predicates; shipdate is
 * read whole).  0 after a full-read launch variant.  Measurement only. */
unsigned long long mgdk_q6_last_sectors(void);
typedef struct mgdk_q1row {
	uint8_t returnflag, linestatus, _pad[6];   /* str heap offsets */
	int64_t sum_qty[2], sum_base_price[2], sum_disc_price[2], sum_charge[2]; /* hge lo,hi */
	int64_t sum_disc[2];
	int64_t count_order;
	mgdk_oid first_row;
	/* BATgroupavg3 of quantity, extendedprice, discount: the average rounded
	 * half away from zero and its remainder (gdk_aggr.c:1996-2095) */
	int64_t avg_qty, avg_price, avg_disc;
	int64_t rem_qty, rem_price, rem_disc;
} mgdk_q1row;
/* Q1 groups (first-occurrence numbering, BATgroup semantics); returns the
 * number of groups in *ngroups (<= maxgroups). */
int mgdk_q1_fused(mgdk_bat *shipdate, mgdk_bat *returnflag, mgdk_bat *linestatus,
		  mgdk_bat *quantity, mgdk_bat *extendedprice, mgdk_bat *discount,
		  mgdk_bat *tax, int32_t dmax, mgdk_q1row *rows, int maxgroups, int *ngroups);

/* the same two plans run operator by operator through the entry points
 * above (what MonetDB's interpreter executes without the fused rewrite) */
int mgdk_q6_opatatime(mgdk_bat *shipdate, mgdk_bat *discount, mgdk_bat *quantity,
		      mgdk_bat *extendedprice, int32_t d0, int32_t d1, int64_t dlo,
		      int64_t dhi, int64_t qmax, void *revenue);
int mgdk_q1_opatatime(mgdk_bat *shipdate, mgdk_bat *returnflag, mgdk_bat *linestatus,
		      mgdk_bat *quantity, mgdk_bat *extendedprice, mgdk_bat *discount,
		      mgdk_bat *tax, int32_t dmax, mgdk_q1row *rows, int maxgroups, int *ngroups);

/* ---- synthetic TPC-H lineitem generated directly in HBM (same values as
 *      oracle/tpch_gen.c); cols: shipdate(date), quantity, extendedprice,
 *      discount, tax (lng), returnflag, linestatus (str, 1-byte offsets) -- */
int mgdk_tpch_lineitem(uint64_t seed, uint64_t row0, uint64_t n, uint64_t sf_parts,
		       mgdk_bat **cols /* [7] */);
/* RANGE-window input of BASELINE config 5: n ascending lng values (gaps
 * U[0,4]) and a partition-start bit column (one partition per plen rows) */
int mgdk_gen_window_column(uint64_t seed, uint64_t n, uint64_t plen, mgdk_bat **vals,
			   mgdk_bat **parts);

/* gdk_analytic_func.c:1959 GDKanalyticalsum / :1626 GDKanalyticalcount
 * (gdk_analytic.h:38-39): per-row aggregate over the row's frame.
 * frame_type 3 = unbounded preceding .. current row (+ peers), 4 = current
 * row (+ peers) .. unbounded following, 5 = whole partition, 6 = current
 * row, otherwise [s[i], e[i]) from GDKanalyticalwindowbounds.  p / o: bit
 * BATs of partition / peer-group starts.  r is caller-allocated (count(b)
 * slots; tp2 = lng or hge for sums, lng for counts). */
int mgdk_GDKanalyticalsum(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
			  int tp1, int tp2, int frame_type);
int mgdk_GDKanalyticalcount(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
			    bool ignore_nils, int tpe, int frame_type);
/* gdk_analytic_func.c :124 GDKanalyticalntile, :230 GDKanalyticalfirst,
 * :312 GDKanalyticallast, :421 GDKanalyticalnthvalue, :671 GDKanalyticallag,
 * :823 GDKanalyticallead, :1264 GDKanalyticalmin / max (gdk_analytic.h:
 * 23-37): r is caller-allocated (count(b) slots of type tpe); p: bit BAT of
 * partition starts (NULL: one partition), o: peer-group starts, s / e:
 * frame bounds.  ntile: exactly one of n (per-row tile counts of type tpe)
 * and ntile (one value of tpe); nth_value: t (lng per row) or *pnth; lag /
 * lead: BUN_NONE (INT64_MAX) gives all nils. */
/* gdk_analytic_bounds.c:95 GDKanalyticaldiff (gdk_analytic.h:21): r (a
 * caller-allocated bit BAT) marks the rows whose value differs from the row
 * before (the partition / peer starts of a sorted column), else p[i] /
 * *npbit / 0; fixed-width types and str */
int mgdk_GDKanalyticaldiff(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, const int8_t *npbit, int tpe);
int mgdk_GDKanalyticalntile(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_bat *n, int tpe, const void *ntile);
int mgdk_GDKanalyticalfirst(mgdk_bat *r, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe);
int mgdk_GDKanalyticallast(mgdk_bat *r, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe);
int mgdk_GDKanalyticalnthvalue(mgdk_bat *r, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, mgdk_bat *t, const int64_t *pnth,
			       int tpe);
int mgdk_GDKanalyticallag(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_BUN lag, const void *default_value, int tpe);
int mgdk_GDKanalyticallead(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_BUN lead, const void *default_value, int tpe);
int mgdk_GDKanalyticalmin(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
			  int frame_type);
int mgdk_GDKanalyticalmax(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
			  int frame_type);
/* gdk_analytic_statistics.c:364 GDKanalyticalavg (gdk_analytic.h:41): dbl
 * average per row over its frame, frame kinds as above; r is a
 * caller-allocated dbl BAT; tpe = type of b (bte..lng, flt, dbl) */
int mgdk_GDKanalyticalavg(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
			  int tpe, int frame_type);
/* gdk_analytic_statistics.c:631 GDKanalyticalavginteger (gdk_analytic.h:42):
 * the average in b's integer type (bte..lng), rounded half away from zero;
 * r is a caller-allocated BAT of that type */
/* gdk_analytic_statistics.c:897-965 GDK_ANALYTICAL_STDEV_VARIANCE
 * (gdk_analytic.h:44-47), :1120-1188 GDK_ANALYTICAL_COVARIANCE (:48-49),
 * :1379 GDKanalytical_correlation (:50): dbl per row over its frame (frame
 * kinds as GDKanalyticalsum; others through the reference's segment tree);
 * r is a caller-allocated dbl BAT; tpe = type of b (bte..hge, flt, dbl) */
int mgdk_GDKanalytical_stddev_samp(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
				   int tpe, int frame_type);
int mgdk_GDKanalytical_stddev_pop(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
				  int tpe, int frame_type);
int mgdk_GDKanalytical_variance_samp(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
				     int tpe, int frame_type);
int mgdk_GDKanalytical_variance_pop(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
				    int tpe, int frame_type);
int mgdk_GDKanalytical_covariance_samp(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b1, mgdk_bat *b2,
				       mgdk_bat *s, mgdk_bat *e, int tpe, int frame_type);
int mgdk_GDKanalytical_covariance_pop(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s,
				      mgdk_bat *e, int tpe, int frame_type);
int mgdk_GDKanalytical_correlation(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s,
				   mgdk_bat *e, int tpe, int frame_type);
/* gdk_analytic_func.c:2479 GDKanalyticalprod (gdk_analytic.h:40): the
 * product in tp2 (bte..hge from narrower or equal integers, flt from flt,
 * dbl from flt / dbl) with the reference's overflow checks */
int mgdk_GDKanalyticalprod(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tp1,
			   int tp2, int frame_type);
int mgdk_GDKanalyticalavginteger(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
				 int tpe, int frame_type);

/* ---- compressed column inputs (sql/backends/monet5/dict.c, for.c):
 *      a DICT column is codes o (bte/sht/int, read unsigned) + the
 *      dictionary u of distinct values; a FOR column is bte/sht offsets
 *      from one minimum.  Selections run on the codes. ---------------- */
int mgdk_DICTcompress(mgdk_bat **o, mgdk_bat **u, mgdk_bat *b, bool ordered, bool smallest_type); /* dict.c:110 */
mgdk_bat *mgdk_DICTdecompress(mgdk_bat *o, mgdk_bat *u);                                         /* dict.c:352 */
mgdk_bat *mgdk_DICTselect(mgdk_bat *lo, mgdk_bat *lc, mgdk_bat *lv, const void *l, const void *h,
			  bool li, bool hi, bool anti);                                         /* dict.c:926 */
mgdk_bat *mgdk_DICTthetaselect(mgdk_bat *lo, mgdk_bat *lc, mgdk_bat *lv, const void *v, const char *op); /* dict.c:788 */
mgdk_bat *mgdk_FORcompress(mgdk_bat *b, int64_t *minval);                                          /* for.c:148 */
mgdk_bat *mgdk_FORdecompress(mgdk_bat *o, int64_t minval, int tp);                                 /* for.c:30 */

/* ---- persistent BAT heaps -> HBM (gdk_bbp.c:595-714 BBP.dir, gdk_heap.c:729
 *      HEAPload): entries of a dbfarm's bat/BBP.dir, and one BAT's tail
 *      (+ string heap) streamed into device memory ------------------------ */
typedef struct mgdk_bbpentry {
	int64_t batid;
	char name[129];
	char type[33];
	int32_t tt;             /* MGDK_* id, -1: unknown type */
	int32_t width;
	int32_t var;            /* has a variable-size heap */
	uint32_t props;         /* BBP.dir property bits (sorted 0x1, revsorted 0x80, key 0x100,
	                           dense 0x200, nonil 0x400, nil 0x800) */
	uint64_t count;
	mgdk_oid hseqbase;
	mgdk_oid tseqbase;
	uint64_t free;          /* tail bytes */
	uint64_t vfree;         /* string heap bytes */
	char tail[256];         /* file names relative to the bat directory */
	char theap[256];
} mgdk_bbpentry;
int mgdk_BBPreaddir(const char *bbp_dir_file, mgdk_bbpentry *out, int maxn, int *n);
mgdk_bat *mgdk_BATload(const char *bat_dir, const mgdk_bbpentry *e);

/* ---- multi-GPU exchange steps (SURVEY.md §8 e).  The reference shards a
 *      plan by row ranges (opt_mitosis.c:150-230) and re-aggregates packed
 *      partials (opt_mergetable.c:1496-1885); across GPUs the group / join
 *      shuffles need a partitioning by VALUE and RCCL buffers: ----------- */
/* order := positions of b (as oids, hseqbase-based) grouped by destination
 * part hash(value) mod-scaled to [0, nparts), stable inside a part;
 * counts[nparts] rows per part.  Integer types and void. */
int mgdk_BAThashpartition(mgdk_bat **order, mgdk_bat *b, int nparts, uint64_t *counts);
/* out[q] = number of rows of the run sorted by (keys, pos) that are below
 * (qk[q], qp[q]); pos NULL: positions 0..n-1 (sample-sort splitters) */
int mgdk_BATlowerbound2(const mgdk_bat *keys, const mgdk_bat *pos, const int64_t *qk, const uint64_t *qp,
			int nq, uint64_t *out);
/* gdk_batop.c:1011 BATappend: append the candidates s of n to b in place
 * (fixed-width tails) */
int mgdk_BATappend(mgdk_bat *b, mgdk_bat *n, mgdk_bat *s, bool force);
/* device-to-device copies between a BAT tail and a device buffer (RCCL) */
int mgdk_BATupload_device(mgdk_bat *b, const void *dev, mgdk_BUN n);
int mgdk_BATdownload_device(const mgdk_bat *b, void *dev);

#ifdef __cplusplus
}
#endif
#endif
