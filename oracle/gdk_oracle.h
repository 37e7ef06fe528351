/*
 * gdk_oracle.h -- CPU restatement of MonetDB GDK's column-operator semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X product path (libmgdk.so).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product never links,
 * calls or falls back to it.
 *
 * It restates (does not copy) the algorithms of the reference
 * rohan-flutterint/MonetDB v11.52.0 (/root/reference, read-only):
 *   select      gdk/gdk_select.c:1342-2084 (BATselect), :2103-2154 (BATthetaselect),
 *               scan normalisation :300-446
 *   candidates  gdk/gdk_cand.c:407 (canditer_init clipping)
 *   project     gdk/gdk_project.c:590-857
 *   calc        gdk/gdk_calc_addsub.c, gdk/gdk_calc_mul.c:23-132,2020-2092,
 *               overflow rules gdk/gdk_calc_private.h:38-140; compare, between,
 *               convert, not, div, mod (gdk_oracle_calc.c)
 *   aggregates  gdk/gdk_aggr.c:65 (BATgroupaggrinit), :708 (dosum), :900, :1018,
 *               :1801 (BATgroupavg), :1996 (BATgroupavg3), :2634 (combine), :3069 (BATgroupcount), AVERAGE_ITER
 *               gdk/gdk_calc_private.h:231-275
 *   group       gdk/gdk_group.c:657-1347 (first-occurrence numbering)
 *   join        gdk/gdk_join.c:4451-4623 (BATjoin: algorithm choice, result
 *               order and properties; gdk_oracle_join.c)
 *   sort        gdk/gdk_batop.c:2266-2827 (BATsort, do_sort), gdk/gdk_rsort.c:21 (stable),
 *               gdk/gdk_qsort.c + gdk_qsort_impl.h (GDKqsort; gdk_oracle_sort.c)
 *   window      gdk/gdk_analytic_bounds.c:187-587, :855-1440 (gdk_oracle_bounds.c)
 *   frames      gdk/gdk_analytic_func.c:1626 (count), :1959 (sum),
 *               gdk/gdk_analytic_statistics.c:364 (avg), :428-700 (avginteger), segment
 *               tree gdk/gdk_analytic.h:52-130
 *   firstn      gdk/gdk_firstn.c:71-97 (heap), :211-1020, :1280
 *   window fns  gdk/gdk_analytic_func.c:124-1300 ntile, first, last,
 *               nth_value, lag, lead, min, max (gdk_oracle_window.c)
 *
 * Parity pinning: see tests/golden/ (fixtures extracted from the reference's
 * own MAL known-answer tests) and DESIGN.md §Oracle.
 */
#ifndef GDK_ORACLE_H
#define GDK_ORACLE_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uint64_t ora_oid;
typedef __int128 ora_hge;

/* GDK type ids (gdk/gdk.h:428-451, HAVE_HGE build) */
enum {
	ORA_void = 0, ORA_msk = 1, ORA_bit = 2, ORA_bte = 3, ORA_sht = 4,
	ORA_int = 5, ORA_oid = 6, ORA_flt = 8, ORA_dbl = 9, ORA_lng = 10,
	ORA_hge = 11, ORA_date = 12, ORA_daytime = 13, ORA_timestamp = 14, ORA_str = 16,
};

#define ORA_OID_NIL ((ora_oid) 1 << 63)

typedef struct ora_bat {
	int32_t type;        /* GDK type id */
	int32_t width;       /* bytes per tail value (str: offset width) */
	uint64_t count;
	ora_oid hseqbase;
	ora_oid tseqbase;    /* void/dense: first value; else ORA_OID_NIL */
	void *base;          /* tail values (NULL for void) */
	char *vheap;         /* str: string heap */
	uint64_t vheapsize;
	uint8_t sorted, revsorted, key, nonil, nil, owned;
	uint8_t _pad[2];
	double unique_est;   /* tunique_est (gdk/gdk.h:740): 0 = unknown */
	uint64_t minpos, maxpos;   /* tminpos / tmaxpos: ORA_BUN_NONE = unknown */
} ora_bat;

#define ORA_BUN_NONE ((uint64_t) INT64_MAX)

/* memory */
ora_bat *ora_new(int type, uint64_t count, ora_oid hseq);
void ora_free(ora_bat *b);
const char *ora_errbuf(void);

/* operators: NULL / -1 on error with message in ora_errbuf() */
ora_bat *ora_select(const ora_bat *b, const ora_bat *s, const void *tl,
		    const void *th, bool li, bool hi, bool anti, bool nil_matches);
ora_bat *ora_thetaselect(const ora_bat *b, const ora_bat *s, const void *val,
			 const char *op);
ora_bat *ora_project(const ora_bat *l, const ora_bat *r);
/* msk BATs (tail = 32-bit words of bits, count = bits): BATunmask
 * (gdk/gdk_cand.c:1464) and BATmaskedcands (:1366) as materialised lists;
 * a msk candidate list anywhere = its BATunmask */
ora_bat *ora_unmask(const ora_bat *b);
ora_bat *ora_maskedcands(ora_oid hseq, uint64_t nr, const ora_bat *masked, bool selected);
/* candidate-list algebra (gdk/gdk_cand.c:46, :184, :259, :1296); the
 * negcands result as the oid list its cand_except form stands for */
ora_bat *ora_mergecand(const ora_bat *a, const ora_bat *b);
ora_bat *ora_intersectcand(const ora_bat *a, const ora_bat *b);
ora_bat *ora_diffcand(const ora_bat *a, const ora_bat *b);
ora_bat *ora_negcands(ora_oid tseq, uint64_t nr, const ora_bat *odels);
/* op: '+', '-', '*'; b1/b2 may be NULL when a constant is given */
ora_bat *ora_calc(char op, const ora_bat *b1, const void *c1, int t1,
		  const ora_bat *b2, const void *c2, int t2,
		  const ora_bat *s, int tp);
/* BATcalc{lt,le,gt,ge,eq,ne,cmp} (op 0..6; gdk/gdk_calc_compare.h), with
 * constants as for ora_calc; s1 / s2 candidate lists of b1 / b2 */
ora_bat *ora_calccmp(int op, const ora_bat *b1, const void *c1, int t1, const ora_bat *b2,
		     const void *c2, int t2, const ora_bat *s1, const ora_bat *s2, bool nil_matches);
/* BATcalcbetween / -cstcst / -batcst / -cstbat (gdk/gdk_calc.c:3968-4206) */
ora_bat *ora_calcbetween(const ora_bat *b, const ora_bat *lo, const void *clo, const ora_bat *hi,
			 const void *chi, int ct, const ora_bat *s, const ora_bat *slo,
			 const ora_bat *shi, bool symmetric, bool linc, bool hinc, bool nils_false,
			 bool anti);
/* BATconvert (gdk/gdk_calc_convert.c:1415) for numeric / oid / bit types */
ora_bat *ora_convert(const ora_bat *b, const ora_bat *s, int tp, int scale1, int scale2, int prec);
ora_bat *ora_calcnot(const ora_bat *b, const ora_bat *s);
/* gdk_calc.c:233-920 negate / absolute / iszero / sign / isnil / isnotnil
 * (op 0..5), :976-2436 min / max / _no_nil (op 6..9; b2 NULL: the constant c
 * of type ct), :2439-3760 and / or / xor / lsh / rsh (op 10..14), :4376
 * ifthenelse (b1 / b2 NULL: the constants of type ct) */
ora_bat *ora_calcunary(int op, const ora_bat *b, const ora_bat *s);
ora_bat *ora_calcminmax(int op, const ora_bat *b1, const ora_bat *b2, const void *c, int ct, const ora_bat *s1,
			const ora_bat *s2);
ora_bat *ora_calcbits(int op, const char *fname, const ora_bat *b1, const void *c1, int t1, const ora_bat *b2,
		      const void *c2, int t2, const ora_bat *s1, const ora_bat *s2);
ora_bat *ora_calcifthenelse(const ora_bat *b, const ora_bat *b1, const void *c1, const ora_bat *b2, const void *c2,
			    int ct);
/* BATcalcdiv / BATcalcmod (+cst variants): op '/' or '%' */
ora_bat *ora_calcdivmod(char op, const ora_bat *b1, const void *c1, int t1, const ora_bat *b2,
			const void *c2, int t2, const ora_bat *s1, const ora_bat *s2, int tp);
int ora_sum(void *res, int tp, const ora_bat *b, const ora_bat *s,
	    bool skip_nils, bool nil_if_empty);
/* BATsort (gdk/gdk_batop.c:2342) with do_sort's choice per run: stable sorts
 * and an exact restatement of GDKqsort (gdk_oracle_sort.c) */
int ora_BATsort(ora_bat **sorted, ora_bat **order, ora_bat **groups, ora_bat *b, const ora_bat *o,
		const ora_bat *g, bool reverse, bool nilslast, bool stable);
void ora_GDKqsort(const ora_bat *v, uint64_t *h, ora_oid *t, uint64_t n, bool reverse, bool nilslast);
int ora_group(ora_bat **groups, ora_bat **extents, ora_bat **histo,
	      ora_bat *b, const ora_bat *s, const ora_bat *g);
ora_bat *ora_groupsum(const ora_bat *b, const ora_bat *g, const ora_bat *e,
		      const ora_bat *s, int tp, bool skip_nils);
ora_bat *ora_groupcount(const ora_bat *b, const ora_bat *g, const ora_bat *e,
			const ora_bat *s, bool skip_nils);
int ora_groupavg3(ora_bat **avgp, ora_bat **remp, ora_bat **cntp,
		  const ora_bat *b, const ora_bat *g, const ora_bat *e,
		  const ora_bat *s, bool skip_nils);
ora_bat *ora_groupavg3combine(const ora_bat *avg, const ora_bat *rem, const ora_bat *cnt,
			       const ora_bat *g, const ora_bat *e, bool skip_nils);
int ora_groupavg(ora_bat **bnp, ora_bat **cntp, const ora_bat *b, const ora_bat *g,
		 const ora_bat *e, const ora_bat *s, bool skip_nils, int scale);
/* gdk_aggr.c:3570 BATmin_skipnil / :3727 BATmax_skipnil: the value into res
 * (a buffer of the width), str: *sres = the string */
int ora_minmax(ora_bat *b, bool skipnil, bool domax, void *res, const char **sres);
/* gdk_aggr.c:1650 BATprod (res of type tp), :1575 BATgroupprod */
int ora_prod(void *res, int tp, const ora_bat *b, const ora_bat *s, bool skip_nils, bool nil_if_empty);
int ora_calcavg(const ora_bat *b, const ora_bat *s, double *avg, uint64_t *vals, int scale);
ora_bat *ora_groupprod(const ora_bat *b, const ora_bat *g, const ora_bat *e, const ora_bat *s, int tp,
		       bool skip_nils);
ora_bat *ora_groupminmax(const ora_bat *b, const ora_bat *g, const ora_bat *e,
			 const ora_bat *s, bool skip_nils, bool domax);
/* BATjoin with its algorithm choice (gdk_oracle_join.c); l and r receive
 * the ordering / key flags the reference caches on them */
/* BATintersect / BATsemijoin's left output (only_misses false) and BATdiff
 * (true) (gdk_join.c:4343-4407, leftjoin :4049); BATleftjoin / BATouterjoin
 * for at most one match per left candidate (-2: several, not restated) */
/* statistics (gdk/gdk_aggr.c:4255-5202): kind 0 stdev / variance, 1
 * covariance, 2 correlation (gdk_oracle_grp.c) */
ora_bat *ora_groupmoments(int kind, const ora_bat *b1, const ora_bat *b2, const ora_bat *g, const ora_bat *e,
			  const ora_bat *s, bool skip_nils, bool issample, bool variance);
int ora_calcmoments(double *res, double *avgp, int kind, const ora_bat *b1, const ora_bat *b2, bool issample,
		    bool variance);
/* doBATgroupquantile (gdk/gdk_aggr.c:3881); g may be NULL */
ora_bat *ora_groupquantile(const ora_bat *b, const ora_bat *g, const ora_bat *e, const ora_bat *s, double quantile,
			   bool skip_nils, bool average);
ora_bat *ora_semijoin_cands(ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr, bool nil_matches,
			    bool max_one, bool only_misses, bool not_in);
int ora_leftjoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr,
		 bool nil_matches, bool outer, bool match_one);
/* leftjoin (gdk_join.c:4049) with its algorithm choice, for several matches
 * per left candidate: BATleftjoin / BATouterjoin / BATsemijoin with r2p /
 * BATmarkjoin (r3p); *algo = the branch taken (gdk_oracle_join.c LJ_*) */
int ora_leftjoin_ex(ora_bat **r1p, ora_bat **r2p, ora_bat **r3p, ora_bat *l, ora_bat *r, const ora_bat *sl,
		    const ora_bat *sr, bool nil_matches, bool nil_on_miss, bool semi, bool max_one, bool min_one,
		    int *algo);
/* gdk_join.c:4367 BATmarkjoin; r2p may be NULL (semi) */
int ora_markjoin(ora_bat **r1p, ora_bat **r2p, ora_bat **r3p, ora_bat *l, ora_bat *r, const ora_bat *sl,
		 const ora_bat *sr);
/* gdk_join.c:3699 thetajoin (mask: 1 EQ, 2 LT, 4 GT of vl op vr), :4626
 * BATbandjoin (c1 / c2 of the columns' type) */
int ora_thetajoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr,
		  int mask, bool nil_matches);
int ora_bandjoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr,
		 const void *c1, const void *c2, bool linc, bool hinc);
/* gdk_join.c:5422 BATrangejoin (rangejoin :5067) */
int ora_rangejoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *rl, ora_bat *rh, const ora_bat *sl,
		  const ora_bat *sr, bool linc, bool hinc, bool anti, bool symmetric);
/* gdk_join.c:3572 BATguess_uniques (s: the candidate BAT, NULL: all of b) */
uint64_t ora_guess_uniques(ora_bat *b, const ora_bat *s);
/* gdk_batop.c:3078 BATcount_no_nil */
uint64_t ora_count_no_nil(const ora_bat *b, const ora_bat *s);
/* gdk_cross.c:138 BATsubcross; outer: :153 BAToutercross (r2p may be NULL) */
int ora_crossproduct(ora_bat **r1p, ora_bat **r2p, const ora_bat *l, const ora_bat *r, const ora_bat *sl,
		     const ora_bat *sr, bool max_one, bool outer);
int ora_join(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r,
	     const ora_bat *sl, const ora_bat *sr, bool nil_matches);
int ora_join_algo(ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr);
/* GDKanalyticalwindowbounds, all units / types (gdk_oracle_bounds.c);
 * r is caller-allocated with count(b) oid slots */
int ora_windowbounds(ora_bat *r, const ora_bat *b, const ora_bat *p, const ora_bat *l, const void *bound,
		     int tp1, int tp2, int unit, bool preceding, ora_oid second_half);
int32_t ora_date_add_day(int32_t dt, int days);
int32_t ora_date_add_month(int32_t dt, int months);
int64_t ora_daytime_add_usec(int64_t t, int64_t usec);
int64_t ora_timestamp_add_usec(int64_t ts, int64_t usec);
int64_t ora_timestamp_add_month(int64_t ts, int m);
/* plain first-N (no group ids, not distinct), heap semantics of
 * gdk/gdk_firstn.c:211-1020 (gdk_oracle_firstn.c) */
ora_bat *ora_firstn(const ora_bat *b, const ora_bat *s, const ora_bat *g, uint64_t n,
		    bool asc, bool nilslast);

/* synthetic TPC-H lineitem (tpch_gen.c) */
typedef struct ora_lineitem {
	uint64_t n;
	int32_t *shipdate;     /* GDK date */
	int64_t *quantity;     /* decimal(15,2) as lng */
	int64_t *extendedprice;
	int64_t *discount;
	int64_t *tax;
	uint8_t *returnflag;   /* 1-byte str offsets into ora_flag_heap */
	uint8_t *linestatus;
} ora_lineitem;
void ora_tpch_lineitem(uint64_t seed, uint64_t row0, uint64_t n, uint64_t sf_parts,
		       int32_t *shipdate, int64_t *quantity, int64_t *extendedprice,
		       int64_t *discount, int64_t *tax, uint8_t *returnflag,
		       uint8_t *linestatus);
int32_t ora_mkdate(int y, int m, int d);

/* op-at-a-time TPC-H pipelines over the oracle operators (pipelines.c) */
int ora_q6(const ora_lineitem *li, int nthreads, ora_hge *revenue);
typedef struct ora_q1row {
	uint8_t returnflag, linestatus, _pad[6];
	ora_hge sum_qty, sum_base_price, sum_disc_price, sum_charge;
	int64_t avg_qty, avg_price, avg_disc;      /* avg3 rounded results */
	int64_t rem_qty, rem_price, rem_disc;
	int64_t count_order;
} ora_q1row;
int ora_q1(const ora_lineitem *li, int nthreads, ora_q1row *rows, int *nrows);

/* windowed aggregates over frames (gdk_oracle_analytic.c); r is
 * caller-allocated with count(b) slots of the result type */
int ora_analyticalsum(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b,
		      const ora_bat *s, const ora_bat *e, int tp1, int tp2, int frame_type);
int ora_analyticalavg(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b,
		      const ora_bat *s, const ora_bat *e, int tpe, int frame_type);
/* gdk_analytic_statistics.c:897-1443 (kind 0 stddev / variance, op 0
 * stddev_samp 1 stddev_pop 2 variance_samp 3 variance_pop; kind 1
 * covariance, op 0 samp 1 pop; kind 2 correlation) and
 * gdk_analytic_func.c:2479 GDKanalyticalprod (gdk_oracle_winstats.c) */
int ora_analyticalstat(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b1, const ora_bat *b2,
		       const ora_bat *s, const ora_bat *e, int kind, int op, int frame_type);
int ora_analyticalprod(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		       const ora_bat *e, int tp2, int frame_type);
int ora_analyticalavginteger(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b,
			     const ora_bat *s, const ora_bat *e, int tpe, int frame_type);
/* gdk_analytic_func.c :124 ntile, :230 first, :312 last, :421 nth_value,
 * :671 lag, :823 lead, :1264 min / max (gdk_oracle_window.c); r is a
 * caller-allocated BAT of count(b) slots of type tpe */
/* gdk_analytic_bounds.c:95 GDKanalyticaldiff: r (bit) marks the rows whose
 * value differs from the previous distinct one, or np[i] / *npbit */
int ora_analyticaldiff(ora_bat *r, const ora_bat *b, const ora_bat *p, const int8_t *npbit, int tpe);
int ora_analyticalntile(ora_bat *r, const ora_bat *b, const ora_bat *p, const ora_bat *n, int tpe,
			const void *ntile);
int ora_analyticalfirst(ora_bat *r, const ora_bat *b, const ora_bat *s, const ora_bat *e, int tpe);
int ora_analyticallast(ora_bat *r, const ora_bat *b, const ora_bat *s, const ora_bat *e, int tpe);
int ora_analyticalnthvalue(ora_bat *r, const ora_bat *b, const ora_bat *s, const ora_bat *e, const ora_bat *t,
			   const int64_t *pnth, int tpe);
int ora_analyticallag(ora_bat *r, const ora_bat *b, const ora_bat *p, uint64_t lag, const void *def, int tpe);
int ora_analyticallead(ora_bat *r, const ora_bat *b, const ora_bat *p, uint64_t lead, const void *def, int tpe);
int ora_analyticalmin(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		      const ora_bat *e, int tpe, int frame_type);
int ora_analyticalmax(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		      const ora_bat *e, int tpe, int frame_type);
int ora_analyticalcount(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b,
			const ora_bat *s, const ora_bat *e, bool ignore_nils, int frame_type);

#ifdef __cplusplus
}
#endif
#endif
