/*
 * gdk_oracle_calc.c -- CPU restatement of the BATcalc comparison, between,
 * conversion, NOT, division and modulo operators.  TEST INFRASTRUCTURE ONLY
 * (see gdk_oracle.h).
 *
 *   compare   gdk/gdk_calc_compare.h:15-995 (op_typeswitchloop,
 *             BATcalcop/-cst/cst-), operators gdk_calc_compare_{lt,le,gt,
 *             ge,eq,ne,generic}.c; nil handling BINARY_3TYPE_FUNC{,_nonil,
 *             _nilmatch} gdk/gdk_calc_private.h:391-535
 *   between   gdk/gdk_calc.c:3770-4206 (BETWEEN, BATcalcbetween*), and3/or3
 *             gdk_calc.c:2590,2826
 *   convert   gdk/gdk_calc_convert.c:98-660 (convertimpl*, convert2bit),
 *             :870-980 (convert_void_any), :1415-1548 (BATconvert)
 *   not       gdk/gdk_calc.c:41-146 (BATcalcnot)
 *   div/mod   gdk/gdk_calc_div.c:21-140, :1880-2060; gdk/gdk_calc_mod.c:21-110,
 *             :1160-1260; BATcalcmuldivmod gdk/gdk_calc_mul.c:2020-2082
 *
 * Mixed-type comparisons follow C's usual arithmetic conversions exactly as
 * the reference's macro expansion does (an int compared with a flt is
 * converted to flt, a lng with a dbl to dbl).  str operands are outside the
 * device path and refused here too.
 */
#include "gdk_oracle_private.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define HGE_NIL ((ora_hge) ((unsigned __int128) 1 << 127))
#define HGE_MAX ((ora_hge) (((unsigned __int128) 1 << 127) - 1))

static int
btype(int t)
{
	/* ATOMbasetype (gdk/gdk_atoms.h:285): date -> int, bit -> bte */
	return t == ORA_date ? ORA_int : t == ORA_bit ? ORA_bte : t;
}

static const char *
tname(int t)
{
	switch (t) {
	case ORA_void: return "void";
	case ORA_bit: return "bit";
	case ORA_bte: return "bte";
	case ORA_sht: return "sht";
	case ORA_int: return "int";
	case ORA_oid: return "oid";
	case ORA_flt: return "flt";
	case ORA_dbl: return "dbl";
	case ORA_lng: return "lng";
	case ORA_hge: return "hge";
	case ORA_date: return "date";
	case ORA_str: return "str";
	}
	return "?";
}

static bool
is_int(int t)
{
	return t == ORA_bte || t == ORA_sht || t == ORA_int || t == ORA_lng || t == ORA_hge;
}

static bool
is_num(int t)
{
	return is_int(t) || t == ORA_flt || t == ORA_dbl;
}

/* one value of a numeric base type, kept in its own domain */
typedef struct {
	int t;          /* base type */
	bool nil;
	ora_hge i;      /* integer types and oid */
	float f;
	double d;
} num;

static num
load(int t, const void *base, uint64_t p)
{
	num v = {.t = t};
	switch (t) {
	case ORA_bte: v.i = ((const int8_t *) base)[p]; v.nil = v.i == INT8_MIN; break;
	case ORA_sht: v.i = ((const int16_t *) base)[p]; v.nil = v.i == INT16_MIN; break;
	case ORA_int: v.i = ((const int32_t *) base)[p]; v.nil = v.i == INT32_MIN; break;
	case ORA_lng: v.i = ((const int64_t *) base)[p]; v.nil = v.i == INT64_MIN; break;
	case ORA_hge: v.i = ((const ora_hge *) base)[p]; v.nil = v.i == HGE_NIL; break;
	case ORA_oid: v.i = (ora_hge) ((const ora_oid *) base)[p]; v.nil = ((const ora_oid *) base)[p] == ORA_OID_NIL; break;
	case ORA_flt: v.f = ((const float *) base)[p]; v.nil = isnan(v.f); break;
	case ORA_dbl: v.d = ((const double *) base)[p]; v.nil = isnan(v.d); break;
	}
	return v;
}

static double
as_dbl(const num *v)
{
	return v->t == ORA_dbl ? v->d : v->t == ORA_flt ? (double) v->f : (double) v->i;
}

static float
as_flt(const num *v)
{
	return v->t == ORA_flt ? v->f : (float) v->i;
}

/* ---------------------------------------------------------------------- */
/* comparisons */

enum { OP_LT, OP_LE, OP_GT, OP_GE, OP_EQ, OP_NE, OP_CMP };

static const char *const cmpfunc[] = {
	"BATcalclt", "BATcalcle", "BATcalcgt", "BATcalcge", "BATcalceq", "BATcalcne", "BATcalccmp",
};

/* OP(a, b) in the domain C's usual arithmetic conversions pick */
static int8_t
apply(int op, const num *a, const num *b)
{
	int lt, gt, le, ge, eq;
	if (a->t == ORA_dbl || b->t == ORA_dbl) {
		double x = as_dbl(a), y = as_dbl(b);
		lt = x < y; gt = x > y; le = x <= y; ge = x >= y; eq = x == y;
	} else if (a->t == ORA_flt || b->t == ORA_flt) {
		float x = as_flt(a), y = as_flt(b);
		lt = x < y; gt = x > y; le = x <= y; ge = x >= y; eq = x == y;
	} else if (a->t == ORA_oid || b->t == ORA_oid) {
		ora_oid x = (ora_oid) a->i, y = (ora_oid) b->i;
		lt = x < y; gt = x > y; le = x <= y; ge = x >= y; eq = x == y;
	} else {
		ora_hge x = a->i, y = b->i;
		lt = x < y; gt = x > y; le = x <= y; ge = x >= y; eq = x == y;
	}
	switch (op) {
	case OP_LT: return lt;
	case OP_LE: return le;
	case OP_GT: return gt;
	case OP_GE: return ge;
	case OP_EQ: return eq;
	case OP_NE: return !eq;
	default: return (int8_t) (gt - lt);
	}
}

/* OP over two flags (the nil_matches branches compare is_nil(v1), is_nil(v2)) */
static int8_t
apply_flags(int op, int x, int y)
{
	num a = {.t = ORA_int, .i = x}, b = {.t = ORA_int, .i = y};
	return apply(op, &a, &b);
}

/* an operand: a BAT (with candidates) or a constant */
typedef struct {
	const ora_bat *b;
	int t;            /* base type passed to op_typeswitchloop (void stays void) */
	const void *c;    /* constant value */
	ora_ci ci;
} opnd;

static uint64_t
pos_of(const opnd *o, uint64_t k)
{
	return o->b ? ci_get(&o->ci, k) - o->b->hseqbase : 0;
}

static const void *
base_of(const opnd *o)
{
	if (o->b == NULL)
		return o->c;
	return o->b->type == ORA_void ? (const void *) &o->b->tseqbase : o->b->base;
}

static ora_bat *
cmp_result(int op, uint64_t n, ora_oid hseq)
{
	return ora_new(op == OP_CMP ? ORA_bte : ORA_bit, n, hseq);
}

/* op_typeswitchloop (gdk_calc_compare.h:15-780) + BATcalcop_intern's
 * properties (:782-825) */
static ora_bat *
cmp_loop(int op, const opnd *l, const opnd *r, bool nonil, bool nil_matches, ora_oid hseq,
	 uint64_t n)
{
	const int t1 = l->t, t2 = r->t;
	const bool nm = nil_matches && (op == OP_EQ || op == OP_NE);
	if (t1 == ORA_str || t2 == ORA_str || !((t1 == ORA_void && (t2 == ORA_oid || t2 == ORA_void)) ||
						 (t1 == ORA_oid && (t2 == ORA_oid || t2 == ORA_void)) ||
						 (is_num(t1) && is_num(t2)))) {
		ora_seterr("%s: bad input types %s,%s.\n", cmpfunc[op], tname(t1), tname(t2));
		return NULL;
	}
	ora_bat *bn = cmp_result(op, n, hseq);
	if (bn == NULL)
		return NULL;
	int8_t *dst = bn->base;
	const int8_t NILV = INT8_MIN;
	uint64_t nils = 0;
	const void *lb = base_of(l), *rb = base_of(r);
	if (t1 == ORA_void) {
		/* gdk_calc_compare.h:36-72 */
		const ora_oid v = l->b ? l->b->tseqbase : *(const ora_oid *) l->c;
		const ora_oid r0 = *(const ora_oid *) rb;
		for (uint64_t k = 0; k < n; k++) {
			uint64_t i = pos_of(l, k), j = pos_of(r, k);
			int8_t res;
			if (v == ORA_OID_NIL || t2 == ORA_void) {
				num a = {.t = ORA_oid, .i = v}, b = {.t = ORA_oid, .i = r0};
				if (v == ORA_OID_NIL || r0 == ORA_OID_NIL)
					res = nm ? apply_flags(op, v == ORA_OID_NIL, r0 == ORA_OID_NIL) : NILV;
				else
					res = apply(op, &a, &b);
			} else {
				ora_oid w = ((const ora_oid *) rb)[r->b ? j : 0];
				if (w == ORA_OID_NIL) {
					res = nm ? apply_flags(op, 0, 1) : NILV;
				} else {
					num a = {.t = ORA_oid, .i = v + i}, b = {.t = ORA_oid, .i = w};
					res = apply(op, &a, &b);
				}
			}
			dst[k] = res;
			nils += res == NILV;
		}
	} else if (t1 == ORA_oid && t2 == ORA_void) {
		/* gdk_calc_compare.h:638-671 */
		const ora_oid v = *(const ora_oid *) rb;
		for (uint64_t k = 0; k < n; k++) {
			uint64_t i = pos_of(l, k), j = pos_of(r, k);
			ora_oid x = ((const ora_oid *) lb)[l->b ? i : 0];
			int8_t res;
			if (v == ORA_OID_NIL) {
				res = nm ? apply_flags(op, x == ORA_OID_NIL, 1) : NILV;
			} else if (x == ORA_OID_NIL) {
				res = nm ? apply_flags(op, 1, 0) : NILV;
			} else {
				num a = {.t = ORA_oid, .i = x}, b = {.t = ORA_oid, .i = v + j};
				res = apply(op, &a, &b);
			}
			dst[k] = res;
			nils += res == NILV;
		}
	} else {
		/* BINARY_3TYPE_FUNC / _nonil / _nilmatch */
		for (uint64_t k = 0; k < n; k++) {
			num a = load(t1, lb, l->b ? pos_of(l, k) : 0);
			num b = load(t2, rb, r->b ? pos_of(r, k) : 0);
			int8_t res;
			if (nonil)
				res = apply(op, &a, &b);
			else if (a.nil || b.nil)
				res = nm ? apply_flags(op, a.nil, b.nil) : NILV;
			else
				res = apply(op, &a, &b);
			dst[k] = res;
			nils += res == NILV;
		}
	}
	bn->sorted = n <= 1 || nils == n;
	bn->revsorted = n <= 1 || nils == n;
	bn->key = n <= 1;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	return bn;
}

static int
optype(const ora_bat *b)
{
	/* ATOMtype(t) == TYPE_oid ? t : ATOMbasetype(t) (gdk_calc_compare.h:866) */
	return b->type == ORA_void || b->type == ORA_oid ? b->type : btype(b->type);
}

static bool
cst_is_nil(int t, const void *v)
{
	num x = load(btype(t), v, 0);
	return x.nil;
}

/* BATcalcop (gdk_calc_compare.h:827-886), BATcalcopcst (:888-925),
 * BATcalccstop (:927-964).  b1 / b2 NULL: the constant c1 / c2 of type
 * t1 / t2 is used. */
ora_bat *
ora_calccmp(int op, const ora_bat *b1, const void *c1, int t1, const ora_bat *b2, const void *c2,
	    int t2, const ora_bat *s1, const ora_bat *s2, bool nil_matches)
{
	opnd l = {.b = b1, .c = c1}, r = {.b = b2, .c = c2};
	if (op < OP_LT || op > OP_CMP || (b1 == NULL && b2 == NULL)) {
		ora_seterr("calccmp: bad arguments");
		return NULL;
	}
	const ora_bat *bb = b1 ? b1 : b2;
	ora_ci ci;
	if (b1 && b2) {
		if (ora_ci_init(&l.ci, b1, s1) < 0 || ora_ci_init(&r.ci, b2, s2) < 0)
			return NULL;
		ora_oid h1 = s1 ? s1->hseqbase : b1->hseqbase, h2 = s2 ? s2->hseqbase : b2->hseqbase;
		if (l.ci.n != r.ci.n || h1 != h2) {
			ora_seterr("inputs not the same size.\n");
			return NULL;
		}
		ci = l.ci;
	} else {
		if (ora_ci_init(&ci, bb, s1) < 0)
			return NULL;
		if (b1)
			l.ci = ci;
		else
			r.ci = ci;
	}
	const ora_oid hseq = s1 ? s1->hseqbase : bb->hseqbase;
	if (ci.n == 0)
		return cmp_result(op, 0, hseq);
	l.t = b1 ? optype(b1) : (t1 == ORA_void || t1 == ORA_oid ? t1 : btype(t1));
	r.t = b2 ? optype(b2) : (t2 == ORA_void || t2 == ORA_oid ? t2 : btype(t2));
	if (b1 && b2 && b1->type == ORA_void && b2->type == ORA_void && l.ci.dense && r.ci.dense) {
		/* BATconstant shortcut (gdk_calc_compare.h:848-861) */
		int8_t res;
		const bool nm = nil_matches && (op == OP_EQ || op == OP_NE);
		if ((b1->tseqbase == ORA_OID_NIL || b2->tseqbase == ORA_OID_NIL) && !nm) {
			res = INT8_MIN;
		} else {
			num a = {.t = ORA_oid, .i = (ora_oid) (b1->tseqbase + l.ci.seq)};
			num b = {.t = ORA_oid, .i = (ora_oid) (b2->tseqbase + r.ci.seq)};
			res = apply(op, &a, &b);
		}
		ora_bat *bn = cmp_result(op, ci.n, b1->hseqbase);
		if (bn == NULL)
			return NULL;
		memset(bn->base, (uint8_t) res, ci.n);
		bn->sorted = bn->revsorted = 1;
		bn->key = ci.n <= 1;
		bn->nil = res == INT8_MIN;
		bn->nonil = !bn->nil;
		return bn;
	}
	bool nonil;
	if (b1 && b2)
		nonil = b1->nonil && b2->nonil;
	else if (b1)
		nonil = b1->nonil && !cst_is_nil(t2, c2);
	else
		nonil = b2->nonil && !cst_is_nil(t1, c1);
	return cmp_loop(op, &l, &r, nonil, nil_matches, hseq, ci.n);
}

/* ---------------------------------------------------------------------- */
/* between (gdk/gdk_calc.c:3770-4206) */

#define BIT_NIL ((int8_t) INT8_MIN)

static int8_t
or3(int8_t a, int8_t b)
{
	return a == 1 || b == 1 ? 1 : a == BIT_NIL || b == BIT_NIL ? BIT_NIL : 0;
}

static int8_t
and3(int8_t a, int8_t b)
{
	return a == 0 || b == 0 ? 0 : a == BIT_NIL || b == BIT_NIL ? BIT_NIL : 1;
}

static int8_t
not3(int8_t a)
{
	return a == BIT_NIL ? BIT_NIL : !a;
}

static int8_t
less3(const num *a, const num *b, bool inc)
{
	if (a->nil || b->nil)
		return BIT_NIL;
	return apply(OP_LT, a, b) || (inc && apply(OP_EQ, a, b));
}

static int8_t
grtr3(const num *a, const num *b, bool inc)
{
	if (a->nil || b->nil)
		return BIT_NIL;
	return apply(OP_LT, b, a) || (inc && apply(OP_EQ, a, b));
}

static int8_t
between3(const num *v, const num *lo, bool linc, const num *hi, bool hinc)
{
	return and3(grtr3(v, lo, linc), less3(v, hi, hinc));
}

static int8_t
BETWEEN(const num *v, const num *lo, const num *hi, bool symmetric, bool linc, bool hinc,
	bool nils_false, bool anti)
{
	if (v->nil)
		return nils_false ? 0 : BIT_NIL;
	int8_t r = symmetric ? or3(between3(v, lo, linc, hi, hinc), between3(v, hi, hinc, lo, linc))
			     : between3(v, lo, linc, hi, hinc);
	return anti ? not3(r) : r;
}

/* BATcalcbetween (b, lo, hi BATs), BATcalcbetweencstcst / batcst / cstbat:
 * lo / hi NULL take the constants clo / chi of type ct. */
ora_bat *
ora_calcbetween(const ora_bat *b, const ora_bat *lo, const void *clo, const ora_bat *hi,
		const void *chi, int ct, const ora_bat *s, const ora_bat *slo, const ora_bat *shi,
		bool symmetric, bool linc, bool hinc, bool nils_false, bool anti)
{
	ora_ci ci, cil, cih;
	if ((lo == NULL || hi == NULL) && btype(b->type) != btype(ct)) {
		ora_seterr("incompatible input types.\n");
		return NULL;
	}
	if (ora_ci_init(&ci, b, s) < 0 || (lo && ora_ci_init(&cil, lo, slo) < 0) ||
	    (hi && ora_ci_init(&cih, hi, shi) < 0))
		return NULL;
	const ora_oid hseq = s ? s->hseqbase : b->hseqbase;
	if ((lo && (cil.n != ci.n || (slo ? slo->hseqbase : lo->hseqbase) != hseq)) ||
	    (hi && (cih.n != ci.n || (shi ? shi->hseqbase : hi->hseqbase) != hseq))) {
		ora_seterr("inputs not the same size.\n");
		return NULL;
	}
	const int t = btype(b->type);
	if (t != ORA_void && ((lo && btype(lo->type) != t) || (hi && btype(hi->type) != t))) {
		ora_seterr("incompatible input types.\n");
		return NULL;
	}
	if (t == ORA_str || (t != ORA_void && t != ORA_oid && !is_num(t))) {
		ora_seterr("BATcalcbetween: bad input type %s.\n", tname(b->type));
		return NULL;
	}
	const bool vd = b->type == ORA_void || (lo && lo->type == ORA_void) || (hi && hi->type == ORA_void);
	if (vd && ((b->type != ORA_void && b->type != ORA_oid) || (lo && lo->type != ORA_void && lo->type != ORA_oid) ||
		   (hi && hi->type != ORA_void && hi->type != ORA_oid))) {
		/* BUNtoid over every operand (gdk_calc.c:4025-4036): oid / void only */
		ora_seterr("incompatible input types.\n");
		return NULL;
	}
	if (lo && hi && b->type == ORA_void && lo->type == ORA_void && hi->type == ORA_void) {
		/* all three dense (gdk_calc.c:4012-4019): one constant */
		num v = {.t = ORA_oid, .i = b->tseqbase, .nil = b->tseqbase == ORA_OID_NIL};
		num l = {.t = ORA_oid, .i = lo->tseqbase, .nil = lo->tseqbase == ORA_OID_NIL};
		num h = {.t = ORA_oid, .i = hi->tseqbase, .nil = hi->tseqbase == ORA_OID_NIL};
		int8_t res = BETWEEN(&v, &l, &h, symmetric, linc, hinc, nils_false, anti);
		ora_bat *bn = ora_new(ORA_bit, ci.n, hseq);
		if (bn == NULL)
			return NULL;
		memset(bn->base, (uint8_t) res, ci.n);
		bn->sorted = bn->revsorted = 1;
		bn->key = ci.n <= 1;
		bn->nil = ci.n >= 1 && res == BIT_NIL;
		bn->nonil = !bn->nil;
		return bn;
	}
	/* a void operand goes through BUNtoid with the result's head at the
	 * first candidate (gdk_calc.c:4025, :4116: COLnew(ci.seq, ...)) */
	ora_bat *bn = ora_new(ORA_bit, ci.n, vd ? (ci.n ? ci_get(&ci, 0) : 0) : hseq);
	if (bn == NULL)
		return NULL;
	int8_t *dst = bn->base;
	uint64_t nils = 0;
	const int tt = vd ? ORA_oid : t;
	for (uint64_t k = 0; k < ci.n; k++) {
		num v, l, h;
		uint64_t i = ci_get(&ci, k) - b->hseqbase;
		if (b->type == ORA_void)
			v = (num) {.t = ORA_oid, .i = (ora_oid) (b->tseqbase + i), .nil = b->tseqbase == ORA_OID_NIL};
		else
			v = load(tt, b->base, i);
		if (lo == NULL) {
			l = load(tt, clo, 0);
		} else {
			uint64_t j = ci_get(&cil, k) - lo->hseqbase;
			if (lo->type == ORA_void)
				l = (num) {.t = ORA_oid, .i = (ora_oid) (lo->tseqbase + j), .nil = lo->tseqbase == ORA_OID_NIL};
			else
				l = load(tt, lo->base, j);
		}
		if (hi == NULL) {
			h = load(tt, chi, 0);
		} else {
			uint64_t j = ci_get(&cih, k) - hi->hseqbase;
			if (hi->type == ORA_void)
				h = (num) {.t = ORA_oid, .i = (ora_oid) (hi->tseqbase + j), .nil = hi->tseqbase == ORA_OID_NIL};
			else
				h = load(tt, hi->base, j);
		}
		dst[k] = BETWEEN(&v, &l, &h, symmetric, linc, hinc, nils_false, anti);
		nils += dst[k] == BIT_NIL;
	}
	bn->sorted = ci.n <= 1 || nils == ci.n;
	bn->revsorted = ci.n <= 1 || nils == ci.n;
	bn->key = ci.n <= 1;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	return bn;
}

/* ---------------------------------------------------------------------- */
/* BATconvert (gdk/gdk_calc_convert.c:1415-1548), numeric and oid types.
 * oid's storage, nil and comparison are lng's, so ATOMbasetype(oid) == lng
 * (gdk/gdk_atoms.c:1720-1737): an oid column converts as a lng column, and
 * a conversion to oid takes convert_lng_oid & co. */

static int
cbtype(int t)
{
	return t == ORA_oid ? ORA_lng : btype(t);
}

static ora_hge
scale_of(int k)
{
	ora_hge v = 1;
	while (k-- > 0)
		v *= 10;
	return v;
}

static ora_hge
imax(int t)
{
	switch (t) {
	case ORA_bte: return INT8_MAX;
	case ORA_sht: return INT16_MAX;
	case ORA_int: return INT32_MAX;
	case ORA_lng: return INT64_MAX;
	default: return HGE_MAX;
	}
}

static int
ibits(int t)
{
	return t == ORA_bte ? 8 : t == ORA_sht ? 16 : t == ORA_int ? 32 : t == ORA_lng ? 64 : 128;
}

static void
fmt_num(char *buf, size_t sz, const num *v)
{
	/* FMT##TYPE1 / CST##TYPE1 (gdk/gdk_calc_private.h:300-321) */
	switch (v->t) {
	case ORA_bte: case ORA_sht: case ORA_int: snprintf(buf, sz, "%d", (int) v->i); break;
	case ORA_lng: snprintf(buf, sz, "%lld", (long long) v->i); break;
	case ORA_hge: snprintf(buf, sz, "%.40Lg (approx. value)", (long double) v->i); break;
	case ORA_flt: snprintf(buf, sz, "%.9g", v->f); break;
	case ORA_dbl: snprintf(buf, sz, "%.17g", v->d); break;
	case ORA_oid: snprintf(buf, sz, "%llu", (unsigned long long) v->i); break;
	}
}

static void
conv_overflow(const num *v, const char *to, int scale, int prec)
{
	/* CONV_OVERFLOW / CONV_OVERFLOW_PREC (gdk_calc_convert.c:148-166) */
	if (prec > 0) {
		ora_seterr("22003!overflow in conversion to DECIMAL(%d,%d).\n", prec, scale);
	} else {
		char a[96];
		fmt_num(a, sizeof(a), v);
		ora_seterr("22003!overflow in conversion of %s to %s.\n", a, to);
	}
}

static void
put_int(int tp, void *base, uint64_t k, ora_hge v)
{
	switch (tp) {
	case ORA_bte: ((int8_t *) base)[k] = (int8_t) v; break;
	case ORA_sht: ((int16_t *) base)[k] = (int16_t) v; break;
	case ORA_int: ((int32_t *) base)[k] = (int32_t) v; break;
	case ORA_lng: ((int64_t *) base)[k] = (int64_t) v; break;
	case ORA_hge: ((ora_hge *) base)[k] = v; break;
	}
}

static void
put_nil(int tp, void *base, uint64_t k)
{
	switch (tp) {
	case ORA_flt: ((float *) base)[k] = nanf(""); break;
	case ORA_dbl: ((double *) base)[k] = nan(""); break;
	case ORA_hge: ((ora_hge *) base)[k] = HGE_NIL; break;
	default: put_int(tp, base, k, -imax(tp) - 1); break;
	}
}

/* the scale factors the reference casts to the C types of the conversion;
 * a factor that does not fit wraps there, and is refused here */
static bool
scales_fit(int st, int dt, bool to_oid, bool to_bit, int scale1, int scale2, int prec)
{
	if (scale1 > 38 || scale2 > 38 || prec > 38)
		return false;
	if (to_oid || to_bit)
		return true;
	if (is_int(st) && is_int(dt))
		return scale_of(scale1 > scale2 ? scale1 - scale2 : 0) <= imax(st) &&
		       scale_of(scale2 > scale1 ? scale2 - scale1 : 0) <= imax(dt) &&
		       scale_of(prec) <= imax(dt);
	if (is_int(st))
		return scale_of(scale1) <= imax(st);
	if (is_int(dt))   /* the device computes v * 10^scale2 exactly up to 10^18 */
		return scale2 <= 18 && scale_of(scale2) <= imax(dt) && scale_of(prec) <= imax(dt);
	return true;
}

/* one value; returns 0, 1 (nil), -1 (overflow: message set) */
static int
conv_one(const num *v, int dt, bool to_oid, bool to_bit, void *dst, uint64_t k, int scale1,
	 int scale2, int prec, bool *reduce)
{
	const int st = v->t;
	if (v->nil) {
		put_nil(dt, dst, k);
		return 1;
	}
	if (to_bit) {
		/* convert2bit_impl (:426-459) */
		*reduce = true;
		((int8_t *) dst)[k] = st == ORA_flt ? v->f != 0 : st == ORA_dbl ? v->d != 0 : v->i != 0;
		return 0;
	}
	if (to_oid) {
		/* convertimpl_oid_enlarge (bte..lng) / _reduce (hge, flt, dbl)
		 * (:168-250); GDK_oid_max = 2^63 - 1 */
		*reduce = false;
		ora_oid o;
		if (is_int(st)) {
			if (v->i < 0 || v->i > (ora_hge) INT64_MAX) {
				conv_overflow(v, "oid", 0, 0);
				return -1;
			}
			o = (ora_oid) v->i;
		} else if (st == ORA_flt) {
			if (v->f < 0 || v->f > (float) INT64_MAX) {
				conv_overflow(v, "oid", 0, 0);
				return -1;
			}
			o = (ora_oid) v->f;
		} else {
			if (v->d < 0 || v->d > (double) INT64_MAX) {
				conv_overflow(v, "oid", 0, 0);
				return -1;
			}
			o = (ora_oid) v->d;
		}
		if (o == ORA_OID_NIL) {
			conv_overflow(v, "oid", 0, 0);
			return -1;
		}
		((ora_oid *) dst)[k] = o;
		return 0;
	}
	if (is_int(st) && is_int(dt)) {
		/* convertimpl (:262-363): scale up (mul) or down (DIVIDE rounds half
		 * away from zero), then the range / precision check */
		const ora_hge div = scale_of(scale1 > scale2 ? scale1 - scale2 : 0);
		const ora_hge mul = scale_of(scale2 > scale1 ? scale2 - scale1 : 0);
		const ora_hge max = imax(dt) / mul, min = -max;
		const ora_hge pr = scale_of(prec) / mul;
		*reduce = div > 1;
		ora_hge x = v->i;
		if (div > 1)
			x = x < 0 ? -((-x + div / 2) / div) : (x + div / 2) / div;
		if (x < min || x > max || (prec && (x >= pr || x <= -pr))) {
			conv_overflow(v, tname(dt), scale2, prec);
			return -1;
		}
		put_int(dt, dst, k, x * mul);
		return 0;
	}
	if (is_int(st)) {
		/* convertimpl_enlarge_float (:98-146): (TYPE2) v / div */
		const ora_hge div = scale_of(scale1);
		if (dt == ORA_flt) {
			*reduce = ibits(st) > FLT_MANT_DIG;
			((float *) dst)[k] = div == 1 ? (float) v->i : (float) v->i / (float) div;
		} else {
			*reduce = ibits(st) > DBL_MANT_DIG;
			((double *) dst)[k] = div == 1 ? (double) v->i : (double) v->i / (double) div;
		}
		return 0;
	}
	if (dt == ORA_flt || dt == ORA_dbl) {
		/* flt -> flt / dbl and dbl -> dbl are exact; dbl -> flt is
		 * convertimpl_reduce_float with rounddbl(x) = x (:639-640) */
		if (st == ORA_dbl && dt == ORA_flt) {
			*reduce = true;
			if (v->d < -FLT_MAX || v->d > FLT_MAX) {
				conv_overflow(v, "flt", 0, 0);
				return -1;
			}
			((float *) dst)[k] = (float) (long double) v->d;
		} else if (dt == ORA_flt) {
			((float *) dst)[k] = v->f;
		} else {
			((double *) dst)[k] = st == ORA_flt ? (double) v->f : v->d;
		}
		return 0;
	}
	/* convertimpl_reduce_float (:365-424): (TYPE2) roundl((ldouble) v * mul),
	 * then the nil and precision checks; the reference's long double is
	 * x87 80-bit, which the oracle's host has too */
	*reduce = true;
	const char *to = dt == ORA_bte ? "bte" : dt == ORA_sht ? "sht" : dt == ORA_int ? "int" : dt == ORA_lng ? "lng" : "hge";
	const ora_hge mul = scale_of(scale2);
	const ora_hge max = imax(dt);
	const ora_hge pr = scale_of(prec);
	const bool out = st == ORA_flt ? (v->f < (float) -max || v->f > (float) max)
				       : (v->d < (double) -max || v->d > (double) max);
	if (out) {
		conv_overflow(v, to, scale2, prec);
		return -1;
	}
	long double x = st == ORA_flt ? (long double) v->f : (long double) v->d;
	long double m = roundl(x * (long double) mul);
	/* out of the type's range the conversion yields the nil value (x87
	 * "integer indefinite") for int and lng; refused the same way for all */
	if (m < -(long double) max || m > (long double) max) {
		conv_overflow(v, to, scale2, prec);
		return -1;
	}
	ora_hge r = (ora_hge) m;
	if (prec && (r >= pr || r <= -pr)) {
		conv_overflow(v, to, scale2, prec);
		return -1;
	}
	put_int(dt, dst, k, r);
	return 0;
}

ora_bat *
ora_convert(const ora_bat *b, const ora_bat *s, int tp, int scale1, int scale2, int prec)
{
	ora_ci ci;
	if (tp == ORA_void)
		tp = ORA_oid;
	if (ora_ci_init(&ci, b, s) < 0)
		return NULL;
	const ora_oid hseq = s ? s->hseqbase : b->hseqbase;
	const int st = b->type == ORA_void ? ORA_void : cbtype(b->type), dt = cbtype(tp);
	const bool to_oid = tp == ORA_oid, to_bit = tp == ORA_bit;
	if ((!is_num(st) && st != ORA_void) || !is_num(dt)) {
		ora_seterr("type combination (convert(%s)->%s) not supported.\n", tname(b->type), tname(tp));
		return NULL;
	}
	if (ci.n == 0 || (b->type == ORA_void && b->tseqbase == ORA_OID_NIL)) {
		/* BATconstant(ci.hseq, tp, nil, ncand) */
		ora_bat *bn = ora_new(tp, ci.n, hseq);
		if (bn == NULL)
			return NULL;
		for (uint64_t k = 0; k < ci.n; k++)
			put_nil(dt, bn->base, k);
		bn->sorted = bn->revsorted = 1;
		bn->key = ci.n <= 1;
		bn->nil = ci.n >= 1;
		bn->nonil = !bn->nil;
		return bn;
	}
	if (ci.n == b->count && !to_bit && st == dt && (!to_oid || b->type == ORA_oid) &&
	    scale1 == 0 && scale2 == 0 && prec == 0) {
		/* COLcopy (gdk_calc_convert.c:1443-1455) */
		ora_bat *bn = ora_new(tp, ci.n, hseq);
		if (bn == NULL)
			return NULL;
		memcpy(bn->base, b->base, ci.n * (size_t) bn->width);
		bn->sorted = b->sorted;
		bn->revsorted = b->revsorted;
		bn->key = b->key;
		bn->nonil = b->nonil;
		bn->nil = b->nil;
		bn->minpos = b->minpos;
		bn->maxpos = b->maxpos;
		bn->unique_est = b->unique_est;
		return bn;
	}
	if (st != ORA_void && !scales_fit(st, dt, to_oid, to_bit, scale1, scale2, prec)) {
		ora_seterr("convert: scale factor does not fit %s\n", tname(tp));
		return NULL;
	}
	ora_bat *bn = ora_new(tp, ci.n, hseq);
	if (bn == NULL)
		return NULL;
	uint64_t nils = 0;
	bool reduce = false;
	if (b->type == ORA_void) {
		/* convert_void_any (:870-979) */
		for (uint64_t k = 0; k < ci.n; k++) {
			ora_oid o = b->tseqbase + (ci_get(&ci, k) - b->hseqbase);
			if (to_bit) {
				((int8_t *) bn->base)[k] = 1;   /* its loop overwrites dst[0] too */
			} else if (dt == ORA_flt) {
				((float *) bn->base)[k] = (float) o;
			} else if (dt == ORA_dbl) {
				((double *) bn->base)[k] = (double) o;
			} else {
				if ((dt == ORA_bte || dt == ORA_sht || dt == ORA_int) && o > (ora_oid) imax(dt)) {
					ora_seterr("22003!overflow in conversion of %llu to %s.\n", (unsigned long long) o,
						   tname(dt));
					ora_free(bn);
					return NULL;
				}
				put_int(dt, bn->base, k, (ora_hge) o);
			}
		}
	} else {
		for (uint64_t k = 0; k < ci.n; k++) {
			num v = load(st, b->base, ci_get(&ci, k) - b->hseqbase);
			int r = conv_one(&v, dt, to_oid, to_bit, bn->base, k, scale1, scale2, prec, &reduce);
			if (r < 0) {
				ora_free(bn);
				return NULL;
			}
			nils += r;
		}
	}
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	/* :1528-1537 (no str on this path) */
	if (!to_bit || ci.n < 2) {
		bn->sorted = nils == 0 && b->sorted;
		bn->revsorted = nils == 0 && b->revsorted;
	} else {
		bn->sorted = bn->revsorted = 0;
	}
	bn->key = (!reduce || ci.n < 2) ? (b->key && nils <= 1) : 0;
	return bn;
}

/* ---------------------------------------------------------------------- */
/* BATcalcnot (gdk/gdk_calc.c:41-146) */
ora_bat *
ora_calcnot(const ora_bat *b, const ora_bat *s)
{
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return NULL;
	const ora_oid hseq = s ? s->hseqbase : b->hseqbase;
	const int t = btype(b->type);
	if (!is_int(t)) {
		ora_seterr("type %s not supported.\n", tname(b->type));
		return NULL;
	}
	ora_bat *bn = ora_new(b->type, ci.n, hseq);
	if (bn == NULL)
		return NULL;
	if (ci.n == 0) {
		bn->sorted = bn->revsorted = 1;
		bn->key = 1;
		bn->nil = 0;
		bn->nonil = 1;
		return bn;
	}
	uint64_t nils = 0;
	for (uint64_t k = 0; k < ci.n; k++) {
		num v = load(t, b->base, ci_get(&ci, k) - b->hseqbase);
		if (v.nil) {
			put_nil(t, bn->base, k);
			nils++;
		} else if (b->type == ORA_bit) {
			((int8_t *) bn->base)[k] = !v.i;
		} else {
			ora_hge r = ~v.i;   /* NOT(x) = ~x; ~max is the nil value */
			if (r == -imax(t) - 1) {
				char a[96];
				fmt_num(a, sizeof(a), &v);
				ora_seterr("22003!overflow in calculation NOT(%s).\n", a);
				ora_free(bn);
				return NULL;
			}
			put_int(t, bn->base, k, r);
		}
	}
	bn->sorted = nils == 0 && b->revsorted;
	bn->revsorted = nils == 0 && b->sorted;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	bn->key = b->key && nils <= 1;
	return bn;
}

/* ---------------------------------------------------------------------- */
/* division and modulo */

static int
rank(int t)
{
	return t == ORA_bte ? 0 : t == ORA_sht ? 1 : t == ORA_int ? 2 : t == ORA_lng ? 3 : t == ORA_hge ? 4
		: t == ORA_flt ? 5 : 6;
}

/* the instantiated DIV_3TYPE / DIV_3TYPE_float / MOD_3TYPE / FMOD_3TYPE
 * combinations (gdk_calc_div.c, gdk_calc_mod.c) */
static bool
divmod_supported(char op, int t1, int t2, int tp)
{
	if (!is_num(t1) || !is_num(t2) || !is_num(tp))
		return false;
	const int r1 = rank(t1), r2 = rank(t2), rp = rank(tp);
	if (op == '/') {
		if (r2 >= 5)   /* float divisor: flt -> flt/dbl, dbl -> dbl */
			return r1 == 6 ? rp == 6 : (r2 == 5 ? rp >= 5 : rp == 6);
		if (r1 >= 5)   /* float dividend, integer divisor */
			return rp >= r1;
		return rp >= r1 || rp >= 5;
	}
	if (r1 <= 4 && r2 <= 4)   /* MOD_3TYPE: result at least the narrower operand */
		return rp <= 4 && rp >= (r1 < r2 ? r1 : r2);
	/* FMOD_3TYPE: one float operand; result its type, or dbl when either is dbl */
	return rp == (r1 == 6 || r2 == 6 ? 6 : 5);
}

ora_bat *
ora_calcdivmod(char op, const ora_bat *b1, const void *c1, int t1, const ora_bat *b2, const void *c2,
	       int t2, const ora_bat *s1, const ora_bat *s2, int tp)
{
	opnd l = {.b = b1, .c = c1}, r = {.b = b2, .c = c2};
	const ora_bat *bb = b1 ? b1 : b2;
	ora_ci ci;
	const char *fname = op == '/' ? (b1 && b2 ? "BATcalcdiv" : b1 ? "BATcalcdivcst" : "BATcalccstdiv")
				      : (b1 && b2 ? "BATcalcmod" : b1 ? "BATcalcmodcst" : "BATcalccstmod");
	if (b1 && b2) {
		if (ora_ci_init(&l.ci, b1, s1) < 0 || ora_ci_init(&r.ci, b2, s2) < 0)
			return NULL;
		ora_oid h1 = s1 ? s1->hseqbase : b1->hseqbase, h2 = s2 ? s2->hseqbase : b2->hseqbase;
		if (l.ci.n != r.ci.n || h1 != h2) {
			ora_seterr("%s: inputs not the same size.\n", fname);
			return NULL;
		}
		ci = l.ci;
	} else {
		if (ora_ci_init(&ci, bb, s1) < 0)
			return NULL;
		if (b1)
			l.ci = ci;
		else
			r.ci = ci;
	}
	const ora_oid hseq = s1 ? s1->hseqbase : bb->hseqbase;
	l.t = btype(b1 ? b1->type : t1);
	r.t = btype(b2 ? b2->type : t2);
	const int dt = btype(tp);
	if (ci.n == 0) {
		ora_bat *bn = ora_new(tp, 0, hseq);
		if (bn) {
			bn->sorted = bn->revsorted = bn->key = bn->nonil = 1;
		}
		return bn;
	}
	if (!divmod_supported(op, l.t, r.t, dt)) {
		ora_seterr("%s: type combination (%s(%s,%s)->%s) not supported.\n", fname, op == '/' ? "div" : "mod",
			   tname(l.t), tname(r.t), tname(dt));
		return NULL;
	}
	ora_bat *bn = ora_new(tp, ci.n, hseq);
	if (bn == NULL)
		return NULL;
	uint64_t nils = 0;
	const void *lb = base_of(&l), *rb = base_of(&r);
	for (uint64_t k = 0; k < ci.n; k++) {
		num a = load(l.t, lb, b1 ? pos_of(&l, k) : 0);
		num b = load(r.t, rb, b2 ? pos_of(&r, k) : 0);
		if (a.nil || b.nil) {
			put_nil(dt, bn->base, k);
			nils++;
			continue;
		}
		const bool bzero = r.t == ORA_flt ? b.f == 0 : r.t == ORA_dbl ? b.d == 0 : b.i == 0;
		if (bzero) {
			ora_seterr("22012!division by zero.\n");
			ora_free(bn);
			return NULL;
		}
		if (op == '/') {
			/* DIV_3TYPE (:21-74): (TYPE3) (lft / rgt) in C's types;
			 * DIV_3TYPE_float (:76-140): (TYPE3) lft / rgt after the
			 * overflow pre-check.  A result beyond the type's range
			 * fails without a message (BUN_NONE + 2). */
			double q;
			if (r.t == ORA_flt || r.t == ORA_dbl) {
				const double ay = r.t == ORA_flt ? (double) fabsf(b.f) : fabs(b.d);
				const double ax = a.t == ORA_flt ? (double) fabsf(a.f) : a.t == ORA_dbl ? fabs(a.d)
						: (double) (a.i < 0 ? -a.i : a.i);
				bool ovf;
				if (dt == ORA_flt)
					ovf = fabsf(b.f) < 1 && FLT_MAX * fabsf(b.f) < (a.t == ORA_flt ? fabsf(a.f) : (float) (a.i < 0 ? -a.i : a.i));
				else
					ovf = ay < 1 && DBL_MAX * ay < ax;
				if (ovf) {
					char u[96], w[96];
					fmt_num(u, sizeof(u), &a);
					fmt_num(w, sizeof(w), &b);
					ora_seterr("22003!overflow in calculation %s/%s.\n", u, w);
					ora_free(bn);
					return NULL;
				}
				q = dt == ORA_flt ? (double) (as_flt(&a) / b.f) : as_dbl(&a) / as_dbl(&b);
			} else if (a.t == ORA_flt) {
				float f = a.f / (float) b.i;
				q = f;
			} else if (a.t == ORA_dbl) {
				q = a.d / (double) b.i;
			} else {
				ora_hge qi = a.i / b.i;
				if (dt == ORA_flt) {
					((float *) bn->base)[k] = (float) qi;
				} else if (dt == ORA_dbl) {
					((double *) bn->base)[k] = (double) qi;
				} else if (qi < -imax(dt) || qi > imax(dt)) {
					ora_seterr("%s", "");
					ora_free(bn);
					return NULL;
				} else {
					put_int(dt, bn->base, k, qi);
				}
				continue;
			}
			const double lim = dt == ORA_flt ? FLT_MAX : DBL_MAX;
			if (q < -lim || q > lim) {
				ora_seterr("%s", "");
				ora_free(bn);
				return NULL;
			}
			if (dt == ORA_flt)
				((float *) bn->base)[k] = (float) q;
			else
				((double *) bn->base)[k] = q;
		} else {
			if (dt == ORA_flt) {
				((float *) bn->base)[k] = fmodf(as_flt(&a), as_flt(&b));
			} else if (dt == ORA_dbl) {
				((double *) bn->base)[k] = fmod(as_dbl(&a), as_dbl(&b));
			} else {
				/* MOD_3TYPE: (TYPE3) lft % rgt -- lft is cast to the
				 * result type first */
				ora_hge x;
				switch (dt) {
				case ORA_bte: x = (int8_t) a.i; break;
				case ORA_sht: x = (int16_t) a.i; break;
				case ORA_int: x = (int32_t) a.i; break;
				case ORA_lng: x = (int64_t) a.i; break;
				default: x = a.i; break;
				}
				put_int(dt, bn->base, k, x % b.i);
			}
		}
	}
	bn->sorted = ci.n <= 1 || nils == ci.n;
	bn->revsorted = ci.n <= 1 || nils == ci.n;
	bn->key = ci.n <= 1;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	return bn;
}

/* ---------------------------------------------------------------------- */
/* the rest of gdk_calc.c's element-wise operators: BATcalcnegate,
 * -absolute, -iszero, -sign (gdk_calc.c:233-800; UNARY_2TYPE_FUNC
 * gdk_calc_private.h:354), -isnil / -isnotnil (:802-920), min / max with
 * their _no_nil and constant forms (MINMAX_TYPE :944, MINMAX_NONIL_TYPE
 * :1150, MINMAX_CST_TYPE :1385, MINMAX_NONIL_CST_TYPE :1535), xor / or / and
 * (:2439-3030; bit: or3 / and3 :2590 / :2826, XORBIT; integers: a result
 * equal to nil is "overflow in calculation"), lsh / rsh (:3059-3760:
 * SHIFT_CHECK, LSH_CHECK, "shift operand too large"), ifthenelse
 * (:4376-4760: a nil condition takes the else branch). */

enum { XO_NEG, XO_ABS, XO_ISZERO, XO_SIGN, XO_ISNIL, XO_ISNOTNIL, XO_MIN, XO_MAX, XO_MINNN, XO_MAXNN, XO_AND,
       XO_OR, XO_XOR, XO_LSH, XO_RSH };

static num
nilnum(int t)
{
	num v = {.t = t, .nil = true, .f = NAN, .d = NAN};
	switch (t) {
	case ORA_bte: v.i = INT8_MIN; break;
	case ORA_sht: v.i = INT16_MIN; break;
	case ORA_int: v.i = INT32_MIN; break;
	case ORA_lng: v.i = INT64_MIN; break;
	case ORA_hge: v.i = HGE_NIL; break;
	case ORA_oid: v.i = (ora_hge) ORA_OID_NIL; break;
	}
	return v;
}

static void
store(int t, void *base, uint64_t k, const num *v)
{
	switch (t) {
	case ORA_bte: ((int8_t *) base)[k] = (int8_t) v->i; break;
	case ORA_sht: ((int16_t *) base)[k] = (int16_t) v->i; break;
	case ORA_int: ((int32_t *) base)[k] = (int32_t) v->i; break;
	case ORA_lng: ((int64_t *) base)[k] = (int64_t) v->i; break;
	case ORA_hge: ((ora_hge *) base)[k] = v->i; break;
	case ORA_oid: ((ora_oid *) base)[k] = (ora_oid) v->i; break;
	case ORA_flt: ((float *) base)[k] = v->f; break;
	case ORA_dbl: ((double *) base)[k] = v->d; break;
	}
}

/* value k of an operand; void columns count from their tseqbase */
static num
getv(const opnd *o, uint64_t k)
{
	if (o->b && o->b->type == ORA_void) {
		const ora_oid s = o->b->tseqbase;
		num v = {.t = ORA_oid, .nil = s == ORA_OID_NIL, .i = (ora_hge) (s == ORA_OID_NIL ? s : s + pos_of(o, k))};
		return v;
	}
	return load(o->t, base_of(o), o->b ? pos_of(o, k) : 0);
}

static bool
lt(const num *a, const num *b)
{
	if (a->t == ORA_flt)
		return a->f < b->f;
	if (a->t == ORA_dbl)
		return a->d < b->d;
	if (a->t == ORA_oid)
		return (unsigned __int128) a->i < (unsigned __int128) b->i;
	return a->i < b->i;
}

static bool
tdense_(const ora_bat *b)
{
	return (b->type == ORA_void || b->type == ORA_oid) && b->tseqbase != ORA_OID_NIL;
}

ora_bat *
ora_calcunary(int op, const ora_bat *b, const ora_bat *s)
{
	opnd o = {.b = b};
	if (ora_ci_init(&o.ci, b, s) < 0)
		return NULL;
	const uint64_t n = o.ci.n;
	const ora_oid hseq = s ? s->hseqbase : b->hseqbase;
	if (op == XO_ISNIL || op == XO_ISNOTNIL) {
		const bool notnil = op == XO_ISNOTNIL;
		if (b->nonil || tdense_(b) || b->type == ORA_void) {
			ora_bat *bn = ora_new(ORA_bit, n, hseq);
			if (bn == NULL)
				return NULL;
			memset(bn->base, (b->nonil || tdense_(b)) ? notnil : !notnil, n);
			bn->sorted = bn->revsorted = 1;
			bn->key = n <= 1;
			bn->nil = 0;
			bn->nonil = 1;
			return bn;
		}
	}
	const int t = b->type == ORA_oid ? ORA_oid : btype(b->type);
	if (!is_num(t) && !((op == XO_ISNIL || op == XO_ISNOTNIL) && t == ORA_oid)) {
		ora_seterr("type %s not supported.\n", tname(b->type));
		return NULL;
	}
	o.t = t;
	const int otp = op == XO_ISZERO || op == XO_ISNIL || op == XO_ISNOTNIL ? ORA_bit : op == XO_SIGN ? ORA_bte
											       : b->type;
	const int ot = btype(otp);
	ora_bat *bn = ora_new(otp, n, hseq);
	if (bn == NULL)
		return NULL;
	uint64_t nils = 0;
	for (uint64_t k = 0; k < n; k++) {
		num v = getv(&o, k), r = v;
		if (op == XO_ISNIL || op == XO_ISNOTNIL) {
			((int8_t *) bn->base)[k] = (int8_t) (v.nil != (op == XO_ISNOTNIL));
			continue;
		}
		if (v.nil) {
			num z = nilnum(ot);
			store(ot, bn->base, k, &z);
			nils++;
			continue;
		}
		switch (op) {
		case XO_NEG: r.i = -v.i; r.f = -v.f; r.d = -v.d; break;
		case XO_ABS: r.i = v.i < 0 ? -v.i : v.i; r.f = fabsf(v.f); r.d = fabs(v.d); break;
		case XO_ISZERO:
			r.t = ORA_bte;
			r.i = t == ORA_flt ? v.f == 0 : t == ORA_dbl ? v.d == 0 : v.i == 0;
			break;
		case XO_SIGN:
			r.t = ORA_bte;
			r.i = t == ORA_flt ? (v.f < 0 ? -1 : v.f > 0) : t == ORA_dbl ? (v.d < 0 ? -1 : v.d > 0)
										 : (v.i < 0 ? -1 : v.i > 0);
			break;
		}
		store(ot, bn->base, k, &r);
	}
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	bn->key = n <= 1;
	switch (op) {
	case XO_NEG:
		bn->sorted = nils == 0 && b->revsorted;
		bn->revsorted = nils == 0 && b->sorted;
		bn->key = b->key && nils <= 1;
		break;
	case XO_SIGN:
		bn->sorted = b->sorted || n <= 1 || nils == n;
		bn->revsorted = b->revsorted || n <= 1 || nils == n;
		break;
	case XO_ISNIL:
		bn->sorted = b->revsorted;
		bn->revsorted = b->sorted;
		break;
	case XO_ISNOTNIL:
		bn->sorted = b->sorted;
		bn->revsorted = b->revsorted;
		break;
	default:
		bn->sorted = bn->revsorted = n <= 1 || nils == n;
		break;
	}
	return bn;
}

/* min / max (b2 NULL: the constant c of type ct) and their _no_nil forms */
ora_bat *
ora_calcminmax(int op, const ora_bat *b1, const ora_bat *b2, const void *c, int ct, const ora_bat *s1,
	       const ora_bat *s2)
{
	const int a1 = b1->type == ORA_void ? ORA_oid : b1->type;
	const int a2 = b2 ? (b2->type == ORA_void ? ORA_oid : b2->type) : (ct == ORA_void ? ORA_oid : ct);
	if (a1 != a2) {
		ora_seterr("inputs have incompatible types\n");
		return NULL;
	}
	opnd l = {.b = b1}, r = {.b = b2, .c = c};
	if (ora_ci_init(&l.ci, b1, s1) < 0 || (b2 && ora_ci_init(&r.ci, b2, s2) < 0))
		return NULL;
	const ora_oid h1 = s1 ? s1->hseqbase : b1->hseqbase;
	if (b2 && (l.ci.n != r.ci.n || h1 != (s2 ? s2->hseqbase : b2->hseqbase))) {
		ora_seterr("inputs not the same size.\n");
		return NULL;
	}
	const int t = a1 == ORA_oid ? ORA_oid : btype(b1->type);
	l.t = r.t = t;
	const uint64_t n = l.ci.n;
	ora_bat *bn = ora_new(a1, n, h1);
	if (bn == NULL)
		return NULL;
	const bool domax = op == XO_MAX || op == XO_MAXNN, nonil = op == XO_MINNN || op == XO_MAXNN;
	const num cv = b2 ? (num) {0} : load(t, c, 0);
	const bool allnil1 = b1->type == ORA_void && b1->tseqbase == ORA_OID_NIL;
	bool nils = false;
	for (uint64_t k = 0; k < n; k++) {
		num p = getv(&l, k), q = b2 ? getv(&r, k) : cv, res;
		if (!b2 && !nonil && (cv.nil || allnil1)) {
			res = nilnum(t);                          /* BATconstantV(nil) */
		} else if (!nonil) {
			if (p.nil || q.nil)
				res = nilnum(t);
			else if (b2)
				res = (domax ? lt(&q, &p) : lt(&p, &q)) ? p : q;     /* p1 OP p2 ? p1 : p2 */
			else
				res = (domax ? lt(&q, &p) : lt(&p, &q)) ? p : q;     /* p1 OP pp2 ? p1 : pp2 */
		} else if (b2) {
			/* MINMAX_NONIL_TYPE: p1 nil -> p2; else (!nil(p2) && p2 OP p1) ? p2 : p1 */
			if (p.nil)
				res = q;
			else
				res = !q.nil && (domax ? lt(&p, &q) : lt(&q, &p)) ? q : p;
		} else {
			/* MINMAX_NONIL_CST_TYPE */
			if (cv.nil)
				res = p;
			else if (p.nil)
				res = cv;
			else
				res = (domax ? lt(&cv, &p) : lt(&p, &cv)) ? p : cv;
		}
		nils |= res.nil;
		store(t, bn->base, k, &res);
	}
	bn->nil = nils;
	bn->nonil = !nils;
	bn->sorted = bn->revsorted = bn->key = n <= 1;
	bn->tseqbase = a1 == ORA_oid && n <= 1 ? (n == 1 ? ((ora_oid *) bn->base)[0] : 0) : ORA_OID_NIL;
	return bn;
}

static const char *const xo_opname[] = {[XO_AND] = "AND", [XO_OR] = "OR", [XO_XOR] = "XOR", [XO_LSH] = "LSH",
					[XO_RSH] = "RSH"};

static void
fmtnum(char *buf, size_t sz, const num *v)
{
	switch (v->t) {
	case ORA_bte: case ORA_sht: case ORA_int: snprintf(buf, sz, "%d", (int) v->i); break;
	case ORA_lng: snprintf(buf, sz, "%lld", (long long) v->i); break;
	case ORA_hge: snprintf(buf, sz, "%.40Lg (approx. value)", (long double) v->i); break;
	default: snprintf(buf, sz, "%llu", (unsigned long long) v->i); break;
	}
}

/* xor / or / and / lsh / rsh of (b1 | c1) with (b2 | c2); fname for the
 * shift message */
ora_bat *
ora_calcbits(int op, const char *fname, const ora_bat *b1, const void *c1, int t1, const ora_bat *b2,
	     const void *c2, int t2, const ora_bat *s1, const ora_bat *s2)
{
	const int ta = b1 ? b1->type : t1, tb = b2 ? b2->type : t2;
	const bool shift = op == XO_LSH || op == XO_RSH;
	if (!shift && btype(ta) != btype(tb)) {
		ora_seterr("incompatible input types.\n");
		return NULL;
	}
	opnd l = {.b = b1, .c = c1}, r = {.b = b2, .c = c2};
	const ora_bat *bb = b1 ? b1 : b2;
	ora_ci ci;
	if (b1 && b2) {
		if (ora_ci_init(&l.ci, b1, s1) < 0 || ora_ci_init(&r.ci, b2, s2) < 0)
			return NULL;
		if (l.ci.n != r.ci.n || (s1 ? s1->hseqbase : b1->hseqbase) != (s2 ? s2->hseqbase : b2->hseqbase)) {
			ora_seterr("inputs not the same size.\n");
			return NULL;
		}
		ci = l.ci;
	} else {
		if (ora_ci_init(&ci, bb, s1) < 0)
			return NULL;
		if (b1)
			l.ci = ci;
		else
			r.ci = ci;
	}
	const ora_oid hseq = s1 ? s1->hseqbase : bb->hseqbase;
	const uint64_t n = ci.n;
	ora_bat *bn = ora_new(ta, n, hseq);
	if (bn == NULL || n == 0)
		return bn;
	l.t = btype(ta);
	r.t = btype(tb);
	if (!is_int(l.t) || !is_int(r.t)) {
		ora_free(bn);
		ora_seterr("%s: bad input type %s.\n", fname, tname(is_int(l.t) ? tb : ta));
		return NULL;
	}
	const int bits = ora_width(l.t) * 8;
	const ora_hge mx = bits == 128 ? HGE_MAX : (((ora_hge) 1 << (bits - 1)) - 1);
	const num NIL = nilnum(l.t);
	uint64_t nils = 0;
	for (uint64_t k = 0; k < n; k++) {
		num p = getv(&l, k), q = getv(&r, k), res = p;
		bool fail = false;
		if (ta == ORA_bit && (op == XO_AND || op == XO_OR)) {
			int8_t v1 = (int8_t) p.i, v2 = (int8_t) q.i;
			res.i = op == XO_OR ? or3(v1, v2) : and3(v1, v2);
			res.nil = res.i == INT8_MIN;
		} else if (p.nil || q.nil) {
			res = NIL;
		} else if (ta == ORA_bit) {
			res.i = (p.i == 0) != (q.i == 0);
		} else if (!shift) {
			res.i = op == XO_AND ? (p.i & q.i) : op == XO_OR ? (p.i | q.i) : (p.i ^ q.i);
			fail = res.i == NIL.i && op != XO_OR;
		} else if (q.i < 0 || q.i >= bits || (op == XO_LSH && (p.i < 0 || p.i > (mx >> (int) q.i)))) {
			fail = true;
		} else {
			res.i = op == XO_LSH ? p.i << (int) q.i : p.i >> (int) q.i;
		}
		if (fail) {
			char x[96], y[96];
			fmtnum(x, sizeof(x), &p);
			fmtnum(y, sizeof(y), &q);
			if (shift)
				ora_seterr("%s: shift operand too large in %s(%s,%s).\n", fname, xo_opname[op], x, y);
			else
				ora_seterr("22003!overflow in calculation %s%s%s.\n", x, xo_opname[op], y);
			ora_free(bn);
			return NULL;
		}
		nils += res.nil || (ta != ORA_bit && (p.nil || q.nil));
		store(l.t, bn->base, k, &res);
	}
	bn->sorted = bn->revsorted = n <= 1 || nils == n;
	bn->key = n <= 1;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	return bn;
}

/* BATcalcifthenelse and its constant forms (b1 / b2 NULL: c1 / c2 of type
 * ct); a void column yields its sequence at the row (gdk_calc.c:4550-4561) */
ora_bat *
ora_calcifthenelse(const ora_bat *b, const ora_bat *b1, const void *c1, const ora_bat *b2, const void *c2, int ct)
{
	const int t1 = b1 ? b1->type : ct, t2 = b2 ? b2->type : ct;
	const int a1 = t1 == ORA_void ? ORA_oid : t1, a2 = t2 == ORA_void ? ORA_oid : t2;
	if ((b1 && b1->count != b->count) || (b2 && b2->count != b->count)) {
		ora_seterr("BATcalcifthenelse: BATs have different lengths.\n");
		return NULL;
	}
	if (b->type != ORA_bit || a1 != a2) {
		ora_seterr("\"then\" and \"else\" BATs have different types.\n");
		return NULL;
	}
	const uint64_t n = b->count;
	ora_bat *bn = ora_new(a1, n, b->hseqbase);
	if (bn == NULL)
		return NULL;
	const int w = ora_width(a1);
	for (uint64_t i = 0; i < n; i++) {
		const int8_t c = ((const int8_t *) b->base)[i];
		const bool take1 = c != 0 && c != INT8_MIN;
		const ora_bat *x = take1 ? b1 : b2;
		const void *cv = take1 ? c1 : c2;
		char *dst = (char *) bn->base + i * w;
		if (x && x->type == ORA_void) {
			const ora_oid v = x->tseqbase + i;
			memcpy(dst, &v, 8);
		} else if (x) {
			memcpy(dst, (const char *) x->base + i * w, w);
		} else {
			memcpy(dst, cv, w);
		}
	}
	const bool nonil1 = b1 ? b1->nonil : !cst_is_nil(ct, c1), nonil2 = b2 ? b2->nonil : !cst_is_nil(ct, c2);
	bn->sorted = bn->revsorted = bn->key = n <= 1;
	bn->nil = 0;
	bn->nonil = nonil1 && nonil2;
	return bn;
}
