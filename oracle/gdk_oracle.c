/*
 * gdk_oracle.c -- CPU restatement of the GDK select / project / calc / sum
 * semantics.  TEST INFRASTRUCTURE ONLY (see gdk_oracle.h).
 */
#include "gdk_oracle_private.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread char errbuf[1024];

const char *
ora_errbuf(void)
{
	return errbuf;
}

void
ora_seterr(const char *fmt, ...)
{
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(errbuf, sizeof(errbuf), fmt, ap);
	va_end(ap);
}

int
ora_width(int type)
{
	switch (type) {
	case ORA_void: return 0;
	case ORA_bit: case ORA_bte: return 1;
	case ORA_sht: return 2;
	case ORA_int: case ORA_date: case ORA_flt: return 4;
	case ORA_oid: case ORA_lng: case ORA_dbl: return 8;
	case ORA_hge: return 16;
	case ORA_str: return 1;
	default: return 0;
	}
}

ora_bat *
ora_new(int type, uint64_t count, ora_oid hseq)
{
	ora_bat *b = calloc(1, sizeof(ora_bat));
	if (b == NULL)
		return NULL;
	b->type = type;
	b->width = ora_width(type);
	b->count = count;
	b->hseqbase = hseq;
	b->tseqbase = type == ORA_void ? 0 : ORA_OID_NIL;
	b->minpos = b->maxpos = ORA_BUN_NONE;
	b->owned = 1;
	if (b->width > 0) {
		b->base = malloc(count * b->width + 16);
		if (b->base == NULL) {
			free(b);
			return NULL;
		}
	}
	return b;
}

void
ora_free(ora_bat *b)
{
	if (b == NULL)
		return;
	if (b->owned) {
		free(b->base);
		free(b->vheap);
	}
	free(b);
}

ora_bat *
ora_dense(ora_oid hseq, ora_oid tseq, uint64_t cnt)
{
	ora_bat *b = ora_new(ORA_void, cnt, hseq);
	if (b == NULL)
		return NULL;
	b->tseqbase = tseq;
	b->sorted = b->key = b->nonil = 1;
	b->revsorted = cnt <= 1;
	return b;
}

/* ---------------------------------------------------------------------- */
/* candidate lists: gdk/gdk_cand.c:407 canditer_init; restated as an
 * explicit (seq, n) dense range or a clipped sorted oid array */

static uint64_t
lower_bound_oid(const ora_oid *a, uint64_t n, ora_oid v)
{
	uint64_t lo = 0, hi = n;
	while (lo < hi) {
		uint64_t m = (lo + hi) / 2;
		if (a[m] < v)
			lo = m + 1;
		else
			hi = m;
	}
	return lo;
}

int
ora_ci_init(ora_ci *ci, const ora_bat *b, const ora_bat *s)
{
	ora_oid lo = b ? b->hseqbase : 0;
	ora_oid hi = b ? b->hseqbase + b->count : ~(ora_oid) 0;
	memset(ci, 0, sizeof(*ci));
	ci->dense = true;
	if (s == NULL) {
		ci->seq = lo;
		ci->n = b ? b->count : 0;
		return 0;
	}
	if (s->count == 0 || (b && b->count == 0))
		return 0;
	if (s->type == ORA_void) {
		ora_oid a = s->tseqbase, e = s->tseqbase + s->count;
		if (a < lo)
			a = lo;
		if (e > hi)
			e = hi;
		if (a < e) {
			ci->seq = a;
			ci->n = e - a;
		}
		return 0;
	}
	if (s->type == ORA_msk) {
		/* a bit BAT stands for the oid list BATunmask makes of it
		 * (gdk_cand.c:1549-1590: hseqbase + i for every set bit i <
		 * count); kept in a per-thread ring of 4 lists */
		static __thread ora_oid *ring[4];
		static __thread unsigned next;
		const uint32_t *w = s->base;
		ora_oid *o = malloc((s->count + 1) * sizeof(ora_oid));
		uint64_t k = 0;
		if (o == NULL) {
			ora_seterr("malloc");
			return -1;
		}
		for (uint64_t i = 0; i < s->count; i++)
			if ((w[i >> 5] >> (i & 31)) & 1)
				o[k++] = s->hseqbase + i;
		free(ring[next & 3]);
		ring[next++ & 3] = o;
		ora_bat tmp = {.type = ORA_oid, .width = 8, .count = k, .base = o};
		return ora_ci_init(ci, b, &tmp);
	}
	if (s->type != ORA_oid) {
		ora_seterr("candidate list must be oid");
		return -1;
	}
	const ora_oid *o = s->base;
	uint64_t p = lower_bound_oid(o, s->count, lo);
	uint64_t q = lower_bound_oid(o, s->count, hi);
	if (p >= q)
		return 0;
	ci->n = q - p;
	if (o[q - 1] - o[p] == q - p - 1) {
		ci->seq = o[p];
	} else {
		ci->dense = false;
		ci->oids = o + p;
	}
	return 0;
}

/* result as candidate list: materialized oid BAT, virtualised when dense
 * (gdk/gdk_select.c:31-89 virtualize) */
static ora_bat *
ora_virtualize(ora_bat *bn)
{
	if (bn->type != ORA_oid)
		return bn;
	const ora_oid *o = bn->base;
	if (bn->count <= 1 || o[bn->count - 1] - o[0] == bn->count - 1) {
		ora_oid seq = bn->count ? o[0] : 0;
		free(bn->base);
		bn->base = NULL;
		bn->type = ORA_void;
		bn->width = 0;
		bn->tseqbase = seq;
	}
	bn->sorted = bn->key = bn->nonil = 1;
	bn->nil = 0;
	bn->revsorted = bn->count <= 1;
	return bn;
}

static ora_bat *
ci_slice(const ora_ci *ci)
{
	if (ci->dense)
		return ora_dense(0, ci->seq, ci->n);
	ora_bat *bn = ora_new(ORA_oid, ci->n, 0);
	if (bn == NULL)
		return NULL;
	memcpy(bn->base, ci->oids, ci->n * sizeof(ora_oid));
	return ora_virtualize(bn);
}

/* ---------------------------------------------------------------------- */
/* nil values (gdk/gdk_atoms.h:155-217): the minimum of each signed
 * integer type, NaN for floats */

#define ORA_bte_nil ((int8_t) INT8_MIN)
#define ORA_sht_nil ((int16_t) INT16_MIN)
#define ORA_int_nil ((int32_t) INT32_MIN)
#define ORA_lng_nil ((int64_t) INT64_MIN)
#define ORA_hge_nil ((ora_hge) ((unsigned __int128) 1 << 127))
#define ORA_HGE_MAX ((ora_hge) (((unsigned __int128) 1 << 127) - 1))

static bool
is_nil_val(int t, const void *v)
{
	switch (t) {
	case ORA_bte: case ORA_bit: return *(const int8_t *) v == ORA_bte_nil;
	case ORA_sht: return *(const int16_t *) v == ORA_sht_nil;
	case ORA_int: case ORA_date: return *(const int32_t *) v == ORA_int_nil;
	case ORA_lng: return *(const int64_t *) v == ORA_lng_nil;
	case ORA_hge: return *(const ora_hge *) v == ORA_hge_nil;
	case ORA_oid: return *(const ora_oid *) v == ORA_OID_NIL;
	case ORA_flt: return isnan(*(const float *) v);
	case ORA_dbl: return isnan(*(const double *) v);
	}
	return false;
}

/* three-way compare with nil smallest (ATOMcmp semantics) */
static int
cmp_val(int t, const void *a, const void *b)
{
#define CMP3(T) do { T x = *(const T *) a, y = *(const T *) b; return (x > y) - (x < y); } while (0)
	switch (t) {
	case ORA_bte: case ORA_bit: CMP3(int8_t);
	case ORA_sht: CMP3(int16_t);
	case ORA_int: case ORA_date: CMP3(int32_t);
	case ORA_lng: CMP3(int64_t);
	case ORA_hge: CMP3(ora_hge);
	case ORA_oid: CMP3(int64_t);   /* oid compares as its storage type lng */
	case ORA_flt: {
		float x = *(const float *) a, y = *(const float *) b;
		if (isnan(x)) return isnan(y) ? 0 : -1;
		if (isnan(y)) return 1;
		return (x > y) - (x < y);
	}
	case ORA_dbl: {
		double x = *(const double *) a, y = *(const double *) b;
		if (isnan(x)) return isnan(y) ? 0 : -1;
		if (isnan(y)) return 1;
		return (x > y) - (x < y);
	}
	}
	return 0;
#undef CMP3
}

static const void *
nilptr(int t)
{
	static const int8_t bn = ORA_bte_nil;
	static const int16_t sn = ORA_sht_nil;
	static const int32_t in = ORA_int_nil;
	static const int64_t ln = ORA_lng_nil;
	static const ora_oid on = ORA_OID_NIL;
	static ora_hge hn;
	static float fn;
	static double dn;
	switch (t) {
	case ORA_bte: case ORA_bit: return &bn;
	case ORA_sht: return &sn;
	case ORA_int: case ORA_date: return &in;
	case ORA_lng: return &ln;
	case ORA_oid: return &on;
	case ORA_hge: hn = ORA_hge_nil; return &hn;
	case ORA_flt: fn = nanf(""); return &fn;
	case ORA_dbl: dn = nan(""); return &dn;
	}
	return NULL;
}

/* ---------------------------------------------------------------------- */
/* BATselect (gdk/gdk_select.c:1342-2084)
 *
 * The reference chooses between hash, binary search on sorted input,
 * order index and scan; all return the same sorted oid list, so the
 * restatement always evaluates the normalised scan predicate
 * (scanfunc, gdk_select.c:300-446) over the candidates.  (The hash path's
 * anti-equi select drops nils even under nil_matches, gdk_select.c:2046-2058;
 * it is only taken for BATs with an existing hash or after >1000 selects on
 * a transient BAT, which this restatement does not model.) */

typedef struct {
	int mode;   /* 0 range, 1 anti, 2 equi, 3 equi-nil */
	bool nil_matches;
} selmode;

#define SCAN_IMPL(T, ISNIL, PREV, NEXT, MINV, MAXV)				\
static uint64_t								\
scan_##T(const ora_bat *b, const ora_ci *ci, T vl, T vh, bool li, bool hi, \
	 bool equi, bool anti, bool nil_matches, bool lval, bool hval,	\
	 bool lnil, ora_oid *dst)					\
{									\
	const T *src = (const T *) b->base;				\
	uint64_t cnt = 0;						\
	if (anti && li) {						\
		if (vl == MINV) {					\
			anti = false; vl = vh; li = !hi; hval = false;	\
		} else {						\
			vl = PREV(vl); li = false;			\
		}							\
	}								\
	if (anti && hi) {						\
		if (vh == MAXV) {					\
			anti = false; vh = vl; hi = !li; lval = false;	\
		} else {						\
			vh = NEXT(vh); hi = false;			\
		}							\
	}								\
	if (!anti) {							\
		if (lval) {						\
			if (!li) {					\
				if (vl == MAXV)				\
					return 0;			\
				vl = NEXT(vl); li = true;		\
			}						\
		} else {						\
			vl = MINV; li = true; lval = true;		\
		}							\
		if (hval) {						\
			if (!hi) {					\
				if (vh == MINV)				\
					return 0;			\
				vh = PREV(vh); hi = true;		\
			}						\
		} else {						\
			vh = MAXV; hi = true; hval = true;		\
		}							\
		if (vl > vh)						\
			return 0;					\
	}								\
	for (uint64_t i = 0; i < ci->n; i++) {				\
		ora_oid o = ci_get(ci, i);				\
		T v = src[o - b->hseqbase];				\
		bool ok;						\
		if (equi)						\
			ok = lnil ? ISNIL(v) : v == vl;			\
		else if (anti)						\
			ok = nil_matches ? (ISNIL(v) || v <= vl || v >= vh) \
				: (!ISNIL(v) && (v <= vl || v >= vh));	\
		else							\
			ok = v >= vl && v <= vh;			\
		if (ok)							\
			dst[cnt++] = o;					\
	}								\
	return cnt;							\
}

#define INIL8(v) ((v) == ORA_bte_nil)
#define INIL16(v) ((v) == ORA_sht_nil)
#define INIL32(v) ((v) == ORA_int_nil)
#define INIL64(v) ((v) == ORA_lng_nil)
#define INIL128(v) ((v) == ORA_hge_nil)
#define ONIL(v) ((v) == ORA_OID_NIL)
#define FNIL(v) isnan(v)
#define PREVI(x) ((x) - 1)
#define NEXTI(x) ((x) + 1)
#define PREVF(x) nextafterf((x), -3.40282346638528859812e+38F)
#define NEXTF(x) nextafterf((x), 3.40282346638528859812e+38F)
#define PREVD(x) nextafter((x), -1.7976931348623157e+308)
#define NEXTD(x) nextafter((x), 1.7976931348623157e+308)

typedef int8_t bte_t;
typedef int16_t sht_t;
typedef int32_t int_t;
typedef int64_t lng_t;
typedef ora_hge hge_t;
typedef ora_oid oid_t;
typedef float flt_t;
typedef double dbl_t;

SCAN_IMPL(bte_t, INIL8, PREVI, NEXTI, (int8_t) (INT8_MIN + 1), (int8_t) INT8_MAX)
SCAN_IMPL(sht_t, INIL16, PREVI, NEXTI, (int16_t) (INT16_MIN + 1), (int16_t) INT16_MAX)
SCAN_IMPL(int_t, INIL32, PREVI, NEXTI, INT32_MIN + 1, INT32_MAX)
SCAN_IMPL(lng_t, INIL64, PREVI, NEXTI, INT64_MIN + 1, INT64_MAX)
SCAN_IMPL(hge_t, INIL128, PREVI, NEXTI, -ORA_HGE_MAX, ORA_HGE_MAX)
SCAN_IMPL(oid_t, ONIL, PREVI, NEXTI, (ora_oid) 0, (ora_oid) INT64_MAX)
/* GDK_flt_min/GDK_dbl_min are the most negative finite values
 * (gdk/gdk_atoms.h:162-165) */
SCAN_IMPL(flt_t, FNIL, PREVF, NEXTF, -3.40282346638528859812e+38F, 3.40282346638528859812e+38F)
SCAN_IMPL(dbl_t, FNIL, PREVD, NEXTD, -1.7976931348623157e+308, 1.7976931348623157e+308)

static ora_bat *
select_nils_complement(const ora_bat *b, const ora_bat *s, const ora_ci *ci)
{
	/* "everything except nil" (gdk_select.c:1482-1509) */
	(void) s;
	ora_bat *bn = ora_new(ORA_oid, ci->n, 0);
	if (bn == NULL)
		return NULL;
	const char *src = b->base;
	uint64_t cnt = 0;
	for (uint64_t i = 0; i < ci->n; i++) {
		ora_oid o = ci_get(ci, i);
		if (b->type == ORA_void || !is_nil_val(b->type, src + (o - b->hseqbase) * b->width))
			((ora_oid *) bn->base)[cnt++] = o;
	}
	bn->count = cnt;
	return ora_virtualize(bn);
}

static int
basetype(int t)
{
	return t == ORA_date ? ORA_int : t == ORA_bit ? ORA_bte : t;
}

/* ---- str select: BATselect's generic part (gdk_select.c:1342-1520) with
 * strCmp (nil "\200" before every string, then strcmp), then
 * fullscan_any (:449-605; fullscan_str's string-elimination fast path,
 * :608-760, returns the same oids by comparing heap offsets) */
static const char ora_str_nil[2] = {'\200', 0};

static const char *
sel_str_at(const ora_bat *b, uint64_t p)
{
	const char *x = (const char *) b->base + p * b->width;
	uint64_t o;
	switch (b->width) {
	case 1: o = *(const uint8_t *) x + 8192u; break;      /* GDK_VAROFFSET */
	case 2: o = *(const uint16_t *) x + 8192u; break;
	case 4: o = *(const uint32_t *) x; break;
	default: o = *(const uint64_t *) x; break;
	}
	return b->vheap + o;
}

static bool
str_isnil(const char *a)
{
	return (unsigned char) a[0] == 0x80 && a[1] == 0;
}

static int
str_cmp(const char *a, const char *b)
{
	bool an = str_isnil(a), bn = str_isnil(b);
	if (an || bn)
		return an ? -!bn : 1;
	int c = strcmp(a, b);
	return (c > 0) - (c < 0);
}

static ora_bat *
select_str(const ora_bat *b, const ora_ci *ci, const char *tl, const char *th, bool li, bool hi, bool anti,
	   bool nil_matches)
{
	const char *nil = ora_str_nil;
	bool lnil = str_cmp(tl, nil) == 0;
	bool lval = !lnil || th == NULL;
	bool equi = th == NULL || (lval && str_cmp(tl, th) == 0);
	bool hval;
	if (lnil && nil_matches && (th == NULL || str_cmp(th, nil) == 0)) {
		equi = true;
		lval = true;
	}
	if (equi) {
		if (th == NULL)
			hi = li;
		th = tl;
		hval = true;
		if (!anti && (!li || !hi))
			return ora_dense(0, 0, 0);
	} else {
		nil_matches = false;
		hval = str_cmp(th, nil) != 0;
	}
	bool all_but_nil = false;
	if (anti) {
		if (lval != hval) {
			const char *tv = tl;
			bool ti = li;
			li = !hi;
			hi = !ti;
			tl = th;
			th = tv;
			ti = lval;
			lval = hval;
			hval = ti;
			lnil = str_cmp(tl, nil) == 0;
			anti = false;
		} else if (!lval && !hval) {
			return ora_dense(0, 0, 0);
		} else if ((equi && (lnil || !(li && hi))) || str_cmp(tl, th) > 0) {
			if (equi && !lnil && nil_matches && !(li && hi))
				return ci_slice(ci);
			all_but_nil = true;
		} else {
			equi = false;
		}
	}
	if (!all_but_nil && hval && (equi ? !li || !hi : str_cmp(tl, th) > 0))
		return ora_dense(0, 0, 0);
	ora_bat *bn = ora_new(ORA_oid, ci->n, 0);
	if (bn == NULL)
		return NULL;
	ora_oid *dst = bn->base;
	uint64_t cnt = 0;
	for (uint64_t i = 0; i < ci->n; i++) {
		const ora_oid o = ci_get(ci, i);
		const char *v = sel_str_at(b, o - b->hseqbase);
		const bool isnil = str_isnil(v);
		bool ok;
		int c;
		if (all_but_nil)
			ok = !isnil;
		else if (equi)
			ok = str_cmp(tl, v) == 0;
		else if (anti)
			ok = (nil_matches && isnil) ||
			     (!isnil && ((lval && ((c = str_cmp(tl, v)) > 0 || (!li && c == 0))) ||
					 (hval && ((c = str_cmp(th, v)) < 0 || (!hi && c == 0)))));
		else
			ok = !isnil && (!lval || (c = str_cmp(tl, v)) < 0 || (li && c == 0)) &&
			     (!hval || (c = str_cmp(th, v)) > 0 || (hi && c == 0));
		if (ok)
			dst[cnt++] = o;
	}
	bn->count = cnt;
	return ora_virtualize(bn);
}

ora_bat *
ora_select(const ora_bat *b, const ora_bat *s, const void *tl, const void *th,
	   bool li, bool hi, bool anti, bool nil_matches)
{
	ora_ci ci;
	if (tl == NULL) {
		ora_seterr("tl value required");
		return NULL;
	}
	if (s && s->type == ORA_oid && !s->sorted) {
		ora_seterr("invalid argument: s must be sorted.\n");
		return NULL;
	}
	if (ora_ci_init(&ci, b, s) < 0)
		return NULL;
	if (ci.n == 0)
		return ora_dense(0, 0, 0);
	if (b->type == ORA_str)
		return select_str(b, &ci, tl, th, li, hi, anti, nil_matches);

	int t = basetype(b->type);
	if (b->type == ORA_void) {
		/* dense oid column: materialise logically as oid values */
		t = ORA_oid;
	}
	const void *nil = nilptr(t);
	bool lnil = nil && cmp_val(t, tl, nil) == 0;
	bool lval = !lnil || th == NULL;
	bool equi = th == NULL || (lval && cmp_val(t, tl, th) == 0);
	bool hval;
	if (lnil && nil_matches && (th == NULL || cmp_val(t, th, nil) == 0)) {
		equi = true;
		lval = true;
	}
	bool antiequi = false;
	(void) antiequi;
	if (equi) {
		if (th == NULL)
			hi = li;
		th = tl;
		hval = true;
		if (!anti && (!li || !hi))
			return ora_dense(0, 0, 0);       /* empty interval */
	} else {
		nil_matches = false;
		hval = cmp_val(t, th, nil) != 0;
	}
	if (anti) {
		if (lval != hval) {
			const void *tv;
			bool ti = li;
			li = !hi;
			hi = !ti;
			tv = tl;
			tl = th;
			th = tv;
			ti = lval;
			lval = hval;
			hval = ti;
			lnil = cmp_val(t, tl, nil) == 0;
			anti = false;
		} else if (!lval && !hval) {
			return ora_dense(0, 0, 0);       /* anti nil-nil range */
		} else if ((equi && (lnil || !(li && hi))) || cmp_val(t, tl, th) > 0) {
			if (equi && !lnil && nil_matches && !(li && hi))
				return ci_slice(&ci);
			return select_nils_complement(b, s, &ci);
		} else {
			antiequi = equi;
			equi = false;
		}
	}
	if (hval && (equi ? !li || !hi : cmp_val(t, tl, th) > 0))
		return ora_dense(0, 0, 0);               /* empty range */

	ora_bat *bn = ora_new(ORA_oid, ci.n, 0);
	if (bn == NULL)
		return NULL;
	uint64_t cnt = 0;
	ora_oid *dst = bn->base;
	if (b->type == ORA_void) {
		/* positional select on a dense column: values are oids */
		ora_bat tmp = *b;
		ora_oid *vals = malloc(b->count * sizeof(ora_oid) + 8);
		for (uint64_t i = 0; i < b->count; i++)
			vals[i] = b->tseqbase + i;
		tmp.base = vals;
		cnt = scan_oid_t(&tmp, &ci, *(const ora_oid *) tl, *(const ora_oid *) th,
				 li, hi, equi, anti, nil_matches, lval, hval, lnil, dst);
		free(vals);
	} else {
		switch (t) {
#define CASE(TT, T) case TT: cnt = scan_##T(b, &ci, *(const T *) tl, *(const T *) th, li, hi, equi, anti, nil_matches, lval, hval, lnil, dst); break
		CASE(ORA_bte, bte_t);
		CASE(ORA_sht, sht_t);
		CASE(ORA_int, int_t);
		CASE(ORA_lng, lng_t);
		CASE(ORA_hge, hge_t);
		CASE(ORA_oid, oid_t);
		CASE(ORA_flt, flt_t);
		CASE(ORA_dbl, dbl_t);
#undef CASE
		default:
			ora_free(bn);
			ora_seterr("select: unsupported type %d", b->type);
			return NULL;
		}
	}
	bn->count = cnt;
	return ora_virtualize(bn);
}

/* BATthetaselect (gdk/gdk_select.c:2103-2154) */
ora_bat *
ora_thetaselect(const ora_bat *b, const ora_bat *s, const void *val, const char *op)
{
	int t = b->type == ORA_void ? ORA_oid : basetype(b->type);
	const void *nil = b->type == ORA_str ? (const void *) ora_str_nil : nilptr(t);
	if (val == NULL || op == NULL) {
		ora_seterr("thetaselect: NULL argument");
		return NULL;
	}
	if (strcmp(op, "eq") == 0)
		return ora_select(b, s, val, NULL, true, true, false, true);
	if (strcmp(op, "ne") == 0)
		return ora_select(b, s, val, NULL, true, true, true, true);
	if (b->type == ORA_str ? str_isnil(val) : cmp_val(t, val, nil) == 0)
		return ora_dense(0, 0, 0);
	if (op[0] == '=' && ((op[1] == '=' && op[2] == 0) || op[1] == 0))
		return ora_select(b, s, val, NULL, true, true, false, false);
	if (op[0] == '!' && op[1] == '=' && op[2] == 0)
		return ora_select(b, s, val, NULL, true, true, true, false);
	if (op[0] == '<') {
		if (op[1] == 0)
			return ora_select(b, s, nil, val, false, false, false, false);
		if (op[1] == '=' && op[2] == 0)
			return ora_select(b, s, nil, val, false, true, false, false);
		if (op[1] == '>' && op[2] == 0)
			return ora_select(b, s, val, NULL, true, true, true, false);
	}
	if (op[0] == '>') {
		if (op[1] == 0)
			return ora_select(b, s, val, nil, false, false, false, false);
		if (op[1] == '=' && op[2] == 0)
			return ora_select(b, s, val, nil, true, false, false, false);
	}
	ora_seterr("unknown operator.\n");
	return NULL;
}

/* ---------------------------------------------------------------------- */
/* BATproject (gdk/gdk_project.c:590-857): out[i] = r[l[i] - r.hseqbase];
 * a nil oid in l yields nil; out-of-range oids are an error. */
/* BATunmask of a msk BAT (gdk_cand.c:1464, its positive-list branch
 * :1549-1599): hseqbase + i for every set bit i < count, virtualised */
ora_bat *
ora_unmask(const ora_bat *b)
{
	if (b->type != ORA_msk) {
		ora_seterr("BATunmask: not a msk BAT");
		return NULL;
	}
	const uint32_t *w = b->base;
	uint64_t k = 0;
	for (uint64_t i = 0; i < b->count; i++)
		k += (w[i >> 5] >> (i & 31)) & 1;
	ora_bat *bn = ora_new(ORA_oid, k, b->hseqbase);
	if (bn == NULL)
		return NULL;
	ora_oid *o = bn->base;
	k = 0;
	for (uint64_t i = 0; i < b->count; i++)
		if ((w[i >> 5] >> (i & 31)) & 1)
			o[k++] = b->hseqbase + i;
	bn->count = k;
	bn->sorted = bn->key = bn->nonil = 1;
	bn->revsorted = k <= 1;
	return ora_virtualize(bn);
}

/* BATmaskedcands (gdk_cand.c:1366-1460) as the oid list it stands for: the
 * mask words of [hseq, hseq + nr) from masked's bits (or their complement),
 * rows past masked's end selected -- returned unmasked (materialised) */
ora_bat *
ora_maskedcands(ora_oid hseq, uint64_t nr, const ora_bat *masked, bool selected)
{
	if (masked->type != ORA_msk) {
		ora_seterr("BATmaskedcands: not a msk BAT");
		return NULL;
	}
	const uint32_t *w = masked->base;
	ora_bat *bn = ora_new(ORA_oid, nr, hseq);
	if (bn == NULL)
		return NULL;
	ora_oid *o = bn->base;
	uint64_t k = 0;
	if (masked->count > 0)
		for (uint64_t i = 0; i < nr; i++) {
			bool bit = i < masked->count ? (((w[i >> 5] >> (i & 31)) & 1) != 0) == selected : true;
			if (bit)
				o[k++] = hseq + i;
		}
	bn->count = k;
	bn->sorted = bn->key = bn->nonil = 1;
	bn->revsorted = k <= 1;
	return ora_virtualize(bn);
}

/* ---------------------------------------------------------------------- */
/* candidate-list algebra (gdk/gdk_cand.c:46-355, :1296-1363).  A list's
 * candidates are its own values (canditer_init(&ci, NULL, b)): a void BAT
 * the range [tseqbase, tseqbase + count), an oid BAT its sorted values. */

static void
cand_list(const ora_bat *b, ora_ci *ci)
{
	ci->dense = b->type == ORA_void;
	ci->seq = b->tseqbase;
	ci->oids = b->type == ORA_void ? NULL : (const ora_oid *) b->base;
	ci->n = b->count;
}

/* a new oid list from `o` with `n` values: properties as the reference
 * sets them, then virtualize (gdk_select.c:31) */
static ora_bat *
cand_result(ora_oid *o, uint64_t n)
{
	ora_bat *bn = ora_new(ORA_oid, n, 0);
	if (bn == NULL)
		return NULL;
	if (n)
		memcpy(bn->base, o, n * sizeof(ora_oid));
	bn->count = n;
	bn->sorted = bn->key = bn->nonil = 1;
	bn->revsorted = n <= 1;
	bn->nil = 0;
	return ora_virtualize(bn);
}

/* BATmergecand (gdk_cand.c:46-166): the two-pointer merge of :131-153;
 * the reference's dense shortcuts (:66-95) give the same sequence */
ora_bat *
ora_mergecand(const ora_bat *a, const ora_bat *b)
{
	ora_ci ca, cb;
	cand_list(a, &ca);
	cand_list(b, &cb);
	ora_oid *o = malloc((ca.n + cb.n + 1) * sizeof(ora_oid));
	if (o == NULL) {
		ora_seterr("malloc");
		return NULL;
	}
	uint64_t i = 0, j = 0, k = 0;
	while (i < ca.n && j < cb.n) {
		const ora_oid x = ci_get(&ca, i), y = ci_get(&cb, j);
		if (x < y) {
			o[k++] = x;
			i++;
		} else if (y < x) {
			o[k++] = y;
			j++;
		} else {
			o[k++] = x;
			i++;
			j++;
		}
	}
	while (i < ca.n)
		o[k++] = ci_get(&ca, i++);
	while (j < cb.n)
		o[k++] = ci_get(&cb, j++);
	ora_bat *bn = cand_result(o, k);
	free(o);
	return bn;
}

/* BATintersectcand (gdk_cand.c:184-252), the loop of :228-240 */
ora_bat *
ora_intersectcand(const ora_bat *a, const ora_bat *b)
{
	ora_ci ca, cb;
	cand_list(a, &ca);
	cand_list(b, &cb);
	ora_oid *o = malloc(((ca.n < cb.n ? ca.n : cb.n) + 1) * sizeof(ora_oid));
	if (o == NULL) {
		ora_seterr("malloc");
		return NULL;
	}
	uint64_t i = 0, j = 0, k = 0;
	while (i < ca.n && j < cb.n) {
		const ora_oid x = ci_get(&ca, i), y = ci_get(&cb, j);
		if (x < y)
			i++;
		else if (y < x)
			j++;
		else {
			o[k++] = x;
			i++;
			j++;
		}
	}
	ora_bat *bn = cand_result(o, k);
	free(o);
	return bn;
}

/* BATdiffcand (gdk_cand.c:259-355), the loop of :331-339 */
ora_bat *
ora_diffcand(const ora_bat *a, const ora_bat *b)
{
	ora_ci ca, cb;
	cand_list(a, &ca);
	cand_list(b, &cb);
	ora_oid *o = malloc((ca.n + 1) * sizeof(ora_oid));
	if (o == NULL) {
		ora_seterr("malloc");
		return NULL;
	}
	uint64_t j = 0, k = 0;
	for (uint64_t i = 0; i < ca.n; i++) {
		const ora_oid x = ci_get(&ca, i);
		while (j < cb.n && ci_get(&cb, j) < x)
			j++;
		if (j == cb.n || x < ci_get(&cb, j))
			o[k++] = x;
	}
	ora_bat *bn = cand_result(o, k);
	free(o);
	return bn;
}

/* BATnegcands (gdk_cand.c:1296-1363): [tseq, tseq + nr) minus the
 * deletions odels[lo, hi) that fall inside it (SORTfndfirst bounds); the
 * reference keeps them as a cand_except vheap -- returned here as the oid
 * list that stands for */
ora_bat *
ora_negcands(ora_oid tseq, uint64_t nr, const ora_bat *odels)
{
	ora_ci cd;
	cand_list(odels, &cd);
	uint64_t lo = 0, hi;
	while (lo < cd.n && ci_get(&cd, lo) < tseq)
		lo++;
	hi = lo;
	while (hi < cd.n && ci_get(&cd, hi) < tseq + nr)
		hi++;
	if (lo == hi || cd.n == 0)
		return ora_dense(0, tseq, nr);
	if (hi - lo == nr)
		return ora_dense(0, tseq, 0);
	ora_oid *o = malloc((nr + 1) * sizeof(ora_oid));
	if (o == NULL) {
		ora_seterr("malloc");
		return NULL;
	}
	uint64_t k = 0, d = lo;
	for (ora_oid x = tseq; x < tseq + nr; x++) {
		if (d < hi && ci_get(&cd, d) == x) {
			d++;
			continue;
		}
		o[k++] = x;
	}
	ora_bat *bn = cand_result(o, k);
	free(o);
	return bn;
}

ora_bat *
ora_project(const ora_bat *l, const ora_bat *r)
{
	if (l->type == ORA_msk) {
		/* gdk_project.c:652-660 */
		ora_bat *m = ora_unmask(l);
		if (m == NULL)
			return NULL;
		ora_bat *bn = ora_project(m, r);
		ora_free(m);
		return bn;
	}
	ora_ci ci;
	if (ora_ci_init(&ci, NULL, l) < 0)
		return NULL;
	int t = r->type;
	uint64_t n = l->count;
	ora_oid rlo = r->hseqbase, rhi = r->hseqbase + r->count;
	if (l->type == ORA_void && n > 0) {
		if (l->tseqbase < rlo || l->tseqbase + n > rhi) {
			ora_seterr("does not match always\n");
			return NULL;
		}
	}
	int ot = t == ORA_void ? ORA_oid : t;
	ora_bat *bn = ora_new(ot, n, l->hseqbase);
	if (bn == NULL)
		return NULL;
	bn->width = r->type == ORA_void ? 8 : r->width;
	if (r->type == ORA_str) {
		free(bn->base);
		bn->base = malloc(n * r->width + 16);
		bn->vheap = malloc(r->vheapsize);
		memcpy(bn->vheap, r->vheap, r->vheapsize);
		bn->vheapsize = r->vheapsize;
	}
	const ora_oid *lo = l->type == ORA_oid ? l->base : NULL;
	bool hasnil = false;
	for (uint64_t i = 0; i < n; i++) {
		ora_oid o = lo ? lo[i] : l->tseqbase + i;
		char *d = (char *) bn->base + i * bn->width;
		if (o == ORA_OID_NIL) {
			if (ot == ORA_str) {
				ora_seterr("project: nil oid on str unsupported");
				ora_free(bn);
				return NULL;
			}
			memcpy(d, nilptr(basetype(ot)), bn->width);
			hasnil = true;
			continue;
		}
		if (o < rlo || o >= rhi) {
			ora_seterr("does not match always\n");
			ora_free(bn);
			return NULL;
		}
		if (r->type == ORA_void) {
			ora_oid v = r->tseqbase == ORA_OID_NIL ? ORA_OID_NIL : r->tseqbase + (o - rlo);
			memcpy(d, &v, 8);
		} else {
			memcpy(d, (const char *) r->base + (o - rlo) * r->width, bn->width);
		}
	}
	bn->nil = hasnil;
	bn->nonil = l->nonil && r->nonil && !hasnil;
	bn->sorted = n <= 1 || (l->sorted && r->sorted) || (l->revsorted && r->revsorted) || r->count <= 1;
	bn->revsorted = n <= 1 || (l->sorted && r->revsorted) || (l->revsorted && r->sorted) || r->count <= 1;
	bn->key = n <= 1 || (l->key && r->key);
	return bn;
}

/* ---------------------------------------------------------------------- */
/* BATcalc{add,sub,mul}[cst] for integer types (gdk/gdk_calc_addsub.c,
 * gdk/gdk_calc_mul.c): nil in either operand gives nil; the result is
 * computed in the result type tp; overflow (result outside
 * [-max, max] of tp, i.e. also hitting the nil value) is the error
 * "22003!overflow in calculation <a><op><b>." (ON_OVERFLOW,
 * gdk/gdk_calc_private.h).  Results are positional over the candidates
 * (hseqbase = first candidate's hseq). */

static bool
get_hge(int t, const void *p, ora_hge *v)
{
	switch (t) {
	case ORA_bte: *v = *(const int8_t *) p; return *v == ORA_bte_nil;
	case ORA_sht: *v = *(const int16_t *) p; return *v == ORA_sht_nil;
	case ORA_int: case ORA_date: *v = *(const int32_t *) p; return *v == ORA_int_nil;
	case ORA_lng: *v = *(const int64_t *) p; return *v == ORA_lng_nil;
	case ORA_hge: *v = *(const ora_hge *) p; return *v == ORA_hge_nil;
	}
	*v = 0;
	return false;
}

static ora_hge
type_max(int tp)
{
	switch (tp) {
	case ORA_bte: return INT8_MAX;
	case ORA_sht: return INT16_MAX;
	case ORA_int: return INT32_MAX;
	case ORA_lng: return INT64_MAX;
	case ORA_hge: return ORA_HGE_MAX;
	}
	return 0;
}

static void
put_hge(int tp, void *p, ora_hge v)
{
	switch (tp) {
	case ORA_bte: *(int8_t *) p = (int8_t) v; break;
	case ORA_sht: *(int16_t *) p = (int16_t) v; break;
	case ORA_int: *(int32_t *) p = (int32_t) v; break;
	case ORA_lng: *(int64_t *) p = (int64_t) v; break;
	case ORA_hge: *(ora_hge *) p = v; break;
	}
}

static void
fmt_val(char *buf, size_t sz, int t, ora_hge v)
{
	switch (basetype(t)) {
	case ORA_bte: case ORA_sht: case ORA_int: snprintf(buf, sz, "%d", (int) v); break;
	case ORA_lng: snprintf(buf, sz, "%lld", (long long) v); break;
	default: snprintf(buf, sz, "%.40Lg (approx. value)", (long double) v); break;
	}
}

ora_bat *
ora_calc(char op, const ora_bat *b1, const void *c1, int t1,
	 const ora_bat *b2, const void *c2, int t2,
	 const ora_bat *s, int tp)
{
	ora_ci ci1, ci2;
	const ora_bat *bb = b1 ? b1 : b2;
	if (bb == NULL) {
		ora_seterr("calc: no BAT operand");
		return NULL;
	}
	if (b1)
		t1 = basetype(b1->type);
	if (b2)
		t2 = basetype(b2->type);
	if (tp != ORA_bte && tp != ORA_sht && tp != ORA_int && tp != ORA_lng && tp != ORA_hge) {
		ora_seterr("calc: unsupported result type");
		return NULL;
	}
	if (b1 && b2) {
		/* BATcalcmuldivmod / BATcalcadd take s1,s2: here the same s */
		if (ora_ci_init(&ci1, b1, s) < 0 || ora_ci_init(&ci2, b2, s) < 0)
			return NULL;
		if (ci1.n != ci2.n) {
			ora_seterr("inputs not the same size.\n");
			return NULL;
		}
	} else {
		if (ora_ci_init(&ci1, bb, s) < 0)
			return NULL;
		ci2 = ci1;
	}
	/* COLnew(ci1.hseq, ...): s's head base, else b's */
	ora_oid hseq = s ? s->hseqbase : bb->hseqbase;
	ora_bat *bn = ora_new(tp, ci1.n, hseq);
	if (bn == NULL)
		return NULL;
	ora_hge max = type_max(tp);
	uint64_t nils = 0;
	for (uint64_t i = 0; i < ci1.n; i++) {
		ora_hge x, y, z;
		bool n1, n2;
		if (b1) {
			ora_oid o = ci_get(&ci1, i) - b1->hseqbase;
			n1 = get_hge(t1, (const char *) b1->base + o * b1->width, &x);
		} else {
			n1 = get_hge(t1, c1, &x);
		}
		if (b2) {
			ora_oid o = ci_get(&ci2, i) - b2->hseqbase;
			n2 = get_hge(t2, (const char *) b2->base + o * b2->width, &y);
		} else {
			n2 = get_hge(t2, c2, &y);
		}
		char *d = (char *) bn->base + i * bn->width;
		if (n1 || n2) {
			memcpy(d, nilptr(tp), bn->width);
			nils++;
			continue;
		}
		bool ovf;
		switch (op) {
		case '+': ovf = __builtin_add_overflow(x, y, &z); break;
		case '-': ovf = __builtin_sub_overflow(x, y, &z); break;
		case '*': ovf = __builtin_mul_overflow(x, y, &z); break;
		default:
			ora_seterr("calc: bad op");
			ora_free(bn);
			return NULL;
		}
		if (ovf || z < -max || z > max) {
			/* ON_OVERFLOW (gdk_calc_private.h:346-352): the operand
			 * values, FMT per type (FMThge "%.40Lg (approx. value)") */
			char a[64], c[64];
			fmt_val(a, sizeof(a), t1, x);
			fmt_val(c, sizeof(c), t2, y);
			ora_seterr("22003!overflow in calculation %s%c%s.\n", a, op, c);
			ora_free(bn);
			return NULL;
		}
		put_hge(tp, d, z);
	}
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	/* result order (gdk_calc_addsub.c:1528-1531, 1590-1593, 1649-1652,
	 * 3208-3209, 3262-3265, 3318-3321; gdk_calc_mul.c:2068-2069,
	 * 2133-2138, 2194-2199): a constant operand keeps the BAT's order (a
	 * negative multiplier or cst - b reverses it), two sorted BATs add to a
	 * sorted result, anything else is unordered; only without nils */
	bool srt = false, rev = false;
	if (nils == 0) {
		if (b1 && b2) {
			if (op == '+') {
				srt = b1->sorted && b2->sorted;
				rev = b1->revsorted && b2->revsorted;
			}
		} else {
			const ora_bat *b = b1 ? b1 : b2;
			int sign = 1;
			if (op == '*') {
				ora_hge c;
				get_hge(b1 ? t2 : t1, b1 ? c2 : c1, &c);
				sign = c > 0 ? 1 : c < 0 ? -1 : 0;
			} else if (op == '-' && !b1) {
				sign = -1;
			}
			srt = (sign >= 0 && b->sorted) || (sign <= 0 && b->revsorted);
			rev = (sign >= 0 && b->revsorted) || (sign <= 0 && b->sorted);
		}
	}
	bn->sorted = srt || ci1.n <= 1 || nils == ci1.n;
	bn->revsorted = rev || ci1.n <= 1 || nils == ci1.n;
	bn->key = ci1.n <= 1;
	return bn;
}

/* ---------------------------------------------------------------------- */
/* BATsum (gdk/gdk_aggr.c:1018 -> dosum :708, AGGR_SUM :429-705):
 * integer sum into tp with overflow -> "22003!overflow in sum aggregate.";
 * nils are skipped when skip_nils, else make the result nil; an empty input
 * gives nil when nil_if_empty, else 0. */

/* dofsum, gdk/gdk_aggr.c:183-427, one group: Shewchuk / msum partials with
 * the reference's handling of intermediate overflow (twopow, infs) and its
 * final correction step.  INFINITES_ALLOWED is not defined in the reference
 * build, so infs counts overflows.  Returns -1 with the overflow message. */
static void
ora_twosum(volatile double *hi, volatile double *lo, double x, double y)
{
	volatile double yr;
	*hi = x + y;
	yr = *hi - x;
	*lo = y - yr;
}

static bool
ora_samesign(double x, double y)
{
	return (x >= 0) == (y >= 0);
}

/* one group's values in input order (NaN = nil) */
int ora_fsum_array(double *out, bool *isnil, const double *vals, uint64_t nv, bool skip_nils, bool nil_if_empty);
int
ora_fsum_array(double *out, bool *isnil, const double *vals, uint64_t nv, bool skip_nils, bool nil_if_empty)
{
	int npartials = 0, maxpartials = 2, infs = 0;
	bool valseen = false;
	double *partials = malloc(maxpartials * sizeof(double));
	double x, y;
	volatile double lo, hi;
	const double twopow = pow(2.0, 1023.0);
	*isnil = false;
	for (uint64_t k = 0; k < nv; k++) {
		x = vals[k];
		if (isnan(x)) {
			if (!skip_nils) {
				*isnil = true;
				free(partials);
				return 0;
			}
			continue;
		}
		valseen = true;
		int i = 0;
		for (int pi = 0; pi < npartials; pi++) {
			y = partials[pi];
			if (fabs(x) < fabs(y)) { double t = x; x = y; y = t; }
			ora_twosum(&hi, &lo, x, y);
			if (isinf(hi)) {
				int sign = hi > 0 ? 1 : -1;
				hi = x - twopow * sign;
				x = hi - twopow * sign;
				infs += sign;
				if (fabs(x) < fabs(y)) { double t = x; x = y; y = t; }
				ora_twosum(&hi, &lo, x, y);
			}
			if (lo != 0)
				partials[i++] = lo;
			x = hi;
		}
		if (x != 0) {
			if (i == maxpartials) {
				maxpartials *= 2;
				partials = realloc(partials, maxpartials * sizeof(double));
			}
			partials[i++] = x;
		}
		npartials = i;
	}
	if (!valseen) {
		*isnil = nil_if_empty;
		*out = 0;
		free(partials);
		return 0;
	}
	if ((infs == 1 || infs == -1) && npartials > 0 && !ora_samesign(infs, partials[npartials - 1])) {
		ora_twosum(&hi, &lo, infs * twopow, partials[npartials - 1] / 2);
		if (isinf(2 * hi)) {
			y = 2 * lo;
			x = hi + y;
			x -= hi;
			if (x == y && npartials > 1 && ora_samesign(lo, partials[npartials - 2])) {
				*out = 2 * (hi + y);
				free(partials);
				return 0;
			}
		} else {
			if (lo) {
				if (npartials == maxpartials)
					partials = realloc(partials, ++maxpartials * sizeof(double));
				partials[npartials - 1] = 2 * lo;
				partials[npartials++] = 2 * hi;
			} else {
				partials[npartials - 1] = 2 * hi;
			}
			infs = 0;
		}
	}
	if (infs != 0) {
		free(partials);
		ora_seterr("22003!overflow in sum aggregate.\n");
		return -1;
	}
	if (npartials == 0) {
		*out = 0;
		free(partials);
		return 0;
	}
	hi = partials[--npartials];
	while (npartials > 0) {
		ora_twosum(&hi, &lo, hi, partials[--npartials]);
		if (lo) {
			partials[npartials++] = lo;
			break;
		}
	}
	if (npartials >= 2 && ora_samesign(partials[npartials - 1], partials[npartials - 2]) &&
	    hi + 2 * partials[npartials - 1] - hi == 2 * partials[npartials - 1]) {
		hi += 2 * partials[npartials - 1];
		partials[npartials - 1] = -partials[npartials - 1];
	}
	free(partials);
	*out = hi;
	return 0;
}

static int
ora_fsum(double *out, bool *isnil, const ora_bat *b, const ora_ci *ci, bool skip_nils, bool nil_if_empty)
{
	double *vals = malloc((ci->n + 1) * sizeof(double));
	for (uint64_t k = 0; k < ci->n; k++) {
		uint64_t p = ci_get(ci, k) - b->hseqbase;
		vals[k] = b->type == ORA_flt ? (double) ((const float *) b->base)[p] : ((const double *) b->base)[p];
	}
	int rc = ora_fsum_array(out, isnil, vals, ci->n, skip_nils, nil_if_empty);
	free(vals);
	return rc;
}

int
ora_sum(void *res, int tp, const ora_bat *b, const ora_bat *s,
	bool skip_nils, bool nil_if_empty)
{
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return -1;
	int t = basetype(b->type);
	if (t == ORA_flt || t == ORA_dbl) {
		double d;
		bool isnil;
		if (ora_fsum(&d, &isnil, b, &ci, skip_nils, nil_if_empty) < 0)
			return -1;
		if (tp == ORA_dbl) {
			*(double *) res = isnil ? nan("") : d;
			return 0;
		}
		float f = (float) d;
		if (!isnil && (isinf(f) || isnan(f))) {
			ora_seterr("22003!overflow in sum aggregate.\n");
			return -1;
		}
		*(float *) res = isnil ? nanf("") : f;
		return 0;
	}
	if (tp == ORA_dbl) {
		/* integers into dbl (gdk_aggr.c:1112-1156): the exact average
		 * (BATcalcavg, sum in hge :2905-2960) times the count; any nil
		 * without skip_nils gives nil; no values gives nil or 0 */
		ora_hge acc = 0;
		uint64_t cnt = 0;
		for (uint64_t i = 0; i < ci.n; i++) {
			ora_hge v;
			if (get_hge(t, (const char *) b->base + (ci_get(&ci, i) - b->hseqbase) * b->width, &v))
				continue;
			acc += v;
			cnt++;
		}
		double avg = cnt ? (double) acc / (double) cnt : 0;
		bool isnil = (cnt == 0 && nil_if_empty) || (cnt < ci.n && !skip_nils);
		*(double *) res = isnil ? nan("") : avg * (double) cnt;
		return 0;
	}
	if (tp != ORA_lng && tp != ORA_hge && tp != ORA_int) {
		ora_seterr("sum: unsupported result type");
		return -1;
	}
	ora_hge max = type_max(tp), acc = 0;
	bool seen = false;
	for (uint64_t i = 0; i < ci.n; i++) {
		ora_hge v;
		if (get_hge(t, (const char *) b->base + (ci_get(&ci, i) - b->hseqbase) * b->width, &v)) {
			if (!skip_nils) {
				memcpy(res, nilptr(tp), ora_width(tp));
				return 0;
			}
			continue;
		}
		ora_hge z;
		if (__builtin_add_overflow(acc, v, &z) || z < -max || z > max) {
			ora_seterr("22003!overflow in sum aggregate.");
			return -1;
		}
		acc = z;
		seen = true;
	}
	if (!seen && nil_if_empty)
		memcpy(res, nilptr(tp), ora_width(tp));
	else
		put_hge(tp, res, acc);
	return 0;
}
