/*
 * gdk_oracle_join.c -- CPU restatement of GDK's BATjoin, including its
 * algorithm choice, result order and result properties.  TEST
 * INFRASTRUCTURE ONLY (see gdk_oracle.h).
 *
 * BATjoin (gdk/gdk_join.c:4451-4623) picks one of five algorithms and the
 * choice decides the ORDER of the (r1, r2) pairs:
 *   selectjoin     one side is a single value (gdk_join.c:363-563):
 *                  per driving candidate in order, the other side's matches
 *                  ascending (a point BATselect);
 *   mergejoin_void the other side is dense (gdk_join.c:571-1020): a range
 *                  BATselect on the driving side, matches computed;
 *   mergejoin      both sides sorted, or one sorted and binary search is
 *                  cheaper than a hash (gdk_join.c:1023-1335, 1941-2780): per
 *                  driving candidate in order, matches ascending;
 *   hashjoin       otherwise (gdk_join.c:2900-3335): per driving candidate in
 *                  order, matches in DESCENDING position (the hash chains are
 *                  built by prepending, gdk/gdk_hash.c:658-704);
 * and "swapped" variants drive from the right side (r2 then ascends).  The
 * hash side is chosen by joincost (gdk_join.c:3586-3689) from the unique
 * value estimates of guess_uniques (:3519-3576).
 *
 * The estimate samples 1000 rows with BATsample (gdk/gdk_sample.c:199),
 * which is seeded from the clock; a BAT of <= 1000 rows is sampled whole, so
 * the estimate -- and the algorithm choice -- is deterministic there.  For
 * larger BATs this restatement (and the device) samples the rows at
 * floor(i * n / 1000), i < 1000: the only place where the choice can differ
 * from a given reference run, and only when the two costs are close.
 * No BAT carries a prebuilt hash here (joincost's rhash / phash are false)
 * and every BAT is transient (the hash-build cost is counted).
 *
 * BATordered / BATordered_rev (gdk/gdk_batop.c:2002-2262) are evaluated
 * lazily in the reference's order and cache what they find in the input
 * descriptors (tsorted, trevsorted, tkey), as the reference does: the cached
 * flags feed later decisions and result properties.
 */
#include "gdk_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

void ora_seterr(const char *fmt, ...);
ora_bat *ora_dense(ora_oid hseq, ora_oid tseq, uint64_t cnt);

typedef struct {
	bool dense;
	ora_oid seq;
	const ora_oid *oids;
	uint64_t n;
} ora_ci;
int ora_ci_init(ora_ci *ci, const ora_bat *b, const ora_bat *s);

static inline ora_oid
ci_get(const ora_ci *ci, uint64_t i)
{
	return ci->dense ? ci->seq + i : ci->oids[i];
}

/* ---- values ---------------------------------------------------------- */

/* value of position p sign-extended to 64 bits: every join type compares
 * as a signed integer with its nil (the type minimum) smallest; oid
 * compares like lng (its storage type, gdk/gdk_atoms.c:1720-1737) */
/* a flt / dbl value as an int64 that compares as dbl_cmp does (nil = NaN
 * below everything, -0.0 == +0.0): the bits of a non-negative double as
 * they are, a negative one's low 63 bits flipped (a flt widens exactly to
 * dbl); equal images <=> equal values, so the hash path's buckets
 * (dblHash hashes -0.0 as 0, gdk_atoms.c:138-145) agree too */
static int64_t
fimage(double x)
{
	if (isnan(x))
		return INT64_MIN;
	if (x == 0)
		return 0;
	int64_t s;
	memcpy(&s, &x, 8);
	return s < 0 ? s ^ INT64_MAX : s;
}

static int64_t
jv(const ora_bat *b, uint64_t p)
{
	switch (b->type) {
	case ORA_flt: return fimage(((const float *) b->base)[p]);
	case ORA_dbl: return fimage(((const double *) b->base)[p]);
	case ORA_void:
		return b->tseqbase == ORA_OID_NIL ? INT64_MIN : (int64_t) (b->tseqbase + p);
	case ORA_bte: case ORA_bit: return ((const int8_t *) b->base)[p];
	case ORA_sht: return ((const int16_t *) b->base)[p];
	case ORA_int: case ORA_date: return ((const int32_t *) b->base)[p];
	default: return ((const int64_t *) b->base)[p];
	}
}

static int64_t
jnilv(int type)
{
	switch (type) {
	case ORA_bte: case ORA_bit: return INT8_MIN;
	case ORA_sht: return INT16_MIN;
	case ORA_int: case ORA_date: return INT32_MIN;
	default: return INT64_MIN;
	}
}

static bool
join_type_ok(int t)
{
	switch (t) {
	case ORA_void: case ORA_bte: case ORA_sht: case ORA_int: case ORA_date:
	case ORA_lng: case ORA_oid: case ORA_daytime: case ORA_timestamp:
	case ORA_flt: case ORA_dbl:
		return true;
	}
	return false;
}

/* ATOMtype: void joins as oid */
static int
atomtype(int t)
{
	return t == ORA_void ? ORA_oid : t;
}

/* BATtdense (gdk/gdk.h): a void or oid BAT with a tseqbase */
static bool
tdense(const ora_bat *b)
{
	return (b->type == ORA_void || b->type == ORA_oid) && b->tseqbase != ORA_OID_NIL;
}

/* ---- BATordered / BATordered_rev (gdk/gdk_batop.c:2002-2262) ------------- */

static bool
ordered(ora_bat *b)
{
	if (b->type == ORA_void || b->sorted || b->count == 0)
		return true;
	bool asc = false, eq = false;
	for (uint64_t p = 1; p < b->count; p++) {
		int64_t x = jv(b, p - 1), y = jv(b, p);
		if (x > y)
			return false;
		if (x < y)
			asc = true;
		else
			eq = true;
	}
	b->sorted = 1;
	if (!asc)
		b->revsorted = 1;
	if (!eq)
		b->key = 1;
	return true;
}

static bool
ordered_rev(ora_bat *b)
{
	if (b->count <= 1 || b->revsorted)
		return true;
	if (b->type == ORA_void)
		return b->tseqbase == ORA_OID_NIL;
	if (tdense(b))
		return false;
	for (uint64_t p = 1; p < b->count; p++)
		if (jv(b, p - 1) < jv(b, p))
			return false;
	b->revsorted = 1;
	return true;
}

/* ---- result builders --------------------------------------------------- */

typedef struct {
	ora_oid *a, *b;
	uint64_t n, cap;
} pairs;

static int
pairs_add(pairs *P, ora_oid x, ora_oid y)
{
	if (P->n == P->cap) {
		uint64_t c = P->cap ? P->cap * 2 : 1024;
		ora_oid *na = realloc(P->a, c * 8), *nb = realloc(P->b, c * 8);
		if (na)
			P->a = na;
		if (nb)
			P->b = nb;
		if (!na || !nb) {
			ora_seterr("out of memory");
			return -1;
		}
		P->cap = c;
	}
	P->a[P->n] = x;
	P->b[P->n] = y;
	P->n++;
	return 0;
}

static ora_bat *
oidbat(const ora_oid *v, uint64_t n)
{
	ora_bat *bn = ora_new(ORA_oid, n, 0);
	if (bn == NULL)
		return NULL;
	if (n)
		memcpy(bn->base, v, n * 8);
	bn->nonil = 1;
	bn->nil = 0;
	return bn;
}

/* properties of an oid column from its values */
typedef struct {
	bool asc, desc, eq, consec;   /* some adjacent pair <, >, ==; all +1 */
} adj;

static adj
adjacent(const ora_oid *v, uint64_t n)
{
	adj r = {false, false, false, true};
	for (uint64_t i = 1; i < n; i++) {
		if (v[i - 1] < v[i])
			r.asc = true;
		else if (v[i - 1] > v[i])
			r.desc = true;
		else
			r.eq = true;
		if (v[i] != v[i - 1] + 1)
			r.consec = false;
	}
	return r;
}

/* virtualize (gdk/gdk_select.c:31-89) of a sorted key oid column */
static void
virtualize(ora_bat *bn)
{
	if (bn->type != ORA_oid)
		return;
	const ora_oid *o = bn->base;
	if (bn->count <= 1 || o[bn->count - 1] - o[0] == bn->count - 1) {
		ora_oid seq = bn->count ? o[0] : 0;
		free(bn->base);
		bn->base = NULL;
		bn->type = ORA_void;
		bn->width = 0;
		bn->tseqbase = seq;
	}
}

/* BATsetcount (gdk/gdk_bat.c:2066-2082): counts <= 1 are ordered both ways */
static void
setcount_props(ora_bat *b)
{
	if (b->count <= 1)
		b->sorted = b->revsorted = 1;
}

static void
out2(ora_bat **r1p, ora_bat **r2p, ora_bat *a, ora_bat *b, bool swapped)
{
	if (swapped) {
		ora_bat *t = a;
		a = b;
		b = t;
	}
	*r1p = a;
	if (r2p)
		*r2p = b;
	else
		ora_free(b);
}

/* nomatch (gdk_join.c:301-360) without nil_on_miss: two empty dense BATs */
static int
nomatch(ora_bat **r1p, ora_bat **r2p)
{
	ora_bat *a = ora_dense(0, 0, 0), *b = ora_dense(0, 0, 0);
	if (!a || !b) {
		ora_free(a);
		ora_free(b);
		return -1;
	}
	out2(r1p, r2p, a, b, false);
	return 0;
}

/* ---- selectjoin (gdk_join.c:363-563) ------------------------------------ */

static int
selectjoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_ci *lci,
	   const ora_bat *sr, bool nil_matches, bool swapped)
{
	ora_oid o = ci_get(lci, 0);
	int64_t v = jv(l, o - l->hseqbase);
	if (!nil_matches && v == jnilv(l->type))
		return nomatch(r1p, r2p);
	/* bn = BATselect(r, sr, v, NULL, true, true, false, false) */
	ora_bat *rr = r, *tmp = NULL;
	if (r->type == ORA_void) {
		/* the restated select reads stored values: materialise */
		tmp = ora_new(ORA_oid, r->count, r->hseqbase);
		if (tmp == NULL)
			return -1;
		for (uint64_t p = 0; p < r->count; p++)
			((int64_t *) tmp->base)[p] = jv(r, p);
		rr = tmp;
	}
	union { int8_t b; int16_t s; int32_t i; int64_t l; float f; double d; } val;
	if (l->type == ORA_flt || l->type == ORA_dbl) {
		/* the point select takes the value itself */
		memcpy(&val, (const char *) l->base + (o - l->hseqbase) * l->width, l->width);
	} else {
		switch (rr->width) {
		case 1: val.b = (int8_t) v; break;
		case 2: val.s = (int16_t) v; break;
		case 4: val.i = (int32_t) v; break;
		default: val.l = v; break;
		}
	}
	ora_bat *bn = ora_select(rr, sr, &val, NULL, true, true, false, false);
	ora_free(tmp);
	if (bn == NULL)
		return -1;
	uint64_t bnc = bn->count;
	if (bnc == 0) {
		ora_free(bn);
		return nomatch(r1p, r2p);
	}
	uint64_t cnt = lci->n * bnc;
	ora_bat *a = ora_new(ORA_oid, cnt, 0), *b = ora_new(ORA_oid, cnt, 0);
	if (!a || !b) {
		ora_free(a);
		ora_free(b);
		ora_free(bn);
		return -1;
	}
	a->sorted = 1;
	a->revsorted = lci->n == 1;
	a->tseqbase = bnc == 1 && lci->dense ? o : ORA_OID_NIL;
	a->key = bnc == 1;
	a->nil = 0;
	a->nonil = 1;
	b->sorted = lci->n == 1 || bnc == 1;
	b->revsorted = bnc == 1;
	b->tseqbase = lci->n == 1 && tdense(bn) ? bn->tseqbase : ORA_OID_NIL;
	b->key = lci->n == 1;
	b->nil = 0;
	b->nonil = 1;
	ora_oid *A = a->base, *B = b->base;
	for (uint64_t i = 0, k = 0; i < lci->n; i++) {
		ora_oid lo = ci_get(lci, i);
		for (uint64_t j = 0; j < bnc; j++, k++) {
			A[k] = lo;
			B[k] = bn->type == ORA_void ? bn->tseqbase + j : ((const ora_oid *) bn->base)[j];
		}
	}
	ora_free(bn);
	setcount_props(a);
	setcount_props(b);
	out2(r1p, r2p, a, b, swapped);
	return 0;
}

/* ---- mergejoin_void (gdk_join.c:571-700, no nil_on_miss) ----------------- */

static int
mergejoin_void(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_bat *sl,
	       const ora_ci *rci, bool swapped)
{
	ora_oid lo = r->tseqbase, hi = lo + r->count;
	if (rci->seq > r->hseqbase)
		lo += rci->seq - r->hseqbase;
	if (rci->seq + rci->n < r->hseqbase + r->count)
		hi -= r->hseqbase + r->count - rci->seq - rci->n;
	/* r1 = BATselect(l, sl, &lo, &hi, true, false, false, false) */
	ora_bat *ll = l, *tmp = NULL;
	if (l->type == ORA_void) {
		tmp = ora_new(ORA_oid, l->count, l->hseqbase);
		if (tmp == NULL)
			return -1;
		for (uint64_t p = 0; p < l->count; p++)
			((int64_t *) tmp->base)[p] = jv(l, p);
		ll = tmp;
	}
	ora_bat *a = ora_select(ll, sl, &lo, &hi, true, false, false, false);
	ora_free(tmp);
	if (a == NULL)
		return -1;
	ora_bat *b;
	if (a->count == 0) {
		b = ora_dense(0, 0, 0);
	} else if (tdense(a) && tdense(l)) {
		b = ora_dense(0, l->tseqbase + a->tseqbase - l->hseqbase + r->hseqbase - r->tseqbase, a->count);
	} else {
		b = ora_new(ORA_oid, a->count, 0);
		if (b) {
			for (uint64_t k = 0; k < a->count; k++) {
				ora_oid o1 = a->type == ORA_void ? a->tseqbase + k : ((const ora_oid *) a->base)[k];
				((ora_oid *) b->base)[k] = (ora_oid) jv(l, o1 - l->hseqbase) - r->tseqbase + r->hseqbase;
			}
			b->key = l->key;
			b->sorted = l->sorted;
			b->revsorted = l->revsorted;
			b->nil = 0;
			b->nonil = 1;
			setcount_props(b);
		}
	}
	if (b == NULL) {
		ora_free(a);
		return -1;
	}
	out2(r1p, r2p, a, b, swapped);
	return 0;
}

/* ---- mergejoin (gdk_join.c:1941-2780; :1023-1335 mergejoin_int / _lng) ---- */

/* the matches of one driving value: the candidate index range [lo, hi) of
 * the sorted other side whose values equal v */
static void
equal_range(const ora_bat *r, const ora_ci *rci, bool rasc, int64_t v, uint64_t *lo, uint64_t *hi)
{
	uint64_t a = 0, b = rci->n;
	while (a < b) {                 /* first index not "before" v */
		uint64_t m = (a + b) / 2;
		int64_t x = jv(r, ci_get(rci, m) - r->hseqbase);
		if (rasc ? x < v : x > v)
			a = m + 1;
		else
			b = m;
	}
	uint64_t c = a, d = rci->n;
	while (c < d) {                 /* first index "after" v */
		uint64_t m = (c + d) / 2;
		int64_t x = jv(r, ci_get(rci, m) - r->hseqbase);
		if (rasc ? x <= v : x >= v)
			c = m + 1;
		else
			d = m;
	}
	*lo = a;
	*hi = c;
}

static int
mergejoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_ci *lci,
	  const ora_ci *rci, bool nil_matches, bool swapped)
{
	const int bt = atomtype(l->type);
	const bool special = lci->dense && lci->n == l->count && rci->dense && rci->n == r->count &&
		l->sorted && r->sorted && l->type != ORA_void &&
		(bt == ORA_int || bt == ORA_date || bt == ORA_lng || bt == ORA_oid ||
		 bt == ORA_daytime || bt == ORA_timestamp);
	const bool lsorted = l->sorted || l->revsorted;   /* lscan > 0 */
	const bool rasc = r->sorted;
	const int64_t lnil = jnilv(l->type);
	pairs P = {0};
	uint64_t groups = 0;            /* matched runs of equal driving values */
	bool nlmulti = false;           /* a matched run of several driving rows */
	for (uint64_t i = 0; i < lci->n; i++) {
		ora_oid lo_ = ci_get(lci, i);
		int64_t v = jv(l, lo_ - l->hseqbase);
		if (v == lnil && !nil_matches)
			continue;
		uint64_t a, b;
		equal_range(r, rci, rasc, v, &a, &b);
		if (a == b)
			continue;
		if (i == 0 || jv(l, ci_get(lci, i - 1) - l->hseqbase) != v)
			groups++;
		else
			nlmulti = true;
		for (uint64_t j = a; j < b; j++)
			if (pairs_add(&P, lo_, ci_get(rci, j)) < 0) {
				free(P.a);
				free(P.b);
				return -1;
			}
	}
	ora_bat *A = oidbat(P.a, P.n), *B = oidbat(P.b, P.n);
	free(P.a);
	free(P.b);
	if (!A || !B) {
		ora_free(A);
		ora_free(B);
		return -1;
	}
	const uint64_t n = A->count;
	adj a1 = adjacent(A->base, n), a2 = adjacent(B->base, n);
	/* r1 ascends with the driving candidates: ordered, revsorted only when
	 * all equal, key when no value has several matches */
	A->sorted = 1;
	A->revsorted = !a1.asc;
	A->key = !a1.eq;
	B->sorted = !a2.desc;
	B->key = !a2.eq && !a2.desc;
	if (special) {
		/* mergejoin_int / _lng keep the dense oid columns as oid */
		B->revsorted = !a2.asc;
		B->key = !nlmulti;
		A->tseqbase = n == 0 ? 0 : (A->key && a1.consec ? ((ora_oid *) A->base)[0] : ORA_OID_NIL);
		B->tseqbase = n == 0 ? 0 : (B->key && !a2.desc && a2.consec ? ((ora_oid *) B->base)[0] : ORA_OID_NIL);
		setcount_props(A);
		setcount_props(B);
	} else {
		if (lsorted) {
			/* every property the loop maintains is the column's own */
			B->revsorted = !a2.asc;
			B->key = !nlmulti;
		} else {
			/* l unsorted: r2 is flagged reverse sorted only within one run,
			 * and key only while it ascends (or for two descending rows of two
			 * runs) -- gdk_join.c:2587-2631 */
			B->revsorted = !a2.asc && groups <= 1;
			B->key = (!a2.desc && !a2.eq) ||
				(n == 2 && ((ora_oid *) B->base)[0] > ((ora_oid *) B->base)[1]);
		}
		setcount_props(A);
		setcount_props(B);
		if (A->key)
			virtualize(A);
		if (n <= 1) {
			B->key = 1;
			virtualize(B);
		}
	}
	out2(r1p, r2p, A, B, swapped);
	return 0;
}

/* ---- hashjoin (gdk_join.c:2900-3335) --------------------------------------- */

static int
hashjoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_ci *lci,
	 const ora_ci *rci, bool nil_matches, bool swapped)
{
	uint64_t cap = 16;
	while (cap < 2 * rci->n)
		cap <<= 1;
	int64_t *head = malloc(cap * sizeof(int64_t));
	int64_t *next = malloc((rci->n + 1) * sizeof(int64_t));
	int64_t *keys = malloc((rci->n + 1) * sizeof(int64_t));
	if (!head || !next || !keys) {
		free(head); free(next); free(keys);
		ora_seterr("out of memory");
		return -1;
	}
	memset(head, 0xff, cap * sizeof(int64_t));
	/* chains by prepending (gdk_hash.c:658-704): DESCENDING position */
	for (uint64_t j = 0; j < rci->n; j++) {
		keys[j] = jv(r, ci_get(rci, j) - r->hseqbase);
		uint64_t h = ((uint64_t) keys[j] * 0x9e3779b97f4a7c15ull) >> 20 & (cap - 1);
		next[j] = head[h];
		head[h] = (int64_t) j;
	}
	const int64_t lnil = jnilv(l->type);
	pairs P = {0};
	for (uint64_t i = 0; i < lci->n; i++) {
		ora_oid lo_ = ci_get(lci, i);
		int64_t v = jv(l, lo_ - l->hseqbase);
		if (v == lnil && !nil_matches)
			continue;
		uint64_t h = ((uint64_t) v * 0x9e3779b97f4a7c15ull) >> 20 & (cap - 1);
		for (int64_t j = head[h]; j >= 0; j = next[j])
			if (keys[j] == v && pairs_add(&P, lo_, ci_get(rci, (uint64_t) j)) < 0) {
				free(head); free(next); free(keys); free(P.a); free(P.b);
				return -1;
			}
	}
	free(head); free(next); free(keys);
	ora_bat *A = oidbat(P.a, P.n), *B = oidbat(P.b, P.n);
	free(P.a);
	free(P.b);
	if (!A || !B) {
		ora_free(A);
		ora_free(B);
		return -1;
	}
	const uint64_t n = A->count;
	adj a1 = adjacent(A->base, n);
	A->sorted = 1;
	A->revsorted = !a1.asc;
	A->key = !a1.eq;
	/* r1 keeps a tseqbase while the matched candidates are consecutive
	 * (lskipped, gdk_join.c:3206-3230), only for a dense left candidate list */
	A->tseqbase = lci->dense && A->key && a1.consec ? 0 : ORA_OID_NIL;
	B->sorted = B->revsorted = 0;
	B->key = l->key;
	B->tseqbase = ORA_OID_NIL;
	if (n <= 1) {
		A->sorted = A->revsorted = A->key = 1;
		A->tseqbase = 0;
		B->sorted = B->revsorted = B->key = 1;
		B->tseqbase = 0;
	}
	if (n > 0) {
		if (A->tseqbase != ORA_OID_NIL)
			A->tseqbase = ((ora_oid *) A->base)[0];
		if (B->tseqbase != ORA_OID_NIL)
			B->tseqbase = ((ora_oid *) B->base)[0];
	}
	double ue = l->unique_est < r->unique_est ? l->unique_est : r->unique_est;
	A->unique_est = B->unique_est = ue;
	out2(r1p, r2p, A, B, swapped);
	return 0;
}

/* ---- cost model (gdk_join.c:3337-3689) ------------------------------------- */

/* count_unique (gdk_join.c:3337-3516): distinct values among the first half
 * and among all of the sampled positions s[0..ns) */
static void
count_unique(ora_bat *b, const ora_oid *s, uint64_t ns, uint64_t *cnt1, uint64_t *cnt2)
{
	uint64_t half = ns / 2;
	if (b->key || ns <= 1 || tdense(b)) {
		*cnt1 = half;
		*cnt2 = ns;
		return;
	}
	(void) ordered(b);
	(void) ordered_rev(b);
	if ((b->sorted && b->revsorted) || (b->type == ORA_void && b->tseqbase == ORA_OID_NIL)) {
		*cnt1 = *cnt2 = 1;
		return;
	}
	int64_t *seen = malloc((ns + 1) * sizeof(int64_t));
	uint64_t ndist = 0;
	*cnt1 = 0;
	for (uint64_t i = 0; i < ns; i++) {
		if (i == half)
			*cnt1 = ndist;
		int64_t v = jv(b, s[i] - b->hseqbase);
		bool found = false;
		for (uint64_t k = 0; k < ndist && !found; k++)
			found = seen[k] == v;
		if (!found)
			seen[ndist++] = v;
	}
	*cnt2 = ndist;
	free(seen);
}

/* the rows BATsample(b, 1000) stands for: all of them up to 1000 rows (the
 * reference's own rule, gdk_sample.c:114-117), else 1000 evenly spaced */
static uint64_t
sample_positions(uint64_t cnt, uint64_t *pos)
{
	if (cnt <= 1000) {
		for (uint64_t i = 0; i < cnt; i++)
			pos[i] = i;
		return cnt;
	}
	for (uint64_t i = 0; i < 1000; i++)
		pos[i] = (uint64_t) ((unsigned __int128) i * cnt / 1000);
	return 1000;
}

/* guess_uniques (gdk_join.c:3518-3576); s is the candidate BAT behind ci
 * (NULL: all of b).  A candidate list is sampled whole (not clipped to b)
 * and the sample projected through it, as BATsample + BATproject do. */
static double
guess_uniques(ora_bat *b, const ora_ci *ci, const ora_bat *s)
{
	if (b->key)
		return (double) ci->n;
	uint64_t pos[1000];
	ora_oid s1[1000];
	uint64_t n2;
	const bool full = s == NULL || (ci->dense && ci->n == b->count);
	if (full) {
		if (b->unique_est != 0)
			return b->unique_est;
		n2 = sample_positions(b->count, pos);
		for (uint64_t i = 0; i < n2; i++)
			s1[i] = b->hseqbase + pos[i];
	} else {
		n2 = sample_positions(s->count, pos);
		for (uint64_t i = 0; i < n2; i++)
			s1[i] = s->type == ORA_void ? s->tseqbase + pos[i] : ((const ora_oid *) s->base)[pos[i]];
	}
	uint64_t n1 = n2 / 2, cnt1, cnt2;
	/* count_unique iterates the sample as a candidate list of b (clipped) */
	uint64_t lo = 0, hi = n2;
	while (lo < hi && s1[lo] < b->hseqbase)
		lo++;
	while (hi > lo && s1[hi - 1] >= b->hseqbase + b->count)
		hi--;
	count_unique(b, s1 + lo, hi - lo, &cnt1, &cnt2);
	double A = (double) (cnt2 - cnt1) / (n2 - n1);
	double B = cnt1 - n1 * A;
	B += A * ci->n;
	if (full && b->unique_est == 0)
		b->unique_est = B;
	return B;
}

/* joincost (gdk_join.c:3586-3689) with no prebuilt hash */
static double
joincost(ora_bat *r, uint64_t lcount, const ora_ci *rci, const ora_bat *sr)
{
	double rcost = 1;
	if (!rci->dense && rci->n > 0)
		rcost += log2((double) rci->n);
	rcost *= lcount;
	const uint64_t cnt = r->count;
	if (!tdense(r)) {
		double ue = r->unique_est;
		if (ue == 0) {
			ora_ci all = {.dense = true, .seq = r->hseqbase, .n = r->count};
			ue = guess_uniques(r, &all, NULL);
		}
		rcost *= 1.1 * ((double) cnt / ue);
		rcost += cnt * 2.0;
	}
	if (rci->n != cnt) {
		double ue = r->unique_est;
		if (ue == 0)
			ue = guess_uniques(r, rci, sr);
		double rccost = 1.1 * ((double) cnt / ue);
		rccost *= lcount;
		rccost += rci->n * 2.0;
		if (rccost < rcost)
			rcost = rccost;
	}
	return rcost;
}

/* ---- str keys: BATjoin compares with strCmp (nil "\200" first, then
 * strcmp's unsigned bytes) and hashes the string (strHash); every algorithm
 * choice, scan and result order only depends on that order and equality,
 * so the pair of str columns joins exactly as the pair of lng columns that
 * hold each string's rank among the distinct strings of both sides (nil ->
 * lng nil).  The ranks come from a qsort of all strings here. */
static const char *
jstr_at(const ora_bat *b, uint64_t p)
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
jstr_nil(const char *s)
{
	return (unsigned char) s[0] == 0x80 && s[1] == 0;
}

static int
jstr_qcmp(const void *a, const void *b)
{
	return strcmp(*(const char *const *) a, *(const char *const *) b);
}

static ora_bat *
jstr_image(const ora_bat *b, const char **dict, uint64_t nd)
{
	ora_bat *m = ora_new(ORA_lng, b->count, b->hseqbase);
	if (m == NULL)
		return NULL;
	int64_t *o = m->base;
	for (uint64_t i = 0; i < b->count; i++) {
		const char *s = jstr_at(b, i);
		if (jstr_nil(s)) {
			o[i] = INT64_MIN;
			continue;
		}
		uint64_t lo = 0, hi = nd;
		while (lo < hi) {
			uint64_t mid = (lo + hi) / 2;
			if (strcmp(dict[mid], s) < 0)
				lo = mid + 1;
			else
				hi = mid;
		}
		o[i] = (int64_t) lo;
	}
	m->sorted = b->sorted;
	m->revsorted = b->revsorted;
	m->key = b->key;
	m->nonil = b->nonil;
	m->nil = b->nil;
	m->unique_est = b->unique_est;
	return m;
}

static int
str_images(const ora_bat *l, const ora_bat *r, ora_bat **lip, ora_bat **rip)
{
	*lip = *rip = NULL;
	const uint64_t n = l->count + r->count;
	const char **dict = malloc((n ? n : 1) * sizeof(char *));
	if (dict == NULL) {
		ora_seterr("malloc");
		return -1;
	}
	uint64_t nd = 0;
	for (int side = 0; side < 2; side++) {
		const ora_bat *b = side ? r : l;
		for (uint64_t i = 0; i < b->count; i++) {
			const char *s = jstr_at(b, i);
			if (!jstr_nil(s))
				dict[nd++] = s;
		}
	}
	qsort(dict, nd, sizeof(char *), jstr_qcmp);
	uint64_t k = 0;
	for (uint64_t i = 0; i < nd; i++)
		if (k == 0 || strcmp(dict[k - 1], dict[i]) != 0)
			dict[k++] = dict[i];
	*lip = jstr_image(l, dict, k);
	*rip = *lip ? jstr_image(r, dict, k) : NULL;
	free(dict);
	if (*rip == NULL) {
		if (*lip)
			ora_free(*lip);
		*lip = NULL;
		return -1;
	}
	return 0;
}

/* what the scans found on the images holds for the strings */
static void
str_flags_back(ora_bat *l, ora_bat *r, ora_bat *li, ora_bat *ri)
{
	l->sorted = li->sorted;
	l->revsorted = li->revsorted;
	l->key = li->key;
	l->unique_est = li->unique_est;
	r->sorted = ri->sorted;
	r->revsorted = ri->revsorted;
	r->key = ri->key;
	r->unique_est = ri->unique_est;
	ora_free(li);
	ora_free(ri);
}

/* ---- BATjoin (gdk_join.c:4451-4623) ---------------------------------------- */

int
ora_join(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r,
	 const ora_bat *sl, const ora_bat *sr, bool nil_matches)
{
	if (l->type == ORA_msk || r->type == ORA_msk) {
		/* msk inputs joined as their BATunmask (gdk_join.c:4500-4517) */
		ora_bat *lm = l->type == ORA_msk ? ora_unmask(l) : NULL;
		ora_bat *rm = r->type == ORA_msk ? ora_unmask(r) : NULL;
		int rc = -1;
		if ((l->type != ORA_msk || lm) && (r->type != ORA_msk || rm))
			rc = ora_join(r1p, r2p, lm ? lm : l, rm ? rm : r, sl, sr, nil_matches);
		if (lm)
			ora_free(lm);
		if (rm)
			ora_free(rm);
		return rc;
	}
	if (atomtype(l->type) != atomtype(r->type)) {
		ora_seterr("BATjoin: inputs not compatible.");
		return -1;
	}
	if (l->type == ORA_str) {
		ora_bat *li, *ri;
		if (str_images(l, r, &li, &ri) < 0)
			return -1;
		int rc = ora_join(r1p, r2p, li, ri, sl, sr, nil_matches);
		str_flags_back(l, r, li, ri);
		return rc;
	}
	if (!join_type_ok(l->type) || !join_type_ok(r->type)) {
		ora_seterr("BATjoin: type not restated");
		return -1;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, r, sr) < 0)
		return -1;
	if (lci.n == 0 || rci.n == 0)
		return nomatch(r1p, r2p);
	if (lci.n == 1 || (ordered(l) && ordered_rev(l)) ||
	    (l->type == ORA_void && l->tseqbase == ORA_OID_NIL))
		return selectjoin(r1p, r2p, l, r, &lci, sr, nil_matches, false);
	if (rci.n == 1 || (ordered(r) && ordered_rev(r)) ||
	    (r->type == ORA_void && r->tseqbase == ORA_OID_NIL))
		return selectjoin(r1p, r2p, r, l, &rci, sl, nil_matches, true);
	if (tdense(r) && rci.dense)
		return mergejoin_void(r1p, r2p, l, r, sl, &rci, false);
	if (tdense(l) && lci.dense)
		return mergejoin_void(r1p, r2p, r, l, sr, &lci, true);
	if ((ordered(l) || ordered_rev(l)) && (ordered(r) || ordered_rev(r)))
		return mergejoin(r1p, r2p, l, r, &lci, &rci, nil_matches, false);
	double lcost = joincost(l, rci.n, &lci, sl);
	double rcost = joincost(r, lci.n, &rci, sr);
	bool swap = lcost < rcost;
	double best = swap ? lcost : rcost;
	if ((ordered(r) || ordered_rev(r)) && lci.n * (log2((double) rci.n) + 1) < best)
		return mergejoin(r1p, r2p, l, r, &lci, &rci, nil_matches, false);
	if ((ordered(l) || ordered_rev(l)) && rci.n * (log2((double) lci.n) + 1) < best)
		return mergejoin(r1p, r2p, r, l, &rci, &lci, nil_matches, true);
	if (swap)
		return hashjoin(r1p, r2p, r, l, &rci, &lci, nil_matches, true);
	return hashjoin(r1p, r2p, l, r, &lci, &rci, nil_matches, false);
}

/* which algorithm ora_join takes (tests assert the branch they mean to
 * cover): 0 nomatch, 1 selectjoin, 2 selectjoin swapped, 3 mergejoin_void,
 * 4 mergejoin_void swapped, 5 mergejoin (both sorted), 6 mergejoin (r
 * sorted, cheaper), 7 mergejoin swapped, 8 hashjoin swapped, 9 hashjoin.
 * Evaluates the same conditions (and caches the same flags). */
int
ora_join_algo(ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr)
{
	if (l->type == ORA_str && r->type == ORA_str) {
		ora_bat *li, *ri;
		if (str_images(l, r, &li, &ri) < 0)
			return -1;
		int a = ora_join_algo(li, ri, sl, sr);
		str_flags_back(l, r, li, ri);
		return a;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, r, sr) < 0)
		return -1;
	if (lci.n == 0 || rci.n == 0)
		return 0;
	if (lci.n == 1 || (ordered(l) && ordered_rev(l)) ||
	    (l->type == ORA_void && l->tseqbase == ORA_OID_NIL))
		return 1;
	if (rci.n == 1 || (ordered(r) && ordered_rev(r)) ||
	    (r->type == ORA_void && r->tseqbase == ORA_OID_NIL))
		return 2;
	if (tdense(r) && rci.dense)
		return 3;
	if (tdense(l) && lci.dense)
		return 4;
	if ((ordered(l) || ordered_rev(l)) && (ordered(r) || ordered_rev(r)))
		return 5;
	double lcost = joincost(l, rci.n, &lci, sl);
	double rcost = joincost(r, lci.n, &rci, sr);
	bool swap = lcost < rcost;
	double best = swap ? lcost : rcost;
	if ((ordered(r) || ordered_rev(r)) && lci.n * (log2((double) rci.n) + 1) < best)
		return 6;
	if ((ordered(l) || ordered_rev(l)) && rci.n * (log2((double) lci.n) + 1) < best)
		return 7;
	return swap ? 8 : 9;
}

/* ---- semi / anti / outer joins (gdk_join.c:4049 leftjoin, :4320-4407) ----
 * BATintersect / BATsemijoin's r1 (semi), BATdiff (only_misses, not_in) and
 * BATleftjoin / BATouterjoin (nil_on_miss, match_one) restated by their
 * result definitions, which every path of leftjoin shares:
 *   a left candidate's matches are the right candidates with an equal value;
 *   a nil never matches unless nil_matches (gdk_join.c:3127, :2338);
 *   semi: the left candidates with a match, once each, in order (virtualized);
 *     max_one: "more than one match" when a candidate has two (:2760);
 *   only_misses: the left candidates without a match; not_in additionally
 *     drops nil left values and returns nothing when a right candidate is nil
 *     (:3027-3060, :2038) -- except on the dense-right path, mergejoin_void
 *     (:4096-4101), which has no not_in and no nil on the right;
 *   empty left or right side: nomatch (:301-360), the misses being every
 *   left candidate;
 *   left / outer join: the matched pairs in left order (outer: a miss gives
 *   (l, nil)); a left candidate with several matches orders them by the
 *   algorithm leftjoin picks, which this restatement does not model, so it is
 *   refused (-2) unless match_one asks for the reference's error. */
typedef struct {
	int64_t v;
	ora_oid o;
} vpair;

static int
vpair_cmp(const void *a, const void *b)
{
	const vpair *x = a, *y = b;
	if (x->v != y->v)
		return x->v < y->v ? -1 : 1;
	return x->o < y->o ? -1 : x->o > y->o;
}

/* leftjoin's algorithms (gdk_join.c:4049-4300; lj_algo below) */
enum { LJ_NOMATCH = 0, LJ_SELECT = 1, LJ_MJVOID = 2, LJ_FETCH = 3, LJ_BITMASK = 4, LJ_MERGE = 5, LJ_SWAP = 6,
       LJ_HASH = 7 };
static int lj_algo(ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr, const ora_ci *lci,
		   const ora_ci *rci, bool nil_matches, bool nil_on_miss, bool semi, bool only_misses, bool not_in,
		   bool max_one, bool min_one, bool want_r2, bool *equal_order);

/* the right candidates' (value, oid), sorted; *rnil: some value is nil */
static vpair *
rpairs(const ora_bat *r, const ora_ci *rci, bool *rnil)
{
	vpair *p = malloc((rci->n + 1) * sizeof(vpair));
	if (p == NULL)
		return NULL;
	*rnil = false;
	const int64_t nil = jnilv(r->type);
	for (uint64_t i = 0; i < rci->n; i++) {
		const ora_oid o = ci_get(rci, i);
		p[i].v = jv(r, o - r->hseqbase);
		p[i].o = o;
		if (r->type != ORA_void && p[i].v == nil)
			*rnil = true;
		if (r->type == ORA_void && r->tseqbase == ORA_OID_NIL)
			*rnil = true;
	}
	qsort(p, rci->n, sizeof(vpair), vpair_cmp);
	return p;
}

static uint64_t
vlower(const vpair *p, uint64_t n, int64_t v)
{
	uint64_t lo = 0, hi = n;
	while (lo < hi) {
		uint64_t m = (lo + hi) / 2;
		if (p[m].v < v)
			lo = m + 1;
		else
			hi = m;
	}
	return lo;
}

static bool
lnil(const ora_bat *l, int64_t v)
{
	if (l->type == ORA_void)
		return l->tseqbase == ORA_OID_NIL;
	return v == jnilv(l->type);
}

/* semi (only_misses = false) or anti (true) join's left output */
ora_bat *
ora_semijoin_cands(ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr, bool nil_matches,
		   bool max_one, bool only_misses, bool not_in)
{
	if (atomtype(l->type) != atomtype(r->type) || !join_type_ok(l->type) || l->type == ORA_flt ||
	    l->type == ORA_dbl) {
		ora_seterr("leftjoin: type not restated");
		return NULL;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, r, sr) < 0)
		return NULL;
	ora_oid *o = malloc((lci.n + 1) * sizeof(ora_oid));
	if (o == NULL) {
		ora_seterr("malloc");
		return NULL;
	}
	uint64_t k = 0;
	if (lci.n == 0 || rci.n == 0) {
		if (only_misses)
			for (uint64_t i = 0; i < lci.n; i++)
				o[k++] = ci_get(&lci, i);
	} else {
		if (tdense(r) && rci.dense)
			not_in = false;             /* mergejoin_void */
		/* mergejoin with an ordered l skips l's nils before its scan when
		 * neither nil_matches nor nil_on_miss is set (gdk_join.c:2093-2100):
		 * BATdiff then does not list them (the other paths do) */
		bool skipnil = false;
		if (only_misses && !not_in && !nil_matches) {
			bool eqo;
			skipnil = lj_algo(l, r, sl, sr, &lci, &rci, nil_matches, false, false, true, false, false, false,
					  false, &eqo) == LJ_MERGE && (l->sorted || l->revsorted);
		}
		bool rnil;
		vpair *p = rpairs(r, &rci, &rnil);
		if (p == NULL) {
			free(o);
			ora_seterr("malloc");
			return NULL;
		}
		if (!(not_in && rnil)) {
			for (uint64_t i = 0; i < lci.n; i++) {
				const ora_oid lo = ci_get(&lci, i);
				const int64_t v = jv(l, lo - l->hseqbase);
				uint64_t cnt = 0;
				if (lnil(l, v) && (!nil_matches || not_in)) {
					if (not_in || skipnil)
						continue;
				} else {
					const uint64_t a = vlower(p, rci.n, v);
					uint64_t b = a;
					while (b < rci.n && p[b].v == v)
						b++;
					cnt = b - a;
				}
				if (cnt > 1 && max_one && !only_misses) {
					free(p);
					free(o);
					ora_seterr("more than one match");
					return NULL;
				}
				if ((cnt > 0) != only_misses)
					o[k++] = lo;
			}
		}
		free(p);
	}
	ora_bat *bn = oidbat(o, k);
	free(o);
	if (bn == NULL)
		return NULL;
	bn->sorted = bn->key = 1;
	bn->revsorted = k <= 1;
	virtualize(bn);
	return bn;
}

/* BATleftjoin (outer = false) / BATouterjoin (outer = true) for right
 * candidates whose values match at most once per left candidate: returns
 * -2 when a left candidate matches twice and match_one is not set */
int
ora_leftjoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr,
	     bool nil_matches, bool outer, bool match_one)
{
	if (atomtype(l->type) != atomtype(r->type) || !join_type_ok(l->type) || l->type == ORA_flt ||
	    l->type == ORA_dbl) {
		ora_seterr("leftjoin: type not restated");
		return -1;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, r, sr) < 0)
		return -1;
	ora_oid *a = malloc((lci.n + 1) * sizeof(ora_oid)), *b = malloc((lci.n + 1) * sizeof(ora_oid));
	bool rnil;
	vpair *p = rci.n ? rpairs(r, &rci, &rnil) : NULL;
	if (a == NULL || b == NULL || (rci.n && p == NULL)) {
		free(a);
		free(b);
		free(p);
		ora_seterr("malloc");
		return -1;
	}
	uint64_t k = 0;
	bool anynil = false;
	for (uint64_t i = 0; i < lci.n; i++) {
		const ora_oid lo = ci_get(&lci, i);
		const int64_t v = jv(l, lo - l->hseqbase);
		uint64_t cnt = 0, at = 0;
		if (rci.n && !(lnil(l, v) && !nil_matches)) {
			at = vlower(p, rci.n, v);
			uint64_t e = at;
			while (e < rci.n && p[e].v == v)
				e++;
			cnt = e - at;
		}
		if (cnt > 1) {
			free(a);
			free(b);
			free(p);
			if (match_one) {
				ora_seterr("more than one match");
				return -1;
			}
			return -2;
		}
		if (cnt == 1) {
			a[k] = lo;
			b[k++] = p[at].o;
		} else if (outer) {
			a[k] = lo;
			b[k++] = ORA_OID_NIL;
			anynil = true;
		}
	}
	free(p);
	ora_bat *x = oidbat(a, k), *y = oidbat(b, k);
	free(a);
	free(b);
	if (x == NULL || y == NULL) {
		ora_free(x);
		ora_free(y);
		return -1;
	}
	x->sorted = x->key = 1;
	x->revsorted = k <= 1;
	y->nil = anynil;
	y->nonil = !anynil;
	*r1p = x;
	*r2p = y;
	return 0;
}

/* BATmarkjoin (gdk_join.c:4367: leftjoin with nil_on_miss, semi when r2p is
 * NULL): every left candidate once, its match (nil on a miss) and a mark:
 * TRUE on a match; on a miss nil when the left value is nil (hashjoin
 * :3127-3133, selectjoin :386-391, mergejoin_void :3100) or a right candidate
 * is nil (defmark, hashjoin :3026-3076, selectjoin :513-527, mergejoin
 * :2033-2036), else FALSE; no right candidates: FALSE everywhere (leftjoin
 * :4144 nomatch with defmark 0).  With r2p, -2 when a left candidate matches
 * twice (the order of several matches is the algorithm's). */
int
ora_markjoin(ora_bat **r1p, ora_bat **r2p, ora_bat **r3p, ora_bat *l, ora_bat *r, const ora_bat *sl,
	     const ora_bat *sr)
{
	if (atomtype(l->type) != atomtype(r->type) || !join_type_ok(l->type) || l->type == ORA_flt ||
	    l->type == ORA_dbl) {
		ora_seterr("markjoin: type not restated");
		return -1;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, r, sr) < 0)
		return -1;
	ora_oid *a = malloc((lci.n + 1) * sizeof(ora_oid)), *b = malloc((lci.n + 1) * sizeof(ora_oid));
	int8_t *m = malloc(lci.n + 1);
	bool rnil = false;
	vpair *p = rci.n ? rpairs(r, &rci, &rnil) : NULL;
	if (a == NULL || b == NULL || m == NULL || (rci.n && p == NULL)) {
		free(a);
		free(b);
		free(m);
		free(p);
		ora_seterr("malloc");
		return -1;
	}
	bool anynil = false, mnil = false;
	for (uint64_t i = 0; i < lci.n; i++) {
		const ora_oid lo = ci_get(&lci, i);
		const int64_t v = jv(l, lo - l->hseqbase);
		uint64_t cnt = 0, at = 0;
		int8_t mk = 0;
		if (rci.n) {
			if (lnil(l, v)) {
				mk = INT8_MIN;
			} else {
				at = vlower(p, rci.n, v);
				uint64_t e = at;
				while (e < rci.n && p[e].v == v)
					e++;
				cnt = e - at;
				mk = cnt ? 1 : rnil ? INT8_MIN : 0;
			}
		}
		if (cnt > 1 && r2p) {
			free(a);
			free(b);
			free(m);
			free(p);
			return -2;
		}
		a[i] = lo;
		b[i] = cnt ? p[at].o : ORA_OID_NIL;
		m[i] = mk;
		anynil |= cnt == 0;
		mnil |= mk == INT8_MIN;
	}
	free(p);
	const uint64_t n = lci.n;
	ora_bat *x = oidbat(a, n), *y = r2p ? oidbat(b, n) : NULL, *z = ora_new(ORA_bit, n, 0);
	free(a);
	free(b);
	if (x == NULL || (r2p && y == NULL) || z == NULL) {
		free(m);
		ora_free(x);
		ora_free(y);
		ora_free(z);
		return -1;
	}
	memcpy(z->base, m, n);
	free(m);
	z->nil = mnil;
	z->nonil = !mnil;
	x->sorted = x->key = 1;
	x->revsorted = n <= 1;
	*r1p = x;
	if (r2p) {
		y->nil = anynil;
		y->nonil = !anynil;
		*r2p = y;
	}
	*r3p = z;
	return 0;
}

/* ---- BATthetajoin / BATbandjoin (gdk/gdk_join.c:3699-3889 thetajoin,
 * :4626-5000 BATbandjoin): the nested loops as the reference runs them --
 * left candidates in order, each one's matches in right-candidate order.
 * theta compares with ATOMcompare (jv's images: nil the smallest, -0.0 ==
 * +0.0); mask 1 EQ, 2 LT, 4 GT (vl op vr).  band: vr - c1 <= vl <= vr + c2
 * in the reference's arithmetic per type (integers widened, flt in dbl, dbl
 * with SUBF / ADDF_WITH_CHECK and their goto rules), nils never match. */

static int
pair_out(ora_bat **r1p, ora_bat **r2p, ora_oid *a, ora_oid *b, uint64_t n)
{
	ora_bat *x = ora_new(ORA_oid, n, 0), *y = ora_new(ORA_oid, n, 0);
	memcpy(x->base, a, n * sizeof(ora_oid));
	memcpy(y->base, b, n * sizeof(ora_oid));
	x->sorted = 1;
	x->nonil = y->nonil = 1;
	*r1p = x;
	*r2p = y;
	return 0;
}

int
ora_thetajoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr, int mask,
	      bool nil_matches)
{
	if (atomtype(l->type) != atomtype(r->type)) {
		ora_seterr("BATthetajoin: inputs not compatible.\n");
		return -1;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, r, sr) < 0)
		return -1;
	const bool lall = l->type == ORA_void && l->tseqbase == ORA_OID_NIL;
	const bool rall = r->type == ORA_void && r->tseqbase == ORA_OID_NIL;
	uint64_t cap = 1024, n = 0;
	ora_oid *a = malloc(cap * sizeof(ora_oid)), *b = malloc(cap * sizeof(ora_oid));
	if ((lall || rall) && !nil_matches)
		goto done;     /* nomatch (:3738-3763) */
	for (uint64_t i = 0; i < lci.n; i++) {
		const ora_oid lo = ci_get(&lci, i);
		const int64_t vl = jv(l, lo - l->hseqbase);
		if (!nil_matches && lnil(l, vl))
			continue;
		for (uint64_t j = 0; j < rci.n; j++) {
			const ora_oid ro = ci_get(&rci, j);
			const int64_t vr = jv(r, ro - r->hseqbase);
			if (!nil_matches && lnil(r, vr))
				continue;
			const int c = (vl > vr) - (vl < vr);
			if (!((mask & 2 && c < 0) || (mask & 4 && c > 0) || (mask & 1 && c == 0)))
				continue;
			if (n == cap) {
				cap *= 2;
				a = realloc(a, cap * sizeof(ora_oid));
				b = realloc(b, cap * sizeof(ora_oid));
			}
			a[n] = lo;
			b[n++] = ro;
		}
	}
done:
	pair_out(r1p, r2p, a, b, n);
	free(a);
	free(b);
	return 0;
}

static bool
band_match(const ora_bat *l, const ora_bat *r, uint64_t pl, uint64_t pr, const void *c1p, const void *c2p,
	   bool linc, bool hinc)
{
	switch (l->type) {
	case ORA_flt: {
		const float vl = ((const float *) l->base)[pl], vr = ((const float *) r->base)[pr];
		const float c1 = *(const float *) c1p, c2 = *(const float *) c2p;
		if (isnan(vr))
			return false;
		double v1 = (double) vr, v2 = v1;
		v1 -= c1;
		if (vl <= v1 && (!linc || vl != v1))
			return false;
		v2 += c2;
		if (vl >= v2 && (!hinc || vl != v2))
			return false;
		return true;
	}
	case ORA_dbl: {
		const double vl = ((const double *) l->base)[pl], vr = ((const double *) r->base)[pr];
		const double c1 = *(const double *) c1p, c2 = *(const double *) c2p;
		if (isnan(vr))
			return false;
		double v1, v2;
		if (c1 < 1 ? DBL_MAX + c1 < vr : -DBL_MAX + c1 > vr) {
			if (c1 < 0)
				return false;
		} else {
			v1 = vr - c1;
			if (vl <= v1 && (!linc || vl != v1))
				return false;
		}
		if (c2 < 1 ? -DBL_MAX - c2 > vr : DBL_MAX - c2 < vr)
			return !(c2 > 0);
		v2 = vr + c2;
		if (vl >= v2 && (!hinc || vl != v2))
			return false;
		return true;
	}
	default: {
		const int64_t vl = jv(l, pl), vr = jv(r, pr);
		if (vr == jnilv(r->type))
			return false;
		ora_hge c1, c2;
		switch (l->type) {
		case ORA_bte: c1 = *(const int8_t *) c1p; c2 = *(const int8_t *) c2p; break;
		case ORA_sht: c1 = *(const int16_t *) c1p; c2 = *(const int16_t *) c2p; break;
		case ORA_int: case ORA_date: c1 = *(const int32_t *) c1p; c2 = *(const int32_t *) c2p; break;
		default: c1 = *(const int64_t *) c1p; c2 = *(const int64_t *) c2p; break;
		}
		const ora_hge v1 = (ora_hge) vr - c1, v2 = (ora_hge) vr + c2;
		if (vl <= v1 && (!linc || vl != v1))
			return false;
		if (vl >= v2 && (!hinc || vl != v2))
			return false;
		return true;
	}
	}
}

int
ora_bandjoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr,
	     const void *c1p, const void *c2p, bool linc, bool hinc)
{
	if (atomtype(l->type) != atomtype(r->type)) {
		ora_seterr("BATbandjoin: inputs not compatible.\n");
		return -1;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, r, sr) < 0)
		return -1;
	uint64_t cap = 1024, n = 0;
	ora_oid *a = malloc(cap * sizeof(ora_oid)), *b = malloc(cap * sizeof(ora_oid));
	bool empty;
	switch (l->type) {
#define BE(T, NILT) { const T c1 = *(const T *) c1p, c2 = *(const T *) c2p; \
		empty = NILT || -c1 > c2 || ((!hinc || !linc) && -c1 == c2); }
	case ORA_bte: BE(int8_t, (c1 == INT8_MIN || c2 == INT8_MIN)) break;
	case ORA_sht: BE(int16_t, (c1 == INT16_MIN || c2 == INT16_MIN)) break;
	case ORA_int: case ORA_date: BE(int32_t, (c1 == INT32_MIN || c2 == INT32_MIN)) break;
	case ORA_lng: BE(int64_t, (c1 == INT64_MIN || c2 == INT64_MIN)) break;
	case ORA_flt: BE(float, (isnan(c1) || isnan(c2))) break;
	case ORA_dbl: BE(double, (isnan(c1) || isnan(c2))) break;
#undef BE
	default:
		free(a);
		free(b);
		ora_seterr("unsupported type\n");
		return -1;
	}
	if (lci.n == 0 || rci.n == 0 || empty)
		goto done;
	for (uint64_t i = 0; i < lci.n; i++) {
		const ora_oid lo = ci_get(&lci, i);
		const uint64_t pl = lo - l->hseqbase;
		bool ln;
		if (l->type == ORA_flt)
			ln = isnan(((const float *) l->base)[pl]);
		else if (l->type == ORA_dbl)
			ln = isnan(((const double *) l->base)[pl]);
		else
			ln = jv(l, pl) == jnilv(l->type);
		if (ln)
			continue;
		for (uint64_t j = 0; j < rci.n; j++) {
			const ora_oid ro = ci_get(&rci, j);
			if (!band_match(l, r, pl, ro - r->hseqbase, c1p, c2p, linc, hinc))
				continue;
			if (n == cap) {
				cap *= 2;
				a = realloc(a, cap * sizeof(ora_oid));
				b = realloc(b, cap * sizeof(ora_oid));
			}
			a[n] = lo;
			b[n++] = ro;
		}
	}
done:
	pair_out(r1p, r2p, a, b, n);
	free(a);
	free(b);
	return 0;
}

/* ---- BATrangejoin (gdk/gdk_join.c:5422-5471, rangejoin :5067-5420) -----
 * l within [rl, rh] per right candidate (linc / hinc: the ends included).
 * Not anti, not symmetric and l sorted or reverse sorted (BATordered /
 * BATordered_rev are computed first, :5071-5075): for each right candidate
 * in order, the l positions of the range by binary search (SORTfndfirst /
 * SORTfndlast), mapped to the left candidates in between -- right-major
 * output.  Otherwise the nested loop: left-major, BETWEEN's three-valued
 * logic (:5040-5064; a nil bound gives nil, which never matches, but its
 * negation under anti is nil too).  An order index would take the first
 * path through it; the oracle (like the device) keeps no order indexes.
 * The result properties come from the reference's extra scan (:5351-5410),
 * restated over the whole result (the scan only stops once nothing can
 * change). */

static uint64_t
ci_lower(const ora_ci *ci, ora_oid o)
{
	if (ci->dense)
		return o <= ci->seq ? 0 : (o - ci->seq < ci->n ? o - ci->seq : ci->n);
	uint64_t a = 0, b = ci->n;
	while (a < b) {
		const uint64_t m = (a + b) / 2;
		if (ci->oids[m] < o)
			a = m + 1;
		else
			b = m;
	}
	return a;
}

/* first position of l (sorted: value >= v / > v; reverse sorted: <= v / < v) */
static uint64_t
sortfnd(const ora_bat *l, bool rev, int64_t v, bool last)
{
	uint64_t a = 0, b = l->count;
	while (a < b) {
		const uint64_t m = (a + b) / 2;
		const int64_t x = jv(l, m);
		const bool before = rev ? (last ? x >= v : x > v) : (last ? x <= v : x < v);
		if (before)
			a = m + 1;
		else
			b = m;
	}
	return a;
}

static int
between3(int64_t v, bool vn, int64_t lo, bool lon, bool linc, int64_t hi, bool hin, bool hinc)
{
	/* 1 true, 0 false, -1 nil */
	const int g = vn || lon ? -1 : (lo < v || (linc && v == lo));
	const int l = vn || hin ? -1 : (v < hi || (hinc && v == hi));
	if (g == 0 || l == 0)
		return 0;
	if (g < 0 || l < 0)
		return -1;
	return 1;
}

static void
oid_props(ora_bat *b)
{
	const ora_oid *d = b->base;
	bool eq = false, lt = false, gt = false, gap = false;
	for (uint64_t i = 1; i < b->count; i++) {
		if (d[i - 1] == d[i])
			eq = true;
		else if (d[i - 1] < d[i]) {
			lt = true;
			gap |= d[i - 1] + 1 != d[i];
		} else
			gt = true;
	}
	b->key = !eq && !gt;
	b->sorted = !gt;
	b->revsorted = !lt;
	b->nil = false;
	b->nonil = true;
	b->tseqbase = !eq && !gt && !gap ? (b->count ? d[0] : 0) : ORA_OID_NIL;
}

int
ora_rangejoin(ora_bat **r1p, ora_bat **r2p, ora_bat *l, ora_bat *rl, ora_bat *rh, const ora_bat *sl,
	      const ora_bat *sr, bool linc, bool hinc, bool anti, bool symmetric)
{
	if (atomtype(l->type) != atomtype(rl->type) || atomtype(l->type) != atomtype(rh->type)) {
		ora_seterr("BATrangejoin: inputs not compatible.\n");
		return -1;
	}
	if (rl->count != rh->count || rl->hseqbase != rh->hseqbase) {
		ora_seterr("BATrangejoin: right inputs not aligned.\n");
		return -1;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, rl, sr) < 0)
		return -1;
	const bool lnilall = l->type == ORA_void && l->tseqbase == ORA_OID_NIL;
	const bool rlnil = rl->type == ORA_void && rl->tseqbase == ORA_OID_NIL;
	const bool rhnil = rh->type == ORA_void && rh->tseqbase == ORA_OID_NIL;
	uint64_t cap = 1024, n = 0;
	ora_oid *a = malloc(cap * sizeof(ora_oid)), *b = malloc(cap * sizeof(ora_oid));
	if (lci.n == 0 || rci.n == 0 || lnilall || (rlnil && rhnil) || ((rlnil || rhnil) && !anti))
		goto done;
	if (rlnil || rhnil) {
		free(a);
		free(b);
		/* anti with a nil bound column: l > rh (or l < rl), gdk_join.c:5448-5460 */
		return ora_thetajoin(r1p, r2p, l, rlnil ? rh : rl, sl, sr, rlnil ? 4 : 2, false);
	}
#define ADD(x, y) do { if (n == cap) { cap *= 2; a = realloc(a, cap * sizeof(ora_oid)); \
			b = realloc(b, cap * sizeof(ora_oid)); } a[n] = (x); b[n++] = (y); } while (0)
	if (!anti && !symmetric && (ordered(l) || ordered_rev(l))) {
		const bool rev = !ordered(l);
		for (uint64_t j = 0; j < rci.n; j++) {
			const ora_oid ro = ci_get(&rci, j);
			const int64_t vlo = jv(rl, ro - rl->hseqbase), vhi = jv(rh, ro - rh->hseqbase);
			if (lnil(rl, vlo) || lnil(rh, vhi))
				continue;
			uint64_t low, high;
			if (!rev) {
				low = sortfnd(l, false, vlo, !linc);
				high = sortfnd(l, false, vhi, hinc);
			} else {
				low = sortfnd(l, true, vhi, !hinc);
				high = sortfnd(l, true, vlo, linc);
			}
			if (high <= low)
				continue;
			const uint64_t cl = ci_lower(&lci, low + l->hseqbase), ch = ci_lower(&lci, high + l->hseqbase);
			for (uint64_t q = cl; q < ch; q++)
				ADD(ci_get(&lci, q), ro);
		}
	} else {
		for (uint64_t i = 0; i < lci.n; i++) {
			const ora_oid lo = ci_get(&lci, i);
			const int64_t v = jv(l, lo - l->hseqbase);
			const bool vn = l->type != ORA_void && lnil(l, v);
			if (vn)
				continue;
			for (uint64_t j = 0; j < rci.n; j++) {
				const ora_oid ro = ci_get(&rci, j);
				const int64_t vlo = jv(rl, ro - rl->hseqbase), vhi = jv(rh, ro - rh->hseqbase);
				const bool ln = lnil(rl, vlo), hn = lnil(rh, vhi);
				int m = between3(v, false, vlo, ln, linc, vhi, hn, hinc);
				if (symmetric) {
					const int m2 = between3(v, false, vhi, hn, hinc, vlo, ln, linc);
					m = m == 1 || m2 == 1 ? 1 : (m < 0 || m2 < 0 ? -1 : 0);
				}
				if (anti)
					m = m < 0 ? -1 : !m;
				if (m == 1)
					ADD(lo, ro);
			}
		}
	}
#undef ADD
done:
	pair_out(r1p, r2p, a, b, n);
	free(a);
	free(b);
	oid_props(*r1p);
	oid_props(*r2p);
	return 0;
}

/* ---- leftjoin's algorithm choice and the order of several matches --------
 * (gdk/gdk_join.c:4049-4300).  What a left candidate's matches are does not
 * depend on the algorithm; their ORDER, which one a semi join with a right
 * output keeps, and a few quirks do:
 *   selectjoin (:363-563; one left candidate or all left values equal): the
 *     matches ascending (a point BATselect), semi keeps the first; max_one ->
 *     "more than one match", min_one (BATouterjoin's match_one) -> "not enough
 *     matches" on a miss (:399-404, the only path that raises it);
 *   mergejoin_void (:571), fetchjoin (:3893), bitmaskjoin (:3956): at most one
 *     match per left candidate; fetchjoin returns the pairs in RIGHT position
 *     order (r1 descends when r is reverse sorted) and, reached without a
 *     check of nil_on_miss (:4156-4168), no nil rows for misses;
 *   mergejoin (:1941-2780): the matches ascending (:2651-2683 emits a run
 *     forwards in both scan directions); semi keeps the LAST of the run when
 *     l and r are scanned in the same order (equal_order, :2091-2107: also
 *     when l is not ordered) -- rci already points past the run and the copy
 *     steps back by nr = 1 (:2661-2668) -- else the first; a sorted l's nil
 *     values are skipped before the scan when neither nil_matches nor
 *     nil_on_miss is set (:2093-2100), so BATdiff does not list them;
 *   hashjoin (:2900-3335): the matches in hash-chain order, DESCENDING
 *     position (chains are built by prepending); semi keeps the first of the
 *     chain, i.e. the last position;
 *   swapped hashjoin (:4203-4295; leftjoin / semi without max_one when
 *     joincost prefers hashing l): the pairs of hashjoin(r, l) -- right
 *     candidates in order, each one's left matches descending -- then r1 / r2
 *     sorted by GDKqsort on r1 (unstable, :4236-4251); semi first reduces the
 *     right side to BATunique (first occurrence of each value, gdk_unique.c),
 *     so every left candidate keeps its FIRST match.
 * mergejoin's memory-pressure term (:4185, BATcount(r) * width >
 * GDK_mem_maxsize / nthreads) depends on the host and is taken as false.
 * BATmarkjoin's reference quirks (the mark column of selectjoin has one row
 * per left candidate whatever the match count, :513-527; fetchjoin returns no
 * mark column) are not reproduced: the marks are one per result row. */

/* BATtvoid (gdk.h): dense or void */
static bool
tvoid(const ora_bat *b)
{
	return tdense(b) || b->type == ORA_void;
}

static int
lj_algo(ora_bat *l, ora_bat *r, const ora_bat *sl, const ora_bat *sr, const ora_ci *lci, const ora_ci *rci,
	bool nil_matches, bool nil_on_miss, bool semi, bool only_misses, bool not_in, bool max_one, bool min_one,
	bool want_r2, bool *equal_order)
{
	*equal_order = true;
	if (lci->n == 0 || rci->n == 0)
		return LJ_NOMATCH;
	if (!only_misses && !not_in &&
	    (lci->n == 1 || (ordered(l) && ordered_rev(l)) || (l->type == ORA_void && l->tseqbase == ORA_OID_NIL)))
		return LJ_SELECT;
	if (tdense(r) && rci->dense)
		return LJ_MJVOID;
	if (tdense(l) && lci->dense && rci->dense && !semi && !max_one && !min_one && !nil_matches && !only_misses &&
	    !not_in && (ordered(r) || ordered_rev(r)))
		return LJ_FETCH;
	if (tdense(l) && lci->dense && !want_r2 && (semi || only_misses) && !nil_on_miss && !not_in && !max_one &&
	    !min_one)
		return LJ_BITMASK;
	if ((ordered(r) || ordered_rev(r)) && (ordered(l) || ordered_rev(l) || tdense(r) || lci->n < 1024)) {
		if (l->sorted || l->revsorted)
			*equal_order = (l->sorted && r->sorted) ||
				(l->revsorted && r->revsorted && !tvoid(l) && !tvoid(r));
		return LJ_MERGE;
	}
	const double rcost = joincost(r, lci->n, rci, sr);
	if (!nil_on_miss && !only_misses && !not_in && !max_one && !min_one) {
		double lcost = joincost(l, rci->n, lci, sl);
		if (semi && !r->key)
			lcost += rci->n;
		lcost += rci->n * log((double) rci->n);
		if (lcost < rcost)
			return LJ_SWAP;
	}
	return LJ_HASH;
}

typedef struct {
	ora_oid *a, *b;
	int8_t *m;
	uint64_t n, cap;
} ljrows;

static int
ljrows_add(ljrows *R, ora_oid x, ora_oid y, int8_t m)
{
	if (R->n == R->cap) {
		uint64_t c = R->cap ? R->cap * 2 : 1024;
		ora_oid *na = realloc(R->a, c * 8), *nb = realloc(R->b, c * 8);
		int8_t *nm = realloc(R->m, c);
		if (na)
			R->a = na;
		if (nb)
			R->b = nb;
		if (nm)
			R->m = nm;
		if (!na || !nb || !nm) {
			ora_seterr("out of memory");
			return -1;
		}
		R->cap = c;
	}
	R->a[R->n] = x;
	R->b[R->n] = y;
	R->m[R->n] = m;
	R->n++;
	return 0;
}

/* the swapped hash join's rows (see above): r1 / r2 of the pairs in
 * hashjoin(r, l)'s order, then GDKqsort on r1 with r2 as payload */
static int
lj_swapped(ljrows *R, ora_bat *l, ora_bat *r, const ora_ci *lci, const ora_ci *rci, bool nil_matches, bool semi)
{
	bool lnil_any;
	vpair *lp = rpairs(l, lci, &lnil_any);          /* l's candidates by (value, oid) */
	if (lp == NULL)
		return -1;
	/* semi and r not known key: BATunique(r, sr), the first candidate of
	 * every distinct value */
	int64_t *seen = NULL;
	uint64_t nseen = 0;
	if (semi && !r->key) {
		seen = malloc((rci->n + 1) * sizeof(int64_t));
		if (seen == NULL) {
			free(lp);
			ora_seterr("malloc");
			return -1;
		}
	}
	pairs P = {0};
	const int64_t rn = jnilv(r->type);
	for (uint64_t j = 0; j < rci->n; j++) {
		const ora_oid ro = ci_get(rci, j);
		const int64_t v = jv(r, ro - r->hseqbase);
		if (seen) {
			/* a value seen before is not in BATunique's list */
			uint64_t a = 0, b = nseen;
			while (a < b) {
				uint64_t m = (a + b) / 2;
				if (seen[m] < v)
					a = m + 1;
				else
					b = m;
			}
			if (a < nseen && seen[a] == v)
				continue;
			memmove(seen + a + 1, seen + a, (nseen - a) * sizeof(int64_t));
			seen[a] = v;
			nseen++;
		}
		const bool isnil = r->type == ORA_void ? r->tseqbase == ORA_OID_NIL : v == rn;
		if (isnil && !nil_matches)
			continue;
		uint64_t a = vlower(lp, lci->n, v), b = a;
		while (b < lci->n && lp[b].v == v)
			b++;
		for (uint64_t k = b; k > a; k--)          /* descending left position */
			if (pairs_add(&P, lp[k - 1].o, ro) < 0) {
				free(lp);
				free(seen);
				free(P.a);
				free(P.b);
				return -1;
			}
	}
	free(lp);
	free(seen);
	if (P.n > 1) {
		ora_bat *v = ora_new(ORA_oid, P.n, 0);
		uint64_t *h = malloc(P.n * sizeof(uint64_t));
		if (v == NULL || h == NULL) {
			ora_free(v);
			free(h);
			free(P.a);
			free(P.b);
			ora_seterr("malloc");
			return -1;
		}
		memcpy(v->base, P.a, P.n * 8);
		for (uint64_t k = 0; k < P.n; k++)
			h[k] = k;
		ora_GDKqsort(v, h, P.b, P.n, false, false);
		for (uint64_t k = 0; k < P.n; k++)
			P.a[k] = ((const ora_oid *) v->base)[h[k]];
		ora_free(v);
		free(h);
	}
	int rc = 0;
	for (uint64_t k = 0; k < P.n && rc == 0; k++)
		rc = ljrows_add(R, P.a[k], P.b[k], 1);
	free(P.a);
	free(P.b);
	return rc;
}

/* leftjoin (gdk_join.c:4049) for the outputs with a right (or mark) column:
 * BATleftjoin (nil_on_miss false, semi false), BATouterjoin (nil_on_miss,
 * match_one = max_one = min_one), BATsemijoin with r2p (semi, max_one),
 * BATmarkjoin (nil_on_miss; semi when r2p is NULL; r3p set).  *algo: the
 * LJ_* branch taken (tests check the shapes they mean to cover). */
int
ora_leftjoin_ex(ora_bat **r1p, ora_bat **r2p, ora_bat **r3p, ora_bat *l, ora_bat *r, const ora_bat *sl,
		const ora_bat *sr, bool nil_matches, bool nil_on_miss, bool semi, bool max_one, bool min_one,
		int *algo)
{
	*r1p = NULL;
	if (r2p)
		*r2p = NULL;
	if (r3p)
		*r3p = NULL;
	if (l->type == ORA_msk || r->type == ORA_msk) {
		ora_bat *lm = l->type == ORA_msk ? ora_unmask(l) : NULL;
		ora_bat *rm = r->type == ORA_msk ? ora_unmask(r) : NULL;
		int rc = -1;
		if ((l->type != ORA_msk || lm) && (r->type != ORA_msk || rm))
			rc = ora_leftjoin_ex(r1p, r2p, r3p, lm ? lm : l, rm ? rm : r, sl, sr, nil_matches, nil_on_miss, semi,
					     max_one, min_one, algo);
		ora_free(lm);
		ora_free(rm);
		return rc;
	}
	if (atomtype(l->type) != atomtype(r->type)) {
		ora_seterr("leftjoin: inputs not compatible.");
		return -1;
	}
	if (l->type == ORA_str) {
		ora_bat *li, *ri;
		if (str_images(l, r, &li, &ri) < 0)
			return -1;
		int rc = ora_leftjoin_ex(r1p, r2p, r3p, li, ri, sl, sr, nil_matches, nil_on_miss, semi, max_one,
					 min_one, algo);
		str_flags_back(l, r, li, ri);
		return rc;
	}
	if (!join_type_ok(l->type) || !join_type_ok(r->type)) {
		ora_seterr("leftjoin: type not restated");
		return -1;
	}
	ora_ci lci, rci;
	if (ora_ci_init(&lci, l, sl) < 0 || ora_ci_init(&rci, r, sr) < 0)
		return -1;
	const bool want_r2 = r2p != NULL;
	bool eqo;
	const int a = lj_algo(l, r, sl, sr, &lci, &rci, nil_matches, nil_on_miss, semi, false, false, max_one, min_one,
			      want_r2, &eqo);
	if (algo)
		*algo = a;
	ljrows R = {0};
	bool rnil = false;
	vpair *p = rci.n ? rpairs(r, &rci, &rnil) : NULL;
	if (rci.n && p == NULL) {
		ora_seterr("malloc");
		return -1;
	}
	int rc = 0;
	if (a == LJ_NOMATCH) {
		/* nomatch (:301-360): the misses with nil (defmark 0, leftjoin :4144) */
		for (uint64_t i = 0; nil_on_miss && i < lci.n && rc == 0; i++)
			rc = ljrows_add(&R, ci_get(&lci, i), ORA_OID_NIL, 0);
	} else if (a == LJ_SWAP) {
		rc = lj_swapped(&R, l, r, &lci, &rci, nil_matches, semi);
	} else {
		/* fetchjoin's rows leave in right position order: with r reverse
		 * sorted the left candidates come out descending */
		const bool rev = a == LJ_FETCH && !r->sorted;
		for (uint64_t ii = 0; ii < lci.n && rc == 0; ii++) {
			const uint64_t i = rev ? lci.n - 1 - ii : ii;
			const ora_oid lo = ci_get(&lci, i);
			const int64_t v = jv(l, lo - l->hseqbase);
			const bool isnil = lnil(l, v);
			uint64_t lo_ = 0, hi_ = 0;
			if (!(isnil && !nil_matches)) {
				lo_ = vlower(p, rci.n, v);
				hi_ = lo_;
				while (hi_ < rci.n && p[hi_].v == v)
					hi_++;
			}
			const uint64_t cnt = hi_ - lo_;
			if (cnt > 1 && max_one) {
				ora_seterr("more than one match");
				rc = -1;
				break;
			}
			if (cnt == 0) {
				if (a == LJ_SELECT && min_one && !(isnil && !nil_matches)) {
					ora_seterr("not enough matches");
					rc = -1;
					break;
				}
				if (nil_on_miss && a != LJ_FETCH)
					rc = ljrows_add(&R, lo, ORA_OID_NIL, (int8_t) (isnil || rnil ? INT8_MIN : 0));
				continue;
			}
			if (semi) {
				const bool last = a == LJ_HASH || (a == LJ_MERGE && eqo);
				rc = ljrows_add(&R, lo, p[last ? hi_ - 1 : lo_].o, 1);
				continue;
			}
			if (a == LJ_HASH) {
				for (uint64_t k = hi_; k > lo_ && rc == 0; k--)
					rc = ljrows_add(&R, lo, p[k - 1].o, 1);
			} else {
				for (uint64_t k = lo_; k < hi_ && rc == 0; k++)
					rc = ljrows_add(&R, lo, p[k].o, 1);
			}
		}
	}
	free(p);
	if (rc < 0) {
		free(R.a);
		free(R.b);
		free(R.m);
		return -1;
	}
	ora_bat *x = oidbat(R.a, R.n), *y = oidbat(R.b, R.n), *z = r3p ? ora_new(ORA_bit, R.n, 0) : NULL;
	if (x == NULL || y == NULL || (r3p && z == NULL)) {
		ora_free(x);
		ora_free(y);
		ora_free(z);
		free(R.a);
		free(R.b);
		free(R.m);
		return -1;
	}
	bool ynil = false, znil = false;
	for (uint64_t k = 0; k < R.n; k++) {
		ynil |= R.b[k] == ORA_OID_NIL;
		znil |= R.m[k] == INT8_MIN;
	}
	if (z) {
		memcpy(z->base, R.m, R.n);
		z->nil = znil;
		z->nonil = !znil;
	}
	adj a1 = adjacent(R.a, R.n);
	free(R.a);
	free(R.b);
	free(R.m);
	x->sorted = !a1.desc;
	x->revsorted = !a1.asc;
	x->key = !a1.eq;
	y->nil = ynil;
	y->nonil = !ynil;
	y->sorted = y->revsorted = y->key = R.n <= 1;
	if (semi && x->sorted && x->key)
		virtualize(x);
	*r1p = x;
	if (r2p)
		*r2p = y;
	else
		ora_free(y);
	if (r3p)
		*r3p = z;
	return 0;
}

/* ---- cross products (gdk/gdk_cross.c) ---------------------------------- */

/* canditer_slice (gdk_cand.c): all candidates, hseqbase 0; void when dense */
static ora_bat *
cross_slice(const ora_ci *ci)
{
	if (ci->dense)
		return ora_dense(0, ci->seq, ci->n);
	ora_bat *b = ora_new(ORA_oid, ci->n, 0);
	if (b == NULL)
		return NULL;
	for (uint64_t i = 0; i < ci->n; i++)
		((ora_oid *) b->base)[i] = ci->oids[i];
	b->sorted = b->key = b->nonil = 1;
	b->revsorted = ci->n <= 1;
	return b;
}

/* BATconstant (gdk_bat.c) of an oid */
static ora_bat *
cross_const(ora_oid v, uint64_t n)
{
	ora_bat *b = ora_new(ORA_oid, n, 0);
	if (b == NULL)
		return NULL;
	for (uint64_t i = 0; i < n; i++)
		((ora_oid *) b->base)[i] = v;
	b->sorted = b->revsorted = b->nonil = 1;
	b->key = n <= 1;
	return b;
}

/* a void column of n nil oids (BATtseqbase(bn, oid_nil), gdk_bat.c:2167) */
static ora_bat *
cross_nilvoid(uint64_t n)
{
	ora_bat *b = ora_dense(0, ORA_OID_NIL, n);
	if (b == NULL)
		return NULL;
	b->sorted = b->revsorted = 1;
	b->key = n <= 1;
	b->nonil = n == 0;
	b->nil = n > 0;
	return b;
}

/* BATcrossci (gdk_cross.c:22) */
static int
cross_ci(ora_bat **r1p, ora_bat **r2p, const ora_ci *c1, const ora_ci *c2)
{
	ora_bat *a = NULL, *b = NULL;
	if (c1->n == 0 || c2->n == 0) {
		a = ora_dense(0, 0, 0);
		if (r2p)
			b = ora_dense(0, 0, 0);
	} else if (c2->n == 1) {
		a = cross_slice(c1);
		if (r2p)
			b = c1->n == 1 ? cross_slice(c2) : cross_const(ci_get(c2, 0), c1->n);
	} else if (c1->n == 1) {
		a = cross_const(ci_get(c1, 0), c2->n);
		if (r2p)
			b = cross_slice(c2);
	} else {
		uint64_t n = c1->n * c2->n, p = 0;
		a = ora_new(ORA_oid, n, 0);
		if (r2p)
			b = ora_new(ORA_oid, n, 0);
		if (a && (b || !r2p)) {
			/* :95-101 left oid repeated, :112-118 the right list again per left */
			for (uint64_t i = 0; i < c1->n; i++)
				for (uint64_t j = 0; j < c2->n; j++, p++) {
					((ora_oid *) a->base)[p] = ci_get(c1, i);
					if (b)
						((ora_oid *) b->base)[p] = ci_get(c2, j);
				}
			a->sorted = a->nonil = 1;
			a->revsorted = a->key = 0;
			if (b) {
				b->nonil = 1;
				b->sorted = b->revsorted = b->key = 0;
			}
		}
	}
	if (a == NULL || (r2p && b == NULL)) {
		ora_free(a);
		ora_free(b);
		ora_seterr("malloc");
		return -1;
	}
	*r1p = a;
	if (r2p)
		*r2p = b;
	return 0;
}

/* BATsubcross (gdk_cross.c:138); outer: BAToutercross (:153) */
int
ora_crossproduct(ora_bat **r1p, ora_bat **r2p, const ora_bat *l, const ora_bat *r, const ora_bat *sl,
		 const ora_bat *sr, bool max_one, bool outer)
{
	ora_ci c1, c2;
	if (ora_ci_init(&c1, l, sl) < 0 || ora_ci_init(&c2, r, sr) < 0)
		return -1;
	if (max_one && c1.n > 0 && c2.n > 1) {
		ora_seterr("more than one match");
		return -1;
	}
	if (outer && (c1.n == 0 || c2.n == 0)) {
		ora_bat *a = c1.n == 0 ? cross_nilvoid(0) : cross_slice(&c1), *b = NULL;
		if (a == NULL || (r2p && (b = cross_nilvoid(c1.n)) == NULL)) {
			ora_free(a);
			ora_seterr("malloc");
			return -1;
		}
		*r1p = a;
		if (r2p)
			*r2p = b;
		return 0;
	}
	return cross_ci(r1p, r2p, &c1, &c2);
}

/* BATguess_uniques (gdk_join.c:3572): guess_uniques over b's candidates s
 * (NULL: all of b) */
uint64_t
ora_guess_uniques(ora_bat *b, const ora_bat *s)
{
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return 0;
	return (uint64_t) guess_uniques(b, &ci, s);
}
