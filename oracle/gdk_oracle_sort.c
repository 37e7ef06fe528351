/*
 * gdk_oracle_sort.c -- CPU restatement of BATsort (gdk/gdk_batop.c:2342-2827)
 * with the reference's choice of sort function per sorted run (do_sort,
 * gdk_batop.c:2266-2304) and an exact restatement of GDKqsort
 * (gdk/gdk_qsort.c:17-524, gdk/gdk_qsort_impl.h:56-204: Bentley & McIlroy's
 * three-way quicksort), whose order of equal values is what an unstable
 * BATsort returns.  TEST INFRASTRUCTURE ONLY (see gdk_oracle.h).
 *
 * Not restated: the persistent order index (gdk_batop.c:2488-2572, 2716-2766)
 * -- a transient BAT reaches it only after a previous sort of the same BAT
 * created one, which the device does not keep either.
 */
#include "gdk_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

void ora_seterr(const char *fmt, ...);
ora_bat *ora_dense(ora_oid hseq, ora_oid tseq, uint64_t cnt);

/* elements are positions into the values v (bn's tail); the payload t holds
 * the order oids; SWAP moves both (the values move with their positions) */
typedef struct {
	const ora_bat *v;     /* values */
	int bt;               /* storage type deciding the comparison */
	bool reverse, nilslast;
	uint64_t *h;          /* positions being sorted */
	ora_oid *t;           /* payload (NULL: none) */
} sctx;

static int
storage(int tt)
{
	switch (tt) {
	case ORA_bit: return ORA_bte;
	case ORA_date: return ORA_int;
	case ORA_oid: case ORA_daytime: case ORA_timestamp: return ORA_lng;
	default: return tt;
	}
}

static const char *
str_at(const ora_bat *b, uint64_t p)
{
	const char *x = (const char *) b->base + p * b->width;
	uint64_t o;
	switch (b->width) {
	case 1: o = *(const uint8_t *) x + 8192u; break;
	case 2: o = *(const uint16_t *) x + 8192u; break;
	case 4: o = *(const uint32_t *) x; break;
	default: o = *(const uint64_t *) x; break;
	}
	return b->vheap + o;
}

static bool
nil_at(const sctx *c, uint64_t p)
{
	const char *x = (const char *) c->v->base + p * c->v->width;
	switch (c->bt) {
	case ORA_bte: return *(const int8_t *) x == INT8_MIN;
	case ORA_sht: return *(const int16_t *) x == INT16_MIN;
	case ORA_int: return *(const int32_t *) x == INT32_MIN;
	case ORA_lng: return *(const int64_t *) x == INT64_MIN;
	case ORA_hge: return *(const ora_hge *) x == (ora_hge) ((unsigned __int128) 1 << 127);
	case ORA_flt: return isnan(*(const float *) x);
	case ORA_dbl: return isnan(*(const double *) x);
	case ORA_str: {
		const char *s = str_at(c->v, p);
		return (uint8_t) s[0] == 0x80 && s[1] == 0;
	}
	}
	return false;
}

/* three-way comparison of two non-nil values (strCmp = strcmp's unsigned
 * byte order for non-nil strings) */
static int
vcmp(const sctx *c, uint64_t p, uint64_t q)
{
	const char *x = (const char *) c->v->base + p * c->v->width;
	const char *y = (const char *) c->v->base + q * c->v->width;
#define C3(T) { T a, b; memcpy(&a, x, sizeof(T)); memcpy(&b, y, sizeof(T)); return (a > b) - (a < b); }
	switch (c->bt) {
	case ORA_bte: C3(int8_t)
	case ORA_sht: C3(int16_t)
	case ORA_int: C3(int32_t)
	case ORA_lng: C3(int64_t)
	case ORA_hge: C3(ora_hge)
	case ORA_flt: C3(float)
	case ORA_dbl: C3(double)
	case ORA_str: {
		int r = strcmp(str_at(c->v, p), str_at(c->v, q));
		return (r > 0) - (r < 0);
	}
	}
#undef C3
	return 0;
}

/* LT of the four comparator families (gdk_qsort.c:29-166): "i sorts
 * strictly before j" in the requested direction, nils at the front (f,
 * f_rev) or the back (l, l_rev) */
static bool
LT(const sctx *c, size_t i, size_t j)
{
	const uint64_t p = c->h[i], q = c->h[j];
	const bool ni = nil_at(c, p), nj = nil_at(c, q);
	if (ni || nj) {
		if (ni && nj)
			return false;
		return c->nilslast ? nj : ni;
	}
	const int r = vcmp(c, p, q);
	return c->reverse ? r > 0 : r < 0;
}

static bool
LE(const sctx *c, size_t i, size_t j)
{
	return !LT(c, j, i);
}

static bool
EQ(const sctx *c, size_t i, size_t j)
{
	const uint64_t p = c->h[i], q = c->h[j];
	const bool ni = nil_at(c, p), nj = nil_at(c, q);
	if (ni || nj)
		return ni && nj;
	return vcmp(c, p, q) == 0;
}

static void
SWAP(const sctx *c, size_t i, size_t j)
{
	uint64_t x = c->h[i];
	c->h[i] = c->h[j];
	c->h[j] = x;
	if (c->t) {
		ora_oid y = c->t[i];
		c->t[i] = c->t[j];
		c->t[j] = y;
	}
}

static size_t
MED3(const sctx *c, size_t a, size_t b, size_t d)
{
	return LT(c, a, b) ? (LT(c, b, d) ? b : (LT(c, a, d) ? d : a))
			   : (LT(c, d, b) ? b : (LT(c, a, d) ? a : d));
}

static void
insertion(const sctx *c, size_t n)
{
	for (size_t b = 1; b < n; b++)
		for (size_t a = b; a > 0 && LT(c, a, a - 1); a--)
			SWAP(c, a, a - 1);
}

#define INSERTSORT 60

/* GDKqsort_impl (gdk_qsort_impl.h:61-204) on c->h[0..n), c->t[0..n) */
static void
qsort_impl(sctx c, size_t n)
{
	size_t a, b, cc, d, r;
	bool swap_cnt;
loop:
	if (n < INSERTSORT) {
		insertion(&c, n);
		return;
	}
	/* pivot: median of three medians of three (INSERTSORT > 40) */
	b = n >> 1;
	a = 0;
	cc = n - 1;
	d = n >> 3;
	a = MED3(&c, a, a + d, a + 2 * d);
	b = MED3(&c, b - d, b, b + d);
	cc = MED3(&c, cc - 2 * d, cc - d, cc);
	b = MED3(&c, a, b, cc);
	if (b != 0)
		SWAP(&c, 0, b);
	/* Dijkstra's Dutch national flag, Bentley & McIlroy's way */
	a = b = 1;
	cc = d = n - 1;
	swap_cnt = false;
	for (;;) {
		while (b <= cc && LE(&c, b, 0)) {
			if (EQ(&c, b, 0)) {
				swap_cnt = true;
				SWAP(&c, a, b);
				a++;
			}
			b++;
		}
		while (b <= cc && LE(&c, 0, cc)) {
			if (EQ(&c, 0, cc)) {
				swap_cnt = true;
				SWAP(&c, cc, d);
				d--;
			}
			cc--;
		}
		if (b > cc)
			break;
		SWAP(&c, b, cc);
		swap_cnt = true;
		b++;
		cc--;
	}
	if (!swap_cnt && n < 1024) {
		insertion(&c, n);
		return;
	}
	r = a < b - a ? a : b - a;
	for (size_t k = 0; k < r; k++)
		SWAP(&c, k, b - r + k);
	r = d - cc < n - d - 1 ? d - cc : n - d - 1;
	for (size_t k = 0; k < r; k++)
		SWAP(&c, b + k, n - r + k);
	if (b - a < d - cc) {
		if ((r = b - a) > 1)
			qsort_impl(c, r);
		if ((r = d - cc) > 1) {
			c.h += n - r;
			if (c.t)
				c.t += n - r;
			n = r;
			goto loop;
		}
	} else {
		if ((r = d - cc) > 1) {
			sctx c2 = c;
			c2.h += n - r;
			if (c2.t)
				c2.t += n - r;
			qsort_impl(c2, r);
		}
		if ((r = b - a) > 1) {
			n = r;
			goto loop;
		}
	}
}

/* GDKrsort / GDKssort / GDKssort_rev: stable sorts, so any stable merge
 * gives their permutation */
static void
stable_sort(sctx *c, size_t n)
{
	uint64_t *th = malloc(n * sizeof(uint64_t));
	ora_oid *tt = c->t ? malloc(n * sizeof(ora_oid)) : NULL;
	for (size_t w = 1; w < n; w *= 2) {
		for (size_t lo = 0; lo < n; lo += 2 * w) {
			size_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
			size_t i = lo, j = mid, k = lo;
			while (i < mid || j < hi) {
				bool takej = i >= mid || (j < hi && LT(c, j, i));
				size_t s = takej ? j++ : i++;
				th[k] = c->h[s];
				if (tt)
					tt[k] = c->t[s];
				k++;
			}
		}
		memcpy(c->h, th, n * sizeof(uint64_t));
		if (tt)
			memcpy(c->t, tt, n * sizeof(ora_oid));
	}
	free(th);
	free(tt);
}

/* do_sort (gdk_batop.c:2266-2304): the LSD radix sort for integer-like
 * types when nils are at their natural end and the sort is stable or longer
 * than 100 values, a stable merge sort when stable is asked, GDKqsort
 * otherwise */
static void
do_sort(sctx *c, size_t n, int tt, bool stable)
{
	if (n <= 1)
		return;
	bool radix = false;
	switch (tt) {
	case ORA_bte: case ORA_sht: case ORA_int: case ORA_lng: case ORA_hge:
	case ORA_date: case ORA_daytime: case ORA_timestamp:
		radix = c->nilslast == c->reverse && (stable || n > 100);
		break;
	default:
		break;
	}
	if (radix || stable)
		stable_sort(c, n);
	else
		qsort_impl(*c, n);
}

static ora_bat *
copy_bat(const ora_bat *b, ora_oid hseq)
{
	ora_bat *bn = ora_new(b->type == ORA_void ? ORA_oid : b->type, b->count, hseq);
	if (bn == NULL)
		return NULL;
	bn->width = b->type == ORA_void ? 8 : b->width;
	if (b->type == ORA_void) {
		for (uint64_t i = 0; i < b->count; i++)
			((ora_oid *) bn->base)[i] = b->tseqbase == ORA_OID_NIL ? ORA_OID_NIL : b->tseqbase + i;
	} else {
		free(bn->base);
		bn->base = malloc(b->count * b->width + 16);
		memcpy(bn->base, b->base, b->count * b->width);
	}
	if (b->vheap) {
		bn->vheap = malloc(b->vheapsize);
		memcpy(bn->vheap, b->vheap, b->vheapsize);
		bn->vheapsize = b->vheapsize;
	}
	bn->sorted = b->sorted;
	bn->revsorted = b->revsorted;
	bn->key = b->key;
	bn->nonil = b->nonil;
	bn->nil = b->nil;
	return bn;
}

static ora_bat *
constant_oid(ora_oid hseq, ora_oid v, uint64_t n)
{
	ora_bat *bn = ora_new(ORA_oid, n, hseq);
	if (bn == NULL)
		return NULL;
	for (uint64_t i = 0; i < n; i++)
		((ora_oid *) bn->base)[i] = v;
	bn->sorted = bn->revsorted = 1;
	bn->key = n <= 1;
	bn->nonil = 1;
	return bn;
}

static ora_oid
oid_of(const ora_bat *b, uint64_t i)
{
	if (b->type == ORA_void)
		return b->tseqbase == ORA_OID_NIL ? ORA_OID_NIL : b->tseqbase + i;
	return ((const ora_oid *) b->base)[i];
}

/* BATgroup_internal(.., bn, NULL, g, NULL, NULL, subsorted = true)
 * (gdk_group.c:712-802, 940-975): consecutive values compared */
static ora_bat *
sort_groups(const sctx *c, const ora_bat *bn, const ora_bat *g)
{
	const uint64_t n = bn->count;
	if (bn->key || n <= 1 || (g && (g->key || g->type == ORA_void)))
		return ora_dense(bn->hseqbase, 0, n);
	ora_bat *gn = ora_new(ORA_oid, n, bn->hseqbase);
	if (gn == NULL)
		return NULL;
	ora_oid ngrp = 0;
	for (uint64_t i = 0; i < n; i++) {
		bool nw = i == 0 || (g && oid_of(g, i) != oid_of(g, i - 1));
		if (!nw) {
			const bool ni = nil_at(c, i), nj = nil_at(c, i - 1);
			nw = (ni || nj) ? !(ni && nj) : vcmp(c, i, i - 1) != 0;
		}
		if (nw)
			ngrp++;
		((ora_oid *) gn->base)[i] = ngrp - 1;
	}
	gn->sorted = 1;
	gn->revsorted = ngrp == 1 || n <= 1;
	gn->key = ngrp == n;
	gn->nonil = 1;
	return gn;
}

int
ora_BATsort(ora_bat **sorted, ora_bat **order, ora_bat **groups, ora_bat *b, const ora_bat *o,
	    const ora_bat *g, bool reverse, bool nilslast, bool stable)
{
	if (sorted) *sorted = NULL;
	if (order) *order = NULL;
	if (groups) *groups = NULL;
	if (b == NULL) {
		ora_seterr("b must exist\n");
		return -1;
	}
	if (stable && reverse != nilslast) {
		ora_seterr("stable sort cannot have reverse != nilslast\n");
		return -1;
	}
	const uint64_t n = b->count;
	if (b->type == ORA_void) {
		b->sorted = 1;
		b->revsorted = b->tseqbase == ORA_OID_NIL || n <= 1;
		b->key = b->tseqbase != ORA_OID_NIL || n <= 1;
	} else if (n <= 1) {
		b->sorted = b->revsorted = 1;
	}
	if (o && ((o->type != ORA_oid && o->type != ORA_void) || o->count != n ||
		  (o->type == ORA_void && o->count && o->tseqbase == ORA_OID_NIL))) {
		ora_seterr("o must have type oid and same size as b\n");
		return -1;
	}
	if (g && ((g->type != ORA_oid && g->type != ORA_void) || !g->sorted || g->count != n ||
		  (g->type == ORA_void && g->count && g->tseqbase == ORA_OID_NIL))) {
		ora_seterr("g must have type oid, sorted on the tail, and same size as b\n");
		return -1;
	}
	if (sorted == NULL && order == NULL) {
		ora_seterr("no place to put the result.\n");
		return -1;
	}
	if (g == NULL && !stable)
		o = NULL;
	if (b->nonil)
		nilslast = reverse;
	/* trivially (sub)sorted (:2422-2472) */
	if (n <= 1 || (reverse == nilslast && (reverse ? b->revsorted : b->sorted) && o == NULL && g == NULL &&
		       (groups == NULL || b->key || (reverse ? b->sorted : b->revsorted)))) {
		if (sorted && (*sorted = copy_bat(b, b->hseqbase)) == NULL)
			goto oom;
		if (order && (*order = ora_dense(b->hseqbase, b->hseqbase, n)) == NULL)
			goto oom;
		if (groups) {
			*groups = b->key ? ora_dense(b->hseqbase, 0, n) : constant_oid(b->hseqbase, 0, n);
			if (*groups == NULL)
				goto oom;
		}
		return 0;
	}
	ora_bat *bn = o ? ora_project(o, b) : copy_bat(b, b->hseqbase);
	if (bn == NULL)
		return -1;
	ora_bat *on = NULL;
	if (order) {
		on = ora_new(ORA_oid, n, b->hseqbase);
		if (on == NULL) {
			ora_free(bn);
			goto oom;
		}
		for (uint64_t p = 0; p < n; p++)
			((ora_oid *) on->base)[p] = o ? oid_of(o, p) : b->hseqbase + p;
		on->key = o ? o->key : 1;
		on->nonil = 1;
		on->sorted = on->revsorted = 0;   /* :2622-2627 */
	}
	uint64_t *pos = malloc((n + 1) * sizeof(uint64_t));
	for (uint64_t p = 0; p < n; p++)
		pos[p] = p;
	sctx c = {.v = bn, .bt = storage(bn->type), .reverse = reverse, .nilslast = nilslast,
		  .h = pos, .t = on ? on->base : NULL};
	if (g) {
		if (g->key || g->type == ORA_void) {
			/* every group a single row: nothing to sort (:2634-2686) */
			if (on) {
				on->sorted = o ? o->sorted : 1;
				on->revsorted = o ? o->revsorted : 0;
				if (n <= 1)
					on->sorted = on->revsorted = 1;
			}
			free(pos);
			if (groups) {
				*groups = copy_bat(g, g->hseqbase);
				if (*groups == NULL) {
					ora_free(bn);
					ora_free(on);
					goto oom;
				}
			}
			if (sorted) *sorted = bn; else ora_free(bn);
			if (order) *order = on;
			return 0;
		}
		uint64_t r = 0, p;
		for (p = 1; p < n; p++) {
			if (oid_of(g, p) != oid_of(g, p - 1)) {
				sctx s = c;
				s.h += r;
				if (s.t)
					s.t += r;
				do_sort(&s, p - r, bn->type, stable);
				r = p;
			}
		}
		sctx s = c;
		s.h += r;
		if (s.t)
			s.t += r;
		do_sort(&s, p - r, bn->type, stable);
		bn->sorted = r == 0 && !reverse && !nilslast;
		bn->revsorted = r == 0 && reverse && nilslast;
	} else {
		if (reverse != nilslast || (reverse ? !bn->revsorted : !bn->sorted))
			do_sort(&c, n, bn->type, stable);
		bn->sorted = !reverse && !nilslast;
		bn->revsorted = reverse && nilslast;
	}
	/* the values follow their positions */
	if (n) {
		char *nb = malloc(n * bn->width + 16);
		for (uint64_t p = 0; p < n; p++)
			memcpy(nb + p * bn->width, (const char *) bn->base + pos[p] * bn->width, bn->width);
		free(bn->base);
		bn->base = nb;
	}
	free(pos);
	bn->minpos = bn->maxpos = ORA_BUN_NONE;
	if (groups) {
		sctx gc = {.v = bn, .bt = storage(bn->type)};
		ora_bat *gn = sort_groups(&gc, bn, g);
		if (gn == NULL) {
			ora_free(bn);
			ora_free(on);
			goto oom;
		}
		if (gn->key && (g == NULL || (g->sorted && g->revsorted)))
			bn->key = 1;
		*groups = gn;
	}
	if (sorted) *sorted = bn; else ora_free(bn);
	if (order) *order = on;
	return 0;
oom:
	if (sorted) { ora_free(*sorted); *sorted = NULL; }
	if (order) { ora_free(*order); *order = NULL; }
	if (groups) { ora_free(*groups); *groups = NULL; }
	ora_seterr("out of memory");
	return -1;
}

/* GDKqsort on its own (gdk_qsort.c:358-524) for the tests: sorts the
 * positions of v (h: the positions, t: payload oids) */
void
ora_GDKqsort(const ora_bat *v, uint64_t *h, ora_oid *t, uint64_t n, bool reverse, bool nilslast)
{
	sctx c = {.v = v, .bt = storage(v->type), .reverse = reverse, .nilslast = nilslast, .h = h, .t = t};
	if (n > 1)
		qsort_impl(c, n);
}
