/*
 * gdk_oracle_firstn.c -- CPU restatement of GDK's plain first-N
 * (BATfirstn without group ids and without distinct): the binary-heap
 * algorithm whose choice among rows tied with the n-th value is part of
 * the result.  TEST INFRASTRUCTURE ONLY (see gdk_oracle.h).
 *
 * Follows gdk/gdk_firstn.c (reference v11.52.0):
 *   siftdown / heapify          :71-97
 *   shuffle_unique              :186-203
 *   BATfirstn_unique            :211-572 (void, sorted / revsorted slices,
 *                               heap over the first n (asc) or the last n
 *                               (desc) candidates)
 *   BATfirstn_unique_with_groups :716-1020 (heap over (group, value) pairs)
 *   BATfirstn dispatch          :1280-1340
 * Sortedness comes from BATordered / BATordered_rev (exact), and the
 * position of the nils in a sorted column from SORTfndlast
 * (gdk/gdk_search.c:486-513, binsearch :100-300): on a reverse-sorted
 * column SORTfndlast(b, nil) is BATcount(b) (nothing sorts after nil in
 * descending order), which is what the slices below reproduce.
 */
#include "gdk_oracle.h"

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

/* value of row p: integers widened to 128 bits (oid as lng: ATOMbasetype,
 * gdk_firstn.c:353), floats as double; nil = smallest (ATOMcmp) */
typedef struct {
	bool nil;
	bool isflt;
	ora_hge i;
	double f;
} fval;

static fval
fget(const ora_bat *b, uint64_t p)
{
	fval v = {0};
	const char *x = (const char *) b->base + p * b->width;
	switch (b->type) {
	case ORA_void:
		v.nil = b->tseqbase == ORA_OID_NIL;
		v.i = (ora_hge) (b->tseqbase + p);
		break;
	case ORA_bit: case ORA_bte: v.i = *(const int8_t *) x; v.nil = v.i == INT8_MIN; break;
	case ORA_sht: v.i = *(const int16_t *) x; v.nil = v.i == INT16_MIN; break;
	case ORA_int: case ORA_date: v.i = *(const int32_t *) x; v.nil = v.i == INT32_MIN; break;
	case ORA_lng: case ORA_oid: v.i = *(const int64_t *) x; v.nil = v.i == INT64_MIN; break;
	case ORA_hge: v.i = *(const ora_hge *) x; v.nil = v.i == (ora_hge) ((unsigned __int128) 1 << 127); break;
	case ORA_flt: v.isflt = true; v.f = *(const float *) x; v.nil = isnan(v.f); break;
	case ORA_dbl: v.isflt = true; v.f = *(const double *) x; v.nil = isnan(v.f); break;
	}
	return v;
}

/* three-way compare, nil smallest */
static int
fcmp(fval a, fval b)
{
	if (a.nil || b.nil)
		return b.nil - a.nil;
	if (a.isflt)
		return (a.f > b.f) - (a.f < b.f);
	return (a.i > b.i) - (a.i < b.i);
}

/* the four orderings of gdk_firstn.c:101-135 and gdk_calc_private.h LT/GT */
enum { OP_LT, OP_nLT, OP_GT, OP_nGT };

static bool
op(int mode, fval a, fval b)
{
	switch (mode) {
	case OP_LT: return fcmp(a, b) < 0;
	case OP_nLT: return !a.nil && (b.nil || fcmp(a, b) < 0);
	case OP_GT: return fcmp(a, b) > 0;
	default: return !b.nil && (a.nil || fcmp(a, b) > 0);
	}
}

typedef struct {
	const ora_bat *b;
	ora_oid hseq;
	int mode;
	bool voidgrp;          /* void b with groups: compare oids (:848-879) */
	bool asc;
	ora_oid *oids;         /* heap of candidate oids */
	ora_oid *goids;        /* their group ids (NULL: no groups) */
	uint64_t n;
} heap;

/* OPER(p1, p2) on heap slots */
static bool
hop(const heap *h, uint64_t p1, uint64_t p2)
{
	if (h->goids) {
		if (h->goids[p1] != h->goids[p2])
			return h->goids[p1] < h->goids[p2];
		if (h->voidgrp)
			return h->asc ? h->oids[p1] < h->oids[p2] : h->oids[p1] > h->oids[p2];
	}
	return op(h->mode, fget(h->b, h->oids[p1] - h->hseq), fget(h->b, h->oids[p2] - h->hseq));
}

static void
hswap(heap *h, uint64_t p1, uint64_t p2)
{
	ora_oid t = h->oids[p1];
	h->oids[p1] = h->oids[p2];
	h->oids[p2] = t;
	if (h->goids) {
		t = h->goids[p1];
		h->goids[p1] = h->goids[p2];
		h->goids[p2] = t;
	}
}

/* gdk_firstn.c:71-91 */
static void
siftdown(heap *h, uint64_t start)
{
	uint64_t pos = start, child = 2 * pos + 1;
	while (child < h->n) {
		if (child + 1 < h->n && !hop(h, child + 1, child))
			child++;
		if (!hop(h, pos, child))
			break;
		hswap(h, pos, child);
		pos = child;
		child = 2 * pos + 1;
	}
}

/* gdk_firstn.c:93-97 */
static void
heapify(heap *h)
{
	for (uint64_t i = h->n / 2; i > 0; i--)
		siftdown(h, i - 1);
}

static int
cmp_oid(const void *a, const void *b)
{
	ora_oid x = *(const ora_oid *) a, y = *(const ora_oid *) b;
	return (x > y) - (x < y);
}

/* candidate slices [a0, a1) u [b0, b1) as a candidate list */
static ora_bat *
slice2(const ora_ci *ci, uint64_t a0, uint64_t a1, uint64_t b0, uint64_t b1)
{
	uint64_t n = (a1 - a0) + (b1 - b0);
	ora_bat *bn = ora_new(ORA_oid, n, 0);
	if (bn == NULL)
		return NULL;
	ora_oid *o = bn->base;
	uint64_t k = 0;
	for (uint64_t i = a0; i < a1; i++)
		o[k++] = ci_get(ci, i);
	for (uint64_t i = b0; i < b1; i++)
		o[k++] = ci_get(ci, i);
	/* virtualise a dense result (gdk_select.c:31-89 via canditer_slice) */
	if (n <= 1 || o[n - 1] - o[0] == n - 1) {
		ora_oid seq = n ? o[0] : 0;
		ora_free(bn);
		return ora_dense(0, seq, n);
	}
	bn->sorted = bn->key = bn->nonil = 1;
	return bn;
}

static ora_bat *
heap_result(heap *h)
{
	qsort(h->oids, h->n, sizeof(ora_oid), cmp_oid);
	ora_bat *bn = ora_new(ORA_oid, h->n, 0);
	if (bn == NULL)
		return NULL;
	memcpy(bn->base, h->oids, h->n * sizeof(ora_oid));
	const ora_oid *o = bn->base;
	if (h->n <= 1 || o[h->n - 1] - o[0] == h->n - 1) {
		ora_oid seq = h->n ? o[0] : 0;
		ora_free(bn);
		return ora_dense(0, seq, h->n);
	}
	bn->sorted = bn->key = bn->nonil = 1;
	return bn;
}

/* BATordered / BATordered_rev and whether b holds a nil */
static void
props(const ora_bat *b, bool *sorted, bool *revsorted, bool *hasnil)
{
	*sorted = *revsorted = true;
	*hasnil = false;
	if (b->type == ORA_void) {
		*hasnil = b->tseqbase == ORA_OID_NIL && b->count > 0;
		*revsorted = b->count <= 1 || b->tseqbase == ORA_OID_NIL;
		return;
	}
	fval prev = {0};
	for (uint64_t i = 0; i < b->count; i++) {
		fval v = fget(b, i);
		*hasnil |= v.nil;
		if (i > 0) {
			int c = fcmp(prev, v);
			if (c > 0)
				*sorted = false;
			if (c < 0)
				*revsorted = false;
		}
		prev = v;
	}
}

static int
heap_mode(bool asc, bool nilslast, bool hasnil)
{
	if (asc)
		return nilslast && hasnil ? OP_nLT : OP_LT;
	return nilslast || !hasnil ? OP_GT : OP_nGT;
}

/* BATfirstn_unique, gdk_firstn.c:211-572 */
static ora_bat *
firstn_unique(const ora_bat *b, const ora_bat *s, uint64_t n, bool asc, bool nilslast)
{
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return NULL;
	uint64_t cnt = ci.n;
	if (n >= cnt)
		return slice2(&ci, 0, cnt, 0, 0);
	if (b->type == ORA_void) {
		if (asc || b->tseqbase == ORA_OID_NIL)
			return slice2(&ci, 0, n, 0, 0);
		return slice2(&ci, cnt - n, cnt, 0, 0);
	}
	bool sorted, revsorted, hasnil;
	props(b, &sorted, &revsorted, &hasnil);
	if (sorted || revsorted) {
		if (nilslast == asc && hasnil) {
			uint64_t pos;
			if (sorted) {
				/* SORTfndlast(b, nil): first non-nil row */
				uint64_t p = 0;
				while (p < b->count && fget(b, p).nil)
					p++;
				pos = 0;
				while (pos < cnt && ci_get(&ci, pos) < b->hseqbase + p)
					pos++;
				if (asc)
					return cnt - pos < n ? slice2(&ci, cnt - n, cnt, 0, 0)
							     : slice2(&ci, pos, pos + n, 0, 0);
				return pos < n ? slice2(&ci, 0, pos, cnt - (n - pos), cnt) : slice2(&ci, 0, n, 0, 0);
			}
			/* reverse sorted: SORTfndlast(b, nil) == BATcount(b) */
			pos = cnt;
			if (asc)
				return pos < n ? slice2(&ci, 0, n, 0, 0) : slice2(&ci, pos - n, pos, 0, 0);
			return cnt - pos < n ? slice2(&ci, 0, n - (cnt - pos), pos, cnt) : slice2(&ci, pos, pos + n, 0, 0);
		}
		if (asc ? sorted : revsorted)
			return slice2(&ci, 0, n, 0, 0);
		return slice2(&ci, cnt - n, cnt, 0, 0);
	}
	heap h = {.b = b, .hseq = b->hseqbase, .mode = heap_mode(asc, nilslast, hasnil), .asc = asc, .n = n};
	h.oids = malloc(n * sizeof(ora_oid));
	if (h.oids == NULL)
		return NULL;
	uint64_t i0, i1;
	if (asc) {
		for (uint64_t i = 0; i < n; i++)
			h.oids[i] = ci_get(&ci, i);
		i0 = n;
		i1 = cnt;
	} else {
		for (uint64_t k = 0; k < n; k++)
			h.oids[n - 1 - k] = ci_get(&ci, cnt - n + k);
		i0 = 0;
		i1 = cnt - n;
	}
	heapify(&h);
	for (uint64_t i = i0; i < i1; i++) {
		ora_oid o = ci_get(&ci, i);
		if (op(h.mode, fget(b, o - h.hseq), fget(b, h.oids[0] - h.hseq))) {
			h.oids[0] = o;
			siftdown(&h, 0);
		}
	}
	ora_bat *bn = heap_result(&h);
	free(h.oids);
	return bn;
}

/* BATfirstn_unique_with_groups, gdk_firstn.c:716-1020 */
static ora_bat *
firstn_unique_with_groups(const ora_bat *b, const ora_bat *s, const ora_bat *g, uint64_t n, bool asc,
			  bool nilslast)
{
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return NULL;
	uint64_t cnt = ci.n;
	if (n > cnt)
		n = cnt;
	if (n == 0)
		return ora_dense(0, 0, 0);
	if (g->type == ORA_void && g->tseqbase != ORA_OID_NIL)
		return slice2(&ci, 0, n, 0, 0);
	bool sorted, revsorted, hasnil;
	props(b, &sorted, &revsorted, &hasnil);
	heap h = {.b = b, .hseq = b->hseqbase, .mode = heap_mode(asc, nilslast, hasnil), .asc = asc, .n = n,
		  .voidgrp = b->type == ORA_void};
	h.oids = malloc(n * sizeof(ora_oid));
	h.goids = malloc(n * sizeof(ora_oid));
	if (h.oids == NULL || h.goids == NULL) {
		free(h.oids);
		free(h.goids);
		return NULL;
	}
	const ora_oid *gv = g->base;
	uint64_t j = 0;
	for (uint64_t i = 0; i < n; i++) {
		h.oids[i] = ci_get(&ci, i);
		h.goids[i] = g->type == ORA_void ? g->tseqbase + j : gv[j];
		j++;
	}
	heapify(&h);
	for (uint64_t i = n; i < cnt; i++, j++) {
		ora_oid o = ci_get(&ci, i);
		ora_oid gj = g->type == ORA_void ? g->tseqbase + j : gv[j];
		bool in;
		if (h.voidgrp)
			in = gj < h.goids[0] || (!asc && gj == h.goids[0]);
		else
			in = gj < h.goids[0] ||
			     (gj == h.goids[0] && op(h.mode, fget(b, o - h.hseq), fget(b, h.oids[0] - h.hseq)));
		if (in) {
			h.oids[0] = o;
			h.goids[0] = gj;
			siftdown(&h, 0);
		}
	}
	ora_bat *bn = heap_result(&h);
	free(h.oids);
	free(h.goids);
	return bn;
}

/* BATfirstn(&topn, NULL, b, s, g, n, asc, nilslast, false), :1280-1340 */
ora_bat *
ora_firstn(const ora_bat *b, const ora_bat *s, const ora_bat *g, uint64_t n, bool asc, bool nilslast)
{
	if (b == NULL) {
		ora_seterr("firstn: b is NULL");
		return NULL;
	}
	if (n == 0 || b->count == 0 || (s != NULL && s->count == 0))
		return ora_dense(0, 0, 0);
	if (g == NULL)
		return firstn_unique(b, s, n, asc, nilslast);
	if (s == NULL || s->count != g->count) {
		ora_seterr("firstn: g requires s, aligned with it");
		return NULL;
	}
	return firstn_unique_with_groups(b, s, g, n, asc, nilslast);
}
