/*
 * gdk_oracle_grp.c -- CPU restatement of GDK grouping, grouped aggregates,
 * hash join, sort and RANGE window bounds.  TEST INFRASTRUCTURE ONLY
 * (see gdk_oracle.h).
 */
#include "gdk_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

void ora_seterr(const char *fmt, ...);
int ora_width(int type);
int ora_fsum_array(double *out, bool *isnil, const double *vals, uint64_t nv, bool skip_nils, bool nil_if_empty);
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

#define HGE_NIL ((ora_hge) ((unsigned __int128) 1 << 127))
#define HGE_MAX ((ora_hge) (((unsigned __int128) 1 << 127) - 1))

/* grouping key of row p: values compare by equality as in GDK's group code
 * (gdk_group.c, flt/dbl by value: -0 == +0, every NaN is the nil) */
static bool val_at(const ora_bat *b, uint64_t p, ora_hge *v);
static bool
grp_key(const ora_bat *b, uint64_t p, ora_hge *v)
{
	if (b->type == ORA_flt || b->type == ORA_dbl) {
		double d = b->type == ORA_flt ? (double) ((const float *) b->base)[p] : ((const double *) b->base)[p];
		if (isnan(d)) {
			*v = (ora_hge) 1 << 100;   /* outside every double image */
			return true;
		}
		if (d == 0.0)
			d = 0.0;
		int64_t bits;
		memcpy(&bits, &d, 8);
		*v = bits;
		return false;
	}
	return val_at(b, p, v);
}

/* value of row p of b widened to 128 bits; returns true when nil */
static bool
val_at(const ora_bat *b, uint64_t p, ora_hge *v)
{
	const char *x = (const char *) b->base + p * b->width;
	switch (b->type) {
	case ORA_void: *v = (ora_hge) (b->tseqbase + p); return false;
	case ORA_bit: case ORA_bte: *v = *(const int8_t *) x; return *v == INT8_MIN;
	case ORA_sht: *v = *(const int16_t *) x; return *v == INT16_MIN;
	case ORA_int: case ORA_date: *v = *(const int32_t *) x; return *v == INT32_MIN;
	case ORA_lng: *v = *(const int64_t *) x; return *v == INT64_MIN;
	case ORA_hge: *v = *(const ora_hge *) x; return *v == HGE_NIL;
	case ORA_oid: *v = (ora_hge) *(const ora_oid *) x; return *(const ora_oid *) x == ORA_OID_NIL;
	case ORA_str:
		/* 1/2/4/8-byte heap offsets; equal strings share offsets in a
		 * duplicate-eliminated heap (gdk/gdk_atoms.h:370-430) */
		switch (b->width) {
		case 1: *v = *(const uint8_t *) x; break;
		case 2: *v = *(const uint16_t *) x; break;
		case 4: *v = *(const uint32_t *) x; break;
		default: *v = *(const uint64_t *) x; break;
		}
		return false;
	}
	*v = 0;
	return false;
}

/* ---------------------------------------------------------------------- */
/* BATgroup (gdk/gdk_group.c:657-1347): group ids are handed out in order
 * of first occurrence of each distinct (g, value) pair over the candidates
 * (GRPnotfound, gdk_group.c:74-100); nil is an ordinary value; extents hold
 * the oid of each group's first row, histo the row count.  groups is
 * aligned with the candidates (hseqbase = first candidate). */

typedef struct {
	ora_hge key;
	ora_oid g;
	ora_oid gid;
	uint64_t pos;      /* b position of the group's first row (str content) */
	int used;
} gslot;

/* a str column whose heap is not duplicate eliminated (GDK_ELIMDOUBLES,
 * gdk/gdk_atoms.h:373-375: heap free >= GDK_ELIMLIMIT = 64 KiB): BATgroup then
 * compares string contents, not offsets (gdk/gdk_group.c:897-919, the hash
 * path :1118-1282 with ATOMcompare = strCmp) */
#define ORA_ELIMLIMIT ((uint64_t) 1 << 16)
static bool
str_by_content(const ora_bat *b)
{
	return b->type == ORA_str && b->vheap != NULL && b->vheapsize >= ORA_ELIMLIMIT;
}

/* the string of row p (VarHeapVal, gdk/gdk_atoms.h:421-436: 1- and 2-byte
 * offsets are relative to GDK_VAROFFSET = 1024 * sizeof(var_t)) */
static const char *
str_of(const ora_bat *b, uint64_t p)
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

static uint64_t
str_hash(const char *s)
{
	uint64_t h = 0xcbf29ce484222325ULL;   /* FNV-1a over the bytes */
	for (; *s; s++)
		h = (h ^ (uint8_t) *s) * 0x100000001b3ULL;
	return h;
}

static uint64_t
ghash(ora_hge k, ora_oid g)
{
	uint64_t x = (uint64_t) k ^ ((uint64_t) (k >> 64) * 0x9e3779b97f4a7c15ULL) ^ (g * 0xbf58476d1ce4e5b9ULL);
	x ^= x >> 31;
	x *= 0x94d049bb133111ebULL;
	return x ^ (x >> 29);
}

static ora_bat *
ora_constant(ora_oid hseq, int type, int64_t v, uint64_t n)
{
	/* BATconstant (gdk/gdk_batop.c:2832-2922) of an oid / lng value */
	ora_bat *bn = ora_new(type, n, hseq);
	if (bn == NULL)
		return NULL;
	for (uint64_t i = 0; i < n; i++)
		((int64_t *) bn->base)[i] = v;
	bn->sorted = bn->revsorted = 1;
	bn->nil = 0;
	bn->nonil = 1;
	bn->key = n <= 1;
	return bn;
}

/* BATgroup (gdk/gdk_group.c:657-1344): the one-element-per-group and
 * single-group shortcuts (:712-800), else first-occurrence group ids with
 * the result properties of :1284-1318 */
int
ora_group(ora_bat **groups, ora_bat **extents, ora_bat **histo,
	  ora_bat *b, const ora_bat *s, const ora_bat *g)
{
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return -1;
	if (g && g->count != ci.n) {
		ora_seterr("b with s and g must be aligned");
		return -1;
	}
	ora_oid hseqb = ci.n ? ci_get(&ci, 0) : 0;
	ora_bat *gn, *en, *hn;
	const bool gdense = g && (g->type == ORA_void || g->tseqbase != ORA_OID_NIL);
	if (b->key || ci.n <= 1 || (g && (g->key || gdense))) {
		/* trivial: one element per group; note the groups BAT has
		 * BATcount(b) rows, as in the reference (:713) */
		gn = ora_dense(hseqb, 0, b->count);
		if (ci.dense || ci.n <= 1) {
			en = ora_dense(0, ci.n ? ci_get(&ci, 0) : 0, ci.n);
		} else {
			en = ora_new(ORA_oid, ci.n, 0);
			if (en) {
				memcpy(en->base, ci.oids, ci.n * 8);
				en->sorted = en->key = en->nonil = 1;
				en->revsorted = ci.n <= 1;
				en->minpos = 0;
				en->maxpos = ci.n - 1;
			}
		}
		hn = ora_constant(0, ORA_lng, 1, ci.n);
		goto out;
	}
	bool gsame = !g;
	if (g) {
		bool asc = false, desc = false;
		for (uint64_t i = 1; i < g->count; i++) {
			ora_oid x = ((const ora_oid *) g->base)[i - 1], y = ((const ora_oid *) g->base)[i];
			asc |= x < y;
			desc |= x > y;
		}
		gsame = !asc && !desc;
	}
	if (b->sorted && b->revsorted && gsame) {
		/* all values equal, one prior group: a single group 0 */
		gn = ora_constant(hseqb, ORA_oid, 0, ci.n);
		en = ora_dense(0, ci_get(&ci, 0), 1);
		hn = ora_constant(0, ORA_lng, (int64_t) ci.n, 1);
		goto out;
	}
	gn = ora_new(ORA_oid, ci.n, hseqb);
	en = ora_new(ORA_oid, ci.n, 0);
	hn = ora_new(ORA_lng, ci.n, 0);
	uint64_t cap = 16;
	while (cap < 2 * ci.n)
		cap <<= 1;
	gslot *tab = calloc(cap, sizeof(gslot));
	if (!gn || !en || !hn || !tab) {
		ora_free(gn); ora_free(en); ora_free(hn); free(tab);
		ora_seterr("out of memory");
		return -1;
	}
	ora_oid *gids = gn->base, *ext = en->base;
	int64_t *cnt = hn->base;
	uint64_t ngrp = 0, maxgrppos = ORA_BUN_NONE;
	const bool content = str_by_content(b);
	for (uint64_t i = 0; i < ci.n; i++) {
		ora_oid o = ci_get(&ci, i);
		const uint64_t p = o - b->hseqbase;
		ora_hge v;
		if (content)
			v = (ora_hge) str_hash(str_of(b, p));   /* equal strings, equal keys */
		else
			(void) grp_key(b, p, &v);
		ora_oid gg = 0;
		if (g)
			gg = g->type == ORA_void ? g->tseqbase + i : ((const ora_oid *) g->base)[i];
		uint64_t h = ghash(v, gg) & (cap - 1);
		while (tab[h].used && !(tab[h].key == v && tab[h].g == gg &&
					(!content || strcmp(str_of(b, tab[h].pos), str_of(b, p)) == 0)))
			h = (h + 1) & (cap - 1);
		if (!tab[h].used) {
			tab[h].used = 1;
			tab[h].key = v;
			tab[h].pos = p;
			tab[h].g = gg;
			tab[h].gid = ngrp;
			ext[ngrp] = o;
			cnt[ngrp] = 0;
			ngrp++;
			maxgrppos = i;
		}
		gids[i] = tab[h].gid;
		cnt[tab[h].gid]++;
	}
	free(tab);
	en->count = hn->count = ngrp;
	gn->nonil = 1;
	gn->nil = 0;
	gn->key = ngrp == ci.n;
	gn->revsorted = ngrp == 1 || ci.n <= 1;
	bool srt = true;
	for (uint64_t i = 1; i < ci.n && srt; i++)
		srt = gids[i - 1] <= gids[i];
	gn->sorted = srt;
	gn->maxpos = maxgrppos;
	gn->unique_est = (double) ngrp;
	en->sorted = en->key = en->nonil = 1;
	en->nil = 0;
	en->revsorted = ngrp == 1;
	en->unique_est = (double) ngrp;
	if (ngrp <= 1 || ext[ngrp - 1] - ext[0] == ngrp - 1) {
		/* virtualize */
		ora_oid seq = ngrp ? ext[0] : 0;
		free(en->base);
		en->base = NULL;
		en->type = ORA_void;
		en->width = 0;
		en->tseqbase = seq;
	}
	if (ngrp == ci.n || ngrp == 1) {
		hn->key = ngrp == 1;
		hn->sorted = hn->revsorted = 1;
	} else {
		hn->key = hn->sorted = hn->revsorted = 0;
	}
	hn->nonil = 1;
	hn->nil = 0;
	if (!g && !s)
		b->unique_est = (double) ngrp;
out:
	if (!gn || !en || !hn) {
		ora_free(gn); ora_free(en); ora_free(hn);
		ora_seterr("out of memory");
		return -1;
	}
	*groups = gn;
	if (extents)
		*extents = en;
	else
		ora_free(en);
	if (histo)
		*histo = hn;
	else
		ora_free(hn);
	return 0;
}

/* ---------------------------------------------------------------------- */
/* grouped aggregates: BATgroupaggrinit (gdk/gdk_aggr.c:65-146) computes the
 * group id range [min, max] from e (count(e) groups starting at
 * e->hseqbase) or from g; g is aligned with the candidates. */

typedef struct {
	ora_ci ci;
	ora_oid min, max;
	uint64_t ngrp;
	const ora_oid *gids;   /* NULL: dense g (gid = g->tseqbase + i) */
	ora_oid gseq;
} aggr_ctx;

static int
aggr_init(aggr_ctx *a, const ora_bat *b, const ora_bat *g, const ora_bat *e,
	  const ora_bat *s)
{
	memset(a, 0, sizeof(*a));
	if (ora_ci_init(&a->ci, b, s) < 0)
		return -1;
	if (g == NULL) {
		ora_seterr("b and g must be aligned\n");
		return -1;
	}
	/* BATgroupaggrinit (gdk_aggr.c:65-110): g has one group id per
	 * candidate and its head starts at the first candidate */
	if (a->ci.n != g->count || (a->ci.n != 0 && ci_get(&a->ci, 0) != g->hseqbase)) {
		ora_seterr("b with s and g must be aligned\n");
		return -1;
	}
	a->gids = g->type == ORA_void ? NULL : g->base;
	a->gseq = g->tseqbase;
	if (e) {
		a->ngrp = e->count;
		a->min = e->hseqbase;
		a->max = e->hseqbase + a->ngrp - 1;
	} else {
		ora_oid mn = ORA_OID_NIL, mx = 0;
		for (uint64_t i = 0; i < g->count; i++) {
			ora_oid x = a->gids ? a->gids[i] : a->gseq + i;
			if (x == ORA_OID_NIL)
				continue;
			if (x < mn) mn = x;
			if (x > mx) mx = x;
		}
		a->min = mn;
		a->max = mx;
		a->ngrp = mx < mn || mn == ORA_OID_NIL ? 0 : mx - mn + 1;
	}
	return 0;
}

static inline bool
aggr_gid(const aggr_ctx *a, uint64_t i, ora_oid *gid)
{
	ora_oid x = a->gids ? a->gids[i] : a->gseq + i;
	if (x < a->min || x > a->max)
		return false;
	*gid = x - a->min;
	return true;
}

static ora_hge
tmax(int tp)
{
	switch (tp) {
	case ORA_bte: return INT8_MAX;
	case ORA_sht: return INT16_MAX;
	case ORA_int: return INT32_MAX;
	case ORA_lng: return INT64_MAX;
	default: return HGE_MAX;
	}
}

static void
put(int tp, void *base, uint64_t i, ora_hge v, bool nil)
{
	switch (tp) {
	case ORA_bit: case ORA_bte: ((int8_t *) base)[i] = nil ? INT8_MIN : (int8_t) v; break;
	case ORA_sht: ((int16_t *) base)[i] = nil ? INT16_MIN : (int16_t) v; break;
	case ORA_int: ((int32_t *) base)[i] = nil ? INT32_MIN : (int32_t) v; break;
	case ORA_lng: ((int64_t *) base)[i] = nil ? INT64_MIN : (int64_t) v; break;
	case ORA_hge: ((ora_hge *) base)[i] = nil ? HGE_NIL : v; break;
	case ORA_oid: ((ora_oid *) base)[i] = nil ? ORA_OID_NIL : (ora_oid) v; break;
	}
}

/* BATgroupsum (gdk/gdk_aggr.c:900, dosum :708 with nil_if_empty=true):
 * a group's sum is nil until its first non-nil value; a nil value makes
 * it nil for good unless skip_nils; overflow is an error. */
ora_bat *
ora_groupsum(const ora_bat *b, const ora_bat *g, const ora_bat *e,
	     const ora_bat *s, int tp, bool skip_nils)
{
	aggr_ctx a;
	if (aggr_init(&a, b, g, e, s) < 0)
		return NULL;
	if (b->type == ORA_flt || b->type == ORA_dbl) {
		/* dofsum with groups (gdk_aggr.c:183-427): msum per group over its
		 * values in candidate order; a nil makes the group nil unless
		 * skip_nils, an empty group is nil */
		ora_bat *bn = ora_new(tp, a.ngrp, a.ngrp ? a.min : 0);
		uint64_t *cnt = calloc(a.ngrp + 1, sizeof(uint64_t)), *pos = calloc(a.ngrp + 1, sizeof(uint64_t));
		double *vals = malloc((a.ci.n + 1) * sizeof(double));
		ora_oid *gof = malloc((a.ci.n + 1) * sizeof(ora_oid));
		for (uint64_t i = 0; i < a.ci.n; i++) {
			ora_oid gid = 0;
			if (a.ngrp != 1 && !aggr_gid(&a, i, &gid)) {
				gof[i] = ORA_OID_NIL;
				continue;
			}
			gof[i] = gid;
			cnt[gid]++;
		}
		uint64_t acc = 0;
		for (uint64_t k = 0; k < a.ngrp; k++) {
			pos[k] = acc;
			acc += cnt[k];
		}
		for (uint64_t i = 0; i < a.ci.n; i++) {
			if (gof[i] == ORA_OID_NIL)
				continue;
			uint64_t p = ci_get(&a.ci, i) - b->hseqbase;
			vals[pos[gof[i]]++] = b->type == ORA_flt ? (double) ((const float *) b->base)[p]
								  : ((const double *) b->base)[p];
		}
		int rc = 0;
		for (uint64_t k = 0; k < a.ngrp && rc == 0; k++) {
			double d;
			bool isnil;
			rc = ora_fsum_array(&d, &isnil, vals + pos[k] - cnt[k], cnt[k], skip_nils, true);
			if (tp == ORA_dbl) {
				((double *) bn->base)[k] = isnil ? nan("") : d;
			} else {
				float f = (float) d;
				if (!isnil && isinf(f)) {
					ora_seterr("22003!overflow in sum aggregate.\n");
					rc = -1;
				}
				((float *) bn->base)[k] = isnil ? nanf("") : f;
			}
		}
		free(cnt); free(pos); free(vals); free(gof);
		if (rc < 0) {
			ora_free(bn);
			return NULL;
		}
		return bn;
	}
	ora_bat *bn = ora_new(tp, a.ngrp, a.ngrp ? a.min : 0);
	ora_hge *acc = calloc(a.ngrp + 1, sizeof(ora_hge));
	uint8_t *st = calloc(a.ngrp + 1, 1);    /* 0 unseen, 1 value, 2 nil */
	if (!bn || !acc || !st) {
		ora_free(bn); free(acc); free(st);
		ora_seterr("out of memory");
		return NULL;
	}
	ora_hge max = tmax(tp);
	/* st bit 0: group seen (a non-nil value arrived), bit 1: sum is nil.
	 * With several groups, a nil arriving before the group's first
	 * non-nil value is forgotten when that value resets the sum to 0
	 * (AGGR_SUM "with groups", gdk_aggr.c:497-527); with a single group
	 * any nil makes the sum nil (:440-470). */
	for (uint64_t i = 0; i < a.ci.n; i++) {
		ora_oid gid;
		if (a.ngrp == 1)
			gid = 0;
		else if (!aggr_gid(&a, i, &gid))
			continue;
		ora_hge v;
		if (val_at(b, ci_get(&a.ci, i) - b->hseqbase, &v)) {
			if (!skip_nils) {
				st[gid] |= 2;
				if (a.ngrp == 1)
					break;
			}
			continue;
		}
		if (!(st[gid] & 1)) {
			st[gid] = 1;
			acc[gid] = 0;
		}
		if (st[gid] & 2)
			continue;
		ora_hge z;
		if (__builtin_add_overflow(acc[gid], v, &z) || z < -max || z > max) {
			ora_seterr("22003!overflow in sum aggregate.\n");
			ora_free(bn); free(acc); free(st);
			return NULL;
		}
		acc[gid] = z;
	}
	bool hasnil = false;
	for (uint64_t k = 0; k < a.ngrp; k++) {
		put(tp, bn->base, k, acc[k], st[k] != 1);
		hasnil |= st[k] != 1;
	}
	bn->nil = hasnil;
	bn->nonil = !hasnil;
	bn->sorted = bn->revsorted = bn->key = a.ngrp <= 1;
	free(acc);
	free(st);
	return bn;
}

/* BATgroupcount (gdk/gdk_aggr.c:3069): lng counts, 0 for empty groups */
ora_bat *
ora_groupcount(const ora_bat *b, const ora_bat *g, const ora_bat *e,
	       const ora_bat *s, bool skip_nils)
{
	aggr_ctx a;
	if (aggr_init(&a, b, g, e, s) < 0)
		return NULL;
	ora_bat *bn = ora_new(ORA_lng, a.ngrp, a.ngrp ? a.min : 0);
	if (!bn)
		return NULL;
	int64_t *c = bn->base;
	memset(c, 0, a.ngrp * 8);
	for (uint64_t i = 0; i < a.ci.n; i++) {
		ora_oid gid;
		if (!aggr_gid(&a, i, &gid))
			continue;
		ora_hge v;
		if (skip_nils && val_at(b, ci_get(&a.ci, i) - b->hseqbase, &v))
			continue;
		c[gid]++;
	}
	/* gdk_aggr.c:3105-3106 (empty: BATconstant of 0), :3185-3190 */
	bn->nonil = 1;
	bn->nil = 0;
	bn->key = a.ngrp <= 1;
	bn->sorted = bn->revsorted = a.ngrp <= 1 || a.ci.n == 0;
	return bn;
}

/* BATgroupavg3 (gdk/gdk_aggr.c:1996-2110): exact average of integers as
 * floor(sum/n) and remainder (AVERAGE_ITER, gdk_calc_private.h:231-275),
 * then rounded half away from zero (non-TRUNCATE_NUMBERS branch:
 * avg<0 rounds when 2*rem > n, avg>=0 when 2*rem >= n, and rem -= n).
 * Empty groups: avg nil, rem 0, count 0; a nil input without skip_nils makes
 * all three nil for the group. */
int
ora_groupavg3(ora_bat **avgp, ora_bat **remp, ora_bat **cntp,
	      const ora_bat *b, const ora_bat *g, const ora_bat *e,
	      const ora_bat *s, bool skip_nils)
{
	aggr_ctx a;
	if (aggr_init(&a, b, g, e, s) < 0)
		return -1;
	int tp = b->type == ORA_date ? ORA_int : b->type;
	ora_bat *bn = ora_new(tp, a.ngrp, a.ngrp ? a.min : 0);
	ora_bat *rn = ora_new(ORA_lng, a.ngrp, a.ngrp ? a.min : 0);
	ora_bat *cn = ora_new(ORA_lng, a.ngrp, a.ngrp ? a.min : 0);
	ora_hge *sum = calloc(a.ngrp + 1, sizeof(ora_hge));
	uint8_t *isnil = calloc(a.ngrp + 1, 1);
	int64_t *cnt = cn ? cn->base : NULL;
	if (!bn || !rn || !cn || !sum || !isnil) {
		ora_free(bn); ora_free(rn); ora_free(cn); free(sum); free(isnil);
		ora_seterr("out of memory");
		return -1;
	}
	memset(cnt, 0, a.ngrp * 8);
	for (uint64_t i = 0; i < a.ci.n; i++) {
		ora_oid gid;
		if (!aggr_gid(&a, i, &gid))
			continue;
		ora_hge v;
		if (val_at(b, ci_get(&a.ci, i) - b->hseqbase, &v)) {
			if (!skip_nils)
				isnil[gid] = 1;
			continue;
		}
		if (isnil[gid])
			continue;
		sum[gid] += v;   /* exact: |sum| < 2^63 * 2^64 */
		cnt[gid]++;
	}
	int64_t *rem = rn->base;
	for (uint64_t k = 0; k < a.ngrp; k++) {
		if (isnil[k]) {
			put(tp, bn->base, k, 0, true);
			rem[k] = INT64_MIN;
			cnt[k] = INT64_MIN;
			continue;
		}
		if (cnt[k] == 0) {
			put(tp, bn->base, k, 0, true);
			rem[k] = 0;
			continue;
		}
		ora_hge n = cnt[k];
		ora_hge q = sum[k] / n, r = sum[k] % n;
		if (r < 0) {      /* floor division, 0 <= r < n */
			q -= 1;
			r += n;
		}
		if (r > 0) {
			if (q < 0) {
				if (2 * r > n) { q++; r -= n; }
			} else {
				if (2 * r >= n) { q++; r -= n; }
			}
		}
		put(tp, bn->base, k, q, false);
		rem[k] = (int64_t) r;
	}
	free(sum);
	free(isnil);
	*avgp = bn;
	*remp = rn;
	*cntp = cn;
	return 0;
}

/* BATgroupavg3combine (gdk/gdk_aggr.c:2634-2960): each group's (avg, rem,
 * cnt) state starts at 0 and folds every row in order with
 * combine_averages_TYPE (:2402-2630): a row with rem < 0 is first
 * normalised (avg--, rem += cnt); the new state is the floor average of
 * the exact total avg1*cnt1 + rem1 + avg2*cnt2 + rem2 over cnt1 + cnt2
 * (the hge branch reaches the same quotient through multdiv).  A nil avg
 * without skip_nils makes the group nil for good; groups with count 0 are
 * nil; the rest are rounded half away from zero (:2702-2716). */
ora_bat *
ora_groupavg3combine(const ora_bat *avg, const ora_bat *rem, const ora_bat *cnt, const ora_bat *g,
		     const ora_bat *e, bool skip_nils)
{
	aggr_ctx a;
	if (aggr_init(&a, avg, g, e, NULL) < 0)
		return NULL;
	if (a.ci.n != rem->count || a.ci.n != cnt->count) {
		ora_seterr("input bats not aligned");
		return NULL;
	}
	const int tp = avg->type;
	ora_bat *bn = ora_new(tp, a.ngrp, a.ngrp ? a.min : 0);
	ora_hge *av = calloc(a.ngrp + 1, sizeof(ora_hge));
	int64_t *rm = calloc(a.ngrp + 1, 8), *ct = calloc(a.ngrp + 1, 8);
	uint8_t *isnil = calloc(a.ngrp + 1, 1);
	if (!bn || !av || !rm || !ct || !isnil) {
		ora_free(bn); free(av); free(rm); free(ct); free(isnil);
		ora_seterr("out of memory");
		return NULL;
	}
	const int64_t *R = rem->base, *K = cnt->base;
	for (uint64_t i = 0; i < a.ci.n; i++) {
		ora_oid gid;
		if (!aggr_gid(&a, i, &gid))
			continue;
		ora_hge v2;
		if (val_at(avg, i, &v2)) {
			if (!skip_nils)
				isnil[gid] = 1;
			continue;
		}
		if (isnil[gid])
			continue;
		int64_t rem2 = R[i], cnt2 = K[i];
		if (rem2 < 0) {
			v2--;
			rem2 += cnt2;
		}
		const int64_t c = ct[gid] + cnt2;
		ora_hge t = av[gid] * ct[gid] + rm[gid] + v2 * cnt2 + rem2;
		ora_hge q = t / c, r = t % c;
		if (r < 0) {
			q--;
			r += c;
		}
		av[gid] = q;
		rm[gid] = (int64_t) r;
		ct[gid] = c;
	}
	bool hasnil = false;
	for (uint64_t k = 0; k < a.ngrp; k++) {
		if (isnil[k] || ct[k] == 0) {
			put(tp, bn->base, k, 0, true);
			hasnil = true;
			continue;
		}
		ora_hge q = av[k];
		if (rm[k] > 0 && (q < 0 ? 2 * rm[k] > ct[k] : 2 * rm[k] >= ct[k]))
			q++;
		put(tp, bn->base, k, q, false);
	}
	bn->nil = hasnil;
	bn->nonil = !hasnil;
	bn->sorted = bn->revsorted = bn->key = a.ngrp <= 1;
	free(av); free(rm); free(ct); free(isnil);
	return bn;
}

/* BATgroupavg (gdk/gdk_aggr.c:1801-1984): average as dbl.
 * Trivial cases first: no candidates or no groups -> all nil, counts 0
 * (:1834-1853); singleton groups (g dense or key+nonil, e aligned) -> the
 * values converted to dbl (BATconvert, no scale applied), counts 1
 * (:1855-1873).  Otherwise integers run AVERAGE_ITER (gdk_calc_private.h:
 * 231-275: floor average + remainder, exact) and give avg + (dbl) rem / cnt
 * (AGGR_AVG :1717-1751); flt/dbl run the order-dependent AVERAGE_ITER_FLOAT
 * (:277-289) in candidate order (AGGR_AVG_FLOAT :1753-1785).  A nil input
 * without skip_nils makes the group nil for good; nil groups have count 0.
 * scale != 0 divides non-nil averages by 10^scale (:1958-1964). */
int
ora_groupavg(ora_bat **bnp, ora_bat **cntp, const ora_bat *b, const ora_bat *g,
	     const ora_bat *e, const ora_bat *s, bool skip_nils, int scale)
{
	aggr_ctx a;
	if (cntp)
		*cntp = NULL;
	if (aggr_init(&a, b, g, e, s) < 0)
		return -1;
	const int tp = b->type;
	const bool isf = tp == ORA_flt || tp == ORA_dbl;
	if (!isf && tp != ORA_bte && tp != ORA_sht && tp != ORA_int && tp != ORA_lng && tp != ORA_hge) {
		ora_seterr("type (%d) not supported.\n", tp);
		return -1;
	}
	const uint64_t ng = a.ngrp;
	const ora_oid hb = ng ? a.min : 0;
	ora_bat *bn, *cn = NULL;
	if (a.ci.n == 0 || ng == 0) {
		bn = ora_new(ORA_dbl, ng, hb);
		for (uint64_t k = 0; k < ng; k++)
			((double *) bn->base)[k] = nan("");
		if (cntp) {
			cn = ora_new(ORA_lng, ng, hb);
			memset(cn->base, 0, ng * 8);
		}
		*bnp = bn;
		if (cntp)
			*cntp = cn;
		return 0;
	}
	const bool gdense = g->tseqbase != ORA_OID_NIL;
	if ((!skip_nils || cntp == NULL || b->nonil) &&
	    (e == NULL || (e->count == a.ci.n && e->hseqbase == b->hseqbase)) &&
	    (gdense || (g->key && g->nonil))) {
		bn = ora_new(ORA_dbl, a.ci.n, s ? s->hseqbase : b->hseqbase);
		for (uint64_t i = 0; i < a.ci.n; i++) {
			const uint64_t p = ci_get(&a.ci, i) - b->hseqbase;
			double d;
			if (isf) {
				d = tp == ORA_flt ? (double) ((const float *) b->base)[p] : ((const double *) b->base)[p];
			} else {
				ora_hge v;
				d = val_at(b, p, &v) ? nan("") : (double) v;
			}
			((double *) bn->base)[i] = d;
		}
		if (cntp) {
			cn = ora_new(ORA_lng, ng, hb);
			for (uint64_t k = 0; k < ng; k++)
				((int64_t *) cn->base)[k] = 1;
			*cntp = cn;
		}
		*bnp = bn;
		return 0;
	}
	bn = ora_new(ORA_dbl, ng, hb);
	cn = ora_new(ORA_lng, ng, hb);
	ora_hge *avg = calloc(ng + 1, sizeof(ora_hge));
	int64_t *rem = calloc(ng + 1, 8);
	double *dbls = bn->base;
	int64_t *cnts = cn->base;
	memset(cnts, 0, ng * 8);
	for (uint64_t k = 0; k < ng; k++)
		dbls[k] = 0;
	for (uint64_t i = 0; i < a.ci.n; i++) {
		ora_oid gid;
		if (!aggr_gid(&a, i, &gid))
			continue;
		const uint64_t p = ci_get(&a.ci, i) - b->hseqbase;
		if (isf) {
			double x = tp == ORA_flt ? (double) ((const float *) b->base)[p] : ((const double *) b->base)[p];
			if (isnan(x)) {
				if (!skip_nils)
					cnts[gid] = INT64_MIN;
				continue;
			}
			if (cnts[gid] == INT64_MIN)
				continue;
			double *av = &dbls[gid];
			const double n = (double) ++cnts[gid];
			if ((*av > 0) == (x > 0))
				*av += (x - *av) / n;
			else
				*av = *av - *av / n + x / n;
			continue;
		}
		ora_hge x;
		if (val_at(b, p, &x)) {
			if (!skip_nils)
				cnts[gid] = INT64_MIN;
			continue;
		}
		if (cnts[gid] == INT64_MIN)
			continue;
		/* AVERAGE_ITER: a + r/n is the running average, 0 <= r < n */
		ora_hge *av = &avg[gid];
		const int64_t n = ++cnts[gid];
		ora_hge an = *av / n, xn = x / n, z1 = xn - an;
		xn = x - xn * n;
		an = *av - an * n;
		unsigned __int128 z2;
		if (xn >= an) {
			z2 = (unsigned __int128) (xn - an);
			while (z2 >= (unsigned __int128) n) {
				z2 -= (unsigned __int128) n;
				z1++;
			}
		} else {
			z2 = (unsigned __int128) (an - xn);
			for (;;) {
				z1--;
				if (z2 < (unsigned __int128) n) {
					z2 = (unsigned __int128) n - z2;
					break;
				}
				z2 -= (unsigned __int128) n;
			}
		}
		*av += z1;
		rem[gid] += (int64_t) z2;
		if (rem[gid] >= n) {
			rem[gid] -= n;
			(*av)++;
		}
	}
	bool nils = false;
	for (uint64_t k = 0; k < ng; k++) {
		if (cnts[k] == 0 || cnts[k] == INT64_MIN) {
			dbls[k] = nan("");
			cnts[k] = 0;
			nils = true;
		} else if (!isf) {
			dbls[k] = (double) avg[k] + (double) rem[k] / cnts[k];
		}
	}
	if (scale != 0) {
		const double fac = pow(10.0, (double) scale);
		for (uint64_t k = 0; k < ng; k++)
			if (!isnan(dbls[k]))
				dbls[k] /= fac;
	}
	bn->nil = nils;
	bn->nonil = !nils;
	free(avg);
	free(rem);
	*bnp = bn;
	if (cntp)
		*cntp = cn;
	else
		ora_free(cn);
	return 0;
}

/* BATgroupmin / BATgroupmax (gdk/gdk_aggr.c:3487-3560, do_groupmin
 * :3247-3362, AGGR_CMP :3207-3240): the POSITION (oid) of each group's
 * minimum / maximum -- the first row holding it; without skip_nils the
 * first nil of the group wins; groups without a value give oid_nil.  MAL's
 * aggr.min / aggr.max project b through it (monetdb5/modules/kernel/aggr.c:
 * 321-348). */
ora_bat *
ora_groupminmax(const ora_bat *b, const ora_bat *g, const ora_bat *e,
		const ora_bat *s, bool skip_nils, bool domax)
{
	aggr_ctx a;
	if (aggr_init(&a, b, g, e, s) < 0)
		return NULL;
	ora_bat *bn = ora_new(ORA_oid, a.ngrp, a.ngrp ? a.min : 0);
	ora_hge *best = calloc(a.ngrp + 1, sizeof(ora_hge));
	uint8_t *isn = calloc(a.ngrp + 1, 1);
	if (!bn || !best || !isn) {
		ora_free(bn); free(best); free(isn);
		return NULL;
	}
	ora_oid *oids = bn->base;
	for (uint64_t k = 0; k < a.ngrp; k++)
		oids[k] = ORA_OID_NIL;
	for (uint64_t i = 0; i < a.ci.n; i++) {
		ora_oid gid;
		if (!aggr_gid(&a, i, &gid))
			continue;
		ora_oid o = ci_get(&a.ci, i);
		ora_hge v;
		bool vn = val_at(b, o - b->hseqbase, &v);
		if (skip_nils && vn)
			continue;
		if (oids[gid] == ORA_OID_NIL) {
			oids[gid] = o;
			best[gid] = v;
			isn[gid] = vn;
		} else if (!isn[gid] && (vn || (domax ? v > best[gid] : v < best[gid]))) {
			oids[gid] = o;
			best[gid] = v;
			isn[gid] = vn;
		}
	}
	uint64_t nils = 0;
	for (uint64_t k = 0; k < a.ngrp; k++)
		nils += oids[k] == ORA_OID_NIL;
	bn->sorted = bn->revsorted = bn->key = a.ngrp <= 1;
	if (a.ci.n == 0)          /* BATconstant(..., oid_nil, ngrp) */
		bn->sorted = bn->revsorted = 1;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	free(best);
	free(isn);
	return bn;
}

/* ---------------------------------------------------------------------- */


/* ---------------------------------------------------------------------- */
/* RANGE frame bounds (gdk/gdk_analytic_bounds.c:994-1294, kernels
 * :273-387, special cases :614 allbounds and :710 peers): partitions start
 * where p is true (and at row 0); PRECEDING walks back from row k while
 * |b[k]-b[j]| <= limit and gives the first row of that run; FOLLOWING walks
 * forward and gives one past the last row; a nil row's frame is its run of
 * nils; a limit of GDK_lng_max is "unbounded".  Results are absolute row
 * numbers.  Supports lng values with a lng limit. */

/* ---------------------------------------------------------------------- */
/* statistics (gdk/gdk_aggr.c:4255-5202): Welford updates per group in
 * candidate order.  AGGR_STDEV (:4561-4601) for dogroupstdev (:4612-4775),
 * AGGR_COVARIANCE (:4808-4848) for dogroupcovariance (:4851-4997),
 * AGGR_CORRELATION (:5013-5054) for BATgroupcorrelation (:5057-5202); the
 * _SINGLE loops (:4257, :4382, :4478) for calcvariance (:4276),
 * calccovariance (:4404) and BATcalccorrelation (:4503).  A nil value makes
 * its group nil for good unless skip_nils (cnts = BUN_NONE); the whole-column
 * forms skip nils and stop with an overflow error at the first infinite
 * accumulator, the grouped ones check the final accumulators. */

#define ST_VAR 0
#define ST_COV 1
#define ST_COR 2
#define CNT_NONE (~(uint64_t) 0)

/* (dbl) of row p; true when nil */
static bool
dbl_at(const ora_bat *b, uint64_t p, double *d)
{
	if (b->type == ORA_flt) {
		*d = ((const float *) b->base)[p];
		return isnan(*d);
	}
	if (b->type == ORA_dbl) {
		*d = ((const double *) b->base)[p];
		return isnan(*d);
	}
	ora_hge v;
	const bool nil = val_at(b, p, &v);
	*d = (double) v;
	return nil;
}

static bool
moment_type(int tp)
{
	return tp == ORA_bte || tp == ORA_sht || tp == ORA_int || tp == ORA_lng || tp == ORA_hge ||
	       tp == ORA_flt || tp == ORA_dbl;
}

static ora_bat *
const_dbl(ora_oid hseq, double v, uint64_t n)
{
	ora_bat *bn = ora_new(ORA_dbl, n, hseq);
	for (uint64_t k = 0; k < n; k++)
		((double *) bn->base)[k] = v;
	bn->sorted = bn->revsorted = 1;
	bn->key = n <= 1;
	bn->nil = n > 0 && isnan(v);
	bn->nonil = !bn->nil;
	return bn;
}

struct moments {
	uint64_t cnt;
	double mean1, mean2, m2, up, down1, down2;
};

/* one Welford step; returns true when the whole-column form overflows */
static bool
moment_step(struct moments *m, int kind, double x, double y, bool single)
{
	m->cnt++;
	const double n = (double) m->cnt;
	const double delta1 = x - m->mean1;
	m->mean1 += delta1 / n;
	if (kind == ST_VAR) {
		m->m2 += delta1 * (x - m->mean1);
		return single && isinf(m->m2);
	}
	const double delta2 = y - m->mean2;
	m->mean2 += delta2 / n;
	if (kind == ST_COV) {
		m->m2 += delta1 * (y - m->mean2);
		return single && isinf(m->m2);
	}
	const double aux = y - m->mean2;
	m->up += delta1 * aux;
	m->down1 += delta1 * (x - m->mean1);
	m->down2 += delta2 * aux;
	return single && (isinf(m->up) || isinf(m->down1) || isinf(m->down2));
}

ora_bat *
ora_groupmoments(int kind, const ora_bat *b1, const ora_bat *b2, const ora_bat *g, const ora_bat *e,
		 const ora_bat *s, bool skip_nils, bool issample, bool variance)
{
	aggr_ctx a;
	if (g == NULL) {
		ora_seterr("b and g must be aligned\n");
		return NULL;
	}
	if (kind != ST_VAR && (b2 == NULL || b1->count != b2->count || b1->type != b2->type)) {
		ora_seterr("b1 and b2 must be aligned\n");
		return NULL;
	}
	if (aggr_init(&a, b1, g, e, s) < 0)
		return NULL;
	const uint64_t ng = a.ngrp;
	if (b1->count == 0 || ng == 0)
		return const_dbl(ng ? a.min : 0, nan(""), ng);
	const bool singles = g->tseqbase != ORA_OID_NIL || (g->key && g->nonil);
	if (kind == ST_VAR) {
		/* :4652-4661 */
		if ((e == NULL || (e->count == a.ci.n && e->hseqbase == b1->hseqbase)) && singles &&
		    (issample || b1->nonil))
			return const_dbl(a.min, issample ? nan("") : 0.0, ng);
	} else if ((e == NULL || (e->count == b1->count &&
				  (e->hseqbase == b1->hseqbase || e->hseqbase == b2->hseqbase))) && singles) {
		/* :4887-4896, :5091-5097 */
		if (kind == ST_COR)
			return const_dbl(a.min, nan(""), ng);
		if (issample || (b1->nonil && b2->nonil))
			return const_dbl(a.min, issample ? nan("") : 0.0, ng);
	}
	if (!moment_type(b1->type)) {
		ora_seterr("type (%d) not supported.\n", b1->type);
		return NULL;
	}
	struct moments *m = calloc(ng, sizeof(*m));
	for (uint64_t i = 0; i < a.ci.n; i++) {
		ora_oid gid;
		if (!aggr_gid(&a, i, &gid))
			continue;
		const uint64_t p = ci_get(&a.ci, i) - b1->hseqbase;
		double x, y = 0;
		bool nil = dbl_at(b1, p, &x);
		if (kind != ST_VAR)
			nil |= dbl_at(b2, p, &y);
		if (nil) {
			if (!skip_nils)
				m[gid].cnt = CNT_NONE;
		} else if (m[gid].cnt != CNT_NONE) {
			moment_step(&m[gid], kind, x, y, false);
		}
	}
	ora_bat *bn = ora_new(ORA_dbl, ng, a.min);
	double *dbls = bn->base;
	uint64_t nils = 0;
	for (uint64_t k = 0; k < ng; k++) {
		const struct moments *q = &m[k];
		if (kind == ST_COR) {
			if (q->cnt <= 1 || q->cnt == CNT_NONE || q->down1 == 0 || q->down2 == 0) {
				dbls[k] = nan("");
				nils++;
			} else if (isinf(q->up) || isinf(q->down1) || isinf(q->down2)) {
				goto overflow;
			} else {
				const double n = (double) q->cnt;
				dbls[k] = (q->up / n) / (sqrt(q->down1 / n) * sqrt(q->down2 / n));
			}
		} else if (q->cnt == 0 || q->cnt == CNT_NONE) {
			dbls[k] = nan("");
			nils++;
		} else if (q->cnt == 1) {
			dbls[k] = issample ? nan("") : 0;
			nils += issample;
		} else if (isinf(q->m2)) {
			goto overflow;
		} else {
			dbls[k] = q->m2 / (double) (q->cnt - issample);
			if (kind == ST_VAR && !variance)
				dbls[k] = sqrt(dbls[k]);
		}
	}
	free(m);
	bn->sorted = bn->revsorted = bn->key = ng <= 1;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	return bn;
overflow:
	free(m);
	ora_free(bn);
	ora_seterr("22003!overflow in calculation.\n");
	return NULL;
}

int
ora_calcmoments(double *res, double *avgp, int kind, const ora_bat *b1, const ora_bat *b2, bool issample,
		bool variance)
{
	*res = nan("");
	if (avgp)
		*avgp = nan("");
	if (!moment_type(b1->type)) {
		ora_seterr("type (%d) not supported.\n", b1->type);
		return -1;
	}
	if (kind != ST_VAR && (b2 == NULL || b1->count != b2->count || b1->type != b2->type)) {
		ora_seterr("b1 and b2 must be aligned\n");
		return -1;
	}
	struct moments m = {0};
	for (uint64_t i = 0; i < b1->count; i++) {
		double x, y = 0;
		bool nil = dbl_at(b1, i, &x);
		if (kind != ST_VAR)
			nil |= dbl_at(b2, i, &y);
		if (nil)
			continue;
		if (moment_step(&m, kind, x, y, true)) {
			ora_seterr("22003!overflow in calculation.\n");
			return -1;
		}
	}
	if (kind == ST_COR) {
		const double n = (double) m.cnt;
		if (m.cnt != 0 && m.down1 != 0 && m.down2 != 0)
			*res = (m.up / n) / (sqrt(m.down1 / n) * sqrt(m.down2 / n));
		return 0;
	}
	if (m.cnt <= (uint64_t) issample)
		return 0;
	if (avgp)
		*avgp = m.mean1;
	*res = m.m2 / (double) (m.cnt - issample);
	if (kind == ST_VAR && !variance)
		*res = sqrt(*res);   /* BATcalcstdev_*: is_dbl_nil(v) ? dbl_nil : sqrt(v) */
	return 0;
}

/* ---------------------------------------------------------------------- */
/* doBATgroupquantile (gdk/gdk_aggr.c:3881-4222): b (and g) at the candidates
 * (BATproject(s, .)), g sorted, b sorted within the groups (BATsort twice);
 * per run of equal group ids (in sorted order) the value at
 * r + p - (BUN) (p + 0.5 - f), f = (p - r - 1) * quantile, r past the nils
 * with skip_nils; the _avg forms interpolate the two neighbours in dbl
 * (DO_QUANTILE_AVG :3860).  Results go to consecutive positions, nil padded
 * to ngrp (:4073-4077); dense g: a copy of b (:3968-3981). */

static bool
nil_at(const ora_bat *b, uint64_t p)
{
	double d;
	if (b->type == ORA_flt || b->type == ORA_dbl)
		return dbl_at(b, p, &d);
	const char *x = (const char *) b->base + p * b->width;
	switch (b->type) {
	case ORA_daytime: case ORA_timestamp: return *(const int64_t *) x == INT64_MIN;
	default: { ora_hge v; return val_at(b, p, &v); }
	}
}

static void
set_nil(ora_bat *bn, uint64_t k)
{
	char *x = (char *) bn->base + k * bn->width;
	switch (bn->type) {
	case ORA_flt: ((float *) bn->base)[k] = nanf(""); break;
	case ORA_dbl: ((double *) bn->base)[k] = nan(""); break;
	case ORA_bit: case ORA_bte: *(int8_t *) x = INT8_MIN; break;
	case ORA_sht: *(int16_t *) x = INT16_MIN; break;
	case ORA_int: case ORA_date: *(int32_t *) x = INT32_MIN; break;
	case ORA_hge: *(ora_hge *) x = HGE_NIL; break;
	default: *(int64_t *) x = INT64_MIN; break;   /* lng, oid, daytime, timestamp */
	}
}

/* the quantile of the sorted run [r, p) of v into bn[k]; true when nil */
static bool
quantile_of(ora_bat *bn, uint64_t k, const ora_bat *v, uint64_t r, uint64_t p, double quantile, bool skip_nils,
	    bool average)
{
	if (skip_nils)
		while (r < p && nil_at(v, r))
			r++;
	if (r == p) {
		set_nil(bn, k);
		return true;
	}
	const double f = (double) (p - r - 1) * quantile;
	if (average) {
		const double lo = floor(f), hi = ceil(f);
		double low, high;
		/* DO_QUANTILE_AVG: low from idxhi, high from idxlo */
		const bool n1 = dbl_at(v, r + (uint64_t) hi, &low), n2 = dbl_at(v, r + (uint64_t) lo, &high);
		if (n1 || n2) {
			set_nil(bn, k);
			return true;
		}
		((double *) bn->base)[k] = (f - lo) * low + (lo + 1 - f) * high;
		return false;
	}
	const uint64_t qi = r + p - (uint64_t) ((double) p + 0.5 - f);
	memcpy((char *) bn->base + k * bn->width, (const char *) v->base + qi * v->width, v->width);
	return nil_at(v, qi);
}

ora_bat *
ora_groupquantile(const ora_bat *b, const ora_bat *g, const ora_bat *e, const ora_bat *s, double quantile,
		  bool skip_nils, bool average)
{
	if (average && !moment_type(b->type)) {
		ora_seterr("incompatible type\n");
		return NULL;
	}
	ora_oid min = 0;
	uint64_t ngrp = 1;
	aggr_ctx a;
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return NULL;
	if (g) {
		if (aggr_init(&a, b, g, e, s) < 0)
			return NULL;
		min = a.min;
		ngrp = a.ngrp;
	}
	if (quantile < 0 || quantile > 1) {
		ora_seterr("cannot determine quantile for p=%f (p has to be in [0,1])\n", quantile);
		return NULL;
	}
	const int rt = average ? ORA_dbl : b->type;
	if (b->count == 0 || ngrp == 0 || isnan(quantile)) {
		ora_bat *bn = ora_new(rt, ngrp, ngrp == 0 ? 0 : min);
		for (uint64_t k = 0; k < ngrp; k++)
			set_nil(bn, k);
		bn->sorted = bn->revsorted = 1;
		bn->key = ngrp <= 1;
		bn->nil = ngrp > 0;
		bn->nonil = ngrp == 0;
		return bn;
	}
	/* BATproject(s, g): g is aligned with the candidates */
	if (g && !ci.dense && ci.n && ci_get(&ci, ci.n - 1) - ci_get(&ci, 0) + 1 != ci.n) {
		ora_seterr("BATproject: does not match always\n");
		return NULL;
	}
	/* b at the candidates, head aligned with g */
	ora_bat *bv = ora_new(b->type, ci.n, g ? g->hseqbase : 0);
	for (uint64_t i = 0; i < ci.n; i++)
		memcpy((char *) bv->base + i * bv->width,
		       (const char *) b->base + (ci_get(&ci, i) - b->hseqbase) * b->width, b->width);
	if (g && g->tseqbase != ORA_OID_NIL) {
		ora_bat *bn = ora_new(rt, ci.n, g->tseqbase);
		for (uint64_t i = 0; i < ci.n; i++) {
			if (average) {
				double d;
				if (dbl_at(bv, i, &d))
					d = nan("");
				((double *) bn->base)[i] = d;
			} else {
				memcpy((char *) bn->base + i * bn->width, (const char *) bv->base + i * bv->width, bv->width);
			}
		}
		ora_free(bv);
		return bn;
	}
	ora_bat *sv = NULL, *gs = NULL, *go = NULL;
	if (g) {
		ora_bat *gp = (ora_bat *) g;
		if (ora_BATsort(&gs, &go, NULL, gp, NULL, NULL, false, false, false) < 0 ||
		    ora_BATsort(&sv, NULL, NULL, bv, go, gs, false, false, false) < 0) {
			ora_free(bv);
			ora_free(gs);
			ora_free(go);
			return NULL;
		}
	} else if (ora_BATsort(&sv, NULL, NULL, bv, NULL, NULL, false, false, false) < 0) {
		ora_free(bv);
		return NULL;
	}
	ora_bat *bn = ora_new(rt, ngrp, g ? min : 0);
	uint64_t nils = 0, k = 0;
	if (g) {
		for (uint64_t r = 0, p; r < ci.n; r = p, k++) {
			ora_hge gr, gq;
			val_at(gs, r, &gr);
			for (p = r + 1; p < ci.n; p++) {
				val_at(gs, p, &gq);
				if (gq != gr)
					break;
			}
			if (k >= ngrp) {
				ora_seterr("BATgroupquantile: more group ids than groups\n");
				ora_free(bn);
				bn = NULL;
				goto done;
			}
			nils += quantile_of(bn, k, sv, r, p, quantile, skip_nils, average);
		}
	} else {
		nils += quantile_of(bn, 0, sv, 0, ci.n, quantile, skip_nils, average);
		k = 1;
	}
	for (; k < ngrp; k++) {
		set_nil(bn, k);
		nils++;
	}
	bn->sorted = bn->revsorted = bn->key = ngrp <= 1;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
done:
	ora_free(bv);
	ora_free(sv);
	ora_free(gs);
	ora_free(go);
	return bn;
}

/* ---------------------------------------------------------------------- */
/* BATmin_skipnil / BATmax_skipnil (gdk/gdk_aggr.c:3570-3844): a cached
 * minpos / maxpos first; an ordered column (BATordered / BATordered_rev,
 * nil the smallest value) answers from its end -- min: the first non-nil
 * row of a sorted column (skipnil) or its first row, the row before the
 * first nil of a reverse-sorted one (skipnil) or its last row; max: the last
 * row of a sorted column, the first of a reverse-sorted one, nil when that
 * row is nil and skipnil -- else do_groupmin / do_groupmax over all rows:
 * the first row holding the extreme, without skipnil the first nil.  The
 * value at that row is copied to res (str: *sres points at the string);
 * the row is cached in the descriptor.  Returns 0, -1 on error. */

/* val_at with the 8-byte temporal types */
static bool
mm_val(const ora_bat *b, uint64_t p, ora_hge *v)
{
	if (b->type == ORA_daytime || b->type == ORA_timestamp) {
		const int64_t x = ((const int64_t *) b->base)[p];
		*v = x;
		return x == INT64_MIN;
	}
	return val_at(b, p, v);
}

/* three-way compare of rows p, q (nil the smallest; flt / dbl compare as
 * doubles, -0.0 == +0.0; str by strcmp) */
static int
mm_cmp(const ora_bat *b, uint64_t p, uint64_t q)
{
	if (b->type == ORA_str) {
		const char *x = str_of(b, p), *y = str_of(b, q);
		const bool nx = (unsigned char) x[0] == 0x80 && x[1] == 0, ny = (unsigned char) y[0] == 0x80 && y[1] == 0;
		if (nx || ny)
			return ny - nx;
		int r = strcmp(x, y);
		return (r > 0) - (r < 0);
	}
	if (b->type == ORA_flt || b->type == ORA_dbl) {
		double x, y;
		const bool nx = dbl_at(b, p, &x), ny = dbl_at(b, q, &y);
		if (nx || ny)
			return ny - nx;
		return (x > y) - (x < y);
	}
	ora_hge x, y;
	const bool nx = mm_val(b, p, &x), ny = mm_val(b, q, &y);
	if (nx || ny)
		return ny - nx;
	return (x > y) - (x < y);
}

static bool
mm_nil(const ora_bat *b, uint64_t p)
{
	if (b->type == ORA_str) {
		const char *x = str_of(b, p);
		return (unsigned char) x[0] == 0x80 && x[1] == 0;
	}
	if (b->type == ORA_flt || b->type == ORA_dbl) {
		double d;
		return dbl_at(b, p, &d);
	}
	ora_hge v;
	return mm_val(b, p, &v);
}

static bool
mm_ordered(ora_bat *b, bool rev)
{
	if (rev ? b->revsorted : b->sorted)
		return true;
	for (uint64_t p = 1; p < b->count; p++) {
		const int c = mm_cmp(b, p - 1, p);
		if (rev ? c < 0 : c > 0)
			return false;
	}
	if (rev)
		b->revsorted = 1;
	else
		b->sorted = 1;
	return true;
}

int
ora_minmax(ora_bat *b, bool skipnil, bool domax, void *res, const char **sres)
{
	const uint64_t n = b->count;
	uint64_t pos = ORA_BUN_NONE;
	const uint64_t cached = domax ? b->maxpos : b->minpos;
	if (b->type == ORA_msk) {
		ora_seterr("non-linear type");
		return -1;
	}
	if (n == 0) {
		pos = ORA_BUN_NONE;
	} else if (b->type == ORA_void) {
		const ora_oid v = b->tseqbase == ORA_OID_NIL ? ORA_OID_NIL : b->tseqbase + (domax ? n - 1 : 0);
		memcpy(res, &v, 8);
		return 0;
	} else if (cached != ORA_BUN_NONE && cached < n) {
		pos = cached;
	} else {
		const bool asc = mm_ordered(b, false), desc = !asc && mm_ordered(b, true);
		if (asc || desc) {
			if (!domax) {
				if (skipnil && !b->nonil) {
					uint64_t q = 0;
					if (asc) {
						while (q < n && mm_nil(b, q))
							q++;
						pos = q == n ? ORA_BUN_NONE : q;
					} else {
						while (q < n && !mm_nil(b, q))
							q++;
						pos = q == 0 ? ORA_BUN_NONE : q - 1;
					}
				} else {
					pos = asc ? 0 : n - 1;
				}
			} else {
				pos = asc ? n - 1 : 0;
				if (skipnil && !b->nonil && mm_nil(b, pos))
					pos = ORA_BUN_NONE;
			}
		} else {
			/* do_groupmin / do_groupmax over all rows */
			uint64_t best = ORA_BUN_NONE;
			bool bnil = false;
			for (uint64_t p = 0; p < n; p++) {
				const bool vn = mm_nil(b, p);
				if (skipnil && vn)
					continue;
				if (best == ORA_BUN_NONE) {
					best = p;
					bnil = vn;
				} else if (!bnil && (vn || (domax ? mm_cmp(b, p, best) > 0 : mm_cmp(b, p, best) < 0))) {
					best = p;
					bnil = vn;
				}
			}
			pos = best;
		}
		if (pos != ORA_BUN_NONE) {
			if (domax)
				b->maxpos = pos;
			else
				b->minpos = pos;
		}
	}
	if (b->type == ORA_str) {
		*sres = pos == ORA_BUN_NONE ? "\200" : str_of(b, pos);
		return 0;
	}
	if (pos == ORA_BUN_NONE) {
		switch (b->type) {
		case ORA_flt: { const float f = NAN; memcpy(res, &f, 4); break; }
		case ORA_dbl: { const double f = NAN; memcpy(res, &f, 8); break; }
		default: put(b->type == ORA_date ? ORA_int : b->type == ORA_daytime || b->type == ORA_timestamp ? ORA_lng : b->type,
			     res, 0, 0, true); break;
		}
		return 0;
	}
	memcpy(res, (const char *) b->base + pos * b->width, b->width);
	return 0;
}

/* ---------------------------------------------------------------------- */
/* BATprod (gdk/gdk_aggr.c:1650) / BATgroupprod (:1575) through doprod
 * (:1340-1548): per group, in candidate order, the macro doprod picks for
 * the result type -- AGGR_PROD (integer results up to lng: a nil value makes
 * the product nil unless skip_nils, a group's first value resets it to 1
 * when nil_if_empty, so nils before it are forgotten; multiply with the
 * overflow check |p| <= max of MULI4_WITH_CHECK), AGGR_PROD_HGE (hge: any row
 * marks the group seen, HGEMUL_CHECK), AGGR_PROD_FLOAT (flt / dbl: as
 * AGGR_PROD with "|v| > 1 && max / |v| < |p|" as the overflow test).  An
 * overflow is "22003!overflow in product aggregate." */

static int
prod_kind(int tp1, int tp2)
{
	switch (tp2) {
	case ORA_bte: return tp1 == ORA_bte ? 0 : -1;
	case ORA_sht: return tp1 == ORA_bte || tp1 == ORA_sht ? 0 : -1;
	case ORA_int: return tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int ? 0 : -1;
	case ORA_lng: return tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int || tp1 == ORA_lng ? 0 : -1;
	case ORA_hge:
		return tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int || tp1 == ORA_lng || tp1 == ORA_hge ? 1 : -1;
	case ORA_flt:
		return tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int || tp1 == ORA_lng || tp1 == ORA_hge ||
			tp1 == ORA_flt ? 2 : -1;
	case ORA_dbl:
		return tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int || tp1 == ORA_lng || tp1 == ORA_hge ||
			tp1 == ORA_flt || tp1 == ORA_dbl ? 2 : -1;
	}
	return -1;
}

/* the running state of one group */
typedef struct {
	ora_hge ip;        /* integer product */
	double fp;         /* float product (flt results rounded to float each step) */
	bool nil, seen;
} pstate;

/* one row; false on overflow */
static bool
prod_step(pstate *s, int kind, int tp1, int tp2, const ora_bat *b, uint64_t p, bool skip_nils, bool nil_if_empty)
{
	bool vn;
	ora_hge iv = 0;
	double fv = 0;
	if (tp1 == ORA_flt || tp1 == ORA_dbl)
		vn = dbl_at(b, p, &fv);
	else
		vn = val_at(b, p, &iv);
	if (kind == 1 && nil_if_empty && !s->seen) {
		s->seen = true;
		s->nil = false;
		s->ip = 1;
	}
	if (vn) {
		if (!skip_nils)
			s->nil = true;
		return true;
	}
	if (kind != 1 && nil_if_empty && !s->seen) {
		s->seen = true;
		s->nil = false;
		s->ip = 1;
		s->fp = 1;
	}
	if (s->nil)
		return true;
	if (kind == 2) {
		/* C's arithmetic: the value converted to the result type */
		if (tp2 == ORA_flt) {
			const float x = tp1 == ORA_flt ? (float) fv : (float) iv;
			const float ax = x < 0 ? -x : x, ap = (float) s->fp < 0 ? -(float) s->fp : (float) s->fp;
			if (ax > 1 && FLT_MAX / ax < ap)
				return false;
			s->fp = (float) ((float) s->fp * x);
		} else {
			const double x = tp1 == ORA_flt || tp1 == ORA_dbl ? fv : (double) iv;
			const double ax = x < 0 ? -x : x, ap = s->fp < 0 ? -s->fp : s->fp;
			if (ax > 1 && DBL_MAX / ax < ap)
				return false;
			s->fp = s->fp * x;
		}
		return true;
	}
	ora_hge r;
	if (__builtin_mul_overflow(iv, s->ip, &r))
		return false;
	const ora_hge mx = tmax(tp2);
	if (r > mx || r < -mx)
		return false;
	s->ip = r;
	return true;
}

static void
prod_put(int tp2, void *base, uint64_t i, const pstate *s)
{
	if (tp2 == ORA_flt)
		((float *) base)[i] = s->nil ? NAN : (float) s->fp;
	else if (tp2 == ORA_dbl)
		((double *) base)[i] = s->nil ? NAN : s->fp;
	else
		put(tp2, base, i, s->ip, s->nil);
}

int
ora_prod(void *res, int tp, const ora_bat *b, const ora_bat *s, bool skip_nils, bool nil_if_empty)
{
	const int kind = prod_kind(b->type, tp);
	if (kind < 0) {
		ora_seterr("type combination (prod) not supported");
		return -1;
	}
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return -1;
	pstate st = {.ip = 1, .fp = 1, .nil = nil_if_empty, .seen = false};
	for (uint64_t i = 0; i < ci.n; i++)
		if (!prod_step(&st, kind, b->type, tp, b, ci_get(&ci, i) - b->hseqbase, skip_nils, nil_if_empty)) {
			ora_seterr("22003!overflow in product aggregate.\n");
			return -1;
		}
	prod_put(tp, res, 0, &st);
	return 0;
}

ora_bat *
ora_groupprod(const ora_bat *b, const ora_bat *g, const ora_bat *e, const ora_bat *s, int tp, bool skip_nils)
{
	aggr_ctx a;
	if (aggr_init(&a, b, g, e, s) < 0)
		return NULL;
	const int kind = prod_kind(b->type, tp);
	if (kind < 0 && a.ci.n && a.ngrp) {
		ora_seterr("type combination (prod) not supported");
		return NULL;
	}
	ora_bat *bn = ora_new(tp, a.ngrp, a.ngrp ? a.min : 0);
	pstate *st = malloc((a.ngrp + 1) * sizeof(pstate));
	if (!bn || !st) {
		ora_free(bn);
		free(st);
		return NULL;
	}
	for (uint64_t k = 0; k < a.ngrp; k++)
		st[k] = (pstate) {.ip = 1, .fp = 1, .nil = true, .seen = false};
	for (uint64_t i = 0; i < a.ci.n; i++) {
		ora_oid gid;
		if (!aggr_gid(&a, i, &gid))
			continue;
		if (!prod_step(&st[gid], kind, b->type, tp, b, ci_get(&a.ci, i) - b->hseqbase, skip_nils, true)) {
			ora_free(bn);
			free(st);
			ora_seterr("22003!overflow in product aggregate.\n");
			return NULL;
		}
	}
	uint64_t nils = 0;
	for (uint64_t k = 0; k < a.ngrp; k++) {
		prod_put(tp, bn->base, k, &st[k]);
		nils += st[k].nil;
	}
	free(st);
	bn->sorted = bn->revsorted = bn->key = a.ngrp <= 1;
	bn->nil = nils != 0;
	bn->nonil = nils == 0;
	return bn;
}

/* BATcalcavg (gdk/gdk_aggr.c:2987-3044): the average of b[s] without nils.
 * Integers: the sum in hge (AVERAGE_TYPE_LNG_HGE :2905-2924), (dbl) sum / n;
 * a sum that leaves hge -- only an hge column can -- is refused, as the
 * device refuses it (the reference continues with its remainder recurrence,
 * :2925-2958).  flt / dbl: AVERAGE_ITER_FLOAT in candidate order
 * (AVERAGE_FLOATTYPE :2970-2984).  scale divides a non-nil result by
 * 10^scale (:3036-3037); *vals = the number of non-nil values. */
int
ora_calcavg(const ora_bat *b, const ora_bat *s, double *avg, uint64_t *vals, int scale)
{
	const int tp = b->type;
	*avg = nan("");
	if (tp != ORA_bte && tp != ORA_sht && tp != ORA_int && tp != ORA_lng && tp != ORA_hge && tp != ORA_flt &&
	    tp != ORA_dbl) {
		ora_seterr("average of type %d unsupported.\n", tp);
		return -1;
	}
	ora_ci ci;
	if (ora_ci_init(&ci, b, s) < 0)
		return -1;
	uint64_t n = 0;
	double a = 0;
	if (tp == ORA_flt || tp == ORA_dbl) {
		for (uint64_t i = 0; i < ci.n; i++) {
			const uint64_t p = ci_get(&ci, i) - b->hseqbase;
			const double x = tp == ORA_flt ? (double) ((const float *) b->base)[p] : ((const double *) b->base)[p];
			if (isnan(x))
				continue;
			const double nn = (double) ++n;
			if ((a > 0) == (x > 0))
				a += (x - a) / nn;
			else
				a = a - a / nn + x / nn;
		}
		a = n > 0 ? a : nan("");
	} else {
		ora_hge sum = 0;
		const ora_hge max = (ora_hge) (((unsigned __int128) 1 << 127) - 1);
		for (uint64_t i = 0; i < ci.n; i++) {
			ora_hge x;
			if (val_at(b, ci_get(&ci, i) - b->hseqbase, &x))
				continue;
			if ((x > 0 && sum > max - x) || (x < 0 && sum < -max - x)) {
				ora_seterr("42000!BATcalcavg: hge sum exceeds the 128-bit device accumulator\n");
				return -1;
			}
			sum += x;
			n++;
		}
		a = n > 0 ? (double) sum / (double) n : nan("");
	}
	if (scale != 0 && !isnan(a))
		a /= pow(10.0, (double) scale);
	*avg = a;
	if (vals)
		*vals = n;
	return 0;
}

/* BATcount_no_nil (gdk/gdk_batop.c:3078): candidates with a non-nil value;
 * nonil / msk: every candidate, void: none when the sequence is nil */
uint64_t
ora_count_no_nil(const ora_bat *b, const ora_bat *s)
{
	ora_ci ci;
	uint64_t cnt = 0;
	if (ora_ci_init(&ci, b, s) < 0)
		return 0;
	if (b->nonil || b->type == ORA_msk)
		return ci.n;
	if (b->type == ORA_void)
		return b->tseqbase == ORA_OID_NIL ? 0 : ci.n;
	for (uint64_t i = 0; i < ci.n; i++) {
		uint64_t p = ci_get(&ci, i) - b->hseqbase;
		ora_hge v;
		if (b->type == ORA_str)
			cnt += (unsigned char) str_of(b, p)[0] != 0x80;
		else if (b->type == ORA_flt)
			cnt += ((const float *) b->base)[p] == ((const float *) b->base)[p];
		else if (b->type == ORA_dbl)
			cnt += ((const double *) b->base)[p] == ((const double *) b->base)[p];
		else if (b->type == ORA_daytime || b->type == ORA_timestamp)
			cnt += ((const int64_t *) b->base)[p] != INT64_MIN;
		else
			cnt += !val_at(b, p, &v);
	}
	return cnt;
}
