/*
 * gdk_oracle_analytic.c -- windowed aggregates over frames (TEST
 * INFRASTRUCTURE ONLY; see gdk_oracle.h).
 *
 * Restates gdk/gdk_analytic_func.c:
 *   GDKanalyticalsum   :1959 (frame kinds :1976-1996, per-kind loops
 *                      :1684-1815, partition walk ANALYTICAL_SUM_CALC :1819)
 *   GDKanalyticalcount :1626 (:1446-1624)
 * and the fanout-16 segment tree of gdk/gdk_analytic.h:52-130
 * (populate_segment_tree / compute_on_segment_tree) with its size rule
 * GDKrebuild_segment_tree (gdk_analytic_func.c:34-62).  Every addition is
 * checked like ADD_WITH_CHECK (gdk/gdk_calc_private.h:53): a result outside
 * [-max, max] of the result type is "22003!overflow in calculation.\n".
 *
 * Partitions: p[i] != 0 starts a partition at row i >= 1 (row 0 always
 * starts one); peers: o[i] != 0 starts a new peer group (ORDER BY value
 * change) -- the reference's np / op arrays.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gdk_oracle.h"

void ora_seterr(const char *fmt, ...);

#define FANOUT 16
#define HGE_MAX ((ora_hge) (((unsigned __int128) 1 << 127) - 1))

typedef struct {
	ora_hge max;       /* result type's max (range [-max, max]) */
	int ovf;
} acc_t;

/* sum, nil-aware: nil = "no value yet" (tp2 nil) */
typedef struct {
	ora_hge v;
	int nil;
} sval;

static sval
sadd(acc_t *a, sval cur, sval x)
{
	if (x.nil)
		return cur;
	if (cur.nil)
		return x;
	ora_hge r;
	if (__builtin_add_overflow(cur.v, x.v, &r) || r > a->max || r < -a->max) {
		a->ovf = 1;
		return cur;
	}
	cur.v = r;
	return cur;
}

static int
ival(const ora_bat *b, uint64_t i, ora_hge *v)
{
	const char *x = (const char *) b->base;
	switch (b->type) {
	case ORA_bte: *v = ((const int8_t *) x)[i]; return *v == INT8_MIN;
	case ORA_sht: *v = ((const int16_t *) x)[i]; return *v == INT16_MIN;
	case ORA_int: case ORA_date: *v = ((const int32_t *) x)[i]; return *v == INT32_MIN;
	case ORA_lng: *v = ((const int64_t *) x)[i]; return *v == INT64_MIN;
	default: return 1;
	}
}

static int
isnil_any(const ora_bat *b, uint64_t i)
{
	ora_hge v;
	switch (b->type) {
	case ORA_flt: { float f = ((const float *) b->base)[i]; return f != f; }
	case ORA_dbl: { double d = ((const double *) b->base)[i]; return d != d; }
	case ORA_oid: return ((const ora_oid *) b->base)[i] == ORA_OID_NIL;
	case ORA_hge: return ((const ora_hge *) b->base)[i] == -HGE_MAX - 1;
	default: return ival(b, i, &v);
	}
}

static void
put_sum(ora_bat *r, int tp2, uint64_t k, sval s)
{
	if (tp2 == ORA_lng)
		((int64_t *) r->base)[k] = s.nil ? INT64_MIN : (int64_t) s.v;
	else
		((ora_hge *) r->base)[k] = s.nil ? -HGE_MAX - 1 : s.v;
}

/* segment tree over n level-0 values (gdk_analytic.h:63-95) */
typedef struct {
	sval *tree;
	uint64_t *off;
	uint64_t nlevels;
} stree;

static int
st_build(stree *t, const sval *lv0, uint64_t n, acc_t *a)
{
	uint64_t total = n, c = n, nl = 1;
	do {
		c = (c + FANOUT - 1) / FANOUT;
		total += c;
		nl++;
	} while (c > 1);
	t->tree = malloc(total * sizeof(sval));
	t->off = malloc(nl * sizeof(uint64_t));
	t->nlevels = nl;
	if (!t->tree || !t->off)
		return -1;
	memcpy(t->tree, lv0, n * sizeof(sval));
	uint64_t to = n, lsize = n, prev = 0, cur = 1;
	t->off[0] = 0;
	while (cur < nl) {
		uint64_t prev_to = to;
		t->off[cur++] = to;
		for (uint64_t pos = 0; pos < lsize; pos += FANOUT) {
			uint64_t end = pos + FANOUT < lsize ? pos + FANOUT : lsize;
			sval acc = {0, 1};
			for (uint64_t x = pos; x < end; x++)
				acc = sadd(a, acc, t->tree[prev + x]);
			t->tree[to++] = acc;
		}
		prev = prev_to;
		lsize = to - prev_to;
	}
	return 0;
}

/* gdk_analytic.h:97-130 */
static sval
st_query(const stree *t, uint64_t begin, uint64_t tend, acc_t *a)
{
	sval acc = {0, 1};
	if (begin >= tend)
		return acc;
	for (uint64_t level = 0; level < t->nlevels; level++) {
		const sval *tl = t->tree + t->off[level];
		uint64_t pb = begin / FANOUT, pe = tend / FANOUT;
		if (pb == pe) {
			for (uint64_t pos = begin; pos < tend; pos++)
				acc = sadd(a, acc, tl[pos]);
			break;
		}
		uint64_t gb = pb * FANOUT;
		if (begin != gb) {
			for (uint64_t pos = begin; pos < gb + FANOUT; pos++)
				acc = sadd(a, acc, tl[pos]);
			pb++;
		}
		uint64_t ge = pe * FANOUT;
		if (tend != ge)
			for (uint64_t pos = ge; pos < tend; pos++)
				acc = sadd(a, acc, tl[pos]);
		begin = pb;
		tend = pe;
	}
	return acc;
}

static int
bit_at(const ora_bat *b, uint64_t i)
{
	return b && ((const int8_t *) b->base)[i] != 0;
}

int
ora_analyticalsum(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		  const ora_bat *e, int tp1, int tp2, int frame_type)
{
	if (!((tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int || tp1 == ORA_lng) &&
	      (tp2 == ORA_lng || tp2 == ORA_hge))) {
		ora_seterr("42000!type combination (sum(%d)->%d) not supported.\n", tp1, tp2);
		return -1;
	}
	const uint64_t cnt = b->count;
	acc_t a = {tp2 == ORA_lng ? (ora_hge) INT64_MAX : HGE_MAX, 0};
	sval *lv0 = malloc((cnt + 1) * sizeof(sval));
	if (!lv0)
		return -1;
	for (uint64_t i = 0; i < cnt; i++) {
		ora_hge v;
		lv0[i].nil = ival(b, i, &v);
		lv0[i].v = lv0[i].nil ? 0 : v;
	}
	const ora_oid *start = s ? s->base : NULL, *end = e ? e->base : NULL;
	int rc = 0;
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt && !a.ovf; i++) {
		if (i < cnt && !bit_at(p, i))
			continue;
		/* partition [k, i) */
		switch (frame_type) {
		case 3: {   /* unbounded preceding .. current row (+ peers) */
			sval cur = {0, 1};
			while (k < i) {
				uint64_t j = k;
				do {
					cur = sadd(&a, cur, lv0[k]);
					k++;
				} while (k < i && !bit_at(o, k));
				for (; j < k; j++)
					put_sum(r, tp2, j, cur);
			}
			break;
		}
		case 4: {   /* current row (+ peers) .. unbounded following */
			sval cur = {0, 1};
			uint64_t l = i - 1;
			for (uint64_t j = l;; j--) {
				cur = sadd(&a, cur, lv0[j]);
				if (bit_at(o, j) || j == k) {
					for (;; l--) {
						put_sum(r, tp2, l, cur);
						if (l == j)
							break;
					}
					if (j == k)
						break;
					l = j - 1;
				}
			}
			k = i;
			break;
		}
		case 5: {   /* all rows of the partition */
			sval cur = {0, 1};
			for (uint64_t j = k; j < i; j++)
				cur = sadd(&a, cur, lv0[j]);
			for (; k < i; k++)
				put_sum(r, tp2, k, cur);
			break;
		}
		case 6:     /* current row */
			for (; k < i; k++)
				put_sum(r, tp2, k, lv0[k]);
			break;
		default: {  /* frames [start, end) through the segment tree */
			stree t = {0};
			const uint64_t j = k;
			if (st_build(&t, lv0 + j, i - j, &a) < 0) {
				free(t.tree);
				free(t.off);
				rc = -1;
				break;
			}
			for (; k < i && !a.ovf; k++)
				put_sum(r, tp2, k, st_query(&t, start[k] - j, end[k] - j, &a));
			free(t.tree);
			free(t.off);
			break;
		}
		}
		if (rc < 0)
			break;
	}
	free(lv0);
	if (rc < 0)
		return -1;
	if (a.ovf) {
		ora_seterr("22003!overflow in calculation.\n");
		return -1;
	}
	r->count = cnt;
	return 0;
}

int
ora_analyticalcount(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		    const ora_bat *e, bool ignore_nils, int frame_type)
{
	const uint64_t cnt = b->count;
	const bool count_all = !ignore_nils || b->nonil;
	int64_t *rb = r->base;
	const ora_oid *start = s ? s->base : NULL, *end = e ? e->base : NULL;
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt; i++) {
		if (i < cnt && !bit_at(p, i))
			continue;
		switch (frame_type) {
		case 3: {
			int64_t cur = 0;
			while (k < i) {
				uint64_t j = k;
				do {
					cur += count_all || !isnil_any(b, k);
					k++;
				} while (k < i && !bit_at(o, k));
				for (; j < k; j++)
					rb[j] = cur;
			}
			break;
		}
		case 4: {
			int64_t cur = 0;
			uint64_t l = i - 1;
			for (uint64_t j = l;; j--) {
				cur += count_all || !isnil_any(b, j);
				if (bit_at(o, j) || j == k) {
					for (;; l--) {
						rb[l] = cur;
						if (l == j)
							break;
					}
					if (j == k)
						break;
					l = j - 1;
				}
			}
			k = i;
			break;
		}
		case 5: {
			int64_t cur = 0;
			for (uint64_t j = k; j < i; j++)
				cur += count_all || !isnil_any(b, j);
			for (; k < i; k++)
				rb[k] = cur;
			break;
		}
		case 6:
			for (; k < i; k++)
				rb[k] = count_all || !isnil_any(b, k);
			break;
		default:
			/* the count over [start, end) (the segment tree adds 0/1
			 * values, which cannot overflow) */
			for (; k < i; k++) {
				int64_t c = 0;
				if (end[k] > start[k]) {
					if (count_all)
						c = (int64_t) (end[k] - start[k]);
					else
						for (ora_oid x = start[k]; x < end[k]; x++)
							c += !isnil_any(b, x);
				}
				rb[k] = c;
			}
			break;
		}
	}
	r->count = cnt;
	return 0;
}
