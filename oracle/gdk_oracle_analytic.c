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
#include <float.h>
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gdk_oracle.h"

void ora_seterr(const char *fmt, ...);
int ora_fsum_array(double *out, bool *isnil, const double *vals, uint64_t nv, bool skip_nils, bool nil_if_empty);

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

/* ---- GDKanalyticalsum over flt / dbl (gdk_analytic_func.c:1795-1817,
 * :1930-1950): frames 3 / 4 / 6 / segment-tree frames add in row order (or
 * the tree's order) with ADD_WITH_CHECK in the result type
 * (gdk_calc_private.h:53-67); frame 5 is dofsum (exact, rounded once). */
typedef struct {
	double v;   /* in the result type (a flt result is kept as its float value) */
	int nil;
	int isflt;
	int ovf;
} fsv;

static double
fround(const fsv *a, double x)
{
	return a->isflt ? (double) (float) x : x;
}

/* ADD_WITH_CHECK(lft, rgt, TPE2, dst, GDK_TPE2_max, overflow) with lft
 * already converted to TPE2 (the comparisons promote it so) */
static double
fadd_check(fsv *a, double lft, double rgt)
{
	if (a->isflt) {
		const float mx = FLT_MAX, l = (float) lft, r = (float) rgt;
		if (r < 1) {
			if (-mx - r > l) { a->ovf = 1; return rgt; }
		} else if (mx - r < l) {
			a->ovf = 1;
			return rgt;
		}
		return (double) (float) (l + r);
	}
	const double mx = DBL_MAX;
	if (rgt < 1) {
		if (-mx - rgt > lft) { a->ovf = 1; return rgt; }
	} else if (mx - rgt < lft) {
		a->ovf = 1;
		return rgt;
	}
	return lft + rgt;
}

/* COMPUTE_LEVELN_SUM_NUM / the sequential frames: cur = x + cur */
static fsv
fsadd(fsv *a, fsv cur, fsv x)
{
	if (x.nil)
		return cur;
	if (cur.nil) {
		cur.v = x.v;
		cur.nil = 0;
		return cur;
	}
	cur.v = fadd_check(a, x.v, cur.v);
	return cur;
}

static void
put_fsum(ora_bat *r, int isflt, uint64_t k, fsv x)
{
	if (isflt)
		((float *) r->base)[k] = x.nil ? nanf("") : (float) x.v;
	else
		((double *) r->base)[k] = x.nil ? nan("") : x.v;
}

static int
fsum_frames(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s, const ora_bat *e,
	    int tp1, int tp2, int frame_type)
{
	const uint64_t cnt = b->count;
	fsv a = {0, 0, tp2 == ORA_flt, 0};
	fsv *lv0 = malloc((cnt + 1) * sizeof(fsv));
	if (!lv0)
		return -1;
	for (uint64_t i = 0; i < cnt; i++) {
		double x = tp1 == ORA_flt ? (double) ((const float *) b->base)[i] : ((const double *) b->base)[i];
		lv0[i] = (fsv) {fround(&a, x), x != x, a.isflt, 0};
	}
	const ora_oid *start = s ? s->base : NULL, *end = e ? e->base : NULL;
	int rc = 0, has_nils = 0;
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt && !a.ovf && rc == 0; i++) {
		if (i < cnt && !bit_at(p, i))
			continue;
		switch (frame_type) {
		case 3: {
			fsv cur = {0, 1, a.isflt, 0};
			while (k < i) {
				uint64_t j = k;
				do {
					cur = fsadd(&a, cur, lv0[k]);
					k++;
				} while (k < i && !bit_at(o, k));
				for (; j < k; j++)
					put_fsum(r, a.isflt, j, cur);
				has_nils |= cur.nil;
			}
			break;
		}
		case 4: {
			fsv cur = {0, 1, a.isflt, 0};
			uint64_t l = i - 1;
			for (uint64_t j = l;; j--) {
				cur = fsadd(&a, cur, lv0[j]);
				if (bit_at(o, j) || j == k) {
					for (;; l--) {
						put_fsum(r, a.isflt, l, cur);
						if (l == j)
							break;
					}
					has_nils |= cur.nil;
					if (j == k)
						break;
					l = j - 1;
				}
			}
			k = i;
			break;
		}
		case 5: {   /* dofsum over the partition, nils skipped, nil if empty */
			double *vals = malloc((i - k + 1) * sizeof(double));
			for (uint64_t j = k; j < i; j++)
				vals[j - k] = lv0[j].nil ? nan("") : (tp1 == ORA_flt ? (double) ((const float *) b->base)[j]
											: ((const double *) b->base)[j]);
			double d = 0;
			bool isnil = false;
			int frc = ora_fsum_array(&d, &isnil, vals, i - k, true, true);
			free(vals);
			if (frc < 0 || (!isnil && a.isflt && (isinf((float) d) || isnan((float) d)))) {
				if (frc == 0)
					ora_seterr("22003!overflow in sum aggregate.\n");
				rc = -2;
				break;
			}
			fsv cur = {a.isflt ? (double) (float) d : d, isnil, a.isflt, 0};
			for (; k < i; k++)
				put_fsum(r, a.isflt, k, cur);
			has_nils |= isnil;
			break;
		}
		case 6:
			for (; k < i; k++) {
				put_fsum(r, a.isflt, k, lv0[k]);
				has_nils |= lv0[k].nil;
			}
			break;
		default: {  /* the reference's tree over the partition, nodes in TPE2 */
			const uint64_t j = k, n = i - k;
			uint64_t total = n, c = n, nl = 1;
			do {
				c = (c + FANOUT - 1) / FANOUT;
				total += c;
				nl++;
			} while (c > 1);
			fsv *tree = malloc(total * sizeof(fsv));
			uint64_t *off = malloc(nl * sizeof(uint64_t));
			memcpy(tree, lv0 + j, n * sizeof(fsv));
			uint64_t to = n, lsize = n, prev = 0, cl = 1;
			off[0] = 0;
			while (cl < nl) {
				uint64_t prev_to = to;
				off[cl++] = to;
				for (uint64_t pos = 0; pos < lsize; pos += FANOUT) {
					uint64_t en = pos + FANOUT < lsize ? pos + FANOUT : lsize;
					fsv acc = {0, 1, a.isflt, 0};
					for (uint64_t x = pos; x < en; x++)
						acc = fsadd(&a, acc, tree[prev + x]);
					tree[to++] = acc;
				}
				prev = prev_to;
				lsize = to - prev_to;
			}
			for (; k < i && !a.ovf; k++) {
				uint64_t begin = start[k] - j, tend = end[k] - j;
				fsv acc = {0, 1, a.isflt, 0};
				if (begin < tend)
					for (uint64_t level = 0; level < nl; level++) {
						const fsv *tl = tree + off[level];
						uint64_t pb = begin / FANOUT, pe = tend / FANOUT;
						if (pb == pe) {
							for (uint64_t pos = begin; pos < tend; pos++)
								acc = fsadd(&a, acc, tl[pos]);
							break;
						}
						uint64_t gb = pb * FANOUT;
						if (begin != gb) {
							for (uint64_t pos = begin; pos < gb + FANOUT; pos++)
								acc = fsadd(&a, acc, tl[pos]);
							pb++;
						}
						uint64_t ge = pe * FANOUT;
						if (tend != ge)
							for (uint64_t pos = ge; pos < tend; pos++)
								acc = fsadd(&a, acc, tl[pos]);
						begin = pb;
						tend = pe;
					}
				put_fsum(r, a.isflt, k, acc);
				has_nils |= acc.nil;
			}
			free(tree);
			free(off);
			break;
		}
		}
	}
	free(lv0);
	if (rc == -2) {
		/* dofsum's message, then the analytic bailout's (GDKerror appends) */
		char m[256];
		snprintf(m, sizeof(m), "%s42000!error while calculating floating-point sum\n", ora_errbuf());
		ora_seterr("%s", m);
		return -1;
	}
	if (rc < 0)
		return -1;
	if (a.ovf) {
		ora_seterr("22003!overflow in calculation.\n");
		return -1;
	}
	r->count = cnt;
	r->nil = has_nils;
	r->nonil = !has_nils;
	return 0;
}

int
ora_analyticalsum(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		  const ora_bat *e, int tp1, int tp2, int frame_type)
{
	if ((tp1 == ORA_flt && (tp2 == ORA_flt || tp2 == ORA_dbl)) || (tp1 == ORA_dbl && tp2 == ORA_dbl))
		return fsum_frames(r, p, o, b, s, e, tp1, tp2, frame_type);
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

/* ---------------------------------------------------------------------- */
/* GDKanalyticalavg (gdk/gdk_analytic_statistics.c:364-423).
 * Integers (bte..lng): the running frames (3, 4, 5) divide the exact 128-bit
 * sum by the count, (dbl) sum / n (ANALYTICAL_AVG_IMP_NUM_* :29-165; the
 * AVERAGE_ITER overflow branch is unreachable below hge); the current row is
 * (dbl) v; general frames walk a fanout-16 segment tree whose nodes are
 * avg_num_deltas {a, n, rr} and whose combine step feeds each non-empty
 * child's a into AVERAGE_ITER (:167-199) -- so an inner node counts its
 * children, not its rows, and the result is a + (dbl) rr / n.
 * flt/dbl: AVERAGE_ITER_FLOAT in the input type (TPE a, :201-316); frame 4
 * never assigns its result, so every row is nil there (:224-246). */

typedef struct {
	int64_t a, n, rr;   /* integers */
	double d;           /* dbl */
	float f;            /* flt */
} anode;

/* AVERAGE_ITER (gdk/gdk_calc_private.h:231-275) in 64-bit arithmetic; for
 * TYPE bte..lng no intermediate leaves TYPE's range */
static void
avg_iter_i(int64_t x, anode *c)
{
	const int64_t n = ++c->n;
	int64_t an = c->a / n, xn = x / n, z1 = xn - an;
	xn = x - xn * n;
	an = c->a - an * n;
	uint64_t z2;
	if (xn >= an) {
		z2 = (uint64_t) (xn - an);
		while (z2 >= (uint64_t) n) {
			z2 -= (uint64_t) n;
			z1++;
		}
	} else {
		z2 = (uint64_t) (an - xn);
		for (;;) {
			z1--;
			if (z2 < (uint64_t) n) {
				z2 = (uint64_t) n - z2;
				break;
			}
			z2 -= (uint64_t) n;
		}
	}
	c->a += z1;
	c->rr += (int64_t) z2;
	if (c->rr >= n) {
		c->rr -= n;
		c->a++;
	}
}

/* AVERAGE_ITER_FLOAT (gdk_calc_private.h:277-289) in TPE arithmetic */
static void
avg_iter_f(float x, anode *c)
{
	c->n++;
	const float n = (float) c->n;
	if ((c->f > 0) == (x > 0))
		c->f += (x - c->f) / n;
	else
		c->f = c->f - c->f / n + x / n;
}

static void
avg_iter_d(double x, anode *c)
{
	c->n++;
	const double n = (double) c->n;
	if ((c->d > 0) == (x > 0))
		c->d += (x - c->d) / n;
	else
		c->d = c->d - c->d / n + x / n;
}

/* fold a node into an accumulator (COMPUTE_LEVELN_AVG_NUM / _FP) */
static void
avg_fold(int tp, anode *acc, const anode *v)
{
	if (v->n == 0)
		return;
	if (tp == ORA_flt)
		avg_iter_f(v->f, acc);
	else if (tp == ORA_dbl)
		avg_iter_d(v->d, acc);
	else
		avg_iter_i(v->a, acc);
}

static double
avg_final(int tp, const anode *c, bool *has_nils)
{
	if (c->n == 0) {
		*has_nils = true;
		return nan("");
	}
	if (tp == ORA_flt)
		return (double) c->f;
	if (tp == ORA_dbl)
		return c->d;
	return (double) c->a + (double) c->rr / (double) c->n;
}

int
ora_analyticalavg(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		  const ora_bat *e, int tpe, int frame_type)
{
	const int tp = b->type;
	if (!(tp == ORA_bte || tp == ORA_sht || tp == ORA_int || tp == ORA_lng || tp == ORA_flt || tp == ORA_dbl)) {
		ora_seterr("42000!average of type %d to dbl unsupported.\n", tpe);
		return -1;
	}
	const bool isf = tp == ORA_flt || tp == ORA_dbl;
	const uint64_t cnt = b->count;
	double *rb = r->base;
	const ora_oid *start = s ? s->base : NULL, *end = e ? e->base : NULL;
	bool has_nils = false;
	anode *lv0 = calloc(cnt + 1, sizeof(anode));
	if (!lv0)
		return -1;
	/* level-0 nodes: {v, 1} or {0} for nil (COMPUTE_LEVEL0_AVG_*) */
	for (uint64_t i = 0; i < cnt; i++) {
		if (isnil_any(b, i))
			continue;
		lv0[i].n = 1;
		if (tp == ORA_flt)
			lv0[i].f = ((const float *) b->base)[i];
		else if (tp == ORA_dbl)
			lv0[i].d = ((const double *) b->base)[i];
		else {
			ora_hge v;
			ival(b, i, &v);
			lv0[i].a = (int64_t) v;
		}
	}
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt; i++) {
		if (i < cnt && !bit_at(p, i))
			continue;
		/* partition [k, i) */
		switch (frame_type) {
		case 3:
			if (isf) {
				anode c = {0};
				double cur = nan("");
				while (k < i) {
					uint64_t j = k;
					do {
						avg_fold(tp, &c, &lv0[k]);
						k++;
					} while (k < i && !bit_at(o, k));
					if (c.n > 0)
						cur = tp == ORA_flt ? (double) c.f : c.d;
					else
						has_nils = true;
					for (; j < k; j++)
						rb[j] = cur;
				}
			} else {
				ora_hge sum = 0;
				int64_t n = 0;
				while (k < i) {
					uint64_t j = k;
					do {
						if (lv0[k].n) {
							sum += lv0[k].a;
							n++;
						}
						k++;
					} while (k < i && !bit_at(o, k));
					double cur = n > 0 ? (double) sum / (double) n : nan("");
					for (; j < k; j++)
						rb[j] = cur;
					has_nils |= n == 0;
				}
			}
			break;
		case 4: {
			ora_hge sum = 0;
			int64_t n = 0;
			uint64_t l = i - 1;
			for (uint64_t j = l;; j--) {
				if (!isf && lv0[j].n) {
					sum += lv0[j].a;
					n++;
				}
				if (bit_at(o, j) || j == k) {
					/* flt/dbl: curval is never assigned (nil) */
					double cur = !isf && n > 0 ? (double) sum / (double) n : nan("");
					for (;; l--) {
						rb[l] = cur;
						if (l == j)
							break;
					}
					has_nils |= cur != cur;
					if (j == k)
						break;
					l = j - 1;
				}
			}
			k = i;
			break;
		}
		case 5: {
			double cur;
			if (isf) {
				anode c = {0};
				for (uint64_t j = k; j < i; j++)
					avg_fold(tp, &c, &lv0[j]);
				cur = c.n > 0 ? (tp == ORA_flt ? (double) c.f : c.d) : nan("");
			} else {
				ora_hge sum = 0;
				int64_t n = 0;
				for (uint64_t j = k; j < i; j++)
					if (lv0[j].n) {
						sum += lv0[j].a;
						n++;
					}
				cur = n > 0 ? (double) sum / (double) n : nan("");
			}
			has_nils |= cur != cur;
			for (; k < i; k++)
				rb[k] = cur;
			break;
		}
		case 6:
			for (; k < i; k++) {
				rb[k] = lv0[k].n == 0 ? nan("")
					: tp == ORA_flt ? (double) lv0[k].f : tp == ORA_dbl ? lv0[k].d : (double) lv0[k].a;
				has_nils |= lv0[k].n == 0;
			}
			break;
		default: {
			/* populate_segment_tree / compute_on_segment_tree
			 * (gdk_analytic.h:63-130) over avg nodes */
			const uint64_t j = k, nc = i - k;
			uint64_t total = nc, c = nc, nl = 1;
			do {
				c = (c + FANOUT - 1) / FANOUT;
				total += c;
				nl++;
			} while (c > 1);
			anode *tree = calloc(total, sizeof(anode));
			uint64_t *off = malloc(nl * sizeof(uint64_t));
			if (!tree || !off) {
				free(tree);
				free(off);
				free(lv0);
				return -1;
			}
			memcpy(tree, lv0 + j, nc * sizeof(anode));
			uint64_t to = nc, lsize = nc, prev = 0, cur = 1;
			off[0] = 0;
			while (cur < nl) {
				uint64_t prev_to = to;
				off[cur++] = to;
				for (uint64_t pos = 0; pos < lsize; pos += FANOUT) {
					uint64_t pend = pos + FANOUT < lsize ? pos + FANOUT : lsize;
					anode acc = {0};
					for (uint64_t x = pos; x < pend; x++)
						avg_fold(tp, &acc, &tree[prev + x]);
					tree[to++] = acc;
				}
				prev = prev_to;
				lsize = to - prev_to;
			}
			for (; k < i; k++) {
				anode acc = {0};
				uint64_t begin = start[k] - j, tend = end[k] - j;
				if (begin < tend)
					for (uint64_t level = 0; level < nl; level++) {
						const anode *tl = tree + off[level];
						uint64_t pb = begin / FANOUT, pe = tend / FANOUT;
						if (pb == pe) {
							for (uint64_t pos = begin; pos < tend; pos++)
								avg_fold(tp, &acc, &tl[pos]);
							break;
						}
						uint64_t gb = pb * FANOUT;
						if (begin != gb) {
							for (uint64_t pos = begin; pos < gb + FANOUT; pos++)
								avg_fold(tp, &acc, &tl[pos]);
							pb++;
						}
						uint64_t ge = pe * FANOUT;
						if (tend != ge)
							for (uint64_t pos = ge; pos < tend; pos++)
								avg_fold(tp, &acc, &tl[pos]);
						begin = pb;
						tend = pe;
					}
				rb[k] = avg_final(tp, &acc, &has_nils);
			}
			free(tree);
			free(off);
			break;
		}
		}
	}
	free(lv0);
	r->count = cnt;
	r->nil = has_nils;
	r->nonil = !has_nils;
	return 0;
}

/* ---------------------------------------------------------------------- */
/* GDKanalyticalavginteger (gdk/gdk_analytic_statistics.c:428-700): the
 * average in the input's integer type.  Every frame keeps AVERAGE_ITER's
 * (avg, rem, ncnt) state -- row by row through the running frames
 * (forward for 3 and 5, backward from the partition end for 4), over
 * avg_int_deltas nodes of the same fanout-16 segment tree as
 * GDKanalyticalavg for general frames -- and ends with
 * ANALYTICAL_AVERAGE_INT_CALC_FINALIZE (:435-446, rounding half away from
 * zero); no rows -> nil; frame 6 copies the values. */

/* compute_on_segment_tree over one partition's tree (levels built by the
 * caller as in ora_analyticalavg): the folded node of [begin, tend) */
static anode
avg_tree_query(int tp, anode *const *lvl, uint64_t nl, uint64_t begin, uint64_t tend)
{
	anode acc = {0};
	if (begin < tend)
		for (uint64_t level = 0; level < nl; level++) {
			const anode *tl = lvl[level];
			uint64_t pb = begin / FANOUT, pe = tend / FANOUT;
			if (pb == pe) {
				for (uint64_t pos = begin; pos < tend; pos++)
					avg_fold(tp, &acc, &tl[pos]);
				break;
			}
			uint64_t gb = pb * FANOUT;
			if (begin != gb) {
				for (uint64_t pos = begin; pos < gb + FANOUT; pos++)
					avg_fold(tp, &acc, &tl[pos]);
				pb++;
			}
			uint64_t ge = pe * FANOUT;
			if (tend != ge)
				for (uint64_t pos = ge; pos < tend; pos++)
					avg_fold(tp, &acc, &tl[pos]);
			begin = pb;
			tend = pe;
		}
	return acc;
}

static void
put_int(ora_bat *r, uint64_t k, int64_t v, bool nil)
{
	switch (r->width) {
	case 1: ((int8_t *) r->base)[k] = nil ? INT8_MIN : (int8_t) v; break;
	case 2: ((int16_t *) r->base)[k] = nil ? INT16_MIN : (int16_t) v; break;
	case 4: ((int32_t *) r->base)[k] = nil ? INT32_MIN : (int32_t) v; break;
	default: ((int64_t *) r->base)[k] = nil ? INT64_MIN : v; break;
	}
}

/* ANALYTICAL_AVERAGE_INT_CALC_FINALIZE into slot k of r */
static void
avgint_put(ora_bat *r, uint64_t k, const anode *c, bool *has_nils)
{
	if (c->n == 0) {
		*has_nils = true;
		put_int(r, k, 0, true);
		return;
	}
	int64_t avg = c->a;
	if (c->rr > 0) {
		if (avg < 0) {
			if (2 * c->rr > c->n)
				avg++;
		} else if (2 * c->rr >= c->n) {
			avg++;
		}
	}
	put_int(r, k, avg, false);
}

int
ora_analyticalavginteger(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
			 const ora_bat *e, int tpe, int frame_type)
{
	const int tp = b->type;
	if (!(tp == ORA_bte || tp == ORA_sht || tp == ORA_int || tp == ORA_lng)) {
		ora_seterr("42000!average of type %d to int unsupported.\n", tpe);
		return -1;
	}
	const uint64_t cnt = b->count;
	const ora_oid *start = s ? s->base : NULL, *end = e ? e->base : NULL;
	bool has_nils = false;
	anode *lv0 = calloc(cnt + 1, sizeof(anode));
	if (!lv0)
		return -1;
	for (uint64_t i = 0; i < cnt; i++) {
		if (isnil_any(b, i))
			continue;
		ora_hge v;
		ival(b, i, &v);
		lv0[i].n = 1;
		lv0[i].a = (int64_t) v;
	}
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt; i++) {
		if (i < cnt && !bit_at(p, i))
			continue;
		/* partition [k, i) */
		if (frame_type == 3) {
			anode c = {0};
			while (k < i) {
				uint64_t j = k;
				do {
					avg_fold(tp, &c, &lv0[k]);
					k++;
				} while (k < i && !bit_at(o, k));
				for (; j < k; j++)
					avgint_put(r, j, &c, &has_nils);
			}
		} else if (frame_type == 4) {
			anode c = {0};
			uint64_t l = i - 1;
			for (uint64_t j = l;; j--) {
				avg_fold(tp, &c, &lv0[j]);
				if (bit_at(o, j) || j == k) {
					for (;; l--) {
						avgint_put(r, l, &c, &has_nils);
						if (l == j)
							break;
					}
					if (j == k)
						break;
					l = j - 1;
				}
			}
			k = i;
		} else if (frame_type == 5) {
			anode c = {0};
			for (uint64_t j = k; j < i; j++)
				avg_fold(tp, &c, &lv0[j]);
			for (; k < i; k++)
				avgint_put(r, k, &c, &has_nils);
		} else if (frame_type == 6) {
			for (; k < i; k++) {
				avgint_put(r, k, &lv0[k], &has_nils);
			}
		} else {
			const uint64_t j = k, nc = i - k;
			uint64_t total = nc, c = nc, nl = 1;
			do {
				c = (c + FANOUT - 1) / FANOUT;
				total += c;
				nl++;
			} while (c > 1);
			anode *tree = calloc(total, sizeof(anode));
			anode **lvl = malloc(nl * sizeof(anode *));
			if (!tree || !lvl) {
				free(tree);
				free(lvl);
				free(lv0);
				return -1;
			}
			memcpy(tree, lv0 + j, nc * sizeof(anode));
			lvl[0] = tree;
			uint64_t to = nc, lsize = nc, prev = 0;
			for (uint64_t cur = 1; cur < nl; cur++) {
				uint64_t prev_to = to;
				lvl[cur] = tree + to;
				for (uint64_t pos = 0; pos < lsize; pos += FANOUT) {
					uint64_t pend = pos + FANOUT < lsize ? pos + FANOUT : lsize;
					anode acc = {0};
					for (uint64_t x = pos; x < pend; x++)
						avg_fold(tp, &acc, &tree[prev + x]);
					tree[to++] = acc;
				}
				prev = prev_to;
				lsize = to - prev_to;
			}
			for (; k < i; k++) {
				anode acc = avg_tree_query(tp, lvl, nl, start[k] - j, end[k] - j);
				avgint_put(r, k, &acc, &has_nils);
			}
			free(tree);
			free(lvl);
		}
	}
	free(lv0);
	r->count = cnt;
	r->nil = has_nils;
	r->nonil = !has_nils;
	return 0;
}
