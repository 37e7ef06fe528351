/*
 * gdk_oracle_winstats.c -- windowed statistics and products over frames
 * (TEST INFRASTRUCTURE ONLY; see gdk_oracle.h).
 *
 * Restates gdk/gdk_analytic_statistics.c:
 *   GDKanalytical_stddev_samp / _stddev_pop / _variance_samp / _variance_pop
 *     (GDK_ANALYTICAL_STDEV_VARIANCE :897-965; per-frame loops :689-792,
 *     segment-tree nodes stdev_var_deltas :794-840)
 *   GDKanalytical_covariance_samp / _pop (:967-1188, covariance_deltas)
 *   GDKanalytical_correlation (:1190-1443, correlation_deltas)
 * and gdk/gdk_analytic_func.c GDKanalyticalprod (:2024-2560: PROD_NUM with
 * MULI4_WITH_CHECK / OP_WITH_CHECK, gdk_calc_private.h:40-46, 133; PROD_FP).
 *
 * Every frame kind folds the same per-row nodes: the running frames in row
 * order (3: forward, results per peer group; 4: backward from the partition
 * end; 5: the partition), 6 the row alone, and every other frame the
 * reference's fanout-16 segment tree (gdk_analytic.h:63-130) per partition
 * with its size rule.  A tree's inner node folds its children as if each
 * were ONE value (COMPUTE_LEVELN_*: the child's `delta` field stands for the
 * child) -- restated as is.  Overflow: the statistics check their
 * accumulators for infinity when a result is produced; the products check
 * every multiplication.
 */
#include <float.h>
#include <math.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gdk_oracle.h"

void ora_seterr(const char *fmt, ...);

#define FANOUT 16
#define HGE_MAX ((ora_hge) (((unsigned __int128) 1 << 127) - 1))

static int
bit_at(const ora_bat *b, uint64_t i)
{
	return b && ((const int8_t *) b->base)[i] != 0;
}

/* (dbl) of row i of a bte..hge / flt / dbl column; true when nil */
static bool
wval(const ora_bat *b, uint64_t i, double *d)
{
	const char *x = b->base;
	switch (b->type) {
	case ORA_bte: { int8_t v = ((const int8_t *) x)[i]; *d = v; return v == INT8_MIN; }
	case ORA_sht: { int16_t v = ((const int16_t *) x)[i]; *d = v; return v == INT16_MIN; }
	case ORA_int: { int32_t v = ((const int32_t *) x)[i]; *d = v; return v == INT32_MIN; }
	case ORA_lng: { int64_t v = ((const int64_t *) x)[i]; *d = (double) v; return v == INT64_MIN; }
	case ORA_hge: { ora_hge v = ((const ora_hge *) x)[i]; *d = (double) v; return v == -HGE_MAX - 1; }
	case ORA_flt: { float v = ((const float *) x)[i]; *d = v; return v != v; }
	default: { double v = ((const double *) x)[i]; *d = v; return v != v; }
	}
}

/* ---- statistics nodes ------------------------------------------------- */

enum { K_VAR, K_COV, K_COR };

typedef struct {
	uint64_t n;
	double mean1, mean2, delta1, delta2, m2, up, down1, down2;
} wnode;

/* COMPUTE_LEVEL0_*: a non-nil row is {n 1, mean v, delta v} */
static void
w_leaf(int kind, wnode *c, const ora_bat *b1, const ora_bat *b2, uint64_t i)
{
	double x, y = 0;
	bool nil = wval(b1, i, &x);
	if (kind != K_VAR)
		nil |= wval(b2, i, &y);
	memset(c, 0, sizeof(*c));
	if (nil)
		return;
	c->n = 1;
	c->mean1 = c->delta1 = x;
	c->mean2 = c->delta2 = y;
}

/* COMPUTE_LEVELN_* (and, with a leaf for v, the running frames' row step) */
static void
w_fold(int kind, wnode *a, const wnode *v)
{
	if (!v->n)
		return;
	a->n++;
	const double n = (double) a->n;
	a->delta1 = v->delta1 - a->mean1;
	a->mean1 += a->delta1 / n;
	if (kind == K_VAR) {
		a->m2 += a->delta1 * (v->delta1 - a->mean1);
		return;
	}
	a->delta2 = v->delta2 - a->mean2;
	a->mean2 += a->delta2 / n;
	if (kind == K_COV) {
		a->m2 += a->delta1 * (v->delta2 - a->mean2);
		return;
	}
	const double aux = v->delta2 - a->mean2;
	a->up += a->delta1 * aux;
	a->down1 += a->delta1 * (v->delta1 - a->mean1);
	a->down2 += a->delta2 * aux;
}

/* the result of a node: op 0 stddev_samp, 1 stddev_pop, 2 variance_samp,
 * 3 variance_pop (K_VAR); 0 samp, 1 pop (K_COV); -1 on overflow */
static int
w_result(int kind, int op, const wnode *a, double *out, bool *has_nils)
{
	if (kind == K_COR) {
		if (isinf(a->up) || isinf(a->down1) || isinf(a->down2))
			return -1;
		const double n = (double) a->n;
		if (a->n != 0 && a->down1 != 0 && a->down2 != 0) {
			*out = (a->up / n) / (sqrt(a->down1 / n) * sqrt(a->down2 / n));
		} else {
			*out = nan("");
			*has_nils = true;
		}
		return 0;
	}
	if (isinf(a->m2))
		return -1;
	const bool sample = kind == K_VAR ? (op & 1) == 0 : op == 0;
	if (a->n > (uint64_t) sample) {
		const double v = a->m2 / (double) (a->n - sample);
		*out = kind == K_VAR && op < 2 ? sqrt(v) : v;
	} else {
		*out = nan("");
		*has_nils = true;
	}
	return 0;
}

static void
tree_levels(uint64_t nc, uint64_t *total, uint64_t *nl)
{
	uint64_t c = nc;
	*total = nc;
	*nl = 1;
	do {
		c = (c + FANOUT - 1) / FANOUT;
		*total += c;
		(*nl)++;
	} while (c > 1);
}

int
ora_analyticalstat(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b1, const ora_bat *b2,
		   const ora_bat *s, const ora_bat *e, int kind, int op, int frame_type)
{
	const int tp = b1->type;
	if (!(tp == ORA_bte || tp == ORA_sht || tp == ORA_int || tp == ORA_lng || tp == ORA_hge || tp == ORA_flt ||
	      tp == ORA_dbl)) {
		ora_seterr("42000!%s of type %d unsupported.\n",
			   kind == K_VAR ? (op < 2 ? "standard deviation" : "variance")
					 : kind == K_COV ? "covariance" : "correlation", tp);
		return -1;
	}
	const uint64_t cnt = b1->count;
	double *rb = r->base;
	const ora_oid *start = s ? s->base : NULL, *end = e ? e->base : NULL;
	bool has_nils = false;
	wnode *lv0 = calloc(cnt + 1, sizeof(wnode));
	if (!lv0)
		return -1;
	for (uint64_t i = 0; i < cnt; i++)
		w_leaf(kind, &lv0[i], b1, b2, i);
	uint64_t k = 0;
	for (uint64_t i = 1; cnt && i <= cnt; i++) {
		if (i < cnt && !bit_at(p, i))
			continue;
		/* partition [k, i) */
		switch (frame_type) {
		case 3: {
			wnode c = {0};
			while (k < i) {
				uint64_t j = k;
				do {
					w_fold(kind, &c, &lv0[k]);
					k++;
				} while (k < i && !bit_at(o, k));
				double v;
				if (w_result(kind, op, &c, &v, &has_nils) < 0)
					goto overflow;
				for (; j < k; j++)
					rb[j] = v;
			}
			break;
		}
		case 4: {
			wnode c = {0};
			uint64_t l = i - 1;
			for (uint64_t j = l;; j--) {
				w_fold(kind, &c, &lv0[j]);
				if (bit_at(o, j) || j == k) {
					double v;
					if (w_result(kind, op, &c, &v, &has_nils) < 0)
						goto overflow;
					for (;; l--) {
						rb[l] = v;
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
			wnode c = {0};
			for (uint64_t j = k; j < i; j++)
				w_fold(kind, &c, &lv0[j]);
			double v;
			if (w_result(kind, op, &c, &v, &has_nils) < 0)
				goto overflow;
			for (; k < i; k++)
				rb[k] = v;
			break;
		}
		case 6: {
			/* the row alone: 0 (population) or nil, whatever the value */
			const bool sample = kind == K_VAR ? (op & 1) == 0 : op == 0;
			const double v = kind == K_COR || sample ? nan("") : 0.0;
			for (; k < i; k++)
				rb[k] = v;
			has_nils = v != v;
			break;
		}
		default: {
			const uint64_t j = k, nc = i - k;
			uint64_t total, nl;
			tree_levels(nc, &total, &nl);
			wnode *tree = calloc(total, sizeof(wnode));
			uint64_t *off = malloc(nl * sizeof(uint64_t));
			if (!tree || !off) {
				free(tree);
				free(off);
				free(lv0);
				return -1;
			}
			memcpy(tree, lv0 + j, nc * sizeof(wnode));
			uint64_t to = nc, lsize = nc, prev = 0, cur = 1;
			off[0] = 0;
			while (cur < nl) {
				uint64_t prev_to = to;
				off[cur++] = to;
				for (uint64_t pos = 0; pos < lsize; pos += FANOUT) {
					uint64_t pend = pos + FANOUT < lsize ? pos + FANOUT : lsize;
					wnode acc = {0};
					for (uint64_t x = pos; x < pend; x++)
						w_fold(kind, &acc, &tree[prev + x]);
					tree[to++] = acc;
				}
				prev = prev_to;
				lsize = to - prev_to;
			}
			int bad = 0;
			for (; k < i && !bad; k++) {
				wnode acc = {0};
				uint64_t begin = start[k] - j, tend = end[k] - j;
				if (begin < tend)
					for (uint64_t level = 0; level < nl; level++) {
						const wnode *tl = tree + off[level];
						uint64_t pb = begin / FANOUT, pe = tend / FANOUT;
						if (pb == pe) {
							for (uint64_t pos = begin; pos < tend; pos++)
								w_fold(kind, &acc, &tl[pos]);
							break;
						}
						uint64_t gb = pb * FANOUT;
						if (begin != gb) {
							for (uint64_t pos = begin; pos < gb + FANOUT; pos++)
								w_fold(kind, &acc, &tl[pos]);
							pb++;
						}
						uint64_t ge = pe * FANOUT;
						if (tend != ge)
							for (uint64_t pos = ge; pos < tend; pos++)
								w_fold(kind, &acc, &tl[pos]);
						begin = pb;
						tend = pe;
					}
				if (w_result(kind, op, &acc, &rb[k], &has_nils) < 0)
					bad = 1;
			}
			free(tree);
			free(off);
			if (bad)
				goto overflow;
			break;
		}
		}
	}
	free(lv0);
	r->count = cnt;
	r->nil = has_nils;
	r->nonil = !has_nils;
	return 0;
overflow:
	free(lv0);
	ora_seterr("22003!overflow in calculation.\n");
	return -1;
}

/* ---- products --------------------------------------------------------- */

typedef struct {
	ora_hge i;
	double d;
	float f;
	int nil;
} pnode;

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

static bool
p_ok(int tp1, int tp2)
{
	switch (tp2) {
	case ORA_bte: return tp1 == ORA_bte;
	case ORA_sht: return tp1 == ORA_bte || tp1 == ORA_sht;
	case ORA_int: return tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int;
	case ORA_lng: return tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int || tp1 == ORA_lng;
	case ORA_hge: return tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int || tp1 == ORA_lng || tp1 == ORA_hge;
	case ORA_flt: return tp1 == ORA_flt;
	case ORA_dbl: return tp1 == ORA_flt || tp1 == ORA_dbl;
	}
	return false;
}

static void
p_leaf(pnode *c, const ora_bat *b, uint64_t i, int tp2)
{
	double d;
	memset(c, 0, sizeof(*c));
	if (tp2 == ORA_flt || tp2 == ORA_dbl) {
		c->nil = wval(b, i, &d);
		if (b->type == ORA_flt)
			c->f = ((const float *) b->base)[i];
		c->d = d;
		return;
	}
	const char *x = b->base;
	switch (b->type) {
	case ORA_bte: c->i = ((const int8_t *) x)[i]; c->nil = c->i == INT8_MIN; break;
	case ORA_sht: c->i = ((const int16_t *) x)[i]; c->nil = c->i == INT16_MIN; break;
	case ORA_int: c->i = ((const int32_t *) x)[i]; c->nil = c->i == INT32_MIN; break;
	case ORA_lng: c->i = ((const int64_t *) x)[i]; c->nil = c->i == INT64_MIN; break;
	default: c->i = ((const ora_hge *) x)[i]; c->nil = c->i == -HGE_MAX - 1; break;
	}
}

/* PROD_NUM / COMPUTE_LEVELN_PROD_* / PROD_FP; false on overflow */
static bool
p_fold(pnode *a, const pnode *v, int tp2)
{
	if (v->nil)
		return true;
	if (a->nil) {
		*a = *v;
		return true;
	}
	if (tp2 == ORA_flt) {
		const float x = v->f;
		if (fabsf(a->f) > 1 && FLT_MAX / fabsf(x) < fabsf(a->f))
			return false;
		a->f *= x;
		return true;
	}
	if (tp2 == ORA_dbl) {
		const double x = v->d;
		if (fabs(a->d) > 1 && DBL_MAX / fabs(x) < fabs(a->d))
			return false;
		a->d *= x;
		return true;
	}
	ora_hge r;
	const ora_hge mx = tmax(tp2);
	if (__builtin_mul_overflow(v->i, a->i, &r) || r > mx || r < -mx)
		return false;
	a->i = r;
	return true;
}

static void
p_put(ora_bat *r, uint64_t k, const pnode *a, int tp2, bool *has_nils)
{
	char *x = r->base;
	*has_nils |= a->nil != 0;
	switch (tp2) {
	case ORA_bte: ((int8_t *) x)[k] = a->nil ? INT8_MIN : (int8_t) a->i; break;
	case ORA_sht: ((int16_t *) x)[k] = a->nil ? INT16_MIN : (int16_t) a->i; break;
	case ORA_int: ((int32_t *) x)[k] = a->nil ? INT32_MIN : (int32_t) a->i; break;
	case ORA_lng: ((int64_t *) x)[k] = a->nil ? INT64_MIN : (int64_t) a->i; break;
	case ORA_hge: ((ora_hge *) x)[k] = a->nil ? -HGE_MAX - 1 : a->i; break;
	case ORA_flt: ((float *) x)[k] = a->nil ? nanf("") : a->f; break;
	default: ((double *) x)[k] = a->nil ? nan("") : a->d; break;
	}
}

int
ora_analyticalprod(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		   const ora_bat *e, int tp2, int frame_type)
{
	if (!p_ok(b->type, tp2)) {
		ora_seterr("42000!type combination (prod(%d)->%d) not supported.\n", b->type, tp2);
		return -1;
	}
	const uint64_t cnt = b->count;
	const ora_oid *start = s ? s->base : NULL, *end = e ? e->base : NULL;
	bool has_nils = false;
	pnode *lv0 = calloc(cnt + 1, sizeof(pnode));
	if (!lv0)
		return -1;
	for (uint64_t i = 0; i < cnt; i++) {
		p_leaf(&lv0[i], b, i, tp2);
		if (tp2 == ORA_dbl && b->type == ORA_flt)
			lv0[i].d = lv0[i].f;
	}
	const pnode none = {.nil = 1};
	uint64_t k = 0;
	for (uint64_t i = 1; cnt && i <= cnt; i++) {
		if (i < cnt && !bit_at(p, i))
			continue;
		switch (frame_type) {
		case 3: {
			pnode c = none;
			while (k < i) {
				uint64_t j = k;
				do {
					if (!p_fold(&c, &lv0[k], tp2))
						goto overflow;
					k++;
				} while (k < i && !bit_at(o, k));
				for (; j < k; j++)
					p_put(r, j, &c, tp2, &has_nils);
			}
			break;
		}
		case 4: {
			pnode c = none;
			uint64_t l = i - 1;
			for (uint64_t j = l;; j--) {
				if (!p_fold(&c, &lv0[j], tp2))
					goto overflow;
				if (bit_at(o, j) || j == k) {
					for (;; l--) {
						p_put(r, l, &c, tp2, &has_nils);
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
			pnode c = none;
			for (uint64_t j = k; j < i; j++)
				if (!p_fold(&c, &lv0[j], tp2))
					goto overflow;
			for (; k < i; k++)
				p_put(r, k, &c, tp2, &has_nils);
			break;
		}
		case 6:
			for (; k < i; k++)
				p_put(r, k, &lv0[k], tp2, &has_nils);
			break;
		default: {
			const uint64_t j = k, nc = i - k;
			uint64_t total, nl;
			tree_levels(nc, &total, &nl);
			pnode *tree = calloc(total, sizeof(pnode));
			uint64_t *off = malloc(nl * sizeof(uint64_t));
			if (!tree || !off) {
				free(tree);
				free(off);
				free(lv0);
				return -1;
			}
			memcpy(tree, lv0 + j, nc * sizeof(pnode));
			uint64_t to = nc, lsize = nc, prev = 0, cur = 1;
			int bad = 0;
			off[0] = 0;
			while (cur < nl && !bad) {
				uint64_t prev_to = to;
				off[cur++] = to;
				for (uint64_t pos = 0; pos < lsize; pos += FANOUT) {
					uint64_t pend = pos + FANOUT < lsize ? pos + FANOUT : lsize;
					pnode acc = none;
					for (uint64_t x = pos; x < pend; x++)
						bad |= !p_fold(&acc, &tree[prev + x], tp2);
					tree[to++] = acc;
				}
				prev = prev_to;
				lsize = to - prev_to;
			}
			for (; k < i && !bad; k++) {
				pnode acc = none;
				uint64_t begin = start[k] - j, tend = end[k] - j;
				if (begin < tend)
					for (uint64_t level = 0; level < nl && !bad; level++) {
						const pnode *tl = tree + off[level];
						uint64_t pb = begin / FANOUT, pe = tend / FANOUT;
						if (pb == pe) {
							for (uint64_t pos = begin; pos < tend; pos++)
								bad |= !p_fold(&acc, &tl[pos], tp2);
							break;
						}
						uint64_t gb = pb * FANOUT;
						if (begin != gb) {
							for (uint64_t pos = begin; pos < gb + FANOUT; pos++)
								bad |= !p_fold(&acc, &tl[pos], tp2);
							pb++;
						}
						uint64_t ge = pe * FANOUT;
						if (tend != ge)
							for (uint64_t pos = ge; pos < tend; pos++)
								bad |= !p_fold(&acc, &tl[pos], tp2);
						begin = pb;
						tend = pe;
					}
				p_put(r, k, &acc, tp2, &has_nils);
			}
			free(tree);
			free(off);
			if (bad)
				goto overflow;
			break;
		}
		}
	}
	free(lv0);
	r->count = cnt;
	r->nil = has_nils;
	r->nonil = !has_nils;
	return 0;
overflow:
	free(lv0);
	ora_seterr("22003!overflow in calculation.\n");
	return -1;
}
