/*
 * gdk_oracle_window.c -- window functions beyond the frame aggregates
 * (TEST INFRASTRUCTURE ONLY; see gdk_oracle.h).
 *
 * Restates gdk/gdk_analytic_bounds.c:95 GDKanalyticaldiff (ANALYTICAL_DIFF_IMP
 * :19-51, the NaN-aware ANALYTICAL_DIFF_FLOAT_IMP :54-92, atomcmp for str
 * :135-170) and gdk/gdk_analytic_func.c:
 *   GDKanalyticalntile    :124 (NTILE_CALC :64-90, partition walk :92-112)
 *   GDKanalyticalfirst    :230 (ANALYTICAL_FIRST_FIXED :215-227)
 *   GDKanalyticallast     :312 (ANALYTICAL_LAST_FIXED :297-309)
 *   GDKanalyticalnthvalue :421 (single :380-397, multi :399-418 -- its
 *                         "lnth - 1 > frame size" test reads the row after
 *                         the frame when lnth - 1 == frame size, kept here)
 *   GDKanalyticallag      :671 (ANALYTICAL_LAG_CALC / _IMP :586-623)
 *   GDKanalyticallead     :823 (LEAD_CALC / ANALYTICAL_LEAD_IMP :744-785)
 *   GDKanalyticalmin/max  :1264 (ANALYTICAL_MIN_MAX: frames 3 :869-888, 4
 *                         :890-915, 5 :917-932, 6 :934-941, others: the
 *                         fanout-16 segment tree, gdk/gdk_analytic.h:64-130)
 * for the fixed-width types (bte, sht, int, lng, hge, flt, dbl and the
 * types stored as them).  Partitions: p[i] != 0 starts a partition at row
 * i; peers: o[i] != 0 starts a peer group.
 */
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gdk_oracle.h"

void ora_seterr(const char *fmt, ...);

/* storage type of a fixed-width value (ATOMbasetype) */
static int
wbase(int t)
{
	switch (t) {
	case ORA_date: return ORA_int;
	case ORA_daytime: case ORA_timestamp: case ORA_oid: return ORA_lng;
	case ORA_bit: return ORA_bte;
	default: return t;
	}
}

static int
wwidth(int t)
{
	switch (wbase(t)) {
	case ORA_bte: return 1;
	case ORA_sht: return 2;
	case ORA_int: case ORA_flt: return 4;
	case ORA_lng: case ORA_dbl: return 8;
	case ORA_hge: return 16;
	default: return 0;
	}
}

static bool
nil_at(int t, const void *base, uint64_t i)
{
	switch (wbase(t)) {
	case ORA_bte: return ((const int8_t *) base)[i] == INT8_MIN;
	case ORA_sht: return ((const int16_t *) base)[i] == INT16_MIN;
	case ORA_int: return ((const int32_t *) base)[i] == INT32_MIN;
	case ORA_lng: return ((const int64_t *) base)[i] == INT64_MIN;
	case ORA_hge: return ((const ora_hge *) base)[i] == (ora_hge) ((unsigned __int128) 1 << 127);
	case ORA_flt: { float f = ((const float *) base)[i]; return f != f; }
	case ORA_dbl: { double d = ((const double *) base)[i]; return d != d; }
	default: return false;
	}
}

static bool
nil_val(int t, const void *v)
{
	return nil_at(t, v, 0);
}

static void
put_nil(int t, void *base, uint64_t i)
{
	switch (wbase(t)) {
	case ORA_bte: ((int8_t *) base)[i] = INT8_MIN; break;
	case ORA_sht: ((int16_t *) base)[i] = INT16_MIN; break;
	case ORA_int: ((int32_t *) base)[i] = INT32_MIN; break;
	case ORA_lng: ((int64_t *) base)[i] = INT64_MIN; break;
	case ORA_hge: ((ora_hge *) base)[i] = (ora_hge) ((unsigned __int128) 1 << 127); break;
	case ORA_flt: ((float *) base)[i] = __builtin_nanf(""); break;
	case ORA_dbl: ((double *) base)[i] = __builtin_nan(""); break;
	}
}

static void
copy_val(int w, void *dst, uint64_t di, const void *src, uint64_t si)
{
	memcpy((char *) dst + di * w, (const char *) src + si * w, w);
}

static void
set_props(ora_bat *r, uint64_t n, bool has_nils)
{
	r->count = n;
	r->nonil = !has_nils;
	r->nil = has_nils;
	r->sorted = r->revsorted = r->key = n <= 1;
}

/* row i starts a partition (row 0 always does) */
static bool
pstart(const ora_bat *p, uint64_t i)
{
	return i == 0 || (p && ((const int8_t *) p->base)[i]);
}

/* ---- ntile ------------------------------------------------------------ */

static int
ntile_val(int t, const void *v, int64_t *out, bool *isnil)
{
	*out = 0;
	*isnil = true;
	switch (t) {
	case ORA_bte: *isnil = *(const int8_t *) v == INT8_MIN; *out = *(const int8_t *) v; return 0;
	case ORA_sht: *isnil = *(const int16_t *) v == INT16_MIN; *out = *(const int16_t *) v; return 0;
	case ORA_int: *isnil = *(const int32_t *) v == INT32_MIN; *out = *(const int32_t *) v; return 0;
	case ORA_lng: *isnil = *(const int64_t *) v == INT64_MIN; *out = *(const int64_t *) v; return 0;
	case ORA_hge: {
		ora_hge h = *(const ora_hge *) v;
		*isnil = h == (ora_hge) ((unsigned __int128) 1 << 127);
		/* (val > GDK_lng_max) ? GDK_lng_max : (lng) val */
		*out = h > (ora_hge) INT64_MAX ? INT64_MAX : (int64_t) h;
		return 0;
	}
	default: return -1;
	}
}

static void
put_int(int t, void *base, uint64_t i, int64_t v)
{
	switch (t) {
	case ORA_bte: ((int8_t *) base)[i] = (int8_t) v; break;
	case ORA_sht: ((int16_t *) base)[i] = (int16_t) v; break;
	case ORA_int: ((int32_t *) base)[i] = (int32_t) v; break;
	case ORA_lng: ((int64_t *) base)[i] = v; break;
	case ORA_hge: ((ora_hge *) base)[i] = v; break;
	}
}

int
ora_analyticalntile(ora_bat *r, const ora_bat *b, const ora_bat *p, const ora_bat *n, int tpe, const void *ntile)
{
	uint64_t cnt = b->count;
	bool has_nils = false;
	int w = wwidth(tpe);
	if (tpe != ORA_bte && tpe != ORA_sht && tpe != ORA_int && tpe != ORA_lng && tpe != ORA_hge) {
		ora_seterr("42000!type %d not supported for the ntile type.\n", tpe);
		return -1;
	}
	if (ntile) {
		int64_t v;
		bool isn;
		ntile_val(tpe, ntile, &v, &isn);
		if (!isn && v <= 0) {
			ora_seterr("42000!ntile must be greater than zero.\n");
			return -1;
		}
	}
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt; i++) {
		if (i < cnt && !pstart(p, i))
			continue;
		/* the partition [k, i) (NTILE_CALC) */
		uint64_t ncnt = i - k;
		for (uint64_t j = 0; k < i; k++, j++) {
			int64_t val;
			bool isn;
			ntile_val(tpe, ntile ? ntile : (const char *) n->base + k * w, &val, &isn);
			if (isn) {
				has_nils = true;
				put_nil(tpe, r->base, k);
				continue;
			}
			if (!ntile && val <= 0) {
				ora_seterr("42000!ntile must be greater than zero.\n");
				return -1;
			}
			uint64_t nval = (uint64_t) val;
			int64_t res;
			if (nval >= ncnt) {
				res = (int64_t) (j + 1);
			} else {
				uint64_t bsize = ncnt / nval, top = ncnt - nval * bsize, small = top * (bsize + 1);
				res = j < small ? (int64_t) (1 + j / (bsize + 1)) : (int64_t) (1 + top + (j - small) / bsize);
			}
			put_int(tpe, r->base, k, res);
		}
	}
	set_props(r, cnt, has_nils);
	return 0;
}

/* ---- first / last / nth_value ------------------------------------------ */

int
ora_analyticalfirst(ora_bat *r, const ora_bat *b, const ora_bat *s, const ora_bat *e, int tpe)
{
	const uint64_t cnt = b->count, *start = s->base, *end = e->base;
	const int w = wwidth(tpe);
	bool has_nils = false;
	if (w == 0) {
		ora_seterr("42000!type not supported");
		return -1;
	}
	for (uint64_t k = 0; k < cnt; k++) {
		if (end[k] > start[k])
			copy_val(w, r->base, k, b->base, start[k]);
		else
			put_nil(tpe, r->base, k);
		has_nils |= nil_at(tpe, r->base, k);
	}
	set_props(r, cnt, has_nils);
	return 0;
}

int
ora_analyticallast(ora_bat *r, const ora_bat *b, const ora_bat *s, const ora_bat *e, int tpe)
{
	const uint64_t cnt = b->count, *start = s->base, *end = e->base;
	const int w = wwidth(tpe);
	bool has_nils = false;
	if (w == 0) {
		ora_seterr("42000!type not supported");
		return -1;
	}
	for (uint64_t k = 0; k < cnt; k++) {
		if (end[k] > start[k])
			copy_val(w, r->base, k, b->base, end[k] - 1);
		else
			put_nil(tpe, r->base, k);
		has_nils |= nil_at(tpe, r->base, k);
	}
	set_props(r, cnt, has_nils);
	return 0;
}

/* t: a lng BAT of per-row n (multi), or NULL with *pnth (single) */
int
ora_analyticalnthvalue(ora_bat *r, const ora_bat *b, const ora_bat *s, const ora_bat *e, const ora_bat *t,
		       const int64_t *pnth, int tpe)
{
	const uint64_t cnt = b->count, *start = s->base, *end = e->base;
	const int w = wwidth(tpe);
	bool has_nils = false;
	if (w == 0 || (t && t->type != ORA_lng)) {
		ora_seterr("42000!type not supported for the nth_value.\n");
		return -1;
	}
	if (t) {
		const int64_t *tp = t->base;
		for (uint64_t k = 0; k < cnt; k++) {
			int64_t lnth = tp[k];
			if (lnth != INT64_MIN && lnth <= 0) {
				ora_seterr("42000!nth_value must be greater than zero.\n");
				return -1;
			}
			if (lnth == INT64_MIN || end[k] <= start[k] || lnth - 1 > (int64_t) (end[k] - start[k])) {
				put_nil(tpe, r->base, k);
				has_nils = true;
			} else {
				/* lnth - 1 == frame size reads the row after the frame
				 * (the reference's bound); past the column it would read
				 * beyond the heap, taken as nil here */
				uint64_t at = start[k] + (uint64_t) (lnth - 1);
				if (at < cnt)
					copy_val(w, r->base, k, b->base, at);
				else
					put_nil(tpe, r->base, k);
				has_nils |= nil_at(tpe, r->base, k);
			}
		}
	} else {
		int64_t nth = *pnth;
		if (nth != INT64_MIN && nth <= 0) {
			ora_seterr("42000!nth_value must be greater than zero.\n");
			return -1;
		}
		if (nth == INT64_MIN) {
			has_nils = true;
			for (uint64_t k = 0; k < cnt; k++)
				put_nil(tpe, r->base, k);
		} else {
			nth--;
			for (uint64_t k = 0; k < cnt; k++) {
				if (end[k] > start[k] && nth < (int64_t) (end[k] - start[k]))
					copy_val(w, r->base, k, b->base, start[k] + (uint64_t) nth);
				else
					put_nil(tpe, r->base, k);
				has_nils |= nil_at(tpe, r->base, k);
			}
		}
	}
	set_props(r, cnt, has_nils);
	return 0;
}

/* ---- lag / lead -------------------------------------------------------- */

#define ORA_BUN_NONE_LAG ((uint64_t) INT64_MAX)

int
ora_analyticallag(ora_bat *r, const ora_bat *b, const ora_bat *p, uint64_t lag, const void *def, int tpe)
{
	const uint64_t cnt = b->count;
	const int w = wwidth(tpe);
	bool has_nils = false;
	if (w == 0) {
		ora_seterr("42000!type not supported");
		return -1;
	}
	if (lag == ORA_BUN_NONE_LAG) {
		for (uint64_t k = 0; k < cnt; k++)
			put_nil(tpe, r->base, k);
		set_props(r, cnt, true);
		return 0;
	}
	/* ANALYTICAL_LAG_CALC per partition [k, i): `lag` defaults, then the
	 * values shifted by lag; has_nils |= lag > 0 && nil(def) per call */
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt + (cnt == 0); i++) {
		if (i < cnt && !pstart(p, i))
			continue;
		uint64_t e = i > cnt ? cnt : i;
		for (uint64_t j = k; j < e; j++) {
			if (j - k < lag) {
				memcpy((char *) r->base + j * w, def, w);
			} else {
				copy_val(w, r->base, j, b->base, j - lag);
				has_nils |= nil_at(tpe, r->base, j);
			}
		}
		has_nils |= lag > 0 && nil_val(tpe, def);
		k = e;
	}
	set_props(r, cnt, has_nils);
	return 0;
}

int
ora_analyticallead(ora_bat *r, const ora_bat *b, const ora_bat *p, uint64_t lead, const void *def, int tpe)
{
	const uint64_t cnt = b->count;
	const int w = wwidth(tpe);
	bool has_nils = false;
	if (w == 0) {
		ora_seterr("42000!type not supported");
		return -1;
	}
	if (lead == ORA_BUN_NONE_LAG) {
		for (uint64_t k = 0; k < cnt; k++)
			put_nil(tpe, r->base, k);
		set_props(r, cnt, true);
		return 0;
	}
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt + (cnt == 0); i++) {
		if (i < cnt && !pstart(p, i))
			continue;
		uint64_t e = i > cnt ? cnt : i;
		for (uint64_t j = k; j < e; j++) {
			if (lead < e - j) {
				copy_val(w, r->base, j, b->base, j + lead);
				has_nils |= nil_at(tpe, r->base, j);
			} else {
				memcpy((char *) r->base + j * w, def, w);
			}
		}
		has_nils |= lead > 0 && nil_val(tpe, def);
		k = e;
	}
	set_props(r, cnt, has_nils);
	return 0;
}

/* ---- min / max over frames --------------------------------------------- */

/* MIN_MAX(a, b) of the reference: MIN(A,B) = ((A) < (B) ? (A) : (B)),
 * MAX(A,B) = ((A) > (B) ? (A) : (B)); returns 1 when the result is a */
static int
pick_a(int t, const void *a, const void *b, bool ismax)
{
	switch (wbase(t)) {
#define PK(T) { T x = *(const T *) a, y = *(const T *) b; return ismax ? x > y : x < y; }
	case ORA_bte: PK(int8_t)
	case ORA_sht: PK(int16_t)
	case ORA_int: PK(int32_t)
	case ORA_lng: PK(int64_t)
	case ORA_hge: PK(ora_hge)
	case ORA_flt: PK(float)
	case ORA_dbl: PK(double)
#undef PK
	}
	return 0;
}

/* curval = MIN_MAX(next, curval) skipping nils (frames 3 / 4 / 5): a nil
 * curval takes next */
static void
fold_next(int t, int w, char *cur, const char *next, bool ismax)
{
	if (nil_val(t, next))
		return;
	if (nil_val(t, cur) || pick_a(t, next, cur, ismax))
		memcpy(cur, next, w);
}

/* COMPUTE_LEVELN: computed = MIN_MAX(computed, VAL) skipping nil VAL */
static void
fold_tree(int t, int w, char *computed, const char *val, bool ismax)
{
	if (nil_val(t, val))
		return;
	if (nil_val(t, computed))
		memcpy(computed, val, w);
	else if (!pick_a(t, computed, val, ismax))
		memcpy(computed, val, w);
}

static int
minmax(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s, const ora_bat *e,
       int tpe, int frame_type, bool ismax)
{
	const uint64_t cnt = b->count;
	const int w = wwidth(tpe);
	const char *bp = b->base;
	char *rb = r->base;
	bool has_nils = false;
	char cur[16], nilv[16];
	if (w == 0) {
		ora_seterr("42000!type not supported");
		return -1;
	}
	put_nil(tpe, nilv, 0);
	const int8_t *op = o ? o->base : NULL;
	uint64_t k = 0;
	for (uint64_t i = 1; i <= cnt; i++) {
		if (i < cnt && !pstart(p, i))
			continue;
		/* partition [k, i) */
		switch (frame_type) {
		case 3:         /* unbounded preceding .. current row: per peer group */
			memcpy(cur, nilv, w);
			for (uint64_t q = k; q < i;) {
				uint64_t j = q;
				do {
					fold_next(tpe, w, cur, bp + q * w, ismax);
					q++;
				} while (q < i && !op[q]);
				for (; j < q; j++)
					memcpy(rb + j * w, cur, w);
				has_nils |= nil_val(tpe, cur);
			}
			break;
		case 4: {       /* current row .. unbounded following */
			memcpy(cur, nilv, w);
			uint64_t l = i - 1;
			for (uint64_t j = l;; j--) {
				fold_next(tpe, w, cur, bp + j * w, ismax);
				if (op[j] || j == k) {
					for (;; l--) {
						memcpy(rb + l * w, cur, w);
						if (l == j)
							break;
					}
					has_nils |= nil_val(tpe, cur);
					if (j == k)
						break;
					l = j - 1;
				}
			}
			break;
		}
		case 5:
			memcpy(cur, nilv, w);
			for (uint64_t j = k; j < i; j++)
				fold_next(tpe, w, cur, bp + j * w, ismax);
			for (uint64_t j = k; j < i; j++)
				memcpy(rb + j * w, cur, w);
			has_nils |= nil_val(tpe, cur);
			break;
		case 6:
			for (uint64_t j = k; j < i; j++) {
				memcpy(rb + j * w, bp + j * w, w);
				has_nils |= nil_at(tpe, bp, j);
			}
			break;
		default: {
			/* the partition's fanout-16 segment tree (gdk_analytic.h:64-95)
			 * and the per-row query walk (:97-130) */
			const uint64_t *start = s->base, *end = e->base;
			uint64_t ncount = i - k, nlevels = 1, counter = ncount, tsize = ncount;
			do {
				counter = (counter + 15) / 16;
				tsize += counter;
				nlevels++;
			} while (counter > 1);
			char *tree = malloc(tsize * w + 16);
			uint64_t *lvl = malloc(nlevels * sizeof(uint64_t));
			if (!tree || !lvl) {
				free(tree);
				free(lvl);
				ora_seterr("malloc");
				return -1;
			}
			uint64_t toff = 0, lsize = ncount, cl = 0;
			lvl[cl++] = 0;
			for (uint64_t x = 0; x < lsize; x++)
				memcpy(tree + (toff++) * w, bp + (k + x) * w, w);
			const char *prev = tree;
			while (cl < nlevels) {
				uint64_t ptoff = toff;
				lvl[cl++] = toff;
				for (uint64_t pos = 0; pos < lsize; pos += 16) {
					uint64_t wd = (lsize < pos + 16 ? lsize : pos + 16) - pos;
					char comp[16];
					memcpy(comp, nilv, w);
					for (uint64_t x = 0; x < wd; x++)
						fold_tree(tpe, w, comp, prev + x * w, ismax);
					memcpy(tree + (toff++) * w, comp, w);
					prev += wd * w;
				}
				lsize = toff - ptoff;
			}
			for (uint64_t q = k; q < i; q++) {
				uint64_t bg = start[q] - k, te = end[q] - k;
				char comp[16];
				memcpy(comp, nilv, w);
				if (bg < te)
					for (uint64_t level = 0; level < nlevels; level++) {
						const char *tl = tree + lvl[level] * w;
						uint64_t pb = bg / 16, pe = te / 16;
						if (pb == pe) {
							for (uint64_t pos = bg; pos < te; pos++)
								fold_tree(tpe, w, comp, tl + pos * w, ismax);
							break;
						}
						uint64_t gb = pb * 16;
						if (bg != gb) {
							for (uint64_t pos = bg; pos < gb + 16; pos++)
								fold_tree(tpe, w, comp, tl + pos * w, ismax);
							pb++;
						}
						uint64_t ge = pe * 16;
						if (te != ge)
							for (uint64_t pos = ge; pos < te; pos++)
								fold_tree(tpe, w, comp, tl + pos * w, ismax);
						bg = pb;
						te = pe;
					}
				memcpy(rb + q * w, comp, w);
				has_nils |= nil_val(tpe, comp);
			}
			free(tree);
			free(lvl);
			break;
		}
		}
		k = i;
	}
	set_props(r, cnt, has_nils);
	return 0;
}

int
ora_analyticalmin(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		  const ora_bat *e, int tpe, int frame_type)
{
	return minmax(r, p, o, b, s, e, tpe, frame_type, false);
}

int
ora_analyticalmax(ora_bat *r, const ora_bat *p, const ora_bat *o, const ora_bat *b, const ora_bat *s,
		  const ora_bat *e, int tpe, int frame_type)
{
	return minmax(r, p, o, b, s, e, tpe, frame_type, true);
}

/* ---- diff ---------------------------------------------------------------- */

static const char *
wstr_at(const ora_bat *b, uint64_t p)
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

static int
wstr_cmp(const char *a, const char *b)
{
	bool an = (unsigned char) a[0] == 0x80 && a[1] == 0, bn = (unsigned char) b[0] == 0x80 && b[1] == 0;
	if (an || bn)
		return an ? -!bn : 1;
	return strcmp(a, b);
}

/* r[i] = the value differs from the last value that differed (TRUE), else
 * np[i] / *npbit / FALSE; floats: two NaNs are the same (when b has nils) */
int
ora_analyticaldiff(ora_bat *r, const ora_bat *b, const ora_bat *p, const int8_t *npbit, int tpe)
{
	const uint64_t cnt = b->count;
	const int8_t *np = p ? p->base : NULL;
	int8_t *rb = r->base;
	const int8_t npb = npbit ? *npbit : 0;
	const int t = tpe == ORA_str ? ORA_str : wbase(tpe);
	uint64_t prev = 0;            /* position of the last differing value */
	for (uint64_t i = 0; i < cnt; i++) {
		bool diff;
		if (t == ORA_str) {
			diff = wstr_cmp(wstr_at(b, prev), wstr_at(b, i)) != 0;
		} else if (t == ORA_flt || t == ORA_dbl) {
			double x = t == ORA_flt ? ((const float *) b->base)[prev] : ((const double *) b->base)[prev];
			double y = t == ORA_flt ? ((const float *) b->base)[i] : ((const double *) b->base)[i];
			diff = x != y && (!b->nonil ? (x == x || y == y) : true);
		} else {
			const int w = wwidth(t);
			diff = memcmp((const char *) b->base + prev * w, (const char *) b->base + i * w, w) != 0;
		}
		if (diff) {
			rb[i] = 1;
			prev = i;
		} else {
			rb[i] = np ? np[i] : npbit ? npb : 0;
		}
	}
	r->count = cnt;
	r->nonil = 1;
	r->nil = 0;
	r->sorted = r->revsorted = r->key = cnt <= 1;
	return 0;
}
