/*
 * gdk_oracle_bounds.c -- window frame bounds (TEST INFRASTRUCTURE ONLY; see
 * gdk_oracle.h).
 *
 * Restates GDKanalyticalwindowbounds (gdk/gdk_analytic_bounds.c:1440) for
 * all three frame units:
 *   unit 0  ROWS    GDKanalyticalrowbounds   :855-992  (walk macros :187-222)
 *   unit 1  RANGE   GDKanalyticalrangebounds :994-1294 (numeric walks :273-369,
 *                   temporal walks :459-556, type tables :389-457, :558-587)
 *   unit 2  GROUPS  GDKanalyticalgroupsbounds :1296-1438 (walks :224-271)
 * with the shortcuts GDKanalyticalallbounds (:589, unbounded) and
 * GDKanalyticalpeers (:710, RANGE limit 0), static limits (`bound`) and
 * per-row limits (`l`), and the reference's error messages and result
 * properties.  Temporal arithmetic restates gdk/gdk_time.c (date_add_day
 * :122, date_add_month :155, daytime_add_usec :336, timestamp_add_usec
 * :436, timestamp_add_month :459) over the packed representations of
 * gdk_time.c:17-51.
 *
 * Rows are visited in the reference's order (partition by partition, row
 * by row), so the first error met is the one reported.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gdk_oracle.h"

void ora_seterr(const char *fmt, ...);

#define HGE_MAX ((ora_hge) (((unsigned __int128) 1 << 127) - 1))
#define HGE_NIL ((ora_hge) ((unsigned __int128) 1 << 127))
#define OID_MAX ((ora_oid) INT64_MAX)

static const char *
tname(int tp)
{
	switch (tp) {
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
	case ORA_daytime: return "daytime";
	case ORA_timestamp: return "timestamp";
	case ORA_str: return "str";
	}
	return "any";
}

/* ---- gdk_time.c restatement ------------------------------------------ */
#define YEAR_MIN (-4712)
#define YEAR_MAX (YEAR_MIN + (1 << 21) / 12 - 1)
#define DAY_USEC (24LL * 60 * 60 * 1000000)
#define DATE_NIL INT32_MIN
#define LNG_NIL INT64_MIN

static int
mdays(int y, int m)
{
	static const int d[13] = {0, 31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
	const int leap = y % 4 == 0 && (y % 100 != 0 || y % 400 == 0);
	return d[m] - (m == 2 && !leap);
}

static int32_t
mkd(int y, int m, int d)
{
	return (int32_t) (((uint32_t) ((y + 4712) * 12 + m - 1) << 5) | (uint32_t) d);
}

static void
split(int32_t dt, int *y, int *m, int *d)
{
	const uint32_t u = (uint32_t) dt;
	*d = (int) (u & 31);
	*m = (int) (((u >> 5) & ((1u << 21) - 1)) % 12 + 1);
	*y = (int) (((u >> 5) & ((1u << 21) - 1)) / 12) - 4712;
}

int32_t
ora_date_add_day(int32_t dt, int days)
{
	if (dt == DATE_NIL || days == INT32_MIN)
		return DATE_NIL;
	if (abs(days) >= 1 << 26)
		return DATE_NIL;
	int y, m, d;
	split(dt, &y, &m, &d);
	d += days;
	while (d <= 0) {
		if (--m == 0) {
			m = 12;
			if (--y < YEAR_MIN)
				return DATE_NIL;
		}
		d += mdays(y, m);
	}
	while (d > mdays(y, m)) {
		d -= mdays(y, m);
		if (++m > 12) {
			m = 1;
			if (++y > YEAR_MAX)
				return DATE_NIL;
		}
	}
	return mkd(y, m, d);
}

int32_t
ora_date_add_month(int32_t dt, int months)
{
	if (dt == DATE_NIL || months == INT32_MIN)
		return DATE_NIL;
	if (abs(months) >= 1 << 21)
		return DATE_NIL;
	int y, m, d;
	split(dt, &y, &m, &d);
	m += months;
	if (m <= 0) {
		y -= (12 - m) / 12;
		if (y < YEAR_MIN)
			return DATE_NIL;
		m = 12 - (-m % 12);
	} else if (m > 12) {
		y += (m - 1) / 12;
		if (y > YEAR_MAX)
			return DATE_NIL;
		m = (m - 1) % 12 + 1;
	}
	if (d > mdays(y, m))
		d = mdays(y, m);
	return mkd(y, m, d);
}

int64_t
ora_daytime_add_usec(int64_t t, int64_t usec)
{
	if (t == LNG_NIL || usec == LNG_NIL)
		return LNG_NIL;
	if (llabs(usec) >= DAY_USEC)
		return LNG_NIL;
	t += usec;
	if (t < 0 || t >= DAY_USEC)
		return LNG_NIL;
	return t;
}

#define TS_TIME(ts) ((int64_t) ((uint64_t) (ts) & ((1ULL << 37) - 1)))
#define TS_DATE(ts) ((int32_t) (((uint64_t) (ts) >> 37) & ((1u << 26) - 1)))
#define MKTS(d, t) ((int64_t) (((uint64_t) (uint32_t) (d) << 37) | (uint64_t) (t)))

int64_t
ora_timestamp_add_usec(int64_t ts, int64_t usec)
{
	if (ts == LNG_NIL || usec == LNG_NIL)
		return LNG_NIL;
	int64_t tm = TS_TIME(ts);
	int32_t dt = TS_DATE(ts);
	tm += usec;
	if (tm < 0) {
		const int add = (int) ((DAY_USEC - 1 - tm) / DAY_USEC);
		tm += add * DAY_USEC;
		dt = ora_date_add_day(dt, -add);
	} else if (tm >= DAY_USEC) {
		dt = ora_date_add_day(dt, (int) (tm / DAY_USEC));
		tm %= DAY_USEC;
	}
	if (dt == DATE_NIL)
		return LNG_NIL;
	return MKTS(dt, tm);
}

int64_t
ora_timestamp_add_month(int64_t ts, int m)
{
	if (ts == LNG_NIL || m == INT32_MIN)
		return LNG_NIL;
	const int64_t tm = TS_TIME(ts);
	const int32_t dt = ora_date_add_month(TS_DATE(ts), m);
	if (dt == DATE_NIL)
		return LNG_NIL;
	return MKTS(dt, tm);
}

/* ---- common -------------------------------------------------------------- */
static int
isbit(const ora_bat *p, uint64_t i)
{
	return p && ((const int8_t *) p->base)[i] != 0;
}

/* integer value of row i of an integer-typed BAT (bte..hge, bit),
 * *nil set for the type's nil */
static ora_hge
ivalue(const ora_bat *b, int tp, uint64_t i, int *nil)
{
	ora_hge v;
	switch (tp) {
	case ORA_bit:
	case ORA_bte: { int8_t x = ((const int8_t *) b->base)[i]; *nil = x == INT8_MIN; v = x; break; }
	case ORA_sht: { int16_t x = ((const int16_t *) b->base)[i]; *nil = x == INT16_MIN; v = x; break; }
	case ORA_int:
	case ORA_date: { int32_t x = ((const int32_t *) b->base)[i]; *nil = x == INT32_MIN; v = x; break; }
	case ORA_lng:
	case ORA_daytime:
	case ORA_timestamp: { int64_t x = ((const int64_t *) b->base)[i]; *nil = x == INT64_MIN; v = x; break; }
	case ORA_hge: { ora_hge x = ((const ora_hge *) b->base)[i]; *nil = x == HGE_NIL; v = x; break; }
	default: *nil = 1; v = 0; break;
	}
	return v;
}

static ora_hge
tmax_of(int tp)
{
	switch (tp) {
	case ORA_bte: return INT8_MAX;
	case ORA_sht: return INT16_MAX;
	case ORA_int: return INT32_MAX;
	case ORA_lng: return INT64_MAX;
	default: return HGE_MAX;
	}
}

static int
is_int_type(int tp)
{
	return tp == ORA_bte || tp == ORA_sht || tp == ORA_int || tp == ORA_lng || tp == ORA_hge;
}

static int
is_mtime(int tp)
{
	return tp == ORA_date || tp == ORA_daytime || tp == ORA_timestamp;
}

/* GDKanalyticalallbounds (:589): every row bound to its partition start
 * (PRECEDING) or end (FOLLOWING) */
static int
allbounds(ora_bat *r, const ora_bat *b, const ora_bat *p, bool preceding)
{
	ora_oid *rb = r->base;
	const uint64_t cnt = b->count;
	uint64_t m = 0;
	for (uint64_t i = 0; i <= cnt; i++) {
		if (i < cnt && !isbit(p, i))
			continue;
		for (uint64_t k = m; k < i; k++)
			rb[k] = preceding ? m : i;
		m = i;
	}
	r->count = cnt;
	r->nonil = 0;
	r->nil = 0;
	return 0;
}

/* equality of two rows for GDKanalyticalpeers (:710): nils match nils */
static int
row_eq(const ora_bat *b, uint64_t x, uint64_t y)
{
	switch (b->type) {
	case ORA_flt: {
		float u = ((const float *) b->base)[x], v = ((const float *) b->base)[y];
		return u == v || (isnan(u) && isnan(v));
	}
	case ORA_dbl: {
		double u = ((const double *) b->base)[x], v = ((const double *) b->base)[y];
		return u == v || (isnan(u) && isnan(v));
	}
	default:
		return memcmp((const char *) b->base + x * b->width, (const char *) b->base + y * b->width,
			      b->width) == 0;
	}
}

/* GDKanalyticalpeers: bound to the first (PRECEDING) / one past the last
 * (FOLLOWING) row of the current row's run of equal values in its partition */
static int
peerbounds(ora_bat *r, const ora_bat *b, const ora_bat *p, bool preceding)
{
	ora_oid *rb = r->base;
	const uint64_t cnt = b->count;
	uint64_t m = 0;
	for (uint64_t i = 0; i <= cnt; i++) {
		if (i < cnt && !isbit(p, i))
			continue;
		uint64_t s = m;
		for (uint64_t k = m; k <= i; k++) {
			if (k == i || !row_eq(b, s, k)) {
				for (uint64_t q = s; q < k; q++)
					rb[q] = preceding ? s : k;
				s = k;
			}
		}
		m = i;
	}
	r->count = cnt;
	r->nonil = 0;
	r->nil = 0;
	return 0;
}

/* limit of row k: from the static bound or l[k]; returns 0 for a valid
 * limit, -1 for nil / negative */
typedef struct {
	int tp2;
	const void *bound;
	const ora_bat *l;
} limsrc;

static int
limit_i(const limsrc *L, uint64_t k, ora_hge *out)
{
	int nil;
	ora_hge v;
	if (L->l)
		v = ivalue(L->l, L->tp2, k, &nil);
	else {
		ora_bat one = {.type = L->tp2, .base = (void *) L->bound};
		v = ivalue(&one, L->tp2, 0, &nil);
	}
	*out = v;
	return nil || v < 0 ? -1 : 0;
}

static int
limit_f(const limsrc *L, uint64_t k, double *out)
{
	double v;
	if (L->tp2 == ORA_flt)
		v = L->l ? ((const float *) L->l->base)[k] : *(const float *) L->bound;
	else
		v = L->l ? ((const double *) L->l->base)[k] : *(const double *) L->bound;
	*out = v;
	return isnan(v) || v < 0 ? -1 : 0;
}

/* ---- ROWS (:855) --------------------------------------------------------- */
static int
rowbounds(ora_bat *r, const ora_bat *b, const ora_bat *p, const ora_bat *l, const void *bound, int tp2,
	  bool preceding, ora_oid second_half, bool groups)
{
	const char *u = groups ? "groups" : "row";
	ora_oid *rb = r->base;
	const uint64_t cnt = b->count;
	if (tp2 != ORA_bte && tp2 != ORA_sht && tp2 != ORA_int && tp2 != ORA_lng && tp2 != ORA_hge) {
		ora_seterr("42000!%s frame bound type %s not supported.\n", groups ? "groups" : "rows", tname(tp2));
		return -1;
	}
	limsrc L = {tp2, bound, l};
	if (l) {
		if (l->nil)
			goto invalid;
	} else {
		/* static: the limit cast to lng, hge clamped to lng max
		 * (:926-962); lng max means unbounded */
		int nil;
		ora_bat one = {.type = tp2, .base = (void *) bound};
		const ora_hge v = ivalue(&one, tp2, 0, &nil);
		if (!nil && v >= INT64_MAX)
			return allbounds(r, b, p, preceding);
		if (nil || v < 0)
			goto invalid;
	}
	const int8_t *bp = groups ? b->base : NULL;
	uint64_t m = 0;
	for (uint64_t i = 0; i <= cnt; i++) {
		if (i < cnt && !isbit(p, i))
			continue;
		for (uint64_t k = m; k < i; k++) {
			ora_hge lv;
			if (limit_i(&L, k, &lv) < 0)
				goto invalid;
			/* per-row hge limits are clamped to oid max (:909-919),
			 * every other limit is used as an oid directly */
			ora_oid rl = lv > (ora_hge) OID_MAX ? OID_MAX : (ora_oid) lv;
			if (!groups) {
				if (preceding)
					rb[k] = rl > k - m ? m : k - rl + second_half;
				else {
					const ora_oid rl2 = rl + second_half;
					rb[k] = rl2 > i - k ? i : k + rl2;
				}
			} else if (preceding) {
				uint64_t j;
				for (j = k;; j--) {
					if (bp[j]) {
						if (rl == 0)
							break;
						rl--;
					}
					if (j == m)
						break;
				}
				rb[k] = j;
			} else {
				uint64_t j;
				for (j = k + 1; j < i; j++) {
					if (bp[j]) {
						if (rl == 0)
							break;
						rl--;
					}
				}
				rb[k] = j;
			}
		}
		m = i;
	}
	r->count = cnt;
	r->nonil = 1;
	r->nil = 0;
	return 0;
invalid:
	ora_seterr("42000!%s frame bound must be non negative and non null.\n", u);
	return -1;
}

/* ---- RANGE (:994) -------------------------------------------------------- */
enum { K_INT, K_FLT, K_DBL, K_MONTH, K_MSEC };

static const char *ERR_OVF = "22003!overflow in calculation.\n";
static const char *ERR_INV = "42000!range frame bound must be non negative and non null.\n";

/* SUB_WITH_CHECK (gdk_calc_private.h:87) in the exact integer domain:
 * overflow iff the true difference lies outside [-max, max] */
static int
isub_ovf(ora_hge v, ora_hge x, ora_hge max)
{
	if (x < 1)
		return max + x < v;
	return -max + x > v;
}

/* the same guard evaluated in float / double arithmetic */
static int
fsub_ovf(float v, float x)
{
	const float max = 3.40282346638528859812e+38F;
	if (x < 1)
		return (float) (max + x) < v;
	return (float) (-max + x) > v;
}

static int
dsub_ovf(double v, double x)
{
	const double max = 1.79769313486231570815e+308;
	if (x < 1)
		return max + x < v;
	return -max + x > v;
}

/* frame test for row j against the current row k: 1 in frame, 0 out,
 * -1 overflow (the walk raises it) */
typedef struct {
	int kind;
	int tp1;
	const ora_bat *b;
	ora_hge tmax;
} rctx;

static int
row_nil(const rctx *c, uint64_t j)
{
	int nil;
	if (c->kind == K_FLT)
		return isnan(((const float *) c->b->base)[j]);
	if (c->kind == K_DBL)
		return isnan(((const double *) c->b->base)[j]);
	ivalue(c->b, c->tp1, j, &nil);
	return nil;
}

static int
range_bounds(ora_bat *r, const rctx *c, const ora_bat *p, const limsrc *L, bool preceding)
{
	ora_oid *rb = r->base;
	const uint64_t cnt = c->b->count;
	uint64_t m = 0;
	for (uint64_t i = 0; i <= cnt; i++) {
		if (i < cnt && !isbit(p, i))
			continue;
		for (uint64_t k = m; k < i; k++) {
			ora_hge il = 0;
			double fl = 0;
			if (c->kind == K_FLT || c->kind == K_DBL) {
				if (limit_f(L, k, &fl) < 0)
					goto invalid;
			} else if (limit_i(L, k, &il) < 0) {
				goto invalid;
			}
			const int vn = row_nil(c, k);
			/* the frame edges of temporal values */
			int64_t vmin = 0, vmax = 0;
			int hasmin = 1, hasmax = 1;
			if (!vn && (c->kind == K_MONTH || c->kind == K_MSEC)) {
				int nil;
				const int64_t v = (int64_t) ivalue(c->b, c->tp1, k, &nil);
				if (c->tp1 == ORA_date) {
					const int32_t d = (int32_t) v;
					int32_t lo, hi;
					if (c->kind == K_MONTH) {
						lo = ora_date_add_month(d, -(int) il);
						hi = ora_date_add_month(d, (int) il);
					} else {
						/* date_add_msec: whole days of the msec limit */
						lo = ora_date_add_day(d, (int) (-(int64_t) il / (24 * 60 * 60 * 1000)));
						hi = ora_date_add_day(d, (int) ((int64_t) il / (24 * 60 * 60 * 1000)));
					}
					hasmin = lo != DATE_NIL;
					hasmax = hi != DATE_NIL;
					vmin = lo;
					vmax = hi;
				} else if (c->tp1 == ORA_daytime) {
					vmin = ora_daytime_add_usec(v, -1000 * (int64_t) il);
					vmax = ora_daytime_add_usec(v, 1000 * (int64_t) il);
					hasmin = vmin != LNG_NIL;
					hasmax = vmax != LNG_NIL;
				} else if (c->kind == K_MONTH) {
					vmin = ora_timestamp_add_month(v, -(int) il);
					vmax = ora_timestamp_add_month(v, (int) il);
					hasmin = vmin != LNG_NIL;
					hasmax = vmax != LNG_NIL;
				} else {
					vmin = ora_timestamp_add_usec(v, -(int64_t) il * 1000);
					vmax = ora_timestamp_add_usec(v, (int64_t) il * 1000);
					hasmin = vmin != LNG_NIL;
					hasmax = vmax != LNG_NIL;
				}
			}
			/* in-frame test of a non-nil row j for a non-nil current row */
#define INFRAME(j, res)								\
			do {							\
				int nil_;					\
				if (c->kind == K_INT) {				\
					const ora_hge v_ = ivalue(c->b, c->tp1, k, &nil_); \
					const ora_hge x_ = ivalue(c->b, c->tp1, (j), &nil_); \
					if (isub_ovf(v_, x_, c->tmax)) { ora_seterr("%s", ERR_OVF); return -1; } \
					const ora_hge d_ = v_ - x_;		\
					(res) = (d_ < 0 ? -d_ : d_) <= il;	\
				} else if (c->kind == K_FLT) {			\
					const float v_ = ((const float *) c->b->base)[k], x_ = ((const float *) c->b->base)[j]; \
					if (fsub_ovf(v_, x_)) { ora_seterr("%s", ERR_OVF); return -1; } \
					const float d_ = v_ - x_;		\
					(res) = !((d_ < 0 ? -d_ : d_) > (float) fl); \
				} else if (c->kind == K_DBL) {			\
					const double v_ = ((const double *) c->b->base)[k], x_ = ((const double *) c->b->base)[j]; \
					if (dsub_ovf(v_, x_)) { ora_seterr("%s", ERR_OVF); return -1; } \
					const double d_ = v_ - x_;		\
					(res) = !((d_ < 0 ? -d_ : d_) > fl);	\
				} else {					\
					const int64_t x_ = (int64_t) ivalue(c->b, c->tp1, (j), &nil_); \
					(res) = !((hasmin && x_ < vmin) || (hasmax && x_ > vmax)); \
				}						\
			} while (0)
			uint64_t j;
			if (preceding) {
				for (j = k;; j--) {
					const int jn = row_nil(c, j);
					if (vn ? !jn : jn) {
						j++;
						break;
					}
					if (!vn) {
						int in;
						INFRAME(j, in);
						if (!in) {
							j++;
							break;
						}
					}
					if (j == m)
						break;
				}
			} else {
				for (j = k + 1; j < i; j++) {
					const int jn = row_nil(c, j);
					if (vn ? !jn : jn)
						break;
					if (!vn) {
						int in;
						INFRAME(j, in);
						if (!in)
							break;
					}
				}
			}
#undef INFRAME
			rb[k] = j;
		}
		m = i;
	}
	r->count = cnt;
	r->nonil = 1;
	r->nil = 0;
	return 0;
invalid:
	ora_seterr("%s", ERR_INV);
	return -1;
}

static int
rangebounds(ora_bat *r, const ora_bat *b, const ora_bat *p, const ora_bat *l, const void *bound, int tp1,
	    int tp2, bool preceding)
{
	if (is_mtime(tp1) && tp2 != ORA_int && tp2 != ORA_lng)
		goto bound_not_supported;
	limsrc L = {tp2, bound, l};
	rctx c = {.tp1 = tp1, .b = b, .tmax = tmax_of(tp1)};
	if (l) {
		if (l->nil)
			goto invalid;
		switch (tp2) {
		case ORA_bte:
		case ORA_sht:
			if (tp1 != ORA_bte && tp1 != ORA_sht && tp1 != ORA_int && tp1 != ORA_lng)
				goto type_not_supported;
			c.kind = K_INT;
			break;
		case ORA_int:
		case ORA_lng:
			if (is_mtime(tp1)) {
				if (tp2 == ORA_int && tp1 == ORA_daytime)
					goto type_not_supported;
				c.kind = tp2 == ORA_int ? K_MONTH : K_MSEC;
			} else if (tp1 != ORA_bte && tp1 != ORA_sht && tp1 != ORA_int && tp1 != ORA_lng) {
				goto type_not_supported;
			} else {
				c.kind = K_INT;
			}
			break;
		case ORA_flt:
			if (tp1 != ORA_flt)
				goto type_not_supported;
			c.kind = K_FLT;
			break;
		case ORA_dbl:
			if (tp1 != ORA_dbl)
				goto type_not_supported;
			c.kind = K_DBL;
			break;
		case ORA_hge:
			if (!is_int_type(tp1))
				goto type_not_supported;
			c.kind = K_INT;
			break;
		default:
			goto bound_not_supported;
		}
		return range_bounds(r, &c, p, &L, preceding);
	}
	switch (tp2) {
	case ORA_bte:
	case ORA_sht:
	case ORA_int:
	case ORA_lng: {
		/* unbounded / current-row shortcuts before the validity check */
		int nil;
		ora_bat one = {.type = tp2, .base = (void *) bound};
		const ora_hge v = ivalue(&one, tp2, 0, &nil);
		const ora_hge vmax = tp2 == ORA_bte ? INT8_MAX : tp2 == ORA_sht ? INT16_MAX
			: tp2 == ORA_int ? INT32_MAX : INT64_MAX;
		if (!nil && v == vmax)
			return allbounds(r, b, p, preceding);
		if (!nil && v == 0)
			return peerbounds(r, b, p, preceding);
		if (nil || v < 0)
			goto invalid;
		if (is_mtime(tp1)) {
			c.kind = tp2 == ORA_int ? K_MONTH : K_MSEC;
			if (tp2 == ORA_int && tp1 == ORA_daytime)
				goto type_not_supported;
		} else if (tp1 == ORA_bte || tp1 == ORA_sht || tp1 == ORA_int || tp1 == ORA_lng) {
			c.kind = K_INT;
		} else {
			goto type_not_supported;
		}
		return range_bounds(r, &c, p, &L, preceding);
	}
	case ORA_flt:
	case ORA_dbl: {
		const double v = tp2 == ORA_flt ? *(const float *) bound : *(const double *) bound;
		if (isnan(v) || v < 0)
			goto invalid;
		if (tp2 == ORA_flt ? *(const float *) bound == 3.40282346638528859812e+38F
				   : v == 1.79769313486231570815e+308)
			return allbounds(r, b, p, preceding);
		if (v == 0)
			return peerbounds(r, b, p, preceding);
		if (tp1 != tp2)
			goto type_not_supported;
		c.kind = tp2 == ORA_flt ? K_FLT : K_DBL;
		return range_bounds(r, &c, p, &L, preceding);
	}
	case ORA_hge: {
		const ora_hge v = *(const ora_hge *) bound;
		if (v == HGE_NIL || v < 0)
			goto invalid;
		if (v == HGE_MAX)
			return allbounds(r, b, p, preceding);
		if (v == 0)
			return peerbounds(r, b, p, preceding);
		if (!is_int_type(tp1))
			goto type_not_supported;
		c.kind = K_INT;
		return range_bounds(r, &c, p, &L, preceding);
	}
	default:
		goto bound_not_supported;
	}
bound_not_supported:
	ora_seterr("42000!range frame bound type %s not supported.\n", tname(tp2));
	return -1;
type_not_supported:
	ora_seterr("42000!type %s not supported for %s frame bound type.\n", tname(tp1), tname(tp2));
	return -1;
invalid:
	ora_seterr("%s", ERR_INV);
	return -1;
}

int
ora_windowbounds(ora_bat *r, const ora_bat *b, const ora_bat *p, const ora_bat *l, const void *bound, int tp1,
		 int tp2, int unit, bool preceding, ora_oid second_half)
{
	switch (unit) {
	case 0:
		return rowbounds(r, b, p, l, bound, tp2, preceding, second_half, false);
	case 1:
		return rangebounds(r, b, p, l, bound, tp1, tp2, preceding);
	case 2:
		if (b->type != ORA_bit) {
			ora_seterr("42000!groups frame bound type must be of type bit.\n");
			return -1;
		}
		return rowbounds(r, b, p, l, bound, tp2, preceding, second_half, true);
	}
	ora_seterr("42000!unit type %d not supported (this is a bug).\n", unit);
	return -1;
}
