// analytic_win.hip -- window functions beyond the frame aggregates on the
// MI355X: GDKanalyticalntile (gdk/gdk_analytic_func.c:124), first (:230),
// last (:312), nth_value (:421), lag (:671), lead (:823) and min / max
// (:1264), the next consumers of the frame bounds of analytic.hip.
//
// The reference walks every partition row by row.  On the device each row
// is answered on its own:
//   * first / last / nth_value read the row's frame [s[i], e[i]);
//   * lag / lead / ntile find the row's partition [ps, pe) by binary search
//     over the compacted partition starts (segments.h) and apply the
//     reference's per-partition rule to the row's offset in it;
//   * min / max answer a range query on a (value, position) order: per
//     32-row block the best position of every prefix and suffix, a sparse
//     table over the block bests, so any [lo, hi) costs two table reads and
//     two block reads (a range inside one block is scanned).  The frame of
//     a row is [ps, end of its peer group) (frame 3), [start of its peer
//     group, pe) (4), [ps, pe) (5), the row (6) or [s[i], e[i]).  Nil never
//     wins; equal values resolve as the reference's scans do: frames 3 / 5
//     keep the earlier row, frame 4 (a backward scan) the later one.  For
//     general frames the reference folds a fanout-16 segment tree whose tie
//     order is neither: equal values are equal, so only a flt / dbl frame
//     whose extreme is both -0.0 and +0.0 can come back with the other
//     zero's sign (parity to ==, not to the bit).
#include <type_traits>

#include "mgdk_internal.h"
#include "segments.h"

using namespace mgdk;

namespace {

// peer-group starts: row 0, a partition start or a peer start
__global__ __launch_bounds__(256) void
k_or_flags_w(const int8_t *p, const int8_t *o, BUN n, int8_t *f)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		f[i] = i == 0 || (p && p[i]) || (o && o[i]);
}

template <typename T>
__device__ __forceinline__ bool
wnil(T v)
{
	return is_nil(v);
}

// the nil of T (flt / dbl: NaN)
template <typename T>
__device__ __forceinline__ T
wnilv()
{
	if constexpr (std::is_same<T, float>::value)
		return __builtin_nanf("");
	else if constexpr (std::is_same<T, double>::value)
		return __builtin_nan("");
	else
		return NilOf<T>::v();
}

// ---- first / last / nth_value ------------------------------------------

// MODE 0 first, 1 last, 2 nth_value with one n (nth0 = n - 1, or -1: nil
// n), 3 nth_value with a per-row lng n (the reference's bound test
// "lnth - 1 > frame size" lets lnth - 1 == size read the row after the
// frame; past the column that read is taken as nil)
template <typename T, int MODE>
__global__ __launch_bounds__(256) void
k_win_fl(const T *b, BUN n, const oid *s, const oid *e, const int64_t *tn, int64_t nth0, T *r, uint32_t *flags)
{
	uint32_t hasnil = 0, bad = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		const oid lo = s[k], hi = e[k];
		T v = wnilv<T>();
		if (MODE == 0) {
			if (hi > lo)
				v = b[lo];
		} else if (MODE == 1) {
			if (hi > lo)
				v = b[hi - 1];
		} else if (MODE == 2) {
			if (nth0 >= 0 && hi > lo && (BUN) nth0 < hi - lo)
				v = b[lo + nth0];
		} else {
			const int64_t ln = tn[k];
			if (ln != INT64_MIN && ln <= 0) {
				bad = 1;
			} else if (ln != INT64_MIN && hi > lo && ln - 1 <= (int64_t) (hi - lo)) {
				const BUN at = lo + (BUN) (ln - 1);
				if (at < n)
					v = b[at];
			}
		}
		r[k] = v;
		hasnil |= wnil(v);
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	bad = block_reduce(bad, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0) {
		publish_or(&flags[0], hasnil);
		publish_or(&flags[1], bad);
	}
}

// ---- lag / lead -------------------------------------------------------------

template <typename T, bool LEAD>
__global__ __launch_bounds__(256) void
k_win_lag(const T *b, BUN n, Starts part, BUN off, T def, T *r, uint32_t *flags)
{
	uint32_t hasnil = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		BUN ps, pe;
		part.seg(k, ps, pe);
		T v;
		if (!LEAD) {
			if (k - ps < off) {
				v = def;
			} else {
				v = b[k - off];
				hasnil |= wnil(v);
			}
		} else {
			if (off < pe - k) {
				v = b[k + off];
				hasnil |= wnil(v);
			} else {
				v = def;
			}
		}
		r[k] = v;
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(&flags[0], hasnil);
}

// ---- ntile ------------------------------------------------------------------

template <typename T>
__device__ __forceinline__ int64_t
ntile_lng(T v)
{
	if constexpr (std::is_same<T, hge>::value)
		return v > (hge) INT64_MAX ? INT64_MAX : (int64_t) v;     // GDK_lng_max clamp (:175)
	else
		return (int64_t) v;
}

template <typename T, bool MULTI>
__global__ __launch_bounds__(256) void
k_win_ntile(const T *nv, T one, BUN n, Starts part, T *r, uint32_t *flags)
{
	uint32_t hasnil = 0, bad = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		BUN ps, pe;
		part.seg(k, ps, pe);
		const T val = MULTI ? nv[k] : one;
		if (wnil(val)) {
			r[k] = wnilv<T>();
			hasnil = 1;
			continue;
		}
		const int64_t x = ntile_lng(val);
		if (x <= 0) {
			bad = 1;
			r[k] = wnilv<T>();
			continue;
		}
		const uint64_t nval = (uint64_t) x, ncnt = pe - ps, j = k - ps;
		uint64_t res;
		if (nval >= ncnt) {
			res = j + 1;
		} else {
			const uint64_t bsize = ncnt / nval, top = ncnt - nval * bsize, small = top * (bsize + 1);
			res = j < small ? 1 + j / (bsize + 1) : 1 + top + (j - small) / bsize;
		}
		r[k] = (T) res;
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	bad = block_reduce(bad, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0) {
		publish_or(&flags[0], hasnil);
		publish_or(&flags[1], bad);
	}
}

// ---- min / max range queries --------------------------------------------------

constexpr BUN MM_BLK = 32;

// the better of positions i and j: a non-nil value beats nil, the smaller
// (MAX: larger) value wins, equal values the earlier (LATE: later) row
template <typename T, bool MAX, bool LATE>
__device__ __forceinline__ BUN
mm_best(const T *b, BUN i, BUN j)
{
	const T x = b[i], y = b[j];
	const bool xn = wnil(x), yn = wnil(y);
	const bool tie_i = LATE ? i > j : i < j;
	if (xn || yn)
		return xn && !yn ? j : !xn && yn ? i : (tie_i ? i : j);
	if (MAX ? x > y : x < y)
		return i;
	if (MAX ? y > x : y < x)
		return j;
	return tie_i ? i : j;
}

// per block: best position of every prefix [block start, i] and suffix
// [i, block end); st0 = the block's best
template <typename T, bool MAX, bool LATE>
__global__ __launch_bounds__(256) void
k_mm_blocks(const T *b, BUN n, BUN *pre, BUN *suf, BUN *st0)
{
	const BUN nb = (n + MM_BLK - 1) / MM_BLK;
	for (BUN bk = (BUN) blockIdx.x * blockDim.x + threadIdx.x; bk < nb; bk += (BUN) gridDim.x * blockDim.x) {
		const BUN a = bk * MM_BLK, z = a + MM_BLK < n ? a + MM_BLK : n;
		BUN c = a;
		for (BUN i = a; i < z; i++) {
			c = i == a ? a : mm_best<T, MAX, LATE>(b, c, i);
			pre[i] = c;
		}
		st0[bk] = c;
		c = z - 1;
		for (BUN i = z; i-- > a;) {
			c = i == z - 1 ? i : mm_best<T, MAX, LATE>(b, i, c);
			suf[i] = c;
		}
	}
}

template <typename T, bool MAX, bool LATE>
__global__ __launch_bounds__(256) void
k_mm_level(const T *b, const BUN *prev, BUN nb, BUN half, BUN *cur)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i + 2 * half <= nb; i += (BUN) gridDim.x * blockDim.x)
		cur[i] = mm_best<T, MAX, LATE>(b, prev[i], prev[i + half]);
}

struct MmTab {
	const BUN *pre, *suf;
	const BUN *lev[40];      // sparse table levels over the blocks
	int nlev;
};

template <typename T, bool MAX, bool LATE>
__device__ __forceinline__ BUN
mm_query(const T *b, const MmTab &t, BUN lo, BUN hi)
{
	const BUN bl = lo / MM_BLK, bh = (hi - 1) / MM_BLK;
	if (bl == bh) {
		BUN c = lo;
		for (BUN i = lo + 1; i < hi; i++)
			c = mm_best<T, MAX, LATE>(b, c, i);
		return c;
	}
	BUN c = mm_best<T, MAX, LATE>(b, t.suf[lo], t.pre[hi - 1]);
	if (bh - bl >= 2) {
		const BUN a = bl + 1, cnt = bh - a;
		const int k = 63 - __clzll((long long) cnt);
		const BUN x = mm_best<T, MAX, LATE>(b, t.lev[k][a], t.lev[k][bh - ((BUN) 1 << k)]);
		c = mm_best<T, MAX, LATE>(b, c, x);
	}
	return c;
}

struct MmArgs {
	BUN n;
	int frame;
	Starts part, peer;
	const oid *s, *e;
	uint32_t *flags;
};

template <typename T, bool MAX, bool LATE>
__global__ __launch_bounds__(256) void
k_mm_query(const T *b, MmTab t, MmArgs a, T *r)
{
	uint32_t hasnil = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < a.n; k += (BUN) gridDim.x * blockDim.x) {
		BUN lo, hi, ps = 0, pe = 0, gs, ge;
		if (a.frame == 3 || a.frame == 4 || a.frame == 5)
			a.part.seg(k, ps, pe);
		switch (a.frame) {
		case 3: a.peer.seg(k, gs, ge); lo = ps; hi = ge; break;
		case 4: a.peer.seg(k, gs, ge); lo = gs; hi = pe; break;
		case 5: lo = ps; hi = pe; break;
		default: lo = a.s[k]; hi = a.e[k]; break;
		}
		T v = wnilv<T>();
		if (hi > lo)
			v = b[mm_query<T, MAX, LATE>(b, t, lo, hi)];
		r[k] = v;
		hasnil |= wnil(v);
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(&a.flags[0], hasnil);
}

template <typename T>
__global__ __launch_bounds__(256) void
k_win_copy(const T *b, BUN n, T *r, uint32_t *flags)
{
	uint32_t hasnil = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		const T v = b[k];
		r[k] = v;
		hasnil |= wnil(v);
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(&flags[0], hasnil);
}

// ---- GDKanalyticaldiff (gdk_analytic_bounds.c:95) -------------------------
// The reference compares each value with the last value that differed;
// equality is transitive here (-0.0 == +0.0, two NaNs the same when b has
// nils), so that value always equals the row before: one compare per row.
template <typename T>
__global__ __launch_bounds__(256) void
k_win_diff(const T *b, BUN n, const int8_t *np, int8_t npb, bool nanaware, int8_t *r)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		bool d = false;
		if (i > 0) {
			const T x = b[i - 1], y = b[i];
			d = x != y;
			if constexpr (std::is_floating_point<T>::value)
				d = d && (!nanaware || x == x || y == y);
		}
		r[i] = d ? 1 : np ? np[i] : npb;
	}
}

__device__ __forceinline__ const uint8_t *
wstr_at(const void *offs, int w, const char *vh, BUN p)
{
	size_t o;
	switch (w) {
	case 1: o = (size_t) ((const uint8_t *) offs)[p] + 8192; break;     // GDK_VAROFFSET
	case 2: o = (size_t) ((const uint16_t *) offs)[p] + 8192; break;
	case 4: o = (size_t) ((const uint32_t *) offs)[p]; break;
	default: o = (size_t) ((const uint64_t *) offs)[p]; break;
	}
	return (const uint8_t *) vh + o;
}

// strCmp != 0: nil ("\200") equals only nil, otherwise bytewise
__global__ __launch_bounds__(256) void
k_win_diff_str(const void *offs, int w, const char *vh, BUN n, const int8_t *np, int8_t npb, int8_t *r)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		bool d = false;
		if (i > 0) {
			const uint8_t *a = wstr_at(offs, w, vh, i - 1), *c = wstr_at(offs, w, vh, i);
			if (a != c) {
				const bool an = a[0] == 0x80 && a[1] == 0, cn = c[0] == 0x80 && c[1] == 0;
				if (an || cn) {
					d = an != cn;
				} else {
					for (;; a++, c++) {
						if (*a != *c) {
							d = true;
							break;
						}
						if (*a == 0)
							break;
					}
				}
			}
		}
		r[i] = d ? 1 : np ? np[i] : npb;
	}
}

// ---- host side -----------------------------------------------------------

// the storage class of a window function's values: 1 bte, 2 sht, 4 int,
// 8 lng, 16 hge, -4 flt, -8 dbl; 0 = not supported
int
wclass(int t)
{
	switch (basetype(t)) {
	case MGDK_bte: case MGDK_bit: return 1;
	case MGDK_sht: return 2;
	case MGDK_int: case MGDK_date: return 4;
	case MGDK_lng: case MGDK_oid: case MGDK_timestamp: case MGDK_daytime: return 8;
	case MGDK_hge: return 16;
	case MGDK_flt: return -4;
	case MGDK_dbl: return -8;
	default: return 0;
	}
}

#define WDISPATCH(CLS, F) \
	switch (CLS) { \
	case 1: F(int8_t); break; \
	case 2: F(int16_t); break; \
	case 4: F(int32_t); break; \
	case 8: F(int64_t); break; \
	case 16: F(hge); break; \
	case -4: F(float); break; \
	default: F(double); break; \
	}

bool
wcheck_r(mgdk_bat *r, mgdk_bat *b, int tpe, const char *fn)
{
	if (r == nullptr || b == nullptr) {
		seterr("%s: NULL argument", fn);
		return false;
	}
	if (wclass(tpe) == 0 || wclass(b->ttype) != wclass(tpe) || wclass(r->ttype) != wclass(tpe)) {
		seterr("42000!%s: type %s not supported on the device path", fn, atomname(tpe));
		return false;
	}
	if (r->theap == nullptr && b->count) {
		seterr("%s: result BAT has no heap", fn);
		return false;
	}
	return true;
}

bool
wcheck_bounds(mgdk_bat *s, mgdk_bat *e, BUN n)
{
	if (s == nullptr || e == nullptr || s->count < n || e->count < n || s->ttype != MGDK_oid || e->ttype != MGDK_oid) {
		seterr("analytic: frame bounds s and e (oid BATs aligned with b) are required");
		return false;
	}
	return true;
}

// flags[0] has nils, flags[1] invalid n; sets r's count and nil properties
int
wfinish(mgdk_bat *r, BUN n, uint32_t *dflags, bool extra_nil, const char *badmsg)
{
	uint32_t *h = (uint32_t *) pinned(16);
	if (!hip_ok(hipMemcpyAsync(h, dflags, 8, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return -1;
	if (h[1]) {
		seterr("%s", badmsg);
		return -1;
	}
	const bool hasnil = h[0] != 0 || extra_nil;
	r->count = n;
	r->tnil = hasnil;
	r->tnonil = !hasnil;
	r->tsorted = r->trevsorted = r->tkey = n <= 1;
	return 0;
}

bool
is_nil_val(int cls, const void *v)
{
	switch (cls) {
	case 1: return *(const int8_t *) v == INT8_MIN;
	case 2: return *(const int16_t *) v == INT16_MIN;
	case 4: return *(const int32_t *) v == INT32_MIN;
	case 8: return *(const int64_t *) v == INT64_MIN;
	case 16: return *(const hge *) v == NilOf<hge>::v();
	case -4: { float f; memcpy(&f, v, 4); return f != f; }
	default: { double d; memcpy(&d, v, 8); return d != d; }
	}
}

bool
bits_ok(mgdk_bat *p, BUN n)
{
	if (p && (p->count != n || width_of(p->ttype) != 1)) {
		seterr("analytic: p and o must be bit BATs aligned with b");
		return false;
	}
	return true;
}

int
fl_run(int mode, mgdk_bat *r, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, mgdk_bat *t, const int64_t *pnth, int tpe,
       const char *fn)
{
	if (!wcheck_r(r, b, tpe, fn))
		return -1;
	const BUN n = b->count;
	if (n == 0) {
		r->count = 0;
		r->tnil = 0;
		r->tnonil = 1;
		return 0;
	}
	if (!wcheck_bounds(s, e, n))
		return -1;
	if (mode == 3 && (t->ttype != MGDK_lng || t->count < n)) {
		seterr("42000!type %s not supported for the nth_value.\n", atomname(t->ttype));
		return -1;
	}
	int64_t nth0 = -1;
	if (mode == 2) {
		if (*pnth != INT64_MIN && *pnth <= 0) {
			seterr("42000!nth_value must be greater than zero.\n");
			return -1;
		}
		nth0 = *pnth == INT64_MIN ? -1 : *pnth - 1;
	}
	// flags in a buffer of their own: make_starts uses meta_buf()
	DevBuf flb(64);
	uint32_t *fl = flb.as<uint32_t>();
	if (fl == nullptr)
		return -1;
	hipStream_t st = stream();
	if (!hip_ok(hipMemsetAsync(fl, 0, 8, st), "memset"))
		return -1;
	const dim3 g(grid_for(n, 1024, 16384)), blk(256);
	const oid *S = (const oid *) s->theap, *E = (const oid *) e->theap;
	const int64_t *tn = t ? (const int64_t *) t->theap : nullptr;
#define FL(T) do { \
		switch (mode) { \
		case 0: hipLaunchKernelGGL((k_win_fl<T, 0>), g, blk, 0, st, (const T *) b->theap, n, S, E, tn, nth0, (T *) r->theap, fl); break; \
		case 1: hipLaunchKernelGGL((k_win_fl<T, 1>), g, blk, 0, st, (const T *) b->theap, n, S, E, tn, nth0, (T *) r->theap, fl); break; \
		case 2: hipLaunchKernelGGL((k_win_fl<T, 2>), g, blk, 0, st, (const T *) b->theap, n, S, E, tn, nth0, (T *) r->theap, fl); break; \
		default: hipLaunchKernelGGL((k_win_fl<T, 3>), g, blk, 0, st, (const T *) b->theap, n, S, E, tn, nth0, (T *) r->theap, fl); break; \
		} } while (0)
	WDISPATCH(wclass(tpe), FL)
#undef FL
	return wfinish(r, n, fl, mode == 2 && nth0 < 0, "42000!nth_value must be greater than zero.\n");
}

int
lag_run(bool lead, mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, BUN off, const void *def, int tpe, const char *fn)
{
	if (!wcheck_r(r, b, tpe, fn))
		return -1;
	if (def == nullptr) {
		seterr("%s: a default value is required", fn);
		return -1;
	}
	const BUN n = b->count;
	const int cls = wclass(tpe);
	if (n == 0) {
		r->count = 0;
		r->tnil = 0;
		r->tnonil = 1;
		return 0;
	}
	if (!bits_ok(p, n))
		return -1;
	// flags in a buffer of their own: make_starts uses meta_buf()
	DevBuf flb(64);
	uint32_t *fl = flb.as<uint32_t>();
	if (fl == nullptr)
		return -1;
	hipStream_t st = stream();
	if (!hip_ok(hipMemsetAsync(fl, 0, 8, st), "memset"))
		return -1;
	const dim3 g(grid_for(n, 1024, 16384)), blk(256);
	if (off == MGDK_BUN_NONE) {
		// BUN_NONE: every row nil (:609-613)
		hge nilv[1];
		switch (cls) {
		case 1: *(int8_t *) nilv = INT8_MIN; break;
		case 2: *(int16_t *) nilv = INT16_MIN; break;
		case 4: *(int32_t *) nilv = INT32_MIN; break;
		case 8: *(int64_t *) nilv = INT64_MIN; break;
		case 16: *nilv = NilOf<hge>::v(); break;
		case -4: { float f = __builtin_nanf(""); memcpy(nilv, &f, 4); break; }
		default: { double d = __builtin_nan(""); memcpy(nilv, &d, 8); break; }
		}
		Starts whole{};
		whole.m = 1;
		whole.n = n;
#define NL(T) do { T dv; memcpy(&dv, nilv, sizeof(T)); \
		hipLaunchKernelGGL((k_win_lag<T, false>), g, blk, 0, st, (const T *) b->theap, n, whole, (BUN) INT64_MAX, dv, (T *) r->theap, fl); } while (0)
		WDISPATCH(cls, NL)
#undef NL
		return wfinish(r, n, fl, true, "");
	}
	Starts part{};
	mgdk_bat *keep = nullptr;
	if (make_starts(p ? (const int8_t *) p->theap : nullptr, n, part, &keep) < 0)
		return -1;
#define LG(T) do { T dv; memcpy(&dv, def, sizeof(T)); \
		if (lead) hipLaunchKernelGGL((k_win_lag<T, true>), g, blk, 0, st, (const T *) b->theap, n, part, off, dv, (T *) r->theap, fl); \
		else hipLaunchKernelGGL((k_win_lag<T, false>), g, blk, 0, st, (const T *) b->theap, n, part, off, dv, (T *) r->theap, fl); } while (0)
	WDISPATCH(cls, LG)
#undef LG
	// has_nils |= (off > 0 && nil(default)) once per partition walk (:590, :760)
	const int rc = wfinish(r, n, fl, off > 0 && is_nil_val(cls, def), "");
	mgdk_BBPunfix(keep);
	return rc;
}

template <typename T, bool MAX, bool LATE>
int
mm_build_query(mgdk_bat *r, mgdk_bat *b, const MmArgs &a)
{
	hipStream_t st = stream();
	const BUN n = a.n, nb = (n + MM_BLK - 1) / MM_BLK;
	int nlev = 1;
	while (((BUN) 1 << nlev) <= nb)
		nlev++;
	DevBuf pre(n * 8 + 8), suf(n * 8 + 8), tab((size_t) nb * nlev * 8 + 8);
	if (!pre.p || !suf.p || !tab.p)
		return -1;
	const T *bv = (const T *) b->theap;
	const dim3 blk(256);
	hipLaunchKernelGGL((k_mm_blocks<T, MAX, LATE>), dim3(grid_for(nb, 256, 16384)), blk, 0, st, bv, n, pre.as<BUN>(),
			   suf.as<BUN>(), tab.as<BUN>());
	MmTab t{};
	t.pre = pre.as<BUN>();
	t.suf = suf.as<BUN>();
	t.nlev = nlev;
	t.lev[0] = tab.as<BUN>();
	for (int l = 1; l < nlev; l++) {
		BUN *cur = tab.as<BUN>() + (size_t) l * nb;
		const BUN half = (BUN) 1 << (l - 1);
		hipLaunchKernelGGL((k_mm_level<T, MAX, LATE>), dim3(grid_for(nb, 1024, 16384)), blk, 0, st, bv,
				   t.lev[l - 1], nb, half, cur);
		t.lev[l] = cur;
	}
	hipLaunchKernelGGL((k_mm_query<T, MAX, LATE>), dim3(grid_for(n, 1024, 16384)), blk, 0, st, bv, t, a,
			   (T *) r->theap);
	return wfinish(r, n, a.flags, false, "");
}

template <typename T>
int
mm_dispatch(bool ismax, bool late, mgdk_bat *r, mgdk_bat *b, const MmArgs &a)
{
	if (ismax)
		return late ? mm_build_query<T, true, true>(r, b, a) : mm_build_query<T, true, false>(r, b, a);
	return late ? mm_build_query<T, false, true>(r, b, a) : mm_build_query<T, false, false>(r, b, a);
}

int
minmax_run(bool ismax, mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
	   int frame_type, const char *fn)
{
	if (!wcheck_r(r, b, tpe, fn))
		return -1;
	const BUN n = b->count;
	if (n == 0) {
		r->count = 0;
		r->tnil = 0;
		r->tnonil = 1;
		return 0;
	}
	if (!bits_ok(p, n) || !bits_ok(o, n))
		return -1;
	const bool frames = !(frame_type >= 3 && frame_type <= 6);
	if (frames && !wcheck_bounds(s, e, n))
		return -1;
	if ((frame_type == 3 || frame_type == 4) && o == nullptr) {
		seterr("analytic: the peer column o is required for this frame");
		return -1;
	}
	hipStream_t st = stream();
	// flags in a buffer of their own: make_starts uses meta_buf()
	DevBuf flb(64);
	uint32_t *fl = flb.as<uint32_t>();
	if (fl == nullptr)
		return -1;
	if (!hip_ok(hipMemsetAsync(fl, 0, 8, st), "memset"))
		return -1;
	const int cls = wclass(tpe);
	if (frame_type == 6) {
		const dim3 g(grid_for(n, 1024, 16384)), blk(256);
#define CP(T) hipLaunchKernelGGL((k_win_copy<T>), g, blk, 0, st, (const T *) b->theap, n, (T *) r->theap, fl)
		WDISPATCH(cls, CP)
#undef CP
		return wfinish(r, n, fl, false, "");
	}
	MmArgs a{};
	a.n = n;
	a.frame = frame_type;
	a.s = frames ? (const oid *) s->theap : nullptr;
	a.e = frames ? (const oid *) e->theap : nullptr;
	a.flags = fl;
	mgdk_bat *kp = nullptr, *kg = nullptr;
	DevBuf gf(n + 8);
	int rc = -1;
	if (!gf.p || make_starts(p ? (const int8_t *) p->theap : nullptr, n, a.part, &kp) < 0)
		goto out;
	if (frame_type == 3 || frame_type == 4) {
		// peer groups restart at every partition start
		hipLaunchKernelGGL(k_or_flags_w, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st,
				   p ? (const int8_t *) p->theap : nullptr, (const int8_t *) o->theap, n, gf.as<int8_t>());
		if (make_starts(gf.as<int8_t>(), n, a.peer, &kg) < 0)
			goto out;
	}
	{
		// frame 4 is a backward scan in the reference: ties keep the later row
		const bool late = frame_type == 4;
#define MM(T) rc = mm_dispatch<T>(ismax, late, r, b, a)
		WDISPATCH(cls, MM)
#undef MM
	}
out:
	mgdk_BBPunfix(kp);
	mgdk_BBPunfix(kg);
	return rc;
}

}  // namespace

extern "C" int
mgdk_GDKanalyticalfirst(mgdk_bat *r, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe)
{
	ProfScope prof("analyticalfirst");
	return fl_run(0, r, b, s, e, nullptr, nullptr, tpe, "GDKanalyticalfirst");
}

extern "C" int
mgdk_GDKanalyticallast(mgdk_bat *r, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe)
{
	ProfScope prof("analyticallast");
	return fl_run(1, r, b, s, e, nullptr, nullptr, tpe, "GDKanalyticallast");
}

extern "C" int
mgdk_GDKanalyticalnthvalue(mgdk_bat *r, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, mgdk_bat *t, const int64_t *pnth,
			   int tpe)
{
	ProfScope prof("analyticalnthvalue");
	if (t == nullptr && pnth == nullptr) {
		seterr("GDKanalyticalnthvalue: nth or t is required");
		return -1;
	}
	return fl_run(t ? 3 : 2, r, b, s, e, t, pnth, tpe, "GDKanalyticalnthvalue");
}

extern "C" int
mgdk_GDKanalyticallag(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_BUN lag, const void *default_value, int tpe)
{
	ProfScope prof("analyticallag");
	return lag_run(false, r, b, p, lag, default_value, tpe, "GDKanalyticallag");
}

extern "C" int
mgdk_GDKanalyticallead(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_BUN lead, const void *default_value, int tpe)
{
	ProfScope prof("analyticallead");
	return lag_run(true, r, b, p, lead, default_value, tpe, "GDKanalyticallead");
}

extern "C" int
mgdk_GDKanalyticalntile(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_bat *n, int tpe, const void *ntile)
{
	ProfScope prof("analyticalntile");
	if (r == nullptr || b == nullptr || ((n == nullptr) == (ntile == nullptr))) {
		seterr("GDKanalyticalntile: exactly one of n and ntile is required");
		return -1;
	}
	const int cls = wclass(tpe);
	if (!(cls == 1 || cls == 2 || cls == 4 || cls == 8 || cls == 16) || basetype(tpe) == MGDK_oid ||
	    wclass(r->ttype) != cls || (n && wclass(n->ttype) != cls)) {
		seterr("42000!type %s not supported for the ntile type.\n", atomname(tpe));
		return -1;
	}
	const BUN cnt = b->count;
	if (ntile) {
		hge v = 0;
		bool isn = is_nil_val(cls, ntile);
		switch (cls) {
		case 1: v = *(const int8_t *) ntile; break;
		case 2: v = *(const int16_t *) ntile; break;
		case 4: v = *(const int32_t *) ntile; break;
		case 8: v = *(const int64_t *) ntile; break;
		default: v = *(const hge *) ntile; break;
		}
		if (!isn && v <= 0) {
			seterr("42000!ntile must be greater than zero.\n");
			return -1;
		}
	}
	if (cnt == 0) {
		r->count = 0;
		r->tnil = 0;
		r->tnonil = 1;
		return 0;
	}
	if (!bits_ok(p, cnt) || (n && n->count < cnt) || r->theap == nullptr) {
		if (n && n->count < cnt)
			seterr("GDKanalyticalntile: n must be aligned with b");
		return -1;
	}
	Starts part{};
	mgdk_bat *keep = nullptr;
	if (make_starts(p ? (const int8_t *) p->theap : nullptr, cnt, part, &keep) < 0)
		return -1;
	hipStream_t st = stream();
	// flags in a buffer of their own: make_starts uses meta_buf()
	DevBuf flb(64);
	uint32_t *fl = flb.as<uint32_t>();
	if (fl == nullptr)
		return -1;
	if (!hip_ok(hipMemsetAsync(fl, 0, 8, st), "memset")) {
		mgdk_BBPunfix(keep);
		return -1;
	}
	const dim3 g(grid_for(cnt, 1024, 16384)), blk(256);
#define NT(T) do { T one{}; if (ntile) memcpy(&one, ntile, sizeof(T)); \
		if (n) hipLaunchKernelGGL((k_win_ntile<T, true>), g, blk, 0, st, (const T *) n->theap, one, cnt, part, (T *) r->theap, fl); \
		else hipLaunchKernelGGL((k_win_ntile<T, false>), g, blk, 0, st, (const T *) nullptr, one, cnt, part, (T *) r->theap, fl); } while (0)
	switch (cls) {
	case 1: NT(int8_t); break;
	case 2: NT(int16_t); break;
	case 4: NT(int32_t); break;
	case 8: NT(int64_t); break;
	default: NT(hge); break;
	}
#undef NT
	const int rc = wfinish(r, cnt, fl, false, "42000!ntile must be greater than zero.\n");
	mgdk_BBPunfix(keep);
	return rc;
}

extern "C" int
mgdk_GDKanalyticalmin(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
		      int frame_type)
{
	ProfScope prof("analyticalmin");
	return minmax_run(false, r, p, o, b, s, e, tpe, frame_type, "GDKanalyticalmin");
}

extern "C" int
mgdk_GDKanalyticalmax(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
		      int frame_type)
{
	ProfScope prof("analyticalmax");
	return minmax_run(true, r, p, o, b, s, e, tpe, frame_type, "GDKanalyticalmax");
}

extern "C" int
mgdk_GDKanalyticaldiff(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, const int8_t *npbit, int tpe)
{
	ProfScope prof("analyticaldiff");
	if (r == nullptr || b == nullptr) {
		seterr("GDKanalyticaldiff: NULL argument");
		return -1;
	}
	const BUN n = b->count;
	const bool str = basetype(tpe) == MGDK_str;
	const int cls = str ? 0 : wclass(tpe);
	if ((!str && cls == 0) || (str && b->tvheap == nullptr) || width_of(r->ttype) != 1) {
		seterr("42000!GDKanalyticaldiff: type %s not supported on the device path", atomname(tpe));
		return -1;
	}
	if (n > 0 && (!bits_ok(p, n) || r->theap == nullptr))
		return -1;
	const int8_t *np = p ? (const int8_t *) p->theap : nullptr;
	const int8_t npb = npbit ? *npbit : 0;
	if (n > 0) {
		const dim3 g(grid_for(n, 1024, 16384)), blk(256);
		hipStream_t st = stream();
		int8_t *rb = (int8_t *) r->theap;
		if (str) {
			hipLaunchKernelGGL(k_win_diff_str, g, blk, 0, st, b->theap, (int) b->twidth, (const char *) b->tvheap, n, np,
					   npb, rb);
		} else {
			const bool nanaware = !b->tnonil;
#define DF(T) hipLaunchKernelGGL((k_win_diff<T>), g, blk, 0, st, (const T *) b->theap, n, np, npb, nanaware, rb)
			WDISPATCH(cls, DF)
#undef DF
		}
		if (!sync())
			return -1;
	}
	r->count = n;
	r->tnonil = 1;
	r->tnil = 0;
	r->tsorted = r->trevsorted = r->tkey = n <= 1;
	return 0;
}
