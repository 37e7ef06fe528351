// bounds.hip -- GDKanalyticalwindowbounds on the MI355X
// (gdk/gdk_analytic_bounds.c:1440): every frame unit, value type and limit
// kind of the reference.
//
//   ROWS   (GDKanalyticalrowbounds :855)    one pass: partition of each row
//          from the partition-start list, the bound is arithmetic
//   GROUPS (GDKanalyticalgroupsbounds :1296) the peer-group starts (set bits
//          of b) compacted once; a row's bound is the (L+1)-th start before /
//          after it, found by binary search -- no walk
//   RANGE  (GDKanalyticalrangebounds :994)
//          - bte..lng values with a static limit: the lng machinery of
//            analytic.hip (narrow types widened once; overflow of the
//            type's own range from the stopping pair)
//          - everything else (hge, flt, dbl, date / daytime / timestamp with
//            month or msec intervals, per-row limits l): one lane per row;
//            when every partition is ordered (asc, nils first / desc, nils
//            last, checked by k_rb_order) the frame edge is found by
//            galloping + binary search with the reference's exact in-frame
//            test (monotone along ordered data), else the reference's linear
//            walk is replayed
//   unbounded (GDKanalyticalallbounds :589) and RANGE limit 0
//          (GDKanalyticalpeers :710): bounds = the enclosing entry of a
//          sorted start list (partition starts / runs of equal values)
//
// Errors are those of the reference, reported for the first row (in the
// reference's row order) that raises one: the kernels record the smallest
// failing row per error kind.
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

// ---- sorted start lists (partition starts, run starts, peer starts) -------
struct Parts {
	const oid *S;       // sorted start rows (NULL: dense Sseq + i)
	oid Sseq;
	BUN ns;
	bool lead;          // row 0 starts a part that S does not list
	BUN m;              // number of parts = ns + lead
	BUN n;
};

__device__ __forceinline__ oid
ps_at(const Parts &P, BUN i)
{
	return P.S ? P.S[i] : P.Sseq + i;
}

__device__ __forceinline__ oid
ps_start(const Parts &P, BUN q)
{
	if (P.lead) {
		if (q == 0)
			return 0;
		q--;
	}
	return ps_at(P, q);
}

__device__ __forceinline__ BUN
ps_end(const Parts &P, BUN q)
{
	return q + 1 < P.m ? ps_start(P, q + 1) : P.n;
}

__device__ __forceinline__ BUN
ps_of(const Parts &P, BUN i)
{
	BUN lo = 0, hi = P.m;
	while (hi - lo > 1) {
		const BUN mid = (lo + hi) / 2;
		if (ps_start(P, mid) <= i) lo = mid; else hi = mid;
	}
	return lo;
}

// number of list entries <= i (upper bound)
__device__ __forceinline__ BUN
ps_upper(const Parts &P, BUN i)
{
	BUN lo = 0, hi = P.ns;
	while (lo < hi) {
		const BUN mid = (lo + hi) / 2;
		if (ps_at(P, mid) <= i) lo = mid + 1; else hi = mid;
	}
	return lo;
}

// number of list entries < i (lower bound)
__device__ __forceinline__ BUN
ps_lower(const Parts &P, BUN i)
{
	BUN lo = 0, hi = P.ns;
	while (lo < hi) {
		const BUN mid = (lo + hi) / 2;
		if (ps_at(P, mid) < i) lo = mid + 1; else hi = mid;
	}
	return lo;
}

__global__ void
k_rb_first(const oid *S, oid *out)
{
	*out = S[0];
}

// ---- limits -----------------------------------------------------------------
struct Lim {
	const void *l;      // per-row limits of type tp2, or NULL
	int tp2;
	hge si;             // static integer limit (validated)
	double sf;          // static flt / dbl limit (validated)
};

// integer limit of row k; false: nil or negative
__device__ __forceinline__ bool
lim_int(const Lim &L, BUN k, hge &v)
{
	if (L.l == nullptr) {
		v = L.si;
		return true;
	}
	bool nil;
	switch (L.tp2) {
	case MGDK_bte: { const int8_t x = ((const int8_t *) L.l)[k]; nil = x == INT8_MIN; v = x; break; }
	case MGDK_sht: { const int16_t x = ((const int16_t *) L.l)[k]; nil = x == INT16_MIN; v = x; break; }
	case MGDK_int: { const int32_t x = ((const int32_t *) L.l)[k]; nil = x == INT32_MIN; v = x; break; }
	case MGDK_lng: { const int64_t x = ((const int64_t *) L.l)[k]; nil = x == INT64_MIN; v = x; break; }
	default: { const hge x = ((const hge *) L.l)[k]; nil = is_nil(x); v = x; break; }
	}
	return !nil && v >= 0;
}

__device__ __forceinline__ bool
lim_flt(const Lim &L, BUN k, double &v)
{
	if (L.l == nullptr) {
		v = L.sf;
		return true;
	}
	v = L.tp2 == MGDK_flt ? (double) ((const float *) L.l)[k] : ((const double *) L.l)[k];
	return !(v != v) && v >= 0;
}

// ---- gdk_time.c (date_add_day :122, date_add_month :155, daytime_add_usec
//      :336, timestamp_add_usec :436, timestamp_add_month :459) ------------
constexpr int32_t DATE_NIL = INT32_MIN;
constexpr int64_t LNG_NIL = INT64_MIN;
constexpr int64_t DAY_USEC = 24LL * 60 * 60 * 1000000;
constexpr int YEAR_MIN = -4712, YEAR_MAX = -4712 + (1 << 21) / 12 - 1;

__device__ __forceinline__ int
mdays(int y, int m)
{
	const bool leap = y % 4 == 0 && (y % 100 != 0 || y % 400 == 0);
	const int d = m == 2 ? 29 : (m == 4 || m == 6 || m == 9 || m == 11) ? 30 : 31;
	return d - (m == 2 && !leap);
}

__device__ __forceinline__ int32_t
mkd(int y, int m, int d)
{
	return (int32_t) (((uint32_t) ((y + 4712) * 12 + m - 1) << 5) | (uint32_t) d);
}

__device__ int32_t
date_add_day(int32_t dt, int days)
{
	if (dt == DATE_NIL || days == INT32_MIN)
		return DATE_NIL;
	if ((days < 0 ? -days : days) >= 1 << 26)
		return DATE_NIL;
	const uint32_t u = (uint32_t) dt;
	int d = (int) (u & 31);
	int m = (int) (((u >> 5) & ((1u << 21) - 1)) % 12 + 1);
	int y = (int) (((u >> 5) & ((1u << 21) - 1)) / 12) - 4712;
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

__device__ int32_t
date_add_month(int32_t dt, int months)
{
	if (dt == DATE_NIL || months == INT32_MIN)
		return DATE_NIL;
	if ((months < 0 ? -months : months) >= 1 << 21)
		return DATE_NIL;
	const uint32_t u = (uint32_t) dt;
	int d = (int) (u & 31);
	int m = (int) (((u >> 5) & ((1u << 21) - 1)) % 12 + 1);
	int y = (int) (((u >> 5) & ((1u << 21) - 1)) / 12) - 4712;
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

__device__ __forceinline__ int64_t
daytime_add_usec(int64_t t, int64_t usec)
{
	if (t == LNG_NIL || usec == LNG_NIL)
		return LNG_NIL;
	if ((usec < 0 ? -usec : usec) >= DAY_USEC)
		return LNG_NIL;
	t += usec;
	return t < 0 || t >= DAY_USEC ? LNG_NIL : t;
}

__device__ int64_t
timestamp_add_usec(int64_t ts, int64_t usec)
{
	if (ts == LNG_NIL || usec == LNG_NIL)
		return LNG_NIL;
	int64_t tm = (int64_t) ((uint64_t) ts & ((1ull << 37) - 1));
	int32_t dt = (int32_t) (((uint64_t) ts >> 37) & ((1u << 26) - 1));
	tm += usec;
	if (tm < 0) {
		const int add = (int) ((DAY_USEC - 1 - tm) / DAY_USEC);
		tm += add * DAY_USEC;
		dt = date_add_day(dt, -add);
	} else if (tm >= DAY_USEC) {
		dt = date_add_day(dt, (int) (tm / DAY_USEC));
		tm %= DAY_USEC;
	}
	if (dt == DATE_NIL)
		return LNG_NIL;
	return (int64_t) (((uint64_t) (uint32_t) dt << 37) | (uint64_t) tm);
}

__device__ int64_t
timestamp_add_month(int64_t ts, int m)
{
	if (ts == LNG_NIL || m == INT32_MIN)
		return LNG_NIL;
	const int64_t tm = (int64_t) ((uint64_t) ts & ((1ull << 37) - 1));
	const int32_t dt = date_add_month((int32_t) (((uint64_t) ts >> 37) & ((1u << 26) - 1)), m);
	if (dt == DATE_NIL)
		return LNG_NIL;
	return (int64_t) (((uint64_t) (uint32_t) dt << 37) | (uint64_t) tm);
}

// ---- the in-frame test of one row against the current row ------------------
enum { K_INT = 0, K_FLT, K_DBL, K_MONTH, K_MSEC };
enum { T_NUM = 0, T_DATE, T_DAYTIME, T_TIMESTAMP };

template <typename V> __device__ __forceinline__ bool vnil(V x) { return is_nil(x); }

// per-row state: the current value and limit, or the temporal frame edges
template <typename V, int KIND, int TK>
struct Frame {
	hge vi, li, tmax;
	float vfl, lfl;
	double vdb, ldb;
	int64_t vmin, vmax;
	bool hasmin, hasmax;

	__device__ __forceinline__ void
	init(V v, hge il, double fl, hge tm)
	{
		tmax = tm;
		if (KIND == K_INT) {
			vi = (hge) v;
			li = il;
		} else if (KIND == K_FLT) {
			vfl = (float) v;
			lfl = (float) fl;
		} else if (KIND == K_DBL) {
			vdb = (double) v;
			ldb = fl;
		} else {
			const int64_t x = (int64_t) v;
			int64_t lo, hi;
			if (TK == T_DATE) {
				if (KIND == K_MONTH) {
					lo = date_add_month((int32_t) x, -(int) il);
					hi = date_add_month((int32_t) x, (int) il);
				} else {
					// date_add_msec: whole days of the msec limit
					lo = date_add_day((int32_t) x, (int) (-(int64_t) il / (24 * 60 * 60 * 1000)));
					hi = date_add_day((int32_t) x, (int) ((int64_t) il / (24 * 60 * 60 * 1000)));
				}
				hasmin = lo != DATE_NIL;
				hasmax = hi != DATE_NIL;
			} else if (TK == T_DAYTIME) {
				lo = daytime_add_usec(x, -1000 * (int64_t) il);
				hi = daytime_add_usec(x, 1000 * (int64_t) il);
				hasmin = lo != LNG_NIL;
				hasmax = hi != LNG_NIL;
			} else if (KIND == K_MONTH) {
				lo = timestamp_add_month(x, -(int) il);
				hi = timestamp_add_month(x, (int) il);
				hasmin = lo != LNG_NIL;
				hasmax = hi != LNG_NIL;
			} else {
				lo = timestamp_add_usec(x, -(int64_t) il * 1000);
				hi = timestamp_add_usec(x, (int64_t) il * 1000);
				hasmin = lo != LNG_NIL;
				hasmax = hi != LNG_NIL;
			}
			vmin = lo;
			vmax = hi;
		}
	}

	// 1: in the frame, 0: outside, 2: the subtraction overflows
	// (SUB_WITH_CHECK, gdk_calc_private.h:87, then ABSOLUTE(calc) > limit)
	__device__ __forceinline__ int
	test(V x) const
	{
		if (KIND == K_INT) {
			const hge xi = (hge) x;
			const bool ovf = xi < 1 ? tmax + xi < vi : -tmax + xi > vi;
			if (ovf)
				return 2;
			const hge d = vi - xi;
			return (d < 0 ? -d : d) <= li;
		} else if (KIND == K_FLT) {
			const float xf = (float) x, mx = 3.40282346638528859812e+38F;
			const bool ovf = xf < 1 ? __fadd_rn(mx, xf) < vfl : __fadd_rn(-mx, xf) > vfl;
			if (ovf)
				return 2;
			const float d = __fsub_rn(vfl, xf);
			return !((d < 0 ? -d : d) > lfl);
		} else if (KIND == K_DBL) {
			const double xd = (double) x, mx = 1.79769313486231570815e+308;
			const bool ovf = xd < 1 ? __dadd_rn(mx, xd) < vdb : __dadd_rn(-mx, xd) > vdb;
			if (ovf)
				return 2;
			const double d = __dsub_rn(vdb, xd);
			return !((d < 0 ? -d : d) > ldb);
		} else {
			const int64_t xi = (int64_t) x;
			return !((hasmin && xi < vmin) || (hasmax && xi > vmax));
		}
	}
};

template <typename V>
struct RArgs {
	const V *b;
	Parts P;
	Lim L;
	bool preceding;
	int order;                   // 0 unordered, 1 asc (nils first), 2 desc (nils last)
	hge tmax;
	oid *out;
	unsigned long long *err;     // [0] first row with an invalid limit, [1] first overflow row
};

template <typename V, int KIND, int TK>
__global__ __launch_bounds__(256) void
k_rb_range(RArgs<V> a)
{
	const BUN n = a.P.n;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		hge il = 0;
		double fl = 0;
		const bool okl = (KIND == K_FLT || KIND == K_DBL) ? lim_flt(a.L, k, fl) : lim_int(a.L, k, il);
		if (!okl) {
			atomicMin(&a.err[0], (unsigned long long) k);
			a.out[k] = k;
			continue;
		}
		const BUN pi = ps_of(a.P, k);
		const BUN m = ps_start(a.P, pi), e = ps_end(a.P, pi);
		const V v = a.b[k];
		const bool vn = vnil(v);
		Frame<V, KIND, TK> F;
		if (!vn)
			F.init(v, il, fl, a.tmax);
		BUN res;
		bool ovf = false;
		if (a.order) {
			const bool desc = a.order == 2;
			BUN lo = m, hi = e;              // nil-run boundary of [m, e)
			while (lo < hi) {
				const BUN mid = (lo + hi) / 2;
				const bool isn = vnil(a.b[mid]);
				if (desc ? !isn : isn) lo = mid + 1; else hi = mid;
			}
			const BUN z0 = lo;
			if (vn) {
				res = desc ? (a.preceding ? z0 : e) : (a.preceding ? m : z0);
			} else if (a.preceding) {
				// smallest j in [va, k] with [j, k] in the frame
				const BUN va = desc ? m : z0;
				BUN good = k, bad = 0;
				bool fb = false;
				for (BUN step = 1; k - va >= step; step <<= 1) {
					const BUN q = k - step;
					if (F.test(a.b[q]) == 1) good = q;
					else { bad = q; fb = true; break; }
				}
				if (!fb && good != va) {
					if (F.test(a.b[va]) == 1) good = va;
					else { bad = va; fb = true; }
				}
				if (fb) {
					while (good - bad > 1) {
						const BUN mid = bad + (good - bad) / 2;
						if (F.test(a.b[mid]) == 1) good = mid; else bad = mid;
					}
					ovf = F.test(a.b[bad]) == 2;
				}
				res = good;
			} else {
				// largest j in [k, vz) with [k, j] in the frame; bound j + 1
				const BUN vz = desc ? z0 : e;
				BUN good = k, bad = vz;
				for (BUN step = 1; k + step < vz; step <<= 1) {
					const BUN q = k + step;
					if (F.test(a.b[q]) == 1) good = q;
					else { bad = q; break; }
				}
				while (bad - good > 1) {
					const BUN mid = good + (bad - good) / 2;
					if (F.test(a.b[mid]) == 1) good = mid; else bad = mid;
				}
				if (bad < vz)
					ovf = F.test(a.b[bad]) == 2;
				res = good + 1;
			}
		} else {
			// the reference's walk (:273-369, :459-556)
			BUN j;
			if (a.preceding) {
				for (j = k;; j--) {
					const bool jn = vnil(a.b[j]);
					if (vn ? !jn : jn) { j++; break; }
					if (!vn) {
						const int t = F.test(a.b[j]);
						if (t == 2) { ovf = true; break; }
						if (t == 0) { j++; break; }
					}
					if (j == m)
						break;
				}
			} else {
				for (j = k + 1; j < e; j++) {
					const bool jn = vnil(a.b[j]);
					if (vn ? !jn : jn)
						break;
					if (!vn) {
						const int t = F.test(a.b[j]);
						if (t == 2) { ovf = true; break; }
						if (t == 0)
							break;
					}
				}
			}
			res = j;
		}
		if (ovf)
			atomicMin(&a.err[1], (unsigned long long) k);
		a.out[k] = res;
	}
}

// order of every partition: bit 0 = some pair violates ascending (nils
// first), bit 1 = some pair violates descending (nils last)
template <typename V>
__global__ __launch_bounds__(256) void
k_rb_order(const V *b, const int8_t *p, BUN n, uint32_t *flags)
{
	uint32_t f = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (BUN) gridDim.x * blockDim.x) {
		if (p && p[i + 1])
			continue;
		const V x = b[i], y = b[i + 1];
		const bool xn = vnil(x), yn = vnil(y);
		if ((!xn && yn) || (!xn && !yn && x > y))
			f |= 1;
		if ((xn && !yn) || (!xn && !yn && x < y))
			f |= 2;
	}
	f = block_reduce(f, [](uint32_t u, uint32_t w) { return u | w; });
	if (threadIdx.x == 0)
		publish_or(flags, f);
}

// run starts of GDKanalyticalpeers: partition starts and value changes
// (nils equal nils, flt / dbl NaN included)
template <typename V>
__global__ __launch_bounds__(256) void
k_rb_runflags(const V *b, const int8_t *p, BUN n, int8_t *f)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		bool s = k == 0 || (p && p[k]);
		if (!s) {
			const V x = b[k - 1], y = b[k];
			s = !(x == y || (vnil(x) && vnil(y)));
		}
		f[k] = s;
	}
}

// bound = start (PRECEDING) / end (FOLLOWING) of the enclosing list entry
__global__ __launch_bounds__(256) void
k_rb_list(Parts P, bool preceding, oid *out)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < P.n; k += (BUN) gridDim.x * blockDim.x) {
		const BUN q = ps_of(P, k);
		out[k] = preceding ? ps_start(P, q) : ps_end(P, q);
	}
}

// ROWS (:187-205): arithmetic on the partition [m, e)
__global__ __launch_bounds__(256) void
k_rb_rows(Parts P, Lim L, bool preceding, oid second_half, oid *out, unsigned long long *err)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < P.n; k += (BUN) gridDim.x * blockDim.x) {
		hge il;
		if (!lim_int(L, k, il)) {
			atomicMin(&err[0], (unsigned long long) k);
			out[k] = k;
			continue;
		}
		const oid rl = il > (hge) INT64_MAX ? (oid) INT64_MAX : (oid) il;
		const BUN q = ps_of(P, k);
		const BUN m = ps_start(P, q), e = ps_end(P, q);
		if (preceding) {
			out[k] = rl > k - m ? m : k - rl + second_half;
		} else {
			const oid rl2 = rl + second_half;
			out[k] = rl2 > e - k ? e : k + rl2;
		}
	}
}

// GROUPS (:224-271): G = the set bits of b (peer-group starts); walking
// back from k the walk stops at the (L+1)-th start it meets, forward at
// the (L+1)-th start after k
__global__ __launch_bounds__(256) void
k_rb_groups(Parts P, Parts G, Lim L, bool preceding, oid *out, unsigned long long *err)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < P.n; k += (BUN) gridDim.x * blockDim.x) {
		hge il;
		if (!lim_int(L, k, il)) {
			atomicMin(&err[0], (unsigned long long) k);
			out[k] = k;
			continue;
		}
		const oid rl = il > (hge) INT64_MAX ? (oid) INT64_MAX : (oid) il;
		const BUN q = ps_of(P, k);
		const BUN m = ps_start(P, q), e = ps_end(P, q);
		const BUN ck = ps_upper(G, k);
		if (preceding) {
			const BUN cm = ps_lower(G, m);
			out[k] = ck > cm && rl < ck - cm ? ps_at(G, ck - 1 - rl) : m;
		} else {
			const BUN idx = ck + rl;
			out[k] = idx < G.ns && idx >= ck && ps_at(G, idx) < e ? ps_at(G, idx) : e;
		}
	}
}

template <typename T>
__global__ __launch_bounds__(256) void
k_rb_widen(const T *in, int64_t *out, BUN n)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const T x = in[i];
		out[i] = x == NilOf<T>::v() ? INT64_MIN : (int64_t) x;
	}
}

// ---- host -------------------------------------------------------------------
// a sorted start list from flags (compact_flags); owns the list BAT
struct HostList {
	Parts P{};
	mgdk_bat *S = nullptr;
	~HostList() { mgdk_BBPunfix(S); }
};

// flags: n bytes, nonzero = start; with_row0: row 0 always starts a part
int
make_list(HostList &H, const int8_t *flags, BUN n, bool with_row0)
{
	H.P.n = n;
	H.P.S = nullptr;
	H.P.Sseq = 0;
	H.P.ns = 0;
	if (flags && n) {
		H.S = compact_flags(flags, n, 0, true);
		if (H.S == nullptr)
			return -1;
		H.P.S = H.S->ttype == MGDK_void ? nullptr : (const oid *) H.S->theap;
		H.P.Sseq = H.S->tseqbase;
		H.P.ns = H.S->count;
	}
	bool first0 = false;
	if (H.P.ns > 0) {
		if (H.P.S == nullptr) {
			first0 = H.P.Sseq == 0;
		} else {
			oid *d = (oid *) meta_buf();
			oid *h = (oid *) pinned(8);
			if (!d || !h)
				return -1;
			hipLaunchKernelGGL(k_rb_first, dim3(1), dim3(1), 0, stream(), H.P.S, d);
			if (!hip_ok(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
				return -1;
			first0 = *h == 0;
		}
	}
	H.P.lead = with_row0 && !first0;
	H.P.m = H.P.ns + (H.P.lead ? 1 : 0);
	return 0;
}

bool
is_mtime(int tp)
{
	return tp == MGDK_date || tp == MGDK_daytime || tp == MGDK_timestamp;
}

bool
is_int(int tp)
{
	return tp == MGDK_bte || tp == MGDK_sht || tp == MGDK_int || tp == MGDK_lng || tp == MGDK_hge;
}

hge
tmax_of(int tp)
{
	switch (tp) {
	case MGDK_bte: return INT8_MAX;
	case MGDK_sht: return INT16_MAX;
	case MGDK_int: return INT32_MAX;
	case MGDK_lng: return INT64_MAX;
	default: return (hge) (((uhge) 1 << 127) - 1);
	}
}

// static integer limit of type tp: value + nil flag
hge
static_int(const void *bound, int tp, bool *nil)
{
	switch (tp) {
	case MGDK_bte: { const int8_t x = *(const int8_t *) bound; *nil = x == INT8_MIN; return x; }
	case MGDK_sht: { const int16_t x = *(const int16_t *) bound; *nil = x == INT16_MIN; return x; }
	case MGDK_int: { const int32_t x = *(const int32_t *) bound; *nil = x == INT32_MIN; return x; }
	case MGDK_lng: { const int64_t x = *(const int64_t *) bound; *nil = x == INT64_MIN; return x; }
	default: { hge x; memcpy(&x, bound, sizeof(x)); *nil = is_nil(x); return x; }
	}
}

// the error of the first failing row (invalid limit / overflow)
int
report(const unsigned long long *h, const char *inv)
{
	if (h[0] == ~0ull && h[1] == ~0ull)
		return 0;
	if (h[0] <= h[1])
		seterr("%s", inv);
	else
		seterr("22003!overflow in calculation.\n");
	return -1;
}

int
run_list_bounds(const HostList &H, bool preceding, oid *out)
{
	if (H.P.n)
		hipLaunchKernelGGL(k_rb_list, dim3(grid_for(H.P.n, 1024, 16384)), dim3(256), 0, stream(), H.P, preceding,
				   out);
	return sync() ? 0 : -1;
}

template <typename V>
int
run_peers(const mgdk_bat *b, const mgdk_bat *p, bool preceding, oid *out)
{
	const BUN n = b->count;
	if (n == 0)
		return 0;
	DevBuf f(n);
	if (!f.p)
		return -1;
	hipLaunchKernelGGL(k_rb_runflags<V>, dim3(grid_for(n, 1024, 16384)), dim3(256), 0, stream(), (const V *) b->theap,
			   p ? (const int8_t *) p->theap : nullptr, n, f.as<int8_t>());
	HostList R;
	if (make_list(R, f.as<int8_t>(), n, false) < 0)
		return -1;
	return run_list_bounds(R, preceding, out);
}

int
peers_any(const mgdk_bat *b, const mgdk_bat *p, bool preceding, oid *out)
{
	switch (b->ttype == MGDK_flt ? MGDK_flt : b->ttype == MGDK_dbl ? MGDK_dbl : basetype(b->ttype)) {
	case MGDK_bte: return run_peers<int8_t>(b, p, preceding, out);
	case MGDK_sht: return run_peers<int16_t>(b, p, preceding, out);
	case MGDK_int: return run_peers<int32_t>(b, p, preceding, out);
	case MGDK_lng: case MGDK_oid: return run_peers<int64_t>(b, p, preceding, out);
	case MGDK_hge: return run_peers<hge>(b, p, preceding, out);
	case MGDK_flt: return run_peers<float>(b, p, preceding, out);
	case MGDK_dbl: return run_peers<double>(b, p, preceding, out);
	}
	seterr("42000!window bounds: type %s not supported on the device path", atomname(b->ttype));
	return -1;
}

template <typename V, int KIND, int TK>
int
run_range(const mgdk_bat *b, const mgdk_bat *p, const HostList &H, const Lim &L, hge tmax, bool preceding, oid *out,
	  const char *inv)
{
	const BUN n = b->count;
	unsigned long long *err = (unsigned long long *) meta_buf();
	uint32_t *flags = (uint32_t *) (err + 2);
	unsigned long long *h = (unsigned long long *) pinned(64);
	if (!err || !h || !hip_ok(hipMemsetAsync(err, 0xff, 16, stream()), "memset") ||
	    !hip_ok(hipMemsetAsync(flags, 0, 4, stream()), "memset"))
		return -1;
	hipLaunchKernelGGL(k_rb_order<V>, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, stream(), (const V *) b->theap,
			   p ? (const int8_t *) p->theap : nullptr, n, flags);
	if (!hip_ok(hipMemcpyAsync(h, flags, 4, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return -1;
	const uint32_t f = *(uint32_t *) h;
	RArgs<V> a;
	a.b = (const V *) b->theap;
	a.P = H.P;
	a.L = L;
	a.preceding = preceding;
	a.order = !(f & 1) ? 1 : !(f & 2) ? 2 : 0;
	a.tmax = tmax;
	a.out = out;
	a.err = err;
	hipLaunchKernelGGL((k_rb_range<V, KIND, TK>), dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream(), a);
	if (!hip_ok(hipMemcpyAsync(h, err, 16, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return -1;
	return report(h, inv);
}

// RANGE over the generic kernel: dispatch on the value type and limit kind
int
range_generic(const mgdk_bat *b, const mgdk_bat *p, const HostList &H, const Lim &L, int tp1, int kind, bool preceding,
	      oid *out, const char *inv)
{
	const hge tmax = tmax_of(basetype(tp1));
	if (kind == K_FLT)
		return run_range<float, K_FLT, T_NUM>(b, p, H, L, tmax, preceding, out, inv);
	if (kind == K_DBL)
		return run_range<double, K_DBL, T_NUM>(b, p, H, L, tmax, preceding, out, inv);
	if (kind == K_INT) {
		switch (basetype(tp1)) {
		case MGDK_bte: return run_range<int8_t, K_INT, T_NUM>(b, p, H, L, tmax, preceding, out, inv);
		case MGDK_sht: return run_range<int16_t, K_INT, T_NUM>(b, p, H, L, tmax, preceding, out, inv);
		case MGDK_int: return run_range<int32_t, K_INT, T_NUM>(b, p, H, L, tmax, preceding, out, inv);
		case MGDK_lng: return run_range<int64_t, K_INT, T_NUM>(b, p, H, L, tmax, preceding, out, inv);
		default: return run_range<hge, K_INT, T_NUM>(b, p, H, L, tmax, preceding, out, inv);
		}
	}
	if (tp1 == MGDK_date)
		return kind == K_MONTH ? run_range<int32_t, K_MONTH, T_DATE>(b, p, H, L, tmax, preceding, out, inv)
				       : run_range<int32_t, K_MSEC, T_DATE>(b, p, H, L, tmax, preceding, out, inv);
	if (tp1 == MGDK_daytime)
		return run_range<int64_t, K_MSEC, T_DAYTIME>(b, p, H, L, tmax, preceding, out, inv);
	return kind == K_MONTH ? run_range<int64_t, K_MONTH, T_TIMESTAMP>(b, p, H, L, tmax, preceding, out, inv)
			       : run_range<int64_t, K_MSEC, T_TIMESTAMP>(b, p, H, L, tmax, preceding, out, inv);
}

}  // namespace

extern "C" int
mgdk_GDKanalyticalwindowbounds(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_bat *l, const void *bound,
			       int tp1, int tp2, int unit, bool preceding, mgdk_oid second_half)
{
	if (r == nullptr || b == nullptr) {
		seterr("GDKanalyticalwindowbounds: NULL argument");
		return -1;
	}
	if ((l == nullptr) == (bound == nullptr)) {
		seterr("GDKanalyticalwindowbounds: exactly one of l and bound must be given");
		return -1;
	}
	const BUN n = b->count;
	if (p && (p->count != n || width_of(p->ttype) != 1)) {
		seterr("window bounds: partition column must be a bit BAT aligned with b");
		return -1;
	}
	if (l && l->count != n) {
		seterr("window bounds: limit column must be aligned with b");
		return -1;
	}
	if (l && basetype(l->ttype) != basetype(tp2)) {
		seterr("window bounds: limit column type %s does not match %s", atomname(l->ttype), atomname(tp2));
		return -1;
	}
	// r is caller-allocated with room for count(b) oids (sql_rank.c:161)
	if (r->ttype != MGDK_oid || (n > 0 && r->theap == nullptr)) {
		seterr("window bounds: result must be an oid BAT");
		return -1;
	}
	if (b->ttype == MGDK_void || b->ttype == MGDK_str) {
		seterr("42000!window bounds: type %s not supported on the device path", atomname(b->ttype));
		return -1;
	}
	ProfScope prof("windowbounds");
	oid *out = (oid *) r->theap;
	const int8_t *pb = p ? (const int8_t *) p->theap : nullptr;
	Lim L{l ? l->theap : nullptr, tp2, 0, 0};
	bool special = false;    // unbounded / peers: the reference leaves tnonil false
	int rc = 0;

	if (unit == 0 || unit == 2) {
		const bool groups = unit == 2;
		const char *inv = groups ? "42000!groups frame bound must be non negative and non null.\n"
					 : "42000!row frame bound must be non negative and non null.\n";
		if (groups && b->ttype != MGDK_bit) {
			seterr("42000!groups frame bound type must be of type bit.\n");
			return -1;
		}
		if (!is_int(tp2)) {
			seterr("42000!%s frame bound type %s not supported.\n", groups ? "groups" : "rows", atomname(tp2));
			return -1;
		}
		if (l) {
			if (l->tnil) {
				seterr("%s", inv);
				return -1;
			}
		} else {
			bool nil;
			const hge v = static_int(bound, tp2, &nil);
			if (!nil && v >= (hge) INT64_MAX)
				special = true;          // GDKanalyticalallbounds
			else if (nil || v < 0) {
				seterr("%s", inv);
				return -1;
			}
			L.si = v;
		}
		HostList H;
		if (make_list(H, pb, n, true) < 0)
			return -1;
		if (special) {
			rc = run_list_bounds(H, preceding, out);
		} else if (n) {
			// the peer-start list first: make_list / compact_flags use the
			// thread's meta buffer that holds the error rows below
			HostList G;
			if (groups && make_list(G, (const int8_t *) b->theap, n, false) < 0)
				return -1;
			unsigned long long *err = (unsigned long long *) meta_buf();
			unsigned long long *h = (unsigned long long *) pinned(64);
			if (!err || !h || !hip_ok(hipMemsetAsync(err, 0xff, 16, stream()), "memset"))
				return -1;
			if (groups) {
				hipLaunchKernelGGL(k_rb_groups, dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream(), H.P, G.P,
						   L, preceding, out, err);
				if (!hip_ok(hipMemcpyAsync(h, err, 16, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
					return -1;
			} else {
				hipLaunchKernelGGL(k_rb_rows, dim3(grid_for(n, 256, 65536)), dim3(256), 0, stream(), H.P, L,
						   preceding, (oid) second_half, out, err);
				if (!hip_ok(hipMemcpyAsync(h, err, 16, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
					return -1;
			}
			rc = report(h, inv);
		}
	} else if (unit == 1) {
		const char *inv = "42000!range frame bound must be non negative and non null.\n";
		if (basetype(b->ttype) != basetype(tp1) && !(b->ttype == MGDK_bit && tp1 == MGDK_bte)) {
			seterr("window bounds: tp1 %s does not match the column type %s", atomname(tp1), atomname(b->ttype));
			return -1;
		}
		if (is_mtime(tp1) && tp2 != MGDK_int && tp2 != MGDK_lng) {
			seterr("42000!range frame bound type %s not supported.\n", atomname(tp2));
			return -1;
		}
		int kind = -1;
		bool fast = false, peers = false;
		hge slimit = 0;
		const bool numint = tp1 == MGDK_bte || tp1 == MGDK_sht || tp1 == MGDK_int || tp1 == MGDK_lng;
		if (l) {
			if (l->tnil) {
				seterr("%s", inv);
				return -1;
			}
			switch (tp2) {
			case MGDK_bte: case MGDK_sht:
				kind = numint ? K_INT : -2;
				break;
			case MGDK_int: case MGDK_lng:
				if (is_mtime(tp1))
					kind = tp2 == MGDK_int ? (tp1 == MGDK_daytime ? -2 : K_MONTH) : K_MSEC;
				else
					kind = numint ? K_INT : -2;
				break;
			case MGDK_flt: kind = tp1 == MGDK_flt ? K_FLT : -2; break;
			case MGDK_dbl: kind = tp1 == MGDK_dbl ? K_DBL : -2; break;
			case MGDK_hge: kind = is_int(tp1) ? K_INT : -2; break;
			default: kind = -1; break;
			}
		} else {
			switch (tp2) {
			case MGDK_bte: case MGDK_sht: case MGDK_int: case MGDK_lng: {
				bool nil;
				const hge v = static_int(bound, tp2, &nil);
				if (!nil && v == tmax_of(tp2)) {
					special = true;
				} else if (!nil && v == 0) {
					special = peers = true;
				} else if (nil || v < 0) {
					seterr("%s", inv);
					return -1;
				} else if (is_mtime(tp1)) {
					kind = tp2 == MGDK_int ? (tp1 == MGDK_daytime ? -2 : K_MONTH) : K_MSEC;
				} else {
					kind = numint ? K_INT : -2;
					fast = numint;
				}
				slimit = v;
				break;
			}
			case MGDK_flt: case MGDK_dbl: {
				const double v = tp2 == MGDK_flt ? (double) *(const float *) bound : *(const double *) bound;
				if (v != v || v < 0) {
					seterr("%s", inv);
					return -1;
				}
				if (tp2 == MGDK_flt ? *(const float *) bound == 3.40282346638528859812e+38F
						    : v == 1.79769313486231570815e+308)
					special = true;
				else if (v == 0)
					special = peers = true;
				else
					kind = tp1 == tp2 ? (tp2 == MGDK_flt ? K_FLT : K_DBL) : -2;
				L.sf = v;
				break;
			}
			case MGDK_hge: {
				bool nil;
				const hge v = static_int(bound, tp2, &nil);
				if (nil || v < 0) {
					seterr("%s", inv);
					return -1;
				}
				if (v == tmax_of(MGDK_hge))
					special = true;
				else if (v == 0)
					special = peers = true;
				else
					kind = is_int(tp1) ? K_INT : -2;
				slimit = v;
				break;
			}
			default:
				kind = -1;
				break;
			}
			L.si = slimit;
		}
		if (!special && kind == -1) {
			seterr("42000!range frame bound type %s not supported.\n", atomname(tp2));
			return -1;
		}
		if (!special && kind == -2) {
			seterr("42000!type %s not supported for %s frame bound type.\n", atomname(tp1), atomname(tp2));
			return -1;
		}
		if (special && !peers) {
			HostList H;
			rc = make_list(H, pb, n, true) < 0 ? -1 : run_list_bounds(H, preceding, out);
		} else if (peers) {
			rc = peers_any(b, p, preceding, out);
			rc = rc < 0 ? -1 : (sync() ? 0 : -1);
		} else if (n == 0) {
			rc = 0;
		} else if (fast) {
			const BUN nn = n;
			const int bt = basetype(tp1);
			const hge tmax = tmax_of(bt);
			const int64_t lim = (int64_t) (slimit < tmax ? slimit : tmax);
			DevBuf wide(bt == MGDK_lng ? 8 : nn * 8 + 8);
			const int64_t *vals = (const int64_t *) b->theap;
			if (bt != MGDK_lng) {
				if (!wide.p)
					return -1;
				const dim3 g(grid_for(nn, 1024, 16384));
				if (bt == MGDK_bte)
					hipLaunchKernelGGL(k_rb_widen<int8_t>, g, dim3(256), 0, stream(),
							   (const int8_t *) b->theap, wide.as<int64_t>(), nn);
				else if (bt == MGDK_sht)
					hipLaunchKernelGGL(k_rb_widen<int16_t>, g, dim3(256), 0, stream(),
							   (const int16_t *) b->theap, wide.as<int64_t>(), nn);
				else
					hipLaunchKernelGGL(k_rb_widen<int32_t>, g, dim3(256), 0, stream(),
							   (const int32_t *) b->theap, wide.as<int64_t>(), nn);
				vals = wide.as<int64_t>();
			}
			rc = range_bounds_int64(r, vals, p, nn, lim, (uint64_t) tmax, false, preceding);
		} else {
			HostList H;
			rc = make_list(H, pb, n, true) < 0 ? -1 : range_generic(b, p, H, L, tp1, kind, preceding, out, inv);
		}
	} else {
		seterr("42000!unit type %d not supported (this is a bug).\n", unit);
		return -1;
	}
	if (rc < 0)
		return -1;
	r->count = n;
	if (n <= 1)
		r->tsorted = r->trevsorted = 1;      // BATsetcount
	// GDKanalyticalallbounds / GDKanalyticalpeers set tnonil = false
	// (:606-607, :851-852), the walks tnonil = (nils == 0) = true; the
	// caller-allocated r keeps its other properties (BATsetcount)
	r->tnonil = !special;
	r->tnil = 0;
	return 0;
}
