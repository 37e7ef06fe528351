// analytic.hip -- RANGE frame bounds of GDKanalyticalwindowbounds on the
// MI355X (gdk/gdk_analytic_bounds.c:1440 -> GDKanalyticalrangebounds :994,
// kernels ANALYTICAL_WINDOW_BOUNDS_RANGE_PRECEDING/FOLLOWING :273-369,
// unbounded GDKanalyticalallbounds :614, limit 0 GDKanalyticalpeers :710).
//
// The reference walks from every row backwards (PRECEDING) or forwards
// (FOLLOWING) while |b[k] - b[j]| <= limit, stopping at nils and at the
// partition start/end: O(n * window).  Inside a partition ordered by the
// window's ORDER BY (nils first ascending, last descending) that walk stops
// exactly where a monotone predicate flips, so the device finds the same
// row by galloping + binary search (O(log window)), and also re-derives the
// only subtraction that could have overflowed (the first violating pair) to
// raise the reference's "22003!overflow in calculation." where it would.
// A check kernel verifies that order; when it does not hold, a per-row
// linear-walk kernel runs instead, so results always match the reference.
// Partitions come from the boolean column p (row 0 always starts one).
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

__global__ __launch_bounds__(256) void
k_part_flags(const int8_t *p, BUN n, int8_t *f)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		f[i] = i == 0 || (p && p[i] != 0);
}

// bit 0: violates ascending-nils-first, bit 1: violates descending-nils-last
__global__ __launch_bounds__(256) void
k_order_check(const int64_t *b, const int8_t *f, BUN n, uint32_t *flags)
{
	uint32_t v = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (BUN) gridDim.x * blockDim.x) {
		if (f[i + 1])
			continue;   // next row starts a new partition
		const int64_t x = b[i], y = b[i + 1];
		const bool xn = x == INT64_MIN, yn = y == INT64_MIN;
		if (!xn && yn) v |= 1;
		else if (!xn && !yn && x > y) v |= 1;
		if (xn && !yn) v |= 2;
		else if (!xn && !yn && x < y) v |= 2;
	}
	for (int o = 32; o > 0; o >>= 1)
		v |= __shfl_xor(v, o);
	if (__lane_id() == 0 && v)
		atomicOr(flags, v);
}

struct WArgs {
	const int64_t *b;
	BUN n;
	const oid *S;       // sorted partition starts (NULL: dense, S[k] = Sseq + k)
	oid Sseq;
	BUN m;              // number of partitions
	int64_t limit;
	bool preceding;
	bool desc;          // partitions sorted descending (nils last)
	bool peers;         // limit == 0: no overflow check (GDKanalyticalpeers)
	bool all;           // unbounded
	oid *out;
	uint32_t *err;      // bit 0: overflow
};

__device__ __forceinline__ oid
pstart(const WArgs &a, BUN k)
{
	return a.S ? a.S[k] : a.Sseq + k;
}

// partition [m, e) containing row i
__device__ __forceinline__ void
partition_of(const WArgs &a, BUN i, BUN &m, BUN &e)
{
	BUN lo = 0, hi = a.m;   // find last k with S[k] <= i
	while (hi - lo > 1) {
		BUN mid = (lo + hi) / 2;
		if (pstart(a, mid) <= i) lo = mid; else hi = mid;
	}
	m = pstart(a, lo);
	e = lo + 1 < a.m ? pstart(a, lo + 1) : a.n;
}

__device__ __forceinline__ uint64_t
absdiff(int64_t x, int64_t y)
{
	return x >= y ? (uint64_t) x - (uint64_t) y : (uint64_t) y - (uint64_t) x;
}

// true difference x - y overflows lng (SUB_WITH_CHECK, incl. == INT64_MIN)
__device__ __forceinline__ bool
sub_ovf(int64_t x, int64_t y)
{
	return absdiff(x, y) > (uint64_t) INT64_MAX;
}

__global__ __launch_bounds__(256) void
k_range_sorted(WArgs a)
{
	uint32_t ovf = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < a.n; k += (BUN) gridDim.x * blockDim.x) {
		BUN m, e;
		partition_of(a, k, m, e);
		if (a.all) {
			a.out[k] = a.preceding ? m : e;
			continue;
		}
		// nil run: ascending -> [m, z0), descending -> [z0, e)
		BUN lo = m, hi = e;
		while (lo < hi) {   // first non-nil (asc) / first nil (desc)
			BUN mid = (lo + hi) / 2;
			bool isn = a.b[mid] == INT64_MIN;
			if (a.desc ? !isn : isn) lo = mid + 1; else hi = mid;
		}
		const BUN z0 = lo;
		const int64_t v = a.b[k];
		if (v == INT64_MIN) {
			if (a.desc)
				a.out[k] = a.preceding ? z0 : e;
			else
				a.out[k] = a.preceding ? m : z0;
			continue;
		}
		const BUN va = a.desc ? m : z0, vz = a.desc ? z0 : e;   // non-nil rows [va, vz)
		const uint64_t lim = (uint64_t) a.limit;
		if (a.preceding) {
			// smallest j in [va, k] with |v - b[j]| <= lim
			BUN good = k, bad = va;   // invariant: ok(good); bad < good or bad==va unknown
			bool found_bad = false;
			for (BUN step = 1;; step <<= 1) {
				if (k - va < step) break;
				BUN j = k - step;
				if (absdiff(v, a.b[j]) <= lim) {
					good = j;
				} else {
					bad = j;
					found_bad = true;
					break;
				}
			}
			if (!found_bad) {
				if (absdiff(v, a.b[va]) <= lim) {
					good = va;
				} else {
					bad = va;
					found_bad = true;
				}
			}
			if (found_bad) {
				while (good - bad > 1) {
					BUN mid = bad + (good - bad) / 2;
					if (absdiff(v, a.b[mid]) <= lim) good = mid; else bad = mid;
				}
				if (!a.peers && sub_ovf(v, a.b[bad]))
					ovf = 1;
			}
			a.out[k] = good;
		} else {
			// largest j in [k, vz) with ok; result j + 1
			BUN good = k, bad = vz;
			bool found_bad = false;
			for (BUN step = 1;; step <<= 1) {
				BUN j = k + step;
				if (j >= vz) break;
				if (absdiff(v, a.b[j]) <= lim) {
					good = j;
				} else {
					bad = j;
					found_bad = true;
					break;
				}
			}
			if (!found_bad) {
				bad = vz;
				// binary search in (good, vz): last ok
				BUN lo2 = good, hi2 = vz;
				while (hi2 - lo2 > 1) {
					BUN mid = lo2 + (hi2 - lo2) / 2;
					if (absdiff(v, a.b[mid]) <= lim) lo2 = mid; else hi2 = mid;
				}
				good = lo2;
				bad = hi2;
				found_bad = bad < vz;
			} else {
				while (bad - good > 1) {
					BUN mid = good + (bad - good) / 2;
					if (absdiff(v, a.b[mid]) <= lim) good = mid; else bad = mid;
				}
			}
			if (found_bad && !a.peers && sub_ovf(v, a.b[bad]))
				ovf = 1;
			a.out[k] = good + 1;
		}
	}
	if (ovf)
		atomicOr(a.err, 1u);
}

// exact restatement of the reference walk for partitions that are not
// ordered (or mixed); O(window) per row
__global__ __launch_bounds__(256) void
k_range_walk(WArgs a)
{
	uint32_t ovf = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < a.n; k += (BUN) gridDim.x * blockDim.x) {
		BUN m, e;
		partition_of(a, k, m, e);
		if (a.all) {
			a.out[k] = a.preceding ? m : e;
			continue;
		}
		const int64_t v = a.b[k];
		const bool vn = v == INT64_MIN;
		const uint64_t lim = (uint64_t) a.limit;
		BUN j;
		if (a.preceding) {
			for (j = k;; j--) {
				const bool jn = a.b[j] == INT64_MIN;
				if (vn ? !jn : jn) { j++; break; }
				if (!vn) {
					if (!a.peers && sub_ovf(v, a.b[j])) { ovf = 1; break; }
					if (absdiff(v, a.b[j]) > lim) { j++; break; }
				}
				if (j == m)
					break;
			}
		} else {
			for (j = k + 1; j < e; j++) {
				const bool jn = a.b[j] == INT64_MIN;
				if (vn ? !jn : jn)
					break;
				if (!vn) {
					if (!a.peers && sub_ovf(v, a.b[j])) { ovf = 1; break; }
					if (absdiff(v, a.b[j]) > lim)
						break;
				}
			}
		}
		a.out[k] = j;
	}
	if (ovf)
		atomicOr(a.err, 1u);
}

}  // namespace

extern "C" int
mgdk_GDKanalyticalwindowbounds(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_bat *l, const void *bound,
			       int tp1, int tp2, int unit, bool preceding, mgdk_oid first_half)
{
	(void) first_half;
	if (r == nullptr || b == nullptr) {
		seterr("GDKanalyticalwindowbounds: NULL argument");
		return -1;
	}
	if (unit != 1) {
		seterr("42000!window bounds: unit %d (rows/groups) not supported on the device path", unit);
		return -1;
	}
	if (l != nullptr || bound == nullptr) {
		seterr("42000!window bounds: per-row (dynamic) bounds not supported on the device path");
		return -1;
	}
	if (basetype(tp1) != MGDK_lng || basetype(b->ttype) != MGDK_lng) {
		seterr("42000!type %s not supported for %s frame bound type.\n", atomname(tp1), atomname(tp2));
		return -1;
	}
	if (tp2 != MGDK_lng) {
		seterr("42000!range frame bound type %s not supported.\n", atomname(tp2));
		return -1;
	}
	if (r->ttype != MGDK_oid) {
		seterr("window bounds: result must be an oid BAT");
		return -1;
	}
	const int64_t limit = *(const int64_t *) bound;
	const bool all = limit == INT64_MAX;
	if (!all && (limit == INT64_MIN || limit < 0)) {
		seterr("42000!range frame bound must be non negative and non null.\n");
		return -1;
	}
	ProfScope prof("windowbounds");
	const BUN n = b->count;
	if (p && (p->count != n || width_of(p->ttype) != 1)) {
		seterr("window bounds: partition column must be a bit BAT aligned with b");
		return -1;
	}
	// r is caller-allocated with room for count(b) oids (sql_rank.c:161
	// allocates it with COLnew(…, BATcount(b), …)); the caller sets nothing else
	mgdk_bat *rr = r;
	if (n > 0 && rr->theap == nullptr) {
		seterr("window bounds: result BAT has no heap");
		return -1;
	}
	hipStream_t st = stream();
	if (n == 0) {
		rr->count = 0;
		return 0;
	}
	DevBuf fl(n + 8), err(16);
	if (!fl.p || !err.p || !hip_ok(hipMemsetAsync(err.p, 0, 16, st), "memset"))
		return -1;
	hipLaunchKernelGGL(k_part_flags, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st,
			   p ? (const int8_t *) p->theap : nullptr, n, fl.as<int8_t>());
	mgdk_bat *S = compact_flags(fl.as<int8_t>(), n, 0);
	if (S == nullptr)
		return -1;
	WArgs a{};
	a.b = (const int64_t *) b->theap;
	a.n = n;
	a.S = S->ttype == MGDK_void ? nullptr : (const oid *) S->theap;
	a.Sseq = S->tseqbase;
	a.m = S->count;
	a.limit = limit;
	a.preceding = preceding;
	a.peers = limit == 0;
	a.all = all;
	a.out = (oid *) rr->theap;
	a.err = err.as<uint32_t>();
	hipLaunchKernelGGL(k_order_check, dim3(grid_for(n, 2048, 4096)), dim3(256), 0, st, a.b, fl.as<int8_t>(), n,
			   err.as<uint32_t>() + 1);
	uint32_t *h = (uint32_t *) pinned(16);
	if (!hip_ok(hipMemcpyAsync(h, err.p, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
		mgdk_BBPunfix(S);
		return -1;
	}
	const uint32_t order = h[1];
	dim3 g(grid_for(n, 256 * 4, 256 * 64)), blk(256);
	if (all || !(order & 1) || !(order & 2)) {
		a.desc = (order & 1) != 0;
		hipLaunchKernelGGL(k_range_sorted, g, blk, 0, st, a);
	} else {
		hipLaunchKernelGGL(k_range_walk, g, blk, 0, st, a);
	}
	if (!hip_ok(hipMemcpyAsync(h, err.p, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
		mgdk_BBPunfix(S);
		return -1;
	}
	mgdk_BBPunfix(S);
	if (h[0] & 1) {
		seterr("22003!overflow in calculation.\n");
		return -1;
	}
	rr->count = n;
	rr->tnonil = 1;
	rr->tnil = 0;
	rr->tsorted = rr->trevsorted = rr->tkey = n <= 1;
	return 0;
}
