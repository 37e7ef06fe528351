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
// row by galloping + binary search, and re-derives the only subtraction that
// could have overflowed (the first violating pair) to raise the reference's
// "22003!overflow in calculation." where it would.  A check kernel verifies
// that order; when it does not hold, a per-row linear-walk kernel restates
// the reference loop, so results always match.
//
// Ordered path (k_range_tile): a workgroup owns 2048 rows; it stages them
// plus a 2048-row halo (before for PRECEDING, after for FOLLOWING) in LDS
// with coalesced loads, and the (<= 128) partitions that overlap the staged
// rows with their nil-run boundaries; every row then searches in LDS (global
// memory only when a frame reaches past the halo) and its bound is stored
// coalesced.  Partitions: the bit column p (row 0 always starts one).
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

// bit 0: violates ascending-nils-first, bit 1: violates descending-nils-last
__global__ __launch_bounds__(256) void
k_order_check(const int64_t *b, const int8_t *p, BUN n, uint32_t *flags)
{
	uint32_t v = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (BUN) gridDim.x * blockDim.x) {
		if (p && p[i + 1] != 0)
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
	const oid *S;       // sorted rows with p == 1 (NULL: dense, S[k] = Sseq + k)
	oid Sseq;
	BUN ns;             // |S|
	bool lead;          // row 0 starts a partition but is not in S
	BUN m;              // number of partitions = ns + lead
	int64_t limit;
	bool preceding;
	bool desc;          // partitions sorted descending (nils last)
	bool peers;         // limit == 0: no overflow check (GDKanalyticalpeers)
	bool all;           // unbounded
	const oid *Z;       // per partition nil-run boundary (ordered path)
	oid *out;
	uint32_t *err;      // bit 0: overflow
};

__device__ __forceinline__ oid
pstart(const WArgs &a, BUN k)
{
	if (a.lead) {
		if (k == 0)
			return 0;
		k--;
	}
	return a.S ? a.S[k] : a.Sseq + k;
}

__device__ __forceinline__ BUN
pend(const WArgs &a, BUN k)
{
	return k + 1 < a.m ? pstart(a, k + 1) : a.n;
}

// index of the partition containing row i
__device__ __forceinline__ BUN
partition_of(const WArgs &a, BUN i)
{
	BUN lo = 0, hi = a.m;
	while (hi - lo > 1) {
		BUN mid = (lo + hi) / 2;
		if (pstart(a, mid) <= i) lo = mid; else hi = mid;
	}
	return lo;
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

// nil-run boundary of every partition: ascending -> first non-nil row,
// descending -> first nil row
__global__ __launch_bounds__(256) void
k_part_nilbound(WArgs a, oid *Z)
{
	for (BUN pi = (BUN) blockIdx.x * blockDim.x + threadIdx.x; pi < a.m; pi += (BUN) gridDim.x * blockDim.x) {
		BUN lo = pstart(a, pi), hi = pend(a, pi);
		while (lo < hi) {
			BUN mid = (lo + hi) / 2;
			bool isn = a.b[mid] == INT64_MIN;
			if (a.desc ? !isn : isn) lo = mid + 1; else hi = mid;
		}
		Z[pi] = lo;
	}
}

constexpr int TR = 8;            // rows per lane
constexpr int TT = 256 * TR;     // rows per tile
constexpr int TH = 2048;         // halo rows
constexpr int PMAX = 128;        // partitions staged per tile

struct Stage {
	const int64_t *sv;
	BUN lo, hi;                  // staged rows [lo, hi)
	const int64_t *b;
	__device__ __forceinline__ int64_t operator()(BUN j) const {
		return (j >= lo && j < hi) ? sv[j - lo] : b[j];
	}
};

// bound of one row in an ordered partition [m, e) with nil boundary z0
__device__ __forceinline__ oid
sorted_bound(const WArgs &a, const Stage &V, BUN k, BUN m, BUN e, BUN z0, uint32_t &ovf)
{
	if (a.all)
		return a.preceding ? m : e;
	const int64_t v = V(k);
	if (v == INT64_MIN) {
		if (a.desc)
			return a.preceding ? z0 : e;
		return a.preceding ? m : z0;
	}
	const BUN va = a.desc ? m : z0, vz = a.desc ? z0 : e;   // non-nil rows
	const uint64_t lim = (uint64_t) a.limit;
	if (a.preceding) {
		// smallest j in [va, k] with |v - b[j]| <= lim
		BUN good = k, bad = va;
		bool fb = false;
		for (BUN step = 1; k - va >= step; step <<= 1) {
			BUN q = k - step;
			if (absdiff(v, V(q)) <= lim) good = q;
			else { bad = q; fb = true; break; }
		}
		if (!fb) {
			if (absdiff(v, V(va)) <= lim) good = va;
			else { bad = va; fb = true; }
		}
		if (fb) {
			while (good - bad > 1) {
				BUN mid = bad + (good - bad) / 2;
				if (absdiff(v, V(mid)) <= lim) good = mid; else bad = mid;
			}
			if (!a.peers && sub_ovf(v, V(bad)))
				ovf = 1;
		}
		return good;
	}
	// largest j in [k, vz) with ok; bound = j + 1
	BUN good = k, bad = vz;
	for (BUN step = 1; k + step < vz; step <<= 1) {
		BUN q = k + step;
		if (absdiff(v, V(q)) <= lim) good = q;
		else { bad = q; break; }
	}
	while (bad - good > 1) {
		BUN mid = good + (bad - good) / 2;
		if (absdiff(v, V(mid)) <= lim) good = mid; else bad = mid;
	}
	if (bad < vz && !a.peers && sub_ovf(v, V(bad)))
		ovf = 1;
	return good + 1;
}

__global__ __launch_bounds__(256) void
k_range_tile(WArgs a)
{
	__shared__ int64_t sv[TT + TH];
	__shared__ oid spst[PMAX + 1];
	__shared__ oid spz[PMAX];
	__shared__ int s_np;
	__shared__ BUN s_plo;
	const BUN t0 = (BUN) blockIdx.x * TT;
	const BUN t1 = t0 + TT < a.n ? t0 + TT : a.n;
	const BUN lo = a.preceding ? (t0 > TH ? t0 - TH : 0) : t0;
	const BUN hi = a.preceding ? t1 : (t1 + TH < a.n ? t1 + TH : a.n);
	for (BUN j = lo + threadIdx.x; j < hi; j += 256)
		sv[j - lo] = a.b[j];
	if (threadIdx.x == 0) {
		BUN plo = partition_of(a, lo), phi = partition_of(a, hi - 1);
		BUN np = phi - plo + 1;
		s_np = np <= PMAX ? (int) np : -1;
		s_plo = plo;
	}
	__syncthreads();
	const int np = s_np;
	const BUN plo = s_plo;
	if (np > 0) {
		for (int i = threadIdx.x; i <= np; i += 256) {
			spst[i] = plo + i < a.m ? pstart(a, plo + i) : a.n;
			if (i < np)
				spz[i] = a.Z[plo + i];
		}
	}
	__syncthreads();
	Stage V{sv, lo, hi, a.b};
	uint32_t ovf = 0;
#pragma unroll
	for (int r = 0; r < TR; r++) {
		const BUN k = t0 + r * 256 + threadIdx.x;
		if (k >= t1)
			break;
		BUN m, e, z0;
		if (np > 0) {
			int l = 0, h = np;   // last i with spst[i] <= k
			while (h - l > 1) {
				int mid = (l + h) / 2;
				if (spst[mid] <= k) l = mid; else h = mid;
			}
			m = spst[l];
			e = spst[l + 1];
			z0 = spz[l];
		} else {
			BUN pi = partition_of(a, k);
			m = pstart(a, pi);
			e = pend(a, pi);
			z0 = a.Z[pi];
		}
		a.out[k] = sorted_bound(a, V, k, m, e, z0, ovf);
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
		const BUN pi = partition_of(a, k);
		const BUN m = pstart(a, pi), e = pend(a, pi);
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

__global__ void
k_first_oid(const oid *S, oid *out)
{
	*out = S[0];
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
	// allocates it with COLnew(..., BATcount(b), ...))
	if (n > 0 && r->theap == nullptr) {
		seterr("window bounds: result BAT has no heap");
		return -1;
	}
	hipStream_t st = stream();
	if (n == 0) {
		r->count = 0;
		return 0;
	}
	// partition starts: the rows with p == 1 (ordered compaction), plus row 0
	mgdk_bat *S = nullptr;
	if (p) {
		S = compact_flags((const int8_t *) p->theap, n, 0, true);
		if (S == nullptr)
			return -1;
	}
	DevBuf err(16);
	if (!err.p || !hip_ok(hipMemsetAsync(err.p, 0, 16, st), "memset")) {
		mgdk_BBPunfix(S);
		return -1;
	}
	WArgs a{};
	a.b = (const int64_t *) b->theap;
	a.n = n;
	if (S) {
		a.S = S->ttype == MGDK_void ? nullptr : (const oid *) S->theap;
		a.Sseq = S->tseqbase;
		a.ns = S->count;
	} else {
		a.S = nullptr;
		a.Sseq = 0;
		a.ns = 0;
	}
	// does row 0 start a partition that S does not list?
	bool first0 = false;
	if (a.ns > 0) {
		if (a.S == nullptr) {
			first0 = a.Sseq == 0;
		} else {
			oid *d = (oid *) meta_buf();
			hipLaunchKernelGGL(k_first_oid, dim3(1), dim3(1), 0, st, a.S, d);
			oid *h = (oid *) pinned(8);
			if (!hip_ok(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
				mgdk_BBPunfix(S);
				return -1;
			}
			first0 = *h == 0;
		}
	}
	a.lead = !first0;
	a.m = a.ns + (a.lead ? 1 : 0);
	a.limit = limit;
	a.preceding = preceding;
	a.peers = limit == 0;
	a.all = all;
	a.out = (oid *) r->theap;
	a.err = err.as<uint32_t>();
	hipLaunchKernelGGL(k_order_check, dim3(grid_for(n, 2048, 4096)), dim3(256), 0, st, a.b,
			   p ? (const int8_t *) p->theap : nullptr, n, err.as<uint32_t>() + 1);
	uint32_t *h = (uint32_t *) pinned(16);
	if (!hip_ok(hipMemcpyAsync(h, err.p, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
		mgdk_BBPunfix(S);
		return -1;
	}
	const uint32_t order = h[1];
	DevBuf Z((a.m + 1) * 8);
	if (!Z.p) {
		mgdk_BBPunfix(S);
		return -1;
	}
	const dim3 blk(256);
	if (all || !(order & 1) || !(order & 2)) {
		a.desc = (order & 1) != 0;
		a.Z = Z.as<oid>();
		hipLaunchKernelGGL(k_part_nilbound, dim3(grid_for(a.m, 256, 8192)), blk, 0, st, a, Z.as<oid>());
		hipLaunchKernelGGL(k_range_tile, dim3((unsigned) ((n + TT - 1) / TT)), blk, 0, st, a);
	} else {
		hipLaunchKernelGGL(k_range_walk, dim3(grid_for(n, 256 * 4, 256 * 64)), blk, 0, st, a);
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
	r->count = n;
	r->tnonil = 1;
	r->tnil = 0;
	r->tsorted = r->trevsorted = r->tkey = n <= 1;
	return 0;
}
