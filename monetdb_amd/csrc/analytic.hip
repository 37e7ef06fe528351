// analytic.hip -- RANGE frame bounds of GDKanalyticalwindowbounds on the
// MI355X (gdk/gdk_analytic_bounds.c:1440 -> GDKanalyticalrangebounds :994,
// kernels ANALYTICAL_WINDOW_BOUNDS_RANGE_PRECEDING/FOLLOWING :273-369,
// unbounded GDKanalyticalallbounds :614, limit 0 GDKanalyticalpeers :710).
//
// The reference walks from every row backwards (PRECEDING) or forwards
// (FOLLOWING) while |b[k] - b[j]| <= limit, stopping at nils and at the
// partition start/end: O(n * window).  Inside a partition ordered by the
// window's ORDER BY (nils first ascending, last descending) that walk stops
// exactly where a monotone predicate flips, and the row it stops at is
// non-decreasing in k; the device therefore advances one pointer per lane
// over consecutive rows (k_range_fast), and re-derives the only subtraction
// that could have overflowed (the first violating pair) to raise the
// reference's "22003!overflow in calculation." where it would.  The same
// pass verifies the order; when neither ascending nor descending order holds
// a per-row linear-walk kernel restates the reference loop, so results always
// match.  Rows whose frame leaves the fast kernel's staged window are fixed
// up by a global gallop + binary search (k_range_fix / k_range_tile) over the
// partition starts S (compaction of p) and nil boundaries Z.
#include <cstdlib>
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

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
	uint64_t tmax;      // max of the value type: |v - b[j]| > tmax overflows (SUB_WITH_CHECK)
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
			if (!a.peers && absdiff(v, V(bad)) > a.tmax)
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
	if (bad < vz && !a.peers && absdiff(v, V(bad)) > a.tmax)
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

// ---------------------------------------------------------------------------
// Fast ordered path (k_range_fast).  Inside an ordered partition the bound of
// row k is monotone non-decreasing in k (also across nil runs and partition
// starts), so the bounds of a tile are a MERGE of the tile's rows with the
// staged rows: staged row j precedes row k in the merge iff j lies before
// k's bound.  Each lane walks a fixed number of merge steps from its own
// diagonal (found by a binary search), so no lane waits on another's data
// dependent loop: ~2 steps per row.  A workgroup owns FT rows and stages
// them plus an FH-row halo (before for PRECEDING, after for FOLLOWING) and
// the partition bits; partition membership inside the stage comes from a
// block max-scan of partition starts, skipped when the stage holds none.
// The same pass checks the order (both directions) so no separate check
// kernel runs; rows whose frame reaches past the halo are listed for a
// fix-up pass with the general machinery (S, Z, global search).  Reads b
// once (+ halo), p once, writes the bound once (coalesced).
// ---------------------------------------------------------------------------

#ifndef MGDK_WIN_FR
#define MGDK_WIN_FR 8
#endif
#ifndef MGDK_WIN_FH
#define MGDK_WIN_FH 256
#endif
#ifndef MGDK_WIN_NT
#define MGDK_WIN_NT 1
#endif
#ifndef MGDK_WIN_XCD
#define MGDK_WIN_XCD 1
#endif
constexpr int FR = MGDK_WIN_FR;          // rows per lane
constexpr int FT = 256 * FR;             // rows per tile
constexpr int FH = MGDK_WIN_FH;          // halo rows
constexpr int FS = FT + FH + 1;          // staged rows at most

__device__ __forceinline__ int
pidx(int i)
{
	return i;
}

struct FArgs {
	const int64_t *b;
	uint64_t tmax;       // |v - b[j]| > tmax overflows (narrow value types widened to lng)
	const int8_t *p;     // partition bits (4-byte aligned); a readable dummy without partitions
	BUN pstep;           // 1, or 0 without partitions
	uint32_t pmask;      // ~0, or 0 without partitions
	BUN n;
	int64_t limit;
	bool preceding;
	bool desc;
	bool peers;
	bool all;
	oid *out;
	uint32_t *flags;     // [0] overflow, [1] order violations (bit0 asc, bit1 desc), [2] unresolved rows,
	                     // [3] a tile needs the wide kernel
	oid *unres;          // unresolved row list
	uint32_t unres_cap;
	const uint32_t *tiles;   // k_range_keys<uint64_t>: the tiles to run (NULL: every tile)
	uint32_t *relist;        // k_range_keys<uint32_t>: tiles it leaves to the 64-bit kernel (count in flags[4])
};

// Partition-start flags of stage rows 4q .. 4q+3 as one little-endian word
// (rows at or past the stage end read as 0).  The host hands over a 4-byte
// aligned flag column (copying a misaligned view) and, without partitions,
// a zero step and mask, so the word load is unconditional on a clamped
// index -- heaps are allocated in >= 256-byte classes, so the aligned word
// holding the last valid byte is always readable -- and the stage's loads
// all stay in flight together instead of each waiting at a branch join.
static_assert(FH % 4 == 0 && FT % 4 == 0, "stage starts must stay word aligned");

__device__ __forceinline__ uint32_t
flags_word(const FArgs &a, BUN lo, int q, int S)
{
	const bool in = 4 * q < S;
	const BUN pos = lo + 4 * (BUN) (in ? q : 0);
	const uint32_t x = *(const uint32_t *) (a.p + pos * a.pstep);
	const BUN rem = a.n - pos;
	const uint32_t m = rem >= 4 ? ~0u : (1u << (8 * rem)) - 1;
	return in ? x & m & a.pmask : 0;
}

__global__ __launch_bounds__(256) void
k_range_fast(FArgs a)
{
	__shared__ int64_t sv[FS];
	__shared__ int16_t spst[FS];         // last partition start (stage index) <= i, -1: before the stage
	__shared__ __attribute__((aligned(16))) uint8_t sp[FS + 4];   // partition start flags of the stage
	__shared__ uint16_t sbd[FT];         // bound of every tile row (stage index)
	__shared__ int32_t s_wmax[4];
	__shared__ int s_hasb;
	__shared__ uint32_t s_ord;
	const int tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const BUN t0 = (BUN) blockIdx.x * FT;
	const BUN t1 = t0 + FT < a.n ? t0 + FT : a.n;
	const BUN lo = a.preceding ? (t0 > FH ? t0 - FH : 0) : t0;
	const BUN hi = a.preceding ? (t1 + 1 < a.n ? t1 + 1 : a.n) : (t1 + FH < a.n ? t1 + FH : a.n);
	const int S = (int) (hi - lo);
	if (tid == 0) {
		s_hasb = 0;
		s_ord = 0;
	}
	{
		// all loads of the stage in flight at once
		constexpr int NB = (FS + 255) / 256;
		int64_t tv[NB];
#pragma unroll
		for (int u = 0; u < NB; u++) {
			const int i = tid + u * 256;
			const int64_t x = a.b[lo + (i < S ? i : 0)];   // clamped: every load in flight
			tv[u] = i < S ? x : 0;
		}
		constexpr int NW = (FS + 3 + 1023) / 1024;
		uint32_t tw[NW];
#pragma unroll
		for (int u = 0; u < NW; u++) {
			const int q = tid + u * 256;      // word q covers stage rows 4q .. 4q+3
			tw[u] = flags_word(a, lo, q, S);
		}
#pragma unroll
		for (int u = 0; u < NB; u++) {
			const int i = tid + u * 256;
			if (i < S)
				sv[pidx(i)] = tv[u];
		}
		bool any = lo == 0;
#pragma unroll
		for (int u = 0; u < NW; u++) {
			const int q = tid + u * 256;
			if (4 * q < S) {
				*(uint32_t *) &sp[4 * q] = tw[u];
				any |= tw[u] != 0;
			}
		}
		if (lo == 0 && tid == 0)
			sp[0] = 1;                    // row 0 always starts a partition
		__syncthreads();
		if (__any(any) && lane == 0)
			s_hasb = 1;
		__syncthreads();
	}
	const bool hasb = s_hasb != 0;
	if (hasb) {
		// block max-scan of partition starts over per-thread chunks
		const int C = (S + 255) / 256;
		const int c0 = tid * C, c1 = c0 + C < S ? c0 + C : S;
		int32_t m = -1;
		for (int i = c0; i < c1; i++)
			if (sp[i])
				m = i;
		int32_t incl = m;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			int32_t u = __shfl_up(incl, o);
			if (lane >= o)
				incl = u > incl ? u : incl;
		}
		if (lane == 63)
			s_wmax[w] = incl;
		__syncthreads();
		int32_t ex = __shfl_up(incl, 1);
		if (lane == 0)
			ex = -1;
		for (int q = 0; q < w; q++)
			ex = s_wmax[q] > ex ? s_wmax[q] : ex;
		m = ex;
		for (int i = c0; i < c1; i++) {
			if (sp[i])
				m = i;
			spst[i] = (int16_t) m;
		}
		__syncthreads();
	}

	const uint64_t lim = (uint64_t) a.limit;
	const bool all = a.all, prec = a.preceding;
	const int NA = (int) (t1 - t0), NB = S, xa = (int) (t0 - lo);
	// ok: staged row j belongs to the frame of the row at stage index xk
	auto ok = [&](int xk, int64_t vk, int j, int64_t vj) -> bool {
		if (hasb && spst[xk] != spst[j])
			return false;
		if (all)
			return true;
		const bool vkn = vk == INT64_MIN, vjn = vj == INT64_MIN;
		return vkn ? vjn : (!vjn && absdiff(vk, vj) <= lim);
	};
	// P(k, j): staged row j lies before the bound of tile row k.  Monotone:
	// true then false in j, and the bound (#j with P) is non-decreasing in k
	// inside ordered partitions -- a merge of the rows with the stage.
	auto P = [&](int k, int j) -> bool {
		if (j >= NB)
			return false;
		const int xk = xa + k;
		if (prec) {
			if (j >= xk)
				return false;
			return !ok(xk, sv[pidx(xk)], j, sv[pidx(j)]);
		}
		if (j <= xk)
			return true;
		return ok(xk, sv[pidx(xk)], j, sv[pidx(j)]);
	};
	{
		// merge path: every lane walks L steps of the (rows x stage) merge
		// from its diagonal; each step emits one bound or passes one row
		const int T = NA + NB;
		const int L = (T + 255) / 256;
		const int d0 = tid * L < T ? tid * L : T;
		int klo = d0 - NB > 0 ? d0 - NB : 0, khi = d0 < NA ? d0 : NA;
		while (klo < khi) {
			const int mid = (klo + khi + 1) >> 1;
			if (!P(mid - 1, d0 - mid))
				klo = mid;
			else
				khi = mid - 1;
		}
		int k = klo, j = d0 - klo;
		for (int st = 0; st < L && k + j < T; st++) {
			const bool pb = k >= NA || P(k, j);
			if (!pb)
				sbd[k] = (uint16_t) j;
			k += pb ? 0 : 1;
			j += pb ? 1 : 0;
		}
	}
	__syncthreads();
	// per row: unresolved frames, the overflow pair, the order of (k, k+1),
	// coalesced result stores
	uint32_t ovf = 0, ord = 0;
	for (int i = tid; i < NA; i += 256) {
		const int xk = xa + i;
		const BUN k = t0 + (BUN) i;
		const int bnd = sbd[i];
		const int64_t vk = sv[pidx(xk)];
		const bool vkn = vk == INT64_MIN;
		if (k + 1 < a.n && !(hasb && spst[xk + 1] == xk + 1)) {
			const int64_t y = sv[pidx(xk + 1)];
			const bool yn = y == INT64_MIN;
			if ((!vkn && yn) || (!vkn && !yn && vk > y))
				ord |= 1;
			if ((vkn && !yn) || (!vkn && !yn && vk < y))
				ord |= 2;
		}
		const bool unres = prec ? (bnd == 0 && lo > 0) : (bnd == NB && hi < a.n);
		if (unres) {
			const uint32_t at = atomicAdd(&a.flags[2], 1u);
			if (at < a.unres_cap)
				a.unres[at] = k;
		} else if (!all && !a.peers && !vkn) {
			// the pair the reference subtracts last (first row outside the frame)
			const int e = prec ? bnd - 1 : bnd;
			if (e >= 0 && e < NB && !(hasb && spst[e] != spst[xk])) {
				const int64_t vb = sv[pidx(e)];
				if (vb != INT64_MIN && absdiff(vk, vb) > a.tmax)
					ovf = 1;
			}
		}
		a.out[k] = lo + (BUN) bnd;
	}
	if (ovf)
		atomicOr(&a.flags[0], 1u);
	if (!all) {
		// one flag update per workgroup, and only for bits not yet published:
		// every tile of ascending data violates "descending", and a same-word
		// atomic per wave would serialise the whole grid
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			ord |= __shfl_xor(ord, o);
		if (lane == 0 && ord)
			atomicOr(&s_ord, ord);
		__syncthreads();
		if (tid == 0 && s_ord) {
			const uint32_t seen = __hip_atomic_load(&a.flags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			if (s_ord & ~seen)
				atomicOr(&a.flags[1], s_ord);
		}
	}
}

// ---------------------------------------------------------------------------
// Narrow-key variant (k_range_keys), the common case.  When the non-nil
// values staged by a tile span less than 2^32, every staged row becomes one
// 64-bit key that is non-decreasing along ordered data:
//     key = partition label (stage-relative) << 33 | flag << 32 | rel
// with flag = "not nil" for ascending partitions (nils first) and "nil" for
// descending ones (nils last), rel = v - min (ascending) or max - v
// (descending), 0 for nils.  The frame edge of row k is then a key threshold
// (partition start / nil run / rel -+ limit, clamped), so one merge step is a
// single 64-bit compare, and no subtraction inside such a tile can overflow
// (|v_k - v_j| < 2^32), so no overflow check is needed.  A tile whose values
// span more sets flags[3]; the host then runs the wide kernel above.
// ---------------------------------------------------------------------------

constexpr uint64_t KMAXREL = 0xffffffffull;

// KT = uint32_t: the common tile -- no partition start in its stage and
// values spanning < 2^31 -- with 32-bit keys flag << 31 | rel, half the key
// LDS (13.8 KiB a workgroup: 8 workgroups per CU instead of 6 with 64-bit
// keys).  Any other tile is listed in a.relist (count flags[4]) and rerun
// by the 64-bit kernel over that list (a.tiles).
template <bool PREC, bool DESC, bool ALL, typename KT = uint64_t>
__global__ __launch_bounds__(256) void
k_range_keys(FArgs a)
{
	constexpr bool K32 = sizeof(KT) == 4;
	constexpr int FB = K32 ? 31 : 32;                    // nil-flag bit
	constexpr KT RMASK = (KT) ((((uint64_t) 1) << FB) - 1);
	__shared__ KT sk[FS];
	__shared__ __attribute__((aligned(16))) uint8_t spu[(FS + 4 > 2 * FT ? FS + 4 : 2 * FT)];  // partition flags, then bounds
	__shared__ int64_t s_min[4], s_max[4];
	__shared__ int s_hasb;
	__shared__ uint32_t s_ord;
	uint8_t *sp = spu;
	uint16_t *sbd = (uint16_t *) spu;
	const int tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const uint32_t tile = (!K32 && a.tiles) ? a.tiles[blockIdx.x] : blockIdx.x;
	const BUN t0 = (BUN) tile * FT;
	const BUN t1 = t0 + FT < a.n ? t0 + FT : a.n;
	const BUN lo = PREC ? (t0 > FH ? t0 - FH : 0) : t0;
	const BUN hi = PREC ? (t1 + 1 < a.n ? t1 + 1 : a.n) : (t1 + FH < a.n ? t1 + FH : a.n);
	const int S = (int) (hi - lo);
	if (tid == 0) {
		s_hasb = 0;
		s_ord = 0;
	}
	constexpr int NB = (FS + 255) / 256;
	int64_t tv[NB];
	int64_t vmin = INT64_MAX, vmax = INT64_MIN;
	{
#pragma unroll
		for (int u = 0; u < NB; u++) {
			const int i = tid + u * 256;
			const int64_t x = a.b[lo + (i < S ? i : 0)];
			tv[u] = i < S ? x : INT64_MIN;
		}
		constexpr int NW = (FS + 3 + 1023) / 1024;
		uint32_t tw[NW];
#pragma unroll
		for (int u = 0; u < NW; u++) {
			const int q = tid + u * 256;
			tw[u] = flags_word(a, lo, q, S);
		}
		bool any = lo == 0;
#pragma unroll
		for (int u = 0; u < NW; u++) {
			const int q = tid + u * 256;
			if (4 * q < S) {
				*(uint32_t *) &sp[4 * q] = tw[u];
				any |= tw[u] != 0;
			}
		}
		if (lo == 0 && tid == 0)
			sp[0] = 1;
		if (!ALL) {
#pragma unroll
			for (int u = 0; u < NB; u++) {
				if (tv[u] != INT64_MIN) {
					vmin = tv[u] < vmin ? tv[u] : vmin;
					vmax = tv[u] > vmax ? tv[u] : vmax;
				}
			}
#pragma unroll
			for (int o = 32; o > 0; o >>= 1) {
				const int64_t x = __shfl_xor(vmin, o), y = __shfl_xor(vmax, o);
				vmin = x < vmin ? x : vmin;
				vmax = y > vmax ? y : vmax;
			}
			if (lane == 0) {
				s_min[w] = vmin;
				s_max[w] = vmax;
			}
		}
		__syncthreads();
		if (__any(any) && lane == 0)
			s_hasb = 1;
		__syncthreads();
	}
	const bool hasb = s_hasb != 0;
	uint64_t base = 0;
	if (!ALL) {
		vmin = s_min[0];
		vmax = s_max[0];
		for (int q = 1; q < 4; q++) {
			vmin = s_min[q] < vmin ? s_min[q] : vmin;
			vmax = s_max[q] > vmax ? s_max[q] : vmax;
		}
		if (vmin <= vmax && (uint64_t) vmax - (uint64_t) vmin > (uint64_t) RMASK) {
			if (tid == 0) {
				if (K32)
					a.relist[atomicAdd(&a.flags[4], 1u)] = tile;   // the 64-bit kernel takes it
				else
					atomicOr(&a.flags[3], 1u);          // wide tile: the host reruns k_range_fast
			}
			return;
		}
		base = DESC ? (uint64_t) vmax : (uint64_t) vmin;
	}
	if (K32 && hasb) {
		if (tid == 0)
			a.relist[atomicAdd(&a.flags[4], 1u)] = tile;       // partition labels need 64-bit keys
		return;
	}
	auto mkkey = [&](uint64_t label, int64_t v) -> KT {
		if (ALL)
			return (KT) (label << 33);
		const bool isnil = v == INT64_MIN;
		const uint64_t flag = DESC ? (isnil ? 1 : 0) : (isnil ? 0 : 1);
		const uint64_t rel = isnil ? 0 : (DESC ? base - (uint64_t) v : (uint64_t) v - base);
		return (KT) ((label << 33) | (flag << FB) | rel);
	};
	if (!hasb) {
#pragma unroll
		for (int u = 0; u < NB; u++) {
			const int i = tid + u * 256;
			if (i < S)
				sk[i] = mkkey(0, tv[u]);
		}
		__syncthreads();
	} else {
#pragma unroll
		for (int u = 0; u < NB; u++) {
			const int i = tid + u * 256;
			if (i < S)
				sk[i] = (KT) tv[u];             // (64-bit keys only: 32-bit tiles left above)
		}
		__syncthreads();
		// partition labels: block max-scan of partition starts (per-thread chunks)
		const int C = (S + 255) / 256;
		const int c0 = tid * C, c1 = c0 + C < S ? c0 + C : S;
		int32_t m = -1;
		for (int i = c0; i < c1; i++)
			if (sp[i])
				m = i;
		int32_t incl = m;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			int32_t u = __shfl_up(incl, o);
			if (lane >= o)
				incl = u > incl ? u : incl;
		}
		__shared__ int32_t s_wmax[4];
		if (lane == 63)
			s_wmax[w] = incl;
		__syncthreads();
		int32_t ex = __shfl_up(incl, 1);
		if (lane == 0)
			ex = -1;
		for (int q = 0; q < w; q++)
			ex = s_wmax[q] > ex ? s_wmax[q] : ex;
		m = ex;
		for (int i = c0; i < c1; i++) {
			if (sp[i])
				m = i;
			sk[i] = mkkey((uint64_t) (m + 1), (int64_t) sk[i]);
		}
		__syncthreads();
	}

	constexpr uint64_t RM = (uint64_t) RMASK;
	const uint64_t lim32 = ALL ? 0 : ((uint64_t) a.limit < RM ? (uint64_t) a.limit : RM);
	// frame threshold of the row with key kk
	auto thr = [&](uint64_t kk) -> uint64_t {
		const uint64_t lab = K32 ? 0 : kk >> 33 << 33;
		if (ALL)
			return PREC ? lab : lab | (K32 ? 0xffffffffull : ((1ull << 33) - 1));
		const uint64_t flag = (kk >> FB) & 1, rel = kk & RM;
		const bool valrow = DESC ? flag == 0 : flag == 1;
		const uint64_t hd = lab | (flag << FB);
		if (PREC)
			return valrow ? hd | (rel > lim32 ? rel - lim32 : 0) : hd;
		return valrow ? hd | (RM - rel > lim32 ? rel + lim32 : RM) : hd | RM;
	};
	const int NA = (int) (t1 - t0), NB2 = S, xa = (int) (t0 - lo);
	// P(k, j): staged row j lies before the bound of tile row k
	auto P = [&](int k, int j) -> bool {
		if (j >= NB2)
			return false;
		const uint64_t t = thr(sk[xa + k]), kj = sk[j];
		return PREC ? kj < t : kj <= t;
	};
	{
		const int T = NA + NB2;
		const int L = (T + 255) / 256;
		const int d0 = tid * L < T ? tid * L : T;
		int klo = d0 - NB2 > 0 ? d0 - NB2 : 0, khi = d0 < NA ? d0 : NA;
		while (klo < khi) {
			const int mid = (klo + khi + 1) >> 1;
			if (!P(mid - 1, d0 - mid))
				klo = mid;
			else
				khi = mid - 1;
		}
		int k = klo, j = d0 - klo;
		uint64_t t = k < NA ? thr(sk[xa + k]) : 0;
		for (int st = 0; st < L && k + j < T; st++) {
			bool pb = true;
			if (k < NA && j < NB2) {
				const uint64_t kj = sk[j];
				pb = PREC ? kj < t : kj <= t;
			} else if (k < NA) {
				pb = false;
			}
			if (!pb) {
				sbd[k] = (uint16_t) j;
				k++;
				if (k < NA)
					t = thr(sk[xa + k]);
			} else {
				j++;
			}
		}
	}
	__syncthreads();
	uint32_t ord = 0, ovf = 0;
	for (int i = tid; i < NA; i += 256) {
		const int xk = xa + i;
		const BUN k = t0 + (BUN) i;
		const int bnd = sbd[i];
		if (!ALL && k + 1 < a.n) {
			const uint64_t x = sk[xk], y = sk[xk + 1];
			if ((x >> 33) == (y >> 33)) {        // same partition
				if (y < x)
					ord |= DESC ? 2u : 1u;
				if (!DESC) {
					const uint64_t fx = (x >> FB) & 1, fy = (y >> FB) & 1;
					if ((fx == 0 && fy == 1) || (fx == 1 && fy == 1 && (y & RM) > (x & RM)))
						ord |= 2u;
				}
			}
		}
		const bool unres = PREC ? (bnd == 0 && lo > 0) : (bnd == NB2 && hi < a.n);
		if (unres) {
			const uint32_t at = atomicAdd(&a.flags[2], 1u);
			if (at < a.unres_cap)
				a.unres[at] = k;
		} else if (!ALL && !a.peers && a.tmax < KMAXREL) {
			// narrow value types: the pair the reference subtracts last (the
			// first row outside the frame) may exceed the type's range even
			// though the tile spans < 2^32
			const int e = PREC ? bnd - 1 : bnd;
			const uint64_t x = sk[xk];
			const bool xval = DESC ? ((x >> FB) & 1) == 0 : ((x >> FB) & 1) == 1;
			if (xval && e >= 0 && e < NB2) {
				const uint64_t y = sk[e];
				const bool yval = DESC ? ((y >> FB) & 1) == 0 : ((y >> FB) & 1) == 1;
				if ((x >> 33) == (y >> 33) && yval) {
					const uint64_t rx = x & RM, ry = y & RM;
					if ((rx > ry ? rx - ry : ry - rx) > a.tmax)
						ovf = 1;
				}
			}
		}
		a.out[k] = lo + (BUN) bnd;
	}
	if (ovf)
		atomicOr(&a.flags[0], 1u);
	if (!ALL) {
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			ord |= __shfl_xor(ord, o);
		if (lane == 0 && ord)
			atomicOr(&s_ord, ord);
		__syncthreads();
		if (tid == 0 && s_ord) {
			const uint32_t seen = __hip_atomic_load(&a.flags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			if (s_ord & ~seen)
				atomicOr(&a.flags[1], s_ord);
		}
	}
}

// ---------------------------------------------------------------------------
// Lean kernel for the common tile of wide values (lng, tmax >= 2^32): no
// nil, at most 16 partition starts in the stage, values within 2^31 of the
// stage's first value (else the tile is listed for the 64-bit kernel).  The general kernels above issue ~2.4 VALU wave-instructions per
// row (PMC: 2.44e9 for 1e9 rows = 4.0 ms of VALU issue on 1024 SIMDs -- the
// whole kernel time).  Here each row's bound is one BRANCHLESS binary search
// over the whole stage, padded to a power of two with keys above every
// threshold: a fixed number of steps, each an LDS read at an immediate
// offset, a compare and a select -- no divergent loop and its exec-mask
// SALU traffic (a per-lane walk measured 1.9e9 SALU + 1.5e9 VALU and was
// slower).  On ordered keys the search over the whole stage equals the
// frame bound (the row's own key satisfies its threshold); on unordered
// keys the result is discarded because the order flags send the column to
// the walk.  Rows map to lanes consecutively, so key reads and bound
// writes are conflict-free and coalesced.
// ---------------------------------------------------------------------------
constexpr int FSP = FS <= 2048 ? 2048 : FS <= 4096 ? 4096 : 8192;   // padded stage
static_assert(FS < FSP, "the stage needs one pad key");

template <bool PREC, bool DESC>
__global__ __launch_bounds__(256) void
k_range_k32(FArgs a)
{
	constexpr int LST = 16;
	__shared__ __attribute__((aligned(16))) uint32_t sk[FSP];
	__shared__ uint32_t s_ord;
	__shared__ int s_nst;
	__shared__ int s_st[LST];
	const int tid = threadIdx.x, lane = __lane_id();
#if MGDK_WIN_XCD
	// XCD-aware order: workgroups go round-robin over the 8 XCDs, so XCD x
	// gets a consecutive run of tiles and a tile's halo was staged by the
	// previous workgroup on the same L2
	const uint32_t per = gridDim.x / 8, rem = gridDim.x % 8, x = blockIdx.x % 8;
	const uint32_t tile = x * per + (x < rem ? x : rem) + blockIdx.x / 8;
#else
	const uint32_t tile = blockIdx.x;
#endif
	const BUN t0 = (BUN) tile * FT;
	const BUN t1 = t0 + FT < a.n ? t0 + FT : a.n;
	const BUN lo = PREC ? (t0 > FH ? t0 - FH : 0) : t0;
	const BUN hi = PREC ? (t1 + 1 < a.n ? t1 + 1 : a.n) : (t1 + FH < a.n ? t1 + FH : a.n);
	const int S = (int) (hi - lo);
	if (tid == 0)
		s_ord = 0;
	const int64_t base = a.b[lo];
	constexpr int NB = (FS + 255) / 256;
	int64_t tv[NB];
#pragma unroll
	for (int u = 0; u < NB; u++) {
		const int i = tid + u * 256;
		tv[u] = a.b[lo + (i < S ? i : S - 1)];
	}
	constexpr int NW = (FS + 3 + 1023) / 1024;
	uint32_t tw[NW];
#pragma unroll
	for (int u = 0; u < NW; u++)
		tw[u] = flags_word(a, lo, tid + u * 256, S);
	bool bad = false;
#pragma unroll
	for (int u = 0; u < NB; u++) {
		const int i = tid + u * 256;
		const uint64_t d = DESC ? (uint64_t) base - (uint64_t) tv[u] : (uint64_t) tv[u] - (uint64_t) base;
		bad |= i < S && (tv[u] == INT64_MIN || d >= 0x80000000ull);
		if (i < S)
			sk[i] = (uint32_t) d;
	}
	for (int i = S + tid; i < FSP; i += 256)
		sk[i] = 0xffffffffu;                // above every threshold
	if (tid == 0)
		s_nst = 0;
	if (__syncthreads_or(bad)) {
		if (tid == 0)
			a.relist[atomicAdd(&a.flags[4], 1u)] = tile;
		return;
	}
	// partition starts after the stage's first row: at most LST of them are
	// listed; a row's search is then confined to its partition
#pragma unroll
	for (int u = 0; u < NW; u++) {
		uint32_t wd = tw[u] & (tid + u * 256 == 0 ? ~0xffu : ~0u);
		while (wd) {
			const int by = __builtin_ctz(wd) >> 3;
			const int pos = 4 * (tid + u * 256) + by;
			if (pos < S) {
				const int at = atomicAdd(&s_nst, 1);
				if (at < LST)
					s_st[at] = pos;
			}
			wd &= ~(0xffu << (8 * by));
		}
	}
	__syncthreads();
	const int nst = s_nst;
	if (nst > LST) {
		if (tid == 0)
			a.relist[atomicAdd(&a.flags[4], 1u)] = tile;
		return;
	}
	const int NA = (int) (t1 - t0), xa = (int) (t0 - lo);
	// thresholds stay below the pad key: valid keys are < 2^31
	const uint32_t lim = (uint64_t) a.limit < 0xfffffffeull ? (uint32_t) a.limit : 0xfffffffeu;
	// the FR searches of a lane run interleaved (independent LDS reads in
	// flight); rows past the tile's end search a clamped row and store nothing
	uint32_t key[FR], t[FR], pos[FR];
#pragma unroll
	for (int u = 0; u < FR; u++) {
		const int r = tid + u * 256;
		key[u] = sk[xa + (r < NA ? r : NA - 1)];
		if (PREC)
			t[u] = key[u] > lim ? key[u] - lim : 0u;
		else
			t[u] = 0xfffffffeu - key[u] > lim ? key[u] + lim : 0xfffffffeu;
		pos[u] = 0;
	}
	// the row's partition within the stage: [ps, pe)
	int ps[FR], pe[FR];
#pragma unroll
	for (int u = 0; u < FR; u++) {
		ps[u] = 0;
		pe[u] = S;
	}
	if (nst == 0) {
#pragma unroll
		for (int h = FSP / 2; h >= 1; h >>= 1) {
#pragma unroll
			for (int u = 0; u < FR; u++) {
				const uint32_t v = sk[pos[u] + h - 1];
				// PREC: lower bound (first j with sk[j] >= key - limit);
				// else upper bound (first j with sk[j] > key + limit)
				pos[u] += (PREC ? v < t[u] : v <= t[u]) ? h : 0;
			}
		}
	} else {
#pragma unroll
		for (int u = 0; u < FR; u++) {
			const int r = tid + u * 256;
			const int xk = xa + (r < NA ? r : NA - 1);
			for (int i = 0; i < nst; i++) {
				const int st = s_st[i];
				if (st <= xk)
					ps[u] = st > ps[u] ? st : ps[u];
				else
					pe[u] = st < pe[u] ? st : pe[u];
			}
		}
		// the predicate is true before ps and false from pe on
#pragma unroll
		for (int h = FSP / 2; h >= 1; h >>= 1) {
#pragma unroll
			for (int u = 0; u < FR; u++) {
				const int j = (int) pos[u] + h - 1;
				const uint32_t v = sk[j];
				const bool c = j < ps[u] || (j < pe[u] && (PREC ? v < t[u] : v <= t[u]));
				pos[u] += c ? h : 0;
			}
		}
	}
	uint32_t ord = 0;
#pragma unroll
	for (int u = 0; u < FR; u++) {
		const int r = tid + u * 256;
		if (r >= NA)
			break;
		const int xk = xa + r;
		const int b = (int) pos[u];
		const BUN row = t0 + (BUN) r;
		const bool unres = PREC ? (b == 0 && ps[u] == 0 && lo > 0) : (b >= S && pe[u] == S && hi < a.n);
		if (unres) {
			const uint32_t at = atomicAdd(&a.flags[2], 1u);
			if (at < a.unres_cap)
				a.unres[at] = row;
		}
#if MGDK_WIN_NT
		__builtin_nontemporal_store(lo + (BUN) (b < S ? b : S), &a.out[row]);
#else
		a.out[row] = lo + (BUN) (b < S ? b : S);
#endif
		if (row + 1 < a.n && xk + 1 < pe[u]) {
			const uint32_t y = sk[xk + 1];
			if (y < key[u])
				ord |= DESC ? 2u : 1u;
			if (!DESC && y > key[u])
				ord |= 2u;
		}
	}
#pragma unroll
	for (int q = 32; q > 0; q >>= 1)
		ord |= __shfl_xor(ord, q);
	if (lane == 0 && ord)
		atomicOr(&s_ord, ord);
	__syncthreads();
	if (tid == 0 && s_ord) {
		const uint32_t seen = __hip_atomic_load(&a.flags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (s_ord & ~seen)
			atomicOr(&a.flags[1], s_ord);
	}
}

// fix-up of the rows k_range_fast could not resolve inside its stage
__global__ __launch_bounds__(256) void
k_range_fix(WArgs a, const oid *rows, uint32_t nrows)
{
	uint32_t ovf = 0;
	Stage V{nullptr, 0, 0, a.b};
	for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nrows; t += gridDim.x * blockDim.x) {
		const BUN k = rows[t];
		const BUN pi = partition_of(a, k);
		a.out[k] = sorted_bound(a, V, k, pstart(a, pi), pend(a, pi), a.Z[pi], ovf);
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
					if (!a.peers && absdiff(v, a.b[j]) > a.tmax) { ovf = 1; break; }
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
					if (!a.peers && absdiff(v, a.b[j]) > a.tmax) { ovf = 1; break; }
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

// S (partition starts as an oid BAT), lead and m of the general machinery
static int
general_setup(WArgs &a, const mgdk_bat *p, BUN n, mgdk_bat **Sp)
{
	hipStream_t st = stream();
	mgdk_bat *S = nullptr;
	if (p) {
		S = compact_flags((const int8_t *) p->theap, n, 0, true);
		if (S == nullptr)
			return -1;
	}
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
	*Sp = S;
	return 0;
}

// RANGE bounds of integer values widened to lng (bte..lng), static limit:
// the ordered fast path with its fix-ups and the unordered walk.  `limit`
// is the effective limit min(limit, tmax) (a frame edge further away than
// the type's max is the overflowing subtraction itself); `all` = unbounded.
// Sets r's values; the caller sets the count and properties.
int
mgdk::range_bounds_int64(mgdk_bat *r, const int64_t *bvals, const mgdk_bat *p, BUN n, int64_t limit,
			 uint64_t tmax, bool all, bool preceding)
{
	hipStream_t st = stream();
	if (n == 0)
		return 0;
	const dim3 blk(256);
	// 1. fast ordered pass, ascending first (the SQL default), descending if
	//    only that order holds
	const uint32_t ucap = (uint32_t) (n / 32 > 65536 ? (n / 32 < (1u << 30) ? n / 32 : (1u << 30)) : 65536);
	DevBuf fl(64), ul((size_t) ucap * 8);
	uint32_t *h = (uint32_t *) pinned(64);
	if (!fl.p || !ul.p || !h)
		return -1;
	FArgs f{};
	f.b = bvals;
	f.tmax = tmax;
	const bool mis = p && ((uintptr_t) p->theap & 3);
	DevBuf pal(mis ? n : 0);
	if (mis) {
		// misaligned view of the partition column: an aligned copy
		if (!pal.p || !hip_ok(hipMemcpyAsync(pal.p, p->theap, n, hipMemcpyDeviceToDevice, st), "memcpy"))
			return -1;
	}
	f.p = !p ? (const int8_t *) fl.p : mis ? (const int8_t *) pal.p : (const int8_t *) p->theap;
	f.pstep = p ? 1 : 0;
	f.pmask = p ? ~0u : 0u;
	f.n = n;
	f.limit = limit;
	f.preceding = preceding;
	f.peers = false;
	f.all = all;
	f.out = (oid *) r->theap;
	f.flags = fl.as<uint32_t>();
	f.unres = ul.as<oid>();
	f.unres_cap = ucap;
	const unsigned ftiles = (unsigned) ((n + FT - 1) / FT);
	static const bool narrow = getenv("MGDK_WIN_K32") ? atoi(getenv("MGDK_WIN_K32")) != 0 : true;
	DevBuf rl((size_t) ftiles * 4 + 64);
	if (!rl.p)
		return -1;
	bool ordered = false;
	for (int pass = 0; pass < 2; pass++) {
		f.desc = pass == 1;
		if (!hip_ok(hipMemsetAsync(fl.p, 0, 64, st), "memset"))
			return -1;
		// 32-bit-key tiles first; the tiles they leave (a partition start in
		// the stage, or values spanning >= 2^31) rerun with 64-bit keys
		f.tiles = nullptr;
		f.relist = rl.as<uint32_t>();
#define RK(KT, G_, P_, D_, A_) hipLaunchKernelGGL((k_range_keys<P_, D_, A_, KT>), dim3(G_), blk, 0, st, f)
#define RKA(KT, G_) do { if (preceding) { \
			if (all) RK(KT, G_, true, false, true); \
			else if (f.desc) RK(KT, G_, true, true, false); \
			else RK(KT, G_, true, false, false); \
		} else { \
			if (all) RK(KT, G_, false, false, true); \
			else if (f.desc) RK(KT, G_, false, true, false); \
			else RK(KT, G_, false, false, false); } } while (0)
		static const bool lean = getenv("MGDK_WIN_LEAN") ? atoi(getenv("MGDK_WIN_LEAN")) != 0 : true;
		if (narrow && lean && !all && tmax >= KMAXREL) {
			// wide values (lng): the lean kernel, its left-over tiles below
			if (preceding) {
				if (f.desc)
					hipLaunchKernelGGL((k_range_k32<true, true>), dim3(ftiles), blk, 0, st, f);
				else
					hipLaunchKernelGGL((k_range_k32<true, false>), dim3(ftiles), blk, 0, st, f);
			} else {
				if (f.desc)
					hipLaunchKernelGGL((k_range_k32<false, true>), dim3(ftiles), blk, 0, st, f);
				else
					hipLaunchKernelGGL((k_range_k32<false, false>), dim3(ftiles), blk, 0, st, f);
			}
			if (!hip_ok(hipMemcpyAsync(h, fl.p, 32, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
				return -1;
			f.tiles = rl.as<uint32_t>();
			if (h[4])
				RKA(uint64_t, h[4]);
		} else if (narrow) {
			RKA(uint32_t, ftiles);
			if (!hip_ok(hipMemcpyAsync(h, fl.p, 32, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
				return -1;
			f.tiles = rl.as<uint32_t>();
			if (h[4])
				RKA(uint64_t, h[4]);
		} else {
			RKA(uint64_t, ftiles);
		}
#undef RKA
#undef RK
		f.tiles = nullptr;
		if (!hip_ok(hipMemcpyAsync(h, fl.p, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			return -1;
		if (h[3]) {
			// some tile spans >= 2^32: the wide kernel (with overflow checks)
			if (!hip_ok(hipMemsetAsync(fl.p, 0, 64, st), "memset"))
				return -1;
			hipLaunchKernelGGL(k_range_fast, dim3(ftiles), blk, 0, st, f);
			if (!hip_ok(hipMemcpyAsync(h, fl.p, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
				return -1;
		}
		const uint32_t viol = h[1];
		if (all || !(viol & (f.desc ? 2u : 1u))) {
			ordered = true;
			break;
		}
		if (viol & 2u)
			break;          // neither order holds
	}
	uint32_t ovf = ordered ? (h[0] & 1) : 0;
	const uint32_t nunres = ordered ? h[2] : 0;
	if (!ordered || nunres > 0) {
		// 2. general machinery: partition starts S, nil boundaries Z
		WArgs a{};
		a.b = bvals;
		a.tmax = tmax;
		a.n = n;
		a.limit = limit;
		a.preceding = preceding;
		a.peers = false;
		a.all = all;
		a.desc = f.desc;
		a.out = (oid *) r->theap;
		a.err = fl.as<uint32_t>() + 4;
		mgdk_bat *S = nullptr;
		if (general_setup(a, p, n, &S) < 0)
			return -1;
		DevBuf Z((a.m + 1) * 8);
		if (!Z.p || !hip_ok(hipMemsetAsync(a.err, 0, 4, st), "memset")) {
			mgdk_BBPunfix(S);
			return -1;
		}
		if (!ordered) {
			hipLaunchKernelGGL(k_range_walk, dim3(grid_for(n, 256 * 4, 256 * 64)), blk, 0, st, a);
		} else {
			a.Z = Z.as<oid>();
			hipLaunchKernelGGL(k_part_nilbound, dim3(grid_for(a.m, 256, 8192)), blk, 0, st, a, Z.as<oid>());
			if (nunres <= ucap)
				hipLaunchKernelGGL(k_range_fix, dim3(grid_for(nunres, 256, 8192)), blk, 0, st, a,
						   (const oid *) ul.p, nunres);
			else
				hipLaunchKernelGGL(k_range_tile, dim3((unsigned) ((n + TT - 1) / TT)), blk, 0, st, a);
		}
		if (!hip_ok(hipMemcpyAsync(h, fl.p, 32, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
			mgdk_BBPunfix(S);
			return -1;
		}
		mgdk_BBPunfix(S);
		ovf = ordered ? (ovf | (h[4] & 1)) : (h[4] & 1);
	}
	if (ovf) {
		seterr("22003!overflow in calculation.\n");
		return -1;
	}
	return 0;
}
