// aggr.hip -- BATsum and the grouped aggregates on the MI355X.
//
// Integer sums are exact: every lane accumulates a 128-bit sum, the partials
// are combined with 64-bit atomics on the two halves (the carry of each low
// add is derived from the value it returned, so the 128-bit total is exact
// and independent of arrival order -- results are bitwise reproducible).
// The reference checks overflow after every add (ADDI_WITH_CHECK,
// gdk/gdk_aggr.c:429-705); a prefix can only leave the result type's range
// if count * max|v| exceeds it, which the kernel also measures; only then a
// one-workgroup ordered pass re-evaluates the prefixes to decide exactly.
//   BATsum       gdk/gdk_aggr.c:1018 (dosum :708; int->dbl via BATcalcavg :1112-1156)
//   BATgroupsum  :900 (nil_if_empty; the "nil before first value" rule :497-527)
//   BATgroupcount :3069, BATgroupavg3 :1996 (rounding :2070-2095),
//   BATgroupmin/max :3487-3844, BATgroupaggrinit :65
#include <cmath>
#include <vector>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

__device__ __forceinline__ hge
ldv(const void *base, int w, BUN p, bool &isnil)
{
	switch (w) {
	case 1: { int8_t v = ((const int8_t *) base)[p]; isnil = v == INT8_MIN; return v; }
	case 2: { int16_t v = ((const int16_t *) base)[p]; isnil = v == INT16_MIN; return v; }
	case 4: { int32_t v = ((const int32_t *) base)[p]; isnil = v == INT32_MIN; return v; }
	case 8: { int64_t v = ((const int64_t *) base)[p]; isnil = v == INT64_MIN; return v; }
	default: { hge v = ((const hge *) base)[p]; isnil = is_nil(v); return v; }
	}
}

__device__ __forceinline__ void
atomic_add128(unsigned long long *lohi, hge v)
{
	const unsigned long long lo = (unsigned long long) (uhge) v;
	const unsigned long long hi = (unsigned long long) ((uhge) v >> 64);
	unsigned long long old = atomicAdd(&lohi[0], lo);
	unsigned long long carry = (old + lo) < old ? 1ull : 0ull;
	if (hi + carry)
		atomicAdd(&lohi[1], hi + carry);
}

__device__ __forceinline__ uint64_t
absbits(hge v)
{
	// ceil-ish magnitude class: top 64 bits of |v| (0 for |v| < 2^64) and low
	uhge a = v < 0 ? (uhge) 0 - (uhge) v : (uhge) v;
	return (a >> 64) ? (uint64_t) (a >> 64) | (1ull << 63) : (uint64_t) a >> 1;
}

// ---- BATsum -----------------------------------------------------------------
struct SumOut {
	unsigned long long sum[2];     // 128-bit total (two's complement)
	unsigned long long cnt;        // non-nil values
	unsigned long long firstnil;   // first nil position (candidate index)
	unsigned long long maxabs;     // magnitude class (absbits)
};

// one workgroup's share of a BATsum, summed by k_sum_fin: a same-address
// atomic from every workgroup serialised at one L2 channel
struct SumPart {
	unsigned long long lo, hi, cnt, firstnil, maxabs, pad[3];
};

template <int W>
__device__ __forceinline__ hge
ldw(const void *base, BUN p, bool &isnil)
{
	if constexpr (W == 1) { const int8_t v = ((const int8_t *) base)[p]; isnil = v == INT8_MIN; return v; }
	else if constexpr (W == 2) { const int16_t v = ((const int16_t *) base)[p]; isnil = v == INT16_MIN; return v; }
	else if constexpr (W == 4) { const int32_t v = ((const int32_t *) base)[p]; isnil = v == INT32_MIN; return v; }
	else if constexpr (W == 8) { const int64_t v = ((const int64_t *) base)[p]; isnil = v == INT64_MIN; return v; }
	else { const hge v = ((const hge *) base)[p]; isnil = is_nil(v); return v; }
}

// W: value width as a template parameter and U rows per thread loaded
// before any is added (a runtime width switch waits for each load)
template <int W, bool DENSE>
__global__ __launch_bounds__(256) void
k_sum(const void *base, oid off, const oid *oids, oid hseq, BUN n, SumPart *parts)
{
	constexpr int U = 8;
	hge s = 0;
	unsigned long long cnt = 0, firstnil = ~0ull, mx = 0;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i0 = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += U * stride) {
		hge v[U];
		bool nl[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * stride, ic = i < n ? i : n - 1;
			v[u] = ldw<W>(base, DENSE ? off + ic : oids[ic] - hseq, nl[u]);
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * stride;
			if (i >= n)
				continue;
			if (nl[u]) {
				firstnil = i < firstnil ? i : firstnil;
				continue;
			}
			s += v[u];
			cnt++;
			const unsigned long long a = absbits(v[u]);
			mx = a > mx ? a : mx;
		}
	}
	s = block_sum128(s);
	cnt = block_reduce(cnt, [](unsigned long long x, unsigned long long y) { return x + y; });
	firstnil = block_reduce(firstnil, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	mx = block_reduce(mx, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	if (threadIdx.x == 0) {
		SumPart p;
		p.lo = (unsigned long long) (uhge) s;
		p.hi = (unsigned long long) ((uhge) s >> 64);
		p.cnt = cnt;
		p.firstnil = firstnil;
		p.maxabs = mx;
		p.pad[0] = p.pad[1] = p.pad[2] = 0;
		parts[blockIdx.x] = p;
	}
}

__global__ __launch_bounds__(256) void
k_sum_fin(const SumPart *parts, uint32_t np, SumOut *o)
{
	hge s = 0;
	unsigned long long cnt = 0, firstnil = ~0ull, mx = 0;
	for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
		const SumPart p = parts[i];
		s += (hge) (((uhge) p.hi << 64) | p.lo);
		cnt += p.cnt;
		firstnil = p.firstnil < firstnil ? p.firstnil : firstnil;
		mx = p.maxabs > mx ? p.maxabs : mx;
	}
	s = block_sum128(s);
	cnt = block_reduce(cnt, [](unsigned long long x, unsigned long long y) { return x + y; });
	firstnil = block_reduce(firstnil, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	mx = block_reduce(mx, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	if (threadIdx.x == 0) {
		o->sum[0] = (unsigned long long) (uhge) s;
		o->sum[1] = (unsigned long long) ((uhge) s >> 64);
		o->cnt = cnt;
		o->firstnil = firstnil;
		o->maxabs = mx;
	}
}

// ordered prefix check for the rare case where overflow is possible: one
// workgroup, each lane a contiguous chunk, then an ordered combine of
// (sum, max prefix, min prefix).  Uses a 192-bit-safe formulation: values are
// at most 128 bits and we stop at the first overflow, so partial sums are
// kept as (hi: int64 guard, 128-bit) via a per-chunk scan.
__global__ __launch_bounds__(256) void
k_sum_ordered(const void *base, int w, bool dense, oid off, const oid *oids, oid hseq, BUN n,
	      hge max, unsigned long long *ovf)
{
	__shared__ hge s_sum[256], s_mx[256], s_mn[256];
	__shared__ int s_has[256], s_bad[256];
	const BUN chunk = (n + 255) / 256;
	const BUN a = threadIdx.x * chunk, e = a + chunk < n ? a + chunk : n;
	hge s = 0, mx = 0, mn = 0;
	int has = 0, bad = 0;
	for (BUN i = a; i < e; i++) {
		BUN p = dense ? off + i : oids[i] - hseq;
		bool isnil;
		hge v = ldv(base, w, p, isnil);
		if (isnil)
			continue;
		uhge r = (uhge) s + (uhge) v;
		hge rs = (hge) r;
		if (((s < 0) == (v < 0)) && ((rs < 0) != (s < 0)))
			bad = 1;   // the chunk's own running sum left 128 bits: overflow for sure
		s = rs;
		if (!has) { mx = mn = s; has = 1; }
		else { mx = s > mx ? s : mx; mn = s < mn ? s : mn; }
	}
	s_sum[threadIdx.x] = s;
	s_mx[threadIdx.x] = mx;
	s_mn[threadIdx.x] = mn;
	s_has[threadIdx.x] = has;
	s_bad[threadIdx.x] = bad;
	__syncthreads();
	if (threadIdx.x == 0) {
		// chunk-local overflow of the 128-bit running sum only matters if
		// the true prefix also overflows, which it then does: any chunk
		// prefix beyond 2^127 plus a prefix sum below max is beyond max?
		// Not in general -- combine exactly with a 192-bit accumulator.
		__int128 acc_lo = 0;
		long long acc_hi = 0;   // acc = acc_hi * 2^128 + (uhge) acc_lo, signed
		bool over = false;
		for (int t = 0; t < 256 && !over; t++) {
			if (s_bad[t]) { over = true; break; }
			if (!s_has[t])
				continue;
			// test base + mx and base + mn against [-max, max]
			for (int q = 0; q < 2 && !over; q++) {
				hge x = q ? s_mn[t] : s_mx[t];
				uhge lo = (uhge) acc_lo + (uhge) x;
				long long hi = acc_hi + ((lo < (uhge) acc_lo) ? 1 : 0) + (x < 0 ? -1 : 0);
				// value = hi*2^128 + lo (lo unsigned)
				if (hi == 0 && (hge) lo >= 0) { if ((hge) lo > max) over = true; }
				else if (hi == -1 && (hge) lo < 0) { if ((hge) lo < -max) over = true; }
				else over = true;
			}
			uhge lo = (uhge) acc_lo + (uhge) s_sum[t];
			acc_hi = acc_hi + ((lo < (uhge) acc_lo) ? 1 : 0) + (s_sum[t] < 0 ? -1 : 0);
			acc_lo = (hge) lo;
		}
		*ovf = over ? 1 : 0;
	}
}

hge
tmax(int tp)
{
	switch (basetype(tp)) {
	case MGDK_bte: return INT8_MAX;
	case MGDK_sht: return INT16_MAX;
	case MGDK_int: return INT32_MAX;
	case MGDK_lng: return INT64_MAX;
	default: return (hge) (((uhge) 1 << 127) - 1);
	}
}

bool
int_type(int t)
{
	t = basetype(t);
	return t == MGDK_bte || t == MGDK_sht || t == MGDK_int || t == MGDK_lng || t == MGDK_hge;
}

void
put_res(void *res, int tp, hge v, bool nil)
{
	switch (basetype(tp)) {
	case MGDK_bte: *(int8_t *) res = nil ? INT8_MIN : (int8_t) v; break;
	case MGDK_sht: *(int16_t *) res = nil ? INT16_MIN : (int16_t) v; break;
	case MGDK_int: *(int32_t *) res = nil ? INT32_MIN : (int32_t) v; break;
	case MGDK_lng: *(int64_t *) res = nil ? INT64_MIN : (int64_t) v; break;
	case MGDK_oid: *(uint64_t *) res = nil ? MGDK_OID_NIL : (uint64_t) v; break;
	default: { hge x = nil ? (hge) ((uhge) 1 << 127) : v; memcpy(res, &x, 16); break; }
	}
}

// magnitude bound from absbits class: returns an upper bound of max|v| as
// a long double (enough to decide "could a prefix overflow")
long double
mag_bound(unsigned long long cls)
{
	if (cls >> 63)
		return ldexpl((long double) ((cls & ~(1ull << 63)) + 1), 64);
	return ((long double) cls + 1) * 2;
}

}  // namespace

int mgdk_fsum(void *res, int tp, mgdk_bat *b, mgdk_bat *s, bool skip_nils, bool nil_if_empty);   // fsum.hip
int mgdk_fgroupsum(const mgdk_bat *b, const Cand &ci, const oid *gids, oid gseq, oid gmin, BUN ngrp, bool skip_nils,
		   int tp, void *res, bool *nils);                                                   // fsum.hip

extern "C" int
mgdk_BATsum(void *res, int tp, mgdk_bat *b, mgdk_bat *s, bool skip_nils, bool nil_if_empty)
{
	if (b == nullptr || res == nullptr) {
		seterr("BATsum: NULL argument");
		return -1;
	}
	if (b->ttype == MGDK_flt || b->ttype == MGDK_dbl)
		return mgdk_fsum(res, tp, b, s, skip_nils, nil_if_empty);   // dofsum, gdk_aggr.c:183
	if (!int_type(b->ttype) || !(int_type(tp) || tp == MGDK_dbl || tp == MGDK_flt)) {
		seterr("type combination (sum(%s)->%s) not supported.\n", atomname(b->ttype), atomname(tp));
		return -1;
	}
	ProfScope prof("sum");
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return -1;
	SumOut *o = (SumOut *) meta_buf();
	const oid off = ci.dense ? ci.seq - b->hseqbase : 0;
	if (ci.n) {
		const unsigned g = grid_for(ci.n, 256 * 8, 2048);
		SumPart *parts = (SumPart *) scratch((size_t) g * sizeof(SumPart));
		if (parts == nullptr)
			return -1;
		const dim3 gd(g), blk(256);
#define KS(W_) do { if (ci.dense) hipLaunchKernelGGL((k_sum<W_, true>), gd, blk, 0, stream(), b->theap, off, ci.oids, b->hseqbase, ci.n, parts); \
		else hipLaunchKernelGGL((k_sum<W_, false>), gd, blk, 0, stream(), b->theap, off, ci.oids, b->hseqbase, ci.n, parts); } while (0)
		switch (b->twidth) {
		case 1: KS(1); break;
		case 2: KS(2); break;
		case 4: KS(4); break;
		case 8: KS(8); break;
		default: KS(16); break;
		}
#undef KS
		hipLaunchKernelGGL(k_sum_fin, dim3(1), dim3(256), 0, stream(), parts, g, o);
	} else {
		SumOut init = {{0, 0}, 0, ~0ull, 0};
		if (!hip_ok(hipMemcpyAsync(o, &init, sizeof(init), hipMemcpyHostToDevice, stream()), "memcpy"))
			return -1;
	}
	SumOut *h = (SumOut *) pinned(sizeof(SumOut));
	if (h == nullptr || !hip_ok(hipMemcpyAsync(h, o, sizeof(SumOut), hipMemcpyDeviceToHost, stream()), "memcpy") ||
	    !sync())
		return -1;
	const hge total = (hge) (((uhge) h->sum[1] << 64) | h->sum[0]);
	const BUN cnt = h->cnt;
	if (tp == MGDK_dbl || tp == MGDK_flt) {
		// integers into floating point: exact average times count
		// (gdk_aggr.c:1112-1156, BATcalcavg :2905-2960 with a hge sum)
		double avg;
		bool nil = false;
		if (cnt == 0) {
			nil = nil_if_empty;
			avg = 0;
		} else {
			avg = (double) total / (double) cnt;
		}
		if (cnt < ci.n && !skip_nils)
			nil = true;
		if (tp == MGDK_dbl)
			*(double *) res = nil ? __builtin_nan("") : avg * (double) cnt;
		else
			*(float *) res = nil ? __builtin_nanf("") : (float) avg * cnt;
		return 0;
	}
	const hge max = tmax(tp);
	const BUN firstnil = (!skip_nils && h->firstnil != ~0ull) ? h->firstnil : ci.n;
	// could any prefix within [0, firstnil) leave [-max, max]?
	long double bound = mag_bound(h->maxabs) * (long double) cnt;
	bool maybe = bound > (long double) max;
	if (maybe) {
		unsigned long long *ov = (unsigned long long *) o;
		hipLaunchKernelGGL(k_sum_ordered, dim3(1), dim3(256), 0, stream(), b->theap, b->twidth, ci.dense, off,
				   ci.oids, b->hseqbase, firstnil, max, ov);
		unsigned long long *hv = (unsigned long long *) pinned(16);
		if (!hip_ok(hipMemcpyAsync(hv, ov, 8, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
			return -1;
		if (*hv) {
			seterr("22003!overflow in sum aggregate.\n");
			return -1;
		}
	}
	if (firstnil < ci.n) {
		put_res(res, tp, 0, true);
		return 0;
	}
	if (cnt == 0) {
		put_res(res, tp, 0, nil_if_empty);
		return 0;
	}
	put_res(res, tp, total, false);
	return 0;
}

// ---- grouped aggregates ------------------------------------------------------
namespace {

// per group accumulators, laid out struct-of-arrays in global memory
struct GAcc {
	unsigned long long *sum;      // [2*ngrp] 128-bit sums
	unsigned long long *cnt;      // [ngrp] non-nil values (or all rows)
	unsigned long long *firstval; // [ngrp] first non-nil candidate index
	unsigned long long *lastnil;  // [ngrp] last nil candidate index + 1 (0 = none)
	long long *mn, *mx;           // [ngrp] min / max (lng-representable types)
	unsigned long long maxabs;    // magnitude class over all values
};

enum { AGG_SUM = 1, AGG_CNT = 2, AGG_POS = 4, AGG_MINMAX = 8 };

// K > 0: few groups -> per-lane register accumulators, one flush per wave
template <int K>
__global__ __launch_bounds__(256) void
k_gaggr(const void *base, int w, oid off, const oid *gids, oid gseq, oid gmin, BUN ngrp, BUN n,
	int what, bool count_all, GAcc acc, unsigned long long *maxabs)
{
	hge s[K > 0 ? K : 1];
	unsigned long long c[K > 0 ? K : 1];
	if constexpr (K > 0) {
#pragma unroll
		for (int k = 0; k < K; k++) { s[k] = 0; c[k] = 0; }
	}
	unsigned long long mx = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		oid g = gids ? gids[i] : gseq + i;
		if (g < gmin || g - gmin >= ngrp)
			continue;
		BUN gi = g - gmin;
		bool isnil;
		hge v = ldv(base, w, off + i, isnil);
		if (isnil) {
			if (what & AGG_POS)
				atomicMax(&acc.lastnil[gi], (unsigned long long) i + 1);
			if (count_all) {
				if constexpr (K > 0) {
#pragma unroll
					for (int k = 0; k < K; k++) c[k] += gi == (BUN) k;
				} else {
					atomicAdd(&acc.cnt[gi], 1ull);
				}
			}
			continue;
		}
		unsigned long long a = absbits(v);
		mx = a > mx ? a : mx;
		if (what & AGG_POS) {
			unsigned long long fv = acc.firstval[gi];
			if (i < fv)
				atomicMin(&acc.firstval[gi], (unsigned long long) i);
		}
		if (what & AGG_MINMAX) {
			atomicMin(&acc.mn[gi], (long long) v);
			atomicMax(&acc.mx[gi], (long long) v);
		}
		if constexpr (K > 0) {
#pragma unroll
			for (int k = 0; k < K; k++) {
				bool m = gi == (BUN) k;
				s[k] += m ? v : (hge) 0;
				c[k] += m;
			}
		} else {
			if (what & AGG_SUM)
				atomic_add128(&acc.sum[2 * gi], v);
			atomicAdd(&acc.cnt[gi], 1ull);
		}
	}
	if constexpr (K > 0) {
#pragma unroll
		for (int k = 0; k < K; k++) {
			hge sk = s[k];
			unsigned long long ck = c[k];
			for (int o = 32; o > 0; o >>= 1) {
				unsigned long long lo = __shfl_xor((unsigned long long) (uhge) sk, o);
				unsigned long long hi = __shfl_xor((unsigned long long) ((uhge) sk >> 64), o);
				sk += (hge) (((uhge) hi << 64) | lo);
				ck += __shfl_xor(ck, o);
			}
			if (__lane_id() == 0 && (BUN) k < ngrp) {
				if (ck) {
					if (what & AGG_SUM)
						atomic_add128(&acc.sum[2 * k], sk);
					atomicAdd(&acc.cnt[k], ck);
				}
			}
		}
	}
	for (int o = 32; o > 0; o >>= 1) {
		unsigned long long t = __shfl_xor(mx, o);
		mx = t > mx ? t : mx;
	}
	if (__lane_id() == 0 && mx)
		publish_max(maxabs, mx);
}

// few groups (K <= 8): every per-group quantity in lane registers -- sums,
// counts, first non-nil position, last nil position, min / max -- so the
// loop has no global loads besides the gid and the value (U rows in flight
// per lane); positions only grow along a lane, so "first" is the first one
// seen and "last" the last one.  One flush of wave-reduced values per wave.
// GT: uint8_t reads the 1-byte group-id image BATgroup keeps with g (<= 255
// groups), oid the 8-byte ids.  W16 = false: values of <= 8 bytes are summed
// exactly as two 64-bit lane accumulators of their low 32 (unsigned) and high
// 32 (signed) bits -- a lane sees < 2^31 rows -- instead of 128-bit adds.
// POS: first non-nil / last nil positions are only tracked when wanted.
template <int VW> struct VTy;
template <> struct VTy<0> { typedef int64_t T; };   // COUNT(*): no values read
template <> struct VTy<1> { typedef int8_t T; };
template <> struct VTy<2> { typedef int16_t T; };
template <> struct VTy<4> { typedef int32_t T; };
template <> struct VTy<8> { typedef int64_t T; };
template <> struct VTy<16> { typedef hge T; };

// VW: value width, a template parameter so that the U loads of a step are
// straight-line code (a runtime width switch puts every load in its own
// block and the compiler then waits for each one before the next)
// per-wave partial of one group (k_gaggr_k writes them, k_gaggr_fin sums
// them): no same-word atomics from thousands of waves, which serialise at
// the L2 (~88 per microsecond per word)
struct GPart {
	unsigned long long lo, hi, cnt, fv, ln;
	long long mn, mx;
	unsigned long long mxa;
};

template <int K, bool MM, bool POS, int VW, typename GT>
__global__ __launch_bounds__(256) void
k_gaggr_k(const void *base, int w, oid off, const GT *gids, oid gseq, oid gmin, BUN ngrp, BUN n, int what,
	  bool count_all, GPart *parts)
{
	constexpr bool W16 = VW == 16;
	typedef typename VTy<VW>::T VT;
	(void) w;
	hge s[W16 ? K : 1];
	unsigned long long slo[W16 ? 1 : K];
	long long shi[W16 ? 1 : K];
	unsigned c[K];
	unsigned long long fv[POS ? K : 1], ln[POS ? K : 1];
	long long mn[MM ? K : 1], mx[MM ? K : 1];
#pragma unroll
	for (int k = 0; k < K; k++) {
		if (W16)
			s[k] = 0;
		else
			slo[k] = 0, shi[k] = 0;
		c[k] = 0;
		if (POS)
			fv[k] = ~0ull, ln[k] = 0;
		if (MM)
			mn[k] = INT64_MAX, mx[k] = INT64_MIN;
	}
	unsigned long long mxa = 0;
	// each wave streams 64 * U consecutive rows per step (row = chunk base +
	// u * 64 + lane: every load instruction covers 64 consecutive values),
	// U independent loads in flight per lane
	constexpr int U = W16 ? 8 : 16;
	constexpr BUN CH = 64 * U;
	const uint32_t gm = (uint32_t) gmin;
	const unsigned lane = __lane_id();
	const BUN nwaves = (BUN) gridDim.x * (blockDim.x / 64);
	// LC: 1-byte ids (the image BATgroup keeps), staged per wave in LDS
	constexpr bool LC = sizeof(GT) == 1;
	__shared__ uint32_t s_gid[4][LC ? 16 * U : 1];
	for (BUN ch = (BUN) blockIdx.x * (blockDim.x / 64) + (threadIdx.x / 64); ch * CH < n; ch += nwaves) {
		// row = chunk base + u * 64 + lane for the values, so every value load
		// instruction covers 64 consecutive values (a lane-contiguous layout
		// makes each instruction touch 64 cache lines).  1-byte ids are read
		// lane-contiguously (one 16- or 8-byte load per lane covers the wave's
		// chunk) and transposed through the wave's LDS slot.
		const BUN i0 = ch * CH + lane;
		constexpr BUN du = 64;
		uint32_t gi[U];
		hge v[U];
		bool nil[U];
		// every load is issued unconditionally (at a clamped index) and masked
		// afterwards: a load under a divergent branch makes the compiler wait
		// for it before the branch joins, which serialises the U loads
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * du;
			const bool ok = i < n;
			const BUN ic = ok ? i : n - 1;
			if (LC) {
				;
			} else {
				const oid g = gids ? (oid) gids[ic] : gseq + ic;
				gi[u] = (!ok || g < gmin || g - gmin >= ngrp) ? ~0u : (uint32_t) (g - gmin);
			}
			// base NULL: COUNT(*) -- every row counts, no value is read
			if constexpr (VW > 0) {
				const VT x = ((const VT *) base)[off + ic];
				v[u] = x;
				nil[u] = is_nil(x);
			} else {
				v[u] = 0;
				nil[u] = false;
			}
		}
		if constexpr (LC) {
			// one aligned id block per lane at a clamped address (a lane past the
			// end reads the last block; its rows are masked below): no branch
			const BUN last = (n - 1) & ~(BUN) (U - 1);
			const BUN ga = ch * CH + (BUN) lane * U;
			const uint8_t *gp = (const uint8_t *) gids + (ga <= last ? ga : last);
			uint32_t wds[U / 4];
			if constexpr (U == 16) {
				const uint4 q = *(const uint4 *) gp;
				wds[0] = q.x, wds[1] = q.y, wds[2] = q.z, wds[3] = q.w;
			} else {
				const uint2 q = *(const uint2 *) gp;
				wds[0] = q.x, wds[1] = q.y;
			}
			uint32_t *sw = s_gid[threadIdx.x / 64];
#pragma unroll
			for (int q = 0; q < U / 4; q++)
				sw[lane * (U / 4) + q] = wds[q];
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			const uint8_t *sb = (const uint8_t *) sw;
			uint32_t gb8[U];
#pragma unroll
			for (int u = 0; u < U; u++)
				gb8[u] = sb[u * 64 + lane];
#pragma unroll
			for (int u = 0; u < U; u++) {
				const BUN i = i0 + (BUN) u * 64;
				gi[u] = i < n ? gb8[u] - gm : ~0u;
			}
			__builtin_amdgcn_wave_barrier();
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * du;
			if (gi[u] >= (uint32_t) ngrp)
				continue;
			if (nil[u]) {
#pragma unroll
				for (int k = 0; k < K; k++) {
					const bool m = gi[u] == (uint32_t) k;
					if (POS)
						ln[k] = m ? i + 1 : ln[k];
					c[k] += (m && count_all);
				}
				continue;
			}
			unsigned long long a;
			if (W16) {
				a = absbits(v[u]);
			} else {
				const long long x = (long long) v[u];
				a = (unsigned long long) (x < 0 ? -x : x) >> 1;
			}
			mxa = a > mxa ? a : mxa;
			const uint32_t lo32 = (uint32_t) (unsigned long long) v[u];
			const int32_t hi32 = (int32_t) ((long long) v[u] >> 32);
#pragma unroll
			for (int k = 0; k < K; k++) {
				const bool m = gi[u] == (uint32_t) k;
				if (W16) {
					s[k] += m ? v[u] : (hge) 0;
				} else {
					slo[k] += m ? lo32 : 0u;
					shi[k] += m ? hi32 : 0;
				}
				c[k] += m;
				if (POS)
					fv[k] = (m && fv[k] == ~0ull) ? i : fv[k];
				if (MM) {
					const long long x = (long long) v[u];
					mn[k] = (m && x < mn[k]) ? x : mn[k];
					mx[k] = (m && x > mx[k]) ? x : mx[k];
				}
			}
		}
	}
#pragma unroll
	for (int k = 0; k < K; k++) {
		hge sk = W16 ? s[k] : (hge) shi[k] * ((hge) 1 << 32) + (hge) slo[k];
		unsigned long long ck = c[k], fk = POS ? fv[k] : ~0ull, lk = POS ? ln[k] : 0;
		long long nk = MM ? mn[k] : 0, xk = MM ? mx[k] : 0;
		for (int o = 32; o > 0; o >>= 1) {
			const unsigned long long lo = __shfl_xor((unsigned long long) (uhge) sk, o);
			const unsigned long long hi = __shfl_xor((unsigned long long) ((uhge) sk >> 64), o);
			sk += (hge) (((uhge) hi << 64) | lo);
			ck += __shfl_xor(ck, o);
			if (POS) {
				const unsigned long long f2 = __shfl_xor(fk, o), l2 = __shfl_xor(lk, o);
				fk = f2 < fk ? f2 : fk;
				lk = l2 > lk ? l2 : lk;
			}
			if (MM) {
				const long long n2 = __shfl_xor(nk, o), x2 = __shfl_xor(xk, o);
				nk = n2 < nk ? n2 : nk;
				xk = x2 > xk ? x2 : xk;
			}
		}
		if (__lane_id() == 0) {
			GPart pp;
			pp.lo = (unsigned long long) (uhge) sk;
			pp.hi = (unsigned long long) ((uhge) sk >> 64);
			pp.cnt = ck;
			pp.fv = fk;
			pp.ln = lk;
			pp.mn = MM ? nk : INT64_MAX;
			pp.mx = MM ? xk : INT64_MIN;
			pp.mxa = 0;
			parts[((BUN) blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * K + k] = pp;
		}
	}
	for (int o = 32; o > 0; o >>= 1) {
		const unsigned long long t = __shfl_xor(mxa, o);
		mxa = t > mxa ? t : mxa;
	}
	if (__lane_id() == 0)
		parts[((BUN) blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * K].mxa = mxa;
}

// one workgroup per group: the sum of the per-wave partials into acc
__global__ __launch_bounds__(256) void
k_gaggr_fin(const GPart *parts, BUN nwaves, int K, BUN ngrp, GAcc acc, unsigned long long *maxabs)
{
	const int k = blockIdx.x;
	uhge s = 0;
	unsigned long long c = 0, fv = ~0ull, ln = 0, mxa = 0;
	long long mn = INT64_MAX, mx = INT64_MIN;
	for (BUN wv = threadIdx.x; wv < nwaves; wv += blockDim.x) {
		const GPart &p = parts[wv * K + k];
		s += ((uhge) p.hi << 64) | p.lo;
		c += p.cnt;
		fv = p.fv < fv ? p.fv : fv;
		ln = p.ln > ln ? p.ln : ln;
		mn = p.mn < mn ? p.mn : mn;
		mx = p.mx > mx ? p.mx : mx;
		if (k == 0)
			mxa = p.mxa > mxa ? p.mxa : mxa;
	}
	s = (uhge) block_sum128((hge) s);
	c = block_reduce(c, [](unsigned long long x, unsigned long long y) { return x + y; });
	fv = block_reduce(fv, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	ln = block_reduce(ln, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	mn = block_reduce(mn, [](long long x, long long y) { return x < y ? x : y; });
	mx = block_reduce(mx, [](long long x, long long y) { return x > y ? x : y; });
	mxa = block_reduce(mxa, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	if (threadIdx.x == 0) {
		if ((BUN) k < ngrp) {
			acc.sum[2 * k] = (unsigned long long) s;
			acc.sum[2 * k + 1] = (unsigned long long) (s >> 64);
			acc.cnt[k] = c;
			acc.firstval[k] = fv;
			acc.lastnil[k] = ln;
			acc.mn[k] = mn;
			acc.mx[k] = mx;
		}
		if (k == 0)
			*maxabs = mxa;
	}
}

// ---- many groups, g sorted (every group a run of consecutive rows, as
// BATgroup numbers ordered keys, a sub-grouping of them or a clustered
// column): a wave owns a range of 64 * GS_U rows and a lane GS_U CONSECUTIVE
// rows of it, all loaded before any is used.  A lane reduces its rows in
// order and stores every run that starts and ends inside them with plain
// stores (no other lane or wave holds that group); only the lane's first and
// last runs meet the neighbouring lanes, through ONE segmented scan over the
// 64 lanes per range.  The range's first run (it may have begun in the
// previous range) and its last (it may go on) are added with atomics.
// (Round 2's one-row-per-lane version ran a 64-lane segmented scan per 64
// rows with one chunk's loads in flight: 7.9 ms for 600M rows.)
constexpr int GS_U = 16;    // rows per lane
constexpr int GS_UA = 8;    // rows per lane when the accumulators are staged in LDS

struct GRun {
	uhge s;
	unsigned long long c, fv, ln;
	long long mn, mx;
	__device__ void clear()
	{
		s = 0;
		c = 0;
		fv = ~0ull;
		ln = 0;
		mn = INT64_MAX;
		mx = INT64_MIN;
	}
	template <bool MM, bool POS>
	__device__ void add(const GRun &o)
	{
		s += o.s;
		c += o.c;
		if (POS) {
			fv = o.fv < fv ? o.fv : fv;
			ln = o.ln > ln ? o.ln : ln;
		}
		if (MM) {
			mn = o.mn < mn ? o.mn : mn;
			mx = o.mx > mx ? o.mx : mx;
		}
	}
	template <bool MM, bool POS>
	__device__ GRun shfl_up(int d) const
	{
		GRun t;
		t.s = ((uhge) __shfl_up((unsigned long long) (s >> 64), d) << 64) | __shfl_up((unsigned long long) s, d);
		t.c = __shfl_up(c, d);
		t.fv = POS ? __shfl_up(fv, d) : ~0ull;
		t.ln = POS ? __shfl_up(ln, d) : 0;
		t.mn = MM ? __shfl_up(mn, d) : INT64_MAX;
		t.mx = MM ? __shfl_up(mx, d) : INT64_MIN;
		return t;
	}
};

__device__ __forceinline__ void put_res_d(void *base, int bt, BUN k, hge v, bool nil);

// BATgroupsum straight into its result column (sums with skip_nils or
// without nils: a group's result is nil only when it has no value): the
// per-group accumulators, their initialisation and the finishing pass go
// away; the groups a range shares with its neighbours leave their partial
// in `edges` (two per range, in range order, so a group's partials are
// consecutive) for k_gedge_sum instead of being added with atomics
struct SOut {
	void *out;
	int bt;
	hge max;
	uint32_t *flags;
	bool on;
};

struct GEdge {
	oid g;
	unsigned long long lo, hi, c;
};

__device__ __forceinline__ uint32_t
sout_put(const SOut &so, BUN gi, uhge s, unsigned long long c)
{
	const hge sv = (hge) s;
	const bool nil = c == 0;
	put_res_d(so.out, so.bt, gi, nil ? 0 : sv, nil);
	return (sv > so.max || sv < -so.max ? 1u : 0u) | (nil ? 2u : 0u);
}

// the groups k_gaggr_sorted adds to with atomics: those of every range's
// first and last row
__global__ __launch_bounds__(256) void
k_gacc_edges(const oid *gids, oid gseq, oid gmin, BUN ngrp, BUN n, BUN RW, GAcc acc, int what)
{
	const BUN nr = (n + RW - 1) / RW;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < nr; k += (BUN) gridDim.x * blockDim.x) {
		const BUN rows[2] = {k * RW, (k + 1) * RW < n ? (k + 1) * RW - 1 : n - 1};
		for (int e = 0; e < 2; e++) {
			const oid g = gids ? gids[rows[e]] : gseq + rows[e];
			if (g < gmin || g - gmin >= ngrp)
				continue;
			const BUN gi = g - gmin;
			if (what & AGG_SUM) {
				acc.sum[2 * gi] = 0;
				acc.sum[2 * gi + 1] = 0;
			}
			acc.cnt[gi] = 0;
			if (what & AGG_POS) {
				acc.firstval[gi] = ~0ull;
				acc.lastnil[gi] = 0;
			}
		}
	}
}

extern __shared__ unsigned long long gs_stage_lds[];

template <int VW, bool MM, bool POS, int U>
__global__ __launch_bounds__(256) void
k_gaggr_sorted(const void *base, oid off, const oid *gids, oid gseq, oid gmin, BUN ngrp, BUN n, bool do_sum,
	       bool count_all, bool vec, bool gapinit, bool stage, GAcc acc, unsigned long long *maxabs, SOut so,
	       GEdge *edges)
{
	typedef typename VTy<VW>::T T;
	// sums / counts only: a range's complete groups (a contiguous id
	// interval) are staged in LDS and stored as contiguous runs -- stored
	// from the lanes that finish them, the 8-byte pieces of neighbouring
	// groups left partial lines behind (PMC: 9.3 GB written for 3.6 GB of
	// accumulators at 150M groups)
	// stage (runtime, sums / counts into accumulators only): the launch
	// gives 3 * RW words of dynamic LDS per wave
	constexpr bool STAGE = !MM && !POS;
	constexpr BUN RW = 64 * U;
	unsigned long long *s_lo = gs_stage_lds + (threadIdx.x >> 6) * 3 * RW, *s_hi = s_lo + RW, *s_c = s_hi + RW;
	const int lane = __lane_id(), wv = threadIdx.x >> 6;
	const BUN nwaves = (BUN) gridDim.x * (blockDim.x / 64);
	const BUN wid = (BUN) blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
	unsigned long long mxa = 0;
	oid sbase = 0, send = 0;     // staged ids: (sbase, send)
	uint32_t sof = 0;            // SOut flags
	auto flush = [&](bool atomic, BUN gi, const GRun &r) {
		if (!atomic && so.on && !(STAGE && stage && gi + gmin > sbase && gi + gmin < send)) {
			sof |= sout_put(so, gi, r.s, r.c);
			return;
		}
		if (STAGE && stage && !atomic && gi + gmin > sbase && gi + gmin < send) {
			const BUN k = gi + gmin - sbase;
			if (do_sum) {
				s_lo[k] = (unsigned long long) r.s;
				s_hi[k] = (unsigned long long) (r.s >> 64);
			}
			s_c[k] = r.c;
		} else if (atomic) {
			if (do_sum && r.s)
				atomic_add128(&acc.sum[2 * gi], (hge) r.s);
			if (r.c)
				atomicAdd(&acc.cnt[gi], r.c);
			if (POS && r.fv != ~0ull)
				atomicMin(&acc.firstval[gi], r.fv);
			if (POS && r.ln)
				atomicMax(&acc.lastnil[gi], r.ln);
			if (MM && r.c) {
				atomicMin(&acc.mn[gi], r.mn);
				atomicMax(&acc.mx[gi], r.mx);
			}
		} else {
			if (do_sum) {
				acc.sum[2 * gi] = (unsigned long long) r.s;
				acc.sum[2 * gi + 1] = (unsigned long long) (r.s >> 64);
			}
			acc.cnt[gi] = r.c;
			if (POS) {
				acc.firstval[gi] = r.fv;
				acc.lastnil[gi] = r.ln;
			}
			if (MM) {
				acc.mn[gi] = r.mn;
				acc.mx[gi] = r.mx;
			}
		}
	};
	auto valid = [&](oid g) { return g >= gmin && g - gmin < ngrp; };
	// gapinit: the accumulators were not initialised (k_gacc_edges set the
	// groups the atomics add to); groups with no row, i.e. the gaps between
	// consecutive ids and before / after them, get the identity here
	// the groups strictly between ids prev and next (prev < next, sorted)
	auto gap = [&](oid prev, oid hi) {
		if (!gapinit || prev >= gmin + ngrp)
			return;
		oid lo = prev + 1;
		lo = lo > gmin ? lo : gmin;
		hi = hi < gmin + ngrp ? hi : gmin + ngrp;
		for (oid h = lo; h < hi; h++) {
			GRun e;
			e.clear();
			flush(false, h - gmin, e);
		}
	};
	for (BUN r0 = wid * RW; r0 < n; r0 += nwaves * RW) {
		const BUN r1 = r0 + RW < n ? r0 + RW : n;
		const BUN l0 = r0 + (BUN) lane * U;
		oid g[U];
		T x[U];
		constexpr bool VEC_OK = VW == 0 || (U * VW) % 16 == 0;
		if (VEC_OK && vec && l0 + U <= r1) {
			// 16-byte loads (the host checked the alignment)
			if (gids) {
				const uint4 *p = (const uint4 *) (gids + l0);
				uint4 q[U / 2];
#pragma unroll
				for (int u = 0; u < U / 2; u++)
					q[u] = p[u];
				__builtin_memcpy(g, q, sizeof g);
			} else {
#pragma unroll
				for (int u = 0; u < U; u++)
					g[u] = gseq + l0 + u;
			}
			if constexpr (VW > 0 && VEC_OK) {
				constexpr int NQ = U * VW / 16;
				const uint4 *p = (const uint4 *) ((const T *) base + off + l0);
				uint4 q[NQ];
#pragma unroll
				for (int u = 0; u < NQ; u++)
					q[u] = p[u];
				__builtin_memcpy(x, q, sizeof x);
			}
		} else {
			// rows past r1 repeat the range's last row: they extend its run
			// and contribute nothing
#pragma unroll
			for (int u = 0; u < U; u++) {
				const BUN ic = l0 + u < r1 ? l0 + u : r1 - 1;
				g[u] = gids ? gids[ic] : gseq + ic;
				if constexpr (VW > 0)
					x[u] = ((const T *) base)[off + ic];
			}
		}
		// the lane's rows in order: P = its first run, cur = the open run
		GRun P, cur;
		P.clear();
		cur.clear();
		bool single = true;
		const oid gF = g[0];
		oid cg = g[0];
		if (STAGE && stage) {
			// the range's first and last ids: groups strictly between them
			// are complete (or empty) in this range; staged when they fit
			const oid a0 = __shfl(g[0], 0), a1 = __shfl(g[U - 1], 63);
			sbase = a0;
			send = a1 - a0 <= RW ? a1 : a0;
			// empty groups keep the identity (also when nothing writes them)
			for (BUN k = lane; k < RW; k += 64) {
				s_lo[k] = 0;
				s_hi[k] = 0;
				s_c[k] = 0;
			}
			__builtin_amdgcn_wave_barrier();
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			if (g[u] != cg) {
				if (single)
					P = cur;
				else if (valid(cg))
					flush(false, cg - gmin, cur);     // a run inside the lane
				if (g[u] > cg + 1)
					gap(cg, g[u]);
				single = false;
				cur.clear();
				cg = g[u];
			}
			const BUN i = l0 + u;
			if (i < r1 && valid(g[u])) {
				bool isnil = false;
				hge v = 0;
				if constexpr (VW > 0) {
					isnil = is_nil(x[u]);
					v = (hge) x[u];
				}
				if (!isnil) {
					cur.s += (uhge) v;
					cur.c++;
					if (POS)
						cur.fv = i < cur.fv ? i : cur.fv;
					if (MM) {
						cur.mn = (long long) v < cur.mn ? (long long) v : cur.mn;
						cur.mx = (long long) v > cur.mx ? (long long) v : cur.mx;
					}
					const unsigned long long ab = absbits(v);
					mxa = ab > mxa ? ab : mxa;
				} else {
					if (count_all)
						cur.c++;
					if (POS)
						cur.ln = i + 1 > cur.ln ? i + 1 : cur.ln;
				}
			}
		}
		const oid gL = cg;
		// the lanes' boundary runs
		const oid gLprev = __shfl_up(gL, 1), gFnext = __shfl_down(gF, 1);
		const bool connects = lane > 0 && gLprev == gF;           // my first run began to my left
		const bool nextconn = lane < 63 && gFnext == gL;         // my last run goes on to my right
		const unsigned long long chain = __ballot(single && (lane == 0 || connects));
		const unsigned long long below = (1ull << lane) - 1;
		// my first run is the range's first (it may have begun in the previous range)
		const bool rfirst = lane == 0 || (connects && (~chain & below) == 0);
		// segmented inclusive scan of the last runs: a lane that is one run
		// and continues its left neighbour's run extends it
		GRun t = cur;
		bool f = !(single && connects);
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const GRun o = t.shfl_up<MM, POS>(d);
			const bool tf = __shfl_up((int) f, d) != 0;
			if (lane >= d) {
				if (!f)
					t.add<MM, POS>(o);
				f |= tf;
			}
		}
		// t = the run ending at my last row, from its start
		const GRun cin = t.shfl_up<MM, POS>(1);
		if (gapinit) {
			if (lane < 63 && gFnext > gL + 1)
				gap(gL, gFnext);
			if (lane == 0) {
				if (r0 == 0) {
					if (gF > gmin && gmin + ngrp > gmin)
						for (oid h = gmin; h < gF && h < gmin + ngrp; h++) {
							GRun e;
							e.clear();
							flush(false, h - gmin, e);
						}
				} else {
					const oid gp = gids ? gids[r0 - 1] : gseq + r0 - 1;
					if (gF > gp + 1)
						gap(gp, gF);
				}
			}
			if (lane == 63 && r1 == n)
				gap(gL, gmin + ngrp);
		}
		if (edges) {
			// the range's shared groups: slot 0 = its first row's group when
			// that group ends inside the range, slot 1 = its last row's group
			bool e0 = false;
			GRun r0run;
			if (!single) {
				if (connects)
					P.add<MM, POS>(cin);
				if (valid(gF)) {
					if (rfirst) {
						e0 = true;
						r0run = P;
					} else {
						flush(false, gF - gmin, P);
					}
				}
				if (!nextconn && valid(gL) && lane < 63)
					flush(false, gL - gmin, cur);
			} else if (!nextconn && valid(gL) && lane < 63) {
				if (rfirst) {
					e0 = true;
					r0run = t;
				} else {
					flush(false, gL - gmin, t);
				}
			}
			const BUN rk = r0 / RW;
			const unsigned long long b0 = __ballot(e0);
			if (e0 || (b0 == 0 && lane == 0)) {
				if (!e0)
					r0run.clear();
				edges[2 * rk] = GEdge{gF, (unsigned long long) r0run.s, (unsigned long long) (r0run.s >> 64),
						      r0run.c};
			}
			if (lane == 63) {
				GRun r1run = single ? t : cur;
				if (!valid(gL))
					r1run.clear();
				edges[2 * rk + 1] = GEdge{gL, (unsigned long long) r1run.s, (unsigned long long) (r1run.s >> 64),
							  r1run.c};
			}
		} else if (!single) {
			if (connects)
				P.add<MM, POS>(cin);
			if (valid(gF))
				flush(rfirst, gF - gmin, P);
			if (!nextconn && valid(gL))
				flush(lane == 63, gL - gmin, cur);
		} else if (!nextconn && valid(gL)) {
			flush(lane == 63 || rfirst, gL - gmin, t);
		}
		if (STAGE && stage && send > sbase + 1) {
			// the staged groups (sbase, send) out as contiguous runs
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			const oid lo = sbase + 1 > gmin ? sbase + 1 : gmin;
			const oid hi = send < gmin + ngrp ? send : gmin + ngrp;
			for (oid h = lo + lane; h < hi; h += 64) {
				const BUN k = h - sbase, gi = h - gmin;
				if (so.on) {
					sof |= sout_put(so, gi, ((uhge) s_hi[k] << 64) | s_lo[k], s_c[k]);
					continue;
				}
				if (do_sum)
					*(ulonglong2 *) &acc.sum[2 * gi] = ulonglong2{s_lo[k], s_hi[k]};
				acc.cnt[gi] = s_c[k];
			}
			__builtin_amdgcn_wave_barrier();
		}
	}
	for (int o = 32; o > 0; o >>= 1) {
		const unsigned long long t = __shfl_xor(mxa, o);
		mxa = t > mxa ? t : mxa;
	}
	if (lane == 0 && mxa)
		publish_max(maxabs, mxa);
	if (so.on) {
		for (int o = 32; o > 0; o >>= 1)
			sof |= __shfl_xor(sof, o);
		if (lane == 0 && sof)
			publish_or(so.flags, sof);
	}
}

// the shared groups' partials summed (a group's entries are consecutive)
__global__ __launch_bounds__(256) void
k_gedge_sum(const GEdge *e, BUN ne, oid gmin, BUN ngrp, SOut so)
{
	uint32_t f = 0;
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < ne; j += (BUN) gridDim.x * blockDim.x) {
		const oid g = e[j].g;
		if ((j > 0 && e[j - 1].g == g) || g < gmin || g - gmin >= ngrp)
			continue;
		uhge s = 0;
		unsigned long long c = 0;
		for (BUN q = j; q < ne && e[q].g == g; q++) {
			s += ((uhge) e[q].hi << 64) | e[q].lo;
			c += e[q].c;
		}
		f |= sout_put(so, g - gmin, s, c);
	}
	for (int o = 32; o > 0; o >>= 1)
		f |= __shfl_xor(f, o);
	if (__lane_id() == 0 && f)
		publish_or(so.flags, f);
}

__global__ void
k_minmax_oid(const oid *g, BUN n, unsigned long long *out)
{
	unsigned long long mn = ~0ull, mx = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		oid x = g[i];
		if (x == MGDK_OID_NIL)
			continue;
		mn = x < mn ? x : mn;
		mx = x > mx ? x : mx;
	}
	mn = block_reduce(mn, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	mx = block_reduce(mx, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	if (threadIdx.x == 0) {
		atomicMin(&out[0], mn);
		atomicMax(&out[1], mx);
	}
}

// BATgroupaggrinit (gdk/gdk_aggr.c:65-146)
// b's values at a materialised candidate list, as a new BAT whose head
// starts at the first candidate (so it is aligned with g, which has one
// group id per candidate); kept alive in a small per-thread ring (nested
// aggregate calls each take their own slot)
static thread_local mgdk_bat *cv_ring[4];
static thread_local unsigned cv_next;

mgdk_bat *
cand_values(mgdk_bat *b, const Cand &ci)
{
	mgdk_bat *l = newbat(0, MGDK_oid, ci.n);
	if (l == nullptr)
		return nullptr;
	if (!hip_ok(hipMemcpyAsync(l->theap, ci.oids, ci.n * sizeof(oid), hipMemcpyDeviceToDevice, stream()), "memcpy")) {
		mgdk_BBPunfix(l);
		return nullptr;
	}
	l->count = ci.n;
	l->tsorted = l->tkey = l->tnonil = 1;
	l->trevsorted = ci.n <= 1;
	mgdk_bat *v = mgdk_BATproject(l, b);
	mgdk_BBPunfix(l);
	if (v == nullptr)
		return nullptr;
	v->hseqbase = ci.first;
	mgdk_BBPunfix(cv_ring[cv_next & 3]);
	cv_ring[cv_next++ & 3] = v;
	return v;
}

// BATgroupaggrinit (gdk/gdk_aggr.c:65); a materialised candidate list is
// resolved once into a gathered value column (*bp is replaced by it)
int
aggr_init(AggrInit *a, mgdk_bat **bp, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s)
{
	*a = AggrInit{};
	mgdk_bat *b = *bp;
	if (cand_init(&a->ci, b, s) < 0)
		return -1;
	if (g == nullptr) {
		seterr("b and g must be aligned\n");
		return -1;
	}
	if (a->ci.n != g->count || (a->ci.n != 0 && a->ci.first != g->hseqbase)) {
		seterr("b with s and g must be aligned\n");
		return -1;
	}
	if (!a->ci.dense) {
		mgdk_bat *v = cand_values(b, a->ci);
		if (v == nullptr || cand_init(&a->ci, v, nullptr) < 0)
			return -1;
		*bp = v;
	}
	a->gids = g->ttype == MGDK_void ? nullptr : (const oid *) g->theap;
	a->g8 = a->gids ? img8_get(g) : nullptr;
	a->gseq = g->tseqbase;
	a->gsorted = g->ttype == MGDK_void || g->tsorted;
	a->gkey = g->ttype == MGDK_void ? g->tseqbase != MGDK_OID_NIL : (g->tkey && g->tsorted);
	if (e) {
		a->ngrp = e->count;
		a->min = e->hseqbase;
		a->max = e->hseqbase + a->ngrp - 1;
		return 0;
	}
	if (a->gids == nullptr) {
		a->min = g->tseqbase;
		a->max = g->tseqbase + g->count - 1;
		a->ngrp = g->count;
		return 0;
	}
	unsigned long long *m = (unsigned long long *) meta_buf();
	unsigned long long init[2] = {~0ull, 0};
	if (!hip_ok(hipMemcpyAsync(m, init, 16, hipMemcpyHostToDevice, stream()), "memcpy"))
		return -1;
	if (g->count)
		hipLaunchKernelGGL(k_minmax_oid, dim3(grid_for(g->count, 2048, 1024)), dim3(256), 0, stream(),
				   a->gids, g->count, m);
	unsigned long long *h = (unsigned long long *) pinned(16);
	if (!hip_ok(hipMemcpyAsync(h, m, 16, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return -1;
	a->min = h[0];
	a->max = h[1];
	a->ngrp = (h[0] == ~0ull || h[1] < h[0]) ? 0 : h[1] - h[0] + 1;
	if (a->ngrp == 0)
		a->min = 0;
	return 0;
}

// accumulator block of run_gaggr: sums and counts 0, first positions ~0,
// last-nil 0, min / max at their identities, the magnitude class 0
// (only the quantities `what` asks for: with as many groups as rows / 4 the
// block is as large as the column)
__global__ __launch_bounds__(256) void
k_gacc_init(GAcc acc, BUN ng, unsigned long long *maxabs, int what)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ng; k += (BUN) gridDim.x * blockDim.x) {
		if (what & AGG_SUM) {
			acc.sum[2 * k] = 0;
			acc.sum[2 * k + 1] = 0;
		}
		acc.cnt[k] = 0;
		if (what & AGG_POS) {
			acc.firstval[k] = ~0ull;
			acc.lastnil[k] = 0;
		}
		if (what & AGG_MINMAX) {
			acc.mn[k] = INT64_MAX;
			acc.mx[k] = INT64_MIN;
		}
	}
	if (blockIdx.x == 0 && threadIdx.x == 0)
		*maxabs = 0;
}

struct GRes {
	std::vector<hge> sum;
	std::vector<unsigned long long> cnt, firstval, lastnil;
	std::vector<long long> mn, mx;
	unsigned long long maxabs;
};

// the grouped accumulators on the device (the thread's scratch buffer:
// valid until its next scratch() user), no read-back
int
gaggr_device(const AggrInit &a, mgdk_bat *b, int what, bool count_all, GAcc &acc, unsigned long long *&maxabs_out,
	     bool full_init = false)
{
	const BUN ng = a.ngrp;
	size_t bytes = ng * (16 + 8 * 5) + 64;
	char *d = (char *) scratch(bytes);
	if (d == nullptr)
		return -1;
	acc.sum = (unsigned long long *) d;
	acc.cnt = acc.sum + 2 * ng;
	acc.firstval = acc.cnt + ng;
	acc.lastnil = acc.firstval + ng;
	acc.mn = (long long *) (acc.lastnil + ng);
	acc.mx = acc.mn + ng;
	unsigned long long *maxabs = (unsigned long long *) (acc.mx + ng);
	hipStream_t st = stream();
	// one init launch, one read-back of the whole accumulator block and one
	// wait: the operator's host round trips, not its kernels, dominated
	// small-group aggregates
	// the host read-back (run_gaggr) copies the whole block: all of it
	// initialised there
	// sorted ids over rows (sums / counts / positions): k_gaggr_sorted
	// initialises the groups itself (gaps) and k_gacc_edges the ones it adds
	// to atomically, so the accumulators are written once instead of twice
	const bool sorted_path = a.ci.n && ng > 8 && a.gsorted && (what & ~(AGG_SUM | AGG_POS | AGG_MINMAX)) == 0;
	static const bool gapinit_on = getenv("MGDK_GAGGR_GAPINIT") ? atoi(getenv("MGDK_GAGGR_GAPINIT")) != 0 : true;
	const bool gapinit = gapinit_on && sorted_path && !full_init && !(what & AGG_MINMAX);
	if (gapinit) {
		if (!hip_ok(hipMemsetAsync(maxabs, 0, 8, st), "memset"))
			return -1;
		const BUN rw = 64 * ((what & (AGG_POS | AGG_MINMAX)) ? GS_U : GS_UA);
		hipLaunchKernelGGL(k_gacc_edges, dim3(grid_for((a.ci.n + rw - 1) / rw, 256, 8192)), dim3(256),
				   0, st, a.gids, a.gseq, a.min, ng, a.ci.n, rw, acc, what);
	} else {
		hipLaunchKernelGGL(k_gacc_init, dim3(grid_for(ng + 1, 1024, 8192)), dim3(256), 0, st, acc, ng, maxabs,
				   full_init ? (AGG_SUM | AGG_POS | AGG_MINMAX) : what);
	}
	const oid off = a.ci.seq - b->hseqbase;
	dim3 g(grid_for(a.ci.n, 256 * 8, 256 * 16)), blk(256);
	// COUNT(*) over few groups needs no values (k_gaggr_k's base == NULL)
	const void *vbase = (what == 0 && count_all && ng <= 8) ? nullptr : b->theap;
	if (a.ci.n) {
#define GK4(K_, MM_, POS_, VW_) do { \
		kk = K_; \
		if (a.g8 && a.min < 256 && a.min + ng <= 256) \
			hipLaunchKernelGGL((k_gaggr_k<K_, MM_, POS_, VW_, uint8_t>), g, blk, 0, st, vbase, b->twidth, off, a.g8, a.gseq, a.min, ng, a.ci.n, what, count_all, parts.as<GPart>()); \
		else \
			hipLaunchKernelGGL((k_gaggr_k<K_, MM_, POS_, VW_, oid>), g, blk, 0, st, vbase, b->twidth, off, a.gids, a.gseq, a.min, ng, a.ci.n, what, count_all, parts.as<GPart>()); } while (0)
#define GK3(K_, MM_, POS_) do { switch (vbase ? b->twidth : 0) { \
		case 0: GK4(K_, MM_, POS_, 0); break; \
		case 1: GK4(K_, MM_, POS_, 1); break; \
		case 2: GK4(K_, MM_, POS_, 2); break; \
		case 4: GK4(K_, MM_, POS_, 4); break; \
		case 8: GK4(K_, MM_, POS_, 8); break; \
		default: GK4(K_, MM_, POS_, 16); break; } } while (0)
#define GK(K_) do { if (what & AGG_MINMAX) GK3(K_, true, true); \
		else if (what & AGG_POS) GK3(K_, false, true); \
		else GK3(K_, false, false); } while (0)
		if (ng <= 8) {
			const BUN nw = (BUN) g.x * 4;
			DevBuf parts(nw * 8 * sizeof(GPart));
			if (parts.p == nullptr)
				return -1;
			int kk = 0;
			if (ng <= 4)
				GK(4);
			else
				GK(8);
			hipLaunchKernelGGL(k_gaggr_fin, dim3(kk), dim3(256), 0, st, parts.as<GPart>(), nw, kk, ng, acc, maxabs);
		}
		else if (a.gsorted && (what & ~(AGG_SUM | AGG_POS | AGG_MINMAX)) == 0) {
			// groups are runs of rows: segmented reduction (k_gaggr_sorted)
			// (k_gacc_edges above uses the same rows per range)
			const bool plain = (what & (AGG_POS | AGG_MINMAX)) == 0;
			const BUN rw = 64 * (plain ? GS_UA : GS_U);
			const BUN nw = (a.ci.n + rw - 1) / rw;
			static const bool stage_on = getenv("MGDK_GS_STAGE") ? atoi(getenv("MGDK_GS_STAGE")) != 0 : true;
			const bool stage = plain && stage_on;
			const size_t lds = stage ? 4 * 3 * rw * 8 : 0;
			const dim3 gs(grid_for(nw, 4, 65535u * 16u));
			const bool sum = (what & AGG_SUM) != 0;
			const void *vb = (what == 0 && count_all) ? nullptr : b->theap;
			// 16-byte loads when a lane's rows start 16-byte aligned
			const bool vec = ((uintptr_t) a.gids & 15) == 0 &&
				(!vb || (((uintptr_t) vb + (uintptr_t) off * b->twidth) & 15) == 0);
#define GS3(VW_, MM_, POS_) do { if (!(MM_) && !(POS_)) \
				hipLaunchKernelGGL((k_gaggr_sorted<VW_, MM_, POS_, GS_UA>), gs, blk, lds, st, vb, off, a.gids, a.gseq, a.min, ng, a.ci.n, sum, count_all, vec, gapinit, stage, acc, maxabs, SOut{}, nullptr); \
			else \
				hipLaunchKernelGGL((k_gaggr_sorted<VW_, MM_, POS_, GS_U>), gs, blk, 0, st, vb, off, a.gids, a.gseq, a.min, ng, a.ci.n, sum, count_all, vec, gapinit, false, acc, maxabs, SOut{}, nullptr); } while (0)
#define GS2(VW_) do { if (what & AGG_MINMAX) GS3(VW_, true, false); \
			else if (what & AGG_POS) GS3(VW_, false, true); \
			else GS3(VW_, false, false); } while (0)
			switch (vb ? b->twidth : 0) {
			case 0: GS2(0); break;
			case 1: GS2(1); break;
			case 2: GS2(2); break;
			case 4: GS2(4); break;
			case 8: GS2(8); break;
			default: GS2(16); break;
			}
#undef GS2
#undef GS3
		} else
			hipLaunchKernelGGL((k_gaggr<0>), g, blk, 0, st, b->theap, b->twidth, off, a.gids, a.gseq, a.min, ng, a.ci.n, what, count_all, acc, maxabs);
	}
	maxabs_out = maxabs;
	return 0;
}

int
run_gaggr(const AggrInit &a, mgdk_bat *b, int what, bool count_all, GRes &r)
{
	const BUN ng = a.ngrp;
	GAcc acc;
	unsigned long long *maxabs;
	if (gaggr_device(a, b, what, count_all, acc, maxabs, true) < 0)
		return -1;
	const char *d = (const char *) acc.sum;
	hipStream_t st = stream();
	r.sum.resize(ng);
	r.cnt.resize(ng);
	r.firstval.resize(ng);
	r.lastnil.resize(ng);
	r.mn.resize(ng);
	r.mx.resize(ng);
	const size_t nblk = (size_t) ng * (16 + 8 * 5) + 8;
	unsigned long long *hb = (unsigned long long *) pinned(nblk);
	if (hb == nullptr || !hip_ok(hipMemcpyAsync(hb, d, nblk, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	const unsigned long long *hs = hb, *hc = hb + 2 * ng, *hf = hc + ng, *hl = hf + ng;
	const long long *hmn = (const long long *) (hl + ng), *hmx = hmn + ng;
	for (BUN k = 0; k < ng; k++) {
		r.sum[k] = (hge) (((uhge) hs[2 * k + 1] << 64) | hs[2 * k]);
		r.cnt[k] = hc[k];
		r.firstval[k] = hf[k];
		r.lastnil[k] = hl[k];
		r.mn[k] = hmn[k];
		r.mx[k] = hmx[k];
	}
	r.maxabs = hb[7 * ng];
	return 0;
}

// ---- results finished on the device (no per-group host loop: a
// high-cardinality GROUP BY has as many groups as rows / 4) --------------
__device__ __forceinline__ void
put_res_d(void *base, int bt, BUN k, hge v, bool nil)
{
	switch (bt) {
	case MGDK_bte: ((int8_t *) base)[k] = nil ? INT8_MIN : (int8_t) v; break;
	case MGDK_sht: ((int16_t *) base)[k] = nil ? INT16_MIN : (int16_t) v; break;
	case MGDK_int: ((int32_t *) base)[k] = nil ? INT32_MIN : (int32_t) v; break;
	case MGDK_lng: ((int64_t *) base)[k] = nil ? INT64_MIN : (int64_t) v; break;
	case MGDK_oid: ((uint64_t *) base)[k] = nil ? MGDK_OID_NIL : (uint64_t) v; break;
	default: ((hge *) base)[k] = nil ? NilOf<hge>::v() : v; break;
	}
}

__device__ __forceinline__ hge
acc_sum(const GAcc &acc, BUN k)
{
	return (hge) (((uhge) acc.sum[2 * k + 1] << 64) | acc.sum[2 * k]);
}

__device__ __forceinline__ void
or_flags(uint32_t *flags, uint32_t f)
{
	f = block_reduce(f, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, f);
}

// BATgroupsum per group (gdk_aggr.c:429-705): nil without a value, and
// without skip_nils when a nil came after the first value (one group: any
// nil); flags bit 0: a group's sum -- itself a prefix -- beyond the type's
// range (overflow), bit 1: a nil result
__global__ __launch_bounds__(256) void
k_gsum_out(GAcc acc, BUN ng, bool empty, int bt, bool skip_nils, hge max, void *out, uint32_t *flags)
{
	uint32_t f = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ng; k += (BUN) gridDim.x * blockDim.x) {
		const hge sv = acc_sum(acc, k);
		const unsigned long long c = acc.cnt[k];
		if (sv > max || sv < -max)
			f |= 1;
		bool nil;
		if (empty || c == 0)
			nil = true;
		else if (skip_nils)
			nil = false;
		else if (ng == 1)
			nil = acc.lastnil[k] != 0;
		else
			nil = acc.lastnil[k] > acc.firstval[k] + 1;
		put_res_d(out, bt, k, nil ? 0 : sv, nil);
		f |= nil ? 2u : 0u;
	}
	or_flags(flags, f);
}

__global__ __launch_bounds__(256) void
k_gcount_out(GAcc acc, BUN ng, long long *out)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ng; k += (BUN) gridDim.x * blockDim.x)
		out[k] = (long long) acc.cnt[k];
}

// BATgroupavg3 per group (gdk_aggr.c:1996-2110, rounding :2070-2095)
// flags bit 1: a nil average, bit 2: a nil remainder / count
__global__ __launch_bounds__(256) void
k_gavg3_out(GAcc acc, BUN ng, bool empty, int bt, bool skip_nils, void *avg, long long *rem, long long *cnt,
	    uint32_t *flags)
{
	uint32_t f = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ng; k += (BUN) gridDim.x * blockDim.x) {
		const unsigned long long n = empty ? 0 : acc.cnt[k];
		if (!empty && !skip_nils && acc.lastnil[k] != 0) {
			put_res_d(avg, bt, k, 0, true);
			rem[k] = INT64_MIN;
			cnt[k] = INT64_MIN;
			f |= 6;
			continue;
		}
		cnt[k] = (long long) n;
		if (n == 0) {
			put_res_d(avg, bt, k, 0, true);
			rem[k] = empty ? INT64_MIN : 0;
			f |= 2;
			continue;
		}
		hge q = acc_sum(acc, k) / (hge) n, m = acc_sum(acc, k) % (hge) n;
		if (m < 0) {
			q -= 1;
			m += (hge) n;
		}
		if (m > 0) {
			if (q < 0) {
				if (2 * m > (hge) n) { q++; m -= (hge) n; }
			} else if (2 * m >= (hge) n) {
				q++;
				m -= (hge) n;
			}
		}
		put_res_d(avg, bt, k, q, false);
		rem[k] = (long long) m;
	}
	or_flags(flags, f);
}

// BATgroupavg of integers (AGGR_AVG, gdk_aggr.c:1717): floor average + its
// remainder as a dbl; flags bit 0: an hge group sum may exceed the 128-bit
// accumulator, bit 1: a nil result
__global__ __launch_bounds__(256) void
k_gavg_out(GAcc acc, BUN ng, bool skip_nils, bool hgein, const unsigned long long *maxabs, double fac,
	   double *out, long long *cnt, uint32_t *flags)
{
	uint32_t f = 0;
	const unsigned long long cls = *maxabs;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ng; k += (BUN) gridDim.x * blockDim.x) {
		const unsigned long long n = acc.cnt[k];
		if (n == 0 || (!skip_nils && acc.lastnil[k] != 0)) {
			out[k] = __builtin_nan("");
			cnt[k] = 0;
			f |= 2;
			continue;
		}
		if (hgein) {
			// mag_bound(cls) * n >= 2^127, in exact integers
			const bool big = (cls >> 63) ? (uhge) ((cls & ~(1ull << 63)) + 1) * n >= ((uhge) 1 << 63)
						     : (uhge) (cls + 1) * n >= ((uhge) 1 << 126);
			f |= big ? 1u : 0u;
		}
		hge q = acc_sum(acc, k) / (hge) n, m = acc_sum(acc, k) % (hge) n;
		if (m < 0) {
			q -= 1;
			m += (hge) n;
		}
		double d = hge_to_dbl(q) + (double) (long long) m / (double) (long long) n;
		if (fac != 1.0)
			d /= fac;
		out[k] = d;
		cnt[k] = (long long) n;
	}
	or_flags(flags, f);
}

// BATgroupavg3combine's result per group from the grouped exact totals and
// counts (gdk_aggr.c:2702-2716); nall / nnon: rows and non-nil rows per
// group (NULL: equal); flags bit 1: a nil result
__global__ __launch_bounds__(256) void
k_avg3c_out(BUN ng, const hge *S, const hge *C, const long long *nall, const long long *nnon, int bt, void *out,
	    uint32_t *flags)
{
	uint32_t f = 0;
	const hge NIL = NilOf<hge>::v();
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ng; k += (BUN) gridDim.x * blockDim.x) {
		const hge sv = S[k], cv = C[k];
		if (sv == NIL || cv == NIL || cv == 0 || (nall && nall[k] != nnon[k])) {
			put_res_d(out, bt, k, 0, true);
			f |= 2;
			continue;
		}
		hge q = sv / cv, r = sv % cv;
		if (r < 0) {
			q -= 1;
			r += cv;
		}
		if (r > 0 && (q < 0 ? 2 * r > cv : 2 * r >= cv))
			q += 1;
		put_res_d(out, bt, k, q, false);
	}
	or_flags(flags, f);
}

// groups of BATgroupmin / max without a value: no non-nil row and no nil
// row that counts (flags bit 1)
__global__ __launch_bounds__(256) void
k_gminmax_nils(GAcc acc, BUN ng, const unsigned long long *firstnil, uint32_t *flags)
{
	uint32_t f = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ng; k += (BUN) gridDim.x * blockDim.x)
		f |= (acc.cnt[k] == 0 && firstnil[k] == ~0ull) ? 2u : 0u;
	or_flags(flags, f);
}

// read a 4-byte flag word after the stream has drained
bool
read_flags(const void *dev, uint32_t *out)
{
	uint32_t *h = (uint32_t *) pinned(16);
	if (h == nullptr || !hip_ok(hipMemcpyAsync(h, dev, 4, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return false;
	*out = h[0];
	return true;
}

// wait = false: the copy is queued from the pinned arena and the caller
// waits once after its last upload (sync())
mgdk_bat *
upload_new(oid hseq, int tp, const void *host, BUN n, bool wait = true)
{
	mgdk_bat *bn = newbat(hseq, tp, n);
	if (bn == nullptr)
		return nullptr;
	const size_t bytes = n * (size_t) bn->twidth;
	const void *src = bytes ? stage_host(host, bytes) : nullptr;
	if ((bytes && (src == nullptr || !hip_ok(hipMemcpyAsync(bn->theap, src, bytes, hipMemcpyHostToDevice, stream()),
						     "hipMemcpyAsync H2D"))) ||
	    (wait && !sync())) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	bn->count = n;
	return bn;
}

void
put_vec(std::vector<char> &buf, int tp, BUN k, hge v, bool nil)
{
	put_res(buf.data() + k * width_of(tp), tp, v, nil);
}


// ---- BATgroupavg (gdk/gdk_aggr.c:1801) ----------------------------------

// singleton groups: BATconvert(b, s, TYPE_dbl) (gdk_calc_convert.c:1415)
__global__ void
k_to_dbl(const void *base, int tp, int w, oid off, BUN n, double *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		double d;
		if (tp == MGDK_flt) {
			d = (double) ((const float *) base)[off + i];
		} else if (tp == MGDK_dbl) {
			d = ((const double *) base)[off + i];
		} else {
			bool nil;
			const hge v = ldv(base, w, off + i, nil);
			d = nil ? __builtin_nan("") : hge_to_dbl(v);
		}
		out[i] = d;
	}
}

constexpr BUN AVG_LDS_BINS = 8192;

// group key of each candidate row for the stable counting sort: gid - min,
// or ngrp for rows whose group is out of range (sorted behind every group)
__global__ __launch_bounds__(256) void
k_avg_keys(const oid *gids, oid gseq, oid gmin, BUN ngrp, BUN n, uint32_t *key, uint32_t *cnt)
{
	// block-private counts in LDS when the groups fit (AVG_LDS_BINS)
	extern __shared__ uint32_t s_cnt[];
	const bool lds = ngrp < AVG_LDS_BINS;
	if (lds)
		for (BUN k = threadIdx.x; k <= ngrp; k += blockDim.x)
			s_cnt[k] = 0;
	__syncthreads();
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const oid g = gids ? gids[i] : gseq + i;
		const uint32_t k = (g < gmin || g - gmin >= ngrp) ? (uint32_t) ngrp : (uint32_t) (g - gmin);
		key[i] = k;
		atomicAdd(lds ? &s_cnt[k] : &cnt[k], 1u);
	}
	if (lds) {
		__syncthreads();
		for (BUN k = threadIdx.x; k <= ngrp; k += blockDim.x)
			if (s_cnt[k])
				atomicAdd(&cnt[k], s_cnt[k]);
	}
}

// AVERAGE_ITER_FLOAT (gdk_calc_private.h:277-289) is order dependent and
// not associative: one lane replays one group's rows in candidate order
// (perm: rows grouped by the stable sort; NULL with one group: every row,
// range-checked through gids).  Eight values are loaded ahead of the
// dependent divisions.
template <typename T>
__global__ void
k_favg_replay(const T *vals, oid off, const uint32_t *perm, const uint64_t *start, const oid *gids, oid gseq,
	      oid gmin, BUN ngrp, BUN n, bool skip_nils, double fac, double *out, long long *cnt)
{
	const BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= ngrp)
		return;
	const BUN j0 = start ? start[k] : 0, j1 = start ? start[k + 1] : n;
	double a = 0;
	long long c = 0;
	bool nil = false;
	constexpr int U = 8;
	for (BUN j = j0; j < j1 && !nil; j += U) {
		double x[U];
		bool ok[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN jj = j + u;
			ok[u] = jj < j1;
			BUN r = 0;
			if (ok[u]) {
				r = perm ? perm[jj] : jj;
				if (!perm) {
					// (gids NULL, gseq nil: every row is in the one group, BATcalcavg)
					const oid g = gids ? gids[r] : gseq == MGDK_OID_NIL ? gmin : gseq + r;
					ok[u] = g >= gmin && g - gmin < ngrp;
				}
			}
			x[u] = ok[u] ? (double) vals[off + r] : 0.0;
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			if (!ok[u] || nil)
				continue;
			if (__builtin_isnan(x[u])) {
				nil = !skip_nils;
				continue;
			}
			const double nn = (double) ++c;
			if ((a > 0) == (x[u] > 0))
				a += (x[u] - a) / nn;
			else
				a = a - a / nn + x[u] / nn;
		}
	}
	if (nil || c == 0) {
		out[k] = __builtin_nan("");
		cnt[k] = 0;
	} else {
		out[k] = fac != 1.0 ? a / fac : a;
		cnt[k] = c;
	}
}

// The parallel form of one large group (fp_parallel_min): block b runs the
// same recurrence over the rows l, l + 256, ... of its tile per lane, then
// the lanes and blocks are merged in order, (a, c) + (b, d) -> a + (b - a) *
// (d / (c + d)): the weighted mean of the partial means.  Only the rounding
// differs from the sequential fold (DESIGN.md states the bound).
struct FAvg {
	double a;
	double c;
	int nil;
};

__device__ __forceinline__ FAvg
favg_comb(const FAvg &x, const FAvg &y)
{
	FAvg r;
	r.nil = x.nil | y.nil;
	if (x.c == 0) {
		r.a = y.a;
		r.c = y.c;
	} else if (y.c == 0) {
		r.a = x.a;
		r.c = x.c;
	} else {
		r.c = x.c + y.c;
		r.a = x.a + (y.a - x.a) * (y.c / r.c);
	}
	return r;
}

template <typename T>
__global__ __launch_bounds__(256) void
k_favg_par(const T *vals, oid off, const oid *gids, oid gseq, oid gmin, BUN n, BUN tile, bool skip_nils, FAvg *part)
{
	__shared__ FAvg lds[256];
	const BUN b0 = (BUN) blockIdx.x * tile, b1 = min(n, b0 + tile);
	FAvg s{0, 0, 0};
	long long c = 0;
	for (BUN r = b0 + threadIdx.x; r < b1; r += 256) {
		const oid g = gids ? gids[r] : gseq == MGDK_OID_NIL ? gmin : gseq + r;
		if (g != gmin)
			continue;
		const double x = (double) vals[off + r];
		if (__builtin_isnan(x)) {
			s.nil |= !skip_nils;
			continue;
		}
		const double nn = (double) ++c;
		if ((s.a > 0) == (x > 0))
			s.a += (x - s.a) / nn;
		else
			s.a = s.a - s.a / nn + x / nn;
	}
	s.c = (double) c;
	s = block_tree(s, [](const FAvg &x, const FAvg &y) { return favg_comb(x, y); }, lds);
	if (threadIdx.x == 0)
		part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void
k_favg_fin(const FAvg *part, unsigned nb, double fac, double *out, long long *cnt)
{
	__shared__ FAvg lds[256];
	const unsigned per = (nb + 255) / 256, p0 = threadIdx.x * per, p1 = min(nb, p0 + per);
	FAvg s{0, 0, 0};
	for (unsigned p = p0; p < p1; p++)
		s = favg_comb(s, part[p]);
	s = block_tree(s, [](const FAvg &x, const FAvg &y) { return favg_comb(x, y); }, lds);
	if (threadIdx.x != 0)
		return;
	if (s.nil || s.c == 0) {
		out[0] = __builtin_nan("");
		cnt[0] = 0;
	} else {
		out[0] = fac != 1.0 ? s.a / fac : s.a;
		cnt[0] = (long long) s.c;
	}
}

// BATgroupavg3combine terms: t = avg * cnt + rem (the row's exact total),
// c = cnt; both nil where avg is nil.  flags[0]: |avg * cnt| beyond 2^126
template <typename T>
__global__ void
k_avg3c_terms(const T *avg, const long long *rem, const long long *cnt, oid off, BUN n, hge *t, long long *c,
	      uint32_t *flags)
{
	uint32_t big = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const T a = avg[off + i];
		if (a == NilOf<T>::v()) {
			t[i] = NilOf<hge>::v();
			c[i] = INT64_MIN;
			continue;
		}
		const long long k = cnt[off + i], r = rem[off + i];
		const hge ha = (hge) a;
		const uhge ua = (uhge) (ha < 0 ? -ha : ha), uk = (uhge) (k < 0 ? -(hge) k : (hge) k);
		// |avg| * |cnt| < 2^126 so the group totals stay inside hge
		if (ua && uk && ua > ((uhge) 1 << 126) / uk)
			big = 1;
		t[i] = ha * (hge) k + (hge) r;
		c[i] = k;
	}
	if (big)
		atomicOr(flags, 1u);
}

// one row per group, row i in group min + i (g strictly increasing over
// exactly the group range): a grouped aggregate is then element-wise
bool
one_row_groups(const AggrInit &a)
{
	const BUN ng = a.ngrp;
	if (!a.gkey || a.ci.n != ng || ng == 0)
		return false;
	if (a.gids == nullptr)
		return a.gseq == a.min;
	// strictly increasing ids, as many as groups: they are the range iff
	// the first is its start and the last its end
	oid *d = (oid *) meta_buf() + 8;
	oid *h = (oid *) pinned(16);
	hipStream_t st = stream();
	if (!hip_ok(hipMemcpyAsync(d, a.gids, 8, hipMemcpyDeviceToDevice, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(d + 1, a.gids + ng - 1, 8, hipMemcpyDeviceToDevice, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return false;
	return h[0] == a.min && h[1] == a.min + ng - 1;
}

// BATgroupsum with one row per group: each group's sum is its row's value
// (nil: no value, so nil; a value beyond the result type overflows)
template <int VW>
__global__ __launch_bounds__(256) void
k_gsum_rows(const void *base, oid off, BUN n, SOut so)
{
	typedef typename VTy<VW>::T T;
	constexpr int U = 8;
	uint32_t f = 0;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i0 = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += U * stride) {
		T x[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + u * stride;
			x[u] = ((const T *) base)[off + (i < n ? i : n - 1)];
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + u * stride;
			if (i >= n)
				break;
			const bool nil = is_nil(x[u]);
			f |= sout_put(so, i, nil ? 0 : (uhge) (hge) x[u], nil ? 0 : 1);
		}
	}
	for (int o = 32; o > 0; o >>= 1)
		f |= __shfl_xor(f, o);
	if (__lane_id() == 0 && f)
		publish_or(so.flags, f);
}

// BATgroupsum over sorted group ids straight into bn (see SOut); false
// when the case does not apply
bool
gsum_sorted_direct(const AggrInit &a, mgdk_bat *b, mgdk_bat *bn, int tp, bool skip_nils, uint32_t *flags, uint32_t *hf,
		   int *rc)
{
	static const bool on = getenv("MGDK_GSUM_DIRECT") ? atoi(getenv("MGDK_GSUM_DIRECT")) != 0 : true;
	const BUN ng = a.ngrp;
	if (!on || !a.gsorted || ng <= 8 || a.ci.n == 0 || !(skip_nils || b->tnonil))
		return false;
	*rc = -1;
	hipStream_t st = stream();
	if (one_row_groups(a)) {
		SOut so1{bn->theap, basetype(tp), tmax(tp), flags, true};
		const oid off1 = a.ci.seq - b->hseqbase;
		const dim3 g1(grid_for(a.ci.n, 256 * 8, 8192)), b1(256);
		switch (b->twidth) {
		case 1: hipLaunchKernelGGL(k_gsum_rows<1>, g1, b1, 0, st, b->theap, off1, a.ci.n, so1); break;
		case 2: hipLaunchKernelGGL(k_gsum_rows<2>, g1, b1, 0, st, b->theap, off1, a.ci.n, so1); break;
		case 4: hipLaunchKernelGGL(k_gsum_rows<4>, g1, b1, 0, st, b->theap, off1, a.ci.n, so1); break;
		case 8: hipLaunchKernelGGL(k_gsum_rows<8>, g1, b1, 0, st, b->theap, off1, a.ci.n, so1); break;
		default: hipLaunchKernelGGL(k_gsum_rows<16>, g1, b1, 0, st, b->theap, off1, a.ci.n, so1); break;
		}
		if (read_flags(flags, hf))
			*rc = 0;
		return true;
	}
	// 16-byte values: 8 rows per lane (register budget), else 16
	// rows per lane: 8 (2.44 ms for 600M rows / 150M groups; 16: 2.75, 32: 3.05)
	static const int ud = getenv("MGDK_GS_DIRECT_U") ? atoi(getenv("MGDK_GS_DIRECT_U")) : GS_UA;
	const int u = b->twidth >= 16 ? GS_UA : (ud == 8 || ud == 32) ? ud : GS_U;
	const BUN rw = 64 * (BUN) u, nr = (a.ci.n + rw - 1) / rw;
	DevBuf eb(nr * 2 * sizeof(GEdge) + 64), mx(64);
	if (!eb.p || !mx.p || !hip_ok(hipMemsetAsync(mx.p, 0, 8, st), "memset"))
		return true;
	const oid off = a.ci.seq - b->hseqbase;
	const bool vec = ((uintptr_t) a.gids & 15) == 0 && (((uintptr_t) b->theap + (uintptr_t) off * b->twidth) & 15) == 0;
	SOut so{bn->theap, basetype(tp), tmax(tp), flags, true};
	const dim3 gs(grid_for(nr, 4, 65535u * 16u)), blk(256);
	GAcc acc{};
	GEdge *e = eb.as<GEdge>();
	unsigned long long *m = mx.as<unsigned long long>();
	// results of 8 bytes or more stored from the lanes that finish the
	// groups measured faster than staged in LDS (2.80 vs 3.07 ms for 600M
	// rows at 16 rows per lane): no LDS, full occupancy
#define GSD_U(VW_, U_) hipLaunchKernelGGL((k_gaggr_sorted<VW_, false, false, U_>), gs, blk, 0, st, b->theap, off, a.gids, a.gseq, a.min, ng, a.ci.n, true, false, vec, true, false, acc, m, so, e)
#define GSD(VW_) do { if (VW_ >= 16 || u == GS_UA) GSD_U(VW_, GS_UA); else if (u == 32) GSD_U(VW_, 32); else GSD_U(VW_, GS_U); } while (0)
	switch (b->twidth) {
	case 1: GSD(1); break;
	case 2: GSD(2); break;
	case 4: GSD(4); break;
	case 8: GSD(8); break;
	default: GSD(16); break;
	}
#undef GSD
#undef GSD_U
	hipLaunchKernelGGL(k_gedge_sum, dim3(grid_for(2 * nr, 1024, 4096)), blk, 0, st, e, 2 * nr, a.min, ng, so);
	// the flags read waits for the stream: eb goes back to the shared cache
	// only after the kernels are done
	if (read_flags(flags, hf))
		*rc = 0;
	return true;
}

}  // namespace

namespace mgdk {

int
group_init(AggrInit *a, mgdk_bat **bp, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s)
{
	return aggr_init(a, bp, g, e, s);
}

GroupRows::GroupRows(BUN n, BUN ng)
	: key(n * 4 + 4), key2(n * 4 + 4), v0(n * 4 + 4), v1(n * 4 + 4), cnt((ng + 1) * 4), start((ng + 1) * 8)
{
}

bool
GroupRows::ok() const
{
	return key.p && key2.p && v0.p && v1.p && cnt.p && start.p;
}

// a stable counting sort of the candidate rows by group (k_avg_keys' keys,
// the exclusive scan of the group sizes, LSD radix passes over the keys)
int
group_rows(const AggrInit &a, GroupRows &gr)
{
	const BUN ng = a.ngrp;
	gr.perm = nullptr;
	gr.start_p = nullptr;
	if (a.ci.n >= 0xffffffffull || ng >= 0xffffffffull) {
		seterr("42000!more than 2^32-1 rows on the device path\n");
		return -1;
	}
	if (ng <= 1)
		return 0;
	hipStream_t st = stream();
	if (!hip_ok(hipMemsetAsync(gr.cnt.p, 0, (ng + 1) * 4, st), "memset"))
		return -1;
	hipLaunchKernelGGL(k_avg_keys, dim3(grid_for(a.ci.n, 2048, 1024)), dim3(256),
			   ng < AVG_LDS_BINS ? (ng + 1) * 4 : 0, st, a.gids, a.gseq, a.min, ng, a.ci.n,
			   gr.key.as<uint32_t>(), gr.cnt.as<uint32_t>());
	int bits = 0;
	while (bits < 32 && (ng >> bits))
		bits++;
	uint32_t *pm = nullptr;
	if (exclusive_scan(gr.cnt.as<uint32_t>(), gr.start.as<uint64_t>(), ng + 1, nullptr) != 0 ||
	    radix_sort_positions32(gr.key.as<uint32_t>(), gr.v0.as<uint32_t>(), gr.key2.as<uint32_t>(),
				   gr.v1.as<uint32_t>(), a.ci.n, bits, &pm) != 0)
		return -1;
	gr.perm = pm;
	gr.start_p = gr.start.as<uint64_t>();
	return 0;
}

mgdk_bat *
cand_values_at(mgdk_bat *b, const Cand &ci)
{
	return cand_values(b, ci);
}

}  // namespace mgdk

extern "C" {

// BATgroupsum (gdk/gdk_aggr.c:900)
mgdk_bat *
mgdk_BATgroupsum(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	if (b != nullptr && (b->ttype == MGDK_flt || b->ttype == MGDK_dbl)) {
		// dofsum with groups (gdk_aggr.c:183), exact per group (fsum.hip)
		ProfScope prof("groupsum");
		AggrInit a;
		if (aggr_init(&a, &b, g, e, s) < 0)
			return nullptr;
		const BUN ng = a.ngrp;
		std::vector<char> out(ng * 8 + 16);
		bool nils = false;
		if (ng && mgdk_fgroupsum(b, a.ci, a.gids, a.gseq, a.min, ng, skip_nils, tp, out.data(), &nils) < 0)
			return nullptr;
		mgdk_bat *bn = upload_new(ng ? a.min : 0, tp, out.data(), ng);
		if (bn) {
			bn->tkey = bn->tsorted = bn->trevsorted = ng <= 1;
			bn->tnil = nils;
			bn->tnonil = !nils;
		}
		return bn;
	}
	if (b == nullptr || !int_type(b->ttype) || !int_type(tp)) {
		seterr("type combination (sum(%s)->%s) not supported.\n", b ? atomname(b->ttype) : "?", atomname(tp));
		return nullptr;
	}
	ProfScope prof("groupsum");
	AggrInit a;
	if (aggr_init(&a, &b, g, e, s) < 0)
		return nullptr;
	const BUN ng = a.ngrp;
	mgdk_bat *bn = newbat(ng ? a.min : 0, tp, ng);
	DevBuf fl(16);
	if (bn == nullptr || fl.p == nullptr || !hip_ok(hipMemsetAsync(fl.p, 0, 16, stream()), "memset")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	uint32_t hf = 0;
	if (ng) {
		int rc = 0;
		bool read = false;
		if (gsum_sorted_direct(a, b, bn, tp, skip_nils, fl.as<uint32_t>(), &hf, &rc)) {
			if (rc < 0) {
				mgdk_BBPunfix(bn);
				return nullptr;
			}
			read = true;
		} else {
			GAcc acc;
			unsigned long long *mx;
			if (gaggr_device(a, b, AGG_SUM | (skip_nils ? 0 : AGG_POS), false, acc, mx) < 0) {
				mgdk_BBPunfix(bn);
				return nullptr;
			}
			hipLaunchKernelGGL(k_gsum_out, dim3(grid_for(ng, 1024, 8192)), dim3(256), 0, stream(), acc, ng,
					   a.ci.n == 0, basetype(tp), skip_nils, tmax(tp), bn->theap, fl.as<uint32_t>());
		}
		if (!read && !read_flags(fl.p, &hf)) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		if (hf & 1) {
			// a prefix of a group could exceed the range only if its final sum
			// does (the final sum is the last prefix)
			seterr("22003!overflow in sum aggregate.\n");
			mgdk_BBPunfix(bn);
			return nullptr;
		}
	}
	bn->count = ng;
	bn->tkey = bn->tsorted = bn->trevsorted = ng <= 1;
	bn->tnil = (hf & 2) != 0;
	bn->tnonil = !bn->tnil;
	return bn;
}

// BATgroupcount (gdk/gdk_aggr.c:3069)
mgdk_bat *
mgdk_BATgroupcount(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	(void) tp;
	if (b == nullptr || !(int_type(b->ttype) || b->ttype == MGDK_oid || b->ttype == MGDK_str)) {
		seterr("42000!BATgroupcount: type not supported on the device path");
		return nullptr;
	}
	ProfScope prof("groupcount");
	AggrInit a;
	if (aggr_init(&a, &b, g, e, s) < 0)
		return nullptr;
	const BUN ng = a.ngrp;
	mgdk_bat *bn = newbat(ng ? a.min : 0, MGDK_lng, ng);
	if (bn == nullptr)
		return nullptr;
	if (ng) {
		// str offsets are never nil in our heaps; oid via lng width
		bool all = !skip_nils || b->tnonil || b->ttype == MGDK_str;
		GAcc acc;
		unsigned long long *mx;
		if (gaggr_device(a, b, 0, all, acc, mx) < 0) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		hipLaunchKernelGGL(k_gcount_out, dim3(grid_for(ng, 1024, 8192)), dim3(256), 0, stream(), acc, ng,
				   (long long *) bn->theap);
		if (!sync()) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
	}
	bn->count = ng;
	{
		// gdk_aggr.c:3105-3106 (empty: BATconstant of 0), :3185-3190
		bn->tnonil = 1;
		bn->tnil = 0;
		bn->tkey = ng <= 1;
		bn->tsorted = bn->trevsorted = ng <= 1 || a.ci.n == 0;
	}
	return bn;
}

// BATgroupavg (gdk/gdk_aggr.c:1801-1984): trivial cases :1834-1873,
// integers AGGR_AVG (:1717) as the exact floor average and remainder of the
// group's 128-bit sum, flt/dbl AGGR_AVG_FLOAT (:1753) replayed per group
// BATcalcavg (gdk/gdk_aggr.c:2987): the average of b[s] without nils and
// their number.  Integers: the exact sum (the device's 128-bit reduction)
// over the count, (dbl) sum / n as AVERAGE_TYPE_LNG_HGE computes it while the
// sum fits (:2905-2924); an hge column whose sum leaves 128 bits -- where
// the reference switches to its remainder recurrence (:2925-2958) -- is
// refused.  flt / dbl: AVERAGE_FLOATTYPE's running mean (:2970-2984),
// replayed in candidate order (the parallel form from fp_parallel_min rows).
// scale: the result divided by 10^scale (:3036-3037).
int
mgdk_BATcalcavg(mgdk_bat *b, mgdk_bat *s, double *avg, mgdk_BUN *vals, int scale)
{
	const double nil = __builtin_nan("");
	if (avg)
		*avg = nil;
	if (b == nullptr || avg == nullptr) {
		seterr("BATcalcavg: NULL argument");
		return -1;
	}
	const int bt = b->ttype;
	if (!(int_type(bt) && bt != MGDK_oid) && bt != MGDK_flt && bt != MGDK_dbl) {
		seterr("average of type %s unsupported.\n", atomname(bt));
		return -1;
	}
	ProfScope prof("calcavg");
	hipStream_t st = stream();
	double a = nil;
	unsigned long long n = 0;
	if (bt == MGDK_flt || bt == MGDK_dbl) {
		Cand ci;
		if (cand_init(&ci, b, s) < 0)
			return -1;
		mgdk_bat *v = b;
		if (!ci.dense) {
			// the gathered values (owned by cand_values' per-thread ring)
			v = cand_values(b, ci);
			if (v == nullptr || cand_init(&ci, v, nullptr) < 0)
				return -1;
		}
		const oid off = ci.n ? ci.seq - v->hseqbase : 0;
		DevBuf out(16), cnt(16);
		bool ok = out.p && cnt.p;
		if (ok && ci.n >= fp_parallel_min() && ci.n > 0) {
			unsigned nb = (unsigned) min((BUN) 2048, (ci.n + 4095) / 4096);
			const BUN tile = (ci.n + nb - 1) / nb;
			nb = (unsigned) ((ci.n + tile - 1) / tile);
			DevBuf part((size_t) nb * sizeof(FAvg));
			ok = part.p != nullptr;
			if (ok) {
				if (bt == MGDK_flt)
					hipLaunchKernelGGL((k_favg_par<float>), dim3(nb), dim3(256), 0, st, (const float *) v->theap, off,
							   (const oid *) nullptr, (oid) MGDK_OID_NIL, (oid) 0, ci.n, tile, true,
							   part.as<FAvg>());
				else
					hipLaunchKernelGGL((k_favg_par<double>), dim3(nb), dim3(256), 0, st, (const double *) v->theap,
							   off, (const oid *) nullptr, (oid) MGDK_OID_NIL, (oid) 0, ci.n, tile, true,
							   part.as<FAvg>());
				hipLaunchKernelGGL(k_favg_fin, dim3(1), dim3(256), 0, st, part.as<FAvg>(), nb, 1.0, out.as<double>(),
						   cnt.as<long long>());
				ok = sync();
			}
		} else if (ok && ci.n > 0) {
			if (bt == MGDK_flt)
				hipLaunchKernelGGL((k_favg_replay<float>), dim3(1), dim3(64), 0, st, (const float *) v->theap, off,
						   (const uint32_t *) nullptr, (const uint64_t *) nullptr, (const oid *) nullptr,
						   (oid) MGDK_OID_NIL, (oid) 0, (BUN) 1, ci.n, true, 1.0, out.as<double>(),
						   cnt.as<long long>());
			else
				hipLaunchKernelGGL((k_favg_replay<double>), dim3(1), dim3(64), 0, st, (const double *) v->theap, off,
						   (const uint32_t *) nullptr, (const uint64_t *) nullptr, (const oid *) nullptr,
						   (oid) MGDK_OID_NIL, (oid) 0, (BUN) 1, ci.n, true, 1.0, out.as<double>(),
						   cnt.as<long long>());
			ok = sync();
		}
		double *h = (double *) pinned(16);
		if (ok && ci.n > 0)
			ok = h && hip_ok(hipMemcpyAsync(h, out.p, 8, hipMemcpyDeviceToHost, st), "memcpy") &&
			     hip_ok(hipMemcpyAsync(h + 1, cnt.p, 8, hipMemcpyDeviceToHost, st), "memcpy") && sync_data();
		if (!ok)
			return -1;
		if (ci.n > 0) {
			long long c;
			memcpy(&c, h + 1, 8);
			n = (unsigned long long) c;
			a = n > 0 ? h[0] : nil;
		}
	} else {
		// the exact sum and count in one reduction; an hge column whose sum
		// could leave 128 bits is checked in order
		hge total = 0;
		Cand ci;
		if (cand_init(&ci, b, s) < 0)
			return -1;
		SumOut *o = (SumOut *) meta_buf();
		if (ci.n) {
			const oid off = ci.dense ? ci.seq - b->hseqbase : 0;
			const unsigned g = grid_for(ci.n, 256 * 8, 2048);
			SumPart *parts = (SumPart *) scratch((size_t) g * sizeof(SumPart));
			if (parts == nullptr)
				return -1;
			const dim3 gd(g), blk(256);
#define KS(W_) do { if (ci.dense) hipLaunchKernelGGL((k_sum<W_, true>), gd, blk, 0, st, b->theap, off, ci.oids, b->hseqbase, ci.n, parts); \
		else hipLaunchKernelGGL((k_sum<W_, false>), gd, blk, 0, st, b->theap, off, ci.oids, b->hseqbase, ci.n, parts); } while (0)
			switch (b->twidth) {
			case 1: KS(1); break;
			case 2: KS(2); break;
			case 4: KS(4); break;
			case 8: KS(8); break;
			default: KS(16); break;
			}
#undef KS
			hipLaunchKernelGGL(k_sum_fin, dim3(1), dim3(256), 0, st, parts, g, o);
			SumOut *h = (SumOut *) pinned(sizeof(SumOut));
			if (h == nullptr || !hip_ok(hipMemcpyAsync(h, o, sizeof(SumOut), hipMemcpyDeviceToHost, st), "memcpy") ||
			    !sync())
				return -1;
			n = h->cnt;
			total = (hge) (((uhge) h->sum[1] << 64) | h->sum[0]);
			if (bt == MGDK_hge && mag_bound(h->maxabs) * (long double) n > (long double) tmax(MGDK_hge)) {
				unsigned long long *ov = (unsigned long long *) o;
				hipLaunchKernelGGL(k_sum_ordered, dim3(1), dim3(256), 0, st, b->theap, b->twidth, ci.dense,
						   ci.dense ? ci.seq - b->hseqbase : 0, ci.oids, b->hseqbase, ci.n, tmax(MGDK_hge), ov);
				unsigned long long *hv = (unsigned long long *) pinned(16);
				if (!hip_ok(hipMemcpyAsync(hv, ov, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
					return -1;
				if (*hv) {
					seterr("42000!BATcalcavg: hge sum exceeds the 128-bit device accumulator\n");
					return -1;
				}
			}
		}
		a = n > 0 ? (double) total / (double) n : nil;
	}
	if (scale != 0 && a == a)
		a /= pow(10.0, (double) scale);
	*avg = a;
	if (vals)
		*vals = (mgdk_BUN) n;
	return 0;
}

int
mgdk_BATgroupavg(mgdk_bat **bnp, mgdk_bat **cntsp, mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp,
		 bool skip_nils, int scale)
{
	if (cntsp)
		*cntsp = nullptr;
	if (tp != MGDK_dbl) {
		seterr("42000!BATgroupavg: result type must be dbl\n");
		return -1;
	}
	if (b == nullptr) {
		seterr("b and g must be aligned\n");
		return -1;
	}
	const int bt = b->ttype;
	const bool isf = bt == MGDK_flt || bt == MGDK_dbl;
	if (!isf && bt != MGDK_bte && bt != MGDK_sht && bt != MGDK_int && bt != MGDK_lng && bt != MGDK_hge) {
		seterr("type (%s) not supported.\n", atomname(bt));
		return -1;
	}
	ProfScope prof("groupavg");
	AggrInit a;
	if (aggr_init(&a, &b, g, e, s) < 0)
		return -1;
	const BUN ng = a.ngrp;
	const oid hb = ng ? a.min : 0;
	hipStream_t st = stream();
	auto constant_lng = [&](long long v) -> mgdk_bat * {
		std::vector<long long> c(ng + 1, v);
		mgdk_bat *cn = upload_new(hb, MGDK_lng, c.data(), ng);
		if (cn) {
			cn->tnonil = 1;
			cn->tkey = cn->tsorted = cn->trevsorted = ng <= 1;
		}
		return cn;
	};
	if (a.ci.n == 0 || ng == 0) {
		std::vector<double> d(ng + 1, __builtin_nan(""));
		mgdk_bat *bn = upload_new(hb, MGDK_dbl, d.data(), ng);
		mgdk_bat *cn = cntsp ? constant_lng(0) : nullptr;
		if (!bn || (cntsp && !cn)) {
			mgdk_BBPunfix(bn);
			mgdk_BBPunfix(cn);
			return -1;
		}
		bn->tnil = ng > 0;
		bn->tnonil = ng == 0;
		*bnp = bn;
		if (cntsp)
			*cntsp = cn;
		return 0;
	}
	const bool gdense = g->tseqbase != MGDK_OID_NIL;
	const oid off = a.ci.seq - b->hseqbase;
	if ((!skip_nils || cntsp == nullptr || b->tnonil) &&
	    (e == nullptr || (e->count == a.ci.n && e->hseqbase == b->hseqbase)) && (gdense || (g->tkey && g->tnonil))) {
		mgdk_bat *bn = newbat(s ? s->hseqbase : b->hseqbase, MGDK_dbl, a.ci.n);
		mgdk_bat *cn = cntsp ? constant_lng(1) : nullptr;
		if (!bn || (cntsp && !cn)) {
			mgdk_BBPunfix(bn);
			mgdk_BBPunfix(cn);
			return -1;
		}
		hipLaunchKernelGGL(k_to_dbl, dim3(grid_for(a.ci.n, 1024, 8192)), dim3(256), 0, st, b->theap, bt, b->twidth,
				   off, a.ci.n, (double *) bn->theap);
		if (!sync()) {
			mgdk_BBPunfix(bn);
			mgdk_BBPunfix(cn);
			return -1;
		}
		bn->count = a.ci.n;
		*bnp = bn;
		if (cntsp)
			*cntsp = cn;
		return 0;
	}
	const double fac = scale != 0 ? pow(10.0, (double) scale) : 1.0;
	mgdk_bat *bn = nullptr, *cn = nullptr;
	bool nils = false;
	if (isf) {
		if (a.ci.n >= 0xffffffffull || ng >= 0xffffffffull) {
			seterr("42000!BATgroupavg: more than 2^32-1 rows on the device path\n");
			return -1;
		}
		bn = newbat(hb, MGDK_dbl, ng);
		cn = newbat(hb, MGDK_lng, ng);
		GroupRows gr(a.ci.n, ng);
		if (!bn || !cn || !gr.ok()) {
			mgdk_BBPunfix(bn);
			mgdk_BBPunfix(cn);
			return -1;
		}
		bool ok = group_rows(a, gr) == 0;
		const uint32_t *perm = gr.perm;
		const uint64_t *sp = gr.start_p;
		if (ok && ng == 1 && a.ci.n >= fp_parallel_min()) {
			unsigned nb = (unsigned) min((BUN) 2048, (a.ci.n + 4095) / 4096);
			const BUN tile = (a.ci.n + nb - 1) / nb;
			nb = (unsigned) ((a.ci.n + tile - 1) / tile);
			DevBuf part((size_t) nb * sizeof(FAvg));
			ok = part.p != nullptr;
			if (ok) {
				if (bt == MGDK_flt)
					hipLaunchKernelGGL((k_favg_par<float>), dim3(nb), dim3(256), 0, st, (const float *) b->theap, off,
							   a.gids, a.gseq, a.min, a.ci.n, tile, skip_nils, part.as<FAvg>());
				else
					hipLaunchKernelGGL((k_favg_par<double>), dim3(nb), dim3(256), 0, st, (const double *) b->theap,
							   off, a.gids, a.gseq, a.min, a.ci.n, tile, skip_nils, part.as<FAvg>());
				hipLaunchKernelGGL(k_favg_fin, dim3(1), dim3(256), 0, st, part.as<FAvg>(), nb, fac,
						   (double *) bn->theap, (long long *) cn->theap);
				ok = sync();
			}
		} else if (ok) {
			const dim3 grid((unsigned) ((ng + 63) / 64)), blk(64);
			if (bt == MGDK_flt)
				hipLaunchKernelGGL((k_favg_replay<float>), grid, blk, 0, st, (const float *) b->theap, off, perm,
						   sp, a.gids, a.gseq, a.min, ng, a.ci.n, skip_nils, fac, (double *) bn->theap,
						   (long long *) cn->theap);
			else
				hipLaunchKernelGGL((k_favg_replay<double>), grid, blk, 0, st, (const double *) b->theap, off,
						   perm, sp, a.gids, a.gseq, a.min, ng, a.ci.n, skip_nils, fac,
						   (double *) bn->theap, (long long *) cn->theap);
			ok = sync();
		}
		if (!ok) {
			mgdk_BBPunfix(bn);
			mgdk_BBPunfix(cn);
			return -1;
		}
		bn->count = cn->count = ng;
		std::vector<long long> hc(ng);
		if (!hip_ok(hipMemcpy(hc.data(), cn->theap, ng * 8, hipMemcpyDeviceToHost), "memcpy")) {
			mgdk_BBPunfix(bn);
			mgdk_BBPunfix(cn);
			return -1;
		}
		for (BUN k = 0; k < ng; k++)
			nils |= hc[k] == 0;
	} else {
		// AVERAGE_ITER's invariant: avg * n + rem == sum, 0 <= rem < n
		bn = newbat(hb, MGDK_dbl, ng);
		cn = newbat(hb, MGDK_lng, ng);
		DevBuf fl(16);
		GAcc acc;
		unsigned long long *mx = nullptr;
		uint32_t hf = 0;
		bool ok = bn && cn && fl.p && hip_ok(hipMemsetAsync(fl.p, 0, 16, st), "memset") &&
			  gaggr_device(a, b, AGG_SUM | (skip_nils ? 0 : AGG_POS), false, acc, mx) == 0;
		if (ok) {
			hipLaunchKernelGGL(k_gavg_out, dim3(grid_for(ng, 1024, 8192)), dim3(256), 0, st, acc, ng, skip_nils,
					   bt == MGDK_hge, mx, scale != 0 ? fac : 1.0, (double *) bn->theap,
					   (long long *) cn->theap, fl.as<uint32_t>());
			ok = read_flags(fl.p, &hf);
		}
		if (ok && (hf & 1)) {
			seterr("42000!BATgroupavg: hge group sum exceeds the 128-bit device accumulator\n");
			ok = false;
		}
		if (!ok) {
			mgdk_BBPunfix(bn);
			mgdk_BBPunfix(cn);
			return -1;
		}
		bn->count = cn->count = ng;
		nils = (hf & 2) != 0;
	}
	bn->tkey = bn->tsorted = bn->trevsorted = ng <= 1;
	bn->tnil = nils;
	bn->tnonil = !nils;
	cn->tkey = cn->tsorted = cn->trevsorted = ng <= 1;
	cn->tnonil = 1;
	*bnp = bn;
	if (cntsp)
		*cntsp = cn;
	else
		mgdk_BBPunfix(cn);
	return 0;
}

// BATgroupavg3combine (gdk/gdk_aggr.c:2634-2960): each group's state is
// folded row by row with combine_averages_TYPE (:2402-2630), which keeps
// avg * cnt + rem == the exact total; the device sums the rows' totals and
// counts per group (order independent) and takes the floor average and its
// remainder, rounded half away from zero (:2702-2716)
mgdk_bat *
mgdk_BATgroupavg3combine(mgdk_bat *avg, mgdk_bat *rem, mgdk_bat *cnt, mgdk_bat *g, mgdk_bat *e, bool skip_nils)
{
	if (avg == nullptr || rem == nullptr || cnt == nullptr || !int_type(avg->ttype)) {
		seterr("42000!BATgroupavg3combine: type not supported on the device path");
		return nullptr;
	}
	ProfScope prof("groupavg3combine");
	AggrInit a;
	if (aggr_init(&a, &avg, g, e, nullptr) < 0)
		return nullptr;
	if (a.ci.n != rem->count || a.ci.n != cnt->count) {
		seterr("input bats not aligned");
		return nullptr;
	}
	const BUN n = a.ci.n, ng = a.ngrp;
	const int tp = avg->ttype;
	if (n == 0 || ng == 0) {
		std::vector<char> nilv(ng * width_of(tp) + 16);
		for (BUN k = 0; k < ng; k++)
			put_vec(nilv, tp, k, 0, true);
		mgdk_bat *bn = upload_new(ng == 0 ? 0 : a.min, tp, nilv.data(), ng);
		if (bn) {
			bn->tnil = ng > 0;
			bn->tnonil = ng == 0;
		}
		return bn;
	}
	hipStream_t st = stream();
	mgdk_bat *T = newbat(avg->hseqbase, MGDK_hge, n), *Cb = newbat(avg->hseqbase, MGDK_lng, n);
	DevBuf fl(64);
	mgdk_bat *S = nullptr, *C = nullptr, *bn = nullptr;
	uint32_t *hf = (uint32_t *) pinned(16);
	if (!T || !Cb || !fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 64, st), "memset"))
		goto out;
	{
		const oid off = a.ci.seq - avg->hseqbase;
		const dim3 gr(grid_for(n, 1024, 8192)), blk(256);
		const long long *R = (const long long *) rem->theap, *K = (const long long *) cnt->theap;
		switch (basetype(tp)) {
		case MGDK_bte: hipLaunchKernelGGL((k_avg3c_terms<int8_t>), gr, blk, 0, st, (const int8_t *) avg->theap, R, K, off, n, (hge *) T->theap, (long long *) Cb->theap, fl.as<uint32_t>()); break;
		case MGDK_sht: hipLaunchKernelGGL((k_avg3c_terms<int16_t>), gr, blk, 0, st, (const int16_t *) avg->theap, R, K, off, n, (hge *) T->theap, (long long *) Cb->theap, fl.as<uint32_t>()); break;
		case MGDK_int: hipLaunchKernelGGL((k_avg3c_terms<int32_t>), gr, blk, 0, st, (const int32_t *) avg->theap, R, K, off, n, (hge *) T->theap, (long long *) Cb->theap, fl.as<uint32_t>()); break;
		case MGDK_lng: hipLaunchKernelGGL((k_avg3c_terms<int64_t>), gr, blk, 0, st, (const int64_t *) avg->theap, R, K, off, n, (hge *) T->theap, (long long *) Cb->theap, fl.as<uint32_t>()); break;
		default: hipLaunchKernelGGL((k_avg3c_terms<hge>), gr, blk, 0, st, (const hge *) avg->theap, R, K, off, n, (hge *) T->theap, (long long *) Cb->theap, fl.as<uint32_t>()); break;
		}
		if (!hip_ok(hipMemcpyAsync(hf, fl.p, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			goto out;
		if (hf[0]) {
			seterr("42000!BATgroupavg3combine: |avg * count| beyond 2^126 is not supported on the device path");
			goto out;
		}
		T->count = Cb->count = n;
		T->tnonil = Cb->tnonil = avg->tnonil;
		T->tnil = Cb->tnil = !avg->tnonil;
		// the group's rows in the same candidate order as avg: T / Cb are
		// aligned with avg's candidates (hseqbase avg->hseqbase + off)
		T->hseqbase = Cb->hseqbase = a.ci.seq;
		// sums over the non-nil rows; without skip_nils a group with any nil
		// avg is nil for good (counted apart: BATgroupsum's own nil rule
		// differs, gdk_aggr.c:497-527)
		S = mgdk_BATgroupsum(T, g, e, nullptr, MGDK_hge, true);
		C = mgdk_BATgroupsum(Cb, g, e, nullptr, MGDK_hge, true);
		if (!S || !C)
			goto out;
		mgdk_bat *N1 = nullptr, *N2 = nullptr;
		if (!skip_nils && !avg->tnonil) {
			N1 = mgdk_BATgroupcount(avg, g, e, nullptr, MGDK_lng, false);
			N2 = N1 ? mgdk_BATgroupcount(avg, g, e, nullptr, MGDK_lng, true) : nullptr;
			if (!N1 || !N2) {
				mgdk_BBPunfix(N1);
				mgdk_BBPunfix(N2);
				goto out;
			}
		}
		bn = newbat(a.min, tp, ng);
		uint32_t hf = 0;
		bool ok = bn && hip_ok(hipMemsetAsync(fl.p, 0, 16, st), "memset");
		if (ok) {
			hipLaunchKernelGGL(k_avg3c_out, dim3(grid_for(ng, 1024, 8192)), dim3(256), 0, st, ng,
					   (const hge *) S->theap, (const hge *) C->theap,
					   N1 ? (const long long *) N1->theap : nullptr,
					   N2 ? (const long long *) N2->theap : nullptr, basetype(tp), bn->theap, fl.as<uint32_t>());
			ok = read_flags(fl.p, &hf);
		}
		mgdk_BBPunfix(N1);
		mgdk_BBPunfix(N2);
		if (!ok) {
			mgdk_BBPunfix(bn);
			bn = nullptr;
			goto out;
		}
		bn->count = ng;
		bn->tnil = (hf & 2) != 0;
		bn->tnonil = !bn->tnil;
		bn->tkey = bn->tsorted = bn->trevsorted = ng <= 1;
	}
out:
	mgdk_BBPunfix(T);
	mgdk_BBPunfix(Cb);
	mgdk_BBPunfix(S);
	mgdk_BBPunfix(C);
	return bn;
}

// BATgroupavg3 (gdk/gdk_aggr.c:1996-2110)
int
mgdk_BATgroupavg3(mgdk_bat **avgp, mgdk_bat **remp, mgdk_bat **cntp, mgdk_bat *b, mgdk_bat *g,
		  mgdk_bat *e, mgdk_bat *s, bool skip_nils)
{
	if (b == nullptr || !int_type(b->ttype)) {
		seterr("42000!BATgroupavg3: type not supported on the device path");
		return -1;
	}
	ProfScope prof("groupavg3");
	AggrInit a;
	if (aggr_init(&a, &b, g, e, s) < 0)
		return -1;
	const BUN ng = a.ngrp;
	const int tp = b->ttype;
	const oid hb = ng ? a.min : 0;
	mgdk_bat *A = newbat(hb, tp, ng), *R = newbat(hb, MGDK_lng, ng), *C = newbat(hb, MGDK_lng, ng);
	DevBuf fl(16);
	uint32_t hf = 0;
	bool ok = A && R && C && fl.p && hip_ok(hipMemsetAsync(fl.p, 0, 16, stream()), "memset");
	if (ok && ng) {
		GAcc acc;
		unsigned long long *mx;
		ok = gaggr_device(a, b, AGG_SUM | (skip_nils ? 0 : AGG_POS), false, acc, mx) == 0;
		if (ok) {
			hipLaunchKernelGGL(k_gavg3_out, dim3(grid_for(ng, 1024, 8192)), dim3(256), 0, stream(), acc, ng,
					   a.ci.n == 0, basetype(tp), skip_nils, A->theap, (long long *) R->theap,
					   (long long *) C->theap, fl.as<uint32_t>());
			ok = read_flags(fl.p, &hf);
		}
	}
	if (!ok) {
		mgdk_BBPunfix(A);
		mgdk_BBPunfix(R);
		mgdk_BBPunfix(C);
		return -1;
	}
	A->count = R->count = C->count = ng;
	// gdk_aggr.c:2012-2027 (no candidates: constants nil / nil / 0), :2298-2303
	const bool empty = a.ci.n == 0;
	A->tnil = (hf & 2) != 0;
	R->tnil = empty ? ng > 0 : (hf & 4) != 0;
	C->tnil = !empty && (hf & 4) != 0;
	A->tnonil = !A->tnil;
	R->tnonil = !R->tnil;
	C->tnonil = !C->tnil;
	A->tkey = R->tkey = C->tkey = empty ? ng <= 1 : ng == 1;
	A->tsorted = R->tsorted = C->tsorted = empty || ng == 1;
	A->trevsorted = R->trevsorted = C->trevsorted = empty || ng == 1;
	*avgp = A;
	*remp = R;
	*cntp = C;
	return 0;
}

}  // extern "C"

namespace {

// ---- BATgroupmin / max over SORTED group ids in one pass: the segmented
// reduction of k_gaggr_sorted with (has a candidate, is nil, best value,
// candidate index) per run -- the first nil wins without skip_nils, else the
// first row holding the extreme; runs combine in row order, so ties keep
// the earlier row.  Results (oids) are stored by the lanes that finish the
// groups, empty groups get oid_nil, the groups a range shares with its
// neighbours go through per-range edge entries (k_gminpos_edges).
struct MRun {
	long long best;
	unsigned long long idx;    // candidate index, ~0: none
	bool isn;
	__device__ void clear()
	{
		best = 0;
		idx = ~0ull;
		isn = false;
	}
	template <bool DOMAX>
	__device__ void add(const MRun &r)    // *this = (*this) followed by r
	{
		if (r.idx == ~0ull || isn)
			return;
		if (idx == ~0ull || r.isn || (DOMAX ? r.best > best : r.best < best))
			*this = r;
	}
	__device__ MRun shfl_up(int d) const
	{
		MRun t;
		t.best = __shfl_up(best, d);
		t.idx = __shfl_up(idx, d);
		t.isn = __shfl_up((int) isn, d) != 0;
		return t;
	}
};

struct MEdge {
	oid g;
	long long best;
	unsigned long long idx;
	unsigned long long isn;
};

struct MOut {
	oid *out;
	bool cdense;
	oid cseq;
	const oid *coids;
	uint32_t *flags;
};

__device__ __forceinline__ uint32_t
mout_put(const MOut &mo, BUN gi, const MRun &r)
{
	const bool nil = r.idx == ~0ull;
	mo.out[gi] = nil ? MGDK_OID_NIL : mo.cdense ? mo.cseq + r.idx : mo.coids[r.idx];
	return nil ? 2u : 0u;
}

template <int VW, bool DOMAX>
__global__ __launch_bounds__(256) void
k_gminpos_sorted(const void *base, oid off, const oid *gids, oid gseq, oid gmin, BUN ngrp, BUN n, bool skip_nils,
		 bool vec, MOut mo, MEdge *edges)
{
	typedef typename VTy<VW>::T T;
	constexpr int U = GS_U;
	constexpr BUN RW = 64 * U;
	const int lane = __lane_id();
	const BUN nwaves = (BUN) gridDim.x * (blockDim.x / 64);
	const BUN wid = (BUN) blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
	uint32_t f = 0;
	auto valid = [&](oid g) { return g >= gmin && g - gmin < ngrp; };
	auto gap = [&](oid prev, oid hi) {   // groups strictly between prev and hi
		if (prev >= gmin + ngrp)
			return;
		oid lo = prev + 1;
		lo = lo > gmin ? lo : gmin;
		hi = hi < gmin + ngrp ? hi : gmin + ngrp;
		MRun e;
		e.clear();
		for (oid h = lo; h < hi; h++)
			f |= mout_put(mo, h - gmin, e);
	};
	for (BUN r0 = wid * RW; r0 < n; r0 += nwaves * RW) {
		const BUN r1 = r0 + RW < n ? r0 + RW : n;
		const BUN l0 = r0 + (BUN) lane * U;
		oid g[U];
		T x[U];
		if (vec && l0 + U <= r1) {
			if (gids) {
				const uint4 *p = (const uint4 *) (gids + l0);
				uint4 q[U / 2];
#pragma unroll
				for (int u = 0; u < U / 2; u++)
					q[u] = p[u];
				__builtin_memcpy(g, q, sizeof g);
			} else {
#pragma unroll
				for (int u = 0; u < U; u++)
					g[u] = gseq + l0 + u;
			}
			constexpr int NQ = U * VW / 16;
			const uint4 *p = (const uint4 *) ((const T *) base + off + l0);
			uint4 q[NQ];
#pragma unroll
			for (int u = 0; u < NQ; u++)
				q[u] = p[u];
			__builtin_memcpy(x, q, sizeof x);
		} else {
#pragma unroll
			for (int u = 0; u < U; u++) {
				const BUN ic = l0 + u < r1 ? l0 + u : r1 - 1;
				g[u] = gids ? gids[ic] : gseq + ic;
				x[u] = ((const T *) base)[off + ic];
			}
		}
		MRun P, cur;
		P.clear();
		cur.clear();
		bool single = true;
		const oid gF = g[0];
		oid cg = g[0];
#pragma unroll
		for (int u = 0; u < U; u++) {
			if (g[u] != cg) {
				if (single)
					P = cur;
				else if (valid(cg))
					f |= mout_put(mo, cg - gmin, cur);
				if (g[u] > cg + 1)
					gap(cg, g[u]);
				single = false;
				cur.clear();
				cg = g[u];
			}
			const BUN i = l0 + u;
			if (i < r1 && valid(g[u])) {
				const bool vn = is_nil(x[u]);
				if (!(skip_nils && vn)) {
					MRun r;
					r.best = (long long) x[u];
					r.idx = i;
					r.isn = vn;
					cur.add<DOMAX>(r);
				}
			}
		}
		const oid gL = cg;
		const oid gLprev = __shfl_up(gL, 1), gFnext = __shfl_down(gF, 1);
		const bool connects = lane > 0 && gLprev == gF;
		const bool nextconn = lane < 63 && gFnext == gL;
		const unsigned long long chain = __ballot(single && (lane == 0 || connects));
		const bool rfirst = lane == 0 || (connects && (~chain & ((1ull << lane) - 1)) == 0);
		// segmented scan of the last runs (a run's earlier part is on the left)
		MRun t = cur;
		bool hd = !(single && connects);
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const MRun o = t.shfl_up(d);
			const bool th = __shfl_up((int) hd, d) != 0;
			if (lane >= d) {
				if (!hd) {
					MRun c = o;
					c.add<DOMAX>(t);
					t = c;
				}
				hd |= th;
			}
		}
		const MRun cin = t.shfl_up(1);
		if (lane < 63 && gFnext > gL + 1)
			gap(gL, gFnext);
		if (lane == 0) {
			if (r0 == 0) {
				MRun e;
				e.clear();
				for (oid h = gmin; h < gF && h < gmin + ngrp; h++)
					f |= mout_put(mo, h - gmin, e);
			} else {
				const oid gp = gids ? gids[r0 - 1] : gseq + r0 - 1;
				if (gF > gp + 1)
					gap(gp, gF);
			}
		}
		if (lane == 63 && r1 == n)
			gap(gL, gmin + ngrp);
		bool e0 = false;
		MRun e0run;
		e0run.clear();
		if (!single) {
			if (connects) {
				MRun c = cin;
				c.add<DOMAX>(P);
				P = c;
			}
			if (valid(gF)) {
				if (rfirst) {
					e0 = true;
					e0run = P;
				} else {
					f |= mout_put(mo, gF - gmin, P);
				}
			}
			if (!nextconn && valid(gL) && lane < 63)
				f |= mout_put(mo, gL - gmin, cur);
		} else if (!nextconn && valid(gL) && lane < 63) {
			if (rfirst) {
				e0 = true;
				e0run = t;
			} else {
				f |= mout_put(mo, gL - gmin, t);
			}
		}
		const BUN rk = r0 / RW;
		if (e0 || (__ballot(e0) == 0 && lane == 0))
			edges[2 * rk] = MEdge{gF, e0run.best, e0run.idx, e0run.isn};
		if (lane == 63) {
			MRun r = single ? t : cur;
			if (!valid(gL))
				r.clear();
			edges[2 * rk + 1] = MEdge{gL, r.best, r.idx, r.isn};
		}
	}
	for (int o = 32; o > 0; o >>= 1)
		f |= __shfl_xor(f, o);
	if (lane == 0 && f)
		publish_or(mo.flags, f);
}

// BATgroupmin / max with one row per group: the row itself, unless its
// value is nil and nils are skipped (then the group has no value)
template <int VW>
__global__ __launch_bounds__(256) void
k_gminpos_rows(const void *base, oid off, BUN n, bool skip_nils, MOut mo)
{
	typedef typename VTy<VW>::T T;
	uint32_t f = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		MRun r;
		r.clear();
		const T x = ((const T *) base)[off + i];
		if (!(skip_nils && is_nil(x))) {
			r.idx = i;
			r.best = (long long) x;
			r.isn = is_nil(x);
		}
		f |= mout_put(mo, i, r);
	}
	for (int o = 32; o > 0; o >>= 1)
		f |= __shfl_xor(f, o);
	if (__lane_id() == 0 && f)
		publish_or(mo.flags, f);
}

template <bool DOMAX>
__global__ __launch_bounds__(256) void
k_gminpos_edges(const MEdge *e, BUN ne, oid gmin, BUN ngrp, MOut mo)
{
	uint32_t f = 0;
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < ne; j += (BUN) gridDim.x * blockDim.x) {
		const oid g = e[j].g;
		if ((j > 0 && e[j - 1].g == g) || g < gmin || g - gmin >= ngrp)
			continue;
		MRun acc;
		acc.clear();
		for (BUN q = j; q < ne && e[q].g == g; q++) {
			MRun r;
			r.best = e[q].best;
			r.idx = e[q].idx;
			r.isn = e[q].isn != 0;
			acc.add<DOMAX>(r);
		}
		f |= mout_put(mo, g - gmin, acc);
	}
	for (int o = 32; o > 0; o >>= 1)
		f |= __shfl_xor(f, o);
	if (__lane_id() == 0 && f)
		publish_or(mo.flags, f);
}

}  // namespace

extern "C" {

// the rows holding each group's extreme value (target) and its first nil:
// smallest candidate index of each (atomicMin, skipped when not smaller)
__global__ __launch_bounds__(256) void
k_gminmax_pos(const void *base, int w, oid off, const oid *gids, oid gseq, oid gmin, BUN ngrp, BUN n,
	      bool skip_nils, const long long *target, unsigned long long *firstnil, unsigned long long *firstbest)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const oid g = gids ? gids[i] : gseq + i;
		if (g < gmin || g - gmin >= ngrp)
			continue;
		const BUN gi = g - gmin;
		bool isnil;
		const hge v = ldv(base, w, off + i, isnil);
		unsigned long long *slot = isnil ? (skip_nils ? nullptr : &firstnil[gi])
						 : ((long long) v == target[gi] ? &firstbest[gi] : nullptr);
		if (slot && i < __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
			atomicMin(slot, (unsigned long long) i);
	}
}

// group k's result: its first nil (no skip_nils), else its first extreme
// row, else oid_nil; candidate index -> candidate oid
__global__ void
k_gminmax_out(BUN ngrp, const unsigned long long *firstnil, const unsigned long long *firstbest, bool dense,
	      oid seq, const oid *oids, oid *out)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ngrp; k += (BUN) gridDim.x * blockDim.x) {
		const unsigned long long p = firstnil[k] != ~0ull ? firstnil[k] : firstbest[k];
		out[k] = p == ~0ull ? MGDK_OID_NIL : dense ? seq + p : oids[p];
	}
}

// BATgroupmin / BATgroupmax (gdk/gdk_aggr.c:3487-3560, do_groupmin
// :3247-3362): the POSITION (oid) of each group's minimum / maximum -- its
// first row; without skip_nils the first nil of the group wins; groups
// without a value give oid_nil.  MAL's aggr.min / aggr.max project b through
// the result (monetdb5/modules/kernel/aggr.c:321-348).
static mgdk_bat *
groupminmax(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, bool skip_nils, bool domax)
{
	// oids (< 2^63, nil = 2^63) order like their signed 64-bit images
	if (b == nullptr || !(int_type(b->ttype) || b->ttype == MGDK_oid) || basetype(b->ttype) == MGDK_hge) {
		seterr("42000!BATgroupmin/max: type not supported on the device path");
		return nullptr;
	}
	Cand c0;                         // the caller's candidates (positions)
	if (cand_init(&c0, b, s) < 0)
		return nullptr;
	AggrInit a;
	if (aggr_init(&a, &b, g, e, s) < 0)
		return nullptr;
	const BUN ng = a.ngrp;
	mgdk_bat *bn = newbat(ng ? a.min : 0, MGDK_oid, ng);
	if (bn == nullptr)
		return nullptr;
	bn->count = ng;
	bn->tsorted = bn->trevsorted = bn->tkey = ng <= 1;
	if (a.ci.n == 0 || ng == 0) {
		// BATconstant(min, TYPE_oid, &oid_nil, ngrp)
		std::vector<oid> nils(ng + 1, MGDK_OID_NIL);
		if (ng && mgdk_BATupload(bn, nils.data(), ng) < 0) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		bn->count = ng;
		bn->tsorted = bn->trevsorted = 1;
		bn->tnil = ng > 0;
		bn->tnonil = ng == 0;
		return bn;
	}
	hipStream_t st = stream();
	static const bool direct = getenv("MGDK_GMINPOS_DIRECT") ? atoi(getenv("MGDK_GMINPOS_DIRECT")) != 0 : true;
	if (direct && a.gsorted && ng > 8 && b->twidth <= 8) {
		// sorted ids: one pass straight into the result (k_gminpos_sorted)
		const BUN rw = 64 * GS_U, nr = (a.ci.n + rw - 1) / rw;
		DevBuf eb(nr * 2 * sizeof(MEdge) + 64), fl(16);
		if (!eb.p || !fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 16, st), "memset")) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		const oid off = a.ci.seq - b->hseqbase;
		const bool vec = ((uintptr_t) a.gids & 15) == 0 &&
			(((uintptr_t) b->theap + (uintptr_t) off * b->twidth) & 15) == 0;
		MOut mo{(oid *) bn->theap, c0.dense, c0.seq, c0.oids, fl.as<uint32_t>()};
		const dim3 gs(grid_for(nr, 4, 65535u * 16u)), blk(256);
		MEdge *ep = eb.as<MEdge>();
		if (one_row_groups(a)) {
			const dim3 g1(grid_for(a.ci.n, 256 * 8, 8192));
			switch (b->twidth) {
			case 1: hipLaunchKernelGGL(k_gminpos_rows<1>, g1, blk, 0, st, b->theap, off, a.ci.n, skip_nils, mo); break;
			case 2: hipLaunchKernelGGL(k_gminpos_rows<2>, g1, blk, 0, st, b->theap, off, a.ci.n, skip_nils, mo); break;
			case 4: hipLaunchKernelGGL(k_gminpos_rows<4>, g1, blk, 0, st, b->theap, off, a.ci.n, skip_nils, mo); break;
			default: hipLaunchKernelGGL(k_gminpos_rows<8>, g1, blk, 0, st, b->theap, off, a.ci.n, skip_nils, mo); break;
			}
			uint32_t hf1 = 0;
			if (!read_flags(fl.p, &hf1)) {
				mgdk_BBPunfix(bn);
				return nullptr;
			}
			bn->tnil = (hf1 & 2) != 0;
			bn->tnonil = !bn->tnil;
			return bn;
		}
#define GMP(VW_, D_) hipLaunchKernelGGL((k_gminpos_sorted<VW_, D_>), gs, blk, 0, st, b->theap, off, a.gids, a.gseq, a.min, ng, a.ci.n, skip_nils, vec, mo, ep)
#define GMP2(VW_) do { if (domax) GMP(VW_, true); else GMP(VW_, false); } while (0)
		switch (b->twidth) {
		case 1: GMP2(1); break;
		case 2: GMP2(2); break;
		case 4: GMP2(4); break;
		default: GMP2(8); break;
		}
#undef GMP2
#undef GMP
		if (domax)
			hipLaunchKernelGGL(k_gminpos_edges<true>, dim3(grid_for(2 * nr, 1024, 4096)), blk, 0, st, ep, 2 * nr,
					   a.min, ng, mo);
		else
			hipLaunchKernelGGL(k_gminpos_edges<false>, dim3(grid_for(2 * nr, 1024, 4096)), blk, 0, st, ep, 2 * nr,
					   a.min, ng, mo);
		uint32_t hf = 0;
		if (!read_flags(fl.p, &hf)) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		bn->tnil = (hf & 2) != 0;
		bn->tnonil = !bn->tnil;
		return bn;
	}
	GAcc acc;
	unsigned long long *mxa;
	if (gaggr_device(a, b, AGG_MINMAX, false, acc, mxa) < 0) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	DevBuf fn(ng * 8 + 8), fb(ng * 8 + 8), fl(16);
	const long long *tgt = domax ? acc.mx : acc.mn;     // each group's extreme value
	if (!fn.p || !fb.p || !fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 16, st), "memset") ||
	    !hip_ok(hipMemsetAsync(fn.p, 0xff, ng * 8, st), "memset") ||
	    !hip_ok(hipMemsetAsync(fb.p, 0xff, ng * 8, st), "memset")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const oid off = a.ci.seq - b->hseqbase;
	hipLaunchKernelGGL(k_gminmax_pos, dim3(grid_for(a.ci.n, 256 * 8, 256 * 16)), dim3(256), 0, st, b->theap,
			   b->twidth, off, a.gids, a.gseq, a.min, ng, a.ci.n, skip_nils, tgt,
			   fn.as<unsigned long long>(), fb.as<unsigned long long>());
	hipLaunchKernelGGL(k_gminmax_out, dim3(grid_for(ng, 256, 4096)), dim3(256), 0, st, ng,
			   fn.as<unsigned long long>(), fb.as<unsigned long long>(), c0.dense, c0.seq, c0.oids,
			   (oid *) bn->theap);
	if (!sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	// groups without a value: no non-nil row and (skip_nils or no nil row)
	hipLaunchKernelGGL(k_gminmax_nils, dim3(grid_for(ng, 1024, 8192)), dim3(256), 0, st, acc, ng,
			   fn.as<unsigned long long>(), fl.as<uint32_t>());
	uint32_t hf = 0;
	if (!read_flags(fl.p, &hf)) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	bn->tnil = (hf & 2) != 0;
	bn->tnonil = !bn->tnil;
	return bn;
}

mgdk_bat *
mgdk_BATgroupmin(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	(void) tp;
	return groupminmax(b, g, e, s, skip_nils, false);
}

mgdk_bat *
mgdk_BATgroupmax(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	(void) tp;
	return groupminmax(b, g, e, s, skip_nils, true);
}

}  // extern "C"

// ---- BATcount_no_nil (gdk/gdk_batop.c:3078) ---------------------------------

namespace {

// non-nil values among the candidates, one atomic per workgroup
template <typename T>
__global__ void
k_count_nonil(const T *__restrict__ v, oid hseq, bool dense, oid seq, const oid *__restrict__ oids, BUN n,
	      unsigned long long *cnt)
{
	unsigned long long c = 0;
	for (BUN i = blockIdx.x * (BUN) blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		c += !is_nil(v[(dense ? seq + i : oids[i]) - hseq]);
	c = block_reduce(c, [](unsigned long long a, unsigned long long b) { return a + b; });
	if (threadIdx.x == 0 && c)
		atomicAdd(cnt, c);
}

// str: the first byte of the string at the offset (1- / 2-byte offsets
// biased by GDK_VAROFFSET) is not the nil string's 0x80
template <typename O>
__global__ void
k_count_nonil_str(const O *__restrict__ off, const char *__restrict__ heap, size_t bias, oid hseq, bool dense,
		  oid seq, const oid *__restrict__ oids, BUN n, unsigned long long *cnt)
{
	unsigned long long c = 0;
	for (BUN i = blockIdx.x * (BUN) blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		c += heap[(size_t) off[(dense ? seq + i : oids[i]) - hseq] + bias] != '\200';
	c = block_reduce(c, [](unsigned long long a, unsigned long long b) { return a + b; });
	if (threadIdx.x == 0 && c)
		atomicAdd(cnt, c);
}

}  // namespace

// the count of b's candidates whose value is not nil; every candidate when b
// is known nil-free (tnonil), a msk BAT, or a void BAT with a sequence (none
// when its sequence is nil).  A count of every row records tnonil in b, as
// the reference does.  The reference cannot fail; here a device error gives
// MGDK_BUN_NONE with the message set, a NULL b 0
extern "C" mgdk_BUN
mgdk_BATcount_no_nil(mgdk_bat *b, mgdk_bat *s)
{
	if (b == nullptr)
		return 0;
	mgdk_bat *held = nullptr;
	if (s && is_complex_cand(s) && (s = held = unmask_cand(s)) == nullptr)
		return MGDK_BUN_NONE;
	struct Unfix {
		mgdk_bat *b;
		~Unfix() { mgdk_BBPunfix(b); }
	} unfix{held};
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return MGDK_BUN_NONE;
	if (b->tnonil || b->ttype == MGDK_msk)
		return ci.n;
	if (b->ttype == MGDK_void)
		return b->tseqbase == MGDK_OID_NIL ? 0 : ci.n;
	BUN cnt = 0;
	if (ci.n > 0) {
		DevBuf acc(8);
		if (!acc.p)
			return MGDK_BUN_NONE;
		hipStream_t st = stream();
		unsigned long long *d = acc.as<unsigned long long>();
		if (!hip_ok(hipMemsetAsync(d, 0, 8, st), "hipMemsetAsync"))
			return MGDK_BUN_NONE;
		const dim3 g(grid_for(ci.n, BLOCK * 16, 256u * 32u)), blk(BLOCK);
		const oid hs = b->hseqbase;
		switch (b->ttype == MGDK_str ? MGDK_str : basetype(b->ttype)) {
		case MGDK_bte: hipLaunchKernelGGL((k_count_nonil<int8_t>), g, blk, 0, st, (const int8_t *) b->theap, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
		case MGDK_sht: hipLaunchKernelGGL((k_count_nonil<int16_t>), g, blk, 0, st, (const int16_t *) b->theap, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
		case MGDK_int: hipLaunchKernelGGL((k_count_nonil<int32_t>), g, blk, 0, st, (const int32_t *) b->theap, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
		case MGDK_lng: hipLaunchKernelGGL((k_count_nonil<int64_t>), g, blk, 0, st, (const int64_t *) b->theap, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
		case MGDK_oid: hipLaunchKernelGGL((k_count_nonil<uint64_t>), g, blk, 0, st, (const uint64_t *) b->theap, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
		case MGDK_hge: hipLaunchKernelGGL((k_count_nonil<hge>), g, blk, 0, st, (const hge *) b->theap, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
		case MGDK_flt: hipLaunchKernelGGL((k_count_nonil<float>), g, blk, 0, st, (const float *) b->theap, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
		case MGDK_dbl: hipLaunchKernelGGL((k_count_nonil<double>), g, blk, 0, st, (const double *) b->theap, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
		case MGDK_str: {
			const char *heap = (const char *) b->tvheap;
			switch (b->twidth) {
			case 1: hipLaunchKernelGGL((k_count_nonil_str<uint8_t>), g, blk, 0, st, (const uint8_t *) b->theap, heap, (size_t) 8192, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
			case 2: hipLaunchKernelGGL((k_count_nonil_str<uint16_t>), g, blk, 0, st, (const uint16_t *) b->theap, heap, (size_t) 8192, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
			case 4: hipLaunchKernelGGL((k_count_nonil_str<uint32_t>), g, blk, 0, st, (const uint32_t *) b->theap, heap, (size_t) 0, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
			default: hipLaunchKernelGGL((k_count_nonil_str<uint64_t>), g, blk, 0, st, (const uint64_t *) b->theap, heap, (size_t) 0, hs, ci.dense, ci.seq, ci.oids, ci.n, d); break;
			}
			break;
		}
		default:
			seterr("BATcount_no_nil: type %s is not on the device path", atomname(b->ttype));
			return MGDK_BUN_NONE;
		}
		unsigned long long h = 0;
		if (!hip_ok(hipGetLastError(), "k_count_nonil") ||
		    !hip_ok(hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, st), "hipMemcpyAsync") || !sync())
			return MGDK_BUN_NONE;
		cnt = (BUN) h;
	}
	if (cnt == b->count) {            // gdk_batop.c:3179 "we learned something"
		b->tnonil = 1;
		b->tnil = 0;
	}
	return cnt;
}
