// fsum.hip -- BATsum of flt / dbl columns on the MI355X (gdk/gdk_aggr.c:1018
// -> dosum :708 -> dofsum :183-427).
//
// dofsum is Shewchuk / Python msum: its result is the exact sum of the
// non-nil values rounded once to double (round half to even), or the
// "22003!overflow in sum aggregate." error when that rounded sum is not a
// finite double (:415-421); a flt result is that double cast to flt (:400-406).
// The device computes the exact sum instead of msum's partials: every value
// is an integer mantissa times 2^E, so the sum is an integer in units of
// 2^Emin.  One pass finds Emin, the highest bit and the count; a second adds
// every mantissa, shifted by E - Emin, into a per-lane two's-complement
// fixed-point integer of L 64-bit limbs (L = 2 or 4, chosen so the range
// plus log2(count) fits), reduced per workgroup; one workgroup adds the
// partials.  The host rounds the L-limb integer to double exactly (guard and
// sticky bits, subnormal results rounded at 2^-1074).  Columns whose values
// span more than ~250 bits of exponent (e.g. 1e-300 beside 1e300) go to an
// LDS superaccumulator of 32-bit digits covering the whole double range
// instead (three 64-bit LDS atomics per value).  An infinite input makes msum's
// accumulator overflow, so it is reported as the reference's overflow
// error.
#include <cmath>
#include <vector>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

struct FRange {
	unsigned long long cnt;        // non-nil values
	unsigned long long firstnil;   // first nil candidate index
	int emin;                      // lowest exponent (of the mantissa LSB) of a nonzero value
	int etop;                      // highest exponent + 53
	unsigned int inf;              // an infinite value was seen
	unsigned int pad;
};

// value -> (negative, integer mantissa, exponent of its LSB); false for zero
template <typename T>
__device__ __forceinline__ bool
fdecomp(T v, bool &neg, uint64_t &mant, int &e)
{
	const double d = (double) v;           // flt -> dbl is exact
	const uint64_t bits = (uint64_t) __double_as_longlong(d);
	neg = bits >> 63;
	const int ex = (int) ((bits >> 52) & 0x7ff);
	mant = bits & ((1ull << 52) - 1);
	if (ex == 0) {
		if (mant == 0)
			return false;
		e = -1074;
	} else {
		mant |= 1ull << 52;
		e = ex - 1075;
	}
	return true;
}

template <typename T>
__device__ __forceinline__ T
fval(const T *base, bool dense, oid off, const oid *oids, oid hseq, BUN i)
{
	return base[dense ? off + i : oids[i] - hseq];
}

template <typename T>
__global__ __launch_bounds__(256) void
k_fsum_range(const T *base, bool dense, oid off, const oid *oids, oid hseq, BUN n, FRange *o)
{
	unsigned long long cnt = 0, firstnil = ~0ull;
	int emin = INT32_MAX, etop = INT32_MIN;
	unsigned inf = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const T v = fval(base, dense, off, oids, hseq, i);
		if (v != v) {
			firstnil = i < firstnil ? i : firstnil;
			continue;
		}
		cnt++;
		if (isinf((double) v)) {
			inf = 1;
			continue;
		}
		bool neg;
		uint64_t m;
		int e;
		if (fdecomp(v, neg, m, e)) {
			emin = e < emin ? e : emin;
			const int top = e + 64 - __builtin_clzll(m);
			etop = top > etop ? top : etop;
		}
	}
	cnt = block_reduce(cnt, [](unsigned long long a, unsigned long long b) { return a + b; });
	if (threadIdx.x == 0 && cnt)
		atomicAdd(&o->cnt, cnt);
	firstnil = block_reduce(firstnil, [](unsigned long long a, unsigned long long b) { return a < b ? a : b; });
	if (threadIdx.x == 0 && firstnil != ~0ull)
		atomicMin(&o->firstnil, firstnil);
	emin = block_reduce(emin, [](int a, int b) { return a < b ? a : b; });
	if (threadIdx.x == 0 && emin != INT32_MAX)
		atomicMin(&o->emin, emin);
	etop = block_reduce(etop, [](int a, int b) { return a > b ? a : b; });
	if (threadIdx.x == 0 && etop != INT32_MIN)
		atomicMax(&o->etop, etop);
	inf = block_reduce(inf, [](unsigned a, unsigned b) { return a | b; });
	if (threadIdx.x == 0 && inf)
		atomicOr(&o->inf, 1u);
}

// acc += (neg ? -1 : 1) * (m << sh), L-limb two's complement
template <int L>
__device__ __forceinline__ void
limb_add(uint64_t (&acc)[L], bool neg, uint64_t m, int sh)
{
	uint64_t add[L];
#pragma unroll
	for (int q = 0; q < L; q++)
		add[q] = 0;
	const int li = sh >> 6, b = sh & 63;
#pragma unroll
	for (int q = 0; q < L; q++) {
		if (q == li)
			add[q] = m << b;
		else if (q == li + 1 && b)
			add[q] = m >> (64 - b);
	}
	if (neg) {
		// two's complement negation of add
		uint64_t c = 1;
#pragma unroll
		for (int q = 0; q < L; q++) {
			const uint64_t x = ~add[q] + c;
			c = (c && x == 0) ? 1 : 0;
			add[q] = x;
		}
	}
	uint64_t c = 0;
#pragma unroll
	for (int q = 0; q < L; q++) {
		const uint64_t s1 = acc[q] + add[q];
		const uint64_t c1 = s1 < acc[q];
		const uint64_t s2 = s1 + c;
		const uint64_t c2 = s2 < s1;
		acc[q] = s2;
		c = c1 | c2;
	}
}

template <int L>
__device__ __forceinline__ void
limb_addv(uint64_t (&acc)[L], const uint64_t (&x)[L])
{
	uint64_t c = 0;
#pragma unroll
	for (int q = 0; q < L; q++) {
		const uint64_t s1 = acc[q] + x[q];
		const uint64_t c1 = s1 < acc[q];
		const uint64_t s2 = s1 + c;
		const uint64_t c2 = s2 < s1;
		acc[q] = s2;
		c = c1 | c2;
	}
}

// per-workgroup partial sums (L limbs each) of the values in units of 2^emin
template <typename T, int L>
__global__ __launch_bounds__(256) void
k_fsum_acc(const T *base, bool dense, oid off, const oid *oids, oid hseq, BUN n, int emin, uint64_t *part)
{
	__shared__ uint64_t s_acc[4][L];
	uint64_t acc[L];
#pragma unroll
	for (int q = 0; q < L; q++)
		acc[q] = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const T v = fval(base, dense, off, oids, hseq, i);
		bool neg;
		uint64_t m;
		int e;
		if (v != v || isinf((double) v) || !fdecomp(v, neg, m, e))
			continue;
		limb_add<L>(acc, neg, m, e - emin);
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) {
		uint64_t x[L];
#pragma unroll
		for (int q = 0; q < L; q++)
			x[q] = __shfl_xor(acc[q], o);
		limb_addv<L>(acc, x);
	}
	const unsigned w = threadIdx.x >> 6;
	if (__lane_id() == 0)
#pragma unroll
		for (int q = 0; q < L; q++)
			s_acc[w][q] = acc[q];
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int k = 1; k < 4; k++) {
			uint64_t x[L];
#pragma unroll
			for (int q = 0; q < L; q++)
				x[q] = s_acc[k][q];
			limb_addv<L>(acc, x);
		}
#pragma unroll
		for (int q = 0; q < L; q++)
			part[(size_t) blockIdx.x * L + q] = acc[q];
	}
}

template <int L>
__global__ __launch_bounds__(64) void
k_fsum_fin(const uint64_t *part, unsigned nparts, uint64_t *out)
{
	uint64_t acc[L];
#pragma unroll
	for (int q = 0; q < L; q++)
		acc[q] = 0;
	for (unsigned k = threadIdx.x; k < nparts; k += 64) {
		uint64_t x[L];
#pragma unroll
		for (int q = 0; q < L; q++)
			x[q] = part[(size_t) k * L + q];
		limb_addv<L>(acc, x);
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) {
		uint64_t x[L];
#pragma unroll
		for (int q = 0; q < L; q++)
			x[q] = __shfl_xor(acc[q], o);
		limb_addv<L>(acc, x);
	}
	if (threadIdx.x == 0)
#pragma unroll
		for (int q = 0; q < L; q++)
			out[q] = acc[q];
}

// wide exponent spread: a per-workgroup LDS superaccumulator of 32-bit
// digits (weight 2^(32 d - 1074)) held in int64 slots; a value adds its
// shifted mantissa as three signed 32-bit chunks (headroom: 2^31 values)
constexpr int FW_DIG = 68;            // 68 * 32 bits cover 2^-1074 .. 2^1101

template <typename T>
__global__ __launch_bounds__(256) void
k_fsum_wide(const T *base, bool dense, oid off, const oid *oids, oid hseq, BUN n, long long *part)
{
	__shared__ long long dig[FW_DIG];
	if (threadIdx.x < FW_DIG)
		dig[threadIdx.x] = 0;
	__syncthreads();
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const T v = fval(base, dense, off, oids, hseq, i);
		bool neg;
		uint64_t m;
		int e;
		if (v != v || isinf((double) v) || !fdecomp(v, neg, m, e))
			continue;
		const int pos = e + 1074;                 // >= 0
		const int d = pos >> 5;
		const uhge x = (uhge) m << (pos & 31);
#pragma unroll
		for (int k = 0; k < 3; k++) {
			const long long c = (long long) (uint32_t) (x >> (32 * k));
			if (c)
				atomicAdd((unsigned long long *) &dig[d + k], (unsigned long long) (neg ? -c : c));
		}
	}
	__syncthreads();
	if (threadIdx.x < FW_DIG)
		part[(size_t) blockIdx.x * FW_DIG + threadIdx.x] = dig[threadIdx.x];
}

__global__ __launch_bounds__(FW_DIG) void
k_fsum_wide_fin(const long long *part, unsigned nparts, long long *out)
{
	long long t = 0;
	for (unsigned k = 0; k < nparts; k++)
		t += part[(size_t) k * FW_DIG + threadIdx.x];
	out[threadIdx.x] = t;
}

// the L-limb two's-complement integer s times 2^emin rounded to double
// (half to even); false when it is not a finite double
bool
round_to_double(const uint64_t *s, int L, int emin, double *res)
{
	uint64_t a[40] = {0};
	const bool neg = s[L - 1] >> 63;
	for (int q = 0; q < L; q++)
		a[q] = s[q];
	if (neg) {
		uint64_t c = 1;
		for (int q = 0; q < L; q++) {
			a[q] = ~a[q] + c;
			c = (c && a[q] == 0) ? 1 : 0;
		}
	}
	int msb = -1;
	for (int q = L - 1; q >= 0 && msb < 0; q--)
		if (a[q])
			msb = q * 64 + 63 - __builtin_clzll(a[q]);
	if (msb < 0) {
		*res = 0.0;
		return true;
	}
	auto bit = [&](int k) -> uint64_t { return k < 0 ? 0 : (a[k >> 6] >> (k & 63)) & 1; };
	// value = a * 2^emin; top bit weight 2^(msb + emin).  Keep 53 bits, or
	// fewer when the result is subnormal (LSB at 2^-1074)
	int lsb = msb > 52 ? msb - 52 : 0;        // bit index of the result's LSB
	if (lsb + emin < -1074)
		lsb = -1074 - emin;
	uint64_t m = 0;
	for (int k = msb; k >= lsb && k >= 0; k--)
		m = (m << 1) | bit(k);
	if (lsb > msb)
		m = 0;
	// round half to even on the bits below lsb
	const uint64_t g = bit(lsb - 1);
	bool sticky = false;
	for (int k = lsb - 2; k >= 0 && !sticky; k--)
		sticky = bit(k) != 0;
	if (g && (sticky || (m & 1)))
		m++;
	const double d = ldexp((double) m, lsb + emin);   // m < 2^54: exact, scaling exact unless overflow
	if (std::isinf(d))
		return false;
	*res = neg ? -d : d;
	return true;
}

template <typename T>
int
fsum_typed(const mgdk_bat *b, const Cand &ci, double *out, bool *isnil, bool skip_nils, bool nil_if_empty)
{
	hipStream_t st = stream();
	FRange *r = (FRange *) meta_buf();
	FRange init = {0, ~0ull, INT32_MAX, INT32_MIN, 0, 0};
	if (!hip_ok(hipMemcpyAsync(r, &init, sizeof(init), hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	const oid off = ci.dense ? ci.seq - b->hseqbase : 0;
	const T *base = (const T *) b->theap;
	const unsigned grid = grid_for(ci.n, 256 * 16, 4096);
	if (ci.n)
		hipLaunchKernelGGL((k_fsum_range<T>), dim3(grid), dim3(256), 0, st, base, ci.dense, off, ci.oids,
				   b->hseqbase, ci.n, r);
	FRange *h = (FRange *) pinned(sizeof(FRange));
	if (!hip_ok(hipMemcpyAsync(h, r, sizeof(FRange), hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	*isnil = false;
	if (!skip_nils && h->firstnil != ~0ull) {          // dofsum :239-251
		*isnil = true;
		return 0;
	}
	if (h->cnt == 0) {                                  // :304-312
		*isnil = nil_if_empty;
		*out = 0;
		return 0;
	}
	if (h->inf) {
		seterr("22003!overflow in sum aggregate.\n");
		return -1;
	}
	if (h->etop == INT32_MIN) {                         // only zeros
		*out = 0;
		return 0;
	}
	int lg = 0;
	while (((unsigned long long) 1 << lg) < h->cnt)
		lg++;
	const int range = h->etop - h->emin + lg + 1;
	const int L = range <= 127 ? 2 : range <= 255 ? 4 : 0;
	if (L == 0) {
		// wide spread: LDS superaccumulator of 32-bit digits
		if (h->cnt >= ((unsigned long long) 1 << 31)) {
			seterr("42000!BATsum: more than 2^31 floating-point values with a wide exponent spread");
			return -1;
		}
		DevBuf wpart((size_t) grid * FW_DIG * 8 + 64), wout(FW_DIG * 8);
		if (!wpart.p || !wout.p)
			return -1;
		hipLaunchKernelGGL((k_fsum_wide<T>), dim3(grid), dim3(256), 0, st, base, ci.dense, off, ci.oids,
				   b->hseqbase, ci.n, wpart.as<long long>());
		hipLaunchKernelGGL(k_fsum_wide_fin, dim3(1), dim3(FW_DIG), 0, st, wpart.as<long long>(), grid,
				   wout.as<long long>());
		long long *hd = (long long *) pinned(FW_DIG * 8);
		if (!hip_ok(hipMemcpyAsync(hd, wout.p, FW_DIG * 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			return -1;
		// digits -> 36 two's-complement 64-bit limbs (weight of bit 0: 2^-1074)
		uint64_t limb[40] = {0};
		hge carry = 0;
		for (int q = 0; q < 36; q++) {
			hge acc = carry;
			for (int half = 0; half < 2; half++) {
				const int d = 2 * q + half;
				if (d < FW_DIG)
					acc += (hge) hd[d] << (32 * half);
			}
			limb[q] = (uint64_t) acc;
			carry = acc >> 64;                       // arithmetic shift
		}
		if (!round_to_double(limb, 36, -1074, out)) {
			seterr("22003!overflow in sum aggregate.\n");
			return -1;
		}
		return 0;
	}
	DevBuf part((size_t) grid * L * 8 + 64);
	uint64_t *dres = (uint64_t *) meta_buf() + 8;
	if (!part.p)
		return -1;
	if (L == 2) {
		hipLaunchKernelGGL((k_fsum_acc<T, 2>), dim3(grid), dim3(256), 0, st, base, ci.dense, off, ci.oids,
				   b->hseqbase, ci.n, h->emin, part.as<uint64_t>());
		hipLaunchKernelGGL((k_fsum_fin<2>), dim3(1), dim3(64), 0, st, part.as<uint64_t>(), grid, dres);
	} else {
		hipLaunchKernelGGL((k_fsum_acc<T, 4>), dim3(grid), dim3(256), 0, st, base, ci.dense, off, ci.oids,
				   b->hseqbase, ci.n, h->emin, part.as<uint64_t>());
		hipLaunchKernelGGL((k_fsum_fin<4>), dim3(1), dim3(64), 0, st, part.as<uint64_t>(), grid, dres);
	}
	uint64_t *hs = (uint64_t *) pinned(64);
	const int emin = h->emin;
	if (!hip_ok(hipMemcpyAsync(hs, dres, L * 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	if (!round_to_double(hs, L, emin, out)) {
		seterr("22003!overflow in sum aggregate.\n");
		return -1;
	}
	return 0;
}

}  // namespace

// BATsum of a flt / dbl column (called by mgdk_BATsum, aggr.hip)
int
mgdk_fsum(void *res, int tp, mgdk_bat *b, mgdk_bat *s, bool skip_nils, bool nil_if_empty)
{
	if (!(tp == MGDK_dbl || (tp == MGDK_flt && b->ttype == MGDK_flt))) {
		seterr("type combination (sum(%s)->%s) not supported.\n", atomname(b->ttype), atomname(tp));
		return -1;
	}
	ProfScope prof("sum");
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return -1;
	double d = 0;
	bool nil = false;
	const int rc = b->ttype == MGDK_flt ? fsum_typed<float>(b, ci, &d, &nil, skip_nils, nil_if_empty)
					    : fsum_typed<double>(b, ci, &d, &nil, skip_nils, nil_if_empty);
	if (rc < 0)
		return -1;
	if (tp == MGDK_dbl) {
		*(double *) res = nil ? __builtin_nan("") : d;
		return 0;
	}
	const float f = (float) d;                          // :400-406
	if (!nil && std::isinf(f)) {
		seterr("22003!overflow in sum aggregate.\n");
		return -1;
	}
	*(float *) res = nil ? __builtin_nanf("") : f;
	return 0;
}

// ---- grouped: BATgroupsum of flt / dbl (dofsum with gids, gdk_aggr.c:183) --
// Per group an exact fixed-point sum in 32-bit digits (weights 2^(32 d +
// emin), int64 slots: 2^31 values of headroom), three signed chunks per
// value; workgroup-private in LDS when the groups' digits fit, flushed with
// one global atomic per non-zero digit, else global atomics directly.
namespace {

template <typename T, bool LDS>
__global__ __launch_bounds__(256) void
k_fgsum(const T *base, bool dense, oid off, const oid *oids, oid hseq, BUN n, const oid *gids, oid gseq, oid gmin,
	BUN ngrp, int emin, int nd, long long *gdig, unsigned long long *gcnt, unsigned *gnil)
{
	extern __shared__ __attribute__((aligned(16))) long long sdig[];
	long long *dig = gdig;
	unsigned long long *cnt = gcnt;
	unsigned *nil = gnil;
	const BUN nslots = ngrp * (BUN) nd;
	if (LDS) {
		dig = sdig;
		cnt = (unsigned long long *) (sdig + nslots);
		nil = (unsigned *) (cnt + ngrp);
		for (BUN q = threadIdx.x; q < nslots; q += blockDim.x)
			dig[q] = 0;
		for (BUN q = threadIdx.x; q < ngrp; q += blockDim.x) {
			cnt[q] = 0;
			nil[q] = 0;
		}
		__syncthreads();
	}
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const oid g = gids ? gids[i] : gseq + i;
		if (g < gmin || g - gmin >= ngrp)
			continue;
		const BUN gi = g - gmin;
		const T v = fval(base, dense, off, oids, hseq, i);
		if (v != v) {
			atomicOr(&nil[gi], 1u);
			continue;
		}
		atomicAdd(&cnt[gi], 1ull);
		bool neg;
		uint64_t m;
		int e;
		if (isinf((double) v) || !fdecomp(v, neg, m, e))
			continue;
		const int pos = e - emin;
		const int d = pos >> 5;
		const uhge x = (uhge) m << (pos & 31);
#pragma unroll
		for (int k = 0; k < 3; k++) {
			const long long c = (long long) (uint32_t) (x >> (32 * k));
			if (c)
				atomicAdd((unsigned long long *) &dig[gi * nd + d + k], (unsigned long long) (neg ? -c : c));
		}
	}
	if (LDS) {
		__syncthreads();
		for (BUN q = threadIdx.x; q < nslots; q += blockDim.x)
			if (dig[q])
				atomicAdd((unsigned long long *) &gdig[q], (unsigned long long) dig[q]);
		for (BUN q = threadIdx.x; q < ngrp; q += blockDim.x) {
			if (cnt[q])
				atomicAdd(&gcnt[q], cnt[q]);
			if (nil[q])
				atomicOr(&gnil[q], 1u);
		}
	}
}

template <typename T>
int
fgroupsum_typed(const mgdk_bat *b, const Cand &ci, const oid *gids, oid gseq, oid gmin, BUN ngrp, bool skip_nils,
		int tp, void *res, bool *nils)
{
	hipStream_t st = stream();
	FRange *r = (FRange *) meta_buf();
	FRange init = {0, ~0ull, INT32_MAX, INT32_MIN, 0, 0};
	if (!hip_ok(hipMemcpyAsync(r, &init, sizeof(init), hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	const oid off = ci.dense ? ci.seq - b->hseqbase : 0;
	const T *base = (const T *) b->theap;
	const unsigned grid = grid_for(ci.n, 256 * 16, 4096);
	if (ci.n)
		hipLaunchKernelGGL((k_fsum_range<T>), dim3(grid), dim3(256), 0, st, base, ci.dense, off, ci.oids,
				   b->hseqbase, ci.n, r);
	FRange *h = (FRange *) pinned(sizeof(FRange));
	if (!hip_ok(hipMemcpyAsync(h, r, sizeof(FRange), hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	if (h->inf) {
		seterr("22003!overflow in sum aggregate.\n");
		return -1;
	}
	if (h->cnt >= ((unsigned long long) 1 << 31)) {
		seterr("42000!BATgroupsum: more than 2^31 floating-point values are not supported on the device path");
		return -1;
	}
	const int emin = h->etop == INT32_MIN ? 0 : h->emin;
	const int nd = h->etop == INT32_MIN ? 4 : (h->etop - emin + 31) / 32 + 4;
	const BUN nslots = ngrp * (BUN) nd;
	DevBuf dig(nslots * 8 + 64), cnt(ngrp * 8 + 64), nilf(ngrp * 4 + 64);
	if (!dig.p || !cnt.p || !nilf.p || !hip_ok(hipMemsetAsync(dig.p, 0, nslots * 8 + 64, st), "memset") ||
	    !hip_ok(hipMemsetAsync(cnt.p, 0, ngrp * 8 + 64, st), "memset") ||
	    !hip_ok(hipMemsetAsync(nilf.p, 0, ngrp * 4 + 64, st), "memset"))
		return -1;
	const size_t lds = nslots * 8 + ngrp * 12 + 16;
	if (ci.n) {
		if (lds <= 48 * 1024)
			hipLaunchKernelGGL((k_fgsum<T, true>), dim3(grid), dim3(256), lds, st, base, ci.dense, off, ci.oids,
					   b->hseqbase, ci.n, gids, gseq, gmin, ngrp, emin, nd, dig.as<long long>(),
					   cnt.as<unsigned long long>(), nilf.as<unsigned>());
		else
			hipLaunchKernelGGL((k_fgsum<T, false>), dim3(grid), dim3(256), 0, st, base, ci.dense, off, ci.oids,
					   b->hseqbase, ci.n, gids, gseq, gmin, ngrp, emin, nd, dig.as<long long>(),
					   cnt.as<unsigned long long>(), nilf.as<unsigned>());
	}
	std::vector<long long> hd(nslots + 1);
	std::vector<unsigned long long> hc(ngrp + 1);
	std::vector<unsigned> hn(ngrp + 1);
	if (!hip_ok(hipMemcpyAsync(hd.data(), dig.p, nslots * 8, hipMemcpyDeviceToHost, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(hc.data(), cnt.p, ngrp * 8, hipMemcpyDeviceToHost, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(hn.data(), nilf.p, ngrp * 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	*nils = false;
	for (BUN k = 0; k < ngrp; k++) {
		bool nil = (!skip_nils && hn[k]) || hc[k] == 0;      // dofsum :239-251, :304-312
		double d = 0;
		if (!nil) {
			uint64_t limb[40] = {0};
			const int nl = nd / 2 + 2;
			hge carry = 0;
			for (int q = 0; q < nl; q++) {
				hge acc = carry;
				for (int half = 0; half < 2; half++) {
					const int j = 2 * q + half;
					if (j < nd)
						acc += (hge) hd[k * nd + j] << (32 * half);
				}
				limb[q] = (uint64_t) acc;
				carry = acc >> 64;
			}
			if (!round_to_double(limb, nl, emin, &d)) {
				seterr("22003!overflow in sum aggregate.\n");
				return -1;
			}
		}
		if (tp == MGDK_dbl) {
			((double *) res)[k] = nil ? __builtin_nan("") : d;
		} else {
			const float f = (float) d;
			if (!nil && std::isinf(f)) {
				seterr("22003!overflow in sum aggregate.\n");
				return -1;
			}
			((float *) res)[k] = nil ? __builtin_nanf("") : f;
		}
		*nils |= nil;
	}
	return 0;
}

}  // namespace

// grouped float sums into res[0..ngrp) (called by mgdk_BATgroupsum, aggr.hip)
int
mgdk_fgroupsum(const mgdk_bat *b, const Cand &ci, const oid *gids, oid gseq, oid gmin, BUN ngrp, bool skip_nils,
	       int tp, void *res, bool *nils)
{
	if (!(tp == MGDK_dbl || (tp == MGDK_flt && b->ttype == MGDK_flt))) {
		seterr("type combination (sum(%s)->%s) not supported.\n", atomname(b->ttype), atomname(tp));
		return -1;
	}
	return b->ttype == MGDK_flt ? fgroupsum_typed<float>(b, ci, gids, gseq, gmin, ngrp, skip_nils, tp, res, nils)
				    : fgroupsum_typed<double>(b, ci, gids, gseq, gmin, ngrp, skip_nils, tp, res, nils);
}
