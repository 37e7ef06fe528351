// tpch.hip -- synthetic TPC-H lineitem generation in HBM and the fused
// Q6 / Q1 column pipelines.
//
// Generation restates oracle/tpch_gen.c (the same counter-based splitmix64
// values, so a row range can be generated on any GPU shard and checked
// against the CPU oracle bit for bit).
//
// Fused pipelines: one streaming pass over the lineitem columns computing
// exactly what the op-at-a-time MAL plans compute:
//   Q6  select(shipdate in [d0,d1)) -> select(disc in [dlo,dhi]) ->
//       thetaselect(qty < qmax) -> project price, disc -> price*disc (hge)
//       -> sum.  28 B/row: each lane handles 4 consecutive rows with 16-B
//       loads (shipdate 1 x 16 B, each lng column 2 x 16 B), keeps an exact
//       128-bit partial, one pair of 64-bit atomics per wave at the end.
//   Q1  thetaselect(shipdate <= dmax) -> group(returnflag) ->
//       subgroup(linestatus) -> sums of qty, price, price*(100-disc),
//       price*(100-disc)*(100+tax), disc and counts (avg3 derives from the
//       exact sums).  38 B/row.  The few (returnflag, linestatus) keys are
//       discovered on a prefix with their first-occurrence rows, then the
//       main pass keeps K register-resident accumulator sets per lane
//       (K <= 8, predicated adds, no atomics in the loop).  Any row whose key
//       was not in the prefix, any nil, or any value outside the ranges for
//       which the 64-bit lane partials are exact makes the call fall back to
//       the op-at-a-time device plan (pipelines.hip), so results are always
//       the reference's.
#include <mutex>
#include <algorithm>
#include <vector>

#include <atomic>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

__device__ __host__ __forceinline__ uint64_t
mix64(uint64_t z)
{
	z += 0x9e3779b97f4a7c15ull;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t
rnd(uint64_t seed, uint64_t row, uint64_t col)
{
	return mix64(seed ^ mix64(row * 16 + col));
}

__device__ __forceinline__ int64_t
urange(uint64_t r, int64_t lo, int64_t hi)
{
	uint64_t span = (uint64_t) (hi - lo + 1);
	return lo + (int64_t) __umul64hi(r, span);
}

constexpr int ORDERDATE_DAYS = 2405;   // 1998-08-02 - 1992-01-01
constexpr int CURRENTDATE_DAY = 1263;  // 1995-06-17 - 1992-01-01
constexpr int TABLE_DAYS = ORDERDATE_DAYS + 121 + 30 + 2;

__global__ __launch_bounds__(256) void
k_lineitem(uint64_t seed, uint64_t row0, uint64_t n, uint64_t sf_parts, const int32_t *table,
	   int32_t *shipdate, int64_t *quantity, int64_t *extendedprice, int64_t *discount,
	   int64_t *tax, uint8_t *returnflag, uint8_t *linestatus)
{
	for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n;
	     i += (uint64_t) gridDim.x * blockDim.x) {
		uint64_t row = row0 + i;
		int od = (int) urange(rnd(seed, row, 0), 0, ORDERDATE_DAYS);
		int sd = od + (int) urange(rnd(seed, row, 1), 1, 121);
		int rd = sd + (int) urange(rnd(seed, row, 2), 1, 30);
		int64_t q = urange(rnd(seed, row, 3), 1, 50);
		int64_t pk = urange(rnd(seed, row, 4), 1, (int64_t) sf_parts);
		int64_t rp = 90000 + ((pk / 10) % 20001) + 100 * (pk % 1000);
		shipdate[i] = table[sd];
		quantity[i] = q * 100;
		extendedprice[i] = q * rp;
		discount[i] = urange(rnd(seed, row, 5), 0, 10);
		tax[i] = urange(rnd(seed, row, 6), 0, 8);
		returnflag[i] = rd <= CURRENTDATE_DAY ? ((rnd(seed, row, 7) >> 63) ? 16 : 0) : 8;
		linestatus[i] = sd > CURRENTDATE_DAY ? 8 : 0;
	}
}

int
isleap(int y)
{
	return y % 4 == 0 && (y % 100 != 0 || y % 400 == 0);
}

int32_t
mkdate(int y, int m, int d)
{
	return (int32_t) ((((uint32_t) ((y + 4712) * 12 + m - 1)) << 5) | (uint32_t) d);
}

std::vector<int32_t>
date_table()
{
	static const int cum[13] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334, 365};
	std::vector<int32_t> t(TABLE_DAYS);
	int y = 1992, doy = 0;
	for (int i = 0; i < TABLE_DAYS; i++) {
		int m = 1;
		while (m < 12 && doy >= cum[m] + (m >= 2 && isleap(y)))
			m++;
		int start = cum[m - 1] + (m > 2 && isleap(y));
		t[i] = mkdate(y, m, doy - start + 1);
		if (++doy == 365 + isleap(y)) {
			doy = 0;
			y++;
		}
	}
	return t;
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

__device__ __forceinline__ hge
wave_sum128(hge s)
{
	for (int o = 32; o > 0; o >>= 1) {
		unsigned long long lo = __shfl_xor((unsigned long long) (uhge) s, o);
		unsigned long long hi = __shfl_xor((unsigned long long) ((uhge) s >> 64), o);
		s += (hge) (((uhge) hi << 64) | lo);
	}
	return s;
}

// ---- Q6 -------------------------------------------------------------------
struct Q6Args {
	const int32_t *sd;
	const int64_t *disc, *qty, *price;
	uint64_t n;          // rows
	int32_t d0, d1;
	int64_t dlo, dhi, qmax;
	unsigned long long *out;   // [2] 128-bit revenue
	struct Q6Part *parts;      // k_q6c / k_q6s: one partial per workgroup (NULL: atomics into out)
};

// one workgroup's exact revenue and (k_q6s) line count: written once per
// workgroup and summed by k_q6_fin -- a same-address atomic from every wave
// of a 16 Ki-wave grid serialised at one L2 channel (0.47 vs 0.26 ms at SF10)
struct Q6Part {
	unsigned long long lo, hi, lines, pad;
};

// the workgroup's sum of the waves' partials (called by every thread)
__device__ __forceinline__ void
q6_publish(const Q6Args &a, hge acc, uint32_t lines)
{
	__shared__ hge s_acc[4];
	__shared__ uint32_t s_lines[4];
	acc = wave_sum128(acc);
	const unsigned w = threadIdx.x >> 6;
	if (__lane_id() == 0) {
		s_acc[w] = acc;
		s_lines[w] = lines;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		hge t = 0;
		unsigned long long l = 0;
		for (unsigned q = 0; q < blockDim.x / 64; q++) {
			t += s_acc[q];
			l += s_lines[q];
		}
		Q6Part pt;
		pt.lo = (unsigned long long) (uhge) t;
		pt.hi = (unsigned long long) ((uhge) t >> 64);
		pt.lines = l;
		pt.pad = 0;
		a.parts[blockIdx.x] = pt;
	}
}

// out[0..1] = exact sum of the partials, out[2] = their line count
__global__ __launch_bounds__(1024) void
k_q6_fin(const Q6Part *parts, uint32_t n, unsigned long long *out)
{
	__shared__ hge s_acc[16];
	__shared__ unsigned long long s_l[16];
	hge t = 0;
	unsigned long long l = 0;
	for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
		const Q6Part p = parts[i];
		t += (hge) (((uhge) p.hi << 64) | p.lo);
		l += p.lines;
	}
	t = wave_sum128(t);
	for (int o = 32; o > 0; o >>= 1)
		l += __shfl_xor(l, o);
	const unsigned w = threadIdx.x >> 6;
	if (__lane_id() == 0) {
		s_acc[w] = t;
		s_l[w] = l;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		hge r = 0;
		unsigned long long lt = 0;
		for (unsigned q = 0; q < blockDim.x / 64; q++) {
			r += s_acc[q];
			lt += s_l[q];
		}
		out[0] = (unsigned long long) (uhge) r;
		out[1] = (unsigned long long) ((uhge) r >> 64);
		out[2] = lt;
	}
}

__device__ __forceinline__ hge
q6_row(const Q6Args &a, int32_t sd, int64_t di, int64_t q, int64_t p)
{
	bool ok = sd != INT32_MIN && sd >= a.d0 && sd < a.d1 && di != INT64_MIN && di >= a.dlo &&
		  di <= a.dhi && q != INT64_MIN && q < a.qmax && p != INT64_MIN;
	return ok ? (hge) p * (hge) di : (hge) 0;
}

template <bool NT, typename V>
__device__ __forceinline__ V
ldv(const V *p)
{
	if constexpr (NT)
		return __builtin_nontemporal_load(p);
	else
		return *p;
}

template <int UNROLL, bool NT = false>
__global__ __launch_bounds__(256) void
k_q6(Q6Args a)
{
	typedef int32_t i4 __attribute__((ext_vector_type(4)));
	typedef int64_t l2 __attribute__((ext_vector_type(2)));
	hge acc = 0;
	const uint64_t nq = a.n / 4;   // full quads
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	uint64_t q = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
	for (; q + (UNROLL - 1) * stride < nq; q += UNROLL * stride) {
		i4 sd[UNROLL];
		l2 d0[UNROLL], d1[UNROLL], q0[UNROLL], q1[UNROLL], p0[UNROLL], p1[UNROLL];
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			uint64_t r = (q + u * stride) * 4;
			sd[u] = ldv<NT>((const i4 *) (a.sd + r));
			d0[u] = ldv<NT>((const l2 *) (a.disc + r));
			d1[u] = ldv<NT>((const l2 *) (a.disc + r + 2));
			q0[u] = ldv<NT>((const l2 *) (a.qty + r));
			q1[u] = ldv<NT>((const l2 *) (a.qty + r + 2));
			p0[u] = ldv<NT>((const l2 *) (a.price + r));
			p1[u] = ldv<NT>((const l2 *) (a.price + r + 2));
		}
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			acc += q6_row(a, sd[u][0], d0[u][0], q0[u][0], p0[u][0]);
			acc += q6_row(a, sd[u][1], d0[u][1], q0[u][1], p0[u][1]);
			acc += q6_row(a, sd[u][2], d1[u][0], q1[u][0], p1[u][0]);
			acc += q6_row(a, sd[u][3], d1[u][1], q1[u][1], p1[u][1]);
		}
	}
	for (; q < nq; q += stride) {
		uint64_t r = q * 4;
		for (int k = 0; k < 4; k++)
			acc += q6_row(a, a.sd[r + k], a.disc[r + k], a.qty[r + k], a.price[r + k]);
	}
	// tail rows
	if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
		uint64_t r = nq * 4 + threadIdx.x;
		acc += q6_row(a, a.sd[r], a.disc[r], a.qty[r], a.price[r]);
	}
	acc = wave_sum128(acc);
	if (__lane_id() == 0 && acc != 0)
		atomic_add128(a.out, acc);
}

// Contiguous-per-instruction variant: a wave owns a 256-row chunk; lane l
// takes rows {2l, 2l+1, 128+2l, 128+2l+1}, so every load instruction of the
// wave covers one contiguous range (512 B of shipdate, 1 KiB of each lng).
template <int UNROLL, bool NT = false>
__global__ __launch_bounds__(256) void
k_q6c(Q6Args a)
{
	typedef int32_t i2 __attribute__((ext_vector_type(2)));
	typedef int64_t l2 __attribute__((ext_vector_type(2)));
	hge acc = 0;
	const unsigned lane = __lane_id();
	const uint64_t nch = a.n / 256;
	const uint64_t nw = (uint64_t) gridDim.x * (blockDim.x / 64);
	uint64_t c = ((uint64_t) blockIdx.x * blockDim.x + threadIdx.x) / 64;
	for (; c + (UNROLL - 1) * nw < nch; c += UNROLL * nw) {
		i2 s0[UNROLL], s1[UNROLL];
		l2 d0[UNROLL], d1[UNROLL], q0[UNROLL], q1[UNROLL], p0[UNROLL], p1[UNROLL];
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const uint64_t r0 = (c + u * nw) * 256 + 2 * lane, r1 = r0 + 128;
			s0[u] = ldv<NT>((const i2 *) (a.sd + r0));
			s1[u] = ldv<NT>((const i2 *) (a.sd + r1));
			d0[u] = ldv<NT>((const l2 *) (a.disc + r0));
			d1[u] = ldv<NT>((const l2 *) (a.disc + r1));
			q0[u] = ldv<NT>((const l2 *) (a.qty + r0));
			q1[u] = ldv<NT>((const l2 *) (a.qty + r1));
			p0[u] = ldv<NT>((const l2 *) (a.price + r0));
			p1[u] = ldv<NT>((const l2 *) (a.price + r1));
		}
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			acc += q6_row(a, s0[u][0], d0[u][0], q0[u][0], p0[u][0]);
			acc += q6_row(a, s0[u][1], d0[u][1], q0[u][1], p0[u][1]);
			acc += q6_row(a, s1[u][0], d1[u][0], q1[u][0], p1[u][0]);
			acc += q6_row(a, s1[u][1], d1[u][1], q1[u][1], p1[u][1]);
		}
	}
	for (; c < nch; c += nw) {
		const uint64_t r0 = c * 256 + 2 * lane, r1 = r0 + 128;
		for (int k = 0; k < 2; k++) {
			acc += q6_row(a, a.sd[r0 + k], a.disc[r0 + k], a.qty[r0 + k], a.price[r0 + k]);
			acc += q6_row(a, a.sd[r1 + k], a.disc[r1 + k], a.qty[r1 + k], a.price[r1 + k]);
		}
	}
	if (blockIdx.x == 0 && threadIdx.x < (a.n & 255)) {
		const uint64_t r = nch * 256 + threadIdx.x;
		acc += q6_row(a, a.sd[r], a.disc[r], a.qty[r], a.price[r]);
	}
	q6_publish(a, acc, 0);
}

// Predicate-cascade variant (late materialisation inside one pass): the
// same 256-row chunks as k_q6c, but a column is read only for the rows
// still qualifying -- shipdate for every row, discount where the date
// holds, quantity where date and discount hold, extendedprice where all
// three do -- as the reference's candidate lists do (each
// select / projection only touches the previous candidates).  A lane whose
// two rows are both out points its load at one shared zero line (an L2
// hit, no HBM traffic), so every load stays unconditional and in flight; a
// 128-B line of a column is fetched only when one of its 16 rows is still
// in.  The workgroup partials carry the count of those lines (the
// roofline's byte count, summed by k_q6_fin into out[2]).  The
// zero lines are spread over 64 KiB (one 16-B slot per lane of 64 waves):
// every inactive lane of the chip on ONE line serialised on its L2 channel.
constexpr uint32_t Q6_ZBYTES = ZERO_REGION;
// BUF: the discount / quantity / extendedprice loads are raw buffer loads
// through a per-chunk descriptor (wave-uniform base, 2 KiB range); a lane
// with no live row passes an out-of-range offset, which the descriptor's
// range check turns into zeros with no memory access at all
// (cdna_hip_programming.md T15 recipe) -- instead of a zero-region load
typedef unsigned int q6u4 __attribute__((ext_vector_type(4)));
template <bool BUF>
__device__ __forceinline__ void
q6_ld(const int64_t *col, uint64_t chunk, uint64_t r, unsigned boff, bool live, const void *z, long long *out)
{
	typedef long long l2 __attribute__((ext_vector_type(2)));
	if constexpr (BUF) {
		// dword3 0x00020000 is the gfx950 (CDNA3/4) descriptor layout whose
		// range check returns zeros for the dead lanes' out-of-range offset;
		// other families lay the word out differently
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "q6_ld<BUF>: buffer descriptor word 3 is laid out for gfx942 / gfx950 only"
#endif
		__amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *) (col + chunk * 256), (short) 0, 2048,
									      0x00020000);
		const q6u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, live ? boff : 0x80000000u, 0, 0);
		out[0] = (long long) (((unsigned long long) v.y << 32) | v.x);
		out[1] = (long long) (((unsigned long long) v.w << 32) | v.z);
	} else {
		const l2 v = __builtin_nontemporal_load(live ? (const l2 *) (col + r) : (const l2 *) z);
		out[0] = v.x;
		out[1] = v.y;
	}
}

template <int UNROLL, bool BUF = false>
__global__ __launch_bounds__(256) void
k_q6s(Q6Args a, const int64_t *zline)
{
	typedef int32_t i2 __attribute__((ext_vector_type(2)));
	typedef int64_t l2 __attribute__((ext_vector_type(2)));
	hge acc = 0;
	uint32_t nlines = 0;
	const unsigned lane = __lane_id();
	const uint64_t nch = a.n / 256;
	const uint64_t nw = (uint64_t) gridDim.x * (blockDim.x / 64);
	const l2 *z = (const l2 *) zline + ((((uint64_t) blockIdx.x * blockDim.x + threadIdx.x)) & (Q6_ZBYTES / 16 - 1));
	// 128-B lines (8 lanes x 16 B) with at least one active lane in a ballot
	auto lines = [](uint64_t b) -> uint32_t {
		b |= b >> 1;
		b |= b >> 2;
		b |= b >> 4;
		return (uint32_t) __popcll(b & 0x0101010101010101ull);
	};
	uint64_t c = ((uint64_t) blockIdx.x * blockDim.x + threadIdx.x) / 64;
	for (; c + (UNROLL - 1) * nw < nch; c += UNROLL * nw) {
		i2 s0[UNROLL], s1[UNROLL];
		l2 v0[UNROLL], v1[UNROLL], d0[UNROLL], d1[UNROLL];
		bool m[UNROLL][4];
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const uint64_t r0 = (c + u * nw) * 256 + 2 * lane, r1 = r0 + 128;
			s0[u] = __builtin_nontemporal_load((const i2 *) (a.sd + r0));
			s1[u] = __builtin_nontemporal_load((const i2 *) (a.sd + r1));
		}
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const int32_t sd[4] = {s0[u][0], s0[u][1], s1[u][0], s1[u][1]};
#pragma unroll
			for (int k = 0; k < 4; k++)
				m[u][k] = sd[k] != INT32_MIN && sd[k] >= a.d0 && sd[k] < a.d1;
		}
		// discount where the date holds
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const uint64_t r0 = (c + u * nw) * 256 + 2 * lane, r1 = r0 + 128;
			const bool a0 = m[u][0] || m[u][1], a1 = m[u][2] || m[u][3];
			nlines += lines(__ballot(a0)) + lines(__ballot(a1));
			{
				long long t0[2], t1[2];
				q6_ld<BUF>(a.disc, c + u * nw, r0, 16u * lane, a0, z, t0);
				q6_ld<BUF>(a.disc, c + u * nw, r1, 1024u + 16u * lane, a1, z, t1);
				d0[u].x = t0[0];
				d0[u].y = t0[1];
				d1[u].x = t1[0];
				d1[u].y = t1[1];
			}
		}
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const int64_t di[4] = {d0[u][0], d0[u][1], d1[u][0], d1[u][1]};
#pragma unroll
			for (int k = 0; k < 4; k++)
				m[u][k] = m[u][k] && di[k] != INT64_MIN && di[k] >= a.dlo && di[k] <= a.dhi;
		}
		// quantity where date and discount hold
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const uint64_t r0 = (c + u * nw) * 256 + 2 * lane, r1 = r0 + 128;
			const bool a0 = m[u][0] || m[u][1], a1 = m[u][2] || m[u][3];
			nlines += lines(__ballot(a0)) + lines(__ballot(a1));
			{
				long long t0[2], t1[2];
				q6_ld<BUF>(a.qty, c + u * nw, r0, 16u * lane, a0, z, t0);
				q6_ld<BUF>(a.qty, c + u * nw, r1, 1024u + 16u * lane, a1, z, t1);
				v0[u].x = t0[0];
				v0[u].y = t0[1];
				v1[u].x = t1[0];
				v1[u].y = t1[1];
			}
		}
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const int64_t q[4] = {v0[u][0], v0[u][1], v1[u][0], v1[u][1]};
#pragma unroll
			for (int k = 0; k < 4; k++)
				m[u][k] = m[u][k] && q[k] != INT64_MIN && q[k] < a.qmax;
		}
		// extendedprice where all three hold
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const uint64_t r0 = (c + u * nw) * 256 + 2 * lane, r1 = r0 + 128;
			const bool a0 = m[u][0] || m[u][1], a1 = m[u][2] || m[u][3];
			nlines += lines(__ballot(a0)) + lines(__ballot(a1));
			{
				long long t0[2], t1[2];
				q6_ld<BUF>(a.price, c + u * nw, r0, 16u * lane, a0, z, t0);
				q6_ld<BUF>(a.price, c + u * nw, r1, 1024u + 16u * lane, a1, z, t1);
				v0[u].x = t0[0];
				v0[u].y = t0[1];
				v1[u].x = t1[0];
				v1[u].y = t1[1];
			}
		}
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const int64_t p[4] = {v0[u][0], v0[u][1], v1[u][0], v1[u][1]};
			const int64_t di[4] = {d0[u][0], d0[u][1], d1[u][0], d1[u][1]};
#pragma unroll
			for (int k = 0; k < 4; k++)
				if (m[u][k] && p[k] != INT64_MIN)
					acc += (hge) p[k] * (hge) di[k];
		}
	}
	for (; c < nch; c += nw) {
		const uint64_t r0 = c * 256 + 2 * lane, r1 = r0 + 128;
		for (int k = 0; k < 2; k++) {
			acc += q6_row(a, a.sd[r0 + k], a.disc[r0 + k], a.qty[r0 + k], a.price[r0 + k]);
			acc += q6_row(a, a.sd[r1 + k], a.disc[r1 + k], a.qty[r1 + k], a.price[r1 + k]);
		}
		nlines += 3 * 16;                        // counted as fully read
	}
	if (blockIdx.x == 0 && threadIdx.x < (a.n & 255)) {
		const uint64_t r = nch * 256 + threadIdx.x;
		acc += q6_row(a, a.sd[r], a.disc[r], a.qty[r], a.price[r]);
	}
	q6_publish(a, acc, nlines);
}

__global__ __launch_bounds__(256) void
k_q6_scalar(Q6Args a)
{
	hge acc = 0;
	for (uint64_t r = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; r < a.n; r += (uint64_t) gridDim.x * blockDim.x)
		acc += q6_row(a, a.sd[r], a.disc[r], a.qty[r], a.price[r]);
	acc = wave_sum128(acc);
	if (__lane_id() == 0 && acc != 0)
		atomic_add128(a.out, acc);
}

// ---- Q1 -------------------------------------------------------------------
constexpr int Q1_MAXK = 8;

struct Q1Args {
	const int32_t *sd;
	const uint8_t *rf, *ls;
	const int64_t *qty, *price, *disc, *tax;
	uint64_t n;
	int32_t dmax;
	int K;
	uint32_t codes[Q1_MAXK];          // rf << 8 | ls
	unsigned long long *acc;          // [K][12]: qty, price, discprice(2), charge(2), disc, count (+pad)
	uint32_t *flags;                  // [0] unknown key, [1] out of range / nil, [2] outside narrow bounds
	int64_t plim;                     // narrow pass: |qty|, |price| < plim
};

#ifndef MGDK_Q1_MODE
#define MGDK_Q1_MODE 2
#endif
#ifndef MGDK_Q1_UNROLL
#define MGDK_Q1_UNROLL 2
#endif
#ifndef MGDK_Q1_BLOCKS
#define MGDK_Q1_BLOCKS 256
#endif
#ifndef MGDK_Q1_LAYOUT
#define MGDK_Q1_LAYOUT 1
#endif

// Narrow Q1 pass: when |qty|, |price| < plim and |disc|, |tax| < 2^8 every
// per-lane partial fits 64 bits (|charge| < plim * 2^18 per row, so
// plim = 2^45 / rows-per-lane, capped at 2^31, set by the host), so a row costs 64-bit arithmetic only; hge appears at the wave
// reduction.  A row outside the bounds raises flags[2] and the host reruns
// the wide (hge) pass.  LDSACC keeps the five sums of each group in
// lane-private LDS slots (one ds_add_u64 per sum per row, no per-group
// predication); otherwise every group's registers take a predicated add.
constexpr int64_t Q1_SMALL = (int64_t) 1 << 8;

template <int K, bool LDSACC, int LAYOUT>
__global__ __launch_bounds__(256) void
k_q1n(Q1Args a)
{
	__shared__ unsigned long long lacc[LDSACC ? K * 5 * 256 : 1];
	int64_t s[K][5];
	uint32_t cnt[K];
#pragma unroll
	for (int k = 0; k < K; k++) {
		cnt[k] = 0;
#pragma unroll
		for (int j = 0; j < 5; j++)
			s[k][j] = 0;
	}
	if (LDSACC) {
		for (int i = threadIdx.x; i < K * 5 * 256; i += 256)
			lacc[i] = 0;
		__syncthreads();
	}
	uint32_t unknown = 0, bad = 0;
	typedef int32_t i4 __attribute__((ext_vector_type(4)));
	typedef int64_t l2 __attribute__((ext_vector_type(2)));
	typedef uint8_t u4 __attribute__((ext_vector_type(4)));
	const uint64_t nq = a.n / 4;
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	const uint64_t pl = (uint64_t) a.plim;
	auto row = [&](int32_t d, uint32_t code, int64_t q, int64_t p, int64_t di, int64_t t) {
		if (d == INT32_MIN || d > a.dmax)
			return;
		bad |= ((uint64_t) (q + a.plim) >= 2 * pl) | ((uint64_t) (p + a.plim) >= 2 * pl) |
		       ((uint64_t) (di + Q1_SMALL) >= 2 * Q1_SMALL) | ((uint64_t) (t + Q1_SMALL) >= 2 * Q1_SMALL);
		// unsigned: wraps (harmlessly) only on rows that raise bad
		const int64_t dp = (int64_t) ((uint64_t) p * (uint64_t) (100 - di));
		const int64_t ch = (int64_t) ((uint64_t) dp * (uint64_t) (100 + t));
		const int64_t v[5] = {q, p, dp, ch, di};
		if (LDSACC) {
			int g = 0;
			bool hit = false;
#pragma unroll
			for (int k = 0; k < K; k++) {
				const bool m = code == a.codes[k];
				g = m ? k : g;
				hit |= m;
				cnt[k] += m;
			}
			unknown |= !hit;
			unsigned long long *slot = lacc + (size_t) g * 5 * 256 + threadIdx.x;
#pragma unroll
			for (int j = 0; j < 5; j++)
				__hip_atomic_fetch_add(slot + j * 256, (unsigned long long) v[j], __ATOMIC_RELAXED,
						       __HIP_MEMORY_SCOPE_WORKGROUP);
		} else {
			bool hit = false;
#pragma unroll
			for (int k = 0; k < K; k++) {
				const bool m = code == a.codes[k];
				hit |= m;
				cnt[k] += m;
#pragma unroll
				for (int j = 0; j < 5; j++)
					s[k][j] += m ? v[j] : 0;
			}
			unknown |= !hit;
		}
	};
	struct Quad {
		i4 sd;
		u4 rf, ls;
		l2 q0, q1, p0, p1, d0, d1, t0, t1;
	};
	auto load = [&](uint64_t r, Quad &x) {
		x.sd = ldv<true>((const i4 *) (a.sd + r));
		x.rf = ldv<true>((const u4 *) (a.rf + r));
		x.ls = ldv<true>((const u4 *) (a.ls + r));
		x.q0 = ldv<true>((const l2 *) (a.qty + r)), x.q1 = ldv<true>((const l2 *) (a.qty + r + 2));
		x.p0 = ldv<true>((const l2 *) (a.price + r)), x.p1 = ldv<true>((const l2 *) (a.price + r + 2));
		x.d0 = ldv<true>((const l2 *) (a.disc + r)), x.d1 = ldv<true>((const l2 *) (a.disc + r + 2));
		x.t0 = ldv<true>((const l2 *) (a.tax + r)), x.t1 = ldv<true>((const l2 *) (a.tax + r + 2));
	};
	auto rows4 = [&](const Quad &x) {
		row(x.sd[0], ((uint32_t) x.rf[0] << 8) | x.ls[0], x.q0[0], x.p0[0], x.d0[0], x.t0[0]);
		row(x.sd[1], ((uint32_t) x.rf[1] << 8) | x.ls[1], x.q0[1], x.p0[1], x.d0[1], x.t0[1]);
		row(x.sd[2], ((uint32_t) x.rf[2] << 8) | x.ls[2], x.q1[0], x.p1[0], x.d1[0], x.t1[0]);
		row(x.sd[3], ((uint32_t) x.rf[3] << 8) | x.ls[3], x.q1[1], x.p1[1], x.d1[1], x.t1[1]);
	};
	if constexpr (LAYOUT == 1) {
	// contiguous layout: a wave owns 256-row chunks; lane l takes rows
	// 2l, 2l+1 and 128+2l, 128+2l+1 (each lng load covers 1 KiB)
	typedef int32_t i2 __attribute__((ext_vector_type(2)));
	typedef uint8_t u2 __attribute__((ext_vector_type(2)));
	struct Chunk {
		i2 s0, s1;
		u2 f0, f1, l0, l1;
		l2 q0, q1, p0, p1, d0, d1, t0, t1;
	};
	const unsigned lane = __lane_id();
	auto cload = [&](uint64_t c, Chunk &x) {
		const uint64_t r0 = c * 256 + 2 * lane, r1 = r0 + 128;
		x.s0 = ldv<true>((const i2 *) (a.sd + r0)), x.s1 = ldv<true>((const i2 *) (a.sd + r1));
		x.f0 = ldv<true>((const u2 *) (a.rf + r0)), x.f1 = ldv<true>((const u2 *) (a.rf + r1));
		x.l0 = ldv<true>((const u2 *) (a.ls + r0)), x.l1 = ldv<true>((const u2 *) (a.ls + r1));
		x.q0 = ldv<true>((const l2 *) (a.qty + r0)), x.q1 = ldv<true>((const l2 *) (a.qty + r1));
		x.p0 = ldv<true>((const l2 *) (a.price + r0)), x.p1 = ldv<true>((const l2 *) (a.price + r1));
		x.d0 = ldv<true>((const l2 *) (a.disc + r0)), x.d1 = ldv<true>((const l2 *) (a.disc + r1));
		x.t0 = ldv<true>((const l2 *) (a.tax + r0)), x.t1 = ldv<true>((const l2 *) (a.tax + r1));
	};
	auto crows = [&](const Chunk &x) {
		row(x.s0[0], ((uint32_t) x.f0[0] << 8) | x.l0[0], x.q0[0], x.p0[0], x.d0[0], x.t0[0]);
		row(x.s0[1], ((uint32_t) x.f0[1] << 8) | x.l0[1], x.q0[1], x.p0[1], x.d0[1], x.t0[1]);
		row(x.s1[0], ((uint32_t) x.f1[0] << 8) | x.l1[0], x.q1[0], x.p1[0], x.d1[0], x.t1[0]);
		row(x.s1[1], ((uint32_t) x.f1[1] << 8) | x.l1[1], x.q1[1], x.p1[1], x.d1[1], x.t1[1]);
	};
	const uint64_t nch = a.n / 256;
	const uint64_t nw = (uint64_t) gridDim.x * (blockDim.x / 64);
	uint64_t c = ((uint64_t) blockIdx.x * blockDim.x + threadIdx.x) / 64;
	// MGDK_Q1_UNROLL chunks in flight per wave
	for (; c + (MGDK_Q1_UNROLL - 1) * nw < nch; c += MGDK_Q1_UNROLL * nw) {
		Chunk x[MGDK_Q1_UNROLL];
#pragma unroll
		for (int u = 0; u < MGDK_Q1_UNROLL; u++)
			cload(c + u * nw, x[u]);
#pragma unroll
		for (int u = 0; u < MGDK_Q1_UNROLL; u++)
			crows(x[u]);
	}
	for (; c < nch; c += nw) {
		Chunk x;
		cload(c, x);
		crows(x);
	}
	if (blockIdx.x == 0 && threadIdx.x < (a.n & 255)) {
		const uint64_t r = nch * 256 + threadIdx.x;
		row(a.sd[r], ((uint32_t) a.rf[r] << 8) | a.ls[r], a.qty[r], a.price[r], a.disc[r], a.tax[r]);
	}
	} else {
	uint64_t qi = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
#if MGDK_Q1_UNROLL > 1
	// two quads in flight per lane
	for (; qi + stride < nq; qi += 2 * stride) {
		Quad x, y;
		load(qi * 4, x);
		load((qi + stride) * 4, y);
		rows4(x);
		rows4(y);
	}
#endif
	for (; qi < nq; qi += stride) {
		Quad x;
		load(qi * 4, x);
		rows4(x);
	}
	if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
		const uint64_t r = nq * 4 + threadIdx.x;
		row(a.sd[r], ((uint32_t) a.rf[r] << 8) | a.ls[r], a.qty[r], a.price[r], a.disc[r], a.tax[r]);
	}
	}
	if (LDSACC) {
		__syncthreads();
#pragma unroll
		for (int k = 0; k < K; k++)
#pragma unroll
			for (int j = 0; j < 5; j++)
				s[k][j] = (int64_t) lacc[((size_t) k * 5 + j) * 256 + threadIdx.x];
	}
#pragma unroll
	for (int k = 0; k < K; k++) {
		hge v[6] = {(hge) s[k][0], (hge) s[k][1], (hge) s[k][2], (hge) s[k][3], (hge) s[k][4], (hge) cnt[k]};
#pragma unroll
		for (int j = 0; j < 6; j++)
			v[j] = wave_sum128(v[j]);
		if (__lane_id() == 0) {
			unsigned long long *acc = a.acc + (size_t) k * 12;
#pragma unroll
			for (int j = 0; j < 6; j++)
				if (v[j] != 0)
					atomic_add128(acc + 2 * j, v[j]);
		}
	}
	for (int o = 32; o > 0; o >>= 1) {
		unknown |= __shfl_xor(unknown, o);
		bad |= __shfl_xor(bad, o);
	}
	if (__lane_id() == 0) {
		if (unknown)
			atomicOr(&a.flags[0], 1u);
		if (bad)
			atomicOr(&a.flags[2], 1u);
	}
}

// first qualifying row of every (returnflag, linestatus) code.  Lanes of a
// wave hold consecutive rows, so per distinct code in the wave only its
// lowest lane (= smallest row) competes for the global atomicMin.
__global__ __launch_bounds__(256) void
k_q1_keys(const int32_t *sd, const uint8_t *rf, const uint8_t *ls, uint64_t n, int32_t dmax,
	  unsigned long long *first)
{
	const unsigned lane = __lane_id();
	for (uint64_t base = (uint64_t) blockIdx.x * blockDim.x; base < n; base += (uint64_t) gridDim.x * blockDim.x) {
		const uint64_t i = base + threadIdx.x;
		bool valid = false;
		uint32_t c = 0;
		if (i < n) {
			int32_t d = sd[i];
			valid = d != INT32_MIN && d <= dmax;
			c = ((uint32_t) rf[i] << 8) | ls[i];
		}
		uint64_t act = __ballot(valid);
		while (act) {
			const int leader = __ffsll((long long) act) - 1;
			const uint32_t lc = __shfl(c, leader);
			const uint64_t same = __ballot(valid && c == lc);
			if ((int) lane == leader && first[lc] > i)
				atomicMin(&first[lc], (unsigned long long) i);
			act &= ~same;
		}
	}
}

__global__ void
k_q1_collect(const unsigned long long *first, uint32_t *cnt, unsigned long long *list)
{
	for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < 65536; c += gridDim.x * blockDim.x) {
		if (first[c] != ~0ull) {
			uint32_t k = atomicAdd(cnt, 1u);
			if (k < 64) {
				list[2 * k] = first[c];
				list[2 * k + 1] = c;
			}
		}
	}
}

constexpr int64_t Q1_LIM = (int64_t) 1 << 31;

template <int K>
__global__ __launch_bounds__(256) void
k_q1(Q1Args a)
{
	int64_t sq[K], sp[K], sdsc[K];
	hge sdp[K], sch[K];
	uint32_t cnt[K];
#pragma unroll
	for (int k = 0; k < K; k++) {
		sq[k] = sp[k] = sdsc[k] = 0;
		sdp[k] = sch[k] = 0;
		cnt[k] = 0;
	}
	uint32_t unknown = 0, bad = 0;
	typedef int32_t i4 __attribute__((ext_vector_type(4)));
	typedef int64_t l2 __attribute__((ext_vector_type(2)));
	typedef uint8_t u4 __attribute__((ext_vector_type(4)));
	const uint64_t nq = a.n / 4;
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	auto row = [&](int32_t d, uint32_t code, int64_t q, int64_t p, int64_t di, int64_t t) {
		if (d == INT32_MIN || d > a.dmax)
			return;
		bad |= (q <= -Q1_LIM) | (q >= Q1_LIM) | (p <= -Q1_LIM) | (p >= Q1_LIM) |
		       (di <= -Q1_LIM) | (di >= Q1_LIM) | (t <= -Q1_LIM) | (t >= Q1_LIM);
		const int64_t dp = p * (100 - di);            // |.| < 2^63
		const hge ch = (hge) dp * (hge) (100 + t);
		bool hit = false;
#pragma unroll
		for (int k = 0; k < K; k++) {
			const bool m = code == a.codes[k];
			hit |= m;
			sq[k] += m ? q : 0;
			sp[k] += m ? p : 0;
			sdsc[k] += m ? di : 0;
			sdp[k] += m ? (hge) dp : (hge) 0;
			sch[k] += m ? ch : (hge) 0;
			cnt[k] += m;
		}
		unknown |= !hit;
	};
	uint64_t qi = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
	for (; qi < nq; qi += stride) {
		const uint64_t r = qi * 4;
		i4 sd = ldv<true>((const i4 *) (a.sd + r));
		u4 rf = ldv<true>((const u4 *) (a.rf + r));
		u4 ls = ldv<true>((const u4 *) (a.ls + r));
		l2 q0 = ldv<true>((const l2 *) (a.qty + r)), q1 = ldv<true>((const l2 *) (a.qty + r + 2));
		l2 p0 = ldv<true>((const l2 *) (a.price + r)), p1 = ldv<true>((const l2 *) (a.price + r + 2));
		l2 d0 = ldv<true>((const l2 *) (a.disc + r)), d1 = ldv<true>((const l2 *) (a.disc + r + 2));
		l2 t0 = ldv<true>((const l2 *) (a.tax + r)), t1 = ldv<true>((const l2 *) (a.tax + r + 2));
		row(sd[0], ((uint32_t) rf[0] << 8) | ls[0], q0[0], p0[0], d0[0], t0[0]);
		row(sd[1], ((uint32_t) rf[1] << 8) | ls[1], q0[1], p0[1], d0[1], t0[1]);
		row(sd[2], ((uint32_t) rf[2] << 8) | ls[2], q1[0], p1[0], d1[0], t1[0]);
		row(sd[3], ((uint32_t) rf[3] << 8) | ls[3], q1[1], p1[1], d1[1], t1[1]);
	}
	if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
		const uint64_t r = nq * 4 + threadIdx.x;
		row(a.sd[r], ((uint32_t) a.rf[r] << 8) | a.ls[r], a.qty[r], a.price[r], a.disc[r], a.tax[r]);
	}
	// lane partials of qty/price/disc are < 2^31 * rows-per-lane; widen
#pragma unroll
	for (int k = 0; k < K; k++) {
		hge v[6] = {(hge) sq[k], (hge) sp[k], sdp[k], sch[k], (hge) sdsc[k], (hge) cnt[k]};
#pragma unroll
		for (int j = 0; j < 6; j++)
			v[j] = wave_sum128(v[j]);
		if (__lane_id() == 0) {
			unsigned long long *acc = a.acc + (size_t) k * 12;
#pragma unroll
			for (int j = 0; j < 6; j++)
				if (v[j] != 0)
					atomic_add128(acc + 2 * j, v[j]);
		}
	}
	for (int o = 32; o > 0; o >>= 1) {
		unknown |= __shfl_xor(unknown, o);
		bad |= __shfl_xor(bad, o);
	}
	if (__lane_id() == 0) {
		if (unknown)
			atomicOr(&a.flags[0], 1u);
		if (bad)
			atomicOr(&a.flags[1], 1u);
	}
}

bool
aligned16(const void *p)
{
	return ((uintptr_t) p & 15) == 0;
}

}  // namespace

namespace mgdk {
int q1_opatatime(mgdk_bat *shipdate, mgdk_bat *rf, mgdk_bat *ls, mgdk_bat *qty, mgdk_bat *price,
		 mgdk_bat *disc, mgdk_bat *tax, int32_t dmax, mgdk_q1row *rows, int maxgroups, int *ngroups);
}

extern "C" {

// RANGE-window benchmark column (BASELINE config 5): n lng values ascending
// by gaps U[0,4] (so every partition is ordered), partition bit every plen rows
__global__ __launch_bounds__(256) void
k_window_gaps(uint64_t seed, uint64_t n, uint64_t plen, uint8_t *gaps, int8_t *p)
{
	for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x) {
		gaps[i] = (uint8_t) urange(rnd(seed, i, 9), 0, 4);
		p[i] = i % plen == 0;
	}
}

__global__ __launch_bounds__(256) void
k_u64_to_lng(const uint64_t *in, uint64_t n, int64_t base, int64_t *out)
{
	for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
		out[i] = base + (int64_t) in[i];
}

int
mgdk_gen_window_column(uint64_t seed, uint64_t n, uint64_t plen, mgdk_bat **vals, mgdk_bat **parts)
{
	mgdk_bat *v = newbat(0, MGDK_lng, n), *p = newbat(0, MGDK_bit, n);
	DevBuf gaps(n + 16), ex(n * 8 + 16);
	if (!v || !p || !gaps.p || !ex.p) {
		mgdk_BBPunfix(v);
		mgdk_BBPunfix(p);
		return -1;
	}
	if (n) {
		hipLaunchKernelGGL(k_window_gaps, dim3(grid_for(n, 1024, 16384)), dim3(256), 0, stream(), seed, n,
				   plen ? plen : n, gaps.as<uint8_t>(), (int8_t *) p->theap);
		uint64_t tot;
		if (exclusive_scan(gaps.as<uint8_t>(), ex.as<uint64_t>(), n, &tot) < 0) {
			mgdk_BBPunfix(v);
			mgdk_BBPunfix(p);
			return -1;
		}
		hipLaunchKernelGGL(k_u64_to_lng, dim3(grid_for(n, 1024, 16384)), dim3(256), 0, stream(), ex.as<uint64_t>(),
				   n, (int64_t) -1000000, (int64_t *) v->theap);
	}
	if (!sync()) {
		mgdk_BBPunfix(v);
		mgdk_BBPunfix(p);
		return -1;
	}
	v->count = p->count = n;
	v->tsorted = 1;
	v->trevsorted = n <= 1;
	v->tkey = 0;
	p->tsorted = p->trevsorted = p->tkey = n <= 1;
	*vals = v;
	*parts = p;
	return 0;
}

int
mgdk_tpch_lineitem(uint64_t seed, uint64_t row0, uint64_t n, uint64_t sf_parts, mgdk_bat **cols)
{
	static const int types[7] = {MGDK_date, MGDK_lng, MGDK_lng, MGDK_lng, MGDK_lng, MGDK_str, MGDK_str};
	mgdk_bat *b[7] = {};
	for (int i = 0; i < 7; i++) {
		b[i] = newbat(row0, types[i] == MGDK_str ? MGDK_bte : types[i], n);
		if (b[i] == nullptr) {
			for (int j = 0; j < i; j++)
				mgdk_BBPunfix(b[j]);
			return -1;
		}
	}
	std::vector<int32_t> tab = date_table();
	DevBuf dt(tab.size() * 4);
	if (!hip_ok(hipMemcpyAsync(dt.p, tab.data(), tab.size() * 4, hipMemcpyHostToDevice, stream()), "memcpy"))
		return -1;
	if (n)
		hipLaunchKernelGGL(k_lineitem, dim3(grid_for(n, 256 * 4, 256 * 64)), dim3(256), 0, stream(), seed, row0, n,
				   sf_parts, dt.as<int32_t>(), (int32_t *) b[0]->theap, (int64_t *) b[1]->theap,
				   (int64_t *) b[2]->theap, (int64_t *) b[3]->theap, (int64_t *) b[4]->theap,
				   (uint8_t *) b[5]->theap, (uint8_t *) b[6]->theap);
	// string heaps: GDK_VAROFFSET (8192) hash header, then 8-aligned strings
	std::vector<char> rfh(8192 + 24, 0), lsh(8192 + 16, 0);
	rfh[8192 + 0] = 'A';
	rfh[8192 + 8] = 'N';
	rfh[8192 + 16] = 'R';
	lsh[8192 + 0] = 'F';
	lsh[8192 + 8] = 'O';
	if (!sync())
		return -1;
	for (int i = 0; i < 7; i++) {
		b[i]->count = n;
		b[i]->tsorted = b[i]->trevsorted = n <= 1;
		b[i]->tkey = n <= 1;
		b[i]->tnonil = 1;
		b[i]->tnil = 0;
		if (types[i] == MGDK_str) {
			b[i]->ttype = MGDK_str;
			std::vector<char> &hp = i == 5 ? rfh : lsh;
			if (mgdk_BATsetvheap(b[i], hp.data(), hp.size()) < 0)
				return -1;
		}
		cols[i] = b[i];
	}
	return 0;
}

// Q6 launch variants (tuning): variant = layout*3 + unroll_idx (+8: nt loads)
//   layout 0: lane owns 4 consecutive rows (k_q6); 1: contiguous (k_q6c)
//   unroll_idx 0,1,2 -> UNROLL 1,2,4;  bpc = workgroups per CU (256 CUs)
// default from tools/q6_tune.py on MI355X (profiles/r01/q6_tune*.log):
// contiguous 256-row chunks per wave (1 KiB per lng load instruction),
// 4 chunks in flight, nontemporal loads, 12 WG/CU (odd WG/CU counts lose
// 5-7 % with this layout)
// tuning hooks: atomics, so a concurrent set/launch never tears (dataflow
// workers call the library concurrently, SURVEY §8 b)
// round 2: the predicate cascade k_q6s with buffer loads (variant 19: 2
// chunks in flight; profiles/r02/q6_cascade/tune_buf*.log: 1.79 ms at SF100
// against 1.89 with zero-region loads (variant 17) and 2.57-2.81 ms for the
// full-read k_q6c).  Round 3 (profiles/r03/q6_tune/): 128 WG/CU instead of
// 16 -- 1.61 vs 1.83 ms on the same box; more, shorter-lived workgroups
// balance the cascade's uneven per-chunk work across the CUs (64: 1.67,
// 160-192: 1.68, 512: 1.79 with more chunks left to the scalar tail loop)
static std::atomic<int> q6_variant{19}, q6_bpc{128};
static thread_local unsigned long long q6_lines = 0;
// fused Q1 main pass (tools/q1_tune.py, profiles/r01/q1_tune.log)
static std::atomic<int> q1_layout{MGDK_Q1_LAYOUT}, q1_blocks{MGDK_Q1_BLOCKS};

static void
launch_q6(Q6Args a, int variant, int bpc, hipStream_t st)
{
	const int v7 = variant & 7;
	if (variant >= 16 || v7 >= 3) {            // k_q6c / k_q6s: per-workgroup partials
		const uint32_t nb = 256u * (unsigned) bpc;
		a.parts = (Q6Part *) scratch((size_t) nb * sizeof(Q6Part));
		if (a.parts == nullptr)
			return;
	}
	if (variant >= 16) {                 // predicate cascade (k_q6s)
		dim3 g(256u * (unsigned) bpc), blk(256);
		const void *zbuf = zero_region();
		if (zbuf == nullptr) {
			variant = 14;
			goto full;
		}
		const int64_t *z = (const int64_t *) zbuf;
		switch (variant) {
		case 17: hipLaunchKernelGGL((k_q6s<2>), g, blk, 0, st, a, z); break;
		case 18: hipLaunchKernelGGL((k_q6s<1>), g, blk, 0, st, a, z); break;
		case 19: hipLaunchKernelGGL((k_q6s<2, true>), g, blk, 0, st, a, z); break;
		case 20: hipLaunchKernelGGL((k_q6s<4, true>), g, blk, 0, st, a, z); break;
		default: hipLaunchKernelGGL((k_q6s<4>), g, blk, 0, st, a, z); break;
		}
		hipLaunchKernelGGL(k_q6_fin, dim3(1), dim3(1024), 0, st, a.parts, g.x, a.out);
		return;
	}
full:
	const bool nt = (variant & 8) != 0;
	const int v = variant & 7;
	dim3 g(256u * (unsigned) bpc), blk(256);
#define Q6L(K, U) do { if (nt) hipLaunchKernelGGL((K<U, true>), g, blk, 0, st, a); \
			else hipLaunchKernelGGL((K<U, false>), g, blk, 0, st, a); } while (0)
	switch (v) {
	case 0: Q6L(k_q6, 1); break;
	case 1: Q6L(k_q6, 2); break;
	case 2: Q6L(k_q6, 4); break;
	case 3: Q6L(k_q6c, 1); break;
	case 4: Q6L(k_q6c, 2); break;
	default: Q6L(k_q6c, 4); break;
	}
#undef Q6L
	if (v >= 3)
		hipLaunchKernelGGL(k_q6_fin, dim3(1), dim3(1024), 0, st, a.parts, g.x, a.out);
}

int mgdk_q6_fused(mgdk_bat *shipdate, mgdk_bat *discount, mgdk_bat *quantity, mgdk_bat *extendedprice,
		  int32_t d0, int32_t d1, int64_t dlo, int64_t dhi, int64_t qmax, void *revenue);

// select the fused Q1 main-pass layout (0: 4-row lanes, 1: 256-row chunks
// per wave) and workgroup count (tuning hook, not ABI)
void
mgdk_q1_set_variant(int layout, int blocks)
{
	q1_layout = layout == 1 ? 1 : 0;
	q1_blocks = blocks > 0 ? blocks : MGDK_Q1_BLOCKS;
}

// select the Q6 launch variant for subsequent calls (tuning hook, not ABI)
void
mgdk_q6_set_variant(int variant, int blocks_per_cu)
{
	q6_variant = variant;
	q6_bpc = blocks_per_cu > 0 ? blocks_per_cu : 8;
}

int
mgdk_q6_fused(mgdk_bat *shipdate, mgdk_bat *discount, mgdk_bat *quantity, mgdk_bat *extendedprice,
	      int32_t d0, int32_t d1, int64_t dlo, int64_t dhi, int64_t qmax, void *revenue)
{
	mgdk_bat *c[4] = {shipdate, discount, quantity, extendedprice};
	const int want[4] = {MGDK_int, MGDK_lng, MGDK_lng, MGDK_lng};
	for (int i = 0; i < 4; i++) {
		if (c[i] == nullptr || basetype(c[i]->ttype) != want[i] || c[i]->count != shipdate->count ||
		    c[i]->hseqbase != shipdate->hseqbase) {
			seterr("42000!q6_fused: lineitem columns must be aligned date/lng BATs");
			return -1;
		}
	}
	Q6Args a;
	a.sd = (const int32_t *) shipdate->theap;
	a.disc = (const int64_t *) discount->theap;
	a.qty = (const int64_t *) quantity->theap;
	a.price = (const int64_t *) extendedprice->theap;
	a.n = shipdate->count;
	a.d0 = d0;
	a.d1 = d1;
	a.dlo = dlo;
	a.dhi = dhi;
	a.qmax = qmax;
	a.out = (unsigned long long *) meta_buf();
	a.parts = nullptr;
	hipStream_t st = stream();
	// out: [0..1] revenue, [2] column lines read by the cascade
	if (!hip_ok(hipMemsetAsync(a.out, 0, 128, st), "memset"))
		return -1;
	{
		ProfScope prof("q6_fused");
		if (a.n) {
			bool al = aligned16(a.sd) && aligned16(a.disc) && aligned16(a.qty) && aligned16(a.price);
			if (al)
				launch_q6(a, q6_variant.load(), q6_bpc.load(), st);
			else
				hipLaunchKernelGGL(k_q6_scalar, dim3(grid_for(a.n, 256 * 4, 256 * 16)), dim3(256), 0, st, a);
		}
	}
	unsigned long long *h = (unsigned long long *) pinned(32);
	if (!hip_ok(hipMemcpyAsync(h, a.out, 24, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	memcpy(revenue, h, 16);
	q6_lines = h[2];
	return 0;
}

// 128-B column lines the calling thread's last fused Q6 read beyond
// shipdate (cascade variant; 0 for the full-read variants), for the bench's
// byte count
extern "C" unsigned long long
mgdk_q6_last_sectors(void)
{
	return q6_lines;
}

int
mgdk_q1_fused(mgdk_bat *shipdate, mgdk_bat *returnflag, mgdk_bat *linestatus, mgdk_bat *quantity,
	      mgdk_bat *extendedprice, mgdk_bat *discount, mgdk_bat *tax, int32_t dmax, mgdk_q1row *rows,
	      int maxgroups, int *ngroups)
{
	mgdk_bat *c[7] = {shipdate, returnflag, linestatus, quantity, extendedprice, discount, tax};
	for (int i = 0; i < 7; i++) {
		if (c[i] == nullptr || c[i]->count != shipdate->count || c[i]->hseqbase != shipdate->hseqbase) {
			seterr("42000!q1_fused: lineitem columns must be aligned");
			return -1;
		}
	}
	bool shape_ok = basetype(shipdate->ttype) == MGDK_int && returnflag->ttype == MGDK_str &&
			returnflag->twidth == 1 && linestatus->ttype == MGDK_str && linestatus->twidth == 1;
	for (int i = 3; i < 7; i++)
		shape_ok = shape_ok && c[i]->ttype == MGDK_lng && aligned16(c[i]->theap);
	shape_ok = shape_ok && aligned16(shipdate->theap) && ((uintptr_t) returnflag->theap & 3) == 0 &&
		   ((uintptr_t) linestatus->theap & 3) == 0;
	if (!shape_ok)
		return q1_opatatime(shipdate, returnflag, linestatus, quantity, extendedprice, discount, tax, dmax,
				    rows, maxgroups, ngroups);
	const uint64_t n = shipdate->count;
	hipStream_t st = stream();
	// 1. keys and their first occurrence on a prefix
	const uint64_t pre = std::min<uint64_t>(n, (uint64_t) 1 << 20);
	DevBuf first(65536 * 8), list(64 * 16 + 64), acc(Q1_MAXK * 12 * 8 + 64);
	uint32_t *cnt = (uint32_t *) ((char *) list.p + 64 * 16);
	if (!hip_ok(hipMemsetAsync(first.p, 0xff, 65536 * 8, st), "memset") ||
	    !hip_ok(hipMemsetAsync(cnt, 0, 16, st), "memset") ||
	    !hip_ok(hipMemsetAsync(acc.p, 0, Q1_MAXK * 12 * 8 + 64, st), "memset"))
		return -1;
	ProfScope prof("q1_fused");
	if (pre)
		hipLaunchKernelGGL(k_q1_keys, dim3(grid_for(pre, 1024, 2048)), dim3(256), 0, st, (const int32_t *) shipdate->theap,
				   (const uint8_t *) returnflag->theap, (const uint8_t *) linestatus->theap, pre, dmax,
				   first.as<unsigned long long>());
	hipLaunchKernelGGL(k_q1_collect, dim3(64), dim3(256), 0, st, first.as<unsigned long long>(), cnt,
			   list.as<unsigned long long>());
	unsigned long long *h = (unsigned long long *) pinned(64 * 16 + 64);
	if (!hip_ok(hipMemcpyAsync(h, list.p, 64 * 16 + 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	uint32_t K = *(uint32_t *) (h + 128);
	if (K == 0 || K > Q1_MAXK || (int) K > maxgroups)
		return q1_opatatime(shipdate, returnflag, linestatus, quantity, extendedprice, discount, tax, dmax,
				    rows, maxgroups, ngroups);
	std::vector<std::pair<unsigned long long, uint32_t>> keys;
	for (uint32_t k = 0; k < K; k++)
		keys.emplace_back(h[2 * k], (uint32_t) h[2 * k + 1]);
	std::sort(keys.begin(), keys.end());
	// 2. main pass
	Q1Args a{};
	a.sd = (const int32_t *) shipdate->theap;
	a.rf = (const uint8_t *) returnflag->theap;
	a.ls = (const uint8_t *) linestatus->theap;
	a.qty = (const int64_t *) quantity->theap;
	a.price = (const int64_t *) extendedprice->theap;
	a.disc = (const int64_t *) discount->theap;
	a.tax = (const int64_t *) tax->theap;
	a.n = n;
	a.dmax = dmax;
	a.K = (int) K;
	for (uint32_t k = 0; k < K; k++)
		a.codes[k] = keys[k].second;
	for (uint32_t k = K; k < Q1_MAXK; k++)
		a.codes[k] = 0xffffffffu;
	a.acc = acc.as<unsigned long long>();
	a.flags = (uint32_t *) (a.acc + Q1_MAXK * 12);
	const int layout = q1_layout;
	dim3 g(grid_for(n / 4 + 1, 256, MGDK_Q1_MODE == 0 ? 4096 : (unsigned) q1_blocks.load())), blk(256);
	const uint64_t threads = (uint64_t) g.x * 256;
	// rows one lane can see: quads (layout 0) or 4 rows per 256-row chunk
	// per wave (layout 1), plus the tail rows
	const uint64_t per_lane = layout == 1 ? 4 * ((n / 256 + threads / 64 - 1) / (threads / 64)) + 1
					      : 4 * ((n / 4 + threads - 1) / threads) + 3;
	a.plim = std::min<int64_t>(Q1_LIM, (int64_t) (((uint64_t) 1 << 45) / per_lane));
	constexpr bool lds = MGDK_Q1_MODE == 2;
#define Q1N(KK) do { if (layout == 1) hipLaunchKernelGGL((k_q1n<KK, lds, 1>), g, blk, 0, st, a); \
		     else hipLaunchKernelGGL((k_q1n<KK, lds, 0>), g, blk, 0, st, a); } while (0)
	if (MGDK_Q1_MODE == 0)
		;
	else if (K <= 1) Q1N(1);
	else if (K <= 2) Q1N(2);
	else if (K <= 4) Q1N(4);
	else Q1N(8);
#undef Q1N
	unsigned long long *hr = (unsigned long long *) pinned(Q1_MAXK * 12 * 8 + 64);
	const size_t accb = Q1_MAXK * 12 * 8 + 16;
	if (MGDK_Q1_MODE != 0) {
		if (!hip_ok(hipMemcpyAsync(hr, acc.p, accb, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			return -1;
	}
	if (MGDK_Q1_MODE == 0 || ((const uint32_t *) (hr + Q1_MAXK * 12))[2] != 0) {
		// wide pass: values beyond the narrow bounds (or narrow pass disabled)
		ProfScope profw("q1_wide");
		if (!hip_ok(hipMemsetAsync(acc.p, 0, Q1_MAXK * 12 * 8 + 64, st), "memset"))
			return -1;
		if (K <= 1) hipLaunchKernelGGL(k_q1<1>, g, blk, 0, st, a);
		else if (K <= 2) hipLaunchKernelGGL(k_q1<2>, g, blk, 0, st, a);
		else if (K <= 4) hipLaunchKernelGGL(k_q1<4>, g, blk, 0, st, a);
		else hipLaunchKernelGGL(k_q1<8>, g, blk, 0, st, a);
		if (!hip_ok(hipMemcpyAsync(hr, acc.p, accb, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			return -1;
	}
	const uint32_t *fl = (const uint32_t *) (hr + Q1_MAXK * 12);
	if (fl[0] || fl[1])
		return q1_opatatime(shipdate, returnflag, linestatus, quantity, extendedprice, discount, tax, dmax,
				    rows, maxgroups, ngroups);
	for (uint32_t k = 0; k < K; k++) {
		mgdk_q1row &r = rows[k];
		memset(&r, 0, sizeof(r));
		r.returnflag = (uint8_t) (keys[k].second >> 8);
		r.linestatus = (uint8_t) (keys[k].second & 0xff);
		r.first_row = shipdate->hseqbase + keys[k].first;
		const unsigned long long *x = hr + k * 12;
		memcpy(r.sum_qty, x + 0, 16);
		memcpy(r.sum_base_price, x + 2, 16);
		memcpy(r.sum_disc_price, x + 4, 16);
		memcpy(r.sum_charge, x + 6, 16);
		memcpy(r.sum_disc, x + 8, 16);
		r.count_order = (int64_t) x[10];
		// aggr.subavg: BATgroupavg3 of the exact group sums
		hge sq, sp, sd;
		memcpy(&sq, x + 0, 16);
		memcpy(&sp, x + 2, 16);
		memcpy(&sd, x + 8, 16);
		avg3_of_sum(sq, r.count_order, &r.avg_qty, &r.rem_qty);
		avg3_of_sum(sp, r.count_order, &r.avg_price, &r.rem_price);
		avg3_of_sum(sd, r.count_order, &r.avg_disc, &r.rem_disc);
	}
	*ngroups = (int) K;
	return 0;
}

}  // extern "C"
