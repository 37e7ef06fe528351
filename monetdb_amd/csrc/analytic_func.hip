// analytic_func.hip -- windowed SUM / COUNT over frames on the MI355X
// (gdk/gdk_analytic_func.c:1959 GDKanalyticalsum, :1626 GDKanalyticalcount;
// SURVEY.md §8(f) row 1, the direct consumer of the RANGE bounds of
// analytic.hip).
//
// The reference walks every partition: running sums for the UNBOUNDED
// frames (:1684-1745), and a fanout-16 segment tree per partition for
// general frames (:1783-1815, gdk/gdk_analytic.h:52-130).  On the device
// every frame is a row interval [lo, hi), so one exact 128-bit exclusive
// prefix sum P of the non-nil values and one prefix count C of them give
//     sum(frame) = P[hi] - P[lo],  nil when C[hi] - C[lo] == 0
// for every frame kind at once (one reduce-then-scan over the column, one
// per-row pass).  Frame intervals:
//     3 unbounded preceding .. current row: [partition start, end of the
//       row's peer group)             4 current row .. unbounded: [start of
//       the peer group, partition end) 5 whole partition   6 the row
//     other: [s[i], e[i]) from GDKanalyticalwindowbounds.
// Overflow of a lng result is the reference's ADD_WITH_CHECK on every
// partial: for the running frames the partials are exactly the partition's
// prefix (3, 5) or suffix (4) sums, checked row by row from P; for the
// segment-tree frames every tree node and query partial is a sum of a
// subset of the partition, so a partition whose sum of |v| fits lng cannot
// overflow -- such partitions are computed exactly, and a partition beyond
// that bound (where the reference's answer depends on its tree's addition
// order) fails loudly instead of guessing.  hge results of integer inputs
// cannot overflow.
#include <type_traits>

#include <cfloat>
#include <cstdio>

#include "mgdk_internal.h"
#include "segments.h"

using namespace mgdk;

namespace {

constexpr int PF_ROWS = 8;                 // contiguous rows per lane
constexpr int PF_TILE = 256 * PF_ROWS;

template <typename T>
__device__ __forceinline__ bool
ldv(const T *b, BUN i, int64_t &v)
{
	const T x = b[i];
	v = (int64_t) x;
	return x == NilOf<T>::v();
}

__device__ __forceinline__ hge
shfl_up128(hge v, int o)
{
	const unsigned long long lo = __shfl_up((unsigned long long) (uhge) v, o);
	const unsigned long long hi = __shfl_up((unsigned long long) ((uhge) v >> 64), o);
	return (hge) (((uhge) hi << 64) | lo);
}

// inclusive scans across a wave
__device__ __forceinline__ hge
wave_scan128(hge v)
{
	const unsigned lane = __lane_id();
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const hge u = shfl_up128(v, o);
		if (lane >= (unsigned) o)
			v += u;
	}
	return v;
}

__device__ __forceinline__ unsigned long long
wave_scan64(unsigned long long v)
{
	const unsigned lane = __lane_id();
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const unsigned long long u = __shfl_up(v, o);
		if (lane >= (unsigned) o)
			v += u;
	}
	return v;
}

struct TileTot {
	hge sum;
	hge abs;
	unsigned long long cnt;
	unsigned long long pad;
};

template <typename T>
__global__ __launch_bounds__(256) void
k_pf_tile(const T *b, BUN n, bool want_abs, TileTot *tot)
{
	const BUN base = (BUN) blockIdx.x * PF_TILE + (BUN) threadIdx.x * PF_ROWS;
	hge s = 0, a = 0;
	unsigned long long c = 0;
#pragma unroll
	for (int q = 0; q < PF_ROWS; q++) {
		const BUN i = base + q;
		int64_t v;
		if (i < n && !ldv(b, i, v)) {
			s += v;
			c++;
			if (want_abs)
				a += v < 0 ? -(hge) v : (hge) v;
		}
	}
	s = block_sum128(s);
	if (want_abs)
		a = block_sum128(a);
	c = block_reduce(c, [](unsigned long long x, unsigned long long y) { return x + y; });
	if (threadIdx.x == 0) {
		tot[blockIdx.x].sum = s;
		tot[blockIdx.x].abs = a;
		tot[blockIdx.x].cnt = c;
	}
}

// exclusive scan of up to 256 tile totals per workgroup, in place; the
// workgroup's total goes to up[blockIdx.x] (a second level scans those)
__global__ __launch_bounds__(256) void
k_pf_scan256(TileTot *tot, BUN ntiles, TileTot *up)
{
	__shared__ hge w_s[4], w_a[4];
	__shared__ unsigned long long w_c[4];
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const BUN t = (BUN) blockIdx.x * 256 + tid;
	TileTot x{};
	if (t < ntiles)
		x = tot[t];
	const hge is = wave_scan128(x.sum), ia = wave_scan128(x.abs);
	const unsigned long long ic = wave_scan64(x.cnt);
	if (lane == 63) {
		w_s[w] = is;
		w_a[w] = ia;
		w_c[w] = ic;
	}
	__syncthreads();
	hge es = is - x.sum, ea = ia - x.abs;
	unsigned long long ec = ic - x.cnt;
	for (unsigned q = 0; q < w; q++) {
		es += w_s[q];
		ea += w_a[q];
		ec += w_c[q];
	}
	if (t < ntiles) {
		tot[t].sum = es;
		tot[t].abs = ea;
		tot[t].cnt = ec;
	}
	if (up && tid == 255) {
		up[blockIdx.x].sum = es + x.sum;
		up[blockIdx.x].abs = ea + x.abs;
		up[blockIdx.x].cnt = ec + x.cnt;
	}
}

__global__ __launch_bounds__(256) void
k_pf_addup(TileTot *tot, BUN ntiles, const TileTot *up)
{
	const BUN t = (BUN) blockIdx.x * 256 + threadIdx.x;
	if (t < ntiles && blockIdx.x > 0) {
		tot[t].sum += up[blockIdx.x].sum;
		tot[t].abs += up[blockIdx.x].abs;
		tot[t].cnt += up[blockIdx.x].cnt;
	}
}

// P[i], C[i] (and A[i]) = sums over rows < i; entry n holds the totals.
// Lanes own PF_ROWS consecutive rows (a thread-local running sum), the
// results go through LDS so the stores are coalesced.  C may be NULL (no
// nils: the count of [lo, hi) is hi - lo).
template <typename T>
__global__ __launch_bounds__(256) void
k_pf_final(const T *b, BUN n, const TileTot *tot, hge *P, unsigned long long *Cn, hge *A)
{
	__shared__ hge w_s[4], w_a[4];
	__shared__ unsigned long long w_c[4];
	__shared__ hge sP[PF_TILE];
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const BUN tb = (BUN) blockIdx.x * PF_TILE;
	const BUN base = tb + (BUN) tid * PF_ROWS;
	int64_t v[PF_ROWS];
	bool nl[PF_ROWS];
	hge s = 0, a = 0;
	unsigned long long c = 0;
#pragma unroll
	for (int q = 0; q < PF_ROWS; q++) {
		const BUN i = base + q;
		nl[q] = i >= n || ldv(b, i, v[q]);
		if (!nl[q]) {
			s += v[q];
			c++;
			if (A)
				a += v[q] < 0 ? -(hge) v[q] : (hge) v[q];
		}
	}
	const hge is = wave_scan128(s);
	const hge ia = A ? wave_scan128(a) : 0;
	const unsigned long long ic = wave_scan64(c);
	if (lane == 63) {
		w_s[w] = is;
		w_a[w] = ia;
		w_c[w] = ic;
	}
	__syncthreads();
	hge es = is - s + tot[blockIdx.x].sum, ea = ia - a + tot[blockIdx.x].abs;
	unsigned long long ec = ic - c + tot[blockIdx.x].cnt;
	for (unsigned q = 0; q < w; q++) {
		es += w_s[q];
		ea += w_a[q];
		ec += w_c[q];
	}
	const BUN nt = n - tb < (BUN) PF_TILE ? n - tb : (BUN) PF_TILE;
	// sums
#pragma unroll
	for (int q = 0; q < PF_ROWS; q++) {
		sP[tid * PF_ROWS + q] = es;
		if (base + q == n - 1)
			P[n] = es + (nl[q] ? 0 : v[q]);
		if (!nl[q])
			es += v[q];
	}
	__syncthreads();
	for (unsigned i = tid; i < nt; i += 256)
		P[tb + i] = sP[i];
	if (Cn) {
		__syncthreads();
		unsigned long long *sC = (unsigned long long *) sP;
#pragma unroll
		for (int q = 0; q < PF_ROWS; q++) {
			sC[tid * PF_ROWS + q] = ec;
			if (base + q == n - 1)
				Cn[n] = ec + (nl[q] ? 0 : 1);
			if (!nl[q])
				ec++;
		}
		__syncthreads();
		for (unsigned i = tid; i < nt; i += 256)
			Cn[tb + i] = sC[i];
	}
	if (A) {
		__syncthreads();
#pragma unroll
		for (int q = 0; q < PF_ROWS; q++) {
			sP[tid * PF_ROWS + q] = ea;
			if (base + q == n - 1)
				A[n] = ea + (nl[q] ? 0 : (v[q] < 0 ? -(hge) v[q] : (hge) v[q]));
			if (!nl[q])
				ea += v[q] < 0 ? -(hge) v[q] : (hge) v[q];
		}
		__syncthreads();
		for (unsigned i = tid; i < nt; i += 256)
			A[tb + i] = sP[i];
	}
}

__global__ __launch_bounds__(256) void
k_or_flags(const int8_t *p, const int8_t *o, BUN n, int8_t *f)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		f[i] = i == 0 || (p && p[i]) || (o && o[i]);
}

struct FArgs {
	BUN n;
	int frame;
	bool other;          // frame given by s / e
	bool lng_out;        // result lng (else hge)
	bool count;          // GDKanalyticalcount
	bool count_all;
	bool avg;            // GDKanalyticalavg of integers: dbl sum / count
	int avgint;          // GDKanalyticalavginteger: output width (0: off)
	Starts part, peer;
	const oid *s, *e;
	const hge *P, *A;
	const unsigned long long *C;
	void *out;
	uint32_t *flags;     // [0] overflow, [1] beyond the exact bound, [2] nils in the result
};

__global__ __launch_bounds__(256) void
k_frames(FArgs a)
{
	uint32_t ovf = 0, big = 0, hasnil = 0;
	const hge MAXL = (hge) INT64_MAX;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (BUN) gridDim.x * blockDim.x) {
		BUN lo, hi, ps = 0, pe = 0;
		if (a.frame == 3 || a.frame == 4 || a.frame == 5 || (a.other && a.A))
			a.part.seg(i, ps, pe);
		switch (a.frame) {
		case 3: {
			BUN gs, ge;
			a.peer.seg(i, gs, ge);
			lo = ps;
			hi = ge;
			break;
		}
		case 4: {
			BUN gs, ge;
			a.peer.seg(i, gs, ge);
			lo = gs;
			hi = pe;
			break;
		}
		case 5: lo = ps; hi = pe; break;
		case 6: lo = i; hi = i + 1; break;
		default: lo = a.s[i]; hi = a.e[i]; break;
		}
		if (hi < lo)
			hi = lo;
		if (a.count) {
			const long long c = a.count_all || !a.C ? (long long) (hi - lo) : (long long) (a.C[hi] - a.C[lo]);
			((long long *) a.out)[i] = c;
			continue;
		}
		const unsigned long long c = a.C ? a.C[hi] - a.C[lo] : hi - lo;
		const hge sum = a.P[hi] - a.P[lo];
		if (a.avgint) {
			// AVERAGE_ITER's state of the frame = floor(sum / n), sum mod n;
			// ANALYTICAL_AVERAGE_INT_CALC_FINALIZE (gdk_analytic_statistics.c:435-446)
			long long q = 0;
			if (c) {
				hge hq = sum / (hge) c, hr = sum % (hge) c;
				if (hr < 0) {
					hq -= 1;
					hr += (hge) c;
				}
				if (hr > 0 && (hq < 0 ? 2 * hr > (hge) c : 2 * hr >= (hge) c))
					hq += 1;
				q = (long long) hq;
			}
			switch (a.avgint) {
			case 1: ((int8_t *) a.out)[i] = c ? (int8_t) q : INT8_MIN; break;
			case 2: ((int16_t *) a.out)[i] = c ? (int16_t) q : INT16_MIN; break;
			case 4: ((int32_t *) a.out)[i] = c ? (int32_t) q : INT32_MIN; break;
			default: ((int64_t *) a.out)[i] = c ? (int64_t) q : INT64_MIN; break;
			}
			hasnil |= c == 0;
			continue;
		}
		if (a.avg) {
			// (dbl) sum / n of ANALYTICAL_AVG_IMP_NUM_* (gdk_analytic_statistics.c:55-165)
			((double *) a.out)[i] = c ? hge_to_dbl(sum) / (double) (long long) c : __builtin_nan("");
			hasnil |= c == 0;
			continue;
		}
		if (a.lng_out) {
			// the reference's partials for this row's partition
			if (a.frame == 3 || a.frame == 5) {
				const hge q = a.P[i + 1] - a.P[ps];
				ovf |= q > MAXL || q < -MAXL;
			} else if (a.frame == 4) {
				const hge q = a.P[pe] - a.P[i];
				ovf |= q > MAXL || q < -MAXL;
			} else if (a.other && a.A) {
				big |= a.A[pe] - a.A[ps] > MAXL;
			}
			((long long *) a.out)[i] = c ? (long long) sum : INT64_MIN;
		} else {
			((hge *) a.out)[i] = c ? sum : NilOf<hge>::v();
		}
		hasnil |= c == 0;
	}
	ovf = block_reduce(ovf, [](uint32_t x, uint32_t y) { return x | y; });
	big = block_reduce(big, [](uint32_t x, uint32_t y) { return x | y; });
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0) {
		publish_or(&a.flags[0], ovf);
		publish_or(&a.flags[1], big);
		publish_or(&a.flags[2], hasnil);
	}
}

// general frames [s[i], e[i]) into a hge result: 8 rows per lane with
// every bound load, then every prefix load in flight (the generic kernel
// above serialises two dependent loads per row)
template <bool HASC>
__global__ __launch_bounds__(256) void
k_frames_other_hge(FArgs a)
{
	constexpr int R = 8;
	const BUN base = (BUN) blockIdx.x * (256 * R) + threadIdx.x;
	BUN lo[R], hi[R];
#pragma unroll
	for (int q = 0; q < R; q++) {
		const BUN i = base + (BUN) q * 256;
		lo[q] = hi[q] = 0;
		if (i < a.n) {
			lo[q] = a.s[i];
			hi[q] = a.e[i];
		}
	}
	hge pl[R], ph[R];
	unsigned long long cl[R], ch[R];
#pragma unroll
	for (int q = 0; q < R; q++) {
		if (hi[q] < lo[q])
			hi[q] = lo[q];
		pl[q] = a.P[lo[q]];
		ph[q] = a.P[hi[q]];
		if (HASC) {
			cl[q] = a.C[lo[q]];
			ch[q] = a.C[hi[q]];
		}
	}
	uint32_t hasnil = 0;
#pragma unroll
	for (int q = 0; q < R; q++) {
		const BUN i = base + (BUN) q * 256;
		if (i < a.n) {
			const unsigned long long c = HASC ? ch[q] - cl[q] : hi[q] - lo[q];
			((hge *) a.out)[i] = c ? ph[q] - pl[q] : NilOf<hge>::v();
			hasnil |= c == 0;
		}
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(&a.flags[2], hasnil);
}

// Fused general frames into a hge result: one workgroup per 2048-row tile
// stages the values under the tile's frames -- [min s, max e), at most
// FW_MAX rows -- in LDS, builds their exact prefix sums / non-nil counts
// there and answers every row from LDS: the column is read about once and
// no n-row prefix arrays are written or re-read.  A tile whose frames span
// more (long or unbounded frames) raises flags[3]; the host then uses the
// global-prefix path for the whole call.
constexpr int FT_ROWS = 2048;
constexpr int FW_MAX = 2560;
constexpr int FW_PER = (FW_MAX + 255) / 256;   // staged values per lane

template <typename T>
__global__ __launch_bounds__(256) void
k_frames_tile_hge(const T *b, BUN n, const oid *S, const oid *E, hge *out, uint32_t *flags)
{
	__shared__ hge sP[FW_MAX + 1];
	__shared__ uint32_t sC[FW_MAX + 1];
	__shared__ hge w_s[4];
	__shared__ uint32_t w_c[4];
	__shared__ unsigned long long s_lo, s_hi;
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const BUN t0 = (BUN) blockIdx.x * FT_ROWS;
	constexpr int R = FT_ROWS / 256;
	BUN lo[R], hi[R];
	unsigned long long mn = ~0ull, mx = 0;
#pragma unroll
	for (int q = 0; q < R; q++) {
		const BUN i = t0 + (BUN) q * 256 + tid;
		lo[q] = hi[q] = 0;
		if (i < n) {
			lo[q] = S[i];
			hi[q] = E[i];
			if (hi[q] < lo[q])
				hi[q] = lo[q];
			mn = lo[q] < mn ? lo[q] : mn;
			mx = hi[q] > mx ? hi[q] : mx;
		}
	}
	if (tid == 0) {
		s_lo = ~0ull;
		s_hi = 0;
	}
	__syncthreads();
	mn = block_reduce(mn, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	if (tid == 0)
		s_lo = mn;
	mx = block_reduce(mx, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	if (tid == 0)
		s_hi = mx;
	__syncthreads();
	const BUN wlo = s_lo, whi = s_hi;
	if (whi > wlo && whi - wlo > (BUN) FW_MAX) {
		if (tid == 0)
			publish_or(&flags[3], 1u);
		return;
	}
	const int W = whi > wlo ? (int) (whi - wlo) : 0;
	// thread tid stages the contiguous values [tid*FW_PER, ...) of the window
	hge ls = 0;
	uint32_t lc = 0;
	int64_t v[FW_PER];
	bool ok[FW_PER];
#pragma unroll
	for (int q = 0; q < FW_PER; q++) {
		const int j = tid * FW_PER + q;
		ok[q] = false;
		v[q] = 0;
		if (j < W) {
			const T x = b[wlo + j];
			ok[q] = !(x == NilOf<T>::v());
			v[q] = ok[q] ? (int64_t) x : 0;
		}
		ls += v[q];
		lc += ok[q];
	}
	const hge is = wave_scan128(ls);
	const unsigned long long ic = wave_scan64(lc);
	if (lane == 63) {
		w_s[w] = is;
		w_c[w] = (uint32_t) ic;
	}
	__syncthreads();
	hge es = is - ls;
	uint32_t ec = (uint32_t) ic - lc;
	for (unsigned q = 0; q < w; q++) {
		es += w_s[q];
		ec += w_c[q];
	}
#pragma unroll
	for (int q = 0; q < FW_PER; q++) {
		const int j = tid * FW_PER + q;
		if (j <= W) {
			sP[j] = es;
			sC[j] = ec;
		}
		es += v[q];
		ec += ok[q];
	}
	if (tid == 255) {                // entry W (= FW_MAX: past every lane's range)
		sP[W] = es;
		sC[W] = ec;
	}
	__syncthreads();
	uint32_t hasnil = 0;
#pragma unroll
	for (int q = 0; q < R; q++) {
		const BUN i = t0 + (BUN) q * 256 + tid;
		if (i < n) {
			const int a0 = (int) (lo[q] - wlo), a1 = (int) (hi[q] - wlo);
			const uint32_t c = sC[a1] - sC[a0];
			out[i] = c ? sP[a1] - sP[a0] : NilOf<hge>::v();
			hasnil |= c == 0;
		}
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (tid == 0)
		publish_or(&flags[2], hasnil);
}

__global__ void
k_first(const oid *L, oid *out)
{
	*out = L[0];
}

}  // namespace

namespace mgdk {

// starts list from flags (nonzero = start); row 0 is always a start
int
make_starts(const int8_t *flags, BUN n, Starts &st, mgdk_bat **keep)
{
	st.n = n;
	*keep = nullptr;
	if (flags == nullptr) {
		st.L = nullptr;
		st.Lseq = 0;
		st.m = 1;
		st.lead = false;
		return 0;
	}
	mgdk_bat *S = compact_flags(flags, n, 0, true);
	if (S == nullptr)
		return -1;
	*keep = S;
	st.L = S->ttype == MGDK_void ? nullptr : (const oid *) S->theap;
	st.Lseq = S->tseqbase;
	bool first0 = false;
	if (S->count > 0) {
		if (st.L == nullptr) {
			first0 = st.Lseq == 0;
		} else {
			oid *d = (oid *) meta_buf();
			hipLaunchKernelGGL(k_first, dim3(1), dim3(1), 0, stream(), st.L, d);
			oid *h = (oid *) pinned(8);
			if (!hip_ok(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
				return -1;
			first0 = *h == 0;
		}
	}
	st.lead = !first0;
	st.m = S->count + (st.lead ? 1 : 0);
	return 0;
}

}  // namespace mgdk

namespace {

bool
sum_in_type(int t)
{
	t = basetype(t);
	return t == MGDK_bte || t == MGDK_sht || t == MGDK_int || t == MGDK_lng;
}

int
run_frames(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int frame_type,
	   bool count, bool count_all, bool lng_out, bool avg = false, int avgint = 0)
{
	const BUN n = b->count;
	hipStream_t st = stream();
	if (r->theap == nullptr && n) {
		seterr("analytic: result BAT has no heap");
		return -1;
	}
	if (n == 0) {
		r->count = 0;
		return 0;
	}
	if ((p && (p->count != n || width_of(p->ttype) != 1)) || (o && (o->count != n || width_of(o->ttype) != 1))) {
		seterr("analytic: p and o must be bit BATs aligned with b");
		return -1;
	}
	const bool frames = !(frame_type >= 3 && frame_type <= 6);
	if (frames && (s == nullptr || e == nullptr || s->count < n || e->count < n || s->ttype != MGDK_oid ||
		       e->ttype != MGDK_oid)) {
		seterr("analytic: frame bounds s and e (oid BATs aligned with b) are required");
		return -1;
	}
	if ((frame_type == 3 || frame_type == 4) && o == nullptr) {
		seterr("analytic: the peer column o is required for this frame");
		return -1;
	}
	// general frames into hge: the fused tile kernel when every tile's frames
	// fit its LDS window
	if (frames && !count && !lng_out && b->twidth <= 8 && basetype(b->ttype) != MGDK_flt &&
	    basetype(b->ttype) != MGDK_dbl) {
		DevBuf ff(64);
		uint32_t *h = (uint32_t *) pinned(16);
		if (!ff.p || !hip_ok(hipMemsetAsync(ff.p, 0, 64, st), "memset"))
			return -1;
		const dim3 g((unsigned) ((n + FT_ROWS - 1) / FT_ROWS)), blk(256);
		const oid *S = (const oid *) s->theap, *E = (const oid *) e->theap;
		hge *R = (hge *) r->theap;
		switch (b->twidth) {
		case 1: hipLaunchKernelGGL((k_frames_tile_hge<int8_t>), g, blk, 0, st, (const int8_t *) b->theap, n, S, E, R, ff.as<uint32_t>()); break;
		case 2: hipLaunchKernelGGL((k_frames_tile_hge<int16_t>), g, blk, 0, st, (const int16_t *) b->theap, n, S, E, R, ff.as<uint32_t>()); break;
		case 4: hipLaunchKernelGGL((k_frames_tile_hge<int32_t>), g, blk, 0, st, (const int32_t *) b->theap, n, S, E, R, ff.as<uint32_t>()); break;
		default: hipLaunchKernelGGL((k_frames_tile_hge<int64_t>), g, blk, 0, st, (const int64_t *) b->theap, n, S, E, R, ff.as<uint32_t>()); break;
		}
		if (!hip_ok(hipMemcpyAsync(h, ff.p, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			return -1;
		if (h[3] == 0) {
			r->count = n;
			r->tnil = h[2] != 0;
			r->tnonil = h[2] == 0;
			r->tsorted = r->trevsorted = r->tkey = n <= 1;
			return 0;
		}
		// some frame spans more than a tile's window: global prefix path below
	}
	// prefix sums / counts over the column
	const bool need_prefix = !(count && count_all);
	// without nils the count of [lo, hi) is hi - lo: no count prefix
	const bool nonil = b->tnonil != 0;
	const bool want_abs = !count && lng_out && frames;
	const BUN ntiles = (n + PF_TILE - 1) / PF_TILE;
	DevBuf tot(ntiles * sizeof(TileTot) + 64), P(need_prefix && !count ? (n + 1) * 16 : 16),
		Cn(need_prefix ? (n + 1) * 8 : 8), A(want_abs ? (n + 1) * 16 : 16), fl(64);
	if (!tot.p || !P.p || !Cn.p || !A.p || !fl.p)
		return -1;
	if (need_prefix) {
		const dim3 g((unsigned) ntiles), blk(256);
		hge *Pp = count ? nullptr : P.as<hge>();
		DevBuf Pd(count ? (n + 1) * 16 : 16);   // sums are computed anyway; keep them apart for counts
		if (!Pd.p)
			return -1;
		if (Pp == nullptr)
			Pp = Pd.as<hge>();
#define PF_TILE_K(T) hipLaunchKernelGGL((k_pf_tile<T>), g, blk, 0, st, (const T *) b->theap, n, want_abs, \
					  tot.as<TileTot>())
#define PF_FINAL_K(T) hipLaunchKernelGGL((k_pf_final<T>), g, blk, 0, st, (const T *) b->theap, n, tot.as<TileTot>(), \
					   Pp, nonil ? nullptr : Cn.as<unsigned long long>(), want_abs ? A.as<hge>() : nullptr)
		switch (b->twidth) {
		case 1: PF_TILE_K(int8_t); break;
		case 2: PF_TILE_K(int16_t); break;
		case 4: PF_TILE_K(int32_t); break;
		default: PF_TILE_K(int64_t); break;
		}
		// two-level exclusive scan of the tile totals
		const BUN nb = (ntiles + 255) / 256;
		if (nb > 256 * 256) {
			seterr("analytic: input too large");
			return -1;
		}
		DevBuf up(nb * sizeof(TileTot) + 64), up2(256 * sizeof(TileTot) + 64);
		if (!up.p || !up2.p)
			return -1;
		hipLaunchKernelGGL(k_pf_scan256, dim3((unsigned) nb), blk, 0, st, tot.as<TileTot>(), ntiles, up.as<TileTot>());
		if (nb > 1) {
			const BUN nb2 = (nb + 255) / 256;
			hipLaunchKernelGGL(k_pf_scan256, dim3((unsigned) nb2), blk, 0, st, up.as<TileTot>(), nb, up2.as<TileTot>());
			if (nb2 > 1) {
				hipLaunchKernelGGL(k_pf_scan256, dim3(1), blk, 0, st, up2.as<TileTot>(), nb2, (TileTot *) nullptr);
				hipLaunchKernelGGL(k_pf_addup, dim3((unsigned) nb2), blk, 0, st, up.as<TileTot>(), nb, up2.as<TileTot>());
			}
			hipLaunchKernelGGL(k_pf_addup, dim3((unsigned) nb), blk, 0, st, tot.as<TileTot>(), ntiles, up.as<TileTot>());
		}
		switch (b->twidth) {
		case 1: PF_FINAL_K(int8_t); break;
		case 2: PF_FINAL_K(int16_t); break;
		case 4: PF_FINAL_K(int32_t); break;
		default: PF_FINAL_K(int64_t); break;
		}
#undef PF_TILE_K
#undef PF_FINAL_K
		if (!sync())
			return -1;
	}
	// segments
	mgdk_bat *Sp = nullptr, *Sg = nullptr;
	FArgs a{};
	a.n = n;
	a.frame = frame_type;
	a.other = frames;
	a.lng_out = lng_out;
	a.count = count;
	a.count_all = count_all;
	a.avg = avg;
	a.avgint = avgint;
	a.s = frames ? (const oid *) s->theap : nullptr;
	a.e = frames ? (const oid *) e->theap : nullptr;
	a.P = P.as<hge>();
	a.A = want_abs ? A.as<hge>() : nullptr;
	a.C = nonil ? nullptr : Cn.as<unsigned long long>();
	a.out = r->theap;
	a.flags = fl.as<uint32_t>();
	int rc = -1;
	DevBuf gf(n + 8);
	if (!gf.p || make_starts(p ? (const int8_t *) p->theap : nullptr, n, a.part, &Sp) < 0)
		goto out;
	if (frame_type == 3 || frame_type == 4) {
		hipLaunchKernelGGL(k_or_flags, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st,
				   p ? (const int8_t *) p->theap : nullptr, (const int8_t *) o->theap, n, gf.as<int8_t>());
		if (make_starts(gf.as<int8_t>(), n, a.peer, &Sg) < 0)
			goto out;
	}
	if (!hip_ok(hipMemsetAsync(fl.p, 0, 64, st), "memset"))
		goto out;
	if (frames && !count && !lng_out) {
		const dim3 g((unsigned) ((n + 2047) / 2048));
		if (a.C)
			hipLaunchKernelGGL((k_frames_other_hge<true>), g, dim3(256), 0, st, a);
		else
			hipLaunchKernelGGL((k_frames_other_hge<false>), g, dim3(256), 0, st, a);
	} else {
		hipLaunchKernelGGL(k_frames, dim3(grid_for(n, 1024, 16384)), dim3(256), 0, st, a);
	}
	{
		uint32_t *h = (uint32_t *) pinned(16);
		if (!hip_ok(hipMemcpyAsync(h, fl.p, 12, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			goto out;
		if (h[0]) {
			seterr("22003!overflow in calculation.\n");
			goto out;
		}
		if (h[1]) {
			seterr("42000!GDKanalyticalsum: a partition's sum of |values| exceeds lng; its lng frame sums "
			       "depend on the segment tree's addition order -- not supported on the device path "
			       "(use a hge result)");
			goto out;
		}
		r->count = n;
		r->tnil = h[2] != 0;
		r->tnonil = h[2] == 0;
		r->tsorted = r->trevsorted = r->tkey = n <= 1;
		rc = 0;
	}
out:
	mgdk_BBPunfix(Sp);
	mgdk_BBPunfix(Sg);
	return rc;
}


// ---- GDKanalyticalavg (gdk/gdk_analytic_statistics.c:364-423) -----------
//
// Integer inputs over the running frames (3, 4, 5) are exact: the frame's
// 128-bit sum from the prefix arrays above, (dbl) sum / n (k_frames, avg).
// Everything else replays the reference's arithmetic, which is order
// dependent:
//   * flt / dbl over frames 3 and 5: AVERAGE_ITER_FLOAT in the input type,
//     row by row through the partition -- one lane per partition
//     (k_avg_replay); frame 4 of flt / dbl never assigns its result (:224-246),
//     so every row is nil;
//   * general frames: the reference's fanout-16 segment tree per partition
//     (gdk_analytic.h:63-130) whose inner nodes fold their non-empty
//     children's averages with AVERAGE_ITER / AVERAGE_ITER_FLOAT (a node
//     counts children, not rows).  The device builds the same trees for
//     every partition at once, one level per launch, and answers each row
//     with the reference's query walk (k_avg_tree_query).
// Level L >= 1 of partition k (start ps) is stored at
//     lvl[L] + (ps >> 4L) + k + m,   m < ceil(nc / 16^L),
// which never overlaps the next partition's nodes, so a level holds
// (n >> 4L) + #partitions + 1 nodes and needs no per-partition offset scan.

constexpr int AVG_MAX_LEVELS = 17;   // 16^16 = 2^64 rows

// AVERAGE_ITER (gdk/gdk_calc_private.h:231-275) in 64-bit arithmetic: for
// bte..lng inputs no intermediate leaves the input type's range
__device__ __forceinline__ void
avg_iter_int(long long x, long long &a, long long &rr, long long &n)
{
	n++;
	long long an = a / n, xn = x / n, z1 = xn - an;
	xn = x - xn * n;
	an = a - an * n;
	unsigned long long z2;
	if (xn >= an) {
		z2 = (unsigned long long) (xn - an);
		while (z2 >= (unsigned long long) n) {
			z2 -= (unsigned long long) n;
			z1++;
		}
	} else {
		z2 = (unsigned long long) (an - xn);
		for (;;) {
			z1--;
			if (z2 < (unsigned long long) n) {
				z2 = (unsigned long long) n - z2;
				break;
			}
			z2 -= (unsigned long long) n;
		}
	}
	a += z1;
	rr += (long long) z2;
	if (rr >= n) {
		rr -= n;
		a++;
	}
}

// avg_num_deltas / avg_fp_deltas and their fold / finalize steps
template <typename T, bool F = std::is_floating_point<T>::value>
struct AvgNode;

template <typename T>
struct AvgNode<T, false> {
	long long a, n, rr;
	__device__ __forceinline__ void zero() { a = n = rr = 0; }
	__device__ __forceinline__ void leaf(const T *b, BUN i)
	{
		const T v = b[i];
		a = v == NilOf<T>::v() ? 0 : (long long) v;
		n = v == NilOf<T>::v() ? 0 : 1;
		rr = 0;
	}
	__device__ __forceinline__ void fold(const AvgNode &c)
	{
		if (c.n)
			avg_iter_int(c.a, a, rr, n);
	}
	__device__ __forceinline__ double result() const
	{
		return (double) a + (double) rr / (double) n;
	}
	// ANALYTICAL_AVERAGE_INT_CALC_FINALIZE (gdk_analytic_statistics.c:435-446)
	__device__ __forceinline__ long long rounded() const
	{
		long long q = a;
		if (rr > 0 && (q < 0 ? 2 * rr > n : 2 * rr >= n))
			q++;
		return q;
	}
};

template <typename T>
struct AvgNode<T, true> {
	T a;
	long long n;
	__device__ __forceinline__ void zero() { a = 0; n = 0; }
	__device__ __forceinline__ void leaf(const T *b, BUN i)
	{
		const T v = b[i];
		a = v != v ? (T) 0 : v;
		n = v != v ? 0 : 1;
	}
	// AVERAGE_ITER_FLOAT (gdk_calc_private.h:277-289) in T arithmetic
	__device__ __forceinline__ void add(T x)
	{
		n++;
		const T nn = (T) n;
		if ((a > 0) == (x > 0))
			a += (x - a) / nn;
		else
			a = a - a / nn + x / nn;
	}
	__device__ __forceinline__ void fold(const AvgNode &c)
	{
		if (c.n)
			add(c.a);
	}
	__device__ __forceinline__ double result() const { return (double) a; }
	__device__ __forceinline__ long long rounded() const { return 0; }
};

struct AvgTree {
	void *lvl[AVG_MAX_LEVELS];   // level L >= 1 node arrays
	int nlev;                    // levels built above the rows
};

__global__ __launch_bounds__(256) void
k_avg_pidx(Starts part, uint32_t *pidx)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < part.n; i += (BUN) gridDim.x * blockDim.x)
		pidx[i] = (uint32_t) part.idx(i);
}

__global__ __launch_bounds__(256) void
k_avg_maxlen(Starts part, unsigned long long *mx)
{
	unsigned long long v = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < part.m; k += (BUN) gridDim.x * blockDim.x)
		v = max(v, (unsigned long long) (part.end_of(k) - part.at(k)));
	v = block_reduce(v, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	if (threadIdx.x == 0 && v)
		atomicMax(mx, v);
}

// populate_segment_tree, level L >= 1: the thread of the first row a node
// covers folds the node's children (level L-1) in order
template <typename T>
__global__ __launch_bounds__(256) void
k_avg_tree_level(const T *b, Starts part, const uint32_t *pidx, AvgTree t, int L)
{
	using N = AvgNode<T>;
	const int sh = 4 * L, shc = sh - 4;
	N *out = (N *) t.lvl[L];
	const N *child = L > 1 ? (const N *) t.lvl[L - 1] : nullptr;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < part.n; i += (BUN) gridDim.x * blockDim.x) {
		const BUN k = pidx[i], ps = part.at(k);
		const BUN rel = i - ps;
		if (rel & (((BUN) 1 << sh) - 1))
			continue;
		const BUN nc = part.end_of(k) - ps;
		const BUN ncl = (nc + ((BUN) 1 << shc) - 1) >> shc;     // nodes on level L-1
		const BUN c0 = (rel >> sh) * 16, c1 = min(c0 + 16, ncl);
		N acc;
		acc.zero();
		for (BUN c = c0; c < c1; c++) {
			N x;
			if (L == 1)
				x.leaf(b, ps + c);
			else
				x = child[(ps >> shc) + k + c];
			acc.fold(x);
		}
		out[(ps >> sh) + k + (rel >> sh)] = acc;
	}
}

// compute_on_segment_tree (gdk_analytic.h:96-130) for [s[i], e[i])
template <typename T, bool IOUT>
__global__ __launch_bounds__(256) void
k_avg_tree_query(const T *b, Starts part, const uint32_t *pidx, AvgTree t, const oid *S, const oid *E,
		 void *out, uint32_t *flags)
{
	using N = AvgNode<T>;
	uint32_t hasnil = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < part.n; i += (BUN) gridDim.x * blockDim.x) {
		const BUN k = pidx[i], ps = part.at(k), nc = part.end_of(k) - ps;
		BUN begin = S[i] > ps ? min((BUN) S[i] - ps, nc) : 0;
		BUN tend = E[i] > ps ? min((BUN) E[i] - ps, nc) : 0;
		N acc;
		acc.zero();
		if (begin < tend) {
			for (int L = 0; L <= t.nlev; L++) {
				const N *lv = L ? (const N *) t.lvl[L] + ((ps >> (4 * L)) + k) : nullptr;
				auto node = [&](BUN pos) {
					N x;
					if (L == 0)
						x.leaf(b, ps + pos);
					else
						x = lv[pos];
					return x;
				};
				BUN pb = begin / 16, pe = tend / 16;
				if (pb == pe) {
					for (BUN pos = begin; pos < tend; pos++)
						acc.fold(node(pos));
					break;
				}
				const BUN gb = pb * 16;
				if (begin != gb) {
					for (BUN pos = begin; pos < gb + 16; pos++)
						acc.fold(node(pos));
					pb++;
				}
				const BUN ge = pe * 16;
				if (tend != ge)
					for (BUN pos = ge; pos < tend; pos++)
						acc.fold(node(pos));
				begin = pb;
				tend = pe;
			}
		}
		if constexpr (IOUT) {
			((T *) out)[i] = acc.n == 0 ? NilOf<T>::v() : (T) acc.rounded();
			hasnil |= acc.n == 0;
		} else if (acc.n == 0) {
			((double *) out)[i] = __builtin_nan("");
			hasnil = 1;
		} else {
			((double *) out)[i] = acc.result();
		}
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, hasnil);
}

// flt / dbl, frames 3 (peer groups from o) and 5: one lane replays one
// partition's rows in order (ANALYTICAL_AVG_IMP_FP_UNBOUNDED_TILL_CURRENT_ROW
// / _ALL_ROWS, gdk_analytic_statistics.c:202-267)
template <typename T>
__global__ __launch_bounds__(64) void
k_avg_replay(const T *b, Starts part, const int8_t *o, bool peers, double *out, uint32_t *flags)
{
	const BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t hasnil = 0;
	if (k < part.m) {
		const BUN ps = part.at(k), pe = part.end_of(k);
		AvgNode<T> c;
		c.zero();
		double cur = __builtin_nan("");
		BUN j = ps;
		for (BUN r = ps; r < pe; r++) {
			const T v = b[r];
			if (v == v)
				c.add(v);
			if (r + 1 == pe || (peers && o[r + 1])) {
				if (c.n > 0)
					cur = (double) c.a;
				else
					hasnil = 1;
				for (; j <= r; j++)
					out[j] = cur;
			}
		}
	}
	if (hasnil)
		publish_or(flags, 1);
}

template <typename T>
__global__ __launch_bounds__(256) void
k_avg_row(const T *b, BUN n, bool nil_all, double *out, uint32_t *flags)
{
	uint32_t hasnil = nil_all && n;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const T v = b[i];
		const bool nil = nil_all || is_nil(v);
		out[i] = nil ? __builtin_nan("") : (double) v;
		hasnil |= nil;
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, hasnil);
}

// integer copy of the values (frame 6 of GDKanalyticalavginteger)
template <typename T>
__global__ __launch_bounds__(256) void
k_avg_copy(const T *b, BUN n, T *out, uint32_t *flags)
{
	uint32_t hasnil = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const T v = b[i];
		out[i] = v;
		hasnil |= is_nil(v);
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, hasnil);
}

template <typename T, bool IOUT = false>
int
run_avg(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int frame_type)
{
	constexpr bool isf = std::is_floating_point<T>::value;
	const BUN n = b->count;
	hipStream_t st = stream();
	const T *bv = (const T *) b->theap;
	void *out = r->theap;
	const bool frames = !(frame_type >= 3 && frame_type <= 6);
	DevBuf fl(64);
	if (!fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 64, st), "memset"))
		return -1;
	mgdk_bat *Sp = nullptr;
	int rc = -1;
	if (IOUT && frame_type == 6) {
		hipLaunchKernelGGL((k_avg_copy<T>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, bv, n, (T *) out,
				   fl.as<uint32_t>());
	} else if (frame_type == 6 || (isf && frame_type == 4)) {
		hipLaunchKernelGGL((k_avg_row<T>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, bv, n,
				   frame_type == 4, (double *) out, fl.as<uint32_t>());
	} else {
		Starts part;
		if (make_starts(p ? (const int8_t *) p->theap : nullptr, n, part, &Sp) < 0)
			goto out;
		if (!frames) {
			// flt / dbl, frames 3 and 5 (integers take run_frames)
			if constexpr (isf)
				hipLaunchKernelGGL((k_avg_replay<T>), dim3((unsigned) ((part.m + 63) / 64)), dim3(64), 0, st, bv,
						   part, frame_type == 3 ? (const int8_t *) o->theap : nullptr, frame_type == 3,
						   (double *) out, fl.as<uint32_t>());
		} else {
			if (n >= 0xffffffffull) {
				seterr("42000!GDKanalyticalavg: more than 2^32-1 rows on the device path\n");
				goto out;
			}
			// levels: until one node covers the longest partition
			unsigned long long *hm = (unsigned long long *) pinned(8);
			DevBuf mx(64), pidx(n * 4 + 4);
			if (!mx.p || !pidx.p || !hip_ok(hipMemsetAsync(mx.p, 0, 8, st), "memset"))
				goto out;
			hipLaunchKernelGGL(k_avg_maxlen, dim3(grid_for(part.m, 1024, 1024)), dim3(256), 0, st, part,
					   mx.as<unsigned long long>());
			hipLaunchKernelGGL(k_avg_pidx, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, part,
					   pidx.as<uint32_t>());
			if (!hip_ok(hipMemcpyAsync(hm, mx.p, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
				goto out;
			AvgTree t{};
			// (nc - 1) >> 4L == 0 for every partition at the top level
			int nlev = 1;
			while (nlev < AVG_MAX_LEVELS - 1 && ((*hm - 1) >> (4 * nlev)) > 0)
				nlev++;
			t.nlev = nlev;
			size_t tot = 0, offs[AVG_MAX_LEVELS] = {0};
			for (int L = 1; L <= nlev; L++) {
				offs[L] = tot;
				tot += ((n >> (4 * L)) + part.m + 1) * sizeof(AvgNode<T>);
				tot = (tot + 255) & ~(size_t) 255;
			}
			DevBuf tree(tot);
			if (!tree.p)
				goto out;
			for (int L = 1; L <= nlev; L++)
				t.lvl[L] = tree.as<char>() + offs[L];
			for (int L = 1; L <= nlev; L++)
				hipLaunchKernelGGL((k_avg_tree_level<T>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, bv,
						   part, pidx.as<uint32_t>(), t, L);
			hipLaunchKernelGGL((k_avg_tree_query<T, IOUT>), dim3(grid_for(n, 256, 16384)), dim3(256), 0, st, bv, part,
					   pidx.as<uint32_t>(), t, (const oid *) s->theap, (const oid *) e->theap, out,
					   fl.as<uint32_t>());
			if (!sync())
				goto out;
		}
	}
	{
		uint32_t *h = (uint32_t *) pinned(16);
		if (!hip_ok(hipMemcpyAsync(h, fl.p, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			goto out;
		r->count = n;
		r->tnil = h[0] != 0;
		r->tnonil = h[0] == 0;
		r->tsorted = r->trevsorted = r->tkey = n <= 1;
		rc = 0;
	}
out:
	mgdk_BBPunfix(Sp);
	return rc;
}

// ---- GDKanalyticalsum over flt / dbl (gdk_analytic_func.c:1795-1817,
// :1930-1950).  Float addition is not associative, so the order is the
// reference's: frames 3 / 4 add row by row (one lane replays one partition),
// general frames walk the reference's fanout-16 tree (built for every
// partition at once, one launch per level) in its own order, every add with
// ADD_WITH_CHECK in the result type T2 (gdk_calc_private.h:53-67); frame 5
// is dofsum: the exact sum of the partition rounded once (the grouped exact
// float sum with the partition as the group).
template <typename T2>
struct FSum {
	T2 v;
	int nil;
	__device__ __forceinline__ void zero() { v = 0; nil = 1; }
	// cur = x + cur (ADD_WITH_CHECK(x, cur, ...)); false on overflow
	__device__ __forceinline__ bool fold(const FSum &x)
	{
		if (x.nil)
			return true;
		if (nil) {
			v = x.v;
			nil = 0;
			return true;
		}
		const T2 mx = sizeof(T2) == 4 ? (T2) FLT_MAX : (T2) DBL_MAX;
		if (v < 1) {
			if (-mx - v > x.v)
				return false;
		} else if (mx - v < x.v) {
			return false;
		}
		v = x.v + v;
		return true;
	}
	template <typename T1>
	__device__ __forceinline__ void leaf(const T1 *b, BUN i)
	{
		const T1 x = b[i];
		nil = x != x;
		v = nil ? (T2) 0 : (T2) x;
	}
};

template <typename T1, typename T2>
__global__ __launch_bounds__(64) void
k_fsum_replay(const T1 *b, Starts part, const int8_t *o, bool forward, T2 *out, uint32_t *flags)
{
	const BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t fl = 0;
	if (k < part.m) {
		const BUN ps = part.at(k), pe = part.end_of(k);
		FSum<T2> cur;
		cur.zero();
		if (forward) {
			BUN j = ps;
			for (BUN r = ps; r < pe && !(fl & 2); r++) {
				FSum<T2> x;
				x.leaf(b, r);
				if (!cur.fold(x))
					fl |= 2;
				if (r + 1 == pe || o[r + 1]) {
					const T2 w = cur.nil ? (T2) __builtin_nan("") : cur.v;
					fl |= cur.nil;
					for (; j <= r; j++)
						out[j] = w;
				}
			}
		} else if (pe > ps) {
			BUN l = pe - 1;
			for (BUN j = pe - 1;; j--) {
				FSum<T2> x;
				x.leaf(b, j);
				if (!cur.fold(x)) {
					fl |= 2;
					break;
				}
				if (o[j] || j == ps) {
					const T2 w = cur.nil ? (T2) __builtin_nan("") : cur.v;
					fl |= cur.nil;
					for (;; l--) {
						out[l] = w;
						if (l == j)
							break;
					}
					if (j == ps)
						break;
					l = j - 1;
				}
			}
		}
	}
	if (fl)
		atomicOr(flags, fl);
}

template <typename T1, typename T2>
__global__ __launch_bounds__(256) void
k_fsum_row(const T1 *b, BUN n, T2 *out, uint32_t *flags)
{
	uint32_t hasnil = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const T1 v = b[i];
		out[i] = (T2) v;
		hasnil |= v != v;
	}
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, hasnil);
}

// frame 5: every row gets its partition's dofsum (psum: dbl per partition);
// a flt result is the dbl sum rounded to flt (and an infinite one overflows)
template <typename T2>
__global__ __launch_bounds__(256) void
k_fsum_bcast(const double *psum, const uint32_t *pidx, BUN n, T2 *out, uint32_t *flags)
{
	uint32_t fl = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const double d = psum[pidx[i]];
		const T2 w = (T2) d;
		out[i] = w;
		if (d != d)
			fl |= 1;
		else if (w - w != w - w)   // infinite after rounding
			fl |= 4;
	}
	fl = block_reduce(fl, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, fl);
}

__global__ __launch_bounds__(256) void
k_pidx_oid(const uint32_t *pidx, BUN n, oid *g)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		g[i] = pidx[i];
}

template <typename T1, typename T2>
__global__ __launch_bounds__(256) void
k_fsum_tree_level(const T1 *b, Starts part, const uint32_t *pidx, AvgTree t, int L, uint32_t *flags)
{
	using N = FSum<T2>;
	const int sh = 4 * L, shc = sh - 4;
	N *out = (N *) t.lvl[L];
	const N *child = L > 1 ? (const N *) t.lvl[L - 1] : nullptr;
	uint32_t fl = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < part.n; i += (BUN) gridDim.x * blockDim.x) {
		const BUN k = pidx[i], ps = part.at(k);
		const BUN rel = i - ps;
		if (rel & (((BUN) 1 << sh) - 1))
			continue;
		const BUN nc = part.end_of(k) - ps;
		const BUN ncl = (nc + ((BUN) 1 << shc) - 1) >> shc;
		const BUN c0 = (rel >> sh) * 16, c1 = min(c0 + 16, ncl);
		N acc;
		acc.zero();
		for (BUN c = c0; c < c1; c++) {
			N x;
			if (L == 1)
				x.leaf(b, ps + c);
			else
				x = child[(ps >> shc) + k + c];
			if (!acc.fold(x))
				fl |= 2;
		}
		out[(ps >> sh) + k + (rel >> sh)] = acc;
	}
	fl = block_reduce(fl, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, fl);
}

template <typename T1, typename T2>
__global__ __launch_bounds__(256) void
k_fsum_tree_query(const T1 *b, Starts part, const uint32_t *pidx, AvgTree t, const oid *S, const oid *E, T2 *out,
		  uint32_t *flags)
{
	using N = FSum<T2>;
	uint32_t fl = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < part.n; i += (BUN) gridDim.x * blockDim.x) {
		const BUN k = pidx[i], ps = part.at(k), nc = part.end_of(k) - ps;
		BUN begin = S[i] > ps ? min((BUN) S[i] - ps, nc) : 0;
		BUN tend = E[i] > ps ? min((BUN) E[i] - ps, nc) : 0;
		N acc;
		acc.zero();
		if (begin < tend) {
			for (int L = 0; L <= t.nlev; L++) {
				const N *lv = L ? (const N *) t.lvl[L] + ((ps >> (4 * L)) + k) : nullptr;
				auto node = [&](BUN pos) {
					N x;
					if (L == 0)
						x.leaf(b, ps + pos);
					else
						x = lv[pos];
					return x;
				};
				BUN pb = begin / 16, pe = tend / 16;
				if (pb == pe) {
					for (BUN pos = begin; pos < tend; pos++)
						if (!acc.fold(node(pos)))
							fl |= 2;
					break;
				}
				const BUN gb = pb * 16;
				if (begin != gb) {
					for (BUN pos = begin; pos < gb + 16; pos++)
						if (!acc.fold(node(pos)))
							fl |= 2;
					pb++;
				}
				const BUN ge = pe * 16;
				if (tend != ge)
					for (BUN pos = ge; pos < tend; pos++)
						if (!acc.fold(node(pos)))
							fl |= 2;
				begin = pb;
				tend = pe;
			}
		}
		out[i] = acc.nil ? (T2) __builtin_nan("") : acc.v;
		fl |= acc.nil;
	}
	fl = block_reduce(fl, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, fl);
}

// ---- the parallel form of frames 3 / 4 over one partition ----------------
// (fp_parallel_min): the running sum as a blocked scan.  Positions q are
// rows in fold order (frame 3: q = row; frame 4: q = n - 1 - row); a
// position ends its peer run where the replay writes (frame 3: o[row + 1]
// or the last row; frame 4: o[row] or row 0).  Pass 1 folds each 4096-
// position tile (16 per lane, the lanes combined in order); pass 2 scans
// the tile totals; pass 3 writes every position's running sum; pass 4 gives
// every position the sum at the end of its run (end positions are never
// rewritten, so it reads them in place).  FSum::fold keeps the replay's
// overflow test and nil rule; only the rounding differs (DESIGN.md states
// the bound).
constexpr unsigned RS_PER = 16, RS_TILE = 256 * RS_PER;

__device__ __forceinline__ BUN
rs_row(BUN q, BUN n, bool fwd)
{
	return fwd ? q : n - 1 - q;
}

__device__ __forceinline__ bool
rs_end(const int8_t *o, BUN q, BUN n, bool fwd)
{
	if (fwd)
		return q + 1 == n || o[q + 1];
	const BUN j = n - 1 - q;
	return j == 0 || o[j];
}

template <typename T2>
__device__ __forceinline__ FSum<T2>
rs_comb(FSum<T2> a, const FSum<T2> &b, uint32_t &fl)
{
	if (!a.fold(b))
		fl |= 2;
	return a;
}

// a lane's RS_PER positions q0 .. q0 + RS_PER - 1 of its tile: values (as
// FSum leaves) and run-end flags.  The tile's values and end bytes are
// loaded row-wise (consecutive lanes, consecutive addresses) into LDS and
// each lane then reads its RS_PER consecutive positions (one pad slot per
// RS_PER keeps those reads off a single bank)
template <typename T1>
struct RsStage {
	T1 v[RS_TILE + RS_TILE / RS_PER];
	int8_t f[RS_TILE];
};

template <typename T1, typename T2>
__device__ __forceinline__ void
rs_load(const T1 *b, const int8_t *o, BUN n, bool fwd, RsStage<T1> &sg, FSum<T2> (&x)[RS_PER], bool (&e)[RS_PER])
{
	const BUN t0 = (BUN) blockIdx.x * RS_TILE;
#pragma unroll
	for (unsigned k = 0; k < RS_PER; k++) {
		const unsigned i = k * 256 + threadIdx.x;
		const BUN q = t0 + i;
		T1 v = (T1) 0;
		int8_t f = 1;
		if (q < n) {
			v = b[rs_row(q, n, fwd)];
			// the end flag's byte: o[q + 1] (frame 3) or o[n - 1 - q] (frame
			// 4); the last position always ends its run
			if (q + 1 < n)
				f = o[fwd ? q + 1 : n - 1 - q];
		}
		sg.v[i + i / RS_PER] = v;
		sg.f[i] = f;
	}
	__syncthreads();
	const unsigned l0 = threadIdx.x * RS_PER;
#pragma unroll
	for (unsigned k = 0; k < RS_PER; k++) {
		const unsigned i = l0 + k;
		const BUN q = t0 + i;
		const T1 v = sg.v[i + i / RS_PER];
		x[k].nil = q >= n || v != v;
		x[k].v = x[k].nil ? (T2) 0 : (T2) v;
		e[k] = q < n && sg.f[i] != 0;
	}
}

template <typename T2>
__device__ __forceinline__ FSum<T2>
rs_shfl_up(const FSum<T2> &v, int d)
{
	FSum<T2> y;
	y.v = __shfl_up(v.v, d);
	y.nil = __shfl_up(v.nil, d);
	return y;
}

// ordered exclusive scan over the block's values (blockDim.x a multiple of
// 64, at most 1024): a wave scan by shuffles, then the waves' totals through
// LDS (one barrier); the same association every launch.  *total = the fold
// of all of them
template <typename T2>
__device__ __forceinline__ FSum<T2>
rs_block_excl(FSum<T2> v, FSum<T2> *wt, uint32_t &fl, FSum<T2> *total)
{
	const unsigned lane = __lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
	FSum<T2> inc = v;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const FSum<T2> y = rs_shfl_up(inc, d);
		if ((int) lane >= d)
			inc = rs_comb(y, inc, fl);
	}
	FSum<T2> ex = rs_shfl_up(inc, 1);
	if (lane == 0)
		ex.zero();
	if (lane == 63)
		wt[w] = inc;
	__syncthreads();
	FSum<T2> wp, all;
	wp.zero();
	all.zero();
	for (unsigned q = 0; q < nw; q++) {
		if (q < w)
			wp = rs_comb(wp, wt[q], fl);
		all = rs_comb(all, wt[q], fl);
	}
	*total = all;
	__syncthreads();            // wt may be reused by the caller
	return rs_comb(wp, ex, fl);
}

template <typename T1, typename T2>
__global__ __launch_bounds__(256) void
k_rs_tile(const T1 *b, const int8_t *o, BUN n, bool fwd, FSum<T2> *tot, BUN *fend, uint32_t *flags)
{
	__shared__ FSum<T2> lds[256];
	__shared__ BUN sm[256];
	__shared__ RsStage<T1> sg;
	const BUN q0 = (BUN) blockIdx.x * RS_TILE + threadIdx.x * RS_PER;
	FSum<T2> x[RS_PER];
	bool e[RS_PER];
	rs_load<T1, T2>(b, o, n, fwd, sg, x, e);
	FSum<T2> acc;
	acc.zero();
	BUN fe = ~(BUN) 0;
	uint32_t fl = 0;
#pragma unroll
	for (int k = (int) RS_PER - 1; k >= 0; k--)
		if (e[k])
			fe = q0 + k;
#pragma unroll
	for (unsigned k = 0; k < RS_PER; k++)
		acc = rs_comb(acc, x[k], fl);
	FSum<T2> total;
	(void) rs_block_excl(acc, lds, fl, &total);
#pragma unroll
	for (int d = 32; d > 0; d >>= 1)
		fe = min(fe, (BUN) __shfl_xor(fe, d));
	if (__lane_id() == 0)
		sm[threadIdx.x >> 6] = fe;
	__syncthreads();
	fe = min(min(sm[0], sm[1]), min(sm[2], sm[3]));
	if (threadIdx.x == 0) {
		tot[blockIdx.x] = total;
		fend[blockIdx.x] = fe;
	}
	if (fl)
		atomicOr(flags, fl);
}

// pre[t] = the fold of the tiles before t (in order); nxt[t] = the first run
// end at or after tile t + 1's first position.  One workgroup of 1024
// threads: thread t folds a contiguous run of tiles (its loads issued
// together), one block scan of the runs, then each thread writes its run's
// prefixes; the suffix minima alike
constexpr unsigned RS_TPT = 32;     // tiles per thread per round (all loaded at once)

template <typename T2>
__global__ __launch_bounds__(1024) void
k_rs_tiles(const FSum<T2> *tot, const BUN *fend, BUN nt, FSum<T2> *pre, BUN *nxt, uint32_t *flags)
{
	__shared__ FSum<T2> wt[16];
	__shared__ BUN wm[16];
	uint32_t fl = 0;
	FSum<T2> carry;
	carry.zero();
	const BUN round = (BUN) 1024 * RS_TPT;
	for (BUN r0 = 0; r0 < nt; r0 += round) {
		const BUN b0 = r0 + (BUN) threadIdx.x * RS_TPT;
		FSum<T2> v[RS_TPT];
#pragma unroll
		for (unsigned k = 0; k < RS_TPT; k++) {
			if (b0 + k < nt)
				v[k] = tot[b0 + k];
			else
				v[k].zero();
		}
		FSum<T2> acc;
		acc.zero();
#pragma unroll
		for (unsigned k = 0; k < RS_TPT; k++)
			acc = rs_comb(acc, v[k], fl);
		FSum<T2> total;
		FSum<T2> run = rs_comb(carry, rs_block_excl(acc, wt, fl, &total), fl);
#pragma unroll
		for (unsigned k = 0; k < RS_TPT; k++) {
			if (b0 + k < nt)
				pre[b0 + k] = run;
			run = rs_comb(run, v[k], fl);
		}
		carry = rs_comb(carry, total, fl);
	}
	// suffix minima of the first ends, rounds from the back
	BUN m = ~(BUN) 0;
	const BUN nr = (nt + round - 1) / round;
	const unsigned lane = __lane_id(), w = threadIdx.x >> 6;
	for (BUN rr = nr; rr-- > 0;) {
		const BUN b0 = rr * round + (BUN) threadIdx.x * RS_TPT;
		BUN f[RS_TPT];
		BUN own = ~(BUN) 0;
#pragma unroll
		for (unsigned k = 0; k < RS_TPT; k++) {
			f[k] = b0 + k < nt ? fend[b0 + k] : ~(BUN) 0;
			own = min(own, f[k]);
		}
		// minimum over the threads after this one: wave suffix minimum,
		// then the later waves
		BUN suf = own;
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const BUN y = (BUN) __shfl_down(suf, d);
			if ((int) lane + d < 64)
				suf = min(suf, y);
		}
		if (lane == 0)
			wm[w] = suf;
		__syncthreads();
		BUN later = m;
		for (unsigned q = w + 1; q < 16; q++)
			later = min(later, wm[q]);
		const BUN nextin = (BUN) __shfl_down(suf, 1);
		BUN after = lane + 1 < 64 ? min(nextin, later) : later;
		const BUN rmin = min(min(min(wm[0], wm[1]), min(wm[2], wm[3])),
				     min(min(min(wm[4], wm[5]), min(wm[6], wm[7])),
					 min(min(min(wm[8], wm[9]), min(wm[10], wm[11])),
					     min(min(wm[12], wm[13]), min(wm[14], wm[15])))));
		__syncthreads();
#pragma unroll
		for (int k = (int) RS_TPT - 1; k >= 0; k--) {
			if (b0 + k < nt)
				nxt[b0 + k] = after;
			after = min(after, f[k]);
		}
		m = min(m, rmin);
	}
	if (fl)
		atomicOr(flags, fl);
}

// pass 3: every position's value -- the running sum at the end of its peer
// run when that end lies inside the tile (read back from LDS), else its own
// running sum for now -- stored row-wise; pass 4 gives the positions of the
// tile's open last run (its end in a later tile) that end's value, read
// from the output in place (end positions are never rewritten)
template <typename T1, typename T2>
__global__ __launch_bounds__(256) void
k_rs_write(const T1 *b, const int8_t *o, BUN n, bool fwd, const FSum<T2> *pre, const BUN *nxt, int pass, T2 *out,
	   uint32_t *flags)
{
	__shared__ FSum<T2> ls[256];
	__shared__ BUN lm[256];
	__shared__ RsStage<T1> sg;
	__shared__ T2 wo[RS_TILE + RS_TILE / RS_PER];
	const BUN t0 = (BUN) blockIdx.x * RS_TILE;
	const BUN q0 = t0 + threadIdx.x * RS_PER;
	const BUN tend = t0 + RS_TILE < n ? t0 + RS_TILE : n;
	uint32_t fl = 0;
	FSum<T2> x[RS_PER];
	bool e[RS_PER];
	rs_load<T1, T2>(b, o, n, fwd, sg, x, e);
	// the first run end at or after each lane's chunk, inside the tile
	BUN fe = ~(BUN) 0;
#pragma unroll
	for (int k = (int) RS_PER - 1; k >= 0; k--)
		if (e[k])
			fe = q0 + k;
	lm[threadIdx.x] = fe;
	__syncthreads();
	for (unsigned d = 1; d < 256; d <<= 1) {
		BUN y = lm[threadIdx.x];
		if (threadIdx.x + d < 256)
			y = min(y, lm[threadIdx.x + d]);
		__syncthreads();
		lm[threadIdx.x] = y;
		__syncthreads();
	}
	const BUN after = threadIdx.x + 1 < 256 ? lm[threadIdx.x + 1] : ~(BUN) 0;
	if (pass == 1) {
		// the open last run: positions whose end is in a later tile
		BUN endq = after != ~(BUN) 0 ? after : nxt[blockIdx.x];
		if (after != ~(BUN) 0)
			return;      // this lane's positions all end inside the tile
#pragma unroll
		for (int k = (int) RS_PER - 1; k >= 0; k--) {
			const BUN q = q0 + k;
			if (q >= n)
				continue;
			if (e[k])
				return;      // this position and the ones before it end inside the tile
			out[rs_row(q, n, fwd)] = out[rs_row(endq, n, fwd)];
		}
		return;
	}
	FSum<T2> acc;
	acc.zero();
#pragma unroll
	for (unsigned k = 0; k < RS_PER; k++)
		acc = rs_comb(acc, x[k], fl);
	FSum<T2> total;
	const FSum<T2> ex = rs_block_excl(acc, ls, fl, &total);
	FSum<T2> run = rs_comb(pre[blockIdx.x], ex, fl);
	const unsigned l0 = threadIdx.x * RS_PER;
#pragma unroll
	for (unsigned k = 0; k < RS_PER; k++) {
		run = rs_comb(run, x[k], fl);
		const unsigned i = l0 + k;
		wo[i + i / RS_PER] = run.nil ? (T2) __builtin_nan("") : run.v;
		if (run.nil && e[k])
			fl |= 1;
	}
	__syncthreads();
	// positions take their run end's value when it is in the tile (end
	// positions keep their own: nothing they read is rewritten)
	BUN endq = after;
#pragma unroll
	for (int k = (int) RS_PER - 1; k >= 0; k--) {
		const BUN q = q0 + k;
		if (e[k]) {
			endq = q;
			continue;
		}
		if (endq != ~(BUN) 0 && q < n) {
			const unsigned j = (unsigned) (endq - t0), i = l0 + k;
			wo[i + i / RS_PER] = wo[j + j / RS_PER];
		}
	}
	__syncthreads();
#pragma unroll
	for (unsigned k = 0; k < RS_PER; k++) {
		const unsigned i = k * 256 + threadIdx.x;
		if (t0 + i < tend)
			out[rs_row(t0 + i, n, fwd)] = wo[i + i / RS_PER];
	}
	if (fl)
		atomicOr(flags, fl);
}

template <typename T1, typename T2>
int
run_fsum_par(const T1 *bv, const int8_t *o, BUN n, bool fwd, T2 *out, uint32_t *flags)
{
	hipStream_t st = stream();
	const BUN nt = (n + RS_TILE - 1) / RS_TILE;
	DevBuf tot(nt * sizeof(FSum<T2>)), pre(nt * sizeof(FSum<T2>)), fend(nt * sizeof(BUN)), nxt(nt * sizeof(BUN));
	if (!tot.p || !pre.p || !fend.p || !nxt.p)
		return -1;
	if (nt > 0xffffffffull) {
		seterr("42000!GDKanalyticalsum: too many rows on the device path\n");
		return -1;
	}
	hipLaunchKernelGGL((k_rs_tile<T1, T2>), dim3((unsigned) nt), dim3(256), 0, st, bv, o, n, fwd,
			   tot.as<FSum<T2>>(), fend.as<BUN>(), flags);
	hipLaunchKernelGGL((k_rs_tiles<T2>), dim3(1), dim3(1024), 0, st, tot.as<FSum<T2>>(), fend.as<BUN>(), nt,
			   pre.as<FSum<T2>>(), nxt.as<BUN>(), flags);
	hipLaunchKernelGGL((k_rs_write<T1, T2>), dim3((unsigned) nt), dim3(256), 0, st, bv, o, n, fwd,
			   pre.as<FSum<T2>>(), nxt.as<BUN>(), 0, out, flags);
	hipLaunchKernelGGL((k_rs_write<T1, T2>), dim3((unsigned) nt), dim3(256), 0, st, bv, o, n, fwd,
			   pre.as<FSum<T2>>(), nxt.as<BUN>(), 1, out, flags);
	return sync() ? 0 : -1;
}

template <typename T1, typename T2>
int
run_fsum(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int frame_type)
{
	const BUN n = b->count;
	hipStream_t st = stream();
	const T1 *bv = (const T1 *) b->theap;
	T2 *out = (T2 *) r->theap;
	const bool frames = !(frame_type >= 3 && frame_type <= 6);
	DevBuf fl(64);
	if (!fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 64, st), "memset"))
		return -1;
	mgdk_bat *Sp = nullptr;
	int rc = -1;
	if (frame_type == 6) {
		hipLaunchKernelGGL((k_fsum_row<T1, T2>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, bv, n, out,
				   fl.as<uint32_t>());
	} else {
		Starts part;
		if (make_starts(p ? (const int8_t *) p->theap : nullptr, n, part, &Sp) < 0)
			goto out;
		if ((frame_type == 3 || frame_type == 4) && part.m == 1 && n >= fp_parallel_min()) {
			if (run_fsum_par<T1, T2>(bv, (const int8_t *) o->theap, n, frame_type == 3, out, fl.as<uint32_t>()) < 0)
				goto out;
		} else if (frame_type == 3 || frame_type == 4) {
			hipLaunchKernelGGL((k_fsum_replay<T1, T2>), dim3((unsigned) ((part.m + 63) / 64)), dim3(64), 0, st, bv, part,
					   (const int8_t *) o->theap, frame_type == 3, out, fl.as<uint32_t>());
		} else {
			if (n >= 0xffffffffull) {
				seterr("42000!GDKanalyticalsum: more than 2^32-1 rows on the device path\n");
				goto out;
			}
			DevBuf pidx(n * 4 + 4);
			if (!pidx.p)
				goto out;
			hipLaunchKernelGGL(k_avg_pidx, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, part, pidx.as<uint32_t>());
			if (frame_type == 5) {
				// dofsum per partition: the exact grouped float sum, the
				// partition index as the group id
				mgdk_bat *g = newbat(0, MGDK_oid, n);
				if (g == nullptr)
					goto out;
				g->count = n;
				hipLaunchKernelGGL(k_pidx_oid, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, pidx.as<uint32_t>(), n,
						   (oid *) g->theap);
				mgdk_bat *en = mgdk_BATdense(0, 0, part.m);
				mgdk_bat *ps = en ? mgdk_BATgroupsum(b, g, en, nullptr, MGDK_dbl, true) : nullptr;
				mgdk_BBPunfix(g);
				mgdk_BBPunfix(en);
				if (ps == nullptr) {
					// dofsum's message, then the analytic bailout's (GDKerror appends)
					char m[512];
					snprintf(m, sizeof(m), "%s42000!error while calculating floating-point sum\n", mgdk_GDKerrbuf());
					seterr("%s", m);
					goto out;
				}
				hipLaunchKernelGGL((k_fsum_bcast<T2>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st,
						   (const double *) ps->theap, pidx.as<uint32_t>(), n, out, fl.as<uint32_t>());
				const bool ok = sync();
				mgdk_BBPunfix(ps);
				if (!ok)
					goto out;
			} else {
				unsigned long long *hm = (unsigned long long *) pinned(8);
				DevBuf mx(64);
				if (!mx.p || !hip_ok(hipMemsetAsync(mx.p, 0, 8, st), "memset"))
					goto out;
				hipLaunchKernelGGL(k_avg_maxlen, dim3(grid_for(part.m, 1024, 1024)), dim3(256), 0, st, part,
						   mx.as<unsigned long long>());
				if (!hip_ok(hipMemcpyAsync(hm, mx.p, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
					goto out;
				AvgTree t{};
				int nlev = 1;
				while (nlev < AVG_MAX_LEVELS - 1 && ((*hm - 1) >> (4 * nlev)) > 0)
					nlev++;
				t.nlev = nlev;
				size_t tot = 0, offs[AVG_MAX_LEVELS] = {0};
				for (int L = 1; L <= nlev; L++) {
					offs[L] = tot;
					tot += ((n >> (4 * L)) + part.m + 1) * sizeof(FSum<T2>);
					tot = (tot + 255) & ~(size_t) 255;
				}
				DevBuf tree(tot);
				if (!tree.p)
					goto out;
				for (int L = 1; L <= nlev; L++)
					t.lvl[L] = tree.as<char>() + offs[L];
				for (int L = 1; L <= nlev; L++)
					hipLaunchKernelGGL((k_fsum_tree_level<T1, T2>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, bv, part,
							   pidx.as<uint32_t>(), t, L, fl.as<uint32_t>());
				hipLaunchKernelGGL((k_fsum_tree_query<T1, T2>), dim3(grid_for(n, 256, 16384)), dim3(256), 0, st, bv, part,
						   pidx.as<uint32_t>(), t, (const oid *) s->theap, (const oid *) e->theap, out,
						   fl.as<uint32_t>());
				if (!sync())
					goto out;
			}
		}
	}
	{
		uint32_t *h = (uint32_t *) pinned(16);
		if (!hip_ok(hipMemcpyAsync(h, fl.p, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			goto out;
		if (h[0] & 4) {
			seterr("22003!overflow in sum aggregate.\n42000!error while calculating floating-point sum\n");
			goto out;
		}
		if (h[0] & 2) {
			seterr("22003!overflow in calculation.\n");
			goto out;
		}
		r->count = n;
		r->tnil = (h[0] & 1) != 0;
		r->tnonil = (h[0] & 1) == 0;
		r->tsorted = r->trevsorted = r->tkey = n <= 1;
		rc = 0;
	}
out:
	mgdk_BBPunfix(Sp);
	return rc;
}

}  // namespace

extern "C" int
mgdk_GDKanalyticalsum(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tp1,
		      int tp2, int frame_type)
{
	if (r == nullptr || b == nullptr) {
		seterr("GDKanalyticalsum: NULL argument");
		return -1;
	}
	const bool fp = (tp1 == MGDK_flt && (tp2 == MGDK_flt || tp2 == MGDK_dbl)) || (tp1 == MGDK_dbl && tp2 == MGDK_dbl);
	if (fp && basetype(b->ttype) == tp1 && r->ttype == tp2) {
		const BUN n = b->count;
		if (n == 0) {
			r->count = 0;
			r->tnil = 0;
			r->tnonil = 1;
			return 0;
		}
		if ((p && (p->count != n || width_of(p->ttype) != 1)) || (o && (o->count != n || width_of(o->ttype) != 1))) {
			seterr("analytic: p and o must be bit BATs aligned with b");
			return -1;
		}
		if (!(frame_type >= 3 && frame_type <= 6) &&
		    (s == nullptr || e == nullptr || s->count < n || e->count < n || s->ttype != MGDK_oid || e->ttype != MGDK_oid)) {
			seterr("analytic: frame bounds s and e (oid BATs aligned with b) are required");
			return -1;
		}
		if ((frame_type == 3 || frame_type == 4) && o == nullptr) {
			seterr("analytic: the peer column o is required for this frame");
			return -1;
		}
		ProfScope prof("analyticalsum");
		if (tp1 == MGDK_flt && tp2 == MGDK_flt)
			return run_fsum<float, float>(r, p, o, b, s, e, frame_type);
		if (tp1 == MGDK_flt)
			return run_fsum<float, double>(r, p, o, b, s, e, frame_type);
		return run_fsum<double, double>(r, p, o, b, s, e, frame_type);
	}
	if (!sum_in_type(tp1) || basetype(b->ttype) != basetype(tp1) || !(tp2 == MGDK_lng || tp2 == MGDK_hge) ||
	    r->ttype != tp2) {
		seterr("42000!type combination (sum(%s)->%s) not supported.\n", atomname(tp1), atomname(tp2));
		return -1;
	}
	ProfScope prof("analyticalsum");
	return run_frames(r, p, o, b, s, e, frame_type, false, false, tp2 == MGDK_lng);
}

extern "C" int
mgdk_GDKanalyticalcount(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
			bool ignore_nils, int tpe, int frame_type)
{
	if (r == nullptr || b == nullptr) {
		seterr("GDKanalyticalcount: NULL argument");
		return -1;
	}
	(void) tpe;
	if (r->ttype != MGDK_lng) {
		seterr("GDKanalyticalcount: result must be a lng BAT");
		return -1;
	}
	const bool count_all = !ignore_nils || b->tnonil;
	if (!count_all && !sum_in_type(b->ttype)) {
		seterr("42000!GDKanalyticalcount: nil-skipping count of %s not supported on the device path",
		       atomname(b->ttype));
		return -1;
	}
	ProfScope prof("analyticalcount");
	return run_frames(r, p, o, b, s, e, frame_type, true, count_all, false);
}

// GDKanalyticalavg (gdk/gdk_analytic_statistics.c:364): r is a
// caller-allocated dbl BAT of count(b) slots
extern "C" int
mgdk_GDKanalyticalavg(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
		      int frame_type)
{
	if (r == nullptr || b == nullptr) {
		seterr("GDKanalyticalavg: NULL argument");
		return -1;
	}
	const int bt = basetype(tpe);
	if (!(bt == MGDK_bte || bt == MGDK_sht || bt == MGDK_int || bt == MGDK_lng || bt == MGDK_flt ||
	      bt == MGDK_dbl)) {
		if (bt == MGDK_hge)
			seterr("42000!GDKanalyticalavg: average of hge is not supported on the device path\n");
		else
			seterr("42000!average of type %s to dbl unsupported.\n", atomname(tpe));
		return -1;
	}
	if (basetype(b->ttype) != bt || r->ttype != MGDK_dbl) {
		seterr("GDKanalyticalavg: b must be of type tpe and r a dbl BAT");
		return -1;
	}
	const BUN n = b->count;
	if (n && r->theap == nullptr) {
		seterr("analytic: result BAT has no heap");
		return -1;
	}
	if (n == 0) {
		r->count = 0;
		r->tnil = 0;
		r->tnonil = 1;
		return 0;
	}
	if ((p && (p->count != n || width_of(p->ttype) != 1)) || (o && (o->count != n || width_of(o->ttype) != 1))) {
		seterr("analytic: p and o must be bit BATs aligned with b");
		return -1;
	}
	const bool frames = !(frame_type >= 3 && frame_type <= 6);
	if (frames && (s == nullptr || e == nullptr || s->count < n || e->count < n || s->ttype != MGDK_oid ||
		       e->ttype != MGDK_oid)) {
		seterr("analytic: frame bounds s and e (oid BATs aligned with b) are required");
		return -1;
	}
	if ((frame_type == 3 || frame_type == 4) && o == nullptr) {
		seterr("analytic: the peer column o is required for this frame");
		return -1;
	}
	ProfScope prof("analyticalavg");
	const bool isf = bt == MGDK_flt || bt == MGDK_dbl;
	if (!isf && (frame_type == 3 || frame_type == 4 || frame_type == 5))
		return run_frames(r, p, o, b, s, e, frame_type, false, false, false, true);
	switch (bt) {
	case MGDK_bte: return run_avg<int8_t>(r, p, o, b, s, e, frame_type);
	case MGDK_sht: return run_avg<int16_t>(r, p, o, b, s, e, frame_type);
	case MGDK_int: return run_avg<int32_t>(r, p, o, b, s, e, frame_type);
	case MGDK_lng: return run_avg<int64_t>(r, p, o, b, s, e, frame_type);
	case MGDK_flt: return run_avg<float>(r, p, o, b, s, e, frame_type);
	default: return run_avg<double>(r, p, o, b, s, e, frame_type);
	}
}

// GDKanalyticalavginteger (gdk/gdk_analytic_statistics.c:631): the average
// in the input's integer type, rounded half away from zero; r is a
// caller-allocated BAT of b's type
extern "C" int
mgdk_GDKanalyticalavginteger(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
			     int frame_type)
{
	if (r == nullptr || b == nullptr) {
		seterr("GDKanalyticalavginteger: NULL argument");
		return -1;
	}
	const int bt = basetype(tpe);
	if (!(bt == MGDK_bte || bt == MGDK_sht || bt == MGDK_int || bt == MGDK_lng)) {
		if (bt == MGDK_hge)
			seterr("42000!GDKanalyticalavginteger: average of hge is not supported on the device path\n");
		else
			seterr("42000!average of type %s to int unsupported.\n", atomname(tpe));
		return -1;
	}
	if (basetype(b->ttype) != bt || basetype(r->ttype) != bt) {
		seterr("GDKanalyticalavginteger: b and r must be of type tpe");
		return -1;
	}
	const BUN n = b->count;
	if (n && r->theap == nullptr) {
		seterr("analytic: result BAT has no heap");
		return -1;
	}
	if (n == 0) {
		r->count = 0;
		r->tnil = 0;
		r->tnonil = 1;
		return 0;
	}
	if ((p && (p->count != n || width_of(p->ttype) != 1)) || (o && (o->count != n || width_of(o->ttype) != 1))) {
		seterr("analytic: p and o must be bit BATs aligned with b");
		return -1;
	}
	const bool frames = !(frame_type >= 3 && frame_type <= 6);
	if (frames && (s == nullptr || e == nullptr || s->count < n || e->count < n || s->ttype != MGDK_oid ||
		       e->ttype != MGDK_oid)) {
		seterr("analytic: frame bounds s and e (oid BATs aligned with b) are required");
		return -1;
	}
	if ((frame_type == 3 || frame_type == 4) && o == nullptr) {
		seterr("analytic: the peer column o is required for this frame");
		return -1;
	}
	ProfScope prof("analyticalavginteger");
	if (frame_type == 3 || frame_type == 4 || frame_type == 5)
		return run_frames(r, p, o, b, s, e, frame_type, false, false, false, false, width_of(bt));
	switch (bt) {
	case MGDK_bte: return run_avg<int8_t, true>(r, p, o, b, s, e, frame_type);
	case MGDK_sht: return run_avg<int16_t, true>(r, p, o, b, s, e, frame_type);
	case MGDK_int: return run_avg<int32_t, true>(r, p, o, b, s, e, frame_type);
	default: return run_avg<int64_t, true>(r, p, o, b, s, e, frame_type);
	}
}
