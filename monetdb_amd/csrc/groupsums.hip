// groupsums.hip -- GROUP BY an ordered key with exact sums, fused: what
// BATgroup (gdk/gdk_group.c:940-975, ordered keys by consecutive comparison)
// followed by BATgroupsum per value column (gdk/gdk_aggr.c:1009-1080,
// skip_nils) and BATproject(extents, keys) produce -- the extents, the
// histogram, the group keys and the per-group sums -- in two passes over the
// keys and ONE over the values, without the per-row group-id column the
// GDK calls hand from one operator to the next.  It is the local step of
// the mergetable GROUP BY plan (opt_mergetable.c:1496-1670 mat_group /
// mat_group_aggr: per piece BATgroup + BATgroupsum, then the merge) as
// dist_group_aggr runs it; a column whose order is not known is refused
// (return 1) and the caller takes the GDK operators.
//
//   count  per 2048-row tile the group starts (row 0, or a key different
//          from the row before), then a scan of the tile counts (the
//          ordered BATgroup's first pass, k_sq_count);
//   sums   per tile: a lane takes 8 CONSECUTIVE rows (keys and values
//          loaded with 16-byte loads), numbers its starts from the tile's
//          prefix and a workgroup scan of the lanes' start counts, stores
//          extent + key at each start, reduces the runs inside the lane and
//          stores every group that starts and ends inside the tile (a
//          segmented scan over the 256 lanes carries a group across lanes);
//          the tile's first and last groups leave (group, partial) records
//          that k_gs_edges combines in order (no atomics).
#include "lookback.h"
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

constexpr int GSU = 8;                 // rows per lane
constexpr BUN GST = 256 * GSU;         // rows per tile
constexpr int GS_MAXV = 4;
#ifndef GS_FUSED_DEFAULT
#define GS_FUSED_DEFAULT 1   // the tile base by look-back inside the sums pass (no count pass)
#endif
#ifndef GS_STAGE
#define GS_STAGE 1       // group outputs staged in LDS and stored as runs (0: per-lane stores)
#endif

template <int NV>
struct GsPart {
	unsigned long long cnt;             // rows
	unsigned long long nn[NV];          // non-nil values per column
	hge s[NV];
	__device__ void clear()
	{
		cnt = 0;
#pragma unroll
		for (int v = 0; v < NV; v++) {
			nn[v] = 0;
			s[v] = 0;
		}
	}
	__device__ void add(const GsPart &o)
	{
		cnt += o.cnt;
#pragma unroll
		for (int v = 0; v < NV; v++) {
			nn[v] += o.nn[v];
			s[v] += o.s[v];
		}
	}
	__device__ GsPart shfl_up(int d) const
	{
		GsPart t;
		t.cnt = __shfl_up(cnt, d);
#pragma unroll
		for (int v = 0; v < NV; v++) {
			t.nn[v] = __shfl_up(nn[v], d);
			const unsigned long long lo = __shfl_up((unsigned long long) s[v], d);
			const unsigned long long hi = __shfl_up((unsigned long long) ((uhge) s[v] >> 64), d);
			t.s[v] = (hge) (((uhge) hi << 64) | lo);
		}
		return t;
	}
};

template <int NV>
struct GsEdge {
	unsigned long long g;               // ~0: none
	GsPart<NV> p;
};

struct GsOut {
	oid *ext;
	int64_t *hist;
	int64_t *key;
	hge *sum[GS_MAXV];
	uint32_t *flags;                    // bit 1: some group sum is nil
};

template <int NV>
__device__ __forceinline__ uint32_t
gs_put(const GsOut &o, unsigned long long g, const GsPart<NV> &p)
{
	uint32_t f = 0;
	o.hist[g] = (int64_t) p.cnt;
#pragma unroll
	for (int v = 0; v < NV; v++) {
		const bool nil = p.nn[v] == 0;
		o.sum[v][g] = nil ? NilOf<hge>::v() : p.s[v];
		f |= nil ? 2u : 0u;
	}
	return f;
}

template <int W>
struct KT;
template <> struct KT<4> { typedef int32_t T; };
template <> struct KT<8> { typedef int64_t T; };

// a wave's 512 rows [r0, r0 + 512) of a W-byte column go through the wave's
// LDS region: loaded with whole 1-KiB pieces per wave instruction (a
// lane-consecutive global load touches 32 lines per instruction instead of
// 8), then each lane takes its 8 consecutive rows back.  Rows past n repeat
// row n - 1.  stage_ld issues the loads (every column's before any store),
// stage_st stores them, stage_rd reads a lane's rows after the wave barrier.
typedef unsigned gs_u4 __attribute__((ext_vector_type(4)));

template <int W>
struct Stage {
	static constexpr int PL = 512 * W / 16 / 64;      // 16-byte pieces per lane
	gs_u4 v[PL];
	bool full;
};

template <int W>
__device__ __forceinline__ void
stage_ld(const typename KT<W>::T *p, BUN r0, BUN n, Stage<W> &s)
{
	const unsigned lane = __lane_id();
	s.full = r0 + 512 <= n;
	if (s.full) {
		const gs_u4 *src = (const gs_u4 *) (p + r0);
#pragma unroll
		for (int q = 0; q < Stage<W>::PL; q++)
			s.v[q] = __builtin_nontemporal_load(src + q * 64 + lane);
	}
}

template <int W>
__device__ __forceinline__ void
stage_st(const typename KT<W>::T *p, BUN r0, BUN n, const Stage<W> &s, typename KT<W>::T *region)
{
	const unsigned lane = __lane_id();
	if (s.full) {
#pragma unroll
		for (int q = 0; q < Stage<W>::PL; q++)
			((gs_u4 *) region)[q * 64 + lane] = s.v[q];
	} else {
		for (unsigned q = lane; q < 512; q += 64)
			region[q] = p[r0 + q < n ? r0 + q : n - 1];
	}
}

__device__ __forceinline__ void
stage_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int W>
__device__ __forceinline__ void
stage_rd(const typename KT<W>::T *region, typename KT<W>::T x[GSU])
{
	constexpr int NQ = GSU * W / 16;
	gs_u4 v[NQ];
#pragma unroll
	for (int q = 0; q < NQ; q++)
		v[q] = ((const gs_u4 *) (region + __lane_id() * GSU))[q];
	__builtin_memcpy(x, v, sizeof(typename KT<W>::T) * GSU);
}

// the key before the lane's first row
template <typename T>
__device__ __forceinline__ T
stage_pred(const T x[GSU], T before, BUN r0)
{
	const T up = __shfl_up(x[GSU - 1], 1);
	return __lane_id() == 0 ? (r0 > 0 ? before : x[0]) : up;
}

template <int KW>
__global__ __launch_bounds__(256) void
k_gs_count(const typename KT<KW>::T *k, BUN n, uint32_t *tcnt)
{
	typedef typename KT<KW>::T T;
	__shared__ T s_stage[4][512];
	const unsigned w = threadIdx.x >> 6;
	const BUN r0 = (BUN) blockIdx.x * GST + (BUN) w * 512;
	const BUN l0 = (BUN) blockIdx.x * GST + (BUN) threadIdx.x * GSU;
	uint32_t c = 0;
	if (r0 < n) {
		T x[GSU];
		Stage<KW> sk;
		stage_ld<KW>(k, r0, n, sk);
		const T before = r0 > 0 ? k[r0 - 1] : 0;
		stage_st<KW>(k, r0, n, sk, s_stage[w]);
		stage_sync();
		stage_rd<KW>(s_stage[w], x);
		T prev = stage_pred<T>(x, before, r0);
#pragma unroll
		for (int u = 0; u < GSU; u++) {
			c += (l0 + u < n) && (l0 + u == 0 || x[u] != prev);
			prev = x[u];
		}
	}
	c = block_reduce(c, [](uint32_t a, uint32_t b) { return a + b; });
	if (threadIdx.x == 0)
		tcnt[blockIdx.x] = c;
}

// LB: the tile's first group id comes from a decoupled look-back over the
// tiles' start counts (mgdk_lb::lookback on lbst, zero before the launch)
// instead of the count pass's prefix tpre.  Tiles are numbered by blockIdx,
// no ticket (293K same-word ticket atomics cost more than the count pass):
// each XCD dispatches its share of the grid in blockIdx order, so the lowest
// unfinished tile is always resident or next on its XCD and the walk always
// ends; a walk that exceeds the spin limit sets lberr and the host reruns
// the two-pass form
template <int KW, int VW, int NV, bool LB>
__global__ __launch_bounds__(256) void
k_gs_sums(const typename KT<KW>::T *k, const void *const *vals, BUN n, oid hseq, const uint64_t *tpre, GsOut o,
	  GsEdge<NV> *edges, uint64_t *lbst, uint32_t *lberr)
{
	__shared__ uint64_t s_tbase;
	typedef typename KT<KW>::T T;
	typedef typename KT<VW>::T V;
	__shared__ GsPart<NV> s_wtot[4];
	__shared__ int s_wflag[4];
	__shared__ uint32_t s_wst[4];
	// the rows' staging area (s_k, s_v), reused once the rows are in
	// registers for the tile's group outputs
	constexpr size_t KBY = 4 * 512 * sizeof(T), VBY = (size_t) NV * 4 * 512 * sizeof(V);
	__shared__ __attribute__((aligned(16))) unsigned char s_raw[KBY + VBY];
	T (*s_k)[512] = (T (*)[512]) s_raw;
	V (*s_v)[4][512] = (V (*)[4][512]) (s_raw + KBY);
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const BUN t = blockIdx.x;
	const BUN t0 = t * GST, l0 = t0 + (BUN) tid * GSU, r0 = t0 + (BUN) w * 512;
	const bool live = l0 < n;
	T x[GSU];
	V y[NV][GSU];
	bool st[GSU];
	uint32_t ns = 0;
	if (r0 < n) {
		// the value columns first: their loads are in flight while the keys
		// are staged and compared
		Stage<VW> sv[NV];
		Stage<KW> sk;
#pragma unroll
		for (int v = 0; v < NV; v++)
			stage_ld<VW>((const V *) vals[v], r0, n, sv[v]);
		stage_ld<KW>(k, r0, n, sk);
		const T before = r0 > 0 ? k[r0 - 1] : 0;
#pragma unroll
		for (int v = 0; v < NV; v++)
			stage_st<VW>((const V *) vals[v], r0, n, sv[v], s_v[v][w]);
		stage_st<KW>(k, r0, n, sk, s_k[w]);
		stage_sync();
#pragma unroll
		for (int v = 0; v < NV; v++)
			stage_rd<VW>(s_v[v][w], y[v]);
		stage_rd<KW>(s_k[w], x);
		T prev = stage_pred<T>(x, before, r0);
#pragma unroll
		for (int u = 0; u < GSU; u++) {
			st[u] = (l0 + u < n) && (l0 + u == 0 || x[u] != prev);
			prev = x[u];
			ns += st[u];
		}
	} else {
#pragma unroll
		for (int u = 0; u < GSU; u++)
			st[u] = false;
	}
	// starts before the lane in the tile: workgroup exclusive scan
	uint32_t xs = ns;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint32_t q = __shfl_up(xs, d);
		if (lane >= (unsigned) d)
			xs += q;
	}
	if (lane == 63)
		s_wst[w] = xs;
	// the lane's runs: pre = rows before its first start, post = from its
	// last start to its end; runs between two of its starts are complete
	GsPart<NV> pre, cur;
	pre.clear();
	cur.clear();
	bool seen = false;
	uint32_t of = 0;
	__syncthreads();
	uint32_t lpre = xs - ns;
	for (unsigned q = 0; q < w; q++)
		lpre += s_wst[q];
	const uint32_t tst = s_wst[0] + s_wst[1] + s_wst[2] + s_wst[3];
	const bool tile_has_start = tst != 0;
	constexpr uint32_t GCAP = (uint32_t) ((KBY + VBY) / (24 + 16 * NV)) & ~1u;
	const bool stg = GS_STAGE && tst <= GCAP;
	// LB with staged outputs: the tile publishes its start count now and
	// numbers its groups from 0 while it reduces and stages them; the
	// look-back runs at the end, when its predecessors have long published
	// (a look-back before the work made every tile wait on the one before
	// it), and only the copy-out and the edge records need the real base
	const bool late = LB && stg;
	uint64_t tbase;
	if constexpr (LB) {
		if (late) {
			// tile 0's base is 0: its inclusive count is known already
			if (tid == 0)
				mgdk_lb::lb_store(&lbst[t], (t == 0 ? mgdk_lb::ST_PRE : mgdk_lb::ST_AGG) | tst);
			tbase = 0;
		} else {
			if (w == 0) {
				// a predecessor's wait is microseconds; 2^20 spins (~1 s) means
				// the dispatch order assumption failed: give up, the host reruns
				const uint64_t ex = mgdk_lb::lookback(lbst, (uint32_t) t, tst, lberr, 1u << 20);
				if (lane == 0)
					s_tbase = ex;
			}
			__syncthreads();
			tbase = s_tbase;
		}
	} else {
		tbase = tpre[t];
	}
	// the groups starting in the tile, [tbase, tbase + tst), are written by
	// this tile only (ext / key all of them, hist / sums all but the last,
	// which the tail edge record carries): staged in LDS (the rows are in
	// registers since the barrier above) and stored as contiguous runs
	// after the tile, when they fit
	oid *l_ext = (oid *) s_raw;
	int64_t *l_key = (int64_t *) (s_raw + 8 * GCAP), *l_hist = (int64_t *) (s_raw + 16 * GCAP);
	hge *l_sum = (hge *) (s_raw + 24 * GCAP);     // [NV][GCAP]
	auto put = [&](unsigned long long g, const GsPart<NV> &p) -> uint32_t {
		const uint64_t j = g - tbase;
		if (!stg || j >= tst)
			return gs_put<NV>(o, g, p);
		uint32_t f = 0;
		l_hist[j] = (int64_t) p.cnt;
#pragma unroll
		for (int v = 0; v < NV; v++) {
			const bool nil = p.nn[v] == 0;
			l_sum[(size_t) v * GCAP + j] = nil ? NilOf<hge>::v() : p.s[v];
			f |= nil ? 2u : 0u;
		}
		return f;
	};
	// group id of the lane's rows: tbase + (starts in the tile up to the row) - 1
	uint64_t gcur = tbase + lpre - 1;
	if (live) {
#pragma unroll
		for (int u = 0; u < GSU; u++) {
			const BUN i = l0 + u;
			if (st[u]) {
				if (seen)
					of |= put(gcur, cur);             // a run inside the lane
				else
					pre = cur;
				seen = true;
				cur.clear();
				gcur++;
				// the key widened to lng (nil stays nil), as dist_group_aggr's widen
				const int64_t kw = KW == 4 && is_nil((int32_t) x[u]) ? INT64_MIN : (int64_t) x[u];
				if (stg) {
					l_ext[gcur - tbase] = hseq + i;
					l_key[gcur - tbase] = kw;
				} else {
					o.ext[gcur] = hseq + i;
					o.key[gcur] = kw;
				}
			}
			if (i < n) {
				cur.cnt++;
#pragma unroll
				for (int v = 0; v < NV; v++) {
					const V a = y[v][u];
					if (!is_nil(a)) {
						cur.nn[v]++;
						cur.s[v] += (hge) a;
					}
				}
			}
		}
	}
	if (!seen) {
		pre = cur;          // no start: the lane continues its left neighbour's group
		cur.clear();
	}
	// segmented inclusive scan over the lanes of v = seen ? post : pre,
	// a segment beginning at every lane with a start
	GsPart<NV> S = seen ? cur : pre;
	bool f = seen;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const GsPart<NV> q = S.shfl_up(d);
		const bool qf = __shfl_up((int) f, d) != 0;
		if (lane >= (unsigned) d) {
			if (!f)
				S.add(q);
			f |= qf;
		}
	}
	// across the 4 waves: each wave's tail (S of lane 63) and whether it holds
	// a start, combined in order into the carry entering wave w
	if (lane == 63) {
		s_wtot[w] = S;
		s_wflag[w] = f;
	}
	__syncthreads();
	GsPart<NV> carry;
	carry.clear();
	bool cflag = false;        // some start in the waves before w
	for (unsigned q = 0; q < w; q++) {
		if (s_wflag[q])
			carry = s_wtot[q];
		else
			carry.add(s_wtot[q]);
		cflag |= s_wflag[q] != 0;
	}
	if (!f)
		S.add(carry);          // no start in lanes 0..lane of this wave: the carry continues
	// S(lane - 1): the open group's partial entering this lane
	GsPart<NV> Sin = S.shfl_up(1);
	const bool fin = __shfl_up((int) f, 1) != 0;
	if (lane == 0) {
		Sin = carry;
	}
	// some start in the tile before this lane
	const bool before = (lane == 0 ? cflag : (fin || cflag));
	// the group of the lane's first rows ends before its first start
	GsPart<NV> tot = Sin;
	tot.add(pre);
	if (seen && before)
		of |= put(tbase + lpre - 1, tot);
	if constexpr (LB) {
		if (late && w == 0) {
			const uint64_t ex = mgdk_lb::lookback(lbst, (uint32_t) t, tst, lberr, 1u << 20);
			if (lane == 0)
				s_tbase = ex;
		}
	}
	if (stg)
		__syncthreads();
	if (late)
		tbase = s_tbase;
	if (seen && !before)
		edges[2 * t] = GsEdge<NV>{tbase - 1, tot};      // the tile's head group
	if (tid == 255) {
		if (!tile_has_start) {
			// one group over the whole tile: head = everything, tail = empty
			edges[2 * t] = GsEdge<NV>{tbase - 1, S};
			GsPart<NV> z;
			z.clear();
			edges[2 * t + 1] = GsEdge<NV>{tbase - 1, z};
		} else {
			edges[2 * t + 1] = GsEdge<NV>{tbase + lpre + ns - 1, S};   // the tile's last group
		}
	}
	if (stg) {
		for (uint32_t j = tid; j < tst; j += 256) {
			o.ext[tbase + j] = l_ext[j];
			o.key[tbase + j] = l_key[j];
		}
		for (uint32_t j = tid; j + 1 < tst; j += 256) {
			o.hist[tbase + j] = l_hist[j];
#pragma unroll
			for (int v = 0; v < NV; v++)
				o.sum[v][tbase + j] = l_sum[(size_t) v * GCAP + j];
		}
	}
	for (int q = 32; q > 0; q >>= 1)
		of |= __shfl_xor(of, q);
	if (lane == 0 && of)
		publish_or(o.flags, of);
}

// the tile edge records in order: a group's records are consecutive; the
// first record of each group sums them and stores the group.  A group over
// more than GS_ECAP records (a key spanning that many tiles) is left to
// k_gs_edges_long: its first record goes to a list instead of one thread
// walking it
constexpr BUN GS_ECAP = 256;

template <int NV>
__global__ __launch_bounds__(256) void
k_gs_edges(const GsEdge<NV> *e, BUN ne, BUN ngrp, GsOut o, uint32_t *longs)
{
	uint32_t f = 0;
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < ne; j += (BUN) gridDim.x * blockDim.x) {
		const unsigned long long g = e[j].g;
		if (g >= ngrp || (j > 0 && e[j - 1].g == g))
			continue;
		GsPart<NV> p = e[j].p;
		BUN q = j + 1;
		for (; q < ne && q < j + GS_ECAP && e[q].g == g; q++)
			p.add(e[q].p);
		if (q < ne && q == j + GS_ECAP && e[q].g == g) {
			longs[1 + atomicAdd(&longs[0], 1u)] = (uint32_t) j;
			continue;
		}
		f |= gs_put<NV>(o, g, p);
	}
	for (int q = 32; q > 0; q >>= 1)
		f |= __shfl_xor(f, q);
	if (__lane_id() == 0 && f)
		publish_or(o.flags, f);
}

// the long groups: one workgroup sums a group's records 256 at a time (a
// group's records are consecutive and its key never comes back, so the
// first chunk that holds another key ends it)
template <int NV>
__global__ __launch_bounds__(256) void
k_gs_edges_long(const GsEdge<NV> *e, BUN ne, BUN ngrp, GsOut o, const uint32_t *longs)
{
	__shared__ GsPart<NV> s_p[4];
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const uint32_t nl = longs[0];
	for (uint32_t k = blockIdx.x; k < nl; k += gridDim.x) {
		const BUN j = longs[1 + k];
		const unsigned long long g = e[j].g;
		GsPart<NV> p;
		p.clear();
		for (BUN c = j;; c += 256) {
			const BUN q = c + tid;
			const bool in = q < ne && e[q].g == g;
			if (in)
				p.add(e[q].p);
			if (__syncthreads_or(!in))
				break;
		}
		for (int d = 32; d > 0; d >>= 1) {
			GsPart<NV> t;
			t.cnt = __shfl_xor(p.cnt, d);
#pragma unroll
			for (int v = 0; v < NV; v++) {
				t.nn[v] = __shfl_xor(p.nn[v], d);
				const unsigned long long lo = __shfl_xor((unsigned long long) p.s[v], d);
				const unsigned long long hi = __shfl_xor((unsigned long long) ((uhge) p.s[v] >> 64), d);
				t.s[v] = (hge) (((uhge) hi << 64) | lo);
			}
			p.add(t);
		}
		if (lane == 0)
			s_p[w] = p;
		__syncthreads();
		if (tid == 0) {
			GsPart<NV> tot = s_p[0];
			for (int q = 1; q < 4; q++)
				tot.add(s_p[q]);
			const uint32_t f = gs_put<NV>(o, g, tot);
			if (f)
				publish_or(o.flags, f);
		}
		__syncthreads();
	}
}

template <int KW, int VW, int NV>
int
gs_run(const void *kb, const void *const *vals_dev, BUN n, oid hseq, const uint64_t *tpre, BUN nt, BUN ngrp,
       GsOut o, void *edges, uint32_t *longs, uint64_t *lbst, uint32_t *lberr)
{
	hipStream_t st = stream();
	if (lbst)
		hipLaunchKernelGGL((k_gs_sums<KW, VW, NV, true>), dim3((unsigned) nt), dim3(256), 0, st,
				   (const typename KT<KW>::T *) kb, vals_dev, n, hseq, tpre, o, (GsEdge<NV> *) edges, lbst, lberr);
	else
		hipLaunchKernelGGL((k_gs_sums<KW, VW, NV, false>), dim3((unsigned) nt), dim3(256), 0, st,
				   (const typename KT<KW>::T *) kb, vals_dev, n, hseq, tpre, o, (GsEdge<NV> *) edges, lbst, lberr);
	const BUN ne = 2 * nt;
	if (!hip_ok(hipMemsetAsync(longs, 0, 4, st), "memset"))
		return -1;
	hipLaunchKernelGGL(k_gs_edges<NV>, dim3(grid_for(ne, 1024, 4096)), dim3(256), 0, st, (const GsEdge<NV> *) edges,
			   ne, ngrp, o, longs);
	hipLaunchKernelGGL(k_gs_edges_long<NV>, dim3(256), dim3(256), 0, st, (const GsEdge<NV> *) edges, ne, ngrp, o,
			   (const uint32_t *) longs);
	return 0;
}

template <int KW, int VW>
int
gs_nv(int nv, const void *kb, const void *const *vals_dev, BUN n, oid hseq, const uint64_t *tpre, BUN nt, BUN ngrp,
      GsOut o, void *edges, uint32_t *longs, uint64_t *lbst, uint32_t *lberr)
{
	switch (nv) {
	case 1: return gs_run<KW, VW, 1>(kb, vals_dev, n, hseq, tpre, nt, ngrp, o, edges, longs, lbst, lberr);
	case 2: return gs_run<KW, VW, 2>(kb, vals_dev, n, hseq, tpre, nt, ngrp, o, edges, longs, lbst, lberr);
	case 3: return gs_run<KW, VW, 3>(kb, vals_dev, n, hseq, tpre, nt, ngrp, o, edges, longs, lbst, lberr);
	default: return gs_run<KW, VW, 4>(kb, vals_dev, n, hseq, tpre, nt, ngrp, o, edges, longs, lbst, lberr);
	}
}

bool
gs_key_ok(const mgdk_bat *b)
{
	const int t = basetype(b->ttype);
	return b->theap != nullptr && (t == MGDK_int || t == MGDK_lng || t == MGDK_oid || t == MGDK_date ||
				       t == MGDK_timestamp || t == MGDK_daytime);
}

bool
gs_val_ok(const mgdk_bat *b)
{
	const int t = basetype(b->ttype);
	return b->theap != nullptr && (t == MGDK_int || t == MGDK_lng);
}

}  // namespace

extern "C" int
mgdk_group_sums_ordered(mgdk_bat **extents, mgdk_bat **histo, mgdk_bat **keys, mgdk_bat **sums, mgdk_bat *b,
			mgdk_bat **vals, int nvals)
{
	*extents = *histo = *keys = nullptr;
	for (int v = 0; v < nvals && sums; v++)
		sums[v] = nullptr;
	if (b == nullptr || vals == nullptr || sums == nullptr || nvals < 1 || nvals > GS_MAXV) {
		seterr("group_sums_ordered: 1 to %d value columns", GS_MAXV);
		return -1;
	}
	const BUN n = b->count;
	if (!gs_key_ok(b))
		return 1;
	for (int v = 0; v < nvals; v++) {
		if (vals[v] == nullptr || vals[v]->count != n || vals[v]->hseqbase != b->hseqbase) {
			seterr("b and g must be aligned\n");
			return -1;
		}
		if (!gs_val_ok(vals[v]) || vals[v]->twidth != vals[0]->twidth ||
		    ((uintptr_t) vals[v]->theap & 15) != 0)
			return 1;
	}
	if (((uintptr_t) b->theap & 15) != 0 || n == 0 || n >= ((BUN) 1 << 40))
		return 1;
	// ordered keys only (equal keys consecutive): BATgroup's consecutive-
	// comparison path; the order is looked up as BATgroup does
	if (!b->tsorted && !b->trevsorted && !mgdk_BATordered(b) && !mgdk_BATordered_rev(b))
		return 1;
	ProfScope prof("group_sums_ordered");
	hipStream_t st = stream();
	const int kw = b->twidth, vw = vals[0]->twidth;
	const BUN nt = (n + GST - 1) / GST;
	// two-pass (default): a count pass + scan first, outputs sized exactly.
	// Fused (MGDK_GS_FUSED=1): the tile's first group id comes from the
	// look-back inside the sums pass, so the keys are read once; the outputs
	// are sized for n groups (56 B per row at two sums, capped at 48 GiB) and
	// the count is the last tile's inclusive prefix; a look-back that did not
	// complete reruns two-pass.  With the look-back after the staging the
	// fused form is 1.4 % faster at SF100 (5.20 vs 5.27 ms,
	// profiles/r05/gsums_late/): the look-back's round trips cost about what
	// the count pass does, so the exact two-pass form stays the default.  A
	// persistent fused form (next tile's rows fetched during the look-back)
	// needed 240 VGPRs in its tile loop, against 98 for one tile per block.
	// Round 6: on this round's boxes (stores slower than round 5's) the fused
	// form is 4 % faster at SF100 (5.24 vs 5.44-5.47 ms, profiles/r06/gsums_fused/)
	// and is the default; MGDK_GS_FUSED=0 selects the two-pass form.
	const bool fused_on = getenv("MGDK_GS_FUSED") ? atoi(getenv("MGDK_GS_FUSED")) != 0 : GS_FUSED_DEFAULT != 0;   // read per call (tests)
	bool fused = fused_on && nt < 0xffffffffull && n * (24 + 16 * (BUN) nvals) <= ((BUN) 48 << 30);
	DevBuf vp(64);
	const size_t esz = sizeof(GsEdge<GS_MAXV>);
	// the tiles' edge records, then the list of groups over more than
	// GS_ECAP records (k_gs_edges_long)
	const size_t lgoff = (2 * nt * esz + 255) & ~(size_t) 255;
	DevBuf edges(lgoff + (2 * nt / GS_ECAP + 2) * 4);
	if (!vp.p || !edges.p)
		return -1;
	uint32_t *longs = (uint32_t *) ((char *) edges.p + lgoff);
	uint32_t *flags = (uint32_t *) meta_buf();
	const void *hv[GS_MAXV] = {};
	for (int v = 0; v < nvals; v++)
		hv[v] = vals[v]->theap;
	if (!hip_ok(hipMemcpyAsync(vp.p, stage_host(hv, sizeof hv), sizeof hv, hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	const void *const *vd = vp.as<const void *const>();
	mgdk_bat *en = nullptr, *hn = nullptr, *kn = nullptr;
	mgdk_bat *sn[GS_MAXV] = {};
	auto drop = [&]() {
		mgdk_BBPunfix(en);
		mgdk_BBPunfix(hn);
		mgdk_BBPunfix(kn);
		en = hn = kn = nullptr;
		for (int v = 0; v < nvals; v++) {
			mgdk_BBPunfix(sn[v]);
			sn[v] = nullptr;
		}
		return -1;
	};
	uint64_t ngrp = 0;
	uint32_t *hf = (uint32_t *) pinned(32);
	if (hf == nullptr)
		return -1;
	for (;;) {
		DevBuf tc(fused ? 8 : nt * 4 + 8), tp(fused ? 8 : nt * 8 + 8), lbs(fused ? nt * 8 + 64 : 8);
		if (!tc.p || !tp.p || !lbs.p)
			return -1;
		uint64_t *lbst = fused ? lbs.as<uint64_t>() : nullptr;
		uint32_t *lberr = fused ? (uint32_t *) (lbst + nt) : nullptr;
		uint64_t cap;
		if (fused) {
			if (!hip_ok(hipMemsetAsync(lbs.p, 0, nt * 8 + 64, st), "memset"))
				return -1;
			cap = n;
		} else {
			if (kw == 4)
				hipLaunchKernelGGL(k_gs_count<4>, dim3((unsigned) nt), dim3(256), 0, st, (const int32_t *) b->theap,
						   n, tc.as<uint32_t>());
			else
				hipLaunchKernelGGL(k_gs_count<8>, dim3((unsigned) nt), dim3(256), 0, st, (const int64_t *) b->theap,
						   n, tc.as<uint32_t>());
			if (exclusive_scan(tc.as<uint32_t>(), tp.as<uint64_t>(), nt, &ngrp) < 0)
				return -1;
			cap = ngrp;
		}
		en = newbat(0, MGDK_oid, cap);
		hn = newbat(0, MGDK_lng, cap);
		kn = newbat(0, MGDK_lng, cap);
		bool ok = en && hn && kn;
		for (int v = 0; v < nvals && ok; v++)
			ok = (sn[v] = newbat(0, MGDK_hge, cap)) != nullptr;
		if (!ok || !hip_ok(hipMemsetAsync(flags, 0, 8, st), "memset"))
			return drop();
		GsOut o{};
		o.ext = (oid *) en->theap;
		o.hist = (int64_t *) hn->theap;
		o.key = (int64_t *) kn->theap;
		for (int v = 0; v < nvals; v++)
			o.sum[v] = (hge *) sn[v]->theap;
		o.flags = flags;
		const uint64_t *tpre = tp.as<uint64_t>();
		if (kw == 4 && vw == 4)
			gs_nv<4, 4>(nvals, b->theap, vd, n, b->hseqbase, tpre, nt, cap, o, edges.p, longs, lbst, lberr);
		else if (kw == 4)
			gs_nv<4, 8>(nvals, b->theap, vd, n, b->hseqbase, tpre, nt, cap, o, edges.p, longs, lbst, lberr);
		else if (vw == 4)
			gs_nv<8, 4>(nvals, b->theap, vd, n, b->hseqbase, tpre, nt, cap, o, edges.p, longs, lbst, lberr);
		else
			gs_nv<8, 8>(nvals, b->theap, vd, n, b->hseqbase, tpre, nt, cap, o, edges.p, longs, lbst, lberr);
		if (!hip_ok(hipMemcpyAsync(hf, flags, 4, hipMemcpyDeviceToHost, st), "memcpy") ||
		    (fused && (!hip_ok(hipMemcpyAsync(hf + 2, lbst + (nt - 1), 8, hipMemcpyDeviceToHost, st), "memcpy") ||
			       !hip_ok(hipMemcpyAsync(hf + 4, lberr, 4, hipMemcpyDeviceToHost, st), "memcpy"))) ||
		    !sync())
			return drop();
		if (!fused)
			break;
		uint64_t last;
		memcpy(&last, hf + 2, 8);
		if (hf[4] == 0 && (last >> 62) == 2) {
			ngrp = last & mgdk_lb::ST_VAL;
			break;
		}
		// a look-back that did not complete: the two-pass form
		drop();
		fused = false;
	}
	const bool anynil = (hf[0] & 2) != 0;
	// properties as BATgroup / BATgroupsum leave them (extents ascending and
	// key, the histogram and sums unknown, keys ordered as b)
	en->count = hn->count = kn->count = ngrp;
	en->tsorted = 1;
	en->trevsorted = ngrp <= 1;
	en->tkey = 1;
	en->tnonil = 1;
	en->tseqbase = MGDK_OID_NIL;
	hn->tsorted = hn->trevsorted = hn->tkey = ngrp <= 1;
	hn->tnonil = 1;
	kn->tsorted = b->tsorted || ngrp <= 1;
	kn->trevsorted = b->trevsorted || ngrp <= 1;
	kn->tkey = 1;
	kn->tnonil = b->tnonil;
	kn->tnil = !b->tnonil && b->tnil;
	for (int v = 0; v < nvals; v++) {
		sn[v]->count = ngrp;
		sn[v]->tsorted = sn[v]->trevsorted = sn[v]->tkey = ngrp <= 1;
		sn[v]->tnonil = !anynil;
		sn[v]->tnil = anynil;
		sums[v] = sn[v];
	}
	*extents = en;
	*histo = hn;
	*keys = kn;
	return 0;
}
