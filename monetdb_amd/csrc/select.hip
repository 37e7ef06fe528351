// select.hip -- BATselect / BATthetaselect on the MI355X.
//
// Host side restates the argument normalisation of BATselect
// (gdk/gdk_select.c:1342-1564, nil/anti table :1288-1340) and of the typed
// scan (scanfunc, :300-446), which reduces every request to one of a few
// closed predicates.  The device side is a single-pass, order-preserving
// stream compaction:
//   * a tile = 8 rows x 256 lanes x 16 B of the column (8 KiB of int32);
//     every lane issues its eight 16-B loads up front (coalesced, 1 KiB per
//     wave instruction), evaluates the predicate and keeps a hit bitmask;
//   * ranks inside a wave come from __ballot + popcount of the per-lane hit
//     counts (no LDS traffic), ranks of the 32 (row, wave) segments of a tile
//     from one wave-level scan in LDS;
//   * the tile's output offset comes from decoupled look-back over
//     per-tile 8-byte status granules {flag:2, count:62} written and polled
//     with agent-scope relaxed atomics (MI355X_MICROARCH.md "Valid forms",
//     R2 granule hand-off), tiles being numbered in dispatch order by an
//     atomic ticket so every predecessor is already resident;
//   * the sorted oid list is written directly; a dense result is
//     virtualised like virtualize() (gdk_select.c:31-89).
// Input bytes are read exactly once; output = 8 B per hit.
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <limits>
#include <vector>

#include "lookback.h"
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

enum SelMode { SEL_RANGE = 0, SEL_ANTI = 1, SEL_EQ = 2, SEL_EQNIL = 3, SEL_NOTNIL = 4 };

template <typename T>
struct SelPred {
	int mode;
	bool nil_matches;
	T vl, vh;
};

// the predicate with the mode fixed at compile time (branch-free per value)
template <int MODE, typename T>
__device__ __forceinline__ bool
sel_eval(const SelPred<T> &p, T v)
{
	if constexpr (MODE == SEL_RANGE)
		return v >= p.vl && v <= p.vh;
	else if constexpr (MODE == SEL_ANTI)
		return p.nil_matches ? (is_nil(v) || v <= p.vl || v >= p.vh)
				     : (!is_nil(v) && (v <= p.vl || v >= p.vh));
	else if constexpr (MODE == SEL_EQ)
		return v == p.vl;
	else if constexpr (MODE == SEL_EQNIL)
		return is_nil(v);
	else
		return !is_nil(v);
}

using namespace mgdk_lb;

template <int BITS>
__device__ __forceinline__ void
wave_rank(uint32_t c, uint64_t lt, uint32_t &excl, uint32_t &tot)
{
	excl = 0;
	tot = 0;
#pragma unroll
	for (int b = 0; b < BITS; b++) {
		uint64_t bal = __ballot((c >> b) & 1u);
		excl += (uint32_t) __popcll(bal & lt) << b;
		tot += (uint32_t) __popcll(bal) << b;
	}
}

template <int V> struct Bits { static constexpr int v = V <= 1 ? 1 : V <= 3 ? 2 : V <= 7 ? 3 : V <= 15 ? 4 : 5; };

template <typename T>
struct SelArgs {
	const T *col;             // b's tail; value of oid o is col[o - hseq]
	oid hseq;
	const T *col_al;          // dense: 16-B aligned base, slot j -> col_al[j]
	const oid *cand_al;       // materialized: 16-B aligned base of candidate oids
	oid cseq;                 // dense: oid of slot `shift`
	uint64_t n;               // number of candidates
	uint32_t shift;           // leading invalid slots (alignment)
	uint32_t ntiles;
	SelPred<T> pred;
	oid *out;
	uint64_t *status;         // [ntiles] look-back granules
	uint32_t *ticket;         // dynamic tile numbering
	uint64_t *meta;           // [0] total count, [1] error flags
	uint64_t *hmeta;          // streamed: meta[0..3] also stored to this pinned host copy (or null)
};

// rows of 256 lanes x 16 B per tile: 32 for a dense scan (128 KiB of input per
// tile, so one tile ticket per 128 KiB: a single counter sustains only ~88
// atomics/us, MI355X_MICROARCH.md "dequeue"), 16 for candidate lists;
// loads are issued in batches of 8 rows
#ifndef MGDK_SEL_EXP
#define MGDK_SEL_EXP 0
#endif
#ifndef MGDK_SEL_STREAM
#define MGDK_SEL_STREAM 1
#endif
#ifndef MGDK_SEL_ROWS
#define MGDK_SEL_ROWS 32
#endif
#ifndef MGDK_SEL_BATCH
#define MGDK_SEL_BATCH 8
#endif
// oids staged in LDS per dense round of the write pass (LDS per workgroup:
// 8 B per slot, so 2048 leaves room for 8 workgroups per CU)
#ifndef MGDK_SEL_SCH
#define MGDK_SEL_SCH 2048
#endif
// the streamed scan's result words go straight to pinned host memory (no
// device-to-host copy after the write pass)
#ifndef MGDK_SEL_HMETA
#define MGDK_SEL_HMETA 1
#endif
template <bool MAT> constexpr int sel_rows() { return MAT ? 16 : MGDK_SEL_ROWS; }
constexpr int BATCH = MGDK_SEL_BATCH;

template <typename T, bool MAT, int MODE>
__global__ __launch_bounds__(256) void
k_select(SelArgs<T> a)
{
	constexpr int V = MAT ? 2 : (int) (16 / sizeof(T));
	constexpr int ROWS = sel_rows<MAT>();
	constexpr int BITS = Bits<V>::v;
	typedef T vec_t __attribute__((ext_vector_type(V)));
	typedef oid ovec_t __attribute__((ext_vector_type(2)));
	__shared__ uint32_t s_tile;
	__shared__ uint32_t s_off[ROWS * 4];
	__shared__ uint64_t s_prefix;

	const unsigned tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	if (tid == 0)
#if MGDK_SEL_EXP & 1
		s_tile = blockIdx.x;
#else
		s_tile = atomicAdd(a.ticket, 1u);
#endif
	__syncthreads();
	const uint32_t tile = s_tile;
	const uint64_t nslots = a.n + a.shift;
	const uint64_t lt = lanemask_lt();
	const uint64_t j_first = (uint64_t) tile * ROWS * 256 * V;
	// interior tiles: every slot valid -> all loads issued before any use
	const bool full = tile > 0 && j_first + (uint64_t) ROWS * 256 * V <= nslots;

	uint32_t hm[ROWS];
	oid cv[MAT ? ROWS * 2 : 1];
	(void) cv;
	if (full) {
#pragma unroll
		for (int b0 = 0; b0 < ROWS; b0 += BATCH) {
			if constexpr (!MAT) {
				vec_t x[BATCH];
#pragma unroll
				for (int r = 0; r < BATCH; r++)
					x[r] = __builtin_nontemporal_load(
						(const vec_t *) (a.col_al + (((uint64_t) tile * ROWS + b0 + r) * 256 + tid) * V));
#pragma unroll
				for (int r = 0; r < BATCH; r++) {
					uint32_t m = 0;
#pragma unroll
					for (int k = 0; k < V; k++)
						m |= (uint32_t) sel_eval<MODE>(a.pred, (T) x[r][k]) << k;
					hm[b0 + r] = m;
				}
			} else {
				ovec_t o[BATCH];
#pragma unroll
				for (int r = 0; r < BATCH; r++)
					o[r] = *(const ovec_t *) (a.cand_al + (((uint64_t) tile * ROWS + b0 + r) * 256 + tid) * 2);
				T v[BATCH * 2];
#pragma unroll
				for (int r = 0; r < BATCH; r++) {
					cv[(b0 + r) * 2] = o[r][0];
					cv[(b0 + r) * 2 + 1] = o[r][1];
					v[r * 2] = a.col[o[r][0] - a.hseq];
					v[r * 2 + 1] = a.col[o[r][1] - a.hseq];
				}
#pragma unroll
				for (int r = 0; r < BATCH; r++)
					hm[b0 + r] = (uint32_t) sel_eval<MODE>(a.pred, v[r * 2]) |
						     ((uint32_t) sel_eval<MODE>(a.pred, v[r * 2 + 1]) << 1);
			}
		}
	} else {
#pragma unroll
		for (int r = 0; r < ROWS; r++) {
			const uint64_t vi = ((uint64_t) tile * ROWS + r) * 256 + tid;
			const uint64_t j0 = vi * V;
			uint32_t m = 0;
			if (j0 < nslots) {
				if constexpr (!MAT) {
					vec_t x = *(const vec_t *) (a.col_al + j0);
#pragma unroll
					for (int k = 0; k < V; k++) {
						uint64_t j = j0 + k;
						bool ok = j >= a.shift && j < nslots && sel_eval<MODE>(a.pred, (T) x[k]);
						m |= (uint32_t) ok << k;
					}
				} else {
					ovec_t o = *(const ovec_t *) (a.cand_al + j0);
#pragma unroll
					for (int k = 0; k < 2; k++) {
						uint64_t j = j0 + k;
						cv[r * 2 + k] = o[k];
						if (j >= a.shift && j < nslots) {
							T v = a.col[o[k] - a.hseq];
							m |= (uint32_t) sel_eval<MODE>(a.pred, v) << k;
						}
					}
				}
			}
			hm[r] = m;
		}
	}
	// per (row, wave) totals
#pragma unroll
	for (int r = 0; r < ROWS; r++) {
		uint32_t ex, tot;
		wave_rank<BITS>((uint32_t) __popc(hm[r]), lt, ex, tot);
		if (lane == 0)
			s_off[r * 4 + wave] = tot;
	}
	__syncthreads();
	if (wave == 0) {
		// exclusive scan of the ROWS*4 (row, wave) segment counts, in
		// order; lane l owns entries [EPL*l, EPL*l + EPL)
		constexpr int EPL = (ROWS * 4 + 63) / 64;
		uint32_t e[EPL], own = 0;
#pragma unroll
		for (int q = 0; q < EPL; q++) {
			const int idx = (int) lane * EPL + q;
			e[q] = idx < ROWS * 4 ? s_off[idx] : 0u;
			own += e[q];
		}
		uint32_t x = own;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			uint32_t y = __shfl_up(x, o);
			if ((int) lane >= o)
				x += y;
		}
		uint32_t run = x - own;
#pragma unroll
		for (int q = 0; q < EPL; q++) {
			const int idx = (int) lane * EPL + q;
			if (idx < ROWS * 4)
				s_off[idx] = run;
			run += e[q];
		}
		uint64_t agg = __shfl(x, 63);
#if MGDK_SEL_EXP & 2
		uint64_t pre = 0;
#else
		uint64_t pre = lookback(a.status, tile, agg, (uint32_t *) &a.meta[1]);
#endif
		if (lane == 0) {
			s_prefix = pre;
			if (tile == a.ntiles - 1)
				a.meta[0] = pre + agg;
		}
	}
	__syncthreads();
	const uint64_t prefix = s_prefix;
#pragma unroll
	for (int r = 0; r < ROWS; r++) {
		uint32_t ex, tot;
		wave_rank<BITS>((uint32_t) __popc(hm[r]), lt, ex, tot);
		uint64_t pos = prefix + s_off[r * 4 + wave] + ex;
		uint32_t m = hm[r];
		const uint64_t j0 = (((uint64_t) tile * ROWS + r) * 256 + tid) * V;
		while (m) {
			int k = __ffs(m) - 1;
			m &= m - 1;
			oid o;
			if constexpr (MAT)
				o = cv[r * 2 + k];
			else
				o = a.cseq + (j0 + k - a.shift);
			a.out[pos++] = o;
		}
	}
}

// Dense-candidate scan in three launches, no look-back and no tickets:
//   k_sel_count  streams the column once: a tile = SROWS rows x 256 lanes x
//                16 B (64 KiB); the predicate bits go to a bitmap in slot
//                order (bit j = candidate slot j: 1 bit per value, n/8 bytes)
//                and the tile's hit count to counts[tile];
//   k_sel_scan   one workgroup: exclusive prefix of the tile counts;
//   k_sel_write  per tile: a workgroup scan of the bitmap words' popcounts
//                ranks every hit; sparse tiles store from the owning lane,
//                dense tiles go in rounds of 4096 slots whose hits are
//                placed in LDS in order and stored as one contiguous run.
// The column is read once; extra traffic is the bitmap twice (2 bits/value).
#ifndef MGDK_SEL_SROWS
#define MGDK_SEL_SROWS 16
#endif
constexpr int SROWS = MGDK_SEL_SROWS;
// results of at least this many oids keep the scan's bitmap (Priv::smap)
constexpr uint64_t SMAP_MIN = 1 << 20;
// rows of 16-B loads per lane: 1- and 2-byte types unpack 16 / 8 values per
// load, so fewer rows keep the count kernel's registers (and occupancy) in
// line with the 4- and 8-byte types (bte at 16 rows: 140 VGPRs, 0.8 TB/s)
template <typename T> constexpr int sel_srows() { return sizeof(T) >= 4 ? SROWS : sizeof(T) == 2 ? SROWS / 2 : SROWS / 4; }

template <typename T> constexpr int sel_v() { return (int) (16 / sizeof(T)); }
// bitmap words per tile and per lane of k_sel_write
template <typename T> constexpr int sel_wpt() { return sel_srows<T>() * 256 * sel_v<T>() / 32; }
template <typename T> constexpr int sel_wpl() { return sel_wpt<T>() >= 256 ? sel_wpt<T>() / 256 : 1; }

template <typename T, int MODE>
__global__ __launch_bounds__(256) void
k_sel_count(SelArgs<T> a, uint32_t *bits, uint32_t *counts)
{
	constexpr int V = sel_v<T>(), L = 32 / V;   // lanes per bitmap word
	constexpr int SR = sel_srows<T>();
	typedef T vec_t __attribute__((ext_vector_type(V)));
	const unsigned tid = threadIdx.x, lane = tid & 63;
	const uint32_t t = blockIdx.x;
	const uint64_t nslots = a.n + a.shift;
	const bool full = (t > 0 || a.shift == 0) && ((uint64_t) t + 1) * SR * 256 * V <= nslots;
	vec_t x[SR];
	if (full) {
#pragma unroll
		for (int r = 0; r < SR; r++)
			x[r] = __builtin_nontemporal_load((const vec_t *) (a.col_al + (((uint64_t) t * SR + r) * 256 + tid) * V));
	} else {
#pragma unroll
		for (int r = 0; r < SR; r++) {
			const uint64_t j0 = (((uint64_t) t * SR + r) * 256 + tid) * V;
			if (j0 < nslots)
				x[r] = *(const vec_t *) (a.col_al + j0);
		}
	}
	uint32_t cnt = 0;
#pragma unroll
	for (int r = 0; r < SR; r++) {
		const uint64_t j0 = (((uint64_t) t * SR + r) * 256 + tid) * V;
		uint32_t m = 0;
		if (full) {
#pragma unroll
			for (int k = 0; k < V; k++)
				m |= (uint32_t) sel_eval<MODE>(a.pred, (T) x[r][k]) << k;
		} else if (j0 < nslots) {
#pragma unroll
			for (int k = 0; k < V; k++) {
				const uint64_t j = j0 + k;
				const bool ok = j >= a.shift && j < nslots && sel_eval<MODE>(a.pred, (T) x[r][k]);
				m |= (uint32_t) ok << k;
			}
		}
		cnt += __popc(m);
		// gather the L lanes' V-bit pieces of one 32-bit word
		uint32_t wv = m << ((lane % L) * V);
#pragma unroll
		for (int o = 1; o < L; o <<= 1)
			wv |= __shfl_xor(wv, o);
		if (lane % L == 0)
			bits[j0 / 32] = wv;
	}
	cnt = block_reduce<uint32_t>(cnt, [](uint32_t p, uint32_t q) { return p + q; });
	if (tid == 0)
		counts[t] = cnt;
}

// k_sel_count over a candidate list that carries its select scan's bitmap
// (Priv::smap) in the same slot space (slot j = oid cseq + j, 16-B aligned in
// b): a value's predicate bit is ANDed with its candidate bit, and a lane
// whose V slots hold no candidate loads from the zero region instead, so a
// column line is fetched only when it holds a candidate.  The candidate
// oids themselves are never read.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void
k_sel_count_c(SelArgs<T> a, const uint32_t *cbits, const void *zero, uint32_t *bits, uint32_t *counts)
{
	constexpr int V = sel_v<T>(), L = 32 / V;
	constexpr int SR = sel_srows<T>();
	typedef T vec_t __attribute__((ext_vector_type(V)));
	const unsigned tid = threadIdx.x, lane = tid & 63;
	const uint32_t t = blockIdx.x;
	const uint64_t nslots = a.n;
	const uint32_t vmask = V == 32 ? ~0u : ((1u << V) - 1);
	const vec_t *z = (const vec_t *) zero + (((uint64_t) t * 256 + tid) & (ZERO_REGION / 16 - 1));
	uint32_t cw[SR];
#pragma unroll
	for (int r = 0; r < SR; r++) {
		const uint64_t j0 = (((uint64_t) t * SR + r) * 256 + tid) * V;
		cw[r] = cbits[(j0 < nslots ? j0 : 0) / 32];
	}
	vec_t x[SR];
	uint32_t cp[SR];
#pragma unroll
	for (int r = 0; r < SR; r++) {
		const uint64_t j0 = (((uint64_t) t * SR + r) * 256 + tid) * V;
		cp[r] = j0 < nslots ? (cw[r] >> (j0 % 32)) & vmask : 0u;
		x[r] = __builtin_nontemporal_load(cp[r] ? (const vec_t *) (a.col_al + j0) : z);
	}
	uint32_t cnt = 0;
#pragma unroll
	for (int r = 0; r < SR; r++) {
		const uint64_t j0 = (((uint64_t) t * SR + r) * 256 + tid) * V;
		uint32_t m = 0;
#pragma unroll
		for (int k = 0; k < V; k++)
			m |= (uint32_t) sel_eval<MODE>(a.pred, (T) x[r][k]) << k;
		m &= cp[r];
		cnt += __popc(m);
		uint32_t wv = m << ((lane % L) * V);
#pragma unroll
		for (int o = 1; o < L; o <<= 1)
			wv |= __shfl_xor(wv, o);
		if (lane % L == 0)
			bits[j0 / 32] = wv;             // zero past the last slot: the write pass reads whole tiles
	}
	cnt = block_reduce<uint32_t>(cnt, [](uint32_t p, uint32_t q) { return p + q; });
	if (tid == 0)
		counts[t] = cnt;
}

// exclusive prefix of counts[0..n) into pre[0..n), total into meta[0]; one
// workgroup walks the counts in chunks of 8192 (thread t loads and stores
// 8 consecutive counts: coalesced 32-B pieces, all loads of a chunk in
// flight), scans each chunk in LDS and carries the total to the next chunk.
// (A thread owning one long run serialised ~70 dependent loads and wrote
// its run with a stride: 0.13 ms for 73 K tiles.)
__global__ __launch_bounds__(1024) void
k_sel_scan(const uint32_t *counts, uint64_t *pre, uint32_t n, uint64_t *meta, uint64_t *hmeta)
{
	__shared__ uint64_t s_wave[16];
	__shared__ uint64_t s_carry;
	const unsigned tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	constexpr int E = 8;
	if (tid == 0)
		s_carry = 0;
	for (uint64_t c0 = 0; c0 < n; c0 += 1024 * E) {
		const uint64_t i0 = c0 + (uint64_t) tid * E;
		uint32_t v[E];
#pragma unroll
		for (int k = 0; k < E; k++)
			v[k] = i0 + k < n ? counts[i0 + k] : 0u;
		uint64_t own = 0;
#pragma unroll
		for (int k = 0; k < E; k++)
			own += v[k];
		uint64_t x = own;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint64_t y = __shfl_up(x, o);
			if ((int) lane >= o)
				x += y;
		}
		if (lane == 63)
			s_wave[wave] = x;
		__syncthreads();
		uint64_t run = s_carry + x - own, tot = 0;
		for (unsigned q = 0; q < 16; q++) {
			run += q < wave ? s_wave[q] : 0;
			tot += s_wave[q];
		}
#pragma unroll
		for (int k = 0; k < E; k++) {
			if (i0 + k < n)
				pre[i0 + k] = run;
			run += v[k];
		}
		__syncthreads();                      // s_wave / s_carry read by all
		if (tid == 0)
			s_carry += tot;
		__syncthreads();
	}
	if (tid == 0) {
		meta[0] = s_carry;
		meta[1] = 0;   // no look-back errors on this path
		if (hmeta) {
			hmeta[0] = s_carry;
			hmeta[1] = 0;
		}
	}
}

template <typename T>
__global__ __launch_bounds__(256) void
k_sel_write(SelArgs<T> a, const uint32_t *bits, const uint64_t *pre)
{
	constexpr int WPT = sel_wpt<T>(), WPL = sel_wpl<T>();
	// slots per dense round (a tile holds a whole number of rounds), SPL per lane
	constexpr int SCH = MGDK_SEL_SCH, SPL = SCH / 256;
	static_assert(SPL == 4 || SPL == 8 || SPL == 16, "4 to 16 slots per lane");
	static_assert((WPT * 32) % SCH == 0, "whole rounds per tile");
	__shared__ oid s_stage[SCH];
	__shared__ uint32_t s_words[WPT];
	__shared__ uint32_t s_wave[4];
	const unsigned tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	// a grid smaller than the tile count strides over the tiles (fewer,
	// longer workgroups for sparse results)
	for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
		__syncthreads();   // the previous tile's s_wave / s_stage / s_words are consumed
		const uint64_t slot0 = (uint64_t) t * WPT * 32;
		const bool active = tid * WPL < WPT;
		uint32_t w[WPL], cnt = 0;
#pragma unroll
		for (int q = 0; q < WPL; q++) {
			w[q] = active ? bits[(uint64_t) t * WPT + tid * WPL + q] : 0u;
			cnt += __popc(w[q]);
		}
		// workgroup exclusive scan of the per-lane counts
		uint32_t x = cnt;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t y = __shfl_up(x, o);
			if ((int) lane >= o)
				x += y;
		}
		if (lane == 63)
			s_wave[wave] = x;
		__syncthreads();
		uint32_t ex = x - cnt;
		for (unsigned q = 0; q < wave; q++)
			ex += s_wave[q];
		const uint32_t hits = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
		if (hits == 0)
			continue;
		const uint64_t prefix = pre[t];
		const oid base = a.cseq + slot0 - a.shift;
		// first / last oid of the whole result (virtualisation test on the host)
		if (cnt > 0 && (ex == 0 ? prefix == 0 : false)) {
			int q = 0;
			while (w[q] == 0)
				q++;
			a.meta[2] = base + ((uint64_t) (tid * WPL + q) * 32 + __ffs(w[q]) - 1);
			if (a.hmeta)
				a.hmeta[2] = a.meta[2];
		}
		if (cnt > 0 && ex + cnt == hits && prefix + hits == a.meta[0]) {
			int q = WPL - 1;
			while (w[q] == 0)
				q--;
			a.meta[3] = base + ((uint64_t) (tid * WPL + q) * 32 + 31 - __clz(w[q]));
			if (a.hmeta)
				a.hmeta[3] = a.meta[3];
		}
		if (hits < 1024) {
			// sparse: the owning lane stores its hits
			uint64_t pos = prefix + ex;
#pragma unroll
			for (int q = 0; q < WPL; q++) {
				uint32_t m = w[q];
				while (m) {
					const int b = __ffs(m) - 1;
					m &= m - 1;
					a.out[pos++] = base + ((uint64_t) (tid * WPL + q) * 32 + b);
				}
			}
			continue;
		}
		if (hits <= (uint32_t) SCH) {
			// all of the tile's hits fit the LDS stage: each lane places its
			// own, then one contiguous store
			uint32_t pos = ex;
#pragma unroll
			for (int q = 0; q < WPL; q++) {
				uint32_t m = w[q];
				while (m) {
					const int b = __ffs(m) - 1;
					m &= m - 1;
					s_stage[pos++] = base + ((uint64_t) (tid * WPL + q) * 32 + b);
				}
			}
			__syncthreads();
			for (uint32_t i = tid; i < hits; i += 256)
				a.out[prefix + i] = s_stage[i];
			continue;
		}
		// very dense: rounds of SCH slots, lane i taking the SPL slots
		// [SPL i, SPL i + SPL) of the round; the round's hits are ranked by a workgroup
		// scan, placed in LDS in order and stored as one run
#pragma unroll
		for (int q = 0; q < WPL; q++)
			if (active)
				s_words[tid * WPL + q] = w[q];
		uint64_t obase = prefix;
		for (int rd = 0; rd < WPT * 32 / SCH; rd++) {
			__syncthreads();   // s_words written / previous round's s_wave, s_stage consumed
			const uint32_t sl = (uint32_t) rd * SCH + tid * SPL;
			const uint32_t piece = (s_words[sl / 32] >> (sl % 32)) & ((1u << SPL) - 1);
			const uint32_t pc = __popc(piece);
			uint32_t y = pc;
#pragma unroll
			for (int o = 1; o < 64; o <<= 1) {
				const uint32_t z = __shfl_up(y, o);
				if ((int) lane >= o)
					y += z;
			}
			if (lane == 63)
				s_wave[wave] = y;
			__syncthreads();
			uint32_t pos = y - pc;
			for (unsigned q = 0; q < wave; q++)
				pos += s_wave[q];
			const uint32_t rhits = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
			uint32_t mm = piece;
			const oid rb = base + sl;
			while (mm) {
				const int bb = __ffs(mm) - 1;
				mm &= mm - 1;
				s_stage[pos++] = rb + bb;
			}
			__syncthreads();
			for (uint32_t i = tid; i < rhits; i += 256)
				a.out[obase + i] = s_stage[i];
			obase += rhits;
		}
	}
}

__global__ void
k_select_fin(const oid *out, uint64_t *meta)
{
	uint64_t n = meta[0];
	meta[2] = n ? out[0] : 0;
	meta[3] = n ? out[n - 1] : 0;
}

// workgroups of k_sel_write: MGDK_SEL_WGRID (0 = one per tile)
static unsigned
sel_wgrid(uint64_t ntiles)
{
	static const unsigned g = getenv("MGDK_SEL_WGRID") ? (unsigned) atoi(getenv("MGDK_SEL_WGRID")) : 0;
	return g && g < ntiles ? g : (unsigned) ntiles;
}

// ---- host-side normalisation -------------------------------------------------
template <typename T> struct Lim {
	static T minv() { return std::numeric_limits<T>::min() + 1; }   // GDK_T_min = nil + 1
	static T maxv() { return std::numeric_limits<T>::max(); }
	static T prev(T x) { return x - 1; }
	static T next(T x) { return x + 1; }
	static bool isnil(T x) { return x == std::numeric_limits<T>::min(); }
	static T nil() { return std::numeric_limits<T>::min(); }
};
template <> struct Lim<uint64_t> {   // oid: nil = 1<<63, GDK_oid_min = 0, max = 2^63-1
	static uint64_t minv() { return 0; }
	static uint64_t maxv() { return ((uint64_t) 1 << 63) - 1; }
	static uint64_t prev(uint64_t x) { return x - 1; }
	static uint64_t next(uint64_t x) { return x + 1; }
	static bool isnil(uint64_t x) { return x == ((uint64_t) 1 << 63); }
	static uint64_t nil() { return (uint64_t) 1 << 63; }
};
template <> struct Lim<hge> {
	static hge maxv() { return (hge) (((uhge) 1 << 127) - 1); }
	static hge minv() { return -maxv(); }
	static hge prev(hge x) { return x - 1; }
	static hge next(hge x) { return x + 1; }
	static bool isnil(hge x) { return x == (hge) ((uhge) 1 << 127); }
	static hge nil() { return (hge) ((uhge) 1 << 127); }
};
template <> struct Lim<float> {
	static float minv() { return -std::numeric_limits<float>::max(); }
	static float maxv() { return std::numeric_limits<float>::max(); }
	static float prev(float x) { return nextafterf(x, -std::numeric_limits<float>::max()); }
	static float next(float x) { return nextafterf(x, std::numeric_limits<float>::max()); }
	static bool isnil(float x) { return std::isnan(x); }
	static float nil() { return std::numeric_limits<float>::quiet_NaN(); }
};
template <> struct Lim<double> {
	static double minv() { return -std::numeric_limits<double>::max(); }
	static double maxv() { return std::numeric_limits<double>::max(); }
	static double prev(double x) { return nextafter(x, -std::numeric_limits<double>::max()); }
	static double next(double x) { return nextafter(x, std::numeric_limits<double>::max()); }
	static bool isnil(double x) { return std::isnan(x); }
	static double nil() { return std::numeric_limits<double>::quiet_NaN(); }
};

template <typename T>
static int
cmp3(T a, T b)
{
	// ATOMcmp: nil smallest and equal to itself
	bool an = Lim<T>::isnil(a), bn = Lim<T>::isnil(b);
	if (an || bn)
		return an && bn ? 0 : an ? -1 : 1;
	return (a > b) - (a < b);
}

// outcome of normalisation
struct Plan {
	enum { EMPTY, ALL, NOTNIL_ALL, SCAN } kind;
};

static mgdk_bat *
empty_result()
{
	return mgdk_BATdense(0, 0, 0);
}

template <typename T>
static mgdk_bat *run_scan_bits(const mgdk_bat *b, const Cand &ci, const SelPred<T> &pred, const SelMap &cm);

template <typename T>
static mgdk_bat *
run_scan(const mgdk_bat *b, const Cand &ci, const SelPred<T> &pred)
{
	// a candidate list that is a whole select result with its scan bitmap,
	// 16-B aligned against b in the same slot space: stream b through it
	// (only for dense enough lists: below the threshold the list's oids and a
	// gather move fewer bytes than streaming every slot of the bitmap)
	static const int min_pct = getenv("MGDK_SEL_BITS_PCT") ? atoi(getenv("MGDK_SEL_BITS_PCT")) : 50;
	SelMap cm;
	if (MGDK_SEL_STREAM && !ci.dense && ci.src && ci.n == ci.src->count && ci.n > 0 && smap_get(ci.src, &cm) &&
	    ci.n * 100 >= (uint64_t) min_pct * cm.nslots &&
	    cm.base >= (int64_t) b->hseqbase && cm.lo >= b->hseqbase && cm.hi < b->hseqbase + b->count &&
	    (((uintptr_t) b->theap + (uintptr_t) (cm.base - (int64_t) b->hseqbase) * sizeof(T)) & 15) == 0)
		return run_scan_bits<T>(b, ci, pred, cm);
	ProfScope prof("select");
	mgdk_bat *bn = newbat(0, MGDK_oid, ci.n);
	if (bn == nullptr)
		return nullptr;
	SelArgs<T> a{};
	a.col = (const T *) b->theap;
	a.hseq = b->hseqbase;
	a.n = ci.n;
	a.pred = pred;
	a.out = (oid *) bn->theap;
	uint64_t items_per_tile;
	if (ci.dense) {
		const T *start = a.col + (ci.seq - b->hseqbase);
		uintptr_t mis = ((uintptr_t) start % 16) / sizeof(T);
		a.col_al = start - mis;
		a.shift = (uint32_t) mis;
		a.cseq = ci.seq;
		items_per_tile = (uint64_t) (MGDK_SEL_STREAM ? sel_srows<T>() : sel_rows<false>()) * 256 * (16 / sizeof(T));
	} else {
		uintptr_t mis = ((uintptr_t) ci.oids % 16) / sizeof(oid);
		a.cand_al = ci.oids - mis;
		a.shift = (uint32_t) mis;
		items_per_tile = (uint64_t) sel_rows<true>() * 256 * 2;
	}
	uint64_t ntiles = (ci.n + a.shift + items_per_tile - 1) / items_per_tile;
	if (ntiles >= (1ull << 31)) {
		seterr("select: input too large");
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	a.ntiles = (uint32_t) ntiles;
	size_t sbytes = (ntiles + 8) * sizeof(uint64_t);
	char *sc = (char *) scratch(sbytes);
	uint64_t *meta = (uint64_t *) meta_buf();
	if (sc == nullptr || meta == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	a.ticket = (uint32_t *) sc;
	a.status = (uint64_t *) sc + 8;
	a.meta = meta;
	hipStream_t st = stream();
	const bool streamed = ci.dense && MGDK_SEL_STREAM;   // count / scan / write, no look-back
	uint64_t *h = (uint64_t *) pinned(64);
	if (h == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	a.hmeta = streamed && MGDK_SEL_HMETA ? h : nullptr;
	if (!streamed && (!hip_ok(hipMemsetAsync(sc, 0, sbytes, st), "hipMemsetAsync") ||
			  !hip_ok(hipMemsetAsync(meta, 0, 64, st), "hipMemsetAsync"))) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	// bitmap + counts + prefixes of the streamed scan: kept with the result
	// as its projection accelerator (Priv::smap) when it stays a list
	struct HeapRef {
		Heap *h;
		~HeapRef() { heap_decref(h); }
	} sbh{streamed ? heap_new(ntiles * (4 * (size_t) sel_wpt<T>() + 4 + 8) + 64) : nullptr};
	struct { void *p; } sb{sbh.h ? sbh.h->base : nullptr};
	uint32_t *smap_bits = nullptr;
	{
		const dim3 g((unsigned) ntiles), blk(256), gw(sel_wgrid(ntiles));
		uint32_t *bits = nullptr, *counts = nullptr;
		uint64_t *pre = nullptr;
		if (streamed) {
			if (sb.p == nullptr) {
				mgdk_BBPunfix(bn);
				return nullptr;
			}
			pre = (uint64_t *) sb.p;
			counts = (uint32_t *) (pre + ntiles);
			bits = counts + ntiles + (ntiles & 1);
			smap_bits = bits;
		}
#define SELS(MODE) do { hipLaunchKernelGGL((k_sel_count<T, MODE>), g, blk, 0, st, a, bits, counts); \
			hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, st, counts, pre, (uint32_t) ntiles, a.meta, a.hmeta); \
			hipLaunchKernelGGL(k_sel_write<T>, gw, blk, 0, st, a, bits, pre); } while (0)
#define SELL(MAT, MODE) do { if (!(MAT) && MGDK_SEL_STREAM) SELS(MODE); \
			     else hipLaunchKernelGGL((k_select<T, MAT, MODE>), g, blk, 0, st, a); } while (0)
#define SELM(MAT) switch (pred.mode) { \
		case SEL_RANGE: SELL(MAT, SEL_RANGE); break; \
		case SEL_ANTI: SELL(MAT, SEL_ANTI); break; \
		case SEL_EQ: SELL(MAT, SEL_EQ); break; \
		case SEL_EQNIL: SELL(MAT, SEL_EQNIL); break; \
		default: SELL(MAT, SEL_NOTNIL); break; }
		if (ci.dense) {
			SELM(false);
		} else {
			SELM(true);
		}
#undef SELM
#undef SELL
#undef SELS
	}
	if (!streamed)
		hipLaunchKernelGGL(k_select_fin, dim3(1), dim3(1), 0, st, (const oid *) bn->theap, meta);
	if ((a.hmeta == nullptr && !hip_ok(hipMemcpyAsync(h, meta, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, st), "memcpy")) ||
	    !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[1] & 1) {
		seterr("HY013!select: look-back did not complete");
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	uint64_t cnt = h[0];
	bn->count = cnt;
	bn->tsorted = bn->tkey = bn->tnonil = 1;
	bn->tnil = 0;
	bn->trevsorted = cnt <= 1;
	if (cnt <= 1 || h[3] - h[2] == cnt - 1) {
		setdense(bn, cnt ? h[2] : 0, cnt);   // virtualize
	} else if (streamed && cnt >= SMAP_MIN) {
		SelMap m{};
		m.pre = (const uint64_t *) sbh.h->base;
		m.bits = smap_bits;
		m.wpt = (uint32_t) sel_wpt<T>();
		m.ntiles = ntiles;
		m.nslots = ci.n + a.shift;
		m.base = (int64_t) (a.cseq - a.shift);
		m.lo = h[2];
		m.hi = h[3];
		smap_set(bn, sbh.h, m);
	}
	return bn;
}

template <typename T>
static mgdk_bat *
run_scan_bits(const mgdk_bat *b, const Cand &ci, const SelPred<T> &pred, const SelMap &cm)
{
	ProfScope prof("select");
	const uint64_t p0 = (uint64_t) (cm.base - (int64_t) b->hseqbase);      // b's position of slot 0
	const uint64_t nslots = std::min<uint64_t>(cm.nslots, b->count - p0);
	mgdk_bat *bn = newbat(0, MGDK_oid, ci.n);
	const void *zero = zero_region();
	if (bn == nullptr || zero == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	SelArgs<T> a{};
	a.col = (const T *) b->theap;
	a.hseq = b->hseqbase;
	a.col_al = a.col + p0;
	a.shift = 0;
	a.cseq = (oid) cm.base;
	a.n = nslots;
	a.pred = pred;
	a.out = (oid *) bn->theap;
	const uint64_t items_per_tile = (uint64_t) sel_srows<T>() * 256 * (16 / sizeof(T));
	const uint64_t ntiles = (nslots + items_per_tile - 1) / items_per_tile;
	if (ntiles >= (1ull << 31)) {
		seterr("select: input too large");
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	a.ntiles = (uint32_t) ntiles;
	uint64_t *meta = (uint64_t *) meta_buf();
	uint64_t *h = (uint64_t *) pinned(64);
	a.meta = meta;
	a.hmeta = MGDK_SEL_HMETA ? h : nullptr;
	struct HeapRef {
		Heap *h;
		~HeapRef() { heap_decref(h); }
	} sbh{heap_new(ntiles * (4 * (size_t) sel_wpt<T>() + 4 + 8) + 64)};
	if (sbh.h == nullptr || meta == nullptr || h == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	uint64_t *pre = (uint64_t *) sbh.h->base;
	uint32_t *counts = (uint32_t *) (pre + ntiles);
	uint32_t *bits = counts + ntiles + (ntiles & 1);
	hipStream_t st = stream();
	const dim3 g((unsigned) ntiles), blk(256), gw(sel_wgrid(ntiles));
#define SELC(MODE) do { hipLaunchKernelGGL((k_sel_count_c<T, MODE>), g, blk, 0, st, a, cm.bits, zero, bits, counts); \
			hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, st, counts, pre, (uint32_t) ntiles, a.meta, a.hmeta); \
			hipLaunchKernelGGL(k_sel_write<T>, gw, blk, 0, st, a, bits, pre); } while (0)
	switch (pred.mode) {
	case SEL_RANGE: SELC(SEL_RANGE); break;
	case SEL_ANTI: SELC(SEL_ANTI); break;
	case SEL_EQ: SELC(SEL_EQ); break;
	case SEL_EQNIL: SELC(SEL_EQNIL); break;
	default: SELC(SEL_NOTNIL); break;
	}
#undef SELC
	if ((a.hmeta == nullptr && !hip_ok(hipMemcpyAsync(h, meta, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, st), "memcpy")) ||
	    !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const uint64_t cnt = h[0];
	bn->count = cnt;
	bn->tsorted = bn->tkey = bn->tnonil = 1;
	bn->tnil = 0;
	bn->trevsorted = cnt <= 1;
	if (cnt <= 1 || h[3] - h[2] == cnt - 1) {
		setdense(bn, cnt ? h[2] : 0, cnt);   // virtualize
	} else if (cnt >= SMAP_MIN) {
		SelMap m{};
		m.pre = pre;
		m.bits = bits;
		m.wpt = (uint32_t) sel_wpt<T>();
		m.ntiles = ntiles;
		m.nslots = nslots;
		m.base = cm.base;
		m.lo = h[2];
		m.hi = h[3];
		smap_set(bn, sbh.h, m);
	}
	return bn;
}

// The body of BATselect after candidate setup, for value type T.
template <typename T>
static mgdk_bat *
select_typed(mgdk_bat *b, const Cand &ci, const T *tlp, const T *thp, bool li, bool hi,
	     bool anti, bool nil_matches)
{
	const T nil = Lim<T>::nil();
	T tl = *tlp, th = thp ? *thp : T{};
	bool th_null = thp == nullptr;
	bool lnil = cmp3(tl, nil) == 0;
	bool lval = !lnil || th_null;
	bool equi = th_null || (lval && cmp3(tl, th) == 0);
	bool hval;
	if (lnil && nil_matches && (th_null || cmp3(th, nil) == 0)) {
		equi = true;
		lval = true;
	}
	if (equi) {
		if (th_null)
			hi = li;
		th = tl;
		hval = true;
		if (!anti && (!li || !hi))
			return empty_result();
	} else {
		nil_matches = false;
		hval = cmp3(th, nil) != 0;
	}
	if (anti) {
		if (lval != hval) {
			bool ti = li;
			li = !hi;
			hi = !ti;
			T tv = tl;
			tl = th;
			th = tv;
			ti = lval;
			lval = hval;
			hval = ti;
			lnil = cmp3(tl, nil) == 0;
			anti = false;
		} else if (!lval && !hval) {
			return empty_result();
		} else if ((equi && (lnil || !(li && hi))) || cmp3(tl, th) > 0) {
			if (equi && !lnil && nil_matches && !(li && hi))
				return cand_slice(ci);
			SelPred<T> p{SEL_NOTNIL, false, tl, th};
			if (b->tnonil)
				return cand_slice(ci);
			return run_scan<T>(b, ci, p);
		} else {
			equi = false;   // anti-equi handled by the scan (gdk_select.c:1519)
		}
	}
	if (hval && (equi ? !li || !hi : cmp3(tl, th) > 0))
		return empty_result();
	if (equi && lnil && b->tnonil)
		return empty_result();
	if (!equi && !lval && !hval && lnil && b->tnonil)
		return cand_slice(ci);

	// scanfunc normalisation (gdk_select.c:300-446)
	T vl = tl, vh = th;
	if (anti && li) {
		if (vl == Lim<T>::minv()) {
			anti = false;
			vl = vh;
			li = !hi;
			hval = false;
		} else {
			vl = Lim<T>::prev(vl);
			li = false;
		}
	}
	if (anti && hi) {
		if (vh == Lim<T>::maxv()) {
			anti = false;
			vh = vl;
			hi = !li;
			lval = false;
		} else {
			vh = Lim<T>::next(vh);
			hi = false;
		}
	}
	if (!anti) {
		if (lval) {
			if (!li) {
				if (vl == Lim<T>::maxv())
					return empty_result();
				vl = Lim<T>::next(vl);
				li = true;
			}
		} else {
			vl = Lim<T>::minv();
			li = true;
			lval = true;
		}
		if (hval) {
			if (!hi) {
				if (vh == Lim<T>::minv())
					return empty_result();
				vh = Lim<T>::prev(vh);
				hi = true;
			}
		} else {
			vh = Lim<T>::maxv();
			hi = true;
			hval = true;
		}
		if (vl > vh)
			return empty_result();
	}
	SelPred<T> p;
	p.vl = vl;
	p.vh = vh;
	p.nil_matches = nil_matches;
	if (equi)
		p.mode = lnil ? SEL_EQNIL : SEL_EQ;
	else if (anti)
		p.mode = SEL_ANTI;
	else
		p.mode = SEL_RANGE;
	return run_scan<T>(b, ci, p);
}

// void (dense oid) column: positional select, values are tseqbase + p
static mgdk_bat *
select_void(mgdk_bat *b, const Cand &ci, const oid *tl, const oid *th, bool li, bool hi,
	    bool anti, bool nil_matches)
{
	// materialise the dense values once, then use the generic path
	mgdk_bat *tmp = newbat(b->hseqbase, MGDK_oid, b->count);
	if (tmp == nullptr)
		return nullptr;
	std::vector<oid> h(b->count);
	for (BUN i = 0; i < b->count; i++)
		h[i] = b->tseqbase == MGDK_OID_NIL ? MGDK_OID_NIL : b->tseqbase + i;
	if (mgdk_BATupload(tmp, h.data(), b->count) < 0) {
		mgdk_BBPunfix(tmp);
		return nullptr;
	}
	tmp->tnonil = b->tseqbase != MGDK_OID_NIL;
	mgdk_bat *r = select_typed<uint64_t>(tmp, ci, tl, th, li, hi, anti, nil_matches);
	mgdk_BBPunfix(tmp);
	return r;
}

}  // namespace

namespace mgdk {
// Ordered compaction of a 0/1 byte array: the sorted list of positions i
// (as oids base + i) with flags[i] == 1.  Used by BATgroup / BATjoin.
mgdk_bat *
compact_flags(const int8_t *flags, BUN n, oid base, bool nonzero)
{
	if (n == 0)
		return empty_result();
	mgdk_bat tmp{};
	tmp.ttype = MGDK_bte;
	tmp.twidth = 1;
	tmp.count = n;
	tmp.hseqbase = base;
	tmp.theap = (void *) flags;
	Cand ci{};
	ci.dense = true;
	ci.seq = base;
	ci.n = n;
	ci.first = base;
	ci.last = base + n - 1;
	SelPred<int8_t> p{SEL_EQ, false, 1, 1};
	if (nonzero) {
		// bit columns: any non-zero byte (true or nil) counts, like `if (np[i])`
		p.mode = SEL_ANTI;
		p.nil_matches = true;
		p.vl = -1;
		p.vh = 1;
	}
	return run_scan<int8_t>(&tmp, ci, p);
}
}  // namespace mgdk

namespace {

// ---- str columns: BATselect's generic part with strCmp, then the
// fullscan_any predicate (gdk/gdk_select.c:449-605) per candidate.
// fullscan_str's string-elimination path (:608-760) compares heap offsets
// instead of bytes when doubles are eliminated -- the same oids.

constexpr char SEL_STR_NIL[2] = {'\x80', 0};

__device__ __forceinline__ const uint8_t *
sel_str_at(const void *offs, int w, const char *vh, BUN p)
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

__device__ __forceinline__ bool
dstr_isnil(const uint8_t *a)
{
	return a[0] == 0x80 && a[1] == 0;
}

// strCmp (gdk_atoms.c): nil before every string, then strcmp's unsigned bytes
__device__ __forceinline__ int
dstr_cmp(const uint8_t *a, const uint8_t *b)
{
	const bool an = dstr_isnil(a), bn = dstr_isnil(b);
	if (an || bn)
		return an ? -(int) !bn : 1;
	for (;; a++, b++) {
		const int x = *a, y = *b;
		if (x != y)
			return x < y ? -1 : 1;
		if (x == 0)
			return 0;
	}
}

struct StrSel {
	const void *offs;
	int w;
	const char *vh;
	oid hseq;
	const uint8_t *tl, *th;     // device copies
	bool li, hi, equi, anti, nil_matches, lval, hval, all_but_nil;
};

// flags over rows [first, first + m): 1 where a candidate row qualifies
__global__ __launch_bounds__(256) void
k_sel_str(StrSel a, bool dense, oid cseq, const oid *coids, BUN ncand, oid first, int8_t *flags)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < ncand; i += (BUN) gridDim.x * blockDim.x) {
		const oid o = dense ? cseq + i : coids[i];
		const uint8_t *v = sel_str_at(a.offs, a.w, a.vh, o - a.hseq);
		const bool isnil = dstr_isnil(v);
		bool ok;
		int c;
		if (a.all_but_nil)
			ok = !isnil;
		else if (a.equi)
			ok = dstr_cmp(a.tl, v) == 0;
		else if (a.anti)
			ok = (a.nil_matches && isnil) ||
			     (!isnil && ((a.lval && ((c = dstr_cmp(a.tl, v)) > 0 || (!a.li && c == 0))) ||
					 (a.hval && ((c = dstr_cmp(a.th, v)) < 0 || (!a.hi && c == 0)))));
		else
			ok = !isnil && (!a.lval || (c = dstr_cmp(a.tl, v)) < 0 || (a.li && c == 0)) &&
			     (!a.hval || (c = dstr_cmp(a.th, v)) > 0 || (a.hi && c == 0));
		flags[o - first] = ok;
	}
}

int
host_str_cmp(const char *a, const char *b)
{
	const bool an = (unsigned char) a[0] == 0x80 && a[1] == 0, bn = (unsigned char) b[0] == 0x80 && b[1] == 0;
	if (an || bn)
		return an ? -(int) !bn : 1;
	const int c = strcmp(a, b);
	return (c > 0) - (c < 0);
}

mgdk_bat *
select_str(mgdk_bat *b, const Cand &ci, const char *tl, const char *th, bool li, bool hi, bool anti,
	   bool nil_matches)
{
	if (b->tvheap == nullptr) {
		seterr("42000!BATselect: str column without a string heap");
		return nullptr;
	}
	const char *nil = SEL_STR_NIL;
	bool lnil = host_str_cmp(tl, nil) == 0;
	bool lval = !lnil || th == nullptr;
	bool equi = th == nullptr || (lval && host_str_cmp(tl, th) == 0);
	bool hval;
	if (lnil && nil_matches && (th == nullptr || host_str_cmp(th, nil) == 0)) {
		equi = true;
		lval = true;
	}
	if (equi) {
		if (th == nullptr)
			hi = li;
		th = tl;
		hval = true;
		if (!anti && (!li || !hi))
			return empty_result();
	} else {
		nil_matches = false;
		hval = host_str_cmp(th, nil) != 0;
	}
	bool all_but_nil = false;
	if (anti) {
		if (lval != hval) {
			const char *tv = tl;
			bool ti = li;
			li = !hi;
			hi = !ti;
			tl = th;
			th = tv;
			ti = lval;
			lval = hval;
			hval = ti;
			lnil = host_str_cmp(tl, nil) == 0;
			anti = false;
		} else if (!lval && !hval) {
			return empty_result();
		} else if ((equi && (lnil || !(li && hi))) || host_str_cmp(tl, th) > 0) {
			// everything except nil (:1482-1509)
			if (equi && !lnil && nil_matches && !(li && hi))
				return cand_slice(ci);
			if (b->tnonil)
				return cand_slice(ci);
			all_but_nil = true;
		} else {
			equi = false;
		}
	}
	if (!all_but_nil && hval && (equi ? !li || !hi : host_str_cmp(tl, th) > 0))
		return empty_result();
	if (equi && lnil && b->tnonil)
		return empty_result();
	const size_t ll = strlen(tl) + 1, hl = strlen(th) + 1;
	const BUN m = ci.last - ci.first + 1;
	DevBuf vals(ll + hl + 16), flags(m + 8);
	hipStream_t st = stream();
	if (!vals.p || !flags.p || !hip_ok(hipMemsetAsync(flags.p, 0, m, st), "memset"))
		return nullptr;
	// each bound's copy is queued right after it is staged: a second
	// stage_host may wrap the arena (sync + reuse from offset 0)
	if (!hip_ok(hipMemcpyAsync(vals.p, stage_host(tl, ll), ll, hipMemcpyHostToDevice, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync((char *) vals.p + ll, stage_host(th, hl), hl, hipMemcpyHostToDevice, st), "memcpy"))
		return nullptr;
	StrSel a{};
	a.offs = b->theap;
	a.w = b->twidth;
	a.vh = (const char *) b->tvheap;
	a.hseq = b->hseqbase;
	a.tl = (const uint8_t *) vals.p;
	a.th = (const uint8_t *) vals.p + ll;
	a.li = li;
	a.hi = hi;
	a.equi = equi;
	a.anti = anti;
	a.nil_matches = nil_matches;
	a.lval = lval;
	a.hval = hval;
	a.all_but_nil = all_but_nil;
	hipLaunchKernelGGL(k_sel_str, dim3(grid_for(ci.n, 1024, 16384)), dim3(256), 0, st, a, ci.dense, ci.seq, ci.oids,
			   ci.n, ci.first, flags.as<int8_t>());
	return compact_flags(flags.as<int8_t>(), m, ci.first);
}

}  // namespace

extern "C" {

mgdk_bat *
mgdk_BATselect(mgdk_bat *b, mgdk_bat *s, const void *tl, const void *th, bool li, bool hi,
	       bool anti, bool nil_matches)
{
	if (b == nullptr) {
		seterr("BATselect: b must exist");
		return nullptr;
	}
	if (tl == nullptr) {
		seterr("tl value required");
		return nullptr;
	}
	if (s && s->ttype != MGDK_msk && !s->tsorted) {
		seterr("invalid argument: s must be sorted.\n");
		return nullptr;
	}
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return nullptr;
	if (ci.n == 0)
		return empty_result();
	switch (basetype(b->ttype)) {
	case MGDK_void:
		return select_void(b, ci, (const oid *) tl, (const oid *) th, li, hi, anti, nil_matches);
	case MGDK_bte:
		return select_typed<int8_t>(b, ci, (const int8_t *) tl, (const int8_t *) th, li, hi, anti, nil_matches);
	case MGDK_sht:
		return select_typed<int16_t>(b, ci, (const int16_t *) tl, (const int16_t *) th, li, hi, anti, nil_matches);
	case MGDK_int:
		return select_typed<int32_t>(b, ci, (const int32_t *) tl, (const int32_t *) th, li, hi, anti, nil_matches);
	case MGDK_lng:
		return select_typed<int64_t>(b, ci, (const int64_t *) tl, (const int64_t *) th, li, hi, anti, nil_matches);
	case MGDK_oid:
		return select_typed<uint64_t>(b, ci, (const uint64_t *) tl, (const uint64_t *) th, li, hi, anti, nil_matches);
	case MGDK_hge:
		return select_typed<hge>(b, ci, (const hge *) tl, (const hge *) th, li, hi, anti, nil_matches);
	case MGDK_flt:
		return select_typed<float>(b, ci, (const float *) tl, (const float *) th, li, hi, anti, nil_matches);
	case MGDK_dbl:
		return select_typed<double>(b, ci, (const double *) tl, (const double *) th, li, hi, anti, nil_matches);
	case MGDK_str:
		return select_str(b, ci, (const char *) tl, (const char *) th, li, hi, anti, nil_matches);
	default:
		seterr("42000!BATselect: type %s not supported on the device path", atomname(b->ttype));
		return nullptr;
	}
}

// BATthetaselect (gdk/gdk_select.c:2103-2154)
mgdk_bat *
mgdk_BATthetaselect(mgdk_bat *b, mgdk_bat *s, const void *val, const char *op)
{
	if (b == nullptr || val == nullptr || op == nullptr) {
		seterr("BATthetaselect: NULL argument");
		return nullptr;
	}
	if (strcmp(op, "eq") == 0)
		return mgdk_BATselect(b, s, val, nullptr, true, true, false, true);
	if (strcmp(op, "ne") == 0)
		return mgdk_BATselect(b, s, val, nullptr, true, true, true, true);
	alignas(16) unsigned char nilv[16];
	bool isnil = false;
	switch (basetype(b->ttype)) {
	case MGDK_str:
		nilv[0] = 0x80;
		nilv[1] = 0;
		isnil = ((const unsigned char *) val)[0] == 0x80 && ((const unsigned char *) val)[1] == 0;
		break;
	case MGDK_bte: *(int8_t *) nilv = INT8_MIN; isnil = *(const int8_t *) val == INT8_MIN; break;
	case MGDK_sht: *(int16_t *) nilv = INT16_MIN; isnil = *(const int16_t *) val == INT16_MIN; break;
	case MGDK_int: *(int32_t *) nilv = INT32_MIN; isnil = *(const int32_t *) val == INT32_MIN; break;
	case MGDK_lng: *(int64_t *) nilv = INT64_MIN; isnil = *(const int64_t *) val == INT64_MIN; break;
	case MGDK_void:
	case MGDK_oid: *(uint64_t *) nilv = MGDK_OID_NIL; isnil = *(const uint64_t *) val == MGDK_OID_NIL; break;
	case MGDK_hge: {
		hge n = (hge) ((uhge) 1 << 127);
		memcpy(nilv, &n, 16);
		isnil = memcmp(val, &n, 16) == 0;
		break;
	}
	case MGDK_flt: *(float *) nilv = std::numeric_limits<float>::quiet_NaN(); isnil = std::isnan(*(const float *) val); break;
	case MGDK_dbl: *(double *) nilv = std::numeric_limits<double>::quiet_NaN(); isnil = std::isnan(*(const double *) val); break;
	default:
		seterr("42000!BATthetaselect: type %s not supported on the device path", atomname(b->ttype));
		return nullptr;
	}
	if (isnil)
		return empty_result();
	if (op[0] == '=' && ((op[1] == '=' && op[2] == 0) || op[1] == 0))
		return mgdk_BATselect(b, s, val, nullptr, true, true, false, false);
	if (op[0] == '!' && op[1] == '=' && op[2] == 0)
		return mgdk_BATselect(b, s, val, nullptr, true, true, true, false);
	if (op[0] == '<') {
		if (op[1] == 0)
			return mgdk_BATselect(b, s, nilv, val, false, false, false, false);
		if (op[1] == '=' && op[2] == 0)
			return mgdk_BATselect(b, s, nilv, val, false, true, false, false);
		if (op[1] == '>' && op[2] == 0)
			return mgdk_BATselect(b, s, val, nullptr, true, true, true, false);
	}
	if (op[0] == '>') {
		if (op[1] == 0)
			return mgdk_BATselect(b, s, val, nilv, false, false, false, false);
		if (op[1] == '=' && op[2] == 0)
			return mgdk_BATselect(b, s, val, nilv, true, false, false, false);
	}
	seterr("unknown operator.\n");
	return nullptr;
}

}  // extern "C"
