// sort.hip -- BATsort on the MI355X (gdk/gdk_batop.c:2342, do_sort :2266-2304).
//
// For integer keys with nilslast == reverse the reference sorts with the
// stable LSD radix sort GDKrsort (gdk/gdk_rsort.c:21); stable float sorts use
// the stable merge sort.  Both produce THE stable permutation, which is what
// this stable LSD radix sort reproduces:
//   key image: order-preserving unsigned key (sign bit flipped; IEEE floats
//   folded; -0 == +0; nil placed first or last as requested; inverted for
//   descending so ties keep input order); 32-bit keys for types up to 4
//   bytes (when nilslast == reverse, so nil keeps its natural image), 64-bit
//   otherwise;
//   passes: 8-bit digits, only digit positions that are not constant over
//   the input (AND/OR reduction) are sorted;
//   the global digit counts of every pass come from ONE pass over the input
//   (LSD passes permute the keys, the counts do not change);
//   per pass: a stable scatter of an 8192-key tile whose output base per
//   digit is the pass's digit start + a decoupled look-back over the
//   tiles' digit counts (each tile publishes its counts before ranking, so
//   the walk back is short; MGDK_SORT_LB=0 restores the per-pass histogram
//   + scan); in the tile each wave
//   ranks its 32 rows of 64 keys against per-wave running digit counters
//   (no workgroup barrier per row), a row's same-digit lanes found through
//   a per-wave LDS lane mask per digit (one OR, one read, one clear;
//   MGDK_SORT_LDSMATCH=0 restores 8 bit-sliced ballots), the tile is
//   reordered by digit in LDS and written out in that order, so equal-digit
//   runs leave as contiguous stores;
//   the LAST pass writes the result columns directly: integer values decoded
//   from the key image (no gather) and the order oids (hseqbase + position).
#include <type_traits>
#include <vector>

#include "lookback.h"
#include "mgdk_internal.h"

// the MSD-then-local form for 4-byte keys of >= 2^22 rows (one look-back
// scatter pass fewer): 7 % slower than the four LSD passes on round 5's
// boxes (2.79 ms), 8 % faster on round 6's, whose scatter passes run at
// 735-906 us instead of 512-586
#ifndef SORT_HYBRID_DEFAULT
#define SORT_HYBRID_DEFAULT 1
#endif

using namespace mgdk;

namespace {

// 4-byte keys: 8 waves x 16 rows (122 VGPRs, 4 waves per SIMD) measured
// 2.80-2.84 ms for 100M int32 against 3.05-3.07 for 4 x 32 (243 VGPRs, 2
// waves per SIMD) on the same boxes with the per-thread look-back
// (profiles/r05/sort); in round 3, with the walk waiting on residency, it
// was the other way round
#ifndef MGDK_SORT_WAVES
#define MGDK_SORT_WAVES 8
#endif
#ifndef MGDK_SORT_ROWS
#define MGDK_SORT_ROWS 16
#endif
#ifndef MGDK_SORT_WAVES8
#define MGDK_SORT_WAVES8 4
#endif
#ifndef MGDK_SORT_ROWS8
#define MGDK_SORT_ROWS8 32
#endif
// scatter tile shape per key width: waves per workgroup x rows of 64 keys
// per wave (the tile's keys and values are staged in LDS)
template <typename K>
struct Tile {
	static constexpr int W = sizeof(K) == 4 ? MGDK_SORT_WAVES : MGDK_SORT_WAVES8;
	static constexpr int R = sizeof(K) == 4 ? MGDK_SORT_ROWS : MGDK_SORT_ROWS8;
	static constexpr int THREADS = 64 * W;
	static constexpr int N = THREADS * R;
	static_assert(W >= 4 && N % 256 == 0, "the digit steps need 256 threads");
};
// 1: a row's peer lanes (same digit) come from a per-wave LDS lane mask per
// digit (one OR, one read, one clear) instead of 8 bit-sliced ballots
#ifndef MGDK_SORT_LOCAL_NOPASS
#define MGDK_SORT_LOCAL_NOPASS 0     // diagnostic builds only: pass C without its LDS passes
#endif
#ifndef MGDK_SORT_LDSMATCH
#define MGDK_SORT_LDSMATCH 1
#endif

template <typename K>
__global__ __launch_bounds__(256) void
k_rs_hist(const K *keys, BUN n, int shift, uint32_t *hist, uint32_t nblocks)
{
	__shared__ uint32_t h[256];
	h[threadIdx.x] = 0;
	__syncthreads();
	const BUN base = (BUN) blockIdx.x * Tile<K>::N;
	constexpr int HR = Tile<K>::N / 256;
	K k[HR];
#pragma unroll
	for (int r = 0; r < HR; r++) {
		const BUN i = base + r * 256 + threadIdx.x;
		k[r] = i < n ? keys[i] : 0;
	}
#pragma unroll
	for (int r = 0; r < HR; r++) {
		const BUN i = base + r * 256 + threadIdx.x;
		if (i < n)
			atomicAdd(&h[(uint32_t) (k[r] >> shift) & 255], 1u);
	}
	__syncthreads();
	hist[(BUN) threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// digit histograms of every pass at once: LSD passes permute the keys, so
// each pass's global digit counts are those of the input (one read)
constexpr int RS_MAXP = 8;
#ifndef MGDK_SORT_GIDV
#define MGDK_SORT_GIDV 1        // group-start count pass with 16-B loads (0: 4-B loads at a 256-row stride)
#endif
#ifndef MGDK_SORT_LBW
#define MGDK_SORT_LBW 8         // predecessors read per step of the scatter's look-back walk (1: one at a time)
#endif
#ifndef MGDK_SORT_NTLOAD
#define MGDK_SORT_NTLOAD 1      // nontemporal key / value loads in the scatter passes (0: plain; 2.84 vs 2.74 ms)
#endif
struct Shifts {
	int s[RS_MAXP];
	int n;
};

template <typename K>
__global__ __launch_bounds__(256) void
k_rs_dhist(const K *keys, BUN n, Shifts sh, uint32_t *out)
{
	__shared__ uint32_t h[RS_MAXP][256];
	for (int p = 0; p < sh.n; p++)
		h[p][threadIdx.x] = 0;
	__syncthreads();
	// 8 keys per thread per step, all loaded before the first is counted
	constexpr int KU = 8;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i0 = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += KU * stride) {
		K k[KU];
#pragma unroll
		for (int u = 0; u < KU; u++) {
			const BUN i = i0 + u * stride;
			k[u] = keys[i < n ? i : n - 1];
		}
#pragma unroll
		for (int u = 0; u < KU; u++)
			if (i0 + u * stride < n)
				for (int p = 0; p < sh.n; p++)
					atomicAdd(&h[p][(uint32_t) (k[u] >> sh.s[p]) & 255], 1u);
	}
	__syncthreads();
	for (int p = 0; p < sh.n; p++)
		if (h[p][threadIdx.x])
			atomicAdd(&out[(sh.s[p] / 8) * 256 + threadIdx.x], h[p][threadIdx.x]);
}

// exclusive scan of each pass's 256 digit counts (one workgroup per pass)
__global__ __launch_bounds__(256) void
k_rs_dscan(const uint32_t *cnt, Shifts sh, uint32_t *gdig)
{
	__shared__ uint32_t ws[4];
	const uint32_t v = cnt[(sh.s[blockIdx.x] / 8) * 256 + threadIdx.x];
	const unsigned lane = __lane_id(), w = threadIdx.x >> 6;
	uint32_t x = v;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t u = __shfl_up(x, o);
		if (lane >= (unsigned) o)
			x += u;
	}
	if (lane == 63)
		ws[w] = x;
	__syncthreads();
	for (unsigned q = 0; q < w; q++)
		x += ws[q];
	gdig[blockIdx.x * 256 + threadIdx.x] = x - v;
}

// the tiles of a pass that sorts inside the buckets of the previous (MSD)
// pass: desc[t] = {first row, rows, first tile of the bucket, tiles of the
// bucket}; the counts / offsets of tile t live at 256 * first + d * tiles +
// (t - first), so one exclusive scan gives every (bucket, digit) its start
struct SegTiles {
	const uint4 *desc;
	const uint32_t *count;      // number of tiles
};

// final pass outputs: decoded value column and order oids
struct FinalOut {
	void *sorted;       // NULL: not requested (or gathered separately)
	void *keys;         // sorted key images (for groups), NULL: not requested
	bool want_keys;
	int vw;             // value width in bytes (1, 2, 4, 8)
	bool reverse;
	bool is64;          // 64-bit key image of a signed/unsigned integer
	bool uns;           // oid
	oid *order;
	oid hseq;
	oid *gid;           // hybrid pass C: group ids written with the rows (NULL: not)
	bool *gid_done;     // set when it did
	uint64_t *gid_last; // ... and the last row's group id
};

template <typename K>
__device__ __forceinline__ void
emit_final(const FinalOut &fo, BUN g, K key, uint32_t v)
{
	if (fo.order)
		fo.order[g] = fo.hseq + v;
	if (fo.keys)
		((K *) fo.keys)[g] = key;
	if (fo.sorted) {
		uint64_t u = (uint64_t) key;
		if (fo.reverse)
			u = ~u;
		if (sizeof(K) == 4) {
			const int32_t x = (int32_t) ((uint32_t) u ^ 0x80000000u);
			switch (fo.vw) {
			case 1: ((int8_t *) fo.sorted)[g] = (int8_t) x; break;
			case 2: ((int16_t *) fo.sorted)[g] = (int16_t) x; break;
			default: ((int32_t *) fo.sorted)[g] = x; break;
			}
		} else {
			((uint64_t *) fo.sorted)[g] = fo.uns ? u : (u ^ (1ull << 63));
		}
	}
}

// LB: the tile's output base per digit comes from a decoupled look-back
// over the tiles' digit counts (tiles numbered by a ticket, so every
// predecessor is resident) plus the pass's global digit start gdig -- no
// per-pass histogram pass and scan.  Otherwise offs holds the digit-major
// exclusive scan of k_rs_hist's counts.
// XCD-grouped tile order (xg > 0): the tiles are dealt to the XCDs in
// groups of xg consecutive tiles, each XCD claiming its own tiles in order
// (a per-XCD ticket; an XCD whose tiles are all claimed takes the next ones
// of another XCD), so neighbouring tiles -- whose runs of a digit are
// adjacent in the output -- complete their shared lines in one L2.  A
// tile's predecessor may then be unclaimed while the tile waits on it, and
// whether it is ever claimed depends on what the dispatcher can place, so
// the look-back counts an unclaimed predecessor's digits itself instead of
// waiting for it (k_rs_scatter): no residency assumption, any group size is
// safe.
__device__ __forceinline__ uint32_t
claim_tile(uint32_t *xtk, uint32_t ntiles, uint32_t xg)
{
	const uint32_t x = (uint32_t) __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;   // HW_REG_XCC_ID
	for (uint32_t k = 0; k < 8; k++) {
		const uint32_t y = (x + k) & 7;
		const uint32_t j = atomicAdd(&xtk[y], 1u);
		const uint32_t t = (j / xg) * 8 * xg + y * xg + j % xg;
		if (t < ntiles)
			return t;
	}
	return ~0u;
}

template <typename K, bool FINAL, bool IDV, bool LB, bool SEG>
__global__ __launch_bounds__(Tile<K>::THREADS) void
k_rs_scatter(const K *keys, const uint32_t *vals, BUN n, int shift, const uint32_t *offs, uint32_t nblocks,
	     K *kout, uint32_t *vout, FinalOut fo, uint32_t *ticket, uint64_t *status, const uint32_t *gdig,
	     uint32_t *err, SegTiles sg, uint32_t xg, uint64_t *znext, K kx)
{
	constexpr int SWAVES = Tile<K>::W, SROWS = Tile<K>::R, STHREADS = Tile<K>::THREADS, STILE = Tile<K>::N;
	__shared__ K sk[STILE];
	__shared__ __attribute__((aligned(16))) uint32_t sv[STILE];
	__shared__ uint32_t wcnt[SWAVES][256]; // per-wave running digit counts, then per-wave bases
	__shared__ uint32_t tstart[256];      // digit start inside the reordered tile
	__shared__ uint32_t gbase[256];       // digit start of this tile in the output
	__shared__ uint32_t s_wt[4];
	__shared__ uint32_t s_tile;
	// threads 0..255 (waves 0-3) own one digit each in the per-digit steps
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const bool dig = tid < 256;
	if (LB || (SEG && xg)) {
		if (tid == 0)
			s_tile = xg ? claim_tile(ticket + 8, SEG ? *sg.count : nblocks, xg) : atomicAdd(ticket, 1u);
		__syncthreads();
	}
	const uint32_t blk = LB || (SEG && xg) ? s_tile : blockIdx.x;
	// SEG: the tile is a piece of one bucket of the previous (MSD) pass
	uint4 sd = {0, 0, 0, 0};
	if (SEG) {
		if (blk >= *sg.count)
			return;
		sd = sg.desc[blk];
	}
	if (LB && blk == ~0u)
		return;     // cannot happen: one tile per workgroup
	// the next LSD pass's look-back status of this tile, zeroed here (the
	// passes alternate between two status arrays: no memset between them)
	if (LB && znext != nullptr && dig)
		znext[(size_t) blk * 256 + tid] = 0ull;
	const BUN tbase = SEG ? (BUN) sd.x : (BUN) blk * STILE;
	const BUN tend = SEG ? tbase + sd.y : n;
	__shared__ uint32_t lh[256];          // LB: the tile's digit counts, published before ranking
	if (LB && dig)
		lh[tid] = 0;
	for (unsigned q = tid; q < SWAVES * 256; q += STHREADS)
		(&wcnt[0][0])[q] = 0;
	if (!LB && dig)
		gbase[tid] = SEG ? offs[(BUN) 256 * sd.z + (BUN) tid * sd.w + (blk - sd.z)] : offs[(BUN) tid * nblocks + blk];
	const BUN base = tbase + (BUN) w * (64 * SROWS);
#if MGDK_SORT_LDSMATCH
	// the wave's 256 digit lane masks live in sv until the tile is placed
	static_assert(SWAVES * 256 * 2 <= STILE, "lane masks fit in sv");
	unsigned long long *wm = (unsigned long long *) sv + (size_t) w * 256;
#pragma unroll
	for (int q = 0; q < 4; q++)
		wm[lane + 64 * q] = 0ull;
#endif
	K k[SROWS];
	uint32_t v[SROWS];
#pragma unroll
	for (int r = 0; r < SROWS; r++) {
		const BUN i = base + r * 64 + lane;
#if MGDK_SORT_NTLOAD
		k[r] = i < tend ? __builtin_nontemporal_load(keys + i) ^ kx : 0;
		v[r] = IDV ? (uint32_t) i : (i < tend ? __builtin_nontemporal_load(vals + i) : 0);
#else
		k[r] = i < tend ? keys[i] ^ kx : 0;
		v[r] = IDV ? (uint32_t) i : (i < tend ? vals[i] : 0);   // first pass: positions
#endif
	}
	__syncthreads();
	if (LB) {
		// publish this tile's digit counts as early as possible, so the
		// look-back of later tiles rarely has to walk far
#pragma unroll
		for (int r = 0; r < SROWS; r++)
			if (base + r * 64 + lane < tend)
				atomicAdd(&lh[(uint32_t) (k[r] >> shift) & 255], 1u);
		__syncthreads();
		if (dig)
			mgdk_lb::lb_store(status + (size_t) blk * 256 + tid,
					  (blk == 0 ? mgdk_lb::ST_PRE : mgdk_lb::ST_AGG) | lh[tid]);
	}
	const uint64_t lt = lanemask_lt();
	uint32_t rk[SROWS];
#pragma unroll
	for (int r = 0; r < SROWS; r++) {
		const BUN i = base + r * 64 + lane;
		const bool valid = i < tend;
		const uint32_t d = (uint32_t) (k[r] >> shift) & 255;
#if MGDK_SORT_LDSMATCH
		// the wave's lanes OR their bit into their digit's mask, read it
		// back whole (a wave's LDS operations complete in order), clear it
		if (valid)
			__hip_atomic_fetch_or(&wm[d], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
		__builtin_amdgcn_wave_barrier();
		const uint64_t peer = valid ? __hip_atomic_load(&wm[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) : 0ull;
		__builtin_amdgcn_wave_barrier();
		if (valid)
			__hip_atomic_store(&wm[d], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
		__builtin_amdgcn_wave_barrier();
#else
		uint64_t peer = __ballot(valid);
#pragma unroll
		for (int b = 0; b < 8; b++) {
			const uint64_t bal = __ballot((d >> b) & 1);
			peer &= ((d >> b) & 1) ? bal : ~bal;
		}
#endif
		const uint32_t before = wcnt[w][d];
		rk[r] = ((before + (uint32_t) __popcll(peer & lt)) << 8) | d;
		if (valid && (peer >> lane) == 1)    // highest lane of its peer group
			wcnt[w][d] = before + (uint32_t) __popcll(peer);
	}
	__syncthreads();
	// digit d = tid: per-wave bases and the tile's digit prefix
	uint32_t tot = 0, incl = 0;
	if (dig) {
		uint32_t run = 0;
#pragma unroll
		for (int q = 0; q < SWAVES; q++) {
			const uint32_t c = wcnt[q][tid];
			wcnt[q][tid] = run;
			run += c;
		}
		tot = incl = run;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t u = __shfl_up(incl, o);
			if (lane >= (unsigned) o)
				incl += u;
		}
		if (lane == 63)
			s_wt[w] = incl;
	}
	__syncthreads();
	if (dig) {
		uint32_t ex = incl - tot;
		for (unsigned q = 0; q < w; q++)
			ex += s_wt[q];
		tstart[tid] = ex;
	}
	__syncthreads();
	// the tile reordered by digit in LDS before the look-back: the rows'
	// registers are free while the walk waits
#pragma unroll
	for (int r = 0; r < SROWS; r++) {
		const BUN i = base + r * 64 + lane;
		if (i < tend) {
			const uint32_t d = rk[r] & 255;
			const uint32_t lpos = tstart[d] + wcnt[w][d] + (rk[r] >> 8);
			sk[lpos] = k[r];
			sv[lpos] = v[r];
		}
	}
	if (LB) {
		// The walk back over the predecessors' digit counts: every thread
		// (digit) walks on its own, as the classic decoupled look-back.  A
		// claimed predecessor is running and publishes its counts before
		// anything it waits for, so waiting on it is safe.  An UNCLAIMED one
		// (XCD claims deal tiles out of order) may never be claimed while we
		// wait -- the dispatcher may have no room for the workgroup that
		// would claim it -- so a thread that finds its predecessor unclaimed
		// stops, and the workgroup then counts that tile's digits itself
		// from its keys (a pure function of the tile) and the thread walks
		// on: every round makes progress whatever is resident, and any claim
		// order is safe.  Claimed <=> its XCD's ticket has passed it (every
		// claim of a tile is an atomicAdd on its owner's ticket,
		// claim_tile).  Without a miss the walk costs one barrier.
		using namespace mgdk_lb;
		uint64_t excl = 0;
		bool done = blk == 0 || !dig;
		int64_t t = (int64_t) blk - 1;
		__shared__ uint32_t fh[256];           // a predecessor's digit counts, counted here
		__shared__ uint32_t s_miss;
		const uint32_t *xtk = ticket + 8;
		for (;;) {
			bool miss = false;
			uint32_t spins = 0;
#if MGDK_SORT_LBW > 1
			// the walk reads a window of LBW predecessors at once (their
			// loads in flight together) and consumes it in order up to the
			// first inclusive prefix or the first tile not yet published
			while (!done) {
				constexpr int LW = MGDK_SORT_LBW;
				uint64_t win[LW];
#pragma unroll
				for (int q = 0; q < LW; q++)
					win[q] = t - q >= 0 ? lb_load(status + (size_t) (t - q) * 256 + tid) : ST_PRE;
				bool stop = false, notready = false;
#pragma unroll
				for (int q = 0; q < LW; q++) {
					if (stop)
						continue;
					const uint64_t sv = win[q];
					if ((sv >> 62) == 0) {
						notready = true;
						stop = true;
						continue;
					}
					excl += sv & ST_VAL;
					if ((sv & ST_PRE) || --t < 0) {
						done = true;
						stop = true;
					}
				}
				if (!notready) {
					spins = 0;
					continue;
				}
				if (xg && (spins & 15) == 0) {
					const uint32_t y = (uint32_t) (t / xg) & 7;
					const uint32_t j = (uint32_t) (t / (8 * (int64_t) xg)) * xg + (uint32_t) (t % xg);
					if (__hip_atomic_load(&xtk[y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= j) {
						miss = true;
						break;
					}
				}
				if (++spins > (1u << 26)) {
					atomicOr(err, 1u);     // cannot happen: claimed tiles publish
					done = true;
					break;
				}
				__builtin_amdgcn_s_sleep(1);
			}
#else
			while (!done) {
				const uint64_t sv = lb_load(status + (size_t) t * 256 + tid);
				if ((sv >> 62) == 0) {
					if (xg && (spins & 15) == 0) {
						const uint32_t y = (uint32_t) (t / xg) & 7;
						const uint32_t j = (uint32_t) (t / (8 * (int64_t) xg)) * xg + (uint32_t) (t % xg);
						if (__hip_atomic_load(&xtk[y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= j) {
							miss = true;
							break;
						}
					}
					if (++spins > (1u << 26)) {
						atomicOr(err, 1u);     // cannot happen: claimed tiles publish
						done = true;
						break;
					}
					__builtin_amdgcn_s_sleep(1);
					continue;
				}
				spins = 0;
				excl += sv & ST_VAL;
				if ((sv & ST_PRE) || --t < 0)
					done = true;
			}
#endif
			if (!__syncthreads_or(miss))
				break;
			// the latest tile some thread is missing: count it here
			if (tid == 0)
				s_miss = 0;
			if (dig)
				fh[tid] = 0;
			__syncthreads();
			if (miss)
				atomicMax(&s_miss, (uint32_t) t + 1);
			__syncthreads();
			const int64_t ft = (int64_t) s_miss - 1;
			const BUN fb = (BUN) ft * STILE, fe = fb + STILE < n ? fb + STILE : n;
#pragma unroll 1
			for (int r = 0; r < SROWS; r += 4) {
				K fk[4];
#pragma unroll
				for (int u = 0; u < 4; u++) {
					const BUN i = fb + (BUN) (r + u) * STHREADS + tid;
					fk[u] = keys[i < fe ? i : fe - 1] ^ kx;
				}
#pragma unroll
				for (int u = 0; u < 4; u++)
					if (fb + (BUN) (r + u) * STHREADS + tid < fe)
						atomicAdd(&fh[(uint32_t) (fk[u] >> shift) & 255], 1u);
			}
			__syncthreads();
			if (miss && t == ft) {
				excl += fh[tid];
				if (--t < 0)
					done = true;
			}
			// a thread missing an earlier tile looks at it again (it may
			// be claimed by now, or is counted in a later round)
			__syncthreads();
		}
		if (dig && blk != 0)
			lb_store(status + (size_t) blk * 256 + tid, ST_PRE | (excl + tot));
		if (dig)
			gbase[tid] = gdig[tid] + (uint32_t) excl;
	}
	__syncthreads();
	const uint32_t nt = (uint32_t) (tend - tbase < (BUN) STILE ? tend - tbase : (BUN) STILE);
#pragma unroll
	for (int u = 0; u < SROWS; u++) {
		const uint32_t i = tid + u * STHREADS;
		if (i < nt) {
			const K key = sk[i];
			const uint32_t d = (uint32_t) (key >> shift) & 255;
			const BUN g = (BUN) gbase[d] + (i - tstart[d]);
			if (FINAL) {
				emit_final<K>(fo, g, key, sv[i]);
			} else {
				kout[g] = key;
				vout[g] = sv[i];
			}
		}
	}
}

template <typename K>
__global__ __launch_bounds__(256) void
k_andor(const K *keys, BUN n, unsigned long long *out)
{
	unsigned long long a = ~0ull, o = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		a &= (unsigned long long) keys[i];
		o |= (unsigned long long) keys[i];
	}
	a = block_reduce(a, [](unsigned long long x, unsigned long long y) { return x & y; });
	o = block_reduce(o, [](unsigned long long x, unsigned long long y) { return x | y; });
	if (threadIdx.x == 0) {
		const unsigned long long ca = __hip_atomic_load(&out[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const unsigned long long co = __hip_atomic_load(&out[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if ((ca & a) != ca)
			atomicAnd(&out[0], a);
		if ((co | o) != co)
			atomicOr(&out[1], o);
	}
}

// no radix pass needed (all keys equal): write the final outputs in place
template <typename K>
__global__ __launch_bounds__(256) void
k_final_copy(const K *keys, const uint32_t *vals, BUN n, FinalOut fo)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		emit_final<K>(fo, i, keys[i], vals ? vals[i] : (uint32_t) i);
}

// key image of a value
template <typename T, typename K>
__device__ __forceinline__ K
keyimg(T v, bool reverse, bool nilslast)
{
	uint64_t u;
	bool isnil;
	if constexpr (sizeof(T) == 4 && (T) 0.5 != 0) {          // float
		isnil = v != v;
		float f = v == 0 ? 0.0f : v;
		uint32_t b = __float_as_uint(f);
		b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
		u = sizeof(K) == 4 ? (uint64_t) b : (uint64_t) b << 32;
	} else if constexpr (sizeof(T) == 8 && (T) 0.5 != 0) {   // double
		isnil = v != v;
		double f = v == 0 ? 0.0 : v;
		uint64_t b = (uint64_t) __double_as_longlong(f);
		u = (b & (1ull << 63)) ? ~b : (b | (1ull << 63));
	} else if constexpr (T(-1) > T(0)) {                     // oid
		isnil = (uint64_t) v == ((uint64_t) 1 << 63);
		u = (uint64_t) v;
	} else {
		isnil = v == NilOf<T>::v();
		u = sizeof(K) == 4 ? (uint64_t) ((uint32_t) (int32_t) v ^ 0x80000000u)
				   : ((uint64_t) (int64_t) v ^ (1ull << 63));
	}
	const uint64_t all1 = sizeof(K) == 4 ? 0xffffffffull : ~0ull;
	if (reverse)
		u = ~u & all1;
	// integer nil is the type minimum: with nilslast == reverse its natural
	// image already sits at the requested end (and stays decodable)
	constexpr bool is_int = !((T) 0.5 != 0);
	if (isnil && !(is_int && reverse == nilslast))
		u = nilslast ? all1 : 0ull;
	return (K) u;
}

// key images + their AND/OR (constant digits are skipped by the passes)
template <typename T, typename K>
__global__ __launch_bounds__(256) void
k_keys(const T *col, BUN n, bool reverse, bool nilslast, K *keys, unsigned long long *andor, uint32_t *dh)
{
	// dh: the digit counts of every byte position (row b = bits 8b..8b+7),
	// for the radix passes' global digit starts (no separate read)
	constexpr int NBYTES = (int) sizeof(K);
	__shared__ uint32_t h[NBYTES][256];
	if (dh) {
		for (int q = 0; q < NBYTES; q++)
			h[q][threadIdx.x] = 0;
		__syncthreads();
	}
	unsigned long long a = ~0ull, o = 0;
	// 8 values per thread per step, all loaded before the first is used
	constexpr int KU = 8;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i0 = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += KU * stride) {
		T x[KU];
#pragma unroll
		for (int u = 0; u < KU; u++) {
			const BUN i = i0 + u * stride;
#if MGDK_SORT_NTLOAD
			x[u] = __builtin_nontemporal_load(col + (i < n ? i : n - 1));
#else
			x[u] = col[i < n ? i : n - 1];
#endif
		}
#pragma unroll
		for (int u = 0; u < KU; u++) {
			const BUN i = i0 + u * stride;
			if (i >= n)
				break;
			const K k = keyimg<T, K>(x[u], reverse, nilslast);
			if (keys)
				keys[i] = k;
			a &= (unsigned long long) k;
			o |= (unsigned long long) k;
			if (dh)
#pragma unroll
				for (int q = 0; q < NBYTES; q++)
					atomicAdd(&h[q][(uint32_t) (k >> (8 * q)) & 255], 1u);
		}
	}
	if (dh) {
		__syncthreads();
		for (int q = 0; q < NBYTES; q++)
			if (h[q][threadIdx.x])
				atomicAdd(&dh[q * 256 + threadIdx.x], h[q][threadIdx.x]);
	}
	a = block_reduce(a, [](unsigned long long x, unsigned long long y) { return x & y; });
	o = block_reduce(o, [](unsigned long long x, unsigned long long y) { return x | y; });
	if (threadIdx.x == 0) {
		// only when it changes the visible value: a same-word atomic from
		// every workgroup serialises
		const unsigned long long ca = __hip_atomic_load(&andor[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const unsigned long long co = __hip_atomic_load(&andor[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if ((ca & a) != ca)
			atomicAnd(&andor[0], a);
		if ((co | o) != co)
			atomicOr(&andor[1], o);
	}
}

template <typename T>
__global__ __launch_bounds__(256) void
k_gather_sorted(const T *col, const oid *order, BUN n, oid hseq, T *sorted)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		sorted[i] = col[order[i] - hseq];
}

template <typename K>
__global__ __launch_bounds__(256) void
k_newgrp(const K *keys, BUN n, uint8_t *flag)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		flag[i] = i > 0 && keys[i] != keys[i - 1];
}

// group ids of a sorted key image: gid[i] = number of i' in [1, i] with
// keys[i'] != keys[i'-1].  Two passes over 4096-key tiles (count, then
// write with a workgroup scan) around a scan of the tile counts: 16 B/row.
constexpr int GTILE = 4096;

// k_gid_count with whole 16-B loads (1 KiB per wave instruction): thread
// tid holds elements t0 + j * 256 V + tid V .. + V - 1 (V per 16 B); the
// element before a lane's first comes from the lane before (shfl) or, for
// lane 0, one scalar load.  keys must be 16-B aligned (the host checks)
template <typename K>
__global__ __launch_bounds__(256) void
k_gid_count_v(const K *keys, BUN n, uint32_t *cnt)
{
	constexpr int V = 16 / (int) sizeof(K), J = GTILE / 256 / V;
	static_assert(J >= 1 && GTILE % (256 * V) == 0, "whole 16-B pieces per thread");
	typedef uint32_t u4 __attribute__((ext_vector_type(4)));
	const BUN t0 = (BUN) blockIdx.x * GTILE;
	const unsigned tid = threadIdx.x, lane = __lane_id();
	const BUN nv = n / V;                  // whole 16-B pieces in the column
	u4 raw[J];
	K before[J];
#pragma unroll
	for (int j = 0; j < J; j++) {
		const BUN e0 = t0 + (BUN) j * 256 * V + (BUN) tid * V, pv = e0 / V;
		raw[j] = __builtin_nontemporal_load((const u4 *) keys + (pv < nv ? pv : (nv ? nv - 1 : 0)));
		before[j] = lane == 0 && e0 > 0 && e0 <= n ? keys[e0 - 1] : (K) 0;
	}
	uint32_t c = 0;
#pragma unroll
	for (int j = 0; j < J; j++) {
		K x[V];
		__builtin_memcpy(x, &raw[j], 16);
		const BUN e0 = t0 + (BUN) j * 256 * V + (BUN) tid * V;
		// a piece past the last whole one: its elements by scalar loads
		if (e0 / V >= nv)
#pragma unroll
			for (int v = 0; v < V; v++)
				x[v] = e0 + v < n ? keys[e0 + v] : (K) 0;
		K prev = __shfl_up(x[V - 1], 1);
		if (lane == 0)
			prev = before[j];
#pragma unroll
		for (int v = 0; v < V; v++) {
			const BUN i = e0 + v;
			c += i > 0 && i < n && x[v] != prev;
			prev = x[v];
		}
	}
	c = block_reduce(c, [](uint32_t a, uint32_t b) { return a + b; });
	if (threadIdx.x == 0)
		cnt[blockIdx.x] = c;
}

template <typename K>
__global__ __launch_bounds__(256) void
k_gid_count(const K *keys, BUN n, uint32_t *cnt)
{
	const BUN t0 = (BUN) blockIdx.x * GTILE;
	constexpr int Q = GTILE / 256;
	K cur[Q], prv[Q];
#pragma unroll
	for (int q = 0; q < Q; q++) {
		// unconditional loads at clamped rows, all in flight
		const BUN i = t0 + threadIdx.x + (BUN) q * 256, ic = i < n ? i : n - 1;
		cur[q] = keys[ic];
		prv[q] = keys[ic > 0 ? ic - 1 : 0];
	}
	uint32_t c = 0;
#pragma unroll
	for (int q = 0; q < Q; q++) {
		const BUN i = t0 + threadIdx.x + (BUN) q * 256;
		c += i > 0 && i < n && cur[q] != prv[q];
	}
	c = block_reduce(c, [](uint32_t a, uint32_t b) { return a + b; });
	if (threadIdx.x == 0)
		cnt[blockIdx.x] = c;
}

// group ids of sorted keys: element j of the tile (= q * 256 + thread) is a
// group start when its key differs from its predecessor's (read straight
// from memory: the same lines, shifted by one key); its id is the tile's
// prefix + the starts before it, ranked by one ballot per row and a 16 x 4
// LDS table of row / wave totals, and stored where it is (coalesced) -- no
// LDS image of the keys or ids, so the tile needs 256 B of LDS instead of
// 52 KiB (3 workgroups per CU before)
template <typename K>
__global__ __launch_bounds__(256) void
k_gid_write(const K *keys, BUN n, const uint64_t *pre, oid *gid)
{
	constexpr int Q = GTILE / 256;
	__shared__ uint32_t s_cnt[Q][4];
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const BUN t0 = (BUN) blockIdx.x * GTILE;
	K cur[Q], prv[Q];
#pragma unroll
	for (int q = 0; q < Q; q++) {
		const BUN i = t0 + (BUN) q * 256 + tid, ic = i < n ? i : n - 1;
		cur[q] = keys[ic];
		prv[q] = keys[ic > 0 ? ic - 1 : 0];
	}
	const uint64_t lt = (1ull << lane) - 1;
	uint64_t bal[Q];
#pragma unroll
	for (int q = 0; q < Q; q++) {
		const BUN i = t0 + (BUN) q * 256 + tid;
		bal[q] = __ballot(i > 0 && i < n && cur[q] != prv[q]);
		if (lane == 0)
			s_cnt[q][w] = (uint32_t) __popcll(bal[q]);
	}
	__syncthreads();
	uint64_t run = pre[blockIdx.x];
#pragma unroll
	for (int q = 0; q < Q; q++) {
		const BUN i = t0 + (BUN) q * 256 + tid;
		uint32_t before = 0, row = 0;
#pragma unroll
		for (unsigned v = 0; v < 4; v++) {
			before += v < w ? s_cnt[q][v] : 0;
			row += s_cnt[q][v];
		}
		if (i < n)
			gid[i] = run + before + (uint32_t) __popcll(bal[q] & lt) + (uint32_t) ((bal[q] >> lane) & 1);
		run += row;
	}
}

__global__ __launch_bounds__(256) void
k_gid(const uint64_t *excl, const uint8_t *flag, BUN n, oid *gid)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		gid[i] = excl[i] + flag[i];
}

// ---- MSD-then-local variant for 4-byte keys with >= 3 varying digits -------
// pass A scatters by the top varying digit d1 (the LSD scatter kernel, stable,
// positions as values); pass B sorts every d1 bucket by the next digit d2
// (tiles cut at bucket borders, one exclusive scan over (bucket, digit,
// tile) counts); every (d1, d2) bucket -- ~n / 65536 rows -- is then sorted
// by its remaining bits inside one workgroup's LDS (stable 4-bit counting
// passes) and written out as the final columns.  Three passes over HBM
// instead of four; the order is the stable one (each step is stable).

// the tiles of pass B: bucket b's rows cut into pieces of `tile` rows
__global__ __launch_bounds__(256) void
k_seg_tiles(const uint32_t *cnt, const uint32_t *start, uint32_t tile, uint4 *desc, uint32_t *count,
	    uint32_t *bfirst, uint32_t *bnt)
{
	__shared__ uint32_t ws[4];
	const unsigned b = threadIdx.x, lane = __lane_id(), w = b >> 6;
	const uint32_t c = cnt[b], t = (c + tile - 1) / tile;
	uint32_t x = t;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t u = __shfl_up(x, o);
		if (lane >= (unsigned) o)
			x += u;
	}
	if (lane == 63)
		ws[w] = x;
	__syncthreads();
	for (unsigned q = 0; q < w; q++)
		x += ws[q];
	const uint32_t first = x - t;
	bfirst[b] = first;
	bnt[b] = t;
	for (uint32_t j = 0; j < t; j++)
		desc[first + j] = make_uint4(start[b] + j * tile, c - j * tile < tile ? c - j * tile : tile, first, t);
	if (b == 255)
		*count = x;
}

// pass B's per-tile digit counts at 256 * first + d * tiles + (t - first)
template <typename K>
__global__ __launch_bounds__(256) void
k_seg_hist(const K *keys, int shift, SegTiles sg, uint32_t *hist)
{
	__shared__ uint32_t h[256];
	const uint32_t t = blockIdx.x;
	if (t >= *sg.count)
		return;
	const uint4 d = sg.desc[t];
	h[threadIdx.x] = 0;
	__syncthreads();
	constexpr int U = 8;
	for (uint32_t i0 = threadIdx.x; i0 < d.y; i0 += U * 256) {
		K k[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t i = i0 + u * 256;
			k[u] = i < d.y ? keys[d.x + i] : 0;
		}
#pragma unroll
		for (int u = 0; u < U; u++)
			if (i0 + u * 256 < d.y)
				atomicAdd(&h[(uint32_t) (k[u] >> shift) & 255], 1u);
	}
	__syncthreads();
	hist[(BUN) 256 * d.z + (BUN) threadIdx.x * d.w + (t - d.z)] = h[threadIdx.x];
}

// padded index of the counting table (one pad word per 16: the scan's
// 16-entry runs per thread fall on different banks)
__device__ __forceinline__ uint32_t
lpad(uint32_t i)
{
	return i + (i >> 4);
}

// one (d1, d2) bucket per one-wave workgroup (no workgroup barriers, many
// buckets per CU): the bucket's rows (R rows of 64 keys at most) are loaded
// with all loads in flight and sorted by their remaining bits in 8-bit
// stable LSD passes, ranked row by row as the scatter passes rank: a row's
// same-digit lanes from a per-digit LDS lane mask (one OR, one read, one
// clear), its rank = the digit's running count + the peers before it; one
// scan of the 256 counts gives the bases, the rows are placed in LDS and read
// back as rows for the next pass.  The sorted bucket leaves in coalesced
// rows.  GID: buckets claimed per XCD; each counts its group starts (its
// first row always starts one: consecutive buckets hold different leading
// digits) by ballots, and a decoupled look-back over the buckets numbers
// them (every bucket fits: the host checked the largest one first)
__device__ __forceinline__ void
wave_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
	__builtin_amdgcn_wave_barrier();
}

// sorts the rows held in k / v (row r = rows 64 r .. 64 r + 63 of the
// bucket, m of them) by the bits of ls; the sorted bucket is left in wk / wv
template <typename K, int R>
__device__ __forceinline__ void
local_sort(K (&k)[R], uint32_t (&v)[R], uint32_t m, const Shifts &ls, K *wk, uint32_t *wv,
	   unsigned long long *msk, uint32_t *dc)
{
	const unsigned lane = __lane_id();
	const uint32_t rows = (m + 63) >> 6;
	const uint64_t lt = (1ull << lane) - 1;
	wave_sync();
	bool sorted_in_lds = false;
	for (int p = 0; p < ls.n && m > 1; p++) {
		const int sh = ls.s[p];
#pragma unroll
		for (int x = 0; x < 4; x++) {
			msk[lane + 64 * x] = 0ull;
			dc[lane + 64 * x] = 0;
		}
		wave_sync();
		uint32_t rk[R];
#pragma unroll
		for (int r = 0; r < R; r++) {
			rk[r] = 0;
			if ((uint32_t) r < rows) {
				const bool valid = lane + 64 * r < m;
				const uint32_t dg = (uint32_t) (k[r] >> sh) & 255;
				if (valid)
					__hip_atomic_fetch_or(&msk[dg], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
				wave_sync();
				const uint64_t peer = valid ? msk[dg] : 0ull;
				const uint32_t before = valid ? dc[dg] : 0;
				wave_sync();
				if (valid) {
					msk[dg] = 0ull;
					if ((peer >> lane) == 1)      // highest lane of its peer group
						dc[dg] = before + (uint32_t) __popcll(peer);
				}
				wave_sync();
				rk[r] = before + (uint32_t) __popcll(peer & lt);
			}
		}
		// exclusive scan of the 256 digit counts (4 per lane)
		uint32_t c4[4], sum = 0;
#pragma unroll
		for (int x = 0; x < 4; x++) {
			c4[x] = dc[4 * lane + x];
			sum += c4[x];
		}
		uint32_t inc = sum;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t t = __shfl_up(inc, o);
			if (lane >= (unsigned) o)
				inc += t;
		}
		uint32_t ex = inc - sum;
		wave_sync();
#pragma unroll
		for (int x = 0; x < 4; x++) {
			dc[4 * lane + x] = ex;
			ex += c4[x];
		}
		wave_sync();
#pragma unroll
		for (int r = 0; r < R; r++) {
			if ((uint32_t) r < rows && lane + 64 * r < m) {
				const uint32_t pos = dc[(uint32_t) (k[r] >> sh) & 255] + rk[r];
				wk[pos] = k[r];
				wv[pos] = v[r];
			}
		}
		wave_sync();
		sorted_in_lds = true;
		if (p + 1 < ls.n) {
#pragma unroll
			for (int r = 0; r < R; r++) {
				if ((uint32_t) r < rows) {
					k[r] = wk[lane + 64 * r];
					v[r] = wv[lane + 64 * r];
				}
			}
		}
	}
	if (!sorted_in_lds) {
#pragma unroll
		for (int r = 0; r < R; r++)
			if (lane + 64 * r < m) {
				wk[lane + 64 * r] = k[r];
				wv[lane + 64 * r] = v[r];
			}
		wave_sync();
	}
}

// the sorted bucket in wk / wv leaves in pairs of rows at even global
// positions (16-byte oid and group-id stores, 8-byte value stores where both
// are in the bucket); GID: run = the group id before the bucket's first row
template <typename K, int R, bool GID>
__device__ __forceinline__ void
local_emit(uint32_t s, uint32_t m, const FinalOut &fo, uint64_t run, const K *wk, const uint32_t *wv)
{
	const unsigned lane = __lane_id();
	const uint64_t lt = (1ull << lane) - 1;
	const uint32_t a = s & 1;
	const uint32_t prow = (m + a + 127) >> 7;
	const bool fast = sizeof(K) == 4 && fo.vw == 4 && fo.sorted && fo.order && !fo.keys;
	typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
	typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
	for (int r = 0; r < R / 2 + 1; r++) {
		if ((uint32_t) r < prow) {
			const int32_t i0 = (int32_t) (128 * r + 2 * lane) - (int32_t) a;   // local index of the pair
			const bool v0 = i0 >= 0 && i0 < (int32_t) m, v1 = i0 + 1 < (int32_t) m;
			const K k0 = v0 ? wk[i0] : (K) 0, k1 = v1 ? wk[i0 + 1] : (K) 0;
			const uint32_t x0 = v0 ? wv[i0] : 0, x1 = v1 ? wv[i0 + 1] : 0;
			uint64_t g0 = 0, g1 = 0;
			if (GID) {
				const bool f0 = v0 && (i0 > 0 ? k0 != wk[i0 - 1] : s > 0);
				const bool f1 = v1 && (i0 + 1 > 0 ? k1 != (v0 ? k0 : wk[i0]) : s > 0);
				const uint64_t b0 = __ballot(f0), b1 = __ballot(f1);
				g0 = run + (uint64_t) (__popcll(b0 & lt) + __popcll(b1 & lt)) + f0;
				g1 = g0 + f1;
				run += (uint64_t) (__popcll(b0) + __popcll(b1));
			}
			const BUN g = (BUN) s + (BUN) i0;
			if (fast && v0 && v1) {
				uint32_t u0 = (uint32_t) k0, u1 = (uint32_t) k1;
				if (fo.reverse) {
					u0 = ~u0;
					u1 = ~u1;
				}
				*(u32x2 *) ((int32_t *) fo.sorted + g) = (u32x2){u0 ^ 0x80000000u, u1 ^ 0x80000000u};
				*(u64x2 *) (fo.order + g) = (u64x2){fo.hseq + x0, fo.hseq + x1};
				if (GID)
					*(u64x2 *) (fo.gid + g) = (u64x2){g0, g1};
			} else {
				if (v0) {
					emit_final<K>(fo, g, k0, x0);
					if (GID)
						fo.gid[g] = g0;
				}
				if (v1) {
					emit_final<K>(fo, g + 1, k1, x1);
					if (GID)
						fo.gid[g + 1] = g1;
				}
			}
		}
	}
}

template <typename K, int R>
__device__ __forceinline__ void
local_load(const K *keys, const uint32_t *vals, uint32_t s, uint32_t m, K (&k)[R], uint32_t (&v)[R])
{
	const unsigned lane = __lane_id();
#pragma unroll
	for (int r = 0; r < R; r++) {
		const uint32_t i = lane + 64 * r, ic = i < m ? i : (m ? m - 1 : 0);
		k[r] = keys[s + ic];
		v[r] = vals[s + ic];
	}
}

template <typename K, int R, bool GID>
__global__ __launch_bounds__(64) void
k_rs_local(const K *keys, const uint32_t *vals, const uint32_t *bs, Shifts ls, FinalOut fo, uint32_t *ovf,
	   uint32_t *ticket, uint64_t *status, uint32_t *err, uint32_t xg)
{
	constexpr int CAP = 64 * R;
	__shared__ K wk[CAP];
	__shared__ uint32_t wv[CAP];
	__shared__ unsigned long long msk[256];
	__shared__ uint32_t dc[256];
	const unsigned lane = __lane_id();
	uint32_t q = blockIdx.x;
	if (GID) {
		// claimed in ticket order: the group ids' look-back needs every
		// predecessor bucket claimed earlier (its distinct-key count is not
		// something a waiting wave can recompute cheaply), so no per-XCD
		// claims here (MGDK_SORT_LOCALXG, round 4, could leave a predecessor
		// unclaimed behind a spinning wave)
		uint32_t t = 0;
		if (lane == 0)
			t = xg ? claim_tile(ticket + 8, 65536, xg) : atomicAdd(ticket, 1u);
		q = __shfl(t, 0);
	}
	const uint32_t s = bs[q], m = bs[q + 1] - s;
	if (m == 0) {
		if (GID)
			(void) mgdk_lb::lookback(status, q, 0, err);
		return;
	}
	if (m > (uint32_t) CAP) {
		// sorted by the host afterwards (rare: the gate expects <= CAP / 2)
		if (lane == 0) {
			const uint32_t o = atomicAdd(&ovf[0], 1u);
			ovf[1 + 2 * o] = s;
			ovf[2 + 2 * o] = m;
		}
		return;
	}
	K k[R];
	uint32_t v[R];
	local_load<K, R>(keys, vals, s, m, k, v);
	local_sort<K, R>(k, v, m, ls, wk, wv, msk, dc);
	uint64_t run = 0;
	if (GID) {
		// group starts in this bucket, counted by ballots
		uint32_t c = 0;
		const uint32_t rows = (m + 63) >> 6;
#pragma unroll
		for (int r = 0; r < R; r++) {
			if ((uint32_t) r < rows) {
				const uint32_t i = lane + 64 * r;
				const bool st = i < m && (i > 0 ? wk[i] != wk[i - 1] : s > 0);
				c += (uint32_t) __popcll(__ballot(st));
			}
		}
		run = mgdk_lb::lookback(status, q, c, err);
	}
	local_emit<K, R, GID>(s, m, fo, run, wk, wv);
}

// BPW consecutive buckets per one-wave workgroup, the next bucket's rows
// loaded while the current one is sorted (no group ids: those need every
// bucket's predecessors, see k_rs_local<GID>)
template <typename K, int R, int BPW>
__global__ __launch_bounds__(64) void
k_rs_local_mb(const K *keys, const uint32_t *vals, const uint32_t *bs, Shifts ls, FinalOut fo, uint32_t *ovf)
{
	constexpr int CAP = 64 * R;
	__shared__ K wk[CAP];
	__shared__ uint32_t wv[CAP];
	__shared__ unsigned long long msk[256];
	__shared__ uint32_t dc[256];
	const unsigned lane = __lane_id();
	const uint32_t q0 = blockIdx.x * BPW;
	const uint32_t bl = lane <= (unsigned) BPW ? bs[q0 + lane] : 0;
	K k[2][R];
	uint32_t v[2][R];
	{
		const uint32_t s0 = __shfl(bl, 0), m0 = __shfl(bl, 1) - s0;
		if (m0 <= (uint32_t) CAP)
			local_load<K, R>(keys, vals, s0, m0, k[0], v[0]);
	}
#pragma unroll
	for (int j = 0; j < BPW; j++) {
		const uint32_t s = __shfl(bl, j), m = __shfl(bl, j + 1) - s;
		if (j + 1 < BPW) {
			const uint32_t s1 = __shfl(bl, j + 1), m1 = __shfl(bl, j + 2) - s1;
			if (m1 <= (uint32_t) CAP)
				local_load<K, R>(keys, vals, s1, m1, k[(j + 1) & 1], v[(j + 1) & 1]);
		}
		if (m == 0)
			continue;
		if (m > (uint32_t) CAP) {
			if (lane == 0) {
				const uint32_t o = atomicAdd(&ovf[0], 1u);
				ovf[1 + 2 * o] = s;
				ovf[2 + 2 * o] = m;
			}
			continue;
		}
		local_sort<K, R>(k[j & 1], v[j & 1], m, ls, wk, wv, msk, dc);
		local_emit<K, R, false>(s, m, fo, 0, wk, wv);
	}
}

// the largest (d1, d2) bucket (decides the LDS capacity / the GID variant)
__global__ __launch_bounds__(256) void
k_bucket_max(const uint32_t *offs, const uint32_t *bfirst, const uint32_t *bnt, const uint32_t *bstart,
	     const uint32_t *bcnt, uint32_t *mx, uint32_t *bs)
{
	const uint32_t q = blockIdx.x * 256 + threadIdx.x, b = q >> 8, d = q & 255;
	const uint32_t nt = bnt[b], f = bfirst[b];
	uint32_t m = 0, s = bstart[b];
	if (nt != 0) {
		s = offs[(BUN) 256 * f + (BUN) d * nt];
		const uint32_t e = d < 255 ? offs[(BUN) 256 * f + (BUN) (d + 1) * nt] : bstart[b] + bcnt[b];
		m = e - s;
	}
	bs[q] = s;
	if (q == 65535)
		bs[65536] = bstart[b] + bcnt[b];
	m = block_reduce(m, [](uint32_t x, uint32_t y) { return x > y ? x : y; });
	if (threadIdx.x == 0)
		atomicMax(mx, m);
}

template <typename K>
__global__ __launch_bounds__(256) void
k_final_copy_at(const K *keys, const uint32_t *vals, BUN m, BUN s, FinalOut fo)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (BUN) gridDim.x * blockDim.x)
		emit_final<K>(fo, s + i, keys[i], vals[i]);
}

// tiles per XCD group of the scatter passes (0: plain ticket order).  The
// first tile of an XCD's group depends on the previous XCD's whole group;
// the tiles of it that are not claimed yet are counted by the waiting tile
// itself (k_rs_scatter), so any group size completes (before that fallback
// 128 / 256 took 9.4 ms / never completed on 100M int32).  Measured with
// the 8 x 16 tile (profiles/r05/sort): 16 2.87, 24 3.06, 32 2.80, 48 3.54,
// 64 3.24, 128 8.0 ms; 8-byte keys keep round 4's 32
static uint32_t
sort_xg(int kw = 4)
{
	const char *e = getenv("MGDK_SORT_XCDG");
	return e ? (uint32_t) atoi(e) : 32u;
}

// src0: when set, `keys` was NOT filled; the first pass reads the column
// src0 and takes src0[i] ^ kx0 as the image (4-byte integers: the sign flip,
// or its complement for a reverse sort); any other use of the images
// materialises them first
template <typename K>
int radix_sort(K *keys, uint32_t *vals, K *keys_alt, uint32_t *vals_alt, BUN n, int bits, const FinalOut *fo,
	       bool positions, bool andor, K **keys_out, uint32_t **vals_out, const uint32_t *digit_hist = nullptr,
	       const K *src0 = nullptr, K kx0 = 0);

template <typename K>
__global__ __launch_bounds__(256) void
k_img_xor(const K *src, BUN n, K kx, K *keys)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		keys[i] = src[i] ^ kx;
}

// k_img_xor that also counts two digits of the images (the MSD-then-local
// path's d1 / d2 when they are not whole bytes, which k_keys's byte counts do
// not give): out[(s / 8) * 256 + digit] as k_rs_dhist lays them out, so the
// keys are not read once more for them
template <typename K>
__global__ __launch_bounds__(256) void
k_img_xor_h2(const K *src, BUN n, K kx, K *keys, int s1, int s2, uint32_t *out)
{
	__shared__ uint32_t h[2][256];
	h[0][threadIdx.x] = 0;
	h[1][threadIdx.x] = 0;
	__syncthreads();
	constexpr int KU = 8;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i0 = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += KU * stride) {
		K k[KU];
#pragma unroll
		for (int u = 0; u < KU; u++) {
			const BUN i = i0 + u * stride;
			k[u] = src[i < n ? i : n - 1] ^ kx;
		}
#pragma unroll
		for (int u = 0; u < KU; u++) {
			const BUN i = i0 + u * stride;
			if (i < n) {
				keys[i] = k[u];
				atomicAdd(&h[0][(uint32_t) (k[u] >> s1) & 255], 1u);
				atomicAdd(&h[1][(uint32_t) (k[u] >> s2) & 255], 1u);
			}
		}
	}
	__syncthreads();
	if (h[0][threadIdx.x])
		atomicAdd(&out[(s1 / 8) * 256 + threadIdx.x], h[0][threadIdx.x]);
	if (h[1][threadIdx.x])
		atomicAdd(&out[(s2 / 8) * 256 + threadIdx.x], h[1][threadIdx.x]);
}

// passes A, B, C (see above); keys / vals hold the input images, the
// alternates are free; cap: the largest (d1, d2) bucket sorted in LDS
template <typename K>
int
radix_hybrid(K *k0, uint32_t *v0, K *k1, uint32_t *v1, BUN n, int s1, int s2, uint64_t diff, const uint32_t *cnt1,
	     const uint32_t *gd1, uint64_t *status, uint32_t *lbm, const FinalOut &fo0, int cap, K **keys_out,
	     uint32_t **vals_out)
{
	hipStream_t st = stream();
	constexpr uint32_t TILE = (uint32_t) Tile<K>::N;
	const uint32_t nblocks = (uint32_t) ((n + TILE - 1) / TILE);
	const uint32_t tmax = nblocks + 256;
	DevBuf desc((size_t) tmax * 16 + 64), meta(4 * 1024), hist((size_t) 256 * tmax * 4 + 64),
		offs((size_t) 256 * tmax * 4 + 64), ovf((size_t) (1 + 2 * 65536) * 4);
	if (!desc.p || !meta.p || !hist.p || !offs.p || !ovf.p)
		return -1;
	uint32_t *count = meta.as<uint32_t>(), *bfirst = count + 256, *bnt = count + 512;
	FinalOut none{};
	// pass A: by d1, positions as values (status and lbm arrive zeroed:
	// radix_sort clears them before it chooses this path)
	if (!hip_ok(hipMemsetAsync(hist.p, 0, (size_t) 256 * tmax * 4, st), "memset") ||
	    !hip_ok(hipMemsetAsync(ovf.p, 0, 4, st), "memset"))
		return -1;
	hipLaunchKernelGGL((k_rs_scatter<K, false, true, true, false>), dim3(nblocks), dim3(Tile<K>::THREADS), 0, st, k0,
			   v0, n, s1, nullptr, nblocks, k1, v1, none, lbm, status, gd1, lbm + 4, SegTiles{}, sort_xg((int) sizeof(K)),
			   nullptr, (K) 0);
	// pass B: by d2 inside the d1 buckets
	hipLaunchKernelGGL(k_seg_tiles, dim3(1), dim3(256), 0, st, cnt1, gd1, TILE, desc.as<uint4>(), count, bfirst,
			   bnt);
	const SegTiles sg{desc.as<uint4>(), count};
	hipLaunchKernelGGL((k_seg_hist<K>), dim3(tmax), dim3(256), 0, st, (const K *) k1, s2, sg, hist.as<uint32_t>());
	if (exclusive_scan(hist.as<uint32_t>(), offs.as<uint32_t>(), (BUN) 256 * tmax, nullptr) < 0 ||
	    !hip_ok(hipMemsetAsync(lbm + 8, 0, 32, st), "memset"))
		return -1;
	hipLaunchKernelGGL((k_rs_scatter<K, false, false, false, true>), dim3(tmax), dim3(Tile<K>::THREADS), 0, st,
			   (const K *) k1, (const uint32_t *) v1, n, s2, offs.as<uint32_t>(), tmax, k0, v0, none, lbm,
			   status, gd1, lbm + 4, sg, sort_xg((int) sizeof(K)), nullptr, (K) 0);
	// pass C: the remaining varying bits, 4 at a time, inside each (d1, d2) bucket
	// the remaining bits in 8-bit LSD digits (the top one may reach into d2,
	// constant inside a bucket)
	Shifts ls{};
	for (int q = 0; q < s2; q += 8)
		if ((diff >> q) & 255)
			ls.s[ls.n++] = q;
	FinalOut fo = fo0;
	if (fo.want_keys)
		fo.keys = k1;
	// every (d1, d2) bucket's start, and the largest bucket (the group ids
	// ride along only when every bucket fits in LDS)
	DevBuf bsb((size_t) (65536 + 1) * 4 + 64);
	uint32_t *mx = count + 768, *hm = (uint32_t *) pinned(16);
	if (!bsb.p || !hm || !hip_ok(hipMemsetAsync(mx, 0, 4, st), "memset"))
		return -1;
	hipLaunchKernelGGL(k_bucket_max, dim3(256), dim3(256), 0, st, (const uint32_t *) offs.as<uint32_t>(),
			   (const uint32_t *) bfirst, (const uint32_t *) bnt, gd1, cnt1, mx, bsb.as<uint32_t>());
	// the LDS capacity from the largest bucket
	if (!hip_ok(hipMemcpyAsync(hm, mx, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	if (hm[0] <= 4096)
		cap = hm[0] <= 1024 ? 1024 : hm[0] <= 2048 ? 2048 : 4096;
	const bool use_fg = getenv("MGDK_SORT_FUSEGID") ? atoi(getenv("MGDK_SORT_FUSEGID")) != 0 : true;
	const bool gid = fo.gid != nullptr && use_fg && hm[0] <= 4096;
	if (!gid)
		fo.gid = nullptr;
	DevBuf gst(gid ? (size_t) 65536 * 8 + 64 : 64);
	if (!gst.p || (gid && !hip_ok(hipMemsetAsync(gst.p, 0, (size_t) 65536 * 8 + 64, st), "memset")))
		return -1;
	// GID: the ticket words and the error flag follow the 65536 status words
	uint32_t *gtk = gid ? (uint32_t *) (gst.as<uint64_t>() + 65536) : gst.as<uint32_t>(), *ger = gtk + 4;
#define LOCAL(R, G) hipLaunchKernelGGL((k_rs_local<K, R, G>), dim3(65536), dim3(64), 0, st, (const K *) k0, \
				       (const uint32_t *) v0, (const uint32_t *) bsb.as<uint32_t>(), ls, fo, ovf.as<uint32_t>(), gtk, \
				       gst.as<uint64_t>(), ger, 0u)
#define LOCALMB(R) hipLaunchKernelGGL((k_rs_local_mb<K, R, 4>), dim3(65536 / 4), dim3(64), 0, st, (const K *) k0, \
				      (const uint32_t *) v0, (const uint32_t *) bsb.as<uint32_t>(), ls, fo, ovf.as<uint32_t>())
	if (cap <= 1024) {
		if (gid) LOCAL(16, true); else LOCALMB(16);
	} else if (cap <= 2048) {
		if (gid) LOCAL(32, true); else LOCALMB(32);
	} else {
		if (gid) LOCAL(64, true); else LOCALMB(64);
	}
#undef LOCALMB
#undef LOCAL
	uint32_t *h = (uint32_t *) pinned(16);
	if (!h || !hip_ok(hipMemcpyAsync(h, ovf.p, 4, hipMemcpyDeviceToHost, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(h + 1, lbm + 4, 4, hipMemcpyDeviceToHost, st), "memcpy") ||
	    (gid && !hip_ok(hipMemcpyAsync(h + 2, ger, 4, hipMemcpyDeviceToHost, st), "memcpy")) ||
	    (gid && !hip_ok(hipMemcpyAsync(h + 4, fo.gid + n - 1, 8, hipMemcpyDeviceToHost, st), "memcpy")) || !sync())
		return -1;
	if (h[1] || (gid && h[2])) {
		seterr("HY013!BATsort: radix look-back did not complete");
		return -1;
	}
	const uint32_t nov = h[0];
	if (nov) {
		std::vector<uint32_t> ov((size_t) 2 * nov);
		if (!hip_ok(hipMemcpyAsync(ov.data(), ovf.as<uint32_t>() + 1, (size_t) 8 * nov, hipMemcpyDeviceToHost, st),
			    "memcpy") ||
		    !sync_data())
			return -1;
		for (uint32_t q = 0; q < nov; q++) {
			const BUN s = ov[2 * q], m = ov[2 * q + 1];
			K *ks;
			uint32_t *vs;
			if (radix_sort<K>(k0 + s, v0 + s, k1 + s, v1 + s, m, 8 * (int) sizeof(K), nullptr, false, false, &ks,
					  &vs) < 0)
				return -1;
			hipLaunchKernelGGL((k_final_copy_at<K>), dim3(grid_for(m, 1024, 8192)), dim3(256), 0, st,
					   (const K *) ks, (const uint32_t *) vs, m, s, fo);
		}
	}
	if (gid && fo0.gid_done) {
		*fo0.gid_done = true;
		if (fo0.gid_last)
			*fo0.gid_last = *(const uint64_t *) (h + 4);
	}
	*keys_out = fo.want_keys ? k1 : k0;
	*vals_out = v0;
	return sync() ? 0 : -1;
}

// stable LSD radix sort of (key, position) pairs; the final pass (when fo
// is given) writes the result columns instead of the pairs
// positions: the values are 0..n-1 and `vals` is uninitialised (the first
// pass generates them); andor: the keys' AND/OR at meta_buf() are already
// computed
template <typename K>
int
radix_sort(K *keys, uint32_t *vals, K *keys_alt, uint32_t *vals_alt, BUN n, int bits, const FinalOut *fo,
	   bool positions, bool andor, K **keys_out, uint32_t **vals_out, const uint32_t *digit_hist, const K *src0,
	   K kx0)
{
	*keys_out = keys;
	*vals_out = vals;
	hipStream_t st = stream();
	if (n == 0)
		return 0;
	unsigned long long *ao = (unsigned long long *) meta_buf();
	if (src0 != nullptr && !andor) {
		hipLaunchKernelGGL((k_img_xor<K>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, src0, n, kx0, keys);
		src0 = nullptr;
	}
	if (!andor) {
		unsigned long long init[2] = {~0ull, 0ull};
		if (!hip_ok(hipMemcpyAsync(ao, init, 16, hipMemcpyHostToDevice, st), "memcpy"))
			return -1;
		hipLaunchKernelGGL((k_andor<K>), dim3(grid_for(n, 8192, 1024)), dim3(256), 0, st, keys, n, ao);
	}
	// the MSD-then-local variant needs the digit counts of d1 and d2 to
	// choose its bucket capacity
	// MGDK_SORT_HYBRID (read on every call so tests can switch it); the
	// default is SORT_HYBRID_DEFAULT
	const bool use_hy = getenv("MGDK_SORT_HYBRID") ? atoi(getenv("MGDK_SORT_HYBRID")) != 0 : SORT_HYBRID_DEFAULT != 0;
	const bool hy_try = use_hy && sizeof(K) == 4 && fo != nullptr && positions && digit_hist != nullptr &&
			    n >= ((BUN) 1 << 22);
	unsigned long long *h = (unsigned long long *) pinned(16 + 4 * 256 * 4);
	if (!h || !hip_ok(hipMemcpyAsync(h, ao, 16, hipMemcpyDeviceToHost, st), "memcpy") ||
	    (hy_try && !hip_ok(hipMemcpyAsync(h + 2, digit_hist, 4 * 256 * 4, hipMemcpyDeviceToHost, st), "memcpy")) ||
	    !sync())
		return -1;
	const uint64_t diff = h[0] ^ h[1];
	std::vector<int> shifts;
	for (int shift = 0; shift < bits; shift += 8)
		if ((diff >> shift) & 255)
			shifts.push_back(shift);   // other digits are constant: identity passes
	const uint32_t nblocks = (uint32_t) ((n + Tile<K>::N - 1) / Tile<K>::N);
	static const bool use_lb = getenv("MGDK_SORT_LB") ? atoi(getenv("MGDK_SORT_LB")) != 0 : true;
	const bool lb = use_lb && !shifts.empty() && shifts.size() <= (size_t) RS_MAXP;
	// the MSD-then-local path's top two varying digits; when they are not
	// whole bytes their counts come with the images' materialisation below
	const int hy_hi = diff ? 63 - __builtin_clzll(diff) : -1;
	const bool hy_h2 = hy_try && hy_hi >= 16 && (hy_hi - 7) % 8 != 0 && src0 != nullptr &&
			   !shifts.empty() && lb;
	DevBuf h2c(hy_h2 ? RS_MAXP * 256 * 4 * 2 + 64 : 64);
	if (!h2c.p)
		return -1;
	if (src0 != nullptr && (shifts.empty() || hy_try || !positions || !lb || !andor || digit_hist == nullptr)) {
		// paths that read the images themselves: materialise them
		if (hy_h2) {
			if (!hip_ok(hipMemsetAsync(h2c.p, 0, RS_MAXP * 256 * 4, st), "memset"))
				return -1;
			hipLaunchKernelGGL((k_img_xor_h2<K>), dim3(grid_for(n, 16384, 2048)), dim3(256), 0, st, src0, n, kx0,
					   keys, hy_hi - 7, hy_hi - 15, h2c.as<uint32_t>());
		} else {
			hipLaunchKernelGGL((k_img_xor<K>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, src0, n, kx0, keys);
		}
		src0 = nullptr;
	}
	DevBuf hist(lb ? 64 : (size_t) 256 * nblocks * 4), offs(lb ? 64 : (size_t) 256 * nblocks * 4);
	// look-back state: two status arrays (pass s uses status[s % 2] and
	// zeroes status[(s + 1) % 2] for the next pass), ticket words per pass
	// (16 words each: ticket, -, -, -, -, ..., 8 XCD tickets), the error flag
	// after them -- zeroed once, not per pass
	DevBuf status(lb ? (size_t) 256 * nblocks * 8 : 64), status2(lb && shifts.size() > 1 ? (size_t) 256 * nblocks * 8 : 64),
		dcnt(RS_MAXP * 256 * 4 * 2 + 64), lbm(64 * (RS_MAXP + 1));
	if (!hist.p || !offs.p || !status.p || !status2.p || !dcnt.p || !lbm.p)
		return -1;
	uint32_t *lb_err = lbm.as<uint32_t>() + 16 * RS_MAXP + 4;
	uint32_t *gdig = dcnt.as<uint32_t>() + RS_MAXP * 256;
	if (lb) {
		Shifts sh{};
		sh.n = (int) shifts.size();
		for (int q = 0; q < sh.n; q++)
			sh.s[q] = shifts[q];
		if (!hip_ok(hipMemsetAsync(lbm.p, 0, 64 * (RS_MAXP + 1), st), "memset") ||
		    !hip_ok(hipMemsetAsync(status.p, 0, (size_t) 256 * nblocks * 8, st), "memset"))
			return -1;
		const uint32_t *dh = digit_hist;
		if (dh == nullptr) {
			if (!hip_ok(hipMemsetAsync(dcnt.p, 0, RS_MAXP * 256 * 4, st), "memset"))
				return -1;
			hipLaunchKernelGGL((k_rs_dhist<K>), dim3(grid_for(n, 16384, 2048)), dim3(256), 0, st, keys, n, sh,
					   dcnt.as<uint32_t>());
			dh = dcnt.as<uint32_t>();
		}
		hipLaunchKernelGGL(k_rs_dscan, dim3(sh.n), dim3(256), 0, st, dh, sh, gdig);
		const int hi = diff ? 63 - __builtin_clzll(diff) : -1;
		if (hy_try && hi >= 16) {
			// d1: the top 8 varying bits, d2: the 8 below them; their counts
			// from the key-image pass when they are whole bytes, else one
			// more read of the keys
			const int s1 = hi - 7, s2 = s1 - 8;
			const uint32_t *hc1, *hc2, *cnt1, *gd1;
			DevBuf hcnt(RS_MAXP * 256 * 4 * 2 + 64);
			if (!hcnt.p)
				return -1;
			if (s1 % 8 == 0) {
				const uint32_t *hc = (const uint32_t *) (h + 2);
				hc1 = hc + (s1 / 8) * 256;
				hc2 = hc + (s2 / 8) * 256;
				cnt1 = dh + (s1 / 8) * 256;
				size_t q = 0;
				while (shifts[q] != s1)
					q++;
				gd1 = gdig + q * 256;
			} else {
				Shifts s12{};
				s12.n = 2;
				s12.s[0] = s2;
				s12.s[1] = s1;
				uint32_t *c = hy_h2 ? h2c.as<uint32_t>() : hcnt.as<uint32_t>(), *g = c + RS_MAXP * 256;
				uint32_t *hh = (uint32_t *) (h + 2);
				if (!hy_h2) {
					if (!hip_ok(hipMemsetAsync(c, 0, RS_MAXP * 256 * 4, st), "memset"))
						return -1;
					hipLaunchKernelGGL((k_rs_dhist<K>), dim3(grid_for(n, 16384, 2048)), dim3(256), 0, st, keys, n,
							   s12, c);
				}
				hipLaunchKernelGGL(k_rs_dscan, dim3(2), dim3(256), 0, st, (const uint32_t *) c, s12, g);
				if (!hip_ok(hipMemcpyAsync(hh, c, (size_t) 4 * 256 * 4, hipMemcpyDeviceToHost, st), "memcpy") ||
				    !sync())
					return -1;
				hc1 = hh + (s1 / 8) * 256;
				hc2 = hh + (s2 / 8) * 256;
				cnt1 = c + (s1 / 8) * 256;
				gd1 = g + 256;
			}
			// expected largest (d1, d2) bucket if the two digits were independent
			uint32_t m1 = 0, m2 = 0;
			for (int b = 0; b < 256; b++) {
				m1 = hc1[b] > m1 ? hc1[b] : m1;
				m2 = hc2[b] > m2 ? hc2[b] : m2;
			}
			const double est = (double) m1 * (double) m2 / (double) n;
			const int cap = est <= 1024 ? 2048 : est <= 2048 ? 4096 : 0;
			if (cap)      // status and lbm as cleared above, untouched since
				return radix_hybrid<K>(keys, vals, keys_alt, vals_alt, n, s1, s2, diff, cnt1, gd1,
						       status.as<uint64_t>(), lbm.as<uint32_t>(), *fo, cap, keys_out, vals_out);
		}
	}
	K *kin = keys, *kout = keys_alt;
	uint32_t *vin = vals, *vout = vals_alt;
	FinalOut none{};
	// the first pass reads the column itself (src0, kx0) when given
	for (size_t s = 0; s < shifts.size(); s++) {
		const int shift = shifts[s];
		const bool fin = fo != nullptr && s + 1 == shifts.size();
		const bool idv = positions && s == 0;
		uint64_t *sts = (s & 1 ? status2 : status).as<uint64_t>();
		uint64_t *znx = lb && s + 1 < shifts.size() ? (s & 1 ? status : status2).as<uint64_t>() : nullptr;
		if (!lb) {
			hipLaunchKernelGGL((k_rs_hist<K>), dim3(nblocks), dim3(256), 0, st, kin, n, shift,
					   hist.as<uint32_t>(), nblocks);
			if (exclusive_scan(hist.as<uint32_t>(), offs.as<uint32_t>(), (BUN) 256 * nblocks, nullptr) < 0)
				return -1;
		}
		FinalOut f2 = fin ? *fo : none;
		if (fin && f2.want_keys)
			f2.keys = kout;
		uint32_t *tk = lbm.as<uint32_t>() + 16 * s, *er = lb_err;
		const uint32_t *gd = gdig + s * 256;
		const K *kfrom = s == 0 && src0 ? src0 : kin;
		const K kx = s == 0 && src0 ? kx0 : (K) 0;
#define SCAT(F, I, L) hipLaunchKernelGGL((k_rs_scatter<K, F, I, L, false>), dim3(nblocks), dim3(Tile<K>::THREADS), 0, st, kfrom, \
					 vin, n, shift, offs.as<uint32_t>(), nblocks, kout, vout, f2, tk, sts, gd, er, \
					 SegTiles{}, sort_xg((int) sizeof(K)), znx, kx)
		if (lb) {
			if (fin) {
				if (idv) SCAT(true, true, true); else SCAT(true, false, true);
			} else {
				if (idv) SCAT(false, true, true); else SCAT(false, false, true);
			}
		} else {
			if (fin) {
				if (idv) SCAT(true, true, false); else SCAT(true, false, false);
			} else {
				if (idv) SCAT(false, true, false); else SCAT(false, false, false);
			}
		}
#undef SCAT
		std::swap(kin, kout);
		std::swap(vin, vout);
	}
	if (fo != nullptr && shifts.empty()) {
		FinalOut f2 = *fo;
		f2.keys = nullptr;            // keys already in order (kin)
		hipLaunchKernelGGL((k_final_copy<K>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, kin,
				   positions ? nullptr : vin, n, f2);
	}
	uint32_t *he = (uint32_t *) pinned(16);
	if (lb && !hip_ok(hipMemcpyAsync(he, lb_err, 4, hipMemcpyDeviceToHost, st), "memcpy"))
		return -1;
	if (!sync())
		return -1;
	if (lb) {
		if (he[0]) {
			seterr("HY013!BATsort: radix look-back did not complete");
			return -1;
		}
	}
	*keys_out = kin;
	*vals_out = positions && shifts.empty() ? nullptr : vin;   // NULL: identity
	return 0;
}

template <typename T>
void
launch_gather(const mgdk_bat *b, const oid *order, void *sorted)
{
	hipLaunchKernelGGL((k_gather_sorted<T>), dim3(grid_for(b->count, 1024, 8192)), dim3(256), 0, stream(),
			   (const T *) b->theap, order, b->count, b->hseqbase, (T *) sorted);
}

// sort b's keys of type T with key width K into sn / on / gn (any may be NULL)
template <typename T, typename K>
int
sort_typed(const mgdk_bat *b, bool reverse, bool nilslast, mgdk_bat *sn, mgdk_bat *on, mgdk_bat *gn)
{
	const BUN n = b->count;
	constexpr bool is_float = (T) 0.5 != 0;
	hipStream_t st = stream();
	DevBuf k0(n * sizeof(K) + 8), k1(n * sizeof(K) + 8), v0(n * 4 + 4), v1(n * 4 + 4), otmp(on ? 8 : n * 8 + 8);
	if (!k0.p || !k1.p || !v0.p || !v1.p || !otmp.p)
		return -1;
	unsigned long long *ao = (unsigned long long *) meta_buf();
	unsigned long long init[2] = {~0ull, 0ull};
	if (!hip_ok(hipMemcpyAsync(ao, init, 16, hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	DevBuf dh(8 * 256 * 4);
	if (!dh.p || !hip_ok(hipMemsetAsync(dh.p, 0, 8 * 256 * 4, st), "memset"))
		return -1;
	// 4-byte signed integers whose image is a plain XOR (no nil, or nils
	// where their natural image puts them): the key-image pass only counts
	// digits, and the first radix pass reads the column itself
	constexpr bool sint4 = sizeof(T) == 4 && sizeof(K) == 4 && !is_float && (T) -1 < (T) 0;
	static const bool direct_on = !getenv("MGDK_SORT_DIRECT") || atoi(getenv("MGDK_SORT_DIRECT")) != 0;
	const bool direct = sint4 && direct_on && (reverse == nilslast || b->tnonil) && ((uintptr_t) b->theap & 3) == 0;
	const K kx0 = (K) (reverse ? 0x7fffffffu : 0x80000000u);
	hipLaunchKernelGGL((k_keys<T, K>), dim3(grid_for(n, 8192, 1024)), dim3(256), 0, st, (const T *) b->theap, n,
			   reverse, nilslast, direct ? (K *) nullptr : k0.as<K>(), ao, dh.as<uint32_t>());
	FinalOut fo{};
	fo.vw = b->twidth;
	fo.reverse = reverse;
	fo.is64 = sizeof(K) == 8;
	fo.uns = basetype(b->ttype) == MGDK_oid;
	fo.hseq = b->hseqbase;
	// floats (and reverse != nilslast images) are not decodable: gather by order
	const bool decodable = !is_float && reverse == nilslast;
	fo.sorted = decodable && sn ? sn->theap : nullptr;
	// groups: from the decoded sorted values when those are written (equal
	// values <=> equal images), so the last pass writes no key images
	const bool gid_vals = gn != nullptr && fo.sorted != nullptr;
	fo.want_keys = gn != nullptr && !gid_vals;
	fo.order = on ? (oid *) on->theap : otmp.as<oid>();
	// the MSD-then-local path may write the group ids with the rows
	bool gid_done = false;
	uint64_t gid_last = 0;
	fo.gid = gn ? (oid *) gn->theap : nullptr;
	fo.gid_done = &gid_done;
	fo.gid_last = &gid_last;
	K *ks;
	uint32_t *vs;
	if (radix_sort<K>(k0.as<K>(), v0.as<uint32_t>(), k1.as<K>(), v1.as<uint32_t>(), n, 8 * (int) sizeof(K), &fo,
			  true, true, &ks, &vs, dh.as<uint32_t>(), direct ? (const K *) b->theap : nullptr,
			  direct ? kx0 : (K) 0) < 0)
		return -1;
	if (sn && !decodable) {
		switch (b->twidth) {
		case 1: launch_gather<int8_t>(b, fo.order, sn->theap); break;
		case 2: launch_gather<int16_t>(b, fo.order, sn->theap); break;
		case 4: launch_gather<int32_t>(b, fo.order, sn->theap); break;
		default: launch_gather<int64_t>(b, fo.order, sn->theap); break;
		}
	}
	if (gn) {
		// groups: a new group wherever the sorted key image changes
		const BUN nt = (n + GTILE - 1) / GTILE;
		// the scan's total and error flag are read with the final sync (no
		// round trip between the count and the write pass)
		DevBuf cnt(nt * 4 + 4), pre(nt * 8 + 8), sws(scan_ws_words(nt) * 8);
		uint64_t tot = 0;
		bool tot_dev = false;
		if (!cnt.p || !pre.p || !sws.p)
			return -1;
		if (gid_done) {
			tot = gid_last;
		} else if (nt > 0) {
			auto gids = [&](auto *src) {
				using KT = std::remove_const_t<std::remove_pointer_t<decltype(src)>>;
				if (MGDK_SORT_GIDV && n >= (BUN) GTILE && ((uintptr_t) src & 15) == 0)
					hipLaunchKernelGGL((k_gid_count_v<KT>), dim3((unsigned) nt), dim3(256), 0, st, src, n,
							   cnt.as<uint32_t>());
				else
					hipLaunchKernelGGL((k_gid_count<KT>), dim3((unsigned) nt), dim3(256), 0, st, src, n,
							   cnt.as<uint32_t>());
				if (exclusive_scan_nosync(cnt.as<uint32_t>(), pre.as<uint64_t>(), nt, sws.as<uint64_t>()) < 0)
					return -1;
				tot_dev = true;
				hipLaunchKernelGGL((k_gid_write<KT>), dim3((unsigned) nt), dim3(256), 0, st, src, n,
						   pre.as<uint64_t>(), (oid *) gn->theap);
				return 0;
			};
			int rc;
			if constexpr (!is_float)
				rc = gid_vals ? gids((const T *) sn->theap) : gids((const K *) ks);
			else
				rc = gids((const K *) ks);
			if (rc < 0)
				return -1;
		}
		uint64_t *ht = (uint64_t *) pinned(16);
		if (tot_dev && !hip_ok(hipMemcpyAsync(ht, sws.as<uint64_t>() + 2, 16, hipMemcpyDeviceToHost, st), "memcpy"))
			return (void) sync(), -1;
		if (!sync())
			return -1;
		if (tot_dev) {
			if ((uint32_t) ht[1]) {
				seterr("HY013!scan: look-back did not complete");
				return -1;
			}
			tot = ht[0];
		}
		gn->count = n;
		gn->tsorted = 1;
		gn->trevsorted = tot == 0;
		gn->tkey = tot + 1 == n || n <= 1;
		gn->tnonil = 1;
	}
	return sync() ? 0 : -1;
}

__global__ __launch_bounds__(256) void
k_fill_ones(uint8_t *f, BUN n)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		f[i] = i > 0;
}

// ---- sub-sorting: BATsort with o (pre-order) and / or g (groups) ---------
// (gdk/gdk_batop.c:2305-2340): b is first rearranged by o, then every run
// of equal g is sorted.  g is sorted ascending, so "sort within runs" is a
// stable sort on the composite (g, key image): LSD -- first by key image,
// then (stably) by group id -- and the result oids are o[perm].

template <typename T, typename K>
__global__ __launch_bounds__(256) void
k_subkeys(const T *col, const oid *o, oid oseq, oid hseq, BUN n, bool reverse, bool nilslast, K *keys)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		keys[i] = keyimg<T, K>(col[(o ? o[i] : oseq + i) - hseq], reverse, nilslast);
}

__global__ __launch_bounds__(256) void
k_gather_gid(const oid *g, oid gseq, const uint32_t *perm, BUN n, uint64_t *out, uint32_t *idx)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint32_t p = perm ? perm[i] : (uint32_t) i;
		out[i] = g ? g[p] : gseq + p;
		idx[i] = p;
	}
}

template <typename T, typename K>
__global__ __launch_bounds__(256) void
k_final_sub(const T *col, const oid *o, oid oseq, oid hseq, const oid *g, oid gseq, const uint32_t *perm, BUN n,
	    bool reverse, bool nilslast, T *sorted, oid *order, uint8_t *flag)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint32_t p = perm ? perm[i] : (uint32_t) i;
		const oid src = o ? o[p] : oseq + p;
		if (order)
			order[i] = src;
		if (sorted)
			sorted[i] = col[src - hseq];
		if (flag) {
			bool nw = i > 0;
			if (nw) {
				const uint32_t q = perm ? perm[i - 1] : (uint32_t) (i - 1);
				const oid sq = o ? o[q] : oseq + q;
				nw = (g && g[p] != g[q]) || keyimg<T, K>(col[src - hseq], reverse, nilslast) !=
								    keyimg<T, K>(col[sq - hseq], reverse, nilslast);
			}
			flag[i] = nw;
		}
	}
}

template <typename T, typename K>
int
sort_sub(const mgdk_bat *b, const mgdk_bat *o, const mgdk_bat *g, bool reverse, bool nilslast, mgdk_bat *sn,
	 mgdk_bat *on, mgdk_bat *gn)
{
	const BUN n = b->count;
	hipStream_t st = stream();
	const oid *op = o && o->ttype != MGDK_void ? (const oid *) o->theap : nullptr;
	const oid oseq = o ? (o->ttype == MGDK_void ? o->tseqbase : 0) : b->hseqbase;
	// g given as a dense (void) column means every row is its own group:
	// nothing to sort inside the groups
	const bool gdense = g && g->ttype == MGDK_void;
	const oid *gp = g && !gdense ? (const oid *) g->theap : nullptr;
	DevBuf k0(n * sizeof(K) + 8), k1(n * sizeof(K) + 8), v0(n * 4 + 4), v1(n * 4 + 4);
	DevBuf g0(n * 8 + 8), g1(n * 8 + 8), w0(n * 4 + 4), w1(n * 4 + 4), fl(n + 8), ex(n * 8 + 8);
	if (!k0.p || !k1.p || !v0.p || !v1.p || !g0.p || !g1.p || !w0.p || !w1.p || !fl.p || !ex.p)
		return -1;
	const dim3 grd(grid_for(n, 1024, 8192)), blk(256);
	uint32_t *perm = nullptr;
	if (!gdense) {
		hipLaunchKernelGGL((k_subkeys<T, K>), grd, blk, 0, st, (const T *) b->theap, op, oseq, b->hseqbase, n, reverse,
				   nilslast, k0.as<K>());
		K *ks;
		if (radix_sort<K>(k0.as<K>(), v0.as<uint32_t>(), k1.as<K>(), v1.as<uint32_t>(), n, 8 * (int) sizeof(K),
				  nullptr, true, false, &ks, &perm) < 0)
			return -1;
		if (g) {
			hipLaunchKernelGGL(k_gather_gid, grd, blk, 0, st, gp, g->tseqbase, perm, n, g0.as<uint64_t>(),
					   w0.as<uint32_t>());
			uint64_t *gs;
			if (radix_sort<uint64_t>(g0.as<uint64_t>(), w0.as<uint32_t>(), g1.as<uint64_t>(), w1.as<uint32_t>(), n,
						 64, nullptr, false, false, &gs, &perm) < 0)
				return -1;
		}
	}
	hipLaunchKernelGGL((k_final_sub<T, K>), grd, blk, 0, st, (const T *) b->theap, op, oseq, b->hseqbase,
			   gdense ? nullptr : gp, g ? g->tseqbase : 0, perm, n, reverse, nilslast,
			   sn ? (T *) sn->theap : nullptr, on ? (oid *) on->theap : nullptr,
			   gn ? fl.as<uint8_t>() : nullptr);
	if (gn) {
		uint64_t tot = 0;
		if (gdense) {
			hipLaunchKernelGGL(k_fill_ones, grd, blk, 0, st, fl.as<uint8_t>(), n);
		}
		if (exclusive_scan(fl.as<uint8_t>(), ex.as<uint64_t>(), n, &tot) < 0)
			return -1;
		hipLaunchKernelGGL(k_gid, grd, blk, 0, st, ex.as<uint64_t>(), fl.as<uint8_t>(), n, (oid *) gn->theap);
		if (!sync())
			return -1;
		gn->count = n;
		gn->tsorted = 1;
		gn->trevsorted = tot == 0;
		gn->tkey = tot + 1 == n || n <= 1;
		gn->tnonil = 1;
	}
	return sync() ? 0 : -1;
}


// ---- small inputs (n <= 1024): one workgroup, one kernel ------------------
// every row's rank in the stable order of (group, key image, position) by
// counting in LDS, then the outputs and the group ids (a workgroup scan of
// the new-group flags).  Replaces the radix machinery's dozen launches and
// round trips when a plan sorts a handful of rows (e.g. Q1's ORDER BY).
constexpr BUN SMALL_SORT = 1024;

template <typename T>
__global__ __launch_bounds__(1024) void
k_small_sort(const T *col, const oid *o, oid oseq, oid hseq, const oid *g, oid gseq, bool hasg, uint32_t n,
	     bool reverse, bool nilslast, T *sorted, oid *order, oid *gid, uint32_t *ngrp)
{
	__shared__ uint64_t sk[SMALL_SORT], sg[SMALL_SORT];
	__shared__ uint32_t sidx[SMALL_SORT], wsum[16];
	const uint32_t i = threadIdx.x, lane = __lane_id(), w = i >> 6;
	if (i < n) {
		const oid src = o ? o[i] : oseq + i;
		sk[i] = keyimg<T, uint64_t>(col[src - hseq], reverse, nilslast);
		sg[i] = hasg ? (g ? g[i] : gseq + i) : 0;
	}
	__syncthreads();
	if (i < n) {
		const uint64_t ki = sk[i], gi = sg[i];
		uint32_t r = 0;
		for (uint32_t j = 0; j < n; j++) {
			const uint64_t kj = sk[j], gj = sg[j];
			r += gj < gi || (gj == gi && (kj < ki || (kj == ki && j < i)));
		}
		sidx[r] = i;
	}
	__syncthreads();
	uint32_t f = 0;
	if (i < n) {
		const uint32_t q = sidx[i];
		const oid src = o ? o[q] : oseq + q;
		if (order)
			order[i] = src;
		if (sorted)
			sorted[i] = col[src - hseq];
		if (i > 0) {
			const uint32_t q0 = sidx[i - 1];
			f = sg[q] != sg[q0] || sk[q] != sk[q0];
		}
	}
	// inclusive scan of the flags: group id of position i
	uint32_t x = f;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint32_t u = __shfl_up(x, d);
		if (lane >= (unsigned) d)
			x += u;
	}
	if (lane == 63)
		wsum[w] = x;
	__syncthreads();
	uint32_t pre = 0;
	for (uint32_t q = 0; q < w; q++)
		pre += wsum[q];
	if (i < n && gid)
		gid[i] = pre + x;
	if (i == n - 1)
		*ngrp = pre + x;
}

template <typename T>
int
sort_small(const mgdk_bat *b, const mgdk_bat *o, const mgdk_bat *g, bool reverse, bool nilslast, mgdk_bat *sn,
	   mgdk_bat *on, mgdk_bat *gn)
{
	const BUN n = b->count;
	hipStream_t st = stream();
	const oid *op = o && o->ttype != MGDK_void ? (const oid *) o->theap : nullptr;
	const oid oseq = o ? (o->ttype == MGDK_void ? o->tseqbase : 0) : b->hseqbase;
	const oid *gp = g && g->ttype != MGDK_void ? (const oid *) g->theap : nullptr;
	uint32_t *m = (uint32_t *) meta_buf(), *h = (uint32_t *) pinned(64);
	if (!hip_ok(hipMemsetAsync(m, 0, 4, st), "memset"))
		return -1;
	if (n)
		hipLaunchKernelGGL((k_small_sort<T>), dim3(1), dim3(1024), 0, st, (const T *) b->theap, op, oseq, b->hseqbase,
				   gp, g ? g->tseqbase : 0, g != nullptr, (uint32_t) n, reverse, nilslast,
				   sn ? (T *) sn->theap : nullptr, on ? (oid *) on->theap : nullptr,
				   gn ? (oid *) gn->theap : nullptr, m);
	if (!hip_ok(hipMemcpyAsync(h, m, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	if (gn) {
		const uint64_t tot = h[0];
		gn->count = n;
		gn->tsorted = 1;
		gn->trevsorted = tot == 0;
		gn->tkey = tot + 1 == n || n <= 1;
		gn->tnonil = 1;
	}
	return 0;
}

// ---- str columns (strCmp, gdk_atoms.h:414: nil first, then strcmp order) ----
// A string sorts as a sequence of 64-bit chunk keys: chunk k holds its bytes
// [7k, 7k + 7) big-endian (0 after the terminator) under a 0x01 tag byte, so
// every non-nil key is positive and compares like strcmp's unsigned bytes;
// the nil string gets lng nil, so the lng sort places it exactly as the
// reference places nil.  Chunk 0 is sorted, each further chunk sub-sorts the
// groups of equal prefixes.
__device__ __forceinline__ const uint8_t *
str_at(const void *offs, int w, const char *vh, BUN i)
{
	size_t o;
	switch (w) {
	case 1: o = (size_t) ((const uint8_t *) offs)[i] + 8192; break;
	case 2: o = (size_t) ((const uint16_t *) offs)[i] + 8192; break;
	case 4: o = (size_t) ((const uint32_t *) offs)[i]; break;
	default: o = (size_t) ((const uint64_t *) offs)[i]; break;
	}
	return (const uint8_t *) vh + o;
}

__device__ __forceinline__ bool
str_isnil(const uint8_t *s)
{
	return s[0] == 0x80 && s[1] == 0;
}

__global__ __launch_bounds__(256) void
k_str_maxlen(const void *offs, int w, const char *vh, BUN n, unsigned long long *maxlen)
{
	unsigned long long m = 0;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
		const uint8_t *p = str_at(offs, w, vh, i);
		if (str_isnil(p))
			continue;
		unsigned long long l = 0;
		while (p[l])
			l++;
		m = l > m ? l : m;
	}
	m = block_reduce(m, [](unsigned long long a, unsigned long long b) { return a > b ? a : b; });
	if (threadIdx.x == 0 && m)
		atomicMax(maxlen, m);
}

__global__ __launch_bounds__(256) void
k_str_chunk(const void *offs, int w, const char *vh, BUN n, int k, int64_t *key)
{
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
		const uint8_t *p = str_at(offs, w, vh, i);
		if (str_isnil(p)) {
			key[i] = INT64_MIN;
			continue;
		}
		int j = 0;
		while (j < 7 * k && p[j])
			j++;
		uint64_t v = 1;
		bool end = j < 7 * k;
		for (int q = 0; q < 7; q++) {
			const uint8_t c = end ? 0 : p[j + q];
			end |= c == 0;
			v = (v << 8) | c;
		}
		key[i] = (int64_t) v;
	}
}

}  // namespace

namespace mgdk {

int
radix_sort_pairs(uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt, BUN n, int bits,
		 uint64_t **keys_out, uint32_t **vals_out)
{
	return radix_sort<uint64_t>(keys, vals, keys_alt, vals_alt, n, bits, nullptr, false, false, keys_out,
				    vals_out);
}

// stable counting sort of positions 0..n-1 by 32-bit keys (e.g. a
// destination rank); *perm receives the buffer holding the permutation
int
radix_sort_positions32(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt, BUN n, int bits,
		       uint32_t **perm)
{
	uint32_t *ko;
	if (radix_sort<uint32_t>(keys, vals, keys_alt, vals_alt, n, bits, nullptr, true, false, &ko, perm) < 0)
		return -1;
	return 0;
}

thread_local int sort_internal = 0;

}  // namespace mgdk

static int sort_core(mgdk_bat **sorted, mgdk_bat **order, mgdk_bat **groups, mgdk_bat *b, mgdk_bat *o,
		     mgdk_bat *g, bool reverse, bool nilslast);

// stable BATsort of a str column through its chunk keys (see k_str_chunk):
// each chunk sub-sorts the runs of equal prefixes stably
static int
sort_str(mgdk_bat **sorted, mgdk_bat **order, mgdk_bat **groups, mgdk_bat *b, mgdk_bat *o, mgdk_bat *g,
	 bool reverse, bool nilslast)
{
	const BUN n = b->count;
	hipStream_t st = stream();
	unsigned long long *m = (unsigned long long *) meta_buf(), *h = (unsigned long long *) pinned(64);
	if (!hip_ok(hipMemsetAsync(m, 0, 8, st), "memset"))
		return -1;
	if (n)
		hipLaunchKernelGGL(k_str_maxlen, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, (const void *) b->theap, (int) b->twidth,
				   (const char *) b->tvheap, n, m);
	if (!hip_ok(hipMemcpyAsync(h, m, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	const int nch = h[0] > 7 ? (int) ((h[0] + 6) / 7) : 1;
	mgdk_bat *co = o, *cg = g, *on = nullptr, *gn = nullptr;
	int rc = 0;
	for (int k = 0; k < nch && rc == 0; k++) {
		mgdk_bat *key = newbat(b->hseqbase, MGDK_lng, n);
		if (!key) {
			rc = -1;
			break;
		}
		if (n)
			hipLaunchKernelGGL(k_str_chunk, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, (const void *) b->theap,
					   (int) b->twidth, (const char *) b->tvheap, n, k, (int64_t *) key->theap);
		key->count = n;
		key->tsorted = key->trevsorted = n <= 1;
		key->tkey = n <= 1;
		key->tnonil = b->tnonil;
		key->tnil = b->tnil;
		const bool wantg = k + 1 < nch || groups != nullptr;
		on = gn = nullptr;
		rc = sort_core(nullptr, &on, wantg ? &gn : nullptr, key, co, cg, reverse, nilslast);
		mgdk_BBPunfix(key);
		if (co != o)
			mgdk_BBPunfix(co);
		if (cg != g)
			mgdk_BBPunfix(cg);
		co = on;
		cg = gn;
	}
	if (rc != 0) {
		if (co != o)
			mgdk_BBPunfix(co);
		if (cg != g)
			mgdk_BBPunfix(cg);
		return -1;
	}
	mgdk_bat *sn = nullptr;
	if (sorted) {
		sn = mgdk_BATproject(co, b);
		if (!sn) {
			mgdk_BBPunfix(co);
			mgdk_BBPunfix(cg);
			return -1;
		}
		sn->tsorted = (g == nullptr && !reverse) || n <= 1;
		sn->trevsorted = (g == nullptr && reverse) || n <= 1;
		sn->tkey = b->tkey;
		sn->tnonil = b->tnonil;
		sn->tnil = b->tnil;
		*sorted = sn;
	}
	if (order) *order = co; else mgdk_BBPunfix(co);
	if (groups) *groups = cg; else mgdk_BBPunfix(cg);
	return 0;
}

// the stable sort: sorted values, order oids and group ids of b rearranged
// by o and sorted within the runs of g (ties in input order)
static int
sort_core(mgdk_bat **sorted, mgdk_bat **order, mgdk_bat **groups, mgdk_bat *b, mgdk_bat *o, mgdk_bat *g,
	  bool reverse, bool nilslast)
{
	if (b->ttype == MGDK_str) {
		ProfScope prof("sort");
		return sort_str(sorted, order, groups, b, o, g, reverse, nilslast);
	}
	const int tt = basetype(b->ttype);
	if (!(tt == MGDK_bte || tt == MGDK_sht || tt == MGDK_int || tt == MGDK_lng || tt == MGDK_oid ||
	      tt == MGDK_flt || tt == MGDK_dbl || tt == MGDK_void)) {
		seterr("42000!BATsort: type %s not supported on the device path", atomname(b->ttype));
		return -1;
	}
	const BUN n = b->count;
	if (n >= ((BUN) 1 << 32)) {
		seterr("42000!BATsort: more than 2^32 rows");
		return -1;
	}
	ProfScope prof("sort");
	mgdk_bat *sn = nullptr, *on = nullptr, *gn = nullptr;
	if (n <= SMALL_SORT && tt != MGDK_void) {
		sn = sorted ? newbat(b->hseqbase, b->ttype, n) : nullptr;
		on = order ? newbat(b->hseqbase, MGDK_oid, n) : nullptr;
		gn = groups ? newbat(b->hseqbase, MGDK_oid, n) : nullptr;
		if ((sorted && !sn) || (order && !on) || (groups && !gn))
			goto fail;
		int rc = 0;
#define SMALL(T) rc = sort_small<T>(b, o, g, reverse, nilslast, sn, on, gn)
		switch (tt) {
		case MGDK_bte: SMALL(int8_t); break;
		case MGDK_sht: SMALL(int16_t); break;
		case MGDK_int: SMALL(int32_t); break;
		case MGDK_flt: SMALL(float); break;
		case MGDK_lng: SMALL(int64_t); break;
		case MGDK_oid: SMALL(uint64_t); break;
		case MGDK_dbl: SMALL(double); break;
		}
#undef SMALL
		if (rc < 0)
			goto fail;
		if (sn) {
			sn->count = n;
			sn->tsorted = (g == nullptr && !reverse) || n <= 1;
			sn->trevsorted = (g == nullptr && reverse) || n <= 1;
			sn->tkey = b->tkey;
			sn->tnonil = b->tnonil;
			sn->tnil = b->tnil;
		}
		if (on) {
			on->count = n;
			on->tkey = 1;
			on->tnonil = 1;
			on->tsorted = on->trevsorted = 0;   // gdk_batop.c:2622-2624
		}
		goto done;
	}
	if (o != nullptr || g != nullptr) {
		if (tt == MGDK_void) {
			seterr("42000!BATsort: sub-sorting a void column is not supported on the device path");
			return -1;
		}
		sn = sorted ? newbat(b->hseqbase, b->ttype, n) : nullptr;
		on = order ? newbat(b->hseqbase, MGDK_oid, n) : nullptr;
		gn = groups ? newbat(b->hseqbase, MGDK_oid, n) : nullptr;
		if ((sorted && !sn) || (order && !on) || (groups && !gn))
			goto fail;
		const bool k32 = b->twidth <= 4 && reverse == nilslast;
		int rc = 0;
#define SUB(T, K) rc = sort_sub<T, K>(b, o, g, reverse, nilslast, sn, on, gn)
		switch (tt) {
		case MGDK_bte: if (k32) SUB(int8_t, uint32_t); else SUB(int8_t, uint64_t); break;
		case MGDK_sht: if (k32) SUB(int16_t, uint32_t); else SUB(int16_t, uint64_t); break;
		case MGDK_int: if (k32) SUB(int32_t, uint32_t); else SUB(int32_t, uint64_t); break;
		case MGDK_flt: if (k32) SUB(float, uint32_t); else SUB(float, uint64_t); break;
		case MGDK_lng: SUB(int64_t, uint64_t); break;
		case MGDK_oid: SUB(uint64_t, uint64_t); break;
		case MGDK_dbl: SUB(double, uint64_t); break;
		}
#undef SUB
		if (rc < 0)
			goto fail;
		if (sn) {
			sn->count = n;
			sn->tsorted = (g == nullptr && !reverse) || n <= 1;
			sn->trevsorted = (g == nullptr && reverse) || n <= 1;
			sn->tkey = b->tkey;
			sn->tnonil = b->tnonil;
			sn->tnil = b->tnil;
			if (b->ttype == MGDK_str)
				share_vheap(sn, b);
		}
		if (on) {
			on->count = n;
			on->tkey = 1;
			on->tnonil = 1;
			on->tsorted = on->trevsorted = 0;   // gdk_batop.c:2622-2624
		}
		goto done;
	}
	if (tt == MGDK_void) {
		// dense column: sorted already (gdk_batop.c:2384-2392)
		sn = mgdk_BATslice(b, 0, n);
		on = mgdk_BATdense(b->hseqbase, b->hseqbase, n);
		if (groups)
			gn = mgdk_BATdense(b->hseqbase, 0, n);
		if (!sn || !on || (groups && !gn))
			goto fail;
		goto done;
	}
	{
		sn = sorted ? newbat(b->hseqbase, b->ttype, n) : nullptr;
		on = order ? newbat(b->hseqbase, MGDK_oid, n) : nullptr;
		if ((sorted && !sn) || (order && !on))
			goto fail;
		// 32-bit key images need nil at its natural end (nilslast == reverse)
		const bool k32 = b->twidth <= 4 && reverse == nilslast;
		gn = groups ? newbat(b->hseqbase, MGDK_oid, n) : nullptr;
		if (groups && !gn)
			goto fail;
		int rc = 0;
#define SORT(T, K) rc = sort_typed<T, K>(b, reverse, nilslast, sn, on, gn)
		switch (tt) {
		case MGDK_bte: if (k32) SORT(int8_t, uint32_t); else SORT(int8_t, uint64_t); break;
		case MGDK_sht: if (k32) SORT(int16_t, uint32_t); else SORT(int16_t, uint64_t); break;
		case MGDK_int: if (k32) SORT(int32_t, uint32_t); else SORT(int32_t, uint64_t); break;
		case MGDK_flt: if (k32) SORT(float, uint32_t); else SORT(float, uint64_t); break;
		case MGDK_lng: SORT(int64_t, uint64_t); break;
		case MGDK_oid: SORT(uint64_t, uint64_t); break;
		case MGDK_dbl: SORT(double, uint64_t); break;
		}
#undef SORT
		if (rc < 0)
			goto fail;
		if (sn) {
			sn->count = n;
			sn->tsorted = !reverse || n <= 1;
			sn->trevsorted = reverse || n <= 1;
			sn->tkey = b->tkey;
			sn->tnonil = b->tnonil;
			sn->tnil = b->tnil;
			if (b->ttype == MGDK_str)
				share_vheap(sn, b);
		}
		if (on) {
			on->count = n;
			on->tkey = 1;
			on->tnonil = 1;
			on->tsorted = on->trevsorted = 0;   // gdk_batop.c:2622-2624
		}
	}
done:
	if (sorted) *sorted = sn; else mgdk_BBPunfix(sn);
	if (order) *order = on; else mgdk_BBPunfix(on);
	if (groups) *groups = gn; else mgdk_BBPunfix(gn);
	return 0;
fail:
	mgdk_BBPunfix(sn);
	mgdk_BBPunfix(on);
	mgdk_BBPunfix(gn);
	return -1;
}

// ---- BATsort (gdk/gdk_batop.c:2342-2827): the reference's control flow ----
// around the stable engine above, and GDKqsort's order of equal values
// (qsort.hip) wherever do_sort (gdk_batop.c:2266-2304) picks the quicksort:
// an unstable sort of a type the radix sort does not take (bit, oid, flt,
// dbl, str), of nils at the unnatural end (reverse != nilslast), or of a run
// of at most 100 rows.
namespace {

struct OSrc {
	const oid *p;
	oid seq;
	__device__ __forceinline__ oid at(BUN i) const { return p ? p[i] : seq + i; }
};

OSrc
osrc(const mgdk_bat *b)
{
	return OSrc{b && b->ttype != MGDK_void ? (const oid *) b->theap : nullptr, b ? b->tseqbase : 0};
}

__global__ __launch_bounds__(256) void
k_qs_ranks(BUN n, OSrc order1, oid h0, OSrc grp1, uint32_t *rank)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		rank[order1.at(i) - h0] = (uint32_t) grp1.at(i);
}

__global__ __launch_bounds__(256) void
k_qs_pay(BUN n, OSrc o, bool has_o, oid hseq, uint64_t *pay)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		pay[i] = has_o ? o.at(i) : hseq + i;
}

__global__ __launch_bounds__(256) void
k_run_starts(BUN n, OSrc g, int8_t *fl)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		fl[i] = i == 0 || g.at(i) != g.at(i - 1);
}

__global__ __launch_bounds__(256) void
k_qs_mark_runs(const uint64_t *st, const uint32_t *len, uint32_t nseg, uint8_t *mark)
{
	const uint32_t k = blockIdx.x;
	if (k >= nseg)
		return;
	for (uint32_t i = threadIdx.x; i < len[k]; i += blockDim.x)
		mark[st[k] + i] = 1;
}

// order oids: the replayed payload in quicksort runs, the stable order
// (through o) elsewhere
__global__ __launch_bounds__(256) void
k_qs_order(BUN n, const uint8_t *mark, const uint64_t *pay, OSrc order1, oid h0, OSrc o, bool has_o, oid hseq,
	   oid *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		if (mark[i]) {
			out[i] = pay[i];
		} else {
			const oid p = order1.at(i) - h0;
			out[i] = has_o ? o.at(p) : hseq + p;
		}
	}
}

__global__ __launch_bounds__(256) void
k_seq_oids(BUN n, oid hseq, oid *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = hseq + i;
}

bool
radix_type(int tt)
{
	switch (tt) {
	case MGDK_bte: case MGDK_sht: case MGDK_int: case MGDK_lng: case MGDK_hge:
	case MGDK_date: case MGDK_daytime: case MGDK_timestamp:
		return true;
	default:
		return false;   // bit, oid, flt, dbl, str: GDKssort / GDKqsort
	}
}

// runs of equal consecutive g (the sub-sorts of gdk_batop.c:2687-2711) as
// (start, length); whole column without g
int
sort_runs(const mgdk_bat *g, BUN n, std::vector<std::pair<uint64_t, uint32_t>> &runs)
{
	runs.clear();
	if (n == 0)
		return 0;
	if (g == nullptr) {
		runs.emplace_back(0, (uint32_t) n);
		return 0;
	}
	DevBuf fl(n + 8);
	if (!fl.p)
		return -1;
	hipLaunchKernelGGL(k_run_starts, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, stream(), n, osrc(g),
			   fl.as<int8_t>());
	mgdk_bat *S = compact_flags(fl.as<int8_t>(), n, 0);
	if (S == nullptr)
		return -1;
	std::vector<oid> st(S->count);
	const int rc = mgdk_BATdownload(S, st.data());
	mgdk_BBPunfix(S);
	if (rc < 0)
		return -1;
	for (size_t k = 0; k < st.size(); k++)
		runs.emplace_back(st[k], (uint32_t) ((k + 1 < st.size() ? st[k + 1] : n) - st[k]));
	return 0;
}

// a materialised order column hseq, hseq + 1, ... (gdk_batop.c:2611-2620)
mgdk_bat *
seq_order(oid hseq, BUN n)
{
	mgdk_bat *on = newbat(hseq, MGDK_oid, n);
	if (on == nullptr)
		return nullptr;
	if (n)
		hipLaunchKernelGGL(k_seq_oids, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, stream(), n, hseq,
				   (oid *) on->theap);
	if (!sync()) {
		mgdk_BBPunfix(on);
		return nullptr;
	}
	on->count = n;
	on->tkey = on->tnonil = 1;
	on->tsorted = 1;
	on->trevsorted = n <= 1;
	return on;
}

// GDKqsort's order for the quicksort runs: stable-sort b (rearranged by o)
// for the ranks, replay the quicksort on those runs, keep the stable order
// in the others
int
sort_qsort(mgdk_bat **order, mgdk_bat **groups, mgdk_bat *b, mgdk_bat *o, mgdk_bat *g, bool reverse,
	   bool nilslast, const std::vector<std::pair<uint64_t, uint32_t>> &qruns)
{
	const BUN n = b->count;
	hipStream_t st = stream();
	mgdk_bat *bn = o ? mgdk_BATproject(o, b) : b;
	if (bn == nullptr)
		return -1;
	mgdk_bat *o1 = nullptr, *g1 = nullptr, *on = nullptr;
	int rc = -1;
	{
		if (sort_core(nullptr, &o1, &g1, bn, nullptr, g, reverse, nilslast) < 0)
			goto out;
		DevBuf rank(n * 4 + 4), pay(n * 8 + 8), mark(n + 8);
		if (!rank.p || !pay.p || !mark.p)
			goto out;
		const dim3 grd(grid_for(n, 1024, 8192)), blk(256);
		hipLaunchKernelGGL(k_qs_ranks, grd, blk, 0, st, n, osrc(o1), bn->hseqbase, osrc(g1), rank.as<uint32_t>());
		hipLaunchKernelGGL(k_qs_pay, grd, blk, 0, st, n, osrc(o), o != nullptr, b->hseqbase, pay.as<uint64_t>());
		if (qsort_replay(rank.as<uint32_t>(), pay.as<uint64_t>(), n, qruns) < 0)
			goto out;
		// mark the replayed runs
		if (!hip_ok(hipMemsetAsync(mark.p, 0, n, st), "memset"))
			goto out;
		if (!qruns.empty()) {
			std::vector<uint64_t> hs(qruns.size());
			std::vector<uint32_t> hl(qruns.size());
			for (size_t k = 0; k < qruns.size(); k++) {
				hs[k] = qruns[k].first;
				hl[k] = qruns[k].second;
			}
			DevBuf ds(hs.size() * 8), dl(hl.size() * 4);
			if (!ds.p || !dl.p ||
			    !hip_ok(hipMemcpyAsync(ds.p, hs.data(), hs.size() * 8, hipMemcpyHostToDevice, st), "memcpy") ||
			    !hip_ok(hipMemcpyAsync(dl.p, hl.data(), hl.size() * 4, hipMemcpyHostToDevice, st), "memcpy"))
				goto out;
			hipLaunchKernelGGL(k_qs_mark_runs, dim3((unsigned) qruns.size()), dim3(256), 0, st, ds.as<uint64_t>(),
					   dl.as<uint32_t>(), (uint32_t) qruns.size(), mark.as<uint8_t>());
			if (!sync())
				goto out;
		}
		on = newbat(b->hseqbase, MGDK_oid, n);
		if (on == nullptr)
			goto out;
		hipLaunchKernelGGL(k_qs_order, grd, blk, 0, st, n, mark.as<uint8_t>(), pay.as<uint64_t>(), osrc(o1),
				   bn->hseqbase, osrc(o), o != nullptr, b->hseqbase, (oid *) on->theap);
		if (!sync())
			goto out;
		on->count = n;
		on->tkey = o ? o->tkey : 1;
		on->tnonil = 1;
		on->tsorted = on->trevsorted = 0;
		*order = on;
		on = nullptr;
		if (groups) {
			*groups = g1;
			g1 = nullptr;
		}
		rc = 0;
	}
out:
	if (bn != b)
		mgdk_BBPunfix(bn);
	mgdk_BBPunfix(o1);
	mgdk_BBPunfix(g1);
	mgdk_BBPunfix(on);
	return rc;
}

// BATsort through an order index (gdk_batop.c:2510-2568): the order is the
// index (its heap shared, where the reference copies it), the sorted column
// its projection, the groups those of the sorted column
int
sort_by_oidx(mgdk_bat **sn, mgdk_bat **on, mgdk_bat **gn, mgdk_bat *b, Heap *oh, size_t ooff, bool want_sorted)
{
	mgdk_bat *o = oidx_bat(oh, ooff, b->hseqbase, b->count);
	o->tsorted = o->trevsorted = 0;
	*on = o;
	if (want_sorted || gn) {
		mgdk_bat *s = mgdk_BATproject(o, b);
		if (s == nullptr)
			return -1;
		s->tsorted = 1;
		*sn = s;
		if (gn) {
			if (mgdk_BATgroup(gn, nullptr, nullptr, s, nullptr, nullptr, nullptr, nullptr) < 0)
				return -1;
			if (want_sorted && (*gn)->tkey)
				s->tkey = 1;
		}
		if (!want_sorted) {
			mgdk_BBPunfix(s);
			*sn = nullptr;
		}
	}
	return 0;
}

}  // namespace

extern "C" int
mgdk_BATsort(mgdk_bat **sorted, mgdk_bat **order, mgdk_bat **groups, mgdk_bat *b, mgdk_bat *o, mgdk_bat *g,
	     bool reverse, bool nilslast, bool stable)
{
	if (sorted) *sorted = nullptr;
	if (order) *order = nullptr;
	if (groups) *groups = nullptr;
	if (b == nullptr) {
		seterr("b must exist\n");
		return -1;
	}
	if (stable && reverse != nilslast) {
		seterr("stable sort cannot have reverse != nilslast\n");
		return -1;
	}
	const BUN n = b->count;
	if (b->ttype == MGDK_void) {
		b->tsorted = 1;
		b->trevsorted = b->tseqbase == MGDK_OID_NIL || n <= 1;
		b->tkey = b->tseqbase != MGDK_OID_NIL || n <= 1;
	} else if (n <= 1) {
		b->tsorted = b->trevsorted = 1;
	}
	if (o != nullptr && ((basetype(o->ttype) != MGDK_oid && o->ttype != MGDK_void) || o->count != n ||
			     (o->ttype == MGDK_void && o->count && o->tseqbase == MGDK_OID_NIL))) {
		seterr("o must have type oid and same size as b\n");
		return -1;
	}
	if (g != nullptr && ((basetype(g->ttype) != MGDK_oid && g->ttype != MGDK_void) || !g->tsorted ||
			     g->count != n || (g->ttype == MGDK_void && g->count && g->tseqbase == MGDK_OID_NIL))) {
		seterr("g must have type oid, sorted on the tail, and same size as b\n");
		return -1;
	}
	if (sorted == nullptr && order == nullptr) {
		seterr("no place to put the result.\n");
		return -1;
	}
	if (g == nullptr && !stable)
		o = nullptr;        // pre-ordering is meaningless for an unstable full sort (:2410-2414)
	if (b->tnonil)
		nilslast = reverse;  // no nils: their placement does not matter (:2415-2420)
	ProfScope prof("BATsort");
	mgdk_bat *sn = nullptr, *on = nullptr, *gn = nullptr;
	bool mk_oidx = false;
	// trivially (sub)sorted (:2422-2472)
	if (n <= 1 || (reverse == nilslast && (reverse ? b->trevsorted : b->tsorted) && o == nullptr && g == nullptr &&
		       (groups == nullptr || b->tkey || (reverse ? b->tsorted : b->trevsorted)))) {
		if (sorted && (sn = mgdk_BATslice(b, 0, n)) == nullptr)
			goto fail;
		if (order && (on = mgdk_BATdense(b->hseqbase, b->hseqbase, n)) == nullptr)
			goto fail;
		if (groups) {
			oid zero = 0;
			gn = b->tkey ? mgdk_BATdense(b->hseqbase, 0, n) : mgdk_BATconstant(b->hseqbase, MGDK_oid, &zero, n);
			if (gn == nullptr)
				goto fail;
		}
		goto done;
	}
	// every group a single row: nothing to sort (:2633-2686)
	if (g && (g->tkey || g->ttype == MGDK_void)) {
		if (sorted && (sn = o ? mgdk_BATproject(o, b) : mgdk_BATslice(b, 0, n)) == nullptr)
			goto fail;
		if (order) {
			if (o) {
				on = mgdk_BATslice(o, 0, n);
				if (on == nullptr)
					goto fail;
				on->hseqbase = b->hseqbase;
				on->tsorted = o->tsorted;
				on->trevsorted = o->trevsorted;
			} else if ((on = seq_order(b->hseqbase, n)) == nullptr) {
				goto fail;
			}
			if (n <= 1)
				on->tsorted = on->trevsorted = 1;
		}
		if (groups) {
			gn = mgdk_BATslice(g, 0, n);
			if (gn == nullptr)
				goto fail;
		}
		goto done;
	}
	// the order index (gdk_batop.c:2488-2572): a column's own, or for a view
	// over a whole column the parent's, serves an unstable sort and a stable
	// one when it was built stable; BATsort builds one when it hands out an
	// order of a column that is not a view (every device BAT is transient)
	{
		bool ostable = false;
		size_t ooff = 0;
		Heap *oh = g == nullptr && !reverse && !nilslast && sort_internal == 0 ?
			oidx_get(b, &ostable, is_view(b) ? OIDX_PARENT : OIDX_OWN, &ooff) : nullptr;
		mk_oidx = g == nullptr && !reverse && !nilslast && order != nullptr && !is_view(b) && oh == nullptr &&
			  sort_internal == 0;
		if (oh && (stable && !ostable))
			heap_decref(oh), oh = nullptr;
		if (oh && o == nullptr) {
			const int rc = sort_by_oidx(&sn, &on, groups ? &gn : nullptr, b, oh, ooff, sorted != nullptr);
			heap_decref(oh);
			if (rc < 0)
				goto fail;
			goto done;
		}
		if (oh)
			heap_decref(oh);
	}
	// positions and ranks of the sorts below are 32-bit: a column of 2^32 or
	// more rows is only sorted through the shortcuts above (a documented
	// difference from the reference, which has no such limit)
	if (n >= ((BUN) 1 << 32)) {
		seterr("42000!BATsort: more than 2^32 rows");
		goto fail;
	}
	{
		// the runs do_sort sorts with GDKqsort
		std::vector<std::pair<uint64_t, uint32_t>> runs, qruns;
		bool single_run = g == nullptr;
		if (!stable) {
			const bool rx = radix_type(b->ttype);
			if (sort_runs(g, n, runs) < 0)
				goto fail;
			single_run = runs.size() <= 1;
			for (auto &r : runs)
				if (r.second > 1 && (!rx || reverse != nilslast || r.second <= 100))
					qruns.push_back(r);
			// without g, a column already in the requested order is left as it
			// is (:2735-2736)
			if (g == nullptr && reverse == nilslast && (reverse ? b->trevsorted : b->tsorted))
				qruns.clear();
		} else if (g) {
			single_run = mgdk_BATordered_rev(g);
		}
		if (!qruns.empty()) {
			if (sort_qsort(&on, groups ? &gn : nullptr, b, o, g, reverse, nilslast, qruns) < 0)
				goto fail;
			if (sorted && (sn = mgdk_BATproject(on, b)) == nullptr)
				goto fail;
			if (!order) {
				mgdk_BBPunfix(on);
				on = nullptr;
			}
		} else {
			if (sort_core(sorted ? &sn : nullptr, &on, groups ? &gn : nullptr, b, o, g, reverse, nilslast) < 0)
				goto fail;
			if (!order) {
				mgdk_BBPunfix(on);
				on = nullptr;
			}
		}
		// the order becomes b's order index (gdk_batop.c:2717-2765)
		if (mk_oidx && on && oidx_put(b, on, stable) < 0)
			goto fail;
		if (sn) {
			// gdk_batop.c:2712-2715, 2749-2750, 2772-2776
			sn->tsorted = single_run && !reverse && !nilslast;
			sn->trevsorted = single_run && reverse && nilslast;
			if (n <= 1)
				sn->tsorted = sn->trevsorted = 1;
			sn->tkey = o ? (o->tkey && b->tkey) : b->tkey;
			sn->tnonil = b->tnonil;
			sn->tnil = b->tnil;
			sn->tnosorted = sn->tnorevsorted = 0;
			sn->tminpos = sn->tmaxpos = MGDK_BUN_NONE;
			if (gn && gn->tkey && (g == nullptr || (g->tsorted && g->trevsorted)))
				sn->tkey = 1;
		}
	}
done:
	if (sorted) *sorted = sn; else mgdk_BBPunfix(sn);
	if (order) *order = on; else mgdk_BBPunfix(on);
	if (groups) *groups = gn; else mgdk_BBPunfix(gn);
	return 0;
fail:
	mgdk_BBPunfix(sn);
	mgdk_BBPunfix(on);
	mgdk_BBPunfix(gn);
	return -1;
}

// ---- order index (gdk/gdk_orderidx.c) --------------------------------------

// BATorderidx (gdk_orderidx.c:184): the column's sort order kept with it
extern "C" int
mgdk_BATorderidx(mgdk_bat *b, bool stable)
{
	if (b->ttype == MGDK_void) {
		seterr("No order index on void type bats\n");
		return -1;
	}
	if (mgdk_BATcheckorderidx(b))
		return 0;
	if (b->ttype == MGDK_oid && b->tseqbase != MGDK_OID_NIL)
		return 0;   // BATtdense
	mgdk_bat *on = nullptr;
	if (mgdk_BATsort(nullptr, &on, nullptr, b, nullptr, nullptr, false, false, stable) < 0)
		return -1;
	int rc = 0;
	if (on->ttype == MGDK_void) {
		// a dense order: the input was sorted (:199-208)
		b->tsorted = 1;
		b->tnosorted = 0;
	} else {
		rc = oidx_put(b, on, stable);
	}
	mgdk_BBPunfix(on);
	return rc;
}

// BATcheckorderidx (gdk_orderidx.c:74)
extern "C" bool
mgdk_BATcheckorderidx(mgdk_bat *b)
{
	if (b == nullptr)
		return false;
	Heap *h = oidx_get(b, nullptr, OIDX_OWN, nullptr);
	heap_decref(h);
	return h != nullptr;
}

// OIDXdestroy (gdk_orderidx.c:534)
extern "C" void
mgdk_OIDXdestroy(mgdk_bat *b)
{
	if (b == nullptr)
		return;
	Priv *p = (Priv *) b->priv;
	const bool v = p->view;
	img8_drop(b);   // drops every accelerator kept with the tail
	p->view = v;
}

// the column's order index (b->torderidx + ORDERIDXOFF) as a new oid BAT, or
// NULL without an error when it has none; stable: the index's stable flag
extern "C" mgdk_bat *
mgdk_BATorderidx_get(mgdk_bat *b, bool *stable)
{
	bool st = false;
	size_t off = 0;
	Heap *h = b ? oidx_get(b, &st, OIDX_OWN, &off) : nullptr;
	if (h == nullptr)
		return nullptr;
	mgdk_bat *o = oidx_bat(h, off, b->hseqbase, b->count);
	heap_decref(h);
	if (stable)
		*stable = st;
	return o;
}
