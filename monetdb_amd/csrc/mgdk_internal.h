// mgdk_internal.h -- shared internals of libmgdk.so (HIP, gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#include "../../include/mgdk.h"

typedef __int128 hge;
typedef unsigned __int128 uhge;
typedef mgdk_oid oid;
typedef mgdk_BUN BUN;

namespace mgdk {

// ---- errors: thread-local GDKerrbuf (gdk/gdk.h:1710,1947) ----------------
void seterr(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
bool hip_ok(hipError_t e, const char *what);

// ---- streams, allocator, scratch ------------------------------------------
hipStream_t stream();                       // per calling thread
hipStream_t stream2();                      // the thread's side stream (NULL if it cannot be made)
bool side_join();                           // the main stream waits for the side stream's queued work
bool side_fork();                           // the side stream waits for the main stream's queued work
void *dalloc(size_t bytes);                 // HBM, cached, >= 256 B aligned
void dfree(void *p);
// per-thread scratch (grows; valid until the next scratch() on this thread)
void *scratch(size_t bytes);
// pinned host staging for small device->host reads
void *pinned(size_t bytes);
// copy of `bytes` of host data in the thread's pinned upload arena (valid
// until its next sync(): queue the H2D copy, then wait once)
void *stage_host(const void *src, size_t bytes);
// 64 KiB of device zeros (created once): the load target of lanes whose
// rows are all filtered out, spread so no single line is hammered
constexpr size_t ZERO_REGION = 65536;
const void *zero_region();
// per-thread 4 KiB device buffer for small results / arguments
void *meta_buf();
bool sync();                                // stream sync + error check + query context
bool sync_data();                           // stream sync + error check (data transfers)

// ---- BAT heap ownership ---------------------------------------------------
struct Heap {
	void *base;
	size_t size;
	int refs;
};
struct Priv {
	Heap *theap;      // may be shared between views (BATslice)
	Heap *tvheap;
	size_t toff;      // byte offset of b->theap into theap->base
	// accelerator kept with the column (as GDK keeps hashes / imprints /
	// order indexes with a BAT): a 1-byte image of an oid tail whose values
	// are all < 255 (BATgroup's group ids for <= 255 groups), read by the
	// grouped aggregates and sub-grouping instead of the 8-byte ids; dropped
	// whenever the tail is written
	Heap *img8;
	BUN img8_n;
	// accelerator of a select result (an oid list from a dense candidate
	// scan): the scan's predicate bitmap (1 bit per candidate slot) and its
	// per-tile hit prefixes, so a projection through the list streams the
	// projected column in row order instead of reading the 8-byte oids and
	// gathering (see SelMap); dropped with img8 whenever the tail is written
	Heap *smap;
	BUN smap_n;
	uint32_t smap_wpt;       // bitmap words per tile
	uint64_t smap_ntiles;
	uint64_t smap_nslots;    // candidate slots covered (incl. the alignment shift)
	int64_t smap_base;       // oid of slot 0
	size_t smap_bits_off;    // byte offset of the bitmap in the heap (the prefixes are at 0)
	oid smap_lo, smap_hi;    // first / last oid of the list
	// the order index (gdk_orderidx.c: b->torderidx): the oids of the column
	// in sorted order.  A view over the whole column also holds its parent's
	// slot (BATsort uses the parent's index for it, gdk_batop.c:2473-2509),
	// so an index the parent gets later is seen; a written tail leaves both
	struct OidxSlot *oidx, *poidx;
	bool view;               // a BATslice view: BATsort builds no index for it
};
struct OidxSlot {
	int refs;
	Heap *idx;               // n oids at byte offset off, or NULL (the heap
	size_t off;              // is shared with the order BAT it came from:
	BUN n;                   // shared heaps are never written in place)
	bool stable;
};
struct SelMap {
	const uint32_t *bits;
	const uint64_t *pre;
	uint32_t wpt;
	uint64_t ntiles, nslots;
	int64_t base;
	oid lo, hi;
};
Heap *heap_new(size_t bytes);                    // refs = 1
void heap_decref(Heap *h);
mgdk_bat *newbat(oid hseq, int tt, BUN cap);     // allocates tail heap
void setdense(mgdk_bat *b, oid tseq, BUN cnt);
void share_vheap(mgdk_bat *dst, const mgdk_bat *src);
int width_of(int tt);
// the 1-byte image of b's oid tail, or NULL (see Priv::img8)
const uint8_t *img8_get(const mgdk_bat *b);
uint8_t *img8_new(mgdk_bat *b);     // allocate an image for b->count values
void img8_drop(mgdk_bat *b);        // drops every accelerator of the tail (img8, smap)
bool smap_get(const mgdk_bat *b, SelMap *m);
void smap_set(mgdk_bat *b, Heap *h, const SelMap &m);   // takes a reference on h
// b's order index (a reference on its heap, release with heap_decref; the
// oids start at *off bytes into it) or NULL: its own (OIDX_OWN), that of the
// column a whole-column view shows (OIDX_PARENT), or either (OIDX_ANY)
enum { OIDX_OWN = 1, OIDX_PARENT = 2, OIDX_ANY = 3 };
Heap *oidx_get(const mgdk_bat *b, bool *stable, int which, size_t *off);
// give b the order index `order` (an oid BAT of b->count rows, whose heap
// is shared, not copied) unless it has one of its own
int oidx_put(mgdk_bat *b, const mgdk_bat *order, bool stable);
// a new oid BAT over an index heap (shares it)
mgdk_bat *oidx_bat(Heap *h, size_t off, oid hseq, BUN n);
void oidx_share(mgdk_bat *v, const mgdk_bat *b);   // v: a view over all of b
// while one lives on a thread, mgdk_BATsort neither uses nor builds order
// indexes: the sorts the device path runs where the reference runs none
// (the reference's own BATsort calls sort temporaries or are mirrored as is)
extern thread_local int sort_internal;
// the first / last oids of a join's two result columns, read back by the
// partitioned hash join with its pair count (one round trip instead of
// three); hashjoin (joinalgo.hip) takes them when a / b are its results
struct JoinEnds {
	const mgdk_bat *a = nullptr, *b = nullptr;
	oid af = 0, al = 0, bf = 0, bl = 0;
};
extern thread_local JoinEnds join_ends;
struct SortInternal {
	SortInternal() { ++sort_internal; }
	~SortInternal() { --sort_internal; }
};
bool is_view(const mgdk_bat *b);
int basetype(int tt);                            // date->int, bit->bte
const char *atomname(int tt);

// rows from which one group / partition of an order-dependent float fold
// takes the parallel form (mgdk_set_fp_parallel_min)
BUN fp_parallel_min();

// ordered pairwise tree over one value per thread of the block (blockDim a
// power of two <= 1024): thread 0 returns comb(v0, v1, ..., v_{n-1}) in
// thread order, the same association for every launch (deterministic)
template <typename S, typename F>
__device__ __forceinline__ S
block_tree(S v, F comb, S *lds)
{
	lds[threadIdx.x] = v;
	__syncthreads();
	for (unsigned st = 1; st < blockDim.x; st <<= 1) {
		if ((threadIdx.x & (2 * st - 1)) == 0)
			lds[threadIdx.x] = comb(lds[threadIdx.x], lds[threadIdx.x + st]);
		__syncthreads();
	}
	return lds[0];
}

// ---- profiling ----------------------------------------------------------
struct ProfScope {
	const char *name;
	hipEvent_t e0, e1;
	bool on;
	explicit ProfScope(const char *n);
	~ProfScope();
};

// ---- launch helpers ---------------------------------------------------------
constexpr int BLOCK = 256;
inline unsigned grid_for(uint64_t items, uint64_t per_block, unsigned cap = 65535u * 64u) {
	uint64_t g = (items + per_block - 1) / per_block;
	if (g == 0) g = 1;
	return g > cap ? cap : (unsigned) g;
}

// ---- candidate description used by kernels --------------------------------
struct Cand {
	bool dense;
	oid seq;              // dense: first candidate
	const oid *oids;      // materialized: device pointer to first candidate
	BUN n;
	oid first, last;      // first/last candidate oid (valid when n > 0)
	const mgdk_bat *src;  // materialized: the list itself (its accelerators)
};
// canditer_init (gdk/gdk_cand.c:407): clip s to b's [hseqbase, hseqbase+count)
int cand_init(Cand *ci, const mgdk_bat *b, const mgdk_bat *s);
// all of ci's candidates as a new candidate list, hseqbase 0 (canditer_slice,
// gdk_cand.c; select.hip): void when dense
mgdk_bat *cand_slice(const Cand &ci);
// index of candidate oid o in ci (canditer_search); BUN NONE-like ~0 on error
BUN cand_index(const Cand &ci, oid o);
// one oid of an oid / void column (host read)
int oid_at(const mgdk_bat *b, BUN p, oid *v);

// a cand_except / cand_mask list (void BAT + ccand_t vheap) as a new ordered
// oid list (BATunmask, gdk_cand.c); the caller owns the result
mgdk_bat *unmask_cand(const mgdk_bat *s);
// a candidate list that is not a dense range or a sorted oid array: the
// cand_except / cand_mask forms (void + ccand_t vheap) and msk bit BATs
inline bool is_complex_cand(const mgdk_bat *s)
{
	return (s->ttype == MGDK_void && s->tvheap && s->tvheapsize > 8) || s->ttype == MGDK_msk;
}
// bytes of the first n values of b's tail (msk: 32-bit words of bits)
size_t tail_bytes(const mgdk_bat *b, BUN n);

// ordered compaction (select.hip): sorted positions base+i with flags[i]==1;
// the result may be a dense (void) BAT.  Uses the thread's scratch buffer.
mgdk_bat *compact_flags(const int8_t *flags, BUN n, oid base, bool nonzero = false);
// a new sorted, duplicate-free oid BAT of n values (cand.hip): candidate-list
// properties, and void when the values are dense (virtualize)
mgdk_bat *cand_finish(mgdk_bat *bn, BUN n);

// device-wide exclusive prefix sums (scan.hip); *total = sum of all inputs
int exclusive_scan(const uint32_t *in, uint32_t *out, BUN n, uint64_t *total);
int exclusive_scan(const uint32_t *in, uint64_t *out, BUN n, uint64_t *total);
int exclusive_scan(const uint8_t *in, uint64_t *out, BUN n, uint64_t *total);
// the same without waiting for the stream: ws (scan_ws_words(n) words, owned
// by the caller until its next sync) receives the total at ws[2] and the
// look-back error flag at ws[3] (low 32 bits)
BUN scan_ws_words(BUN n);
int exclusive_scan_nosync(const uint32_t *in, uint64_t *out, BUN n, uint64_t *ws);

// stable LSD radix sort of (key, payload) pairs in place (sort.hip); keys
// are order-preserving unsigned images; `bits` = significant key bits.
// Returns the buffers holding the result (the input pair or the spare).
int radix_sort_pairs(uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt,
		     BUN n, int bits, uint64_t **keys_out, uint32_t **vals_out);

// leftjoin's algorithm choice (joinalgo.hip; gdk_join.c:4049-4300)
enum { LJ_NOMATCH = 0, LJ_SELECT = 1, LJ_MJVOID = 2, LJ_FETCH = 3, LJ_BITMASK = 4, LJ_MERGE = 5, LJ_SWAP = 6,
       LJ_HASH = 7 };
int leftjoin_algo(mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, const Cand &lc, const Cand &rc,
		  bool nil_matches, bool nil_on_miss, bool semi, bool only_misses, bool not_in, bool max_one,
		  bool min_one, bool want_r2, bool *equal_order);
// BATjoin's key images for flt / dbl and str (joinalgo.hip)
mgdk_bat *join_float_image(const mgdk_bat *b);
int join_str_images(mgdk_bat *l, mgdk_bat *r, mgdk_bat **lip, mgdk_bat **rip);
void join_image_flags_back(mgdk_bat *l, mgdk_bat *r, const mgdk_bat *li, const mgdk_bat *ri);
// GDKqsort's permutation (qsort.hip) of every segment (start, len) of the
// rows (rank, pay): ranks are the rows' dense ranks in the requested order
int qsort_replay(uint32_t *rank, uint64_t *pay, BUN n, const std::vector<std::pair<uint64_t, uint32_t>> &segs);

// stable sort of the positions 0..n-1 by 32-bit keys (sort.hip); when no
// pass is needed (all keys equal) *perm is left NULL: identity
int radix_sort_positions32(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt, BUN n,
			   int bits, uint32_t **perm);

// RANGE bounds over lng images of bte..lng values with a static limit
// (analytic.hip): ordered fast path + fix-ups + unordered walk; `limit` is
// min(limit, tmax), overflow when |v - b[j]| of the stopping pair > tmax
int range_bounds_int64(mgdk_bat *r, const int64_t *bvals, const mgdk_bat *p, BUN n, int64_t limit,
		       uint64_t tmax, bool all, bool preceding);

// BATgroupavg3's result for one group from its exact sum and count
// (gdk_aggr.c:2070-2095): floor average and remainder, then rounded half
// away from zero
inline void
avg3_of_sum(hge s, int64_t n, int64_t *avg, int64_t *rem)
{
	hge q = s / n, r = s % n;
	if (r < 0) {
		q -= 1;
		r += n;
	}
	if (r > 0) {
		if (q < 0) {
			if (2 * r > n) {
				q++;
				r -= n;
			}
		} else if (2 * r >= n) {
			q++;
			r -= n;
		}
	}
	*avg = (int64_t) q;
	*rem = (int64_t) r;
}

// RAII device temporary (not the per-thread scratch)
struct DevBuf {
	void *p = nullptr;
	explicit DevBuf(size_t bytes) { p = dalloc(bytes ? bytes : 1); }
	~DevBuf() { dfree(p); }
	DevBuf(const DevBuf &) = delete;
	DevBuf &operator=(const DevBuf &) = delete;
	template <typename T> T *as() const { return (T *) p; }
};

// BATgroupaggrinit (gdk/gdk_aggr.c:65; aggr.hip): candidates, group id range
// and the form of g.  group_init replaces *bp by b's values gathered at a
// materialised candidate list (then ci is dense over them)
struct AggrInit {
	Cand ci;
	oid min, max;
	BUN ngrp;
	const oid *gids;   // NULL: dense g
	const uint8_t *g8; // 1-byte image of gids kept by BATgroup (or NULL)
	oid gseq;
	bool gsorted;      // g non-decreasing: every group a run of rows
	bool gkey;         // g strictly increasing (or dense): at most one row per group
};
int group_init(AggrInit *a, mgdk_bat **bp, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s);
// b's values at a materialised candidate list, head at the first candidate
// (kept alive by a small per-thread ring: use before the next few calls)
mgdk_bat *cand_values_at(mgdk_bat *b, const Cand &ci);
// the candidate rows grouped by group id, candidate order kept within a
// group (aggr.hip): rows perm[start[k]] .. perm[start[k+1] - 1] of group k;
// perm NULL: the identity; start_p NULL (one group): every row, whose ids
// the reader range-checks.  Rows outside the group range sort behind.
struct GroupRows {
	DevBuf key, key2, v0, v1, cnt, start;
	const uint32_t *perm = nullptr;
	const uint64_t *start_p = nullptr;
	GroupRows(BUN n, BUN ng);
	bool ok() const;
};
int group_rows(const AggrInit &a, GroupRows &gr);

}  // namespace mgdk


// ---- device-side helpers ------------------------------------------------
template <typename T> struct NilOf;
template <> struct NilOf<int8_t> { static __device__ __host__ constexpr int8_t v() { return INT8_MIN; } };
template <> struct NilOf<int16_t> { static __device__ __host__ constexpr int16_t v() { return INT16_MIN; } };
template <> struct NilOf<int32_t> { static __device__ __host__ constexpr int32_t v() { return INT32_MIN; } };
template <> struct NilOf<int64_t> { static __device__ __host__ constexpr int64_t v() { return INT64_MIN; } };
template <> struct NilOf<uint64_t> { static __device__ __host__ constexpr uint64_t v() { return (uint64_t) 1 << 63; } };
template <> struct NilOf<hge> { static __device__ __host__ constexpr hge v() { return (hge) ((uhge) 1 << 127); } };

template <typename T>
__device__ __host__ inline bool is_nil(T v) { return v == NilOf<T>::v(); }
__device__ __host__ inline bool is_nil(float v) { return v != v; }
__device__ __host__ inline bool is_nil(double v) { return v != v; }

// wave64 helpers
__device__ inline unsigned lane_id() { return __lane_id(); }
__device__ inline uint64_t lanemask_lt() {
	unsigned l = __lane_id();
	return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// ---- block reductions (blockDim.x == 256, every thread calls) -------------
// One global atomic per WORKGROUP, not per wave: same-word device atomics
// serialise at ~88/us (MI355X_MICROARCH.md "fanin"/"dequeue"), so a grid of
// thousands of waves each hitting one word would be bound by the atomic.
// The result is valid in thread 0.
template <typename T, typename F>
__device__ __forceinline__ T
block_reduce(T v, F op)
{
	__shared__ T s_red[4];
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v = op(v, __shfl_xor(v, o));
	__syncthreads();                 // s_red may still be read by a previous call
	if (__lane_id() == 0)
		s_red[threadIdx.x >> 6] = v;
	__syncthreads();
	if (threadIdx.x == 0)
		v = op(op(s_red[0], s_red[1]), op(s_red[2], s_red[3]));
	return v;
}

__device__ __forceinline__ hge
block_sum128(hge s)
{
	unsigned long long lo = (unsigned long long) (uhge) s, hi = (unsigned long long) ((uhge) s >> 64);
	__shared__ unsigned long long s_lo[4], s_hi[4];
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) {
		const unsigned long long l2 = __shfl_xor(lo, o), h2 = __shfl_xor(hi, o);
		const uhge t = (((uhge) hi << 64) | lo) + (((uhge) h2 << 64) | l2);
		lo = (unsigned long long) t;
		hi = (unsigned long long) (t >> 64);
	}
	__syncthreads();
	if (__lane_id() == 0) {
		s_lo[threadIdx.x >> 6] = lo;
		s_hi[threadIdx.x >> 6] = hi;
	}
	__syncthreads();
	uhge t = 0;
	if (threadIdx.x == 0)
		for (int q = 0; q < 4; q++)
			t += ((uhge) s_hi[q] << 64) | s_lo[q];
	return (hge) t;
}

// thread 0 of a workgroup: set bits in a flag word, skipping the atomic when
// they are already visible
__device__ __forceinline__ void
publish_or(uint32_t *flag, uint32_t bits)
{
	if (bits && (bits & ~__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
		atomicOr(flag, bits);
}

// raise a device-wide maximum, skipping the atomic when a value at least as
// large is already visible: one same-word atomic per wave of a large grid
// serialises at the L2 (~88 per microsecond)
__device__ __forceinline__ void
publish_max(unsigned long long *m, unsigned long long v)
{
	if (v > __hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
		atomicMax(m, v);
}

// 128-bit integer -> double, round to nearest even: the top 64 significant
// bits with a sticky bit below them convert exactly like the full value
__device__ __forceinline__ double
hge_to_dbl(hge v)
{
	if (v >= (hge) INT64_MIN && v <= (hge) INT64_MAX)
		return (double) (long long) v;
	const bool neg = v < 0;
	const uhge u = neg ? (uhge) 0 - (uhge) v : (uhge) v;
	const unsigned long long hi = (unsigned long long) (u >> 64);
	if (hi == 0)
		return neg ? -(double) (unsigned long long) u : (double) (unsigned long long) u;
	const int shift = 64 - __builtin_clzll(hi);                 // 1..64
	unsigned long long top = (unsigned long long) (u >> shift);
	if (u & (((uhge) 1 << shift) - 1))
		top |= 1;
	const double d = ldexp((double) top, shift);
	return neg ? -d : d;
}
