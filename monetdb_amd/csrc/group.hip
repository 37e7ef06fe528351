// group.hip -- BATgroup on the MI355X (gdk/gdk_group.c:657-1347).
//
// GDK numbers groups in order of FIRST OCCURRENCE of each distinct
// (prior group, value) pair over the candidates (GRPnotfound,
// gdk_group.c:74-100); a GPU hash table is unordered, so the numbering is
// recovered from first positions:
//   A  insert: every candidate finds its slot -- a direct index for 1/2-byte
//      keys (bte/sht/str offsets, GRP_small_values' domain, :607-654) or an
//      open-addressing table keyed by a CAS-claimed representative row --
//      and lowers the slot's first position with a pre-checked atomicMin;
//   B  flags[i] = (slot(i).first == i); the ordered compaction kernel of
//      select.hip turns them into the sorted first positions = extents, in
//      group-id order;
//   C  slot -> group id map from the extents;
//   D  group id per row + histogram (LDS-privatised counts for <= 4096
//      groups) + the sortedness property.
// nil is an ordinary value (all nils form one group); float keys compare by
// value (+0 == -0, every NaN is nil).
#include <cstdlib>
#include <vector>

#include <type_traits>
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

struct KeySrc {
	const void *base;
	int w;
	int kind;          // 0 signed int, 1 unsigned (str offsets), 2 flt, 3 dbl
	bool dense;
	oid off;           // dense: position of candidate 0
	const oid *oids;   // materialized candidates
	oid hseq;
	const oid *g;      // prior groups aligned with candidates (NULL: none)
	const uint8_t *g8; // their 1-byte image kept with g (NULL: none)
	oid gseq;          // dense prior groups: gseq + i
	bool has_g;
};

__device__ __forceinline__ void
key_at(const KeySrc &s, BUN i, uint64_t &k0, uint64_t &k1, uint64_t &gg)
{
	BUN p = s.dense ? s.off + i : s.oids[i] - s.hseq;
	k1 = 0;
	switch (s.w) {
	case 1: k0 = s.kind == 1 ? ((const uint8_t *) s.base)[p] : (uint64_t) (uint8_t) ((const int8_t *) s.base)[p]; break;
	case 2: k0 = ((const uint16_t *) s.base)[p]; break;
	case 4:
		if (s.kind == 2) {
			float f = ((const float *) s.base)[p];
			if (f != f) k0 = 0x7fc00000u;
			else if (f == 0.0f) k0 = 0;
			else k0 = __float_as_uint(f);
		} else {
			k0 = ((const uint32_t *) s.base)[p];
		}
		break;
	case 8:
		if (s.kind == 3) {
			double d = ((const double *) s.base)[p];
			if (d != d) k0 = 0x7ff8000000000000ull;
			else if (d == 0.0) k0 = 0;
			else k0 = (uint64_t) __double_as_longlong(d);
		} else {
			k0 = ((const uint64_t *) s.base)[p];
		}
		break;
	default:
		k0 = ((const uint64_t *) s.base)[2 * p];
		k1 = ((const uint64_t *) s.base)[2 * p + 1];
		break;
	}
	gg = s.has_g ? (s.g8 ? (uint64_t) s.g8[i] : s.g ? s.g[i] : s.gseq + i) : 0;
}

__device__ __forceinline__ uint64_t
hmix(uint64_t a, uint64_t b, uint64_t c)
{
	uint64_t x = a * 0x9e3779b97f4a7c15ull ^ (b + 0x632be59bd9b4e019ull) * 0xbf58476d1ce4e5b9ull ^ c * 0x94d049bb133111ebull;
	x ^= x >> 31;
	x *= 0xd6e8feb86659fd93ull;
	return x ^ (x >> 32);
}

constexpr uint64_t EMPTY = ~0ull;

// direct: slot = gg * D + k0 (1/2-byte keys), no probing
template <bool DIRECT>
__global__ __launch_bounds__(256) void
k_grp_insert(KeySrc s, BUN n, uint64_t mask, int dshift, unsigned long long *s_row,
	     unsigned long long *s_min, uint32_t *hidx, uint32_t *err)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		uint64_t k0, k1, gg;
		key_at(s, i, k0, k1, gg);
		uint64_t h;
		if (DIRECT) {
			h = (gg << dshift) | k0;
		} else {
			h = hmix(k0, k1, gg) & mask;
			uint32_t probes = 0;
			for (;;) {
				unsigned long long r = s_row[h];
				if (r == EMPTY) {
					r = atomicCAS(&s_row[h], EMPTY, (unsigned long long) i);
					if (r == EMPTY)
						break;
				}
				uint64_t r0, r1, rg;
				key_at(s, r, r0, r1, rg);
				if (r0 == k0 && r1 == k1 && rg == gg)
					break;
				h = (h + 1) & mask;
				if (++probes > mask) {
					atomicOr(err, 1u);
					break;
				}
			}
		}
		hidx[i] = (uint32_t) h;
		if (s_min[h] > i)
			atomicMin(&s_min[h], (unsigned long long) i);
	}
}

__global__ __launch_bounds__(256) void
k_grp_flags(BUN n, const uint32_t *hidx, const unsigned long long *s_min, int8_t *flags)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		flags[i] = s_min[hidx[i]] == i;
}

__global__ __launch_bounds__(256) void
k_grp_map(BUN ngrp, const oid *E, oid Eseq, const uint32_t *hidx, uint32_t *gidmap, bool cdense,
	  oid cseq, const oid *coids, oid *ext)
{
	for (BUN e = (BUN) blockIdx.x * blockDim.x + threadIdx.x; e < ngrp; e += (BUN) gridDim.x * blockDim.x) {
		BUN p = E ? E[e] : Eseq + e;
		gidmap[hidx[p]] = (uint32_t) e;
		ext[e] = cdense ? cseq + p : coids[p];
	}
}

template <bool LDSHIST>
__global__ __launch_bounds__(256) void
k_grp_assign(BUN n, const uint32_t *hidx, const uint32_t *gidmap, oid *gid, BUN ngrp,
	     unsigned long long *histo, uint32_t *unsorted)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
	if (LDSHIST) {
		for (BUN k = threadIdx.x; k < ngrp; k += blockDim.x)
			s_hist[k] = 0;
		__syncthreads();
	}
	uint32_t uns = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		uint32_t g = gidmap[hidx[i]];
		gid[i] = g;
		if (i > 0 && gidmap[hidx[i - 1]] > g)
			uns = 1;
		if (LDSHIST)
			atomicAdd(&s_hist[g], 1u);
		else
			atomicAdd(&histo[g], 1ull);
	}
	uns = block_reduce(uns, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(unsorted, uns);
	if (LDSHIST) {
		__syncthreads();
		for (BUN k = threadIdx.x; k < ngrp; k += blockDim.x)
			if (s_hist[k])
				atomicAdd(&histo[k], (unsigned long long) s_hist[k]);
	}
}

__global__ void
k_max_oid(const oid *g, BUN n, unsigned long long *out)
{
	unsigned long long mx = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		if (g[i] != MGDK_OID_NIL && g[i] > mx)
			mx = g[i];
	mx = block_reduce(mx, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	if (threadIdx.x == 0)
		atomicMax(out, mx);
}


// ---------------------------------------------------------------------------
// Low-cardinality path (<= GL_MAXG groups; keys that fit one 64-bit image:
// (prior group << 32 | key) for keys of <= 4 bytes, the key alone for 8-byte
// keys without prior groups).  Three kernels, no per-row global atomics:
//   first  each workgroup (64 Ki rows) builds an LDS table of its distinct
//          keys with their first row, then merges it into a 4 Ki-slot
//          global table (one CAS + one atomicMin per distinct key per tile);
//   order  one workgroup sorts the occupied slots by first row (bitonic in
//          LDS): rank = group id (first occurrence), extents;
//   assign each workgroup copies the table + slot->id map into LDS and
//          writes every row's group id, an LDS histogram and the order flag.
// The image ~0 is kept in a slot of its own (GL_SLOTS).  Overflow of either
// table (more distinct keys than fit) sends BATgroup to the global path.
// ---------------------------------------------------------------------------

constexpr uint32_t GL_SLOTS = 4096;
constexpr uint32_t GL_MAXG = 3072;
constexpr uint64_t GL_EMPTY = ~0ull;
#ifndef MGDK_GL_TILE
#define MGDK_GL_TILE 32768      // 32 Ki: 0.411 vs 0.423 ms (64 Ki) vs 0.434 (128 Ki), 100M x 1000
#endif
constexpr BUN GL_TILE = MGDK_GL_TILE;     // rows per assign workgroup (and per prefix tile)
constexpr BUN GL_FTILE = 8192;
#ifndef MGDK_GL_NT_STORE
#define MGDK_GL_NT_STORE 1        // nontemporal id stores in the 4-byte assign pass
#endif
#ifndef MGDK_GL_NT_LOAD
#define MGDK_GL_NT_LOAD 1
#endif
#ifndef MGDK_GL_CSTORE
#define MGDK_GL_CSTORE 1          // ids stored as whole 1-KiB pieces per wave instruction
#endif            // rows per workgroup of the first-occurrence pass

__device__ __forceinline__ uint64_t
gl_key(const KeySrc &s, BUN i)
{
	uint64_t k0, k1, gg;
	key_at(s, i, k0, k1, gg);
	return s.has_g ? (gg << 32) | k0 : k0;
}

// typed key image for dense candidates over integer keys (W = 1, 2, 4, 8
// bytes, zero-extended as key_at does for kinds 0 / 1) and prior groups
// G = 0 none, 1 the 1-byte image, 2 an oid column, 3 dense; W == 0 takes
// the generic key_at.  No branch on the width: a load under a runtime
// switch is waited for before the switch joins (DESIGN §4 lesson).
template <int W, int G>
__device__ __forceinline__ uint64_t
gl_key_t(const KeySrc &s, BUN i)
{
	if constexpr (W == 0) {
		return gl_key(s, i);
	} else {
		const BUN p = s.off + i;
		uint64_t k;
		if constexpr (W == 1)
			k = ((const uint8_t *) s.base)[p];
		else if constexpr (W == 2)
			k = ((const uint16_t *) s.base)[p];
		else if constexpr (W == 4)
			k = ((const uint32_t *) s.base)[p];
		else
			k = ((const uint64_t *) s.base)[p];
		if constexpr (G == 1)
			return ((uint64_t) s.g8[i] << 32) | k;
		else if constexpr (G == 2)
			return ((uint64_t) s.g[i] << 32) | k;
		else if constexpr (G == 3)
			return ((uint64_t) (s.gseq + i) << 32) | k;
		else
			return k;
	}
}

constexpr int GL_U = 8;                   // rows per thread in flight

__device__ __forceinline__ uint32_t
gl_hash(uint64_t k)
{
	return (uint32_t) ((k * 0x9E3779B97F4A7C15ull) >> 52);
}

template <int W, int G>
__global__ __launch_bounds__(1024) void
k_gl_first(KeySrc s, BUN n, BUN tile0, unsigned long long *gkey, unsigned long long *gmin, uint32_t *err)
{
	__shared__ unsigned long long lkey[GL_SLOTS];
	__shared__ uint32_t lmin[GL_SLOTS + 1];
	const unsigned tid = threadIdx.x;
	for (uint32_t q = tid; q < GL_SLOTS; q += blockDim.x) {
		lkey[q] = GL_EMPTY;
		lmin[q] = ~0u;
	}
	if (tid == 0)
		lmin[GL_SLOTS] = ~0u;
	__syncthreads();
	// GL_FTILE rows per workgroup from tile tile0 on: many small tables
	// fill the chip where one per 64 Ki-row tile left it idle
	const BUN a = tile0 * GL_TILE + (BUN) blockIdx.x * GL_FTILE, e = min(n, a + GL_FTILE);
	bool ovf = false;
	for (BUN i0 = a + tid; i0 < e; i0 += (BUN) GL_U * blockDim.x) {
		uint64_t kk[GL_U];
#pragma unroll
		for (int u = 0; u < GL_U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x;
			kk[u] = gl_key_t<W, G>(s, i < e ? i : e - 1);       // clamped, all in flight
		}
#pragma unroll
		for (int u = 0; u < GL_U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x;
			if (i >= e)
				continue;
			const uint64_t k = kk[u];
			const uint32_t r = (uint32_t) (i - a);
			if (k == GL_EMPTY) {
				atomicMin(&lmin[GL_SLOTS], r);
				continue;
			}
			uint32_t h = gl_hash(k);
			for (uint32_t pr = 0;; pr++) {
				unsigned long long o = lkey[h];
				if (o == GL_EMPTY)
					o = atomicCAS(&lkey[h], GL_EMPTY, k);
				if (o == GL_EMPTY || o == k) {
					if (lmin[h] > r)
						atomicMin(&lmin[h], r);
					break;
				}
				h = (h + 1) & (GL_SLOTS - 1);
				if (pr >= GL_SLOTS) {
					ovf = true;
					break;
				}
			}
		}
	}
	if (__any(ovf) && __lane_id() == 0)
		atomicOr(err, 1u);
	__syncthreads();
	for (uint32_t q = tid; q <= GL_SLOTS; q += blockDim.x) {
		if (lmin[q] == ~0u)
			continue;
		const unsigned long long first = a + lmin[q];
		if (q == GL_SLOTS) {
			if (gmin[GL_SLOTS] > first)
				atomicMin(&gmin[GL_SLOTS], first);
			continue;
		}
		const uint64_t k = lkey[q];
		uint32_t h = gl_hash(k);
		for (uint32_t pr = 0;; pr++) {
			unsigned long long o = gkey[h];
			if (o == GL_EMPTY)
				o = atomicCAS(&gkey[h], GL_EMPTY, k);
			if (o == GL_EMPTY || o == k) {
				if (gmin[h] > first)
					atomicMin(&gmin[h], first);
				break;
			}
			h = (h + 1) & (GL_SLOTS - 1);
			if (pr >= GL_SLOTS) {
				atomicOr(err, 1u);
				break;
			}
		}
	}
}

// occupied slots ranked by first row (counting ranks over the compacted
// keys first << 13 | slot, all distinct) -> group ids, extents.  Every
// workgroup compacts the table in slot order (a scan, so all workgroups
// hold the same list) and ranks its share of the entries
constexpr unsigned GL_ORDER_SPLIT = 4;
constexpr unsigned GL_ORDER_WG = (GL_MAXG * GL_ORDER_SPLIT + 255) / 256;
// the tables' and flags' initial state in ONE launch (three memsets cost
// ~10 us of blit launches on a 0.4 ms call)
__global__ __launch_bounds__(256) void
k_gl_init(unsigned long long *gkey, unsigned long long *gmin, uint32_t *m)
{
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i <= GL_SLOTS; i += gridDim.x * blockDim.x) {
		gkey[i] = ~0ull;
		gmin[i] = ~0ull;
	}
	if (blockIdx.x == 0 && threadIdx.x < 4)
		m[threadIdx.x] = 0;
}

// also clears the histogram (GL_MAXG + 1 words) and the assign pass's two
// flags m[2], m[3], which the assign pass that follows accumulates into
__global__ __launch_bounds__(256) void
k_gl_order(const unsigned long long *gmin, uint32_t *gmap, bool cdense, oid cseq, const oid *coids, oid *ext,
	   uint32_t *ngrp, unsigned long long *histo)
{
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i <= GL_MAXG; i += gridDim.x * blockDim.x)
		histo[i] = 0ull;
	if (blockIdx.x == 0 && threadIdx.x < 2)
		ngrp[1 + threadIdx.x] = 0;
	__shared__ unsigned long long sk[GL_SLOTS + 1];
	__shared__ uint32_t ws[4];
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	// thread t holds slots 16 t .. 16 t + 15 (and thread 255 the extra slot GL_SLOTS)
	constexpr uint32_t PER = GL_SLOTS / 256;
	unsigned long long f[PER + 1];
	uint32_t cnt = 0;
#pragma unroll
	for (uint32_t x = 0; x < PER; x++) {
		f[x] = gmin[tid * PER + x];
		cnt += f[x] != ~0ull;
	}
	f[PER] = tid == 255 ? gmin[GL_SLOTS] : ~0ull;
	cnt += f[PER] != ~0ull;
	uint32_t inc = cnt;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t t = __shfl_up(inc, o);
		if (lane >= (unsigned) o)
			inc += t;
	}
	if (lane == 63)
		ws[w] = inc;
	__syncthreads();
	uint32_t pos = inc - cnt;
	for (unsigned k = 0; k < w; k++)
		pos += ws[k];
	const uint32_t c = ws[0] + ws[1] + ws[2] + ws[3];
#pragma unroll
	for (uint32_t x = 0; x <= PER; x++)
		if (f[x] != ~0ull)
			sk[pos++] = (f[x] << 13) | (x < PER ? tid * PER + x : GL_SLOTS);
	__syncthreads();
	// GL_ORDER_SPLIT consecutive lanes count one entry's rank over
	// interleaved quarters of the list and add their counts
	const uint32_t sub = tid % GL_ORDER_SPLIT;
	for (uint32_t i0 = (blockIdx.x * blockDim.x + tid) / GL_ORDER_SPLIT; i0 < (c + 63) / 64 * 64;
	     i0 += gridDim.x * blockDim.x / GL_ORDER_SPLIT) {
		const uint32_t i = i0 < c ? i0 : 0;
		const unsigned long long v = sk[i];
		uint32_t r = 0;
		for (uint32_t j = sub; j < c; j += GL_ORDER_SPLIT)
			r += sk[j] < v;
#pragma unroll
		for (int o = 1; o < (int) GL_ORDER_SPLIT; o <<= 1)
			r += __shfl_xor(r, o);
		if (sub == 0 && i0 < c) {
			const uint32_t slot = (uint32_t) (v & 8191);
			gmap[slot] = r;
			if (r < GL_MAXG)     // more groups: the path does not apply
				ext[r] = cdense ? cseq + (BUN) (v >> 13) : coids[v >> 13];
		}
	}
	if (tid == 0 && blockIdx.x == 0)
		*ngrp = c;
}

__device__ __forceinline__ uint32_t
gl_lookup(const unsigned long long *lkey, const uint32_t *lmap, uint64_t k)
{
	if (k == GL_EMPTY)
		return lmap[GL_SLOTS];
	uint32_t h = gl_hash(k);
	for (;;) {
		const unsigned long long o = lkey[h];
		if (o == k)
			return lmap[h];
		if (o == GL_EMPTY)
			return ~0u;             // not in the table (the table keeps an empty slot)
		h = (h + 1) & (GL_SLOTS - 1);
	}
}

// The assign kernels are queued right behind the order pass, before the host
// knows the group count: they read it (gm[1]) and the first pass's overflow
// flag (gm[0]) themselves, return at once when the table overflowed (the
// host then takes the global path), write the 1-byte image only for <= 255
// groups and copy the first / last extent for the host's virtualisation test
// -- one host round trip per BATgroup instead of two
#define GL_ASSIGN_PROLOGUE \
	const uint32_t ngrp = gm[1]; \
	if (gm[0] != 0 || ngrp > GL_MAXG) \
		return; \
	if (ngrp > 255) \
		img = nullptr; \
	if (blockIdx.x == 0 && threadIdx.x == 0 && ngrp > 0) { \
		flo[0] = ext[0]; \
		flo[1] = ext[ngrp - 1]; \
	}

template <int W, int G>
__global__ __launch_bounds__(1024) void
k_gl_assign(KeySrc s, BUN n, const unsigned long long *gkey, const uint32_t *gmap, const uint32_t *gm, oid *gid,
	    uint8_t *img, unsigned long long *histo, uint32_t *unsorted, uint32_t *miss, const oid *ext, oid *flo)
{
	GL_ASSIGN_PROLOGUE;
	__shared__ unsigned long long lkey[GL_SLOTS];
	__shared__ uint32_t lmap[GL_SLOTS + 1];
	__shared__ uint32_t lh[GL_MAXG];
	const unsigned tid = threadIdx.x, lane = __lane_id();
	for (uint32_t q = tid; q < GL_SLOTS; q += blockDim.x) {
		lkey[q] = gkey[q];
		lmap[q] = gmap[q];
	}
	if (tid == 0)
		lmap[GL_SLOTS] = gmap[GL_SLOTS];
	for (uint32_t q = tid; q < ngrp; q += blockDim.x)
		lh[q] = 0;
	__syncthreads();
	const BUN a = (BUN) blockIdx.x * GL_TILE, e = min(n, a + GL_TILE);
	uint32_t uns = 0;
	bool mis = false;
	for (BUN i0 = a + tid; i0 < e; i0 += (BUN) GL_U * blockDim.x) {
		uint64_t kk[GL_U], kp[GL_U];
#pragma unroll
		for (int u = 0; u < GL_U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x, ic = i < e ? i : e - 1;
			kk[u] = gl_key_t<W, G>(s, ic);
			// lane 0's predecessor lies in the previous wave's rows; loaded
			// by every lane (the same lines): a load under a lane-0 branch
			// would be waited for before the branch joins, one row at a time
			kp[u] = gl_key_t<W, G>(s, ic > 0 ? ic - 1 : 0);
		}
#pragma unroll
		for (int u = 0; u < GL_U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x;
			uint32_t g = 0;
			if (i < e) {
				g = gl_lookup(lkey, lmap, kk[u]);
				if (g == ~0u) {
					mis = true;         // first seen past the scanned prefix
					g = 0;
				} else {
					gid[i] = g;
					if (img)
						img[i] = (uint8_t) g;
					atomicAdd(&lh[g], 1u);
				}
			}
			uint32_t gp = __shfl_up(g, 1);
			if (lane == 0 && i > 0 && i < e)
				gp = gl_lookup(lkey, lmap, kp[u]);
			if (i > 0 && i < e && gp > g)
				uns = 1;
		}
	}
	if (__any(uns) && lane == 0)
		publish_or(unsorted, 1u);
	if (__any(mis) && lane == 0)
		publish_or(miss, 1u);
	__syncthreads();
	for (uint32_t q = tid; q < ngrp; q += blockDim.x)
		if (lh[q])
			atomicAdd(&histo[q], (unsigned long long) lh[q]);
}

// the assign pass for dense integer keys of W = 4 or 8 bytes without prior
// groups: a lane takes V = 16 / W CONSECUTIVE rows per step (one 16-byte
// key load; every wave instruction covers 1 KiB of keys) and stores their
// ids as 16-byte pieces; the order flag compares each row with the one
// before it (the lane's previous row, or the key before the lane's first)
template <int W>
__global__ __launch_bounds__(1024) void
k_gl_assign_v(KeySrc s, BUN n, const unsigned long long *gkey, const uint32_t *gmap, const uint32_t *gm, oid *gid,
	      uint8_t *img, unsigned long long *histo, uint32_t *unsorted, uint32_t *miss, const oid *ext, oid *flo)
{
	GL_ASSIGN_PROLOGUE;
	typedef typename std::conditional<W == 4, uint32_t, uint64_t>::type K;
	constexpr int V = 16 / W;
	__shared__ unsigned long long lkey[GL_SLOTS];
	__shared__ uint32_t lmap[GL_SLOTS + 1];
	__shared__ uint32_t lh[GL_MAXG];
	const unsigned tid = threadIdx.x;
	for (uint32_t q = tid; q < GL_SLOTS; q += blockDim.x) {
		lkey[q] = gkey[q];
		lmap[q] = gmap[q];
	}
	if (tid == 0)
		lmap[GL_SLOTS] = gmap[GL_SLOTS];
	for (uint32_t q = tid; q < ngrp; q += blockDim.x)
		lh[q] = 0;
	__syncthreads();
	const BUN a = (BUN) blockIdx.x * GL_TILE, e = min(n, a + GL_TILE);
	const K *kb = (const K *) s.base + s.off;
	uint32_t uns = 0;
	bool mis = false;
	typedef K kv __attribute__((ext_vector_type(V)));
	constexpr BUN STEP = 1024 * V;
	for (BUN r0 = a + (BUN) tid * V; r0 < e; r0 += STEP) {
		K k[V];
		if (r0 + V <= e) {
			const kv x = __builtin_nontemporal_load((const kv *) (kb + r0));
#pragma unroll
			for (int u = 0; u < V; u++)
				k[u] = x[u];
		} else {
#pragma unroll
			for (int u = 0; u < V; u++)
				k[u] = kb[r0 + u < e ? r0 + u : e - 1];
		}
		const K before = kb[r0 > 0 ? r0 - 1 : 0];
		uint32_t g[V], gp = 0;
#pragma unroll
		for (int u = 0; u < V; u++) {
			g[u] = gl_lookup(lkey, lmap, (uint64_t) k[u]);
			if (g[u] == ~0u) {
				mis = true;
				g[u] = 0;
			}
		}
		if (r0 > 0)
			gp = gl_lookup(lkey, lmap, (uint64_t) before);
		mis |= gp == ~0u && r0 > 0;
#pragma unroll
		for (int u = 0; u < V; u++) {
			const BUN i = r0 + u;
			if (i < e) {
				atomicAdd(&lh[g[u]], 1u);
				const uint32_t prev = u == 0 ? gp : g[u - 1];
				if (i > 0 && prev > g[u])
					uns = 1;
			}
		}
		if (r0 + V <= e) {
			typedef unsigned long long o2 __attribute__((ext_vector_type(2)));
#pragma unroll
			for (int u = 0; u < V; u += 2)
				__builtin_nontemporal_store((o2){g[u], g[u + 1]}, (o2 *) (gid + r0 + u));
			if (img) {
				if constexpr (V == 4) {
					const uint32_t w4 = g[0] | (g[1] << 8) | (g[2] << 16) | (g[3] << 24);
					*(uint32_t *) (img + r0) = w4;
				} else {
					*(uint16_t *) (img + r0) = (uint16_t) (g[0] | (g[1] << 8));
				}
			}
		} else {
#pragma unroll
			for (int u = 0; u < V; u++)
				if (r0 + u < e) {
					gid[r0 + u] = g[u];
					if (img)
						img[r0 + u] = (uint8_t) g[u];
				}
		}
	}
	if (__any(uns) && __lane_id() == 0)
		publish_or(unsorted, 1u);
	if (__any(mis) && __lane_id() == 0)
		publish_or(miss, 1u);
	__syncthreads();
	for (uint32_t q = tid; q < ngrp; q += blockDim.x)
		if (lh[q])
			atomicAdd(&histo[q], (unsigned long long) lh[q]);
}

// the assign pass for dense 4-byte keys without prior groups: the table is
// rebuilt per workgroup as ONE 8-byte LDS word per slot (key << 32 | id,
// ~0 = empty) under a 32-bit hash, so a probe is one LDS read and one
// 32-bit compare (the 8-byte key table + id map took two reads and 64-bit
// arithmetic), and the smaller table leaves room for a third workgroup per CU
__device__ __forceinline__ uint32_t
gl_hash32(uint32_t k)
{
	return (k * 0x9E3779B1u) >> 20;
}

__global__ __launch_bounds__(1024) void
k_gl_assign_v32(KeySrc s, BUN n, const unsigned long long *gkey, const uint32_t *gmap, const uint32_t *gm, oid *gid,
		uint8_t *img, unsigned long long *histo, uint32_t *unsorted, uint32_t *miss, const oid *ext, oid *flo)
{
	GL_ASSIGN_PROLOGUE;
	static_assert(GL_SLOTS == 4096, "12-bit hash");
	constexpr int V = 4;
	__shared__ unsigned long long tab[GL_SLOTS];
	__shared__ uint32_t lh[GL_MAXG];
	const unsigned tid = threadIdx.x;
	for (uint32_t q = tid; q < GL_SLOTS; q += blockDim.x)
		tab[q] = GL_EMPTY;
	for (uint32_t q = tid; q < ngrp; q += blockDim.x)
		lh[q] = 0;
	__syncthreads();
	for (uint32_t q = tid; q < GL_SLOTS; q += blockDim.x) {
		const unsigned long long k = gkey[q];
		if (k == GL_EMPTY)
			continue;
		const unsigned long long ent = (k << 32) | gmap[q];
		uint32_t h = gl_hash32((uint32_t) k);
		while (atomicCAS(&tab[h], GL_EMPTY, ent) != GL_EMPTY)
			h = (h + 1) & (GL_SLOTS - 1);
	}
	__syncthreads();
	auto look = [&](uint32_t k) -> uint32_t {
		uint32_t h = gl_hash32(k);
		for (;;) {
			const unsigned long long e = tab[h];
			if (e == GL_EMPTY)
				return ~0u;
			if ((uint32_t) (e >> 32) == k)
				return (uint32_t) e;
			h = (h + 1) & (GL_SLOTS - 1);
		}
	};
	const uint32_t *kb = (const uint32_t *) s.base + s.off;
	uint32_t uns = 0;
	bool mis = false;
	typedef uint32_t kv __attribute__((ext_vector_type(V)));
	constexpr BUN STEP = 1024 * V;
	// a grid smaller than the tile count keeps its table for several tiles
	for (BUN a = (BUN) blockIdx.x * GL_TILE; a < n; a += (BUN) gridDim.x * GL_TILE) {
		const BUN e = min(n, a + GL_TILE);
		for (BUN r0 = a + (BUN) tid * V; r0 < e; r0 += STEP) {
			uint32_t k[V];
			if (r0 + V <= e) {
#if MGDK_GL_NT_LOAD
				const kv x = __builtin_nontemporal_load((const kv *) (kb + r0));
#else
				const kv x = *(const kv *) (kb + r0);
#endif
#pragma unroll
				for (int u = 0; u < V; u++)
					k[u] = x[u];
			} else {
#pragma unroll
				for (int u = 0; u < V; u++)
					k[u] = kb[r0 + u < e ? r0 + u : e - 1];
			}
			const uint32_t before = kb[r0 > 0 ? r0 - 1 : 0];
			uint32_t g[V], gp = 0;
#pragma unroll
			for (int u = 0; u < V; u++) {
				g[u] = look(k[u]);
				if (g[u] == ~0u) {
					mis = true;
					g[u] = 0;
				}
			}
			if (r0 > 0)
				gp = look(before);
			mis |= gp == ~0u && r0 > 0;
#pragma unroll
			for (int u = 0; u < V; u++) {
				const BUN i = r0 + u;
				if (i < e) {
					atomicAdd(&lh[g[u]], 1u);
					const uint32_t prev = u == 0 ? gp : g[u - 1];
					if (i > 0 && prev > g[u])
						uns = 1;
				}
			}
			if (r0 + V <= e) {
				typedef unsigned long long o2 __attribute__((ext_vector_type(2)));
#if MGDK_GL_CSTORE
				// the wave's 256 ids as two 1-KiB pieces: store q takes rows
				// 128 q + 2 l, 2 l + 1 of the wave, held by lane 32 q + l / 2
				// (elements 2 (l & 1), + 1) -- one contiguous run per store
				// instruction instead of 16-B pieces at a 32-B stride
				const BUN wbase = r0 - (BUN) (tid & 63) * V;
				if (wbase + 256 <= e) {
					const unsigned l = tid & 63;
#pragma unroll
					for (int q = 0; q < 2; q++) {
						const int src = 32 * q + (int) (l >> 1);
						const uint32_t a0 = __shfl(g[0], src), a1 = __shfl(g[1], src);
						const uint32_t a2 = __shfl(g[2], src), a3 = __shfl(g[3], src);
						const bool odd = l & 1;
						const o2 val = (o2){odd ? a2 : a0, odd ? a3 : a1};
#if MGDK_GL_NT_STORE
						__builtin_nontemporal_store(val, (o2 *) (gid + wbase + 128 * q + 2 * l));
#else
						*(o2 *) (gid + wbase + 128 * q + 2 * l) = val;
#endif
					}
				} else
#endif
#pragma unroll
				for (int u = 0; u < V; u += 2) {
#if MGDK_GL_NT_STORE
					__builtin_nontemporal_store((o2){g[u], g[u + 1]}, (o2 *) (gid + r0 + u));
#else
					*(o2 *) (gid + r0 + u) = (o2){g[u], g[u + 1]};
#endif
				}
				if (img) {
					const uint32_t w4 = g[0] | (g[1] << 8) | (g[2] << 16) | (g[3] << 24);
					*(uint32_t *) (img + r0) = w4;
				}
			} else {
#pragma unroll
				for (int u = 0; u < V; u++)
					if (r0 + u < e) {
						gid[r0 + u] = g[u];
						if (img)
							img[r0 + u] = (uint8_t) g[u];
					}
			}
		}
	}
	if (__any(uns) && __lane_id() == 0)
		publish_or(unsorted, 1u);
	if (__any(mis) && __lane_id() == 0)
		publish_or(miss, 1u);
	__syncthreads();
	for (uint32_t q = tid; q < ngrp; q += blockDim.x)
		if (lh[q])
			atomicAdd(&histo[q], (unsigned long long) lh[q]);
}

// returns 1 when the path does not apply (too many groups).  The first
// pass reads only a prefix of GL_PREFIX tiles first: the groups it finds
// are numbered, and they are ALL the groups unless the assign pass meets a
// key the prefix did not hold (flagged) -- then the first pass reads every
// tile and the assign runs again.  A prefix group's first row lies inside
// the prefix, before any later group's, so the ids are the first-occurrence
// numbering either way (gdk_group.c:1118-1282).
constexpr unsigned GL_PREFIX = 4;

int
group_lds(const KeySrc &ks, BUN n, const Cand &ci, oid hseqb, mgdk_bat **gnp, mgdk_bat **enp, mgdk_bat **hnp)
{
	hipStream_t st = stream();
	DevBuf gkey((GL_SLOTS + 1) * 8), gmin((GL_SLOTS + 1) * 8), gmap((GL_SLOTS + 1) * 4);
	uint32_t *m = (uint32_t *) meta_buf();
	uint32_t *h = (uint32_t *) pinned(64);
	if (!gkey.p || !gmin.p || !gmap.p || m == nullptr || h == nullptr)
		return -1;
	hipLaunchKernelGGL(k_gl_init, dim3((GL_SLOTS + 256) / 256), dim3(256), 0, st, gkey.as<unsigned long long>(),
			   gmin.as<unsigned long long>(), m);
	const unsigned tiles = (unsigned) ((n + GL_TILE - 1) / GL_TILE);
	static const unsigned prefix = getenv("MGDK_GROUP_PREFIX") ? (unsigned) atoi(getenv("MGDK_GROUP_PREFIX")) : GL_PREFIX;
	// typed fast path: dense candidates, integer keys of 1-8 bytes
	const int fw = ks.dense && ks.kind <= 1 && ks.w <= 8 ? ks.w : 0;
	const int fg = !ks.has_g ? 0 : ks.g8 ? 1 : ks.g ? 2 : 3;
#define GL_LAUNCH(K, ...) do { \
		switch (fw * 4 + fg) { \
		case 4: hipLaunchKernelGGL((K<1, 0>), __VA_ARGS__); break; \
		case 5: hipLaunchKernelGGL((K<1, 1>), __VA_ARGS__); break; \
		case 6: hipLaunchKernelGGL((K<1, 2>), __VA_ARGS__); break; \
		case 7: hipLaunchKernelGGL((K<1, 3>), __VA_ARGS__); break; \
		case 8: hipLaunchKernelGGL((K<2, 0>), __VA_ARGS__); break; \
		case 9: hipLaunchKernelGGL((K<2, 1>), __VA_ARGS__); break; \
		case 10: hipLaunchKernelGGL((K<2, 2>), __VA_ARGS__); break; \
		case 11: hipLaunchKernelGGL((K<2, 3>), __VA_ARGS__); break; \
		case 16: hipLaunchKernelGGL((K<4, 0>), __VA_ARGS__); break; \
		case 17: hipLaunchKernelGGL((K<4, 1>), __VA_ARGS__); break; \
		case 18: hipLaunchKernelGGL((K<4, 2>), __VA_ARGS__); break; \
		case 19: hipLaunchKernelGGL((K<4, 3>), __VA_ARGS__); break; \
		case 32: hipLaunchKernelGGL((K<8, 0>), __VA_ARGS__); break; \
		case 33: hipLaunchKernelGGL((K<8, 1>), __VA_ARGS__); break; \
		case 34: hipLaunchKernelGGL((K<8, 2>), __VA_ARGS__); break; \
		case 35: hipLaunchKernelGGL((K<8, 3>), __VA_ARGS__); break; \
		default: hipLaunchKernelGGL((K<0, 0>), __VA_ARGS__); break; \
		} } while (0)
	unsigned done = 0;          // tiles the first pass has read
	unsigned upto = prefix > 0 && prefix < tiles ? prefix : tiles;
	for (;;) {
		const BUN frows = min(n, (BUN) upto * GL_TILE) - (BUN) done * GL_TILE;
		GL_LAUNCH(k_gl_first, dim3((unsigned) ((frows + GL_FTILE - 1) / GL_FTILE)), dim3(1024), 0, st, ks, n, (BUN) done,
			  gkey.as<unsigned long long>(), gmin.as<unsigned long long>(), &m[0]);
		done = upto;
		// group count not known yet: ids, extents and histogram sized for
		// the largest count this path takes; the ordering pass writes the
		// extents in place and clears the histogram
		mgdk_bat *en = newbat(0, MGDK_oid, GL_MAXG), *hn = newbat(0, MGDK_lng, GL_MAXG + 1), *gn = newbat(hseqb, MGDK_oid, n);
		auto unfix3 = [&]() {
			mgdk_BBPunfix(en);
			mgdk_BBPunfix(hn);
			mgdk_BBPunfix(gn);
		};
		if (!en || !hn || !gn) {
			unfix3();
			return -1;
		}
		hipLaunchKernelGGL(k_gl_order, dim3(GL_ORDER_WG), dim3(256), 0, st, gmin.as<unsigned long long>(), gmap.as<uint32_t>(),
				   ci.dense, ci.seq, ci.oids, (oid *) en->theap, &m[1], (unsigned long long *) hn->theap);
		gn->count = n;
		uint8_t *img = img8_new(gn);   // dropped below unless <= 255 groups
		if (img == nullptr) {
			unfix3();
			return -1;
		}
		// the vector form needs 16-byte aligned keys and ids
		const bool vec = fg == 0 && (fw == 4 || fw == 8) && (((uintptr_t) ks.base + ks.off * fw) & 15) == 0 &&
				 ((uintptr_t) gn->theap & 15) == 0 && ((uintptr_t) img & 3) == 0;
		static const bool v32 = getenv("MGDK_GROUP_V32") ? atoi(getenv("MGDK_GROUP_V32")) != 0 : true;
		const oid *extp = (const oid *) en->theap;
		oid *flo = (oid *) (m + 4);       // after the flags: one 32-B download
		// MGDK_GROUP_GRID: workgroups of the 4-byte assign pass (each keeps its
		// LDS table over grid-strided tiles); 0 = one per tile
		static const unsigned agrid = getenv("MGDK_GROUP_GRID") ? (unsigned) atoi(getenv("MGDK_GROUP_GRID")) : 0;
		if (vec && fw == 4 && v32)
			hipLaunchKernelGGL(k_gl_assign_v32, dim3(agrid && agrid < tiles ? agrid : tiles), dim3(1024), 0, st, ks, n, gkey.as<unsigned long long>(),
					   gmap.as<uint32_t>(), (const uint32_t *) m, (oid *) gn->theap, img,
					   (unsigned long long *) hn->theap, &m[2], &m[3], extp, flo);
		else if (vec && fw == 4)
			hipLaunchKernelGGL(k_gl_assign_v<4>, dim3(tiles), dim3(1024), 0, st, ks, n, gkey.as<unsigned long long>(),
					   gmap.as<uint32_t>(), (const uint32_t *) m, (oid *) gn->theap, img,
					   (unsigned long long *) hn->theap, &m[2], &m[3], extp, flo);
		else if (vec)
			hipLaunchKernelGGL(k_gl_assign_v<8>, dim3(tiles), dim3(1024), 0, st, ks, n, gkey.as<unsigned long long>(),
					   gmap.as<uint32_t>(), (const uint32_t *) m, (oid *) gn->theap, img,
					   (unsigned long long *) hn->theap, &m[2], &m[3], extp, flo);
		else
			GL_LAUNCH(k_gl_assign, dim3(tiles), dim3(1024), 0, st, ks, n, gkey.as<unsigned long long>(),
				  gmap.as<uint32_t>(), (const uint32_t *) m, (oid *) gn->theap, img,
				  (unsigned long long *) hn->theap, &m[2], &m[3], extp, flo);
		if (!hip_ok(hipMemcpyAsync(h, m, 32, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
			unfix3();
			return -1;
		}
		if (h[0] || h[1] > GL_MAXG) {
			unfix3();
			return 1;
		}
		const uint32_t ngrp = h[1];
		oid fl2[2];
		memcpy(fl2, h + 4, 16);
		if (ngrp > 255)
			img8_drop(gn);
		if (h[3]) {
			// a key the prefix did not hold: read the remaining tiles too
			unfix3();
			if (done == tiles) {
				seterr("BATgroup: a key missing from the complete table");
				return -1;
			}
			upto = tiles;
			continue;
		}
		gn->count = n;
		en->count = ngrp;
		hn->count = ngrp;
		gn->tsorted = h[2] == 0;
		gn->trevsorted = ngrp == 1 || n <= 1;
		gn->tkey = ngrp == n;
		gn->tnonil = 1;
		en->tsorted = en->tkey = en->tnonil = 1;
		en->trevsorted = ngrp == 1;
		hn->tkey = ngrp == 1;
		hn->tsorted = hn->trevsorted = ngrp == n || ngrp == 1;
		hn->tnonil = 1;
		// tmaxpos: the row that started the last group (maxgrppos,
		// gdk_group.c:99,1313)
		gn->tmaxpos = ngrp > 0 ? cand_index(ci, fl2[1]) : MGDK_BUN_NONE;
		if (ngrp > 0 && fl2[1] - fl2[0] == ngrp - 1)
			setdense(en, fl2[0], ngrp);
		*gnp = gn;
		*enp = en;
		*hnp = hn;
		return 0;
	}
#undef GL_LAUNCH
}

// ---------------------------------------------------------------------------
// Direct path for 1-byte keys (bte / bit / str with 1-byte offsets) with at
// most 32 prior groups -- GRP_small_values' domain (gdk_group.c:607-654):
// slot = prior group * 256 + key, at most 8192 slots, so every table is a
// plain LDS array (no hashing, no probing).
//   first  each workgroup (64 Ki rows, 16 independent rows per lane in
//          flight) records the first row of every slot it sees, merged into
//          the global table with one atomicMin per occupied slot;
//   order  one workgroup ranks the occupied slots by first row;
//   assign writes each row's group id (and the 1-byte image for <= 255
//          groups), counts per group in lane registers for <= 8 groups
//          (LDS atomics otherwise) and the order flag.
// ---------------------------------------------------------------------------
constexpr uint32_t GS_MAXSLOTS = 8192;
constexpr BUN GS_TILE = 65536;
constexpr int GS_U = 16;

// MODE 0: dense 1-byte keys; 1: dense keys + the prior groups' 1-byte image;
// 2: anything else (key_at).  Modes 0 / 1 are straight-line loads (a
// branchy loader makes the compiler wait for each load before the next).
template <int MODE>
__device__ __forceinline__ uint32_t
gs_slot(const KeySrc &s, BUN i)
{
	if constexpr (MODE == 0) {
		return ((const uint8_t *) s.base)[s.off + i];
	} else if constexpr (MODE == 1) {
		return ((uint32_t) s.g8[i] << 8) | ((const uint8_t *) s.base)[s.off + i];
	} else {
		uint64_t k0, k1, gg;
		key_at(s, i, k0, k1, gg);
		return (uint32_t) ((gg << 8) | (k0 & 0xff));
	}
}

template <int MODE>
__global__ __launch_bounds__(256) void
k_gs_first(KeySrc s, BUN n, uint32_t nslots, unsigned long long *gmin)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t lmin[];   // [nslots]: LDS sized to the slots used
	const unsigned tid = threadIdx.x;
	for (uint32_t q = tid; q < nslots; q += blockDim.x)
		lmin[q] = ~0u;
	__syncthreads();
	const BUN a = (BUN) blockIdx.x * GS_TILE, e = min(n, a + GS_TILE);
	for (BUN i0 = a; i0 < e; i0 += (BUN) blockDim.x * GS_U) {
		uint32_t sl[GS_U];
#pragma unroll
		for (int u = 0; u < GS_U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x + tid;
			const uint32_t x = gs_slot<MODE>(s, i < e ? i : e - 1);   // unconditional load, clamped
			sl[u] = i < e ? x : ~0u;
		}
#pragma unroll
		for (int u = 0; u < GS_U; u++) {
			const uint32_t r = (uint32_t) (i0 - a) + (uint32_t) u * blockDim.x + tid;
			if (sl[u] < nslots && lmin[sl[u]] > r)
				atomicMin(&lmin[sl[u]], r);
		}
	}
	__syncthreads();
	for (uint32_t q = tid; q < nslots; q += blockDim.x)
		if (lmin[q] != ~0u) {
			const unsigned long long f = a + lmin[q];
			if (gmin[q] > f)
				atomicMin(&gmin[q], f);
		}
}

__global__ __launch_bounds__(1024) void
k_gs_order(const unsigned long long *gmin, uint32_t nslots, uint32_t *gmap, bool cdense, oid cseq, const oid *coids,
	   oid *ext, uint32_t *ngrp)
{
	__shared__ unsigned long long sk[GS_MAXSLOTS];
	__shared__ uint32_t s_cnt;
	const unsigned tid = threadIdx.x;
	if (tid == 0)
		s_cnt = 0;
	__syncthreads();
	for (uint32_t q = tid; q < nslots; q += blockDim.x) {
		const unsigned long long f = gmin[q];
		if (f != ~0ull)
			sk[atomicAdd(&s_cnt, 1u)] = (f << 13) | q;
	}
	__syncthreads();
	const uint32_t c = s_cnt;
	for (uint32_t i = tid; i < c; i += blockDim.x) {
		const unsigned long long v = sk[i];
		uint32_t r = 0;
		for (uint32_t j = 0; j < c; j++)
			r += sk[j] < v;
		const uint32_t slot = (uint32_t) (v & 8191);
		gmap[slot] = r;
		ext[r] = cdense ? cseq + (BUN) (v >> 13) : coids[v >> 13];
	}
	if (tid == 0)
		*ngrp = c;
}

template <int K, int MODE>
__global__ __launch_bounds__(256) void
k_gs_assign(KeySrc s, BUN n, const uint32_t *gmap, uint32_t nslots, uint32_t ngrp, oid *gid, uint8_t *img,
	    unsigned long long *histo, uint32_t *unsorted)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t lmap[];   // [nslots] + [ngrp] histogram (K == 0)
	uint32_t *lh = lmap + nslots;
	const unsigned tid = threadIdx.x, lane = __lane_id();
	for (uint32_t q = tid; q < nslots; q += blockDim.x)
		lmap[q] = gmap[q];
	if (K == 0)
		for (uint32_t q = tid; q < ngrp; q += blockDim.x)
			lh[q] = 0;
	__syncthreads();
	uint32_t cnt[K > 0 ? K : 1];
#pragma unroll
	for (int k = 0; k < (K > 0 ? K : 1); k++)
		cnt[k] = 0;
	const BUN a = (BUN) blockIdx.x * GS_TILE, e = min(n, a + GS_TILE);
	uint32_t uns = 0;
	for (BUN i0 = a; i0 < e; i0 += (BUN) blockDim.x * GS_U) {
		uint32_t sl[GS_U];
#pragma unroll
		for (int u = 0; u < GS_U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x + tid;
			const uint32_t x = gs_slot<MODE>(s, i < e ? i : e - 1);   // unconditional load, clamped
			sl[u] = i < e ? x : ~0u;
		}
		uint32_t prev = 0;
		if (lane == 0 && i0 + tid > 0 && i0 + tid < e)
			prev = lmap[gs_slot<MODE>(s, i0 + tid - 1)];
#pragma unroll
		for (int u = 0; u < GS_U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x + tid;
			const uint32_t g = sl[u] < nslots ? lmap[sl[u]] : 0;
			if (i < e) {
				gid[i] = g;
				if (img)
					img[i] = (uint8_t) g;
				if (K > 0) {
#pragma unroll
					for (int k = 0; k < K; k++)
						cnt[k] += g == (uint32_t) k;
				} else {
					atomicAdd(&lh[g], 1u);
				}
			}
			// order flag: the previous row is the previous lane's (lane 0:
			// the last lane of the previous row group, looked up directly)
			uint32_t gp = __shfl_up(g, 1);
			if (lane == 0) {
				if (u == 0)
					gp = prev;
				else if (i < e)     // rows past the tile end read nothing
					gp = lmap[gs_slot<MODE>(s, i - 1)];
			}
			if (i > 0 && i < e && gp > g)
				uns = 1;
		}
	}
	if (__any(uns) && lane == 0)
		publish_or(unsorted, 1u);
	if (K > 0) {
		// per-workgroup counts to histo_part[tile][k] (summed by k_gs_hist):
		// no same-word atomics from every wave
		__shared__ uint32_t s_c[4][K > 0 ? K : 1];
#pragma unroll
		for (int k = 0; k < K; k++) {
			uint32_t c = cnt[k];
			for (int o = 32; o > 0; o >>= 1)
				c += __shfl_xor(c, o);
			if (lane == 0)
				s_c[tid / 64][k] = c;
		}
		__syncthreads();
		if (tid < (unsigned) K)
			histo[(BUN) blockIdx.x * K + tid] = (unsigned long long) s_c[0][tid] + s_c[1][tid] + s_c[2][tid] + s_c[3][tid];
	} else {
		__syncthreads();
		for (uint32_t q = tid; q < ngrp; q += blockDim.x)
			if (lh[q])
				atomicAdd(&histo[q], (unsigned long long) lh[q]);
	}
}

// modes 0 / 1 with 16-byte aligned keys: 16-byte key / prior-id loads per
// lane, transposed through LDS so that the id and image stores coalesce; the
// order flag across lanes by shuffles
template <int K, int MODE>
__global__ __launch_bounds__(256) void
k_gs_assign16(KeySrc s, BUN n, const uint32_t *gmap, uint32_t nslots, uint32_t ngrp, oid *gid, uint8_t *img,
	      unsigned long long *histo, uint32_t *unsorted)
{
	extern __shared__ __attribute__((aligned(16))) uint32_t lmap[];   // [nslots] + [ngrp] histogram (K == 0)
	uint32_t *lh = lmap + nslots;
	const unsigned tid = threadIdx.x, lane = __lane_id();
	for (uint32_t q = tid; q < nslots; q += blockDim.x)
		lmap[q] = gmap[q];
	if (K == 0)
		for (uint32_t q = tid; q < ngrp; q += blockDim.x)
			lh[q] = 0;
	__syncthreads();
	uint32_t cnt[K > 0 ? K : 1];
#pragma unroll
	for (int k = 0; k < (K > 0 ? K : 1); k++)
		cnt[k] = 0;
	const BUN a = (BUN) blockIdx.x * GS_TILE, e = min(n, a + GS_TILE);
	uint32_t uns = 0;
	const uint8_t *keys = (const uint8_t *) s.base + s.off;
	// keys (and prior ids) are read lane-contiguously -- one 16-byte load per
	// lane covers the wave's 1024 rows -- and transposed through the wave's
	// LDS slot, so that row = wave base + u * 64 + lane and every id / image
	// store instruction writes 64 consecutive rows (16-row runs per lane made
	// each store touch 64 cache lines).  Block addresses are clamped to the
	// last aligned block (rows past the tile end are masked), so no branch.
	__shared__ uint4 s_kq[4][64], s_gq[4][MODE == 1 ? 64 : 1];
	const unsigned w = tid / 64;
	const BUN last = (n - 1) & ~(BUN) 15;
	for (BUN wb = a + (BUN) w * 1024; wb < e; wb += (BUN) blockDim.x * 16) {
		const BUN ga = wb + (BUN) lane * 16 <= last ? wb + (BUN) lane * 16 : last;
		s_kq[w][lane] = *(const uint4 *) (keys + ga);
		if (MODE == 1)
			s_gq[w][lane] = *(const uint4 *) (s.g8 + ga);
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		const uint8_t *kb = (const uint8_t *) s_kq[w], *gb = (const uint8_t *) s_gq[w];
		uint32_t g[16];
#pragma unroll
		for (int u = 0; u < 16; u++) {
			const uint32_t k = kb[u * 64 + lane];
			const uint32_t pg = MODE == 1 ? gb[u * 64 + lane] : 0u;
			const uint32_t sl = (pg << 8) | k;     // bytes past n (masked rows) may hold anything
			g[u] = lmap[sl < nslots ? sl : 0];
		}
		__builtin_amdgcn_wave_barrier();
		// the row before the wave base: looked up directly (lane 0)
		uint32_t gprev = 0;
		if (lane == 0 && wb > 0)
			gprev = lmap[gs_slot<MODE>(s, wb - 1)];
#pragma unroll
		for (int u = 0; u < 16; u++) {
			const BUN i = wb + (BUN) u * 64 + lane;
			const bool ok = i < e;
			if (ok) {
				gid[i] = g[u];
				if (img)
					img[i] = (uint8_t) g[u];
			}
			if (K > 0) {
#pragma unroll
				for (int k = 0; k < K; k++)
					cnt[k] += ok && g[u] == (uint32_t) k;
			} else if (ok) {
				atomicAdd(&lh[g[u]], 1u);
			}
			// previous row: lane - 1 of this step; for lane 0 lane 63 of the
			// step before (or the looked-up row before the wave base)
			const uint32_t up = __shfl_up(g[u], 1);
			const uint32_t l63 = __shfl(g[u > 0 ? u - 1 : 0], 63);
			const uint32_t gp = lane ? up : u == 0 ? gprev : l63;
			if (ok && i > 0 && gp > g[u])
				uns = 1;
		}
	}
	if (__any(uns) && lane == 0)
		publish_or(unsorted, 1u);
	if (K > 0) {
		// per-workgroup counts to histo_part[tile][k] (summed by k_gs_hist):
		// no same-word atomics from every wave
		__shared__ uint32_t s_c[4][K > 0 ? K : 1];
#pragma unroll
		for (int k = 0; k < K; k++) {
			uint32_t c = cnt[k];
			for (int o = 32; o > 0; o >>= 1)
				c += __shfl_xor(c, o);
			if (lane == 0)
				s_c[tid / 64][k] = c;
		}
		__syncthreads();
		if (tid < (unsigned) K)
			histo[(BUN) blockIdx.x * K + tid] = (unsigned long long) s_c[0][tid] + s_c[1][tid] + s_c[2][tid] + s_c[3][tid];
	} else {
		__syncthreads();
		for (uint32_t q = tid; q < ngrp; q += blockDim.x)
			if (lh[q])
				atomicAdd(&histo[q], (unsigned long long) lh[q]);
	}
}

// histo[k] = the sum of the per-tile counts (one workgroup per group)
__global__ __launch_bounds__(256) void
k_gs_hist(const unsigned long long *part, BUN tiles, int K, BUN ngrp, unsigned long long *histo)
{
	const int k = blockIdx.x;
	unsigned long long c = 0;
	for (BUN t = threadIdx.x; t < tiles; t += blockDim.x)
		c += part[t * K + k];
	c = block_reduce(c, [](unsigned long long x, unsigned long long y) { return x + y; });
	if (threadIdx.x == 0 && (BUN) k < ngrp)
		histo[k] = c;
}

int
group_small(const KeySrc &ks, BUN n, uint32_t nslots, const Cand &ci, oid hseqb, mgdk_bat **gnp, mgdk_bat **enp,
	    mgdk_bat **hnp)
{
	hipStream_t st = stream();
	DevBuf gmin(GS_MAXSLOTS * 8), gmap(GS_MAXSLOTS * 4), ext(GS_MAXSLOTS * 8);
	uint32_t *m = (uint32_t *) meta_buf();
	uint32_t *h = (uint32_t *) pinned(32);
	if (!gmin.p || !gmap.p || !ext.p)
		return -1;
	if (!hip_ok(hipMemsetAsync(gmin.p, 0xff, nslots * 8, st), "memset") || !hip_ok(hipMemsetAsync(m, 0, 16, st), "memset"))
		return -1;
	const unsigned tiles = (unsigned) ((n + GS_TILE - 1) / GS_TILE);
	const int mode = (ks.dense && !ks.has_g) ? 0 : (ks.dense && ks.g8) ? 1 : 2;
	if (mode == 0)
		hipLaunchKernelGGL((k_gs_first<0>), dim3(tiles), dim3(256), nslots * 4, st, ks, n, nslots, gmin.as<unsigned long long>());
	else if (mode == 1)
		hipLaunchKernelGGL((k_gs_first<1>), dim3(tiles), dim3(256), nslots * 4, st, ks, n, nslots, gmin.as<unsigned long long>());
	else
		hipLaunchKernelGGL((k_gs_first<2>), dim3(tiles), dim3(256), nslots * 4, st, ks, n, nslots, gmin.as<unsigned long long>());
	hipLaunchKernelGGL(k_gs_order, dim3(1), dim3(1024), 0, st, gmin.as<unsigned long long>(), nslots, gmap.as<uint32_t>(),
			   ci.dense, ci.seq, ci.oids, ext.as<oid>(), &m[1]);
	if (!hip_ok(hipMemcpyAsync(h, m, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	const uint32_t ngrp = h[1];
	mgdk_bat *en = newbat(0, MGDK_oid, ngrp), *hn = newbat(0, MGDK_lng, ngrp), *gn = newbat(hseqb, MGDK_oid, n);
	uint8_t *img = nullptr;
	if (gn)
		gn->count = n;
	if (!en || !hn || !gn || !hip_ok(hipMemsetAsync(hn->theap, 0, ngrp * 8 + 8, st), "memset") ||
	    !hip_ok(hipMemcpyAsync(en->theap, ext.p, ngrp * 8, hipMemcpyDeviceToDevice, st), "memcpy") ||
	    (ngrp <= 255 && (img = img8_new(gn)) == nullptr)) {
		mgdk_BBPunfix(en);
		mgdk_BBPunfix(hn);
		mgdk_BBPunfix(gn);
		return -1;
	}
	DevBuf hpart((BUN) tiles * 8 * 8);
	if (hpart.p == nullptr) {
		mgdk_BBPunfix(en);
		mgdk_BBPunfix(hn);
		mgdk_BBPunfix(gn);
		return -1;
	}
	unsigned long long *hdst = ngrp <= 8 ? hpart.as<unsigned long long>() : (unsigned long long *) hn->theap;
	const int kk = ngrp <= 1 ? 1 : ngrp <= 4 ? 4 : 8;
#define GSA2(K_, M_) hipLaunchKernelGGL((k_gs_assign<K_, M_>), dim3(tiles), dim3(256), (nslots + ((K_) == 0 ? ngrp : 0)) * 4, st, ks, n, gmap.as<uint32_t>(), nslots, ngrp, \
				   (oid *) gn->theap, img, hdst, &m[2])
#define GSA16(K_, M_) hipLaunchKernelGGL((k_gs_assign16<K_, M_>), dim3(tiles), dim3(256), (nslots + ((K_) == 0 ? ngrp : 0)) * 4, st, ks, n, gmap.as<uint32_t>(), nslots, ngrp, \
				   (oid *) gn->theap, img, hdst, &m[2])
	const bool al16 = (((uintptr_t) ks.base + ks.off) & 15) == 0;
#define GSA(K_) do { if (mode == 0 && al16) GSA16(K_, 0); else if (mode == 1 && al16) GSA16(K_, 1); \
		else if (mode == 0) GSA2(K_, 0); else if (mode == 1) GSA2(K_, 1); else GSA2(K_, 2); } while (0)
	if (ngrp <= 1)
		GSA(1);
	else if (ngrp <= 4)
		GSA(4);
	else if (ngrp <= 8)
		GSA(8);
	else
		GSA(0);
#undef GSA
#undef GSA2
#undef GSA16
	if (ngrp <= 8 && ngrp > 0)
		hipLaunchKernelGGL(k_gs_hist, dim3(kk), dim3(256), 0, st, hpart.as<unsigned long long>(), (BUN) tiles, kk, (BUN) ngrp,
				   (unsigned long long *) hn->theap);
	// the first / last extent into the pinned buffer too (not pageable stack memory)
	oid fl[2] = {0, 0};
	if (!hip_ok(hipMemcpyAsync(h, m, 12, hipMemcpyDeviceToHost, st), "memcpy") ||
	    (ngrp > 0 && (!hip_ok(hipMemcpyAsync(h + 4, ext.p, 8, hipMemcpyDeviceToHost, st), "memcpy") ||
			  !hip_ok(hipMemcpyAsync(h + 6, ext.as<oid>() + ngrp - 1, 8, hipMemcpyDeviceToHost, st), "memcpy"))) ||
	    !sync()) {
		mgdk_BBPunfix(en);
		mgdk_BBPunfix(hn);
		mgdk_BBPunfix(gn);
		return -1;
	}
	en->count = ngrp;
	hn->count = ngrp;
	if (ngrp > 0)
		memcpy(fl, h + 4, 16);
	gn->tsorted = h[2] == 0;
	gn->trevsorted = ngrp == 1 || n <= 1;
	gn->tkey = ngrp == n;
	gn->tnonil = 1;
	en->tsorted = en->tkey = en->tnonil = 1;
	en->trevsorted = ngrp == 1;
	hn->tkey = ngrp == 1;
	hn->tsorted = hn->trevsorted = ngrp == n || ngrp == 1;
	hn->tnonil = 1;
	gn->tmaxpos = ngrp > 0 ? cand_index(ci, fl[1]) : MGDK_BUN_NONE;
	if (ngrp > 0 && fl[1] - fl[0] == ngrp - 1)
		setdense(en, fl[0], ngrp);
	*gnp = gn;
	*enp = en;
	*hnp = hn;
	return 0;
}

mgdk_bat *
dense_or_copy(const Cand &ci)
{
	if (ci.dense)
		return mgdk_BATdense(0, ci.seq, ci.n);
	mgdk_bat *bn = newbat(0, MGDK_oid, ci.n);
	if (bn && hip_ok(hipMemcpyAsync(bn->theap, ci.oids, ci.n * 8, hipMemcpyDeviceToDevice, stream()), "memcpy") && sync()) {
		bn->count = ci.n;
		bn->tsorted = bn->tkey = bn->tnonil = 1;
		bn->trevsorted = ci.n <= 1;
		return bn;
	}
	mgdk_BBPunfix(bn);
	return nullptr;
}

// ---- ordered keys: GRP_compare_consecutive_values (gdk_group.c:103-175,
// chosen at :940-975 when b is sorted or reverse sorted and g is ordered):
// a new group wherever the (prior group, value) pair differs from the row
// before, so ids are a running count of those starts
__global__ __launch_bounds__(256) void
k_grp_seq_flags(KeySrc s, BUN n, uint8_t *fl)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		uint64_t a0, a1, ag, b0, b1, bg;
		key_at(s, i, a0, a1, ag);
		bool nw = i == 0;
		if (!nw) {
			key_at(s, i - 1, b0, b1, bg);
			nw = a0 != b0 || a1 != b1 || ag != bg;
		}
		fl[i] = nw;
	}
}

__global__ __launch_bounds__(256) void
k_grp_seq_ids(BUN n, const uint8_t *fl, const uint64_t *ex, oid *gid, uint64_t *spos)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint64_t k = ex[i] + fl[i] - 1;
		gid[i] = k;
		if (fl[i])
			spos[k] = i;
	}
}

__global__ __launch_bounds__(256) void
k_grp_seq_ext(BUN ngrp, BUN n, const uint64_t *spos, bool cdense, oid cseq, const oid *coids, oid *en,
	      int64_t *hn)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ngrp; k += (BUN) gridDim.x * blockDim.x) {
		const uint64_t p = spos[k];
		en[k] = cdense ? cseq + p : coids[p];
		if (hn)                         // (uniform: no histogram asked for)
			hn[k] = (int64_t) ((k + 1 < ngrp ? spos[k + 1] : n) - p);
	}
}

// histogram from extents that hold the group starts as oids (dense
// candidates: the write pass stored cseq + start row straight into them)
__global__ __launch_bounds__(256) void
k_grp_seq_hist(BUN ngrp, oid end, const oid *en, int64_t *hn)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < ngrp; k += (BUN) gridDim.x * blockDim.x)
		hn[k] = (int64_t) ((k + 1 < ngrp ? en[k + 1] : end) - en[k]);
}

// Dense candidates: the same starts in two passes over the keys instead of
// flags -> 8-byte scan -> ids (three passes and 8 B of scan per row): a
// count of the starts per 2048-row tile, a scan of the tile counts, then
// the starts again, ranked in the tile by one ballot per 64 rows and a
// 32-entry LDS scan, the ids stored where the rows are.  Key width, float
// normalisation and the prior-group source are template parameters, so
// every key load of a lane is in flight before the first compare.
constexpr int SQU = 8;
constexpr BUN SQT = 256 * SQU;

template <int W, bool FL>
__device__ __forceinline__ void
keyw(const void *base, BUN p, uint64_t &k0, uint64_t &k1)
{
	k1 = 0;
	if constexpr (W == 1) {
		k0 = ((const uint8_t *) base)[p];
	} else if constexpr (W == 2) {
		k0 = ((const uint16_t *) base)[p];
	} else if constexpr (W == 4) {
		const uint32_t u = ((const uint32_t *) base)[p];
		if (FL) {
			const float f = __uint_as_float(u);
			k0 = f != f ? 0x7fc00000u : f == 0.0f ? 0 : u;
		} else {
			k0 = u;
		}
	} else if constexpr (W == 8) {
		const uint64_t u = ((const uint64_t *) base)[p];
		if (FL) {
			const double d = __longlong_as_double((long long) u);
			k0 = d != d ? 0x7ff8000000000000ull : d == 0.0 ? 0 : u;
		} else {
			k0 = u;
		}
	} else {
		k0 = ((const uint64_t *) base)[2 * p];
		k1 = ((const uint64_t *) base)[2 * p + 1];
	}
}

// GK: 0 no prior groups, 1 their 1-byte image, 2 oid ids, 3 dense ids
template <int GK>
__device__ __forceinline__ uint64_t
gval(const KeySrc &s, BUN i)
{
	if constexpr (GK == 0)
		return 0;
	else if constexpr (GK == 1)
		return s.g8[i];
	else if constexpr (GK == 2)
		return s.g[i];
	else
		return s.gseq + i;
}

// start flags of the tile's rows t0 + u * 256 + tid (row 0 starts)
template <int W, bool FL, int GK>
__device__ __forceinline__ void
sq_starts(const KeySrc &s, BUN n, BUN t0, bool st[SQU])
{
	uint64_t a0[SQU], a1[SQU], ag[SQU], b0[SQU], b1[SQU], bg[SQU];
#pragma unroll
	for (int u = 0; u < SQU; u++) {
		const BUN i = t0 + (BUN) u * 256 + threadIdx.x;
		const BUN ic = i < n ? i : n - 1, ip = ic ? ic - 1 : 0;
		keyw<W, FL>(s.base, s.off + ic, a0[u], a1[u]);
		keyw<W, FL>(s.base, s.off + ip, b0[u], b1[u]);
		ag[u] = gval<GK>(s, ic);
		bg[u] = gval<GK>(s, ip);
	}
#pragma unroll
	for (int u = 0; u < SQU; u++) {
		const BUN i = t0 + (BUN) u * 256 + threadIdx.x;
		st[u] = i < n && (i == 0 || a0[u] != b0[u] || a1[u] != b1[u] || ag[u] != bg[u]);
	}
}

template <int W, bool FL, int GK>
__global__ __launch_bounds__(256) void
k_sq_count(KeySrc s, BUN n, uint32_t *tcnt)
{
	bool st[SQU];
	sq_starts<W, FL, GK>(s, n, (BUN) blockIdx.x * SQT, st);
	uint32_t c = 0;
#pragma unroll
	for (int u = 0; u < SQU; u++)
		c += st[u];
	c = block_reduce(c, [](uint32_t x, uint32_t y) { return x + y; });
	if (threadIdx.x == 0)
		tcnt[blockIdx.x] = c;
}

template <int W, bool FL, int GK>
__global__ __launch_bounds__(256) void
k_sq_write(KeySrc s, BUN n, const uint64_t *tpre, oid *gid, uint64_t *spos, uint64_t soff)
{
	__shared__ uint32_t tab[SQU * 4];
	const int lane = __lane_id(), w = threadIdx.x >> 6;
	const BUN t0 = (BUN) blockIdx.x * SQT;
	bool st[SQU];
	sq_starts<W, FL, GK>(s, n, t0, st);
	unsigned long long bal[SQU];
#pragma unroll
	for (int u = 0; u < SQU; u++) {
		bal[u] = __ballot(st[u]);
		if (lane == 0)
			tab[u * 4 + w] = (uint32_t) __popcll(bal[u]);
	}
	__syncthreads();
	if (threadIdx.x < 64) {
		// exclusive scan of the (row group, wave) counts in row order
		uint32_t v = threadIdx.x < SQU * 4 ? tab[threadIdx.x] : 0, x = v;
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const uint32_t t = __shfl_up(x, d);
			if (lane >= d)
				x += t;
		}
		if (threadIdx.x < SQU * 4)
			tab[threadIdx.x] = x - v;
	}
	__syncthreads();
	const uint64_t base = tpre[blockIdx.x];
	const unsigned long long lt = (1ull << lane) - 1;
#pragma unroll
	for (int u = 0; u < SQU; u++) {
		const BUN i = t0 + (BUN) u * 256 + threadIdx.x;
		if (i < n) {
			// starts up to and including row i, minus one
			const uint64_t k = base + tab[u * 4 + w] + (uint64_t) __popcll(bal[u] & lt) + st[u] - 1;
			gid[i] = k;
			if (st[u])
				spos[k] = soff + i;
		}
	}
}

template <int W, bool FL, int GK>
static int
sq_ids(const KeySrc &ks, BUN n, DevBuf &tc, DevBuf &tp, oid *gid, uint64_t *spos, uint64_t *ngrp, bool write,
       uint64_t soff)
{
	hipStream_t st = stream();
	const BUN nt = (n + SQT - 1) / SQT;
	if (!write) {
		hipLaunchKernelGGL((k_sq_count<W, FL, GK>), dim3(nt), dim3(256), 0, st, ks, n, tc.as<uint32_t>());
		return exclusive_scan(tc.as<uint32_t>(), tp.as<uint64_t>(), nt, ngrp);
	}
	hipLaunchKernelGGL((k_sq_write<W, FL, GK>), dim3(nt), dim3(256), 0, st, ks, n, tp.as<uint64_t>(), gid, spos, soff);
	return 0;
}

template <int W, bool FL>
static int
sq_ids_g(const KeySrc &ks, BUN n, DevBuf &tc, DevBuf &tp, oid *gid, uint64_t *spos, uint64_t *ngrp, bool write,
	 uint64_t soff)
{
	if (!ks.has_g)
		return sq_ids<W, FL, 0>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
	if (ks.g8)
		return sq_ids<W, FL, 1>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
	if (ks.g)
		return sq_ids<W, FL, 2>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
	return sq_ids<W, FL, 3>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
}

static int
sq_dispatch(const KeySrc &ks, BUN n, DevBuf &tc, DevBuf &tp, oid *gid, uint64_t *spos, uint64_t *ngrp, bool write,
	    uint64_t soff = 0)
{
	switch (ks.w) {
	case 1: return sq_ids_g<1, false>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
	case 2: return sq_ids_g<2, false>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
	case 4: return ks.kind == 2 ? sq_ids_g<4, true>(ks, n, tc, tp, gid, spos, ngrp, write, soff)
				    : sq_ids_g<4, false>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
	case 8: return ks.kind == 3 ? sq_ids_g<8, true>(ks, n, tc, tp, gid, spos, ngrp, write, soff)
				    : sq_ids_g<8, false>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
	default: return sq_ids_g<16, false>(ks, n, tc, tp, gid, spos, ngrp, write, soff);
	}
}

int
group_ordered(const KeySrc &ks, BUN n, const Cand &ci, oid hseqb, mgdk_bat **gnp, mgdk_bat **enp,
	      mgdk_bat **hnp, bool want_h)
{
	hipStream_t st = stream();
	const dim3 grd(grid_for(n, 1024, 8192)), blk(256);
	static const bool two = getenv("MGDK_GROUP_SEQ2") ? atoi(getenv("MGDK_GROUP_SEQ2")) != 0 : true;
	const bool fast = two && ks.dense && n > 0;
	// dense candidates: the write pass stores each group's start (cseq +
	// row) straight into the extents; the histogram, when wanted, is the
	// difference of neighbouring extents (no start-row array, no pass that
	// reads it to write the extents)
	const bool direct = fast && ci.dense;
	const BUN nt = (n + SQT - 1) / SQT;
	DevBuf fl(fast ? 0 : n + 8), ex(fast ? 0 : n * 8 + 8), tc(fast ? nt * 4 + 8 : 0), tp(fast ? nt * 8 + 8 : 0);
	if ((!fast && (!fl.p || !ex.p)) || (fast && (!tc.p || !tp.p)))
		return -1;
	uint64_t ngrp = 0;
	if (fast) {
		if (sq_dispatch(ks, n, tc, tp, nullptr, nullptr, &ngrp, false) < 0)
			return -1;
	} else {
		hipLaunchKernelGGL(k_grp_seq_flags, grd, blk, 0, st, ks, n, fl.as<uint8_t>());
		if (exclusive_scan(fl.as<uint8_t>(), ex.as<uint64_t>(), n, &ngrp) < 0)
			return -1;
	}
	DevBuf spos(direct ? 8 : ngrp * 8 + 8);
	mgdk_bat *gn = newbat(hseqb, MGDK_oid, n), *en = newbat(0, MGDK_oid, ngrp);
	mgdk_bat *hn = want_h ? newbat(0, MGDK_lng, ngrp) : nullptr;
	if (!gn || !en || (want_h && !hn) || !spos.p) {
		mgdk_BBPunfix(gn);
		mgdk_BBPunfix(en);
		mgdk_BBPunfix(hn);
		return -1;
	}
	uint64_t *starts = direct ? (uint64_t *) en->theap : spos.as<uint64_t>();
	if (fast)
		sq_dispatch(ks, n, tc, tp, (oid *) gn->theap, starts, nullptr, true, direct ? ci.seq : 0);
	else
		hipLaunchKernelGGL(k_grp_seq_ids, grd, blk, 0, st, n, fl.as<uint8_t>(), ex.as<uint64_t>(), (oid *) gn->theap,
				   spos.as<uint64_t>());
	if (direct) {
		if (want_h && ngrp)
			hipLaunchKernelGGL(k_grp_seq_hist, dim3(grid_for(ngrp, 1024, 8192)), blk, 0, st, ngrp,
					   (oid) (ci.seq + n), (const oid *) en->theap, (int64_t *) hn->theap);
	} else {
		hipLaunchKernelGGL(k_grp_seq_ext, dim3(grid_for(ngrp, 1024, 8192)), blk, 0, st, ngrp, n, spos.as<uint64_t>(),
				   ci.dense, ci.seq, ci.oids, (oid *) en->theap, want_h ? (int64_t *) hn->theap : nullptr);
	}
	uint64_t *hl = (uint64_t *) pinned(16);
	if (!hip_ok(hipMemcpyAsync(hl, starts + ngrp - 1, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
		mgdk_BBPunfix(gn);
		mgdk_BBPunfix(en);
		mgdk_BBPunfix(hn);
		return -1;
	}
	gn->count = n;
	gn->tsorted = 1;
	gn->trevsorted = ngrp == 1 || n <= 1;
	gn->tkey = ngrp == n;
	gn->tnonil = 1;
	gn->tmaxpos = direct ? hl[0] - ci.seq : hl[0];
	en->count = ngrp;
	en->tsorted = en->tkey = en->tnonil = 1;
	en->trevsorted = ngrp == 1;
	if (hn) {
		hn->count = ngrp;
		hn->tkey = ngrp == 1;
		hn->tsorted = hn->trevsorted = ngrp == n || ngrp == 1;
		hn->tnonil = 1;
	}
	oid fl2[2];
	if (oid_at(en, 0, &fl2[0]) < 0 || oid_at(en, ngrp - 1, &fl2[1]) < 0) {
		mgdk_BBPunfix(gn);
		mgdk_BBPunfix(en);
		mgdk_BBPunfix(hn);
		return -1;
	}
	if (fl2[1] - fl2[0] == ngrp - 1)
		setdense(en, fl2[0], ngrp);
	*gnp = gn;
	*enp = en;
	*hnp = hn;
	return 0;
}

int
key_kind(int tt)
{
	switch (tt) {
	case MGDK_str: return 1;
	case MGDK_flt: return 2;
	case MGDK_dbl: return 3;
	default: return 0;
	}
}

}  // namespace

// BATgroup by the storage value (for str: by heap offset, exact when the
// heap is duplicate eliminated)
static int
group_core(mgdk_bat **groups, mgdk_bat **extents, mgdk_bat **histo, mgdk_bat *b, mgdk_bat *s,
	   mgdk_bat *g, mgdk_bat *e, mgdk_bat *h)
{
	(void) h;
	if (b == nullptr || groups == nullptr) {
		seterr("b must exist\n");
		return -1;
	}
	if (b->ttype == MGDK_void || b->ttype == MGDK_msk) {
		seterr("42000!BATgroup: type %s not supported on the device path", atomname(b->ttype));
		return -1;
	}
	ProfScope prof("group");
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return -1;
	const BUN n = ci.n;
	const oid hseqb = n ? ci.first : 0;
	if (g && g->count != n) {
		seterr("b with s and g must be aligned\n");
		return -1;
	}
	mgdk_bat *gn = nullptr, *en = nullptr, *hn = nullptr;
	bool grouped = false;   // the general path ran (it sets the estimates)
	// trivial: one element per group (gdk_group.c:712-767)
	if (b->tkey || n <= 1 || (g && (g->tkey || g->ttype == MGDK_void))) {
		gn = mgdk_BATdense(hseqb, 0, b->count);
		en = dense_or_copy(ci);
		long long one = 1;
		hn = mgdk_BATconstant(0, MGDK_lng, &one, n);
		if (!gn || !en || !hn)
			goto fail;
		goto done;
	}
	// the order of b is established first (gdk_group.c:764-765), so a
	// sorted column whose property is not set yet (e.g. the concatenation of
	// the ranks' sorted partial keys after an exchange) takes the
	// consecutive-comparison path below; str order is by content, which the
	// offsets do not show
	if (b->ttype != MGDK_str) {
		(void) mgdk_BATordered(b);
		(void) mgdk_BATordered_rev(b);
	}
	// all values equal and no (or a constant) prior grouping: one group
	// (gdk_group.c:768-770 evaluates BATordered / BATordered_rev on g)
	if (b->tsorted && b->trevsorted && (!g || (mgdk_BATordered(g) && mgdk_BATordered_rev(g)))) {
		oid zero = 0;
		gn = mgdk_BATconstant(hseqb, MGDK_oid, &zero, n);
		en = mgdk_BATdense(0, ci.first, 1);
		long long cnt = (long long) n;
		hn = mgdk_BATconstant(0, MGDK_lng, &cnt, 1);
		if (!gn || !en || !hn)
			goto fail;
		gn->tsorted = gn->trevsorted = 1;
		gn->tkey = n <= 1;
		goto done;
	}
	grouped = true;
	{
		KeySrc ks{};
		ks.base = b->theap;
		ks.w = b->twidth;
		ks.kind = key_kind(b->ttype);
		ks.dense = ci.dense;
		ks.off = ci.dense ? ci.seq - b->hseqbase : 0;
		ks.oids = ci.oids;
		ks.hseq = b->hseqbase;
		ks.has_g = g != nullptr;
		ks.g = g && g->ttype == MGDK_oid ? (const oid *) g->theap : nullptr;
		ks.g8 = ks.g ? img8_get(g) : nullptr;
		ks.gseq = g ? g->tseqbase : 0;
		hipStream_t st = stream();
		// prior group range for the direct table
		uint64_t gmax = 0;
		oid gm = MGDK_OID_NIL;
		// the largest prior group id without a scan when g says where it is
		// (gdk_group.c:745-757: last / first row of an ordered g, tmaxpos)
		if (ks.g && (g->tsorted || g->trevsorted || g->tmaxpos != MGDK_BUN_NONE)) {
			const BUN p = g->tsorted ? n - 1 : g->trevsorted ? 0 : g->tmaxpos;
			if (oid_at(g, p, &gm) < 0)
				return -1;
		}
		if (ks.g && gm != MGDK_OID_NIL) {
			gmax = gm;
		} else if (ks.g) {
			unsigned long long *m = (unsigned long long *) meta_buf();
			if (!hip_ok(hipMemsetAsync(m, 0, 8, st), "memset"))
				return -1;
			hipLaunchKernelGGL(k_max_oid, dim3(grid_for(n, 4096, 1024)), dim3(256), 0, st, ks.g, n, m);
			unsigned long long *hm = (unsigned long long *) pinned(8);
			if (!hip_ok(hipMemcpyAsync(hm, m, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
				return -1;
			gmax = *hm;
		} else if (g) {
			gmax = g->tseqbase + n;
		}
		// ordered keys (and ordered prior groups): consecutive comparison
		// (gdk_group.c:940-975); 1- and 2-byte keys keep the table paths
		if (ks.w >= 4 && (b->tsorted || b->trevsorted) &&
		    (!g || mgdk_BATordered(g) || mgdk_BATordered_rev(g))) {
			if (group_ordered(ks, n, ci, hseqb, &gn, &en, &hn, histo != nullptr) < 0)
				goto fail;
			goto done;
		}
		// 1-byte keys under <= 32 prior groups: direct LDS tables
		static const bool small_on = getenv("MGDK_GROUP_SMALL") ? atoi(getenv("MGDK_GROUP_SMALL")) != 0 : true;
		if (small_on && ks.w == 1 && ks.kind <= 1 && (!ks.has_g || gmax < 32)) {
			const uint32_t nslots = (uint32_t) ((ks.has_g ? gmax + 1 : 1) << 8);
			if (group_small(ks, n, nslots, ci, hseqb, &gn, &en, &hn) < 0)
				goto fail;
			goto done;
		}
		// low-cardinality path first (falls through when it does not apply)
		static const bool lds_on = getenv("MGDK_GROUP_LDS") ? atoi(getenv("MGDK_GROUP_LDS")) != 0 : true;
		if (lds_on && ks.w <= 8 && (!ks.has_g || (ks.w <= 4 && gmax < 0xffffffffull)) && n < ((BUN) 1 << 50)) {
			const int rc = group_lds(ks, n, ci, hseqb, &gn, &en, &hn);
			if (rc < 0)
				goto fail;
			if (rc == 0)
				goto done;
		}
		const bool small = (ks.kind <= 1 && ks.w <= 2);
		int dshift = ks.w * 8;
		bool direct = small && ((gmax + 1) << dshift) <= ((uint64_t) 1 << 24);
		uint64_t T;
		if (direct) {
			T = (gmax + 1) << dshift;
		} else {
			T = 1024;
			while (T < 2 * n)
				T <<= 1;
			if (T > ((uint64_t) 1 << 32)) {
				seterr("HY013!BATgroup: too many rows for the device hash table");
				return -1;
			}
		}
		DevBuf d_row(direct ? 8 : T * 8), d_min(T * 8), d_hidx(n * 4), d_flags(n), d_map(T * 4);
		DevBuf d_err(16);
		if (!d_row.p || !d_min.p || !d_hidx.p || !d_flags.p || !d_map.p || !d_err.p)
			return -1;
		if (!hip_ok(hipMemsetAsync(d_min.p, 0xff, T * 8, st), "memset") ||
		    (!direct && !hip_ok(hipMemsetAsync(d_row.p, 0xff, T * 8, st), "memset")) ||
		    !hip_ok(hipMemsetAsync(d_err.p, 0, 16, st), "memset"))
			return -1;
		dim3 grd(grid_for(n, 256 * 4, 256 * 64)), blk(256);
		if (direct)
			hipLaunchKernelGGL((k_grp_insert<true>), grd, blk, 0, st, ks, n, T - 1, dshift,
					   d_row.as<unsigned long long>(), d_min.as<unsigned long long>(),
					   d_hidx.as<uint32_t>(), d_err.as<uint32_t>());
		else
			hipLaunchKernelGGL((k_grp_insert<false>), grd, blk, 0, st, ks, n, T - 1, dshift,
					   d_row.as<unsigned long long>(), d_min.as<unsigned long long>(),
					   d_hidx.as<uint32_t>(), d_err.as<uint32_t>());
		hipLaunchKernelGGL(k_grp_flags, grd, blk, 0, st, n, d_hidx.as<uint32_t>(),
				   d_min.as<unsigned long long>(), d_flags.as<int8_t>());
		mgdk_bat *E = compact_flags(d_flags.as<int8_t>(), n, 0);
		if (E == nullptr)
			return -1;
		const BUN ngrp = E->count;
		en = newbat(0, MGDK_oid, ngrp);
		hn = newbat(0, MGDK_lng, ngrp);
		gn = newbat(hseqb, MGDK_oid, n);
		if (!en || !hn || !gn) {
			mgdk_BBPunfix(E);
			goto fail;
		}
		hipLaunchKernelGGL(k_grp_map, dim3(grid_for(ngrp, 256, 4096)), blk, 0, st, ngrp,
				   E->ttype == MGDK_void ? nullptr : (const oid *) E->theap, E->tseqbase,
				   d_hidx.as<uint32_t>(), d_map.as<uint32_t>(), ci.dense, ci.seq, ci.oids,
				   (oid *) en->theap);
		if (!hip_ok(hipMemsetAsync(hn->theap, 0, ngrp * 8, st), "memset")) {
			mgdk_BBPunfix(E);
			goto fail;
		}
		uint32_t *uns = d_err.as<uint32_t>() + 1;
		if (ngrp <= 4096)
			hipLaunchKernelGGL((k_grp_assign<true>), grd, blk, ngrp * 4, st, n, d_hidx.as<uint32_t>(),
					   d_map.as<uint32_t>(), (oid *) gn->theap, ngrp,
					   (unsigned long long *) hn->theap, uns);
		else
			hipLaunchKernelGGL((k_grp_assign<false>), grd, blk, 0, st, n, d_hidx.as<uint32_t>(),
					   d_map.as<uint32_t>(), (oid *) gn->theap, ngrp,
					   (unsigned long long *) hn->theap, uns);
		uint32_t *herr = (uint32_t *) pinned(16);
		if (!hip_ok(hipMemcpyAsync(herr, d_err.p, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
			mgdk_BBPunfix(E);
			goto fail;
		}
		mgdk_BBPunfix(E);
		if (herr[0]) {
			seterr("HY013!BATgroup: hash table overflow");
			goto fail;
		}
		gn->count = n;
		en->count = ngrp;
		hn->count = ngrp;
		gn->tsorted = herr[1] == 0;
		gn->trevsorted = ngrp == 1 || n <= 1;
		gn->tkey = ngrp == n;
		gn->tnonil = 1;
		en->tsorted = en->tkey = en->tnonil = 1;
		en->trevsorted = ngrp == 1;
		bool hs = ngrp == n || ngrp == 1;
		hn->tkey = ngrp == 1;
		hn->tsorted = hn->trevsorted = hs;
		hn->tnonil = 1;
		// tmaxpos (gdk_group.c:99,1313), extents virtualised when dense
		if (ngrp > 0) {
			oid fl[2];
			if (oid_at(en, 0, &fl[0]) < 0 || oid_at(en, ngrp - 1, &fl[1]) < 0)
				goto fail;
			gn->tmaxpos = cand_index(ci, fl[1]);
			if (fl[1] - fl[0] == ngrp - 1)
				setdense(en, fl[0], ngrp);
		}
	}
done:
	if (grouped && en) {
		// BATgroup's estimates (gdk_group.c:1291,1314-1318)
		const BUN ngrp = en->count;
		gn->tunique_est = (double) ngrp;
		en->tunique_est = (double) ngrp;
		if (!g && !e && !s)
			b->tunique_est = (double) ngrp;
	}
	*groups = gn;
	if (extents)
		*extents = en;
	else
		mgdk_BBPunfix(en);
	if (histo)
		*histo = hn;
	else
		mgdk_BBPunfix(hn);
	return 0;
fail:
	mgdk_BBPunfix(gn);
	mgdk_BBPunfix(en);
	mgdk_BBPunfix(hn);
	return -1;
}

// ---- str columns whose heap is not duplicate eliminated -------------------
// GDK groups strings by their offsets only when the heap is fully duplicate
// eliminated, i.e. smaller than GDK_ELIMLIMIT = 64 KiB (gdk_group.c:897-919,
// GDK_ELIMDOUBLES gdk_atoms.h:373-375); larger heaps keep equal strings at
// different offsets and the reference compares contents (strCmp, its hash
// path :1118-1282).  On the device:
//   1  group by (prior group, offset) -- a refinement of the content
//      grouping, numbered by first occurrence;
//   2  per offset group: the string of its first row and its prior group;
//      a 64-bit content hash of that string;
//   3  group the offset groups (in id order = first-occurrence order) by
//      (prior group, hash): first-occurrence numbering of the content
//      classes, because an offset group's first row precedes another's iff
//      its id is smaller;
//   4  every offset group's string is compared byte for byte with its
//      class representative's (a hash collision reruns with another seed);
//   5  row ids through the id map, extents through the representatives,
//      histogram = grouped sum of the offset groups' counts.
namespace {

constexpr uint64_t ELIMLIMIT = (uint64_t) 1 << 16;

struct OidSrc {
	const oid *p;     // NULL: dense
	oid seq;
	__device__ __forceinline__ oid at(BUN i) const { return p ? p[i] : seq + i; }
};

OidSrc
oid_src(const mgdk_bat *b)
{
	return OidSrc{b->ttype == MGDK_void ? nullptr : (const oid *) b->theap, b->tseqbase};
}

// VarHeapVal (gdk_atoms.h:421-436): 1- and 2-byte offsets are relative to
// GDK_VAROFFSET = 1024 * sizeof(var_t)
__device__ __forceinline__ const uint8_t *
str_ptr(const void *offs, int w, const char *vh, BUN p)
{
	size_t o;
	switch (w) {
	case 1: o = (size_t) ((const uint8_t *) offs)[p] + 8192; break;
	case 2: o = (size_t) ((const uint16_t *) offs)[p] + 8192; break;
	case 4: o = (size_t) ((const uint32_t *) offs)[p]; break;
	default: o = (size_t) ((const uint64_t *) offs)[p]; break;
	}
	return (const uint8_t *) vh + o;
}

// step 2: the b position and prior group of every offset group's first row
__global__ __launch_bounds__(256) void
k_sg_rep(BUN n, OidSrc gid0, OidSrc ext0, bool cdense, oid cseq, const oid *coids, oid bhseq,
	 const oid *g, uint64_t *rep_pos, oid *rep_g)
{
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
		const oid k = gid0.at(i);
		const oid o = cdense ? cseq + i : coids[i];
		if (ext0.at(k) == o) {
			rep_pos[k] = o - bhseq;
			if (rep_g)
				rep_g[k] = g[i];
		}
	}
}

__global__ __launch_bounds__(256) void
k_sg_hash(BUN K, const uint64_t *rep_pos, const void *offs, int w, const char *vh, uint64_t seed, int64_t *h)
{
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
		const uint8_t *s = str_ptr(offs, w, vh, rep_pos[k]);
		uint64_t x = seed ^ 0xcbf29ce484222325ULL;
		for (; *s; s++)
			x = (x ^ *s) * 0x100000001b3ULL;
		x ^= x >> 31;
		x *= 0x94d049bb133111ebULL;
		x ^= x >> 29;
		h[k] = (int64_t) x;
	}
}

// step 4: 1 in *bad when an offset group's string differs from its class
// representative's
__global__ __launch_bounds__(256) void
k_sg_verify(BUN K, OidSrc gid1, OidSrc ext1, const uint64_t *rep_pos, const void *offs, int w, const char *vh,
	    uint32_t *bad)
{
	uint32_t diff = 0;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
		const oid r = ext1.at(gid1.at(k));
		if (r == k)
			continue;
		const uint8_t *a = str_ptr(offs, w, vh, rep_pos[k]), *c = str_ptr(offs, w, vh, rep_pos[r]);
		size_t j = 0;
		while (a[j] && a[j] == c[j])
			j++;
		diff |= a[j] != c[j];
	}
	diff = block_reduce(diff, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(bad, diff);
}

// step 5: row ids through the map; bit 0 of *flags: a row's id is below its
// predecessor's (the ids are not sorted)
__global__ __launch_bounds__(256) void
k_sg_final(BUN n, OidSrc gid0, OidSrc gid1, oid *gn, uint32_t *flags)
{
	uint32_t down = 0;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
		const oid v = gid1.at(gid0.at(i));
		gn[i] = v;
		if (i > 0)
			down |= gid1.at(gid0.at(i - 1)) > v;
	}
	down = block_reduce(down, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(flags, down);
}

__global__ __launch_bounds__(256) void
k_sg_extents(BUN K1, OidSrc ext0, OidSrc ext1, oid *en)
{
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN c = (BUN) blockIdx.x * blockDim.x + threadIdx.x; c < K1; c += stride)
		en[c] = ext0.at(ext1.at(c));
}

// a scratch column of n rows whose properties are all unknown
mgdk_bat *
plain_col(int tt, BUN n)
{
	mgdk_bat *b = newbat(0, tt, n);
	if (b) {
		b->count = n;
		b->tsorted = b->trevsorted = b->tkey = b->tnonil = b->tnil = 0;
	}
	return b;
}

int
group_str_content(mgdk_bat **groups, mgdk_bat **extents, mgdk_bat **histo, mgdk_bat *b, mgdk_bat *s,
		  mgdk_bat *g, const Cand &ci)
{
	const BUN n = ci.n;
	const oid hseqb = n ? ci.first : 0;
	const double est_b = b->tunique_est;
	mgdk_bat *gn0 = nullptr, *en0 = nullptr, *hn0 = nullptr;
	if (group_core(&gn0, &en0, &hn0, b, s, g, nullptr, nullptr) < 0)
		return -1;
	b->tunique_est = est_b;
	const BUN K = en0->count;
	mgdk_bat *gn = nullptr, *en = nullptr, *hn = nullptr;
	mgdk_bat *H = nullptr, *G = nullptr, *g1 = nullptr, *e1 = nullptr;
	hipStream_t st = stream();
	int rc = -1;
	BUN K1 = 0;
	{
		DevBuf d_pos(K * 8), d_flag(16);
		if (!d_pos.p || !d_flag.p)
			goto out;
		H = plain_col(MGDK_lng, K);
		if (H == nullptr || (g && (G = plain_col(MGDK_oid, K)) == nullptr))
			goto out;
		hipLaunchKernelGGL(k_sg_rep, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, n, oid_src(gn0),
				   oid_src(en0), ci.dense, ci.seq, ci.oids, b->hseqbase,
				   g ? (const oid *) g->theap : nullptr, d_pos.as<uint64_t>(),
				   G ? (oid *) G->theap : nullptr);
		for (uint64_t seed = 0;; seed++) {
			if (seed == 4) {
				seterr("HY013!BATgroup: string hash collisions");
				goto out;
			}
			hipLaunchKernelGGL(k_sg_hash, dim3(grid_for(K, 256, 8192)), dim3(256), 0, st, K,
					   d_pos.as<uint64_t>(), b->theap, b->twidth, (const char *) b->tvheap,
					   seed * 0x9e3779b97f4a7c15ULL, (int64_t *) H->theap);
			if (!sync() || group_core(&g1, &e1, nullptr, H, nullptr, G, nullptr, nullptr) < 0)
				goto out;
			uint32_t *hf = (uint32_t *) pinned(16);
			if (!hip_ok(hipMemsetAsync(d_flag.p, 0, 16, st), "memset"))
				goto out;
			hipLaunchKernelGGL(k_sg_verify, dim3(grid_for(K, 256, 8192)), dim3(256), 0, st, K, oid_src(g1),
					   oid_src(e1), d_pos.as<uint64_t>(), b->theap, b->twidth,
					   (const char *) b->tvheap, d_flag.as<uint32_t>());
			if (!hip_ok(hipMemcpyAsync(hf, d_flag.p, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
				goto out;
			if (hf[0] == 0)
				break;
			mgdk_BBPunfix(g1);
			mgdk_BBPunfix(e1);
			g1 = e1 = nullptr;
		}
		K1 = e1->count;
		gn = newbat(hseqb, MGDK_oid, n);
		en = newbat(0, MGDK_oid, K1);
		if (gn == nullptr || en == nullptr || !hip_ok(hipMemsetAsync(d_flag.p, 0, 16, st), "memset"))
			goto out;
		hipLaunchKernelGGL(k_sg_final, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, n, oid_src(gn0),
				   oid_src(g1), (oid *) gn->theap, d_flag.as<uint32_t>());
		hipLaunchKernelGGL(k_sg_extents, dim3(grid_for(K1, 256, 8192)), dim3(256), 0, st, K1, oid_src(en0),
				   oid_src(e1), (oid *) en->theap);
		uint32_t *hf = (uint32_t *) pinned(16);
		if (!hip_ok(hipMemcpyAsync(hf, d_flag.p, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			goto out;
		gn->count = n;
		gn->tsorted = hf[0] == 0;
		gn->trevsorted = K1 == 1 || n <= 1;
		gn->tkey = K1 == n;
		gn->tnonil = 1;
		gn->tnil = 0;
		en->count = K1;
		en->tsorted = en->tkey = en->tnonil = 1;
		en->trevsorted = K1 == 1;
		hn = mgdk_BATgroupsum(hn0, g1, e1, nullptr, MGDK_lng, true);
		if (hn == nullptr)
			goto out;
		hn->tkey = K1 == 1;
		hn->tsorted = hn->trevsorted = K1 == n || K1 == 1;
		hn->tnonil = 1;
		hn->tnil = 0;
		hn->tminpos = hn->tmaxpos = MGDK_BUN_NONE;
		hn->tunique_est = 0;
		if (K1 > 0) {
			oid fl[2];
			if (oid_at(en, 0, &fl[0]) < 0 || oid_at(en, K1 - 1, &fl[1]) < 0)
				goto out;
			gn->tmaxpos = cand_index(ci, fl[1]);
			if (fl[1] - fl[0] == K1 - 1)
				setdense(en, fl[0], K1);
		}
		gn->tunique_est = en->tunique_est = (double) K1;
		rc = 0;
	}
out:
	mgdk_BBPunfix(gn0);
	mgdk_BBPunfix(en0);
	mgdk_BBPunfix(hn0);
	mgdk_BBPunfix(H);
	mgdk_BBPunfix(G);
	mgdk_BBPunfix(g1);
	mgdk_BBPunfix(e1);
	if (rc < 0) {
		mgdk_BBPunfix(gn);
		mgdk_BBPunfix(en);
		mgdk_BBPunfix(hn);
		return -1;
	}
	*groups = gn;
	if (extents)
		*extents = en;
	else
		mgdk_BBPunfix(en);
	if (histo)
		*histo = hn;
	else
		mgdk_BBPunfix(hn);
	return 0;
}

}  // namespace

extern "C" int
mgdk_BATgroup(mgdk_bat **groups, mgdk_bat **extents, mgdk_bat **histo, mgdk_bat *b, mgdk_bat *s,
	      mgdk_bat *g, mgdk_bat *e, mgdk_bat *h)
{
	if (b != nullptr && groups != nullptr && b->ttype == MGDK_str && b->tvheap != nullptr &&
	    b->tvheapsize >= ELIMLIMIT) {
		Cand ci;
		if (cand_init(&ci, b, s) < 0)
			return -1;
		if (g && g->count != ci.n) {
			seterr("b with s and g must be aligned\n");
			return -1;
		}
		// the shortcuts of gdk_group.c:712-802 hold by content (tkey and
		// the order properties of a str column are about its strings)
		const bool trivial = b->tkey || ci.n <= 1 || (g && (g->tkey || g->ttype == MGDK_void));
		const bool single = b->tsorted && b->trevsorted &&
				    (!g || (mgdk_BATordered(g) && mgdk_BATordered_rev(g)));
		if (!trivial && !single) {
			ProfScope prof("group_str");
			const int rc = group_str_content(groups, extents, histo, b, s, g, ci);
			if (rc == 0 && !g && !e && !s)
				b->tunique_est = (*groups)->tunique_est;
			return rc;
		}
	}
	return group_core(groups, extents, histo, b, s, g, e, h);
}

// BATunique (gdk/gdk_unique.c:30): the candidate list of the first
// occurrence of every distinct value of b[s] -- the extents of BATgroup
// (gdk_unique.c:18-22 says as much), so the same device path computes it.
extern "C" mgdk_bat *
mgdk_BATunique(mgdk_bat *b, mgdk_bat *s)
{
	mgdk_bat *g = nullptr, *e = nullptr;
	if (mgdk_BATgroup(&g, &e, nullptr, b, s, nullptr, nullptr, nullptr) < 0)
		return nullptr;
	mgdk_BBPunfix(g);
	return e;
}
