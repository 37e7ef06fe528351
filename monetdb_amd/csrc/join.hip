// join.hip -- the hash path of BATjoin on the MI355X
// (gdk/gdk_join.c:4451 BATjoin -> :2900 hashjoin, probe loop HASHJOIN
// :2781-2895; hash build gdk/gdk_hash.c:658-704).
//
// GDK's result order: r1 follows the left candidates in order; the matches
// of one left row come in DESCENDING right position, because the chains of
// the right-side hash are built by prepending.  The device reproduces that
// order without chains.
//
// Main path (open addressing):
//   build  every right candidate j is inserted with one CAS into a linear
//          probing table of 2*|r| slots, slot = key image + (j+1) packed in
//          8 bytes (<= 4-byte keys) or 16 bytes (8-byte keys); the largest
//          displacement is recorded.  A key's entries all lie within
//          [home, home + maxdisp], so a probe touches one or two cache lines
//          (table of 15M int keys = 240 MB: MALL-resident on the MI355X);
//   probe  ONE pass over the left side: a tile of 16 x 256 rows issues all
//          its key loads, then all its first-slot loads, counts the matches
//          of every row, ranks them (wave scans + a 64-entry LDS scan) and
//          takes the tile's output offset from decoupled look-back
//          (lookback.h); rows with one match write it directly, rows with
//          several emit them by descending right position (repeated
//          max-below selection over the row's cluster).  The output is
//          sized |l| up front; when a join produces more pairs the probe is
//          simply rerun with the exact size.
// Fallback (heavy duplicate build keys: displacement > DMAX_DUP): CSR table from
//   a stable radix sort of (bucket, position) pairs (sort.hip) and a
//   two-pass count/scan/write probe that walks each bucket backwards.
// nil never matches unless nil_matches.  Integer key types (bte..lng, date,
// oid).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "lookback.h"
#include "mgdk_internal.h"

using namespace mgdk;
using namespace mgdk_lb;

namespace {

struct Side {
	const void *base;
	int w;
	bool uns;          // oid: unsigned
	bool dense;
	oid off;           // dense: position of candidate 0
	const oid *oids;   // materialized candidates
	oid hseq;
	oid cseq;          // dense: oid of candidate 0
	oid tseq;          // void side (base == nullptr): value of position 0
	uint32_t *nofit;   // partitioned paths, 8-byte keys: set when a value has no 4-byte image
};

__device__ __forceinline__ uint64_t
key_of(const Side &s, BUN i, bool &isnil)
{
	BUN p = s.dense ? s.off + i : s.oids[i] - s.hseq;
	switch (s.w) {
	case 1: { int8_t v = ((const int8_t *) s.base)[p]; isnil = v == INT8_MIN; return (uint64_t) (int64_t) v; }
	case 2: { int16_t v = ((const int16_t *) s.base)[p]; isnil = v == INT16_MIN; return (uint64_t) (int64_t) v; }
	case 4: { int32_t v = ((const int32_t *) s.base)[p]; isnil = v == INT32_MIN; return (uint64_t) (int64_t) v; }
	default: {
		if (s.base == nullptr) {        // void: dense oids (nil tseqbase: all nil)
			isnil = s.tseq == MGDK_OID_NIL;
			return isnil ? s.tseq : s.tseq + p;
		}
		uint64_t v = ((const uint64_t *) s.base)[p];
		isnil = s.uns ? v == ((uint64_t) 1 << 63) : (int64_t) v == INT64_MIN;
		return v;
	}
	}
}

__device__ __forceinline__ oid
oid_of(const Side &s, BUN i)
{
	return s.dense ? s.cseq + i : s.oids[i];
}

__device__ __forceinline__ uint64_t
hash64(uint64_t x)
{
	x ^= x >> 33;
	x *= 0xff51afd7ed558ccdull;
	x ^= x >> 33;
	x *= 0xc4ceb9fe1a85ec53ull;
	return x ^ (x >> 33);
}

// ---------------------------------------------------------------------------
// open-addressing table
// ---------------------------------------------------------------------------

// displacement bounds of the main path: linear probing at load 1/2 keeps the
// largest displacement of 10^8 keys well below DMAX; with duplicate build
// keys the multi-match write walks a row's cluster once per match, so the
// table is only used while every cluster stays short (DMAX_DUP)
constexpr uint32_t DMAX = 1024;
constexpr uint32_t DMAX_DUP = 64;
constexpr uint64_t TAB_PAD = DMAX + 8;   // slots past `cap`: probing never wraps
// rows per lane in a probe tile (register budget: 8-byte keys carry 16-B slots)
template <int KW> constexpr int jrows() { return KW == 4 ? 8 : 8; }

struct alignas(16) Slot16 {
	uint64_t key;
	uint64_t pos1;                   // candidate index + 1; 0 = empty
};

// A probe reads a window of W consecutive slots with its first load.
template <int KW> struct Tab;
template <> struct Tab<4> {
	typedef unsigned long long slot_t;
	static constexpr int W = 2;
	static __device__ __forceinline__ uint32_t pos1(slot_t s) { return (uint32_t) (s >> 32); }
	static __device__ __forceinline__ bool same(slot_t s, uint64_t k) { return (uint32_t) s == (uint32_t) k; }
	static __device__ __forceinline__ slot_t load(const slot_t *t, uint64_t h) { return t[h]; }
};
template <> struct Tab<8> {
	typedef Slot16 slot_t;
	static constexpr int W = 1;
	static __device__ __forceinline__ uint32_t pos1(const slot_t &s) { return (uint32_t) s.pos1; }
	static __device__ __forceinline__ bool same(const slot_t &s, uint64_t k) { return s.key == k; }
	static __device__ __forceinline__ slot_t load(const slot_t *t, uint64_t h)
	{
		ulonglong2 v = *(const ulonglong2 *) &t[h];
		Slot16 s;
		s.key = v.x;
		s.pos1 = v.y;
		return s;
	}
};

__device__ __forceinline__ uint64_t
home_of(uint64_t k, uint64_t cap)
{
	return __umul64hi(hash64(k), cap);
}

// meta[2] = largest displacement, meta[3] = 1 when two right candidates
// share a key (then every probe scans its whole cluster)
template <int KW>
__global__ __launch_bounds__(256) void
k_lp_build(Side r, BUN n, uint64_t cap, bool nil_matches, typename Tab<KW>::slot_t *t, uint32_t *maxd,
	   uint32_t *dup)
{
	uint32_t md = 0;
	bool dp = false;
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		const uint64_t k = key_of(r, j, isnil);
		if (isnil && !nil_matches)
			continue;
		uint64_t h = home_of(k, cap);
		uint32_t d = 0;
		if constexpr (KW == 4) {
			// every slot passed over was observed with its final content,
			// so a duplicate placed earlier in the cluster is always seen
			const unsigned long long v = ((unsigned long long) (j + 1) << 32) | (uint32_t) k;
			for (;;) {
				unsigned long long o = t[h];
				if (o == 0ull)
					o = atomicCAS(&t[h], 0ull, v);
				if (o == 0ull)
					break;
				dp |= (uint32_t) o == (uint32_t) k;
				h++;
				if (++d > DMAX)
					break;
			}
		} else {
			while (t[h].pos1 != 0ull ||
			       atomicCAS((unsigned long long *) &t[h].pos1, 0ull, (unsigned long long) (j + 1)) != 0ull) {
				h++;
				if (++d > DMAX)
					break;
			}
			if (d <= DMAX)
				t[h].key = k;
		}
		md = d > md ? d : md;
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) {
		uint32_t x = __shfl_xor(md, o);
		md = x > md ? x : md;
	}
	if (__any(dp) && __lane_id() == 0)
		atomicOr(dup, 1u);
	if (__lane_id() == 0 && md)
		atomicMax(maxd, md);
}

// 8-byte keys: keys are stored after the slot is claimed, so duplicates are
// found in a second pass -- candidate j scans its cluster up to its own slot
__global__ __launch_bounds__(256) void
k_lp_dupcheck(Side r, BUN n, uint64_t cap, bool nil_matches, const Slot16 *t, uint32_t *dup)
{
	bool dp = false;
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		const uint64_t k = key_of(r, j, isnil);
		if (isnil && !nil_matches)
			continue;
		uint64_t h = home_of(k, cap);
		for (uint32_t d = 0; d <= DMAX; d++, h++) {
			const uint64_t p1 = t[h].pos1;
			if (p1 == j + 1 || p1 == 0)
				break;
			if (t[h].key == k) {
				dp = true;
				break;
			}
		}
	}
	if (__any(dp) && __lane_id() == 0)
		atomicOr(dup, 1u);
}

struct ProbeArgs {
	Side l, r;
	BUN n;
	uint64_t cap;
	uint32_t maxd;
	const uint32_t *maxd_dev;   // non-NULL: the build's largest displacement, read on the device
	bool nil_matches;
	uint32_t *ticket;
	uint64_t *status;
	uint32_t ntiles;
	uint64_t *meta;       // [0] total pairs, [1] look-back error
	oid *r1, *r2;
	uint64_t ocap;
	bool nt;              // nontemporal result stores
};

// UNIQ: no two right candidates share a key -> a probe stops at its first
// match.  Otherwise it scans the cluster to the first empty slot (or to
// home + maxd), counting matches and keeping the largest position.
template <int KW, bool UNIQ>
__global__ __launch_bounds__(256) void
k_lp_probe(ProbeArgs a, const typename Tab<KW>::slot_t *t)
{
	typedef Tab<KW> TB;
	typedef typename TB::slot_t slot_t;
	constexpr int JR = jrows<KW>(), JTILE = 256 * JR, W = TB::W;
	__shared__ uint32_t s_tot[64];     // [r][wave], zero-padded to 64
	__shared__ uint64_t s_off[64];
	__shared__ uint32_t s_tile;
	__shared__ uint64_t s_pre;
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	if (tid == 0)
		s_tile = atomicAdd(a.ticket, 1u);
	if (JR * 4 < 64 && tid < 64)
		s_tot[tid] = 0;
	__syncthreads();
	const uint32_t tile = s_tile;
	const BUN base = (BUN) tile * JTILE + tid;
	const uint32_t maxd = a.maxd_dev ? min(*a.maxd_dev, DMAX) : a.maxd;

	uint64_t key[JR];
	bool ok[JR];
#pragma unroll
	for (int r = 0; r < JR; r++) {
		const BUN i = base + (BUN) r * 256;
		bool isnil = true;
		key[r] = i < a.n ? key_of(a.l, i, isnil) : 0;
		ok[r] = i < a.n && (!isnil || a.nil_matches);
	}
	uint64_t hm[JR];
	slot_t sv[JR][W];
#pragma unroll
	for (int r = 0; r < JR; r++) {
		hm[r] = home_of(key[r], a.cap);
#pragma unroll
		for (int q = 0; q < W; q++)
			sv[r][q] = ok[r] ? TB::load(t, hm[r] + q) : slot_t{};
	}
	uint32_t c[JR], best[JR];
#pragma unroll
	for (int r = 0; r < JR; r++) {
		c[r] = 0;
		best[r] = 0;
		if (!ok[r])
			continue;
		uint64_t h = hm[r];
		uint32_t d = 0;
		slot_t win[W];
#pragma unroll
		for (int q = 0; q < W; q++)
			win[q] = sv[r][q];
		for (;;) {
			bool stop = false;
#pragma unroll
			for (int q = 0; q < W; q++) {
				if (stop)
					break;
				const uint32_t p1 = TB::pos1(win[q]);
				if (p1 == 0) {
					stop = true;
					break;
				}
				if (TB::same(win[q], key[r])) {
					c[r]++;
					best[r] = p1 > best[r] ? p1 : best[r];
					if (UNIQ) {
						stop = true;
						break;
					}
				}
				if (d >= maxd) {
					stop = true;
					break;
				}
				d++;
			}
			if (stop)
				break;
			h += W;
#pragma unroll
			for (int q = 0; q < W; q++)
				win[q] = TB::load(t, h + q);
		}
	}
	// ranks: wave scan per row slot r, then a 64-entry scan over (r, wave)
	uint32_t ex[JR];
#pragma unroll
	for (int r = 0; r < JR; r++) {
		uint32_t v = c[r];
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			uint32_t u = __shfl_up(v, o);
			if (lane >= (unsigned) o)
				v += u;
		}
		ex[r] = v - c[r];
		if (lane == 63)
			s_tot[r * 4 + w] = v;
	}
	__syncthreads();
	if (w == 0) {
		uint64_t v = s_tot[lane];
		const uint64_t own = v;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			uint64_t u = __shfl_up(v, o);
			if (lane >= (unsigned) o)
				v += u;
		}
		s_off[lane] = v - own;
		const uint64_t agg = __shfl(v, 63);
		const uint64_t pre = lookback(a.status, tile, agg, (uint32_t *) &a.meta[1]);
		if (lane == 0) {
			s_pre = pre;
			if (tile == a.ntiles - 1)
				a.meta[0] = pre + agg;
		}
	}
	__syncthreads();
	const uint64_t pre = s_pre;
#pragma unroll
	for (int r = 0; r < JR; r++) {
		if (c[r] == 0)
			continue;
		uint64_t pos = pre + s_off[r * 4 + w] + ex[r];
		if (pos + c[r] > a.ocap)
			continue;                      // host reruns with the exact size
		const BUN i = base + (BUN) r * 256;
		const oid lo = oid_of(a.l, i);
		if (a.nt) {
			__builtin_nontemporal_store(lo, &a.r1[pos]);
			__builtin_nontemporal_store(oid_of(a.r, best[r] - 1), &a.r2[pos]);
		} else {
			a.r1[pos] = lo;
			a.r2[pos] = oid_of(a.r, best[r] - 1);
		}
		if (UNIQ)
			continue;
		uint32_t prev = best[r];
		for (uint32_t m = 1; m < c[r]; m++) {
			// next largest candidate index below prev among this key's entries
			uint32_t nb = 0;
			uint64_t h = hm[r];
			for (uint32_t d = 0;; d++, h++) {
				const slot_t s = TB::load(t, h);
				const uint32_t p1 = TB::pos1(s);
				if (p1 == 0)
					break;
				if (TB::same(s, key[r]) && p1 < prev && p1 > nb)
					nb = p1;
				if (d >= maxd)
					break;
			}
			pos++;
			a.r1[pos] = lo;
			a.r2[pos] = oid_of(a.r, nb - 1);
			prev = nb;
		}
	}
}

// ---------------------------------------------------------------------------
// CSR fallback
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void
k_build_keys(Side r, BUN n, uint64_t mask, uint64_t *bucket, uint32_t *idx, uint32_t *cnt)
{
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		uint64_t k = key_of(r, j, isnil);
		uint64_t b = hash64(k) & mask;
		bucket[j] = b;
		idx[j] = (uint32_t) j;
		atomicAdd(&cnt[b], 1u);
	}
}

__global__ __launch_bounds__(256) void
k_build_gather(Side r, BUN n, const uint32_t *sidx, uint64_t *skey, uint8_t *snil)
{
	for (BUN e = (BUN) blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		skey[e] = key_of(r, sidx[e], isnil);
		snil[e] = isnil;
	}
}

template <bool WRITE>
__global__ __launch_bounds__(256) void
k_probe(Side l, BUN n, uint64_t mask, const uint64_t *boff, const uint64_t *skey, const uint8_t *snil,
	const uint32_t *sidx, Side r, bool nil_matches, uint32_t *cnt, const uint64_t *ooff, oid *r1, oid *r2)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		uint64_t k = key_of(l, i, isnil);
		uint32_t c = 0;
		if (!isnil || nil_matches) {
			uint64_t b = hash64(k) & mask;
			const uint64_t e0 = boff[b], e1 = boff[b + 1];
			if (WRITE) {
				uint64_t pos = ooff[i];
				const oid lo = oid_of(l, i);
				for (uint64_t e = e1; e > e0; e--) {
					if (skey[e - 1] == k && (bool) snil[e - 1] == isnil) {
						r1[pos] = lo;
						r2[pos] = oid_of(r, sidx[e - 1]);
						pos++;
					}
				}
			} else {
				for (uint64_t e = e0; e < e1; e++)
					c += skey[e] == k && (bool) snil[e] == isnil;
			}
		}
		if (!WRITE)
			cnt[i] = c;
	}
}

void
side_init(Side &s, const mgdk_bat *b, const Cand &c)
{
	s.base = b->ttype == MGDK_void ? nullptr : b->theap;
	s.w = b->ttype == MGDK_void ? 8 : b->twidth;
	s.uns = basetype(b->ttype) == MGDK_oid || b->ttype == MGDK_void;
	s.tseq = b->tseqbase;
	s.dense = c.dense;
	s.off = c.dense ? c.seq - b->hseqbase : 0;
	s.oids = c.oids;
	s.hseq = b->hseqbase;
	s.cseq = c.seq;
}

// error return after launches: the stream drains before the caller's
// buffers go back to the shared allocator cache
int
sync_fail()
{
	(void) side_join();                 // work queued on the side stream too
	(void) sync();
	return -1;
}

void
unfix2(mgdk_bat *a, mgdk_bat *b)
{
	mgdk_BBPunfix(a);
	mgdk_BBPunfix(b);
}

// open-addressing path; returns 1 when the build exceeded DMAX (caller
// falls back), 0 on success, -1 on error
template <int KW>
int
join_lp(const Side &L, BUN nl, const Side &R, BUN nr, bool nil_matches, mgdk_bat **ap, mgdk_bat **bp, bool *ukey)
{
	typedef typename Tab<KW>::slot_t slot_t;
	hipStream_t st = stream();
	static const int cap_pct = getenv("MGDK_JOIN_CAP_PCT") ? atoi(getenv("MGDK_JOIN_CAP_PCT")) : 200;
	static const bool nt = getenv("MGDK_JOIN_NT") ? atoi(getenv("MGDK_JOIN_NT")) != 0 : false;
	uint64_t cap = nr * (uint64_t) (cap_pct < 110 ? 110 : cap_pct) / 100;
	cap = cap > 64 ? cap : 64;
	const uint64_t tslots = cap + TAB_PAD;
	DevBuf tab(tslots * sizeof(slot_t));
	uint64_t *meta = (uint64_t *) meta_buf();
	uint64_t *h = (uint64_t *) pinned(64);
	if (!tab.p || !meta || !h)
		return -1;
	if (!hip_ok(hipMemsetAsync(tab.p, 0, tslots * sizeof(slot_t), st), "memset") ||
	    !hip_ok(hipMemsetAsync(meta, 0, 64, st), "memset"))
		return -1;
	hipLaunchKernelGGL((k_lp_build<KW>), dim3(grid_for(nr, 1024, 16384)), dim3(256), 0, st, R, nr, cap, nil_matches,
			   tab.as<slot_t>(), (uint32_t *) &meta[2], (uint32_t *) &meta[3]);
	if (KW == 8)
		hipLaunchKernelGGL(k_lp_dupcheck, dim3(grid_for(nr, 1024, 16384)), dim3(256), 0, st, R, nr, cap,
				   nil_matches, (const Slot16 *) tab.p, (uint32_t *) &meta[3]);
	// small build sides: no host round trip between build and probe -- the
	// probe reads the displacement bound on the device and handles
	// duplicates (the general probe is exact for unique keys too); the
	// build's outcome is checked with the probe's, and a bad one discards
	// the probe (a round trip costs more than the probe of a small join)
	const bool onesync = nr < 65536;
	uint32_t maxd = DMAX;
	bool uniq = false;
	if (!onesync) {
		if (!hip_ok(hipMemcpyAsync(h, meta, 32, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			return -1;
		maxd = (uint32_t) h[2];
		uniq = h[3] == 0;
		if (maxd > DMAX || (!uniq && maxd > DMAX_DUP))
			return 1;
	}

	const uint64_t jtile = 256 * jrows<KW>();
	const uint64_t ntiles = (nl + jtile - 1) / jtile;
	if (ntiles >= (1ull << 31)) {
		seterr("42000!BATjoin: input too large");
		return -1;
	}
	ProbeArgs a{};
	a.l = L;
	a.r = R;
	a.n = nl;
	a.cap = cap;
	a.maxd = maxd;
	a.maxd_dev = onesync ? (const uint32_t *) &meta[2] : nullptr;
	a.nil_matches = nil_matches;
	a.nt = nt;
	a.ntiles = (uint32_t) ntiles;
	a.meta = meta;
	uint64_t ocap = nl;
	for (int attempt = 0; attempt < 2; attempt++) {
		mgdk_bat *ra = newbat(0, MGDK_oid, ocap), *rb = newbat(0, MGDK_oid, ocap);
		size_t sbytes = (ntiles + 8) * sizeof(uint64_t);
		char *sc = (char *) scratch(sbytes);
		if (!ra || !rb || !sc) {
			unfix2(ra, rb);
			return -1;
		}
		a.ticket = (uint32_t *) sc;
		a.status = (uint64_t *) sc + 8;
		a.r1 = (oid *) ra->theap;
		a.r2 = (oid *) rb->theap;
		a.ocap = ocap;
		if (!hip_ok(hipMemsetAsync(sc, 0, sbytes, st), "memset") ||
		    !hip_ok(hipMemsetAsync(meta, 0, 16, st), "memset")) {   // [0], [1]: the build's [2], [3] stay
			unfix2(ra, rb);
			return -1;
		}
		if (uniq)
			hipLaunchKernelGGL((k_lp_probe<KW, true>), dim3((unsigned) ntiles), dim3(256), 0, st, a,
					   (const slot_t *) tab.p);
		else
			hipLaunchKernelGGL((k_lp_probe<KW, false>), dim3((unsigned) ntiles), dim3(256), 0, st, a,
					   (const slot_t *) tab.p);
		if (!hip_ok(hipMemcpyAsync(h, meta, 32, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
			unfix2(ra, rb);
			return -1;
		}
		if (onesync && ((uint32_t) h[2] > DMAX || (h[3] != 0 && (uint32_t) h[2] > DMAX_DUP))) {
			unfix2(ra, rb);
			return 1;                       // the build overflowed: the CSR path
		}
		if (h[1] & 1) {
			seterr("HY013!BATjoin: look-back did not complete");
			unfix2(ra, rb);
			return -1;
		}
		const uint64_t nout = h[0];
		if (nout <= ocap) {
			ra->count = rb->count = nout;
			*ukey = onesync ? h[3] == 0 : uniq;
			*ap = ra;
			*bp = rb;
			return 0;
		}
		unfix2(ra, rb);
		ocap = nout;
	}
	seterr("BATjoin: probe result size changed between runs");
	return -1;
}

int
join_csr(const Side &L, BUN nl, const Side &R, BUN nr, bool nil_matches, mgdk_bat **ap, mgdk_bat **bp)
{
	hipStream_t st = stream();
	uint64_t B = 1;
	int bits = 0;
	while (B < nr) {
		B <<= 1;
		bits++;
	}
	if (bits < 8) {
		bits = 8;
		B = 256;
	}
	const uint64_t mask = B - 1;
	DevBuf bk(nr * 8 + 8), bk2(nr * 8 + 8), bi(nr * 4 + 4), bi2(nr * 4 + 4), bcnt(B * 4), boff((B + 1) * 8);
	DevBuf skey(nr * 8 + 8), snil(nr + 8), lcnt(nl * 4 + 4), ooff(nl * 8 + 8);
	if (!bk.p || !bk2.p || !bi.p || !bi2.p || !bcnt.p || !boff.p || !skey.p || !snil.p || !lcnt.p || !ooff.p)
		return -1;
	if (!hip_ok(hipMemsetAsync(bcnt.p, 0, B * 4, st), "memset"))
		return -1;
	if (nr)
		hipLaunchKernelGGL(k_build_keys, dim3(grid_for(nr, 1024, 8192)), dim3(256), 0, st, R, nr, mask,
				   bk.as<uint64_t>(), bi.as<uint32_t>(), bcnt.as<uint32_t>());
	uint64_t *sk;
	uint32_t *si;
	if (radix_sort_pairs(bk.as<uint64_t>(), bi.as<uint32_t>(), bk2.as<uint64_t>(), bi2.as<uint32_t>(), nr, bits,
			     &sk, &si) < 0)
		return -1;
	uint64_t tot = 0;
	if (exclusive_scan(bcnt.as<uint32_t>(), boff.as<uint64_t>(), B, &tot) < 0)
		return -1;
	if (!hip_ok(hipMemcpyAsync(boff.as<uint64_t>() + B, &tot, 8, hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	if (nr)
		hipLaunchKernelGGL(k_build_gather, dim3(grid_for(nr, 1024, 8192)), dim3(256), 0, st, R, nr, si,
				   skey.as<uint64_t>(), snil.as<uint8_t>());
	if (nl)
		hipLaunchKernelGGL((k_probe<false>), dim3(grid_for(nl, 1024, 8192)), dim3(256), 0, st, L, nl, mask,
				   boff.as<uint64_t>(), skey.as<uint64_t>(), snil.as<uint8_t>(), si, R, nil_matches,
				   lcnt.as<uint32_t>(), nullptr, nullptr, nullptr);
	uint64_t nout = 0;
	if (exclusive_scan(lcnt.as<uint32_t>(), ooff.as<uint64_t>(), nl, &nout) < 0)
		return -1;
	mgdk_bat *a = newbat(0, MGDK_oid, nout), *b = newbat(0, MGDK_oid, nout);
	if (!a || !b) {
		unfix2(a, b);
		return -1;
	}
	if (nl && nout)
		hipLaunchKernelGGL((k_probe<true>), dim3(grid_for(nl, 1024, 8192)), dim3(256), 0, st, L, nl, mask,
				   boff.as<uint64_t>(), skey.as<uint64_t>(), snil.as<uint8_t>(), si, R, nil_matches,
				   nullptr, ooff.as<uint64_t>(), (oid *) a->theap, (oid *) b->theap);
	if (!sync()) {
		unfix2(a, b);
		return -1;
	}
	a->count = b->count = nout;
	*ap = a;
	*bp = b;
	return 0;
}


// ---------------------------------------------------------------------------
// Radix-partitioned path (4-byte keys, unique build keys): the build side is
// cut into P = 2^pbits hash partitions of <= ~8 Ki keys, each of which
// becomes an LDS-resident open-addressing table (16 Ki slots, 128 KiB) in the
// workgroup that probes it; the probe side is cut into the same partitions.
// Both cuts are three passes over the side in 32 Ki-row subtiles: a
// histogram per (subtile, partition), a column scan, and a scatter of
// (key, row) entries whose slot comes from an LDS counter (no global
// atomics; a subtile's entries of one partition form one contiguous run).
// The probe workgroup rewrites each of its entries in place as
// (match + 1, row).  The left order is restored per subtile: the restore
// workgroup reads its subtile's run in every partition, drops each match
// into an LDS array indexed by row, and compacts the matched rows in order
// (output offset by decoupled look-back over the subtiles).  Every global
// access is a stream or a short contiguous run; the only random accesses are
// LDS ones.  Duplicate build keys (detected during the LDS build) or an
// oversized partition send the join to the open-addressing path.
// ---------------------------------------------------------------------------

constexpr uint32_t PJ_SUBROWS = 32768;     // rows per subtile (the restore's LDS array)
constexpr int PJ_SUBS = 1;                 // subtiles per histogram workgroup
constexpr uint32_t PJ_SLOTS = 16384;       // LDS hash slots per build partition (128 KiB)
constexpr uint32_t PJ_MAXFILL = 12288;     // largest build partition accepted
constexpr int PJ_MAXPBITS = 11;            // <= 2048 partitions (LDS counters)
constexpr uint32_t PJ_LDS_SUBS = 4096;     // probe subtiles whose run offsets the probe stages in LDS

// one 32-bit multiplicative (Fibonacci) hash per key: the partition is its
// top pbits, the LDS home the next 14 bits.  A 64-bit mixer costs two
// quarter-rate 64-bit multiplies per key, which bounded these passes;
// skewed inputs are caught by the partition-size check (PJ_MAXFILL).
__device__ __forceinline__ uint32_t
pj_hash(uint32_t key)
{
	return key * 0x9E3779B1u;
}

__device__ __forceinline__ uint32_t
pj_part32(uint32_t key, int pbits)
{
	return pj_hash(key) >> (32 - pbits);
}

__device__ __forceinline__ uint32_t
pj_home(uint32_t key, int pbits)
{
	return (pj_hash(key) >> (32 - pbits - 14)) & 16383;
}

// home bucket of a key in a table of nbp buckets: the hash bits below the
// partition bits, scaled
__device__ __forceinline__ uint32_t
gt_home(uint32_t hk, int pbits, uint32_t nbp)
{
	return __umulhi(hk << pbits, nbp);
}

// 1024-thread workgroup reduction (16 waves); result valid in thread 0
template <typename T, typename F>
__device__ __forceinline__ T
block_reduce16(T v, F op)
{
	__shared__ T s_r16[16];
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v = op(v, __shfl_xor(v, o));
	__syncthreads();
	if (__lane_id() == 0)
		s_r16[threadIdx.x >> 6] = v;
	__syncthreads();
	if (threadIdx.x == 0)
		for (int q = 1; q < 16; q++)
			v = op(v, s_r16[q]);
	return v;
}

// 8-byte key as the 4-byte key image of the partitioned paths: values in
// [INT32_MIN + 1, INT32_MAX] keep their bits, nil becomes the 4-byte nil
// image; any other value does not fit (*fits = false).  The image is
// injective on the values that fit, so equal images mean equal keys.
__device__ __forceinline__ uint32_t
narrow_key(const Side &s, uint64_t v, bool isnil, bool &fits)
{
	if (isnil) {
		fits = true;
		return 0x80000000u;
	}
	const int64_t x = (int64_t) v;
	fits = s.uns ? v <= 0x7fffffffull : (x > (int64_t) INT32_MIN && x <= (int64_t) INT32_MAX);
	return (uint32_t) x;
}

// 16 consecutive keys of side s from candidate index i0 as 4-byte images
// (vector loads for a dense side with 16-byte aligned rows); ok[q] = exists,
// counts and (8-byte keys) has a 4-byte image -- a value without one is
// flagged in s.nofit (the build side then falls back; a probe value without
// one cannot match a build side whose values all fit)
__device__ __forceinline__ void
pj_keys16(const Side &s, BUN i0, BUN n, bool skipnil, uint32_t k[16], bool ok[16])
{
	if (s.w == 4 && s.dense && i0 + 16 <= n && ((s.off + i0) & 3) == 0) {
		typedef int32_t i4 __attribute__((ext_vector_type(4)));
		const i4 *src = (const i4 *) ((const int32_t *) s.base + s.off + i0);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const i4 v = __builtin_nontemporal_load(src + q);
			k[4 * q] = (uint32_t) v.x;
			k[4 * q + 1] = (uint32_t) v.y;
			k[4 * q + 2] = (uint32_t) v.z;
			k[4 * q + 3] = (uint32_t) v.w;
		}
#pragma unroll
		for (int q = 0; q < 16; q++)
			ok[q] = !(skipnil && k[q] == 0x80000000u);
		return;
	}
	bool bad = false;
	if (s.w == 8 && s.base && s.dense && i0 + 16 <= n && ((s.off + i0) & 1) == 0) {
		typedef long long l2 __attribute__((ext_vector_type(2)));
		const l2 *src = (const l2 *) ((const int64_t *) s.base + s.off + i0);
		const uint64_t nilv = s.uns ? (1ull << 63) : (uint64_t) INT64_MIN;
#pragma unroll
		for (int q = 0; q < 8; q++) {
			const l2 v = __builtin_nontemporal_load(src + q);
#pragma unroll
			for (int e = 0; e < 2; e++) {
				const uint64_t x = (uint64_t) (e ? v.y : v.x);
				bool fits;
				const bool isnil = x == nilv;
				k[2 * q + e] = narrow_key(s, x, isnil, fits);
				ok[2 * q + e] = fits && !(isnil && skipnil);
				bad |= !fits;
			}
		}
	} else {
#pragma unroll
		for (int q = 0; q < 16; q++) {
			ok[q] = false;
			k[q] = 0;
			if (i0 + q < n) {
				bool isnil, fits = true;
				const uint64_t v = key_of(s, i0 + q, isnil);
				k[q] = s.w == 8 ? narrow_key(s, v, isnil, fits) : (uint32_t) v;
				ok[q] = fits && !(isnil && skipnil);
				bad |= !fits;
			}
		}
	}
	if (bad && s.nofit)
		atomicOr(s.nofit, 1u);
}

// histogram: cnt[sub][p] = rows of subtile sub in partition p
__global__ __launch_bounds__(1024) void
k_pj_hist(Side s, BUN n, int pbits, bool skipnil, uint32_t *cnt)
{
	__shared__ uint32_t c[1u << PJ_MAXPBITS];
	const uint32_t P = 1u << pbits;
	for (int k = 0; k < PJ_SUBS; k++) {
		const BUN sub = (BUN) blockIdx.x * PJ_SUBS + k;
		const BUN a = sub * PJ_SUBROWS;
		if (a >= n)
			break;
		const BUN e = min(n, a + PJ_SUBROWS);
		for (uint32_t p = threadIdx.x; p < P; p += blockDim.x)
			c[p] = 0;
		__syncthreads();
		for (BUN i0 = a + (BUN) threadIdx.x * 16; i0 < e; i0 += (BUN) blockDim.x * 16) {
			uint32_t k[16];
			bool ok[16];
			pj_keys16(s, i0, e, skipnil, k, ok);
#pragma unroll
			for (int q = 0; q < 16; q++)
				if (ok[q])
					atomicAdd(&c[pj_part32(k[q], pbits)], 1u);
		}
		__syncthreads();
		for (uint32_t p = threadIdx.x; p < P; p += blockDim.x)
			cnt[sub * P + p] = c[p];
		__syncthreads();
	}
}

// XCD-aware remap (cdna_hip_programming.md T1, bijective form): workgroups
// are dealt round-robin to the 8 XCDs; XCD x gets the contiguous index block
// [x q + min(x, r), ...) of the G = 8 q + r indices, so neighbouring runs of
// one partition (written by neighbouring subtiles / partitions) are stored
// through the same L2, where their partial lines merge
__device__ __forceinline__ uint32_t
xcd_block(uint32_t b, uint32_t G)
{
	const uint32_t x = b & 7, k = b >> 3, q = G >> 3, r = G & 7;
	return x * q + (x < r ? x : r) + k;
}

// scatter of (key, row) entries: one workgroup per subtile, in halves of
// 16 Ki rows that are counting-sorted by partition in LDS first, so each
// partition's piece of the run is stored by consecutive lanes.  Both halves'
// keys are loaded before the first is ranked (straight-line loads on a full,
// aligned dense subtile), so the second half's loads are in flight while the
// first half is staged and stored.
constexpr uint32_t PJ_HALF = PJ_SUBROWS / 2;
constexpr int PJ_RPT = PJ_HALF / 1024;         // rows per thread per half

template <bool FULL>
__device__ __forceinline__ void
pj_scatter_sub(const Side &s, BUN n, int pbits, bool skipnil, BUN a0, uint2 *ent, uint2 *stage, uint32_t *hist,
	       uint32_t *start, uint32_t *gcur, uint32_t *wsum)
{
	const uint32_t P = 1u << pbits;
	const unsigned tid = threadIdx.x;
	static_assert(PJ_RPT == 16, "16 rows per thread");
	uint32_t kk[2][PJ_RPT];
	bool ok[2][PJ_RPT];
#pragma unroll
	for (int half = 0; half < 2; half++) {
		const BUN i0 = a0 + (BUN) half * PJ_HALF + (BUN) tid * 16;
		if constexpr (FULL) {
			typedef int32_t i4 __attribute__((ext_vector_type(4)));
			const i4 *src = (const i4 *) ((const int32_t *) s.base + s.off + i0);
#pragma unroll
			for (int q = 0; q < 4; q++) {
				const i4 v = __builtin_nontemporal_load(src + q);
				kk[half][4 * q] = (uint32_t) v.x;
				kk[half][4 * q + 1] = (uint32_t) v.y;
				kk[half][4 * q + 2] = (uint32_t) v.z;
				kk[half][4 * q + 3] = (uint32_t) v.w;
			}
#pragma unroll
			for (int q = 0; q < 16; q++)
				ok[half][q] = !(skipnil && kk[half][q] == 0x80000000u);
		} else {
			pj_keys16(s, i0, min(n, a0 + (BUN) (half + 1) * PJ_HALF), skipnil, kk[half], ok[half]);
		}
	}
#pragma unroll
	for (int half = 0; half < 2; half++) {
		const BUN a = a0 + (BUN) half * PJ_HALF;
		if (!FULL && a >= n)
			break;
		for (uint32_t p = tid; p < P; p += blockDim.x)
			hist[p] = 0;
		__syncthreads();
		uint32_t pp[PJ_RPT], rk[PJ_RPT];
#pragma unroll
		for (int q = 0; q < PJ_RPT; q++)
			pp[q] = ok[half][q] ? pj_part32(kk[half][q], pbits) : ~0u;
#pragma unroll
		for (int q = 0; q < PJ_RPT; q++)
			if (pp[q] != ~0u)
				rk[q] = atomicAdd(&hist[pp[q]], 1u);
		__syncthreads();
		// exclusive scan of hist[0..P) into start (P <= 4096: 4 per thread)
		uint32_t loc[4], t = 0;
		const uint32_t per = (P + 1023) / 1024;
		for (uint32_t q = 0; q < per; q++) {
			const uint32_t p = tid * per + q;
			loc[q] = p < P ? hist[p] : 0;
			t += loc[q];
		}
		uint32_t x = t;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t u = __shfl_up(x, o);
			if (__lane_id() >= (unsigned) o)
				x += u;
		}
		if (__lane_id() == 63)
			wsum[tid >> 6] = x;
		__syncthreads();
		uint32_t pre = x - t, total = 0;
		for (uint32_t w = 0; w < 16; w++) {
			pre += w < (tid >> 6) ? wsum[w] : 0;
			total += wsum[w];
		}
		for (uint32_t q = 0; q < per; q++) {
			const uint32_t p = tid * per + q;
			if (p < P)
				start[p] = pre;
			pre += loc[q];
		}
		__syncthreads();
#pragma unroll
		for (int q = 0; q < PJ_RPT; q++)
			if (pp[q] != ~0u)
				stage[start[pp[q]] + rk[q]] = make_uint2(kk[half][q], (uint32_t) (a + (BUN) tid * 16 + q));
		__syncthreads();
		for (uint32_t j = tid; j < total; j += blockDim.x) {
			const uint2 en = stage[j];
			const uint32_t p = pj_part32(en.x, pbits);
			ent[gcur[p] + (j - start[p])] = en;
		}
		__syncthreads();
		for (uint32_t p = tid; p < P; p += blockDim.x)
			gcur[p] += hist[p];
		__syncthreads();
	}
}

__global__ __launch_bounds__(1024) void
k_pj_scatter(Side s, BUN n, int pbits, bool skipnil, const uint32_t *off, const uint32_t *base, uint2 *ent)
{
	__shared__ uint2 stage[PJ_HALF];
	__shared__ uint32_t hist[1u << PJ_MAXPBITS], start[1u << PJ_MAXPBITS], gcur[1u << PJ_MAXPBITS];
	__shared__ uint32_t wsum[16];
	const uint32_t P = 1u << pbits;
	const BUN sub = xcd_block(blockIdx.x, gridDim.x);
	const BUN a0 = sub * PJ_SUBROWS;
	for (uint32_t p = threadIdx.x; p < P; p += blockDim.x)
		gcur[p] = base[p] + off[sub * P + p];
	if (s.w == 4 && s.dense && a0 + PJ_SUBROWS <= n && ((s.off + a0) & 3) == 0)
		pj_scatter_sub<true>(s, n, pbits, skipnil, a0, ent, stage, hist, start, gcur, wsum);
	else
		pj_scatter_sub<false>(s, n, pbits, skipnil, a0, ent, stage, hist, start, gcur, wsum);
}

// column-exclusive prefix of cnt[nsub][P] (64 columns x 16 row groups per
// workgroup); tot[p] = column total
__global__ __launch_bounds__(1024) void
k_pj_colscan(const uint32_t *cnt, uint32_t nsub, uint32_t P, uint32_t *off, uint32_t *tot)
{
	__shared__ uint32_t part[16][64];
	const uint32_t cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
	const uint32_t col = blockIdx.x * 64 + cl;
	const uint32_t per = (nsub + 15) / 16;
	const uint32_t r0 = min(nsub, grp * per), r1 = min(nsub, r0 + per);
	uint32_t sum = 0;
#pragma unroll 8
	for (uint32_t r = r0; r < r1; r++)
		sum += cnt[(size_t) r * P + col];
	part[grp][cl] = sum;
	__syncthreads();
	uint32_t pre = 0;
	for (uint32_t g = 0; g < grp; g++)
		pre += part[g][cl];
#pragma unroll 8
	for (uint32_t r = r0; r < r1; r++) {
		const uint32_t v = cnt[(size_t) r * P + col];
		off[(size_t) r * P + col] = pre;
		pre += v;
	}
	if (grp == 15)
		tot[col] = pre;
}

// base[p] = exclusive prefix of tot (one workgroup; P <= 4096)
__global__ __launch_bounds__(1024) void
k_pj_base(const uint32_t *tot, uint32_t P, uint32_t *base, uint32_t *maxtot)
{
	__shared__ uint32_t wsum[16];
	__shared__ uint32_t carry;
	if (threadIdx.x == 0)
		carry = 0;
	uint32_t mx = 0;
	for (uint32_t b = 0; b < P; b += 1024) {
		__syncthreads();
		const uint32_t p = b + threadIdx.x;
		const uint32_t v = p < P ? tot[p] : 0;
		mx = v > mx ? v : mx;
		uint32_t x = v;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t u = __shfl_up(x, o);
			if (__lane_id() >= (unsigned) o)
				x += u;
		}
		if (__lane_id() == 63)
			wsum[threadIdx.x >> 6] = x;
		__syncthreads();
		uint32_t wpre = 0;
		for (uint32_t w = 0; w < (threadIdx.x >> 6); w++)
			wpre += wsum[w];
		if (p < P)
			base[p] = carry + wpre + x - v;
		__syncthreads();
		if (threadIdx.x == 1023)
			carry += wpre + x;
	}
	__syncthreads();
	if (threadIdx.x == 0)
		base[P] = carry;
	mx = block_reduce16(mx, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
	if (threadIdx.x == 0)
		*maxtot = mx;
}

// one workgroup per partition: LDS table of the build entries, then each
// probe entry of the partition is answered and stored, as (match position +
// 1 or 0, row), at its subtile-major place in the flat array (the column of
// run offsets deltaT[p][*] staged in LDS).  The table is nbp 16-byte buckets
// (2 slots, linear probing over slots from an even home slot) sized from the
// largest build partition, in dynamic LDS together with the offsets column:
// at ~80 % load a 15M-row build side needs < 80 KiB, so two workgroups share
// a CU and one's table build overlaps the other's probe.
__global__ __launch_bounds__(1024) void
k_pj_probe(const uint2 *bent, const uint32_t *bbase, const uint2 *pent, const uint32_t *pbase, int pbits,
	   uint32_t nbp, const uint32_t *deltaT, uint32_t nsub, bool ldsd, uint2 *flat, uint32_t *dupflag)
{
	extern __shared__ __attribute__((aligned(16))) unsigned long long dyn[];
	unsigned long long *tab = dyn;
	uint32_t *sdelta = (uint32_t *) (dyn + 2 * nbp);
	const uint32_t p = xcd_block(blockIdx.x, gridDim.x), ns = 2 * nbp;
	for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x)
		tab[i] = 0ull;
	const uint32_t *dcol = deltaT + (size_t) p * nsub;
	if (ldsd)
		for (uint32_t i = threadIdx.x; i < nsub; i += blockDim.x)
			sdelta[i] = dcol[i];
	__syncthreads();
	// the first batch of probe entries is loaded while the table is built,
	// and every later batch while the previous one is answered
	constexpr int U = 8;
	const uint32_t q0 = pbase[p], q1 = pbase[p + 1];
	uint2 cur[U];
#pragma unroll
	for (int u = 0; u < U; u++) {
		const uint32_t e = q0 + threadIdx.x + u * blockDim.x;
		cur[u] = pent[e < q1 ? e : q0];
	}
	const uint32_t b0 = bbase[p], b1 = bbase[p + 1];
	bool dup = false;
	for (uint32_t e = b0 + threadIdx.x; e < b1; e += blockDim.x) {
		const uint2 en = bent[e];
		const unsigned long long v = ((unsigned long long) (en.y + 1) << 32) | en.x;
		uint32_t h = 2 * gt_home(pj_hash(en.x), pbits, nbp);
		for (;;) {
			const unsigned long long o = atomicCAS(&tab[h], 0ull, v);
			if (o == 0ull)
				break;
			if ((uint32_t) o == en.x) {
				dup = true;
				break;
			}
			h = h + 1 == ns ? 0 : h + 1;
		}
	}
	if (__any(dup) && __lane_id() == 0)
		atomicOr(dupflag, 1u);
	__syncthreads();
	const ulonglong2 *bk = (const ulonglong2 *) tab;
	for (uint32_t e0 = q0 + threadIdx.x; e0 < q1; e0 += U * blockDim.x) {
		uint2 en[U], nxt[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			en[u] = cur[u];
			const uint32_t e = e0 + (U + u) * blockDim.x;
			nxt[u] = pent[e < q1 ? e : q0];
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			uint32_t b = gt_home(pj_hash(en[u].x), pbits, nbp), m = 0;
			for (;;) {
				const ulonglong2 sl = bk[b];
				if (sl.x == 0ull)
					break;
				if ((uint32_t) sl.x == en[u].x) {
					m = (uint32_t) (sl.x >> 32);
					break;
				}
				if (sl.y == 0ull)
					break;
				if ((uint32_t) sl.y == en[u].x) {
					m = (uint32_t) (sl.y >> 32);
					break;
				}
				b = b + 1 == nbp ? 0 : b + 1;
			}
			en[u].x = m;
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t e = e0 + u * blockDim.x;
			const uint32_t sub = en[u].y / PJ_SUBROWS;
			if (e < q1)
				flat[e + (ldsd ? sdelta[sub] : dcol[sub])] = en[u];
		}
#pragma unroll
		for (int u = 0; u < U; u++)
			cur[u] = nxt[u];
	}
}

// deltaT[p][sub] = (subtile-major start of the run of (sub, p)) - (its start
// in the partition-major entries), mod 2^32: the probe stores entry e of
// that run at e + delta, so each subtile's results end up contiguous for the
// restore.  64 x 64 tiles transposed through LDS.
__global__ __launch_bounds__(256) void
k_pj_delta(const uint32_t *offT, const uint32_t *poff, const uint32_t *pbase, uint32_t nsub, uint32_t P,
	   uint32_t *deltaT)
{
	__shared__ uint32_t t[64][65];
	const uint32_t s0 = blockIdx.x * 64, p0 = blockIdx.y * 64;
	for (uint32_t k = threadIdx.x; k < 64 * 64; k += blockDim.x) {
		const uint32_t r = k / 64, c = k % 64, sub = s0 + r, p = p0 + c;
		if (sub < nsub && p < P)
			t[r][c] = offT[(size_t) sub * P + p] - pbase[p] - poff[(size_t) sub * P + p];
	}
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < 64 * 64; k += blockDim.x) {
		const uint32_t r = k / 64, c = k % 64, p = p0 + r, sub = s0 + c;
		if (sub < nsub && p < P)
			deltaT[(size_t) p * nsub + sub] = t[c][r];
	}
}

// the emit's LDS (per workgroup)
struct EmitLds {
	uint32_t rmask[1024], rbase[1024], wsum[16];
	uint64_t pre;
};

// first half: thread tid counts the rows [32 tid, 32 tid + 32) -- a match
// mask and the run's exclusive offset, so the write below can walk the rows
// in order (consecutive lanes -> consecutive positions) without barriers --
// and wave 0 takes the subtile's output offset by look-back (in e.pre after
// the closing barrier)
__device__ __forceinline__ void
pj_emit_scan(const uint32_t *res, uint32_t sub, uint32_t rows, uint32_t nsub, uint64_t *status, uint64_t *meta,
	     EmitLds &e)
{
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	static_assert(PJ_SUBROWS == 32 * 1024, "32 rows per thread");
	const uint32_t r0 = tid * 32, rb = tid * 33;
	uint32_t msk = 0;
#pragma unroll
	for (int k = 0; k < 32; k++)
		msk |= (uint32_t) ((r0 + k < rows) && res[rb + k] != 0) << k;
	const uint32_t c = __popc(msk);
	uint32_t x = c;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t u = __shfl_up(x, o);
		if (lane >= (unsigned) o)
			x += u;
	}
	if (lane == 63)
		e.wsum[w] = x;
	__syncthreads();
	uint32_t wpre = 0, tot = 0;
	for (uint32_t q = 0; q < 16; q++) {
		wpre += q < w ? e.wsum[q] : 0;
		tot += e.wsum[q];
	}
	e.rmask[tid] = msk;
	e.rbase[tid] = wpre + x - c;
	if (w == 0) {
		const uint64_t pre = lookback(status, sub, tot, (uint32_t *) &meta[1]);
		if (lane == 0) {
			e.pre = pre;
			if (sub == nsub - 1)
				meta[0] = pre + tot;
		}
	}
	__syncthreads();
}

// second half: the pairs of the matched rows at their output positions
__device__ __forceinline__ void
pj_emit_write(const uint32_t *res, BUN a, uint32_t rows, const Side &L, const Side &R, const EmitLds &e, oid *r1,
	      oid *r2)
{
	const uint64_t pre = e.pre;
	for (uint32_t r = threadIdx.x; r < rows; r += blockDim.x) {
		const uint32_t run = r >> 5, bit = r & 31;
		const uint32_t mk = e.rmask[run];
		if ((mk >> bit) & 1) {
			const uint64_t o = pre + e.rbase[run] + __popc(mk & ((1u << bit) - 1));
			r1[o] = oid_of(L, a + r);
			r2[o] = oid_of(R, res[r + run] - 1);
		}
	}
}

// the subtile's matches back in row order (shared by both restores):
// res[r + r / 32] = match position + 1 of row r (0: none); output offset by
// decoupled look-back over the subtiles (numbered by ticket)
__device__ __forceinline__ void
pj_emit(const uint32_t *res, uint32_t sub, BUN a, uint32_t rows, uint32_t nsub, const Side &L, const Side &R,
	uint64_t *status, uint64_t *meta, oid *r1, oid *r2)
{
	__shared__ EmitLds e;
	pj_emit_scan(res, sub, rows, nsub, status, meta, e);
	pj_emit_write(res, a, rows, L, R, e, r1, r2);
}

// one workgroup per subtile (ticketed): matches back into row order; the
// subtile's probe results are the contiguous range [offT[sub][0],
// offT[sub + 1][0]) of the flat array
__global__ __launch_bounds__(1024) void
k_pj_restore(const uint2 *flat, const uint32_t *offT, uint32_t P, uint64_t total, BUN n, uint32_t nsub, Side L,
	     Side R, uint32_t *ticket, uint64_t *status, uint64_t *meta, oid *r1, oid *r2)
{
	// res[row + row / 32]: one pad word per 32 rows, so the 32-row runs of
	// consecutive threads fall in different banks
	__shared__ uint32_t res[PJ_SUBROWS + PJ_SUBROWS / 32];
	__shared__ uint32_t s_sub;
	const unsigned tid = threadIdx.x;
	if (tid == 0)
		s_sub = atomicAdd(ticket, 1u);
	for (uint32_t i = tid; i < PJ_SUBROWS + PJ_SUBROWS / 32; i += blockDim.x)
		res[i] = 0;
	__syncthreads();
	const uint32_t sub = s_sub;
	const BUN a = (BUN) sub * PJ_SUBROWS;
	const uint32_t rows = (uint32_t) min((BUN) PJ_SUBROWS, n - a);
	const uint32_t f0 = offT[(size_t) sub * P];
	const uint32_t f1 = sub + 1 < nsub ? offT[(size_t) (sub + 1) * P] : (uint32_t) total;
	constexpr int U = 8;
	for (uint32_t j0 = f0 + tid; j0 < f1; j0 += U * blockDim.x) {
		uint2 en[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t j = j0 + u * blockDim.x;
			en[u] = j < f1 ? flat[j] : make_uint2(0, (uint32_t) a);
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t r = en[u].y - (uint32_t) a;
			if (en[u].x)
				res[r + (r >> 5)] = en[u].x;
		}
	}
	__syncthreads();
	pj_emit(res, sub, a, rows, nsub, L, R, status, meta, r1, r2);
}

// ---------------------------------------------------------------------------
// Probe side with subtile-local runs (round 5, default; MGDK_JOIN_PART=3 runs
// the cut / probe / restore above).  The cut above stores each (subtile,
// partition) run at its partition-major place: ~8 entries of 8 B per run,
// written as 64-B pieces by different workgroups (1.9 TB/s), after a
// histogram pass over the keys.  Here every subtile keeps its own region:
//   k_pj2_cut     one pass, no histogram: the subtile's keys counting-sorted
//                 by partition in LDS and stored contiguously (4-B key images
//                 in pkey, the 2-B row inside the subtile in prow, split so
//                 the probe reads keys only) + the run starts poff[s][0..P]
//                 (uint16; poff[s][P] = the subtile's entries);
//   k_pj2_offt    the run starts transposed (partition-major);
//   k_pj2_probe   one workgroup per partition builds its LDS table and answers
//                 its run of every subtile: a wave takes the runs of 64
//                 subtiles at once, numbers their entries by a wave scan of
//                 the run lengths and lets lane l take entries l, l + 64, ...
//                 (a binary search over the 64 run starts finds an entry's
//                 run), so the key loads of a run are consecutive lanes; the
//                 4-B answer (match + 1, 0 = none) goes to the key's own index
//                 in pans;
//   k_pj2_restore per subtile: the answers dropped into the LDS row array
//                 through prow, then pj_emit.
// Probe-side bytes per row: 4 read + 6 written, 4 + 4, 6 + 16 (40 B) against
// 4, 4 + 8, 8 + 8, 8 + 16 (56 B) for the plan above.
// ---------------------------------------------------------------------------

constexpr size_t PJ2_CUT_LDS = ((size_t) (1u << PJ_MAXPBITS) + PJ_SUBROWS) * 4;
// the probe's LDS: table buckets + the waves' run lists (16 x 64 x 8 B)
constexpr uint32_t PJ2_MAXB = (160 * 1024 - 16 * 64 * 8) / 16;
constexpr uint32_t PJ2_MAXFILL = PJ2_MAXB * 2 * 4 / 5;       // <= 80 % load

__global__ __launch_bounds__(1024) void
k_pj2_cut(Side s, BUN n, int pbits, bool skipnil, uint32_t *pkey, uint16_t *prow, uint16_t *poff, uint64_t *rzero)
{
	// the restore's ticket words and look-back status, cleared here instead
	// of by a memset of their own: 8 words, then one per subtile
	if (rzero != nullptr && threadIdx.x < 8 && (blockIdx.x == 0 || threadIdx.x == 0))
		rzero[blockIdx.x == 0 ? threadIdx.x : 8 + blockIdx.x] = 0;
	if (rzero != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
		rzero[8] = 0;
	extern __shared__ __attribute__((aligned(16))) uint32_t sm2[];
	uint32_t *hist = sm2;                          // counters, then run starts
	uint32_t *stk = sm2 + (1u << PJ_MAXPBITS);     // the run-ordered keys, then rows
	__shared__ uint32_t wsum[16];
	const uint32_t P = 1u << pbits;
	const unsigned tid = threadIdx.x, lane = __lane_id();
	const uint32_t sub = blockIdx.x;
	const BUN a = (BUN) sub * PJ_SUBROWS;
	for (uint32_t p = tid; p < P; p += blockDim.x)
		hist[p] = 0;
	uint32_t kk[2][16], rk[2][16];
	bool ok[2][16];
	// a full, aligned dense 4-byte subtile: lane-consecutive 16-B loads (one
	// 1-KiB piece per wave instruction), key (half, q) = row
	// (half * 4 + q / 4) * 4096 + tid * 4 + q % 4; otherwise 16 consecutive
	// rows per thread and half, key (half, q) = row half * 16384 + tid * 16 + q
	const bool fast = s.w == 4 && s.dense && a + PJ_SUBROWS <= n && ((s.off + a) & 3) == 0;
	if (fast) {
		typedef int32_t i4 __attribute__((ext_vector_type(4)));
		const i4 *src = (const i4 *) ((const int32_t *) s.base + s.off + a);
#pragma unroll
		for (int half = 0; half < 2; half++)
#pragma unroll
			for (int q4 = 0; q4 < 4; q4++) {
				const i4 v = __builtin_nontemporal_load(src + (half * 4 + q4) * 1024 + tid);
				kk[half][4 * q4] = (uint32_t) v.x;
				kk[half][4 * q4 + 1] = (uint32_t) v.y;
				kk[half][4 * q4 + 2] = (uint32_t) v.z;
				kk[half][4 * q4 + 3] = (uint32_t) v.w;
			}
#pragma unroll
		for (int half = 0; half < 2; half++)
#pragma unroll
			for (int q = 0; q < 16; q++)
				ok[half][q] = !(skipnil && kk[half][q] == 0x80000000u);
	} else {
#pragma unroll
		for (int half = 0; half < 2; half++)
			pj_keys16(s, a + (BUN) half * PJ_HALF + (BUN) tid * 16, n, skipnil, kk[half], ok[half]);
	}
	__syncthreads();
#pragma unroll
	for (int half = 0; half < 2; half++)
#pragma unroll
		for (int q = 0; q < 16; q++)
			if (ok[half][q])
				rk[half][q] = atomicAdd(&hist[pj_part32(kk[half][q], pbits)], 1u);
	__syncthreads();
	// exclusive scan of the counters in place (P <= 2048: two per thread)
	static_assert((1u << PJ_MAXPBITS) <= 2048, "two counters per thread");
	const uint32_t p0 = 2 * tid;
	const uint32_t c0 = p0 < P ? hist[p0] : 0, c1 = p0 + 1 < P ? hist[p0 + 1] : 0;
	uint32_t x = c0 + c1;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t u = __shfl_up(x, o);
		if (lane >= (unsigned) o)
			x += u;
	}
	if (lane == 63)
		wsum[tid >> 6] = x;
	__syncthreads();
	uint32_t pre = x - c0 - c1, total = 0;
	for (uint32_t w = 0; w < 16; w++) {
		pre += w < (tid >> 6) ? wsum[w] : 0;
		total += wsum[w];
	}
	uint16_t *po = poff + (size_t) sub * (P + 1);
	if (p0 < P) {
		hist[p0] = pre;
		po[p0] = (uint16_t) pre;
	}
	if (p0 + 1 < P) {
		hist[p0 + 1] = pre + c0;
		po[p0 + 1] = (uint16_t) (pre + c0);
	}
	if (tid == 0)
		po[P] = (uint16_t) total;      // <= PJ_SUBROWS = 32768 fits
	__syncthreads();
#pragma unroll
	for (int half = 0; half < 2; half++)
#pragma unroll
		for (int q = 0; q < 16; q++)
			if (ok[half][q]) {
				rk[half][q] += hist[pj_part32(kk[half][q], pbits)];
				stk[rk[half][q]] = kk[half][q];
			}
	__syncthreads();
	// whole 16-B pieces: the region holds PJ_SUBROWS entries, so rounding
	// the count up to a multiple of 4 (8 for the rows) stays inside it
	typedef uint32_t u4 __attribute__((ext_vector_type(4)));
	u4 *dk = (u4 *) (pkey + a);
	for (uint32_t j = tid; 4 * j < total; j += blockDim.x)
		__builtin_nontemporal_store(((const u4 *) stk)[j], dk + j);
	__syncthreads();
	uint16_t *str = (uint16_t *) stk;
#pragma unroll
	for (int half = 0; half < 2; half++)
#pragma unroll
		for (int q = 0; q < 16; q++)
			if (ok[half][q])
				str[rk[half][q]] = (uint16_t) (fast ? (half * 4 + q / 4) * 4096 + tid * 4 + q % 4
								 : half * PJ_HALF + tid * 16 + q);
	__syncthreads();
	u4 *dr = (u4 *) (prow + a);
	for (uint32_t j = tid; 8 * j < total; j += blockDim.x)
		__builtin_nontemporal_store(((const u4 *) stk)[j], dr + j);
}

// poffT[p][s] = poff[s][p] for p in [0, P]: 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void
k_pj2_offt(const uint16_t *poff, uint32_t nsub, uint32_t P, uint16_t *poffT)
{
	__shared__ uint16_t t[64][65];
	const uint32_t s0 = blockIdx.x * 64, q0 = blockIdx.y * 64;
	for (uint32_t k = threadIdx.x; k < 64 * 64; k += blockDim.x) {
		const uint32_t r = k / 64, c = k % 64;
		if (s0 + r < nsub && q0 + c <= P)
			t[r][c] = poff[(size_t) (s0 + r) * (P + 1) + q0 + c];
	}
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < 64 * 64; k += blockDim.x) {
		const uint32_t r = k / 64, c = k % 64;
		if (s0 + c < nsub && q0 + r <= P)
			poffT[(size_t) (q0 + r) * nsub + s0 + c] = t[c][r];
	}
}

#ifndef PJ2_SIDE
#define PJ2_SIDE 1      // the probe side's cut on the thread's side stream, beside the build side's passes
#endif
#ifndef PJ2_BC
#define PJ2_BC 0        // 1: the build side cut like the probe side (k_pj2_cut, subtile-local runs; measured slower: the
                        // probe then gathers ~16-entry runs from every build subtile, 444 against 270 us)
#endif
#ifndef PJ2_SWAP
#define PJ2_SWAP 1      // 1: the build side's cut on the side stream, the probe side's on the main one
#endif
#ifndef PJ2_RALL
#define PJ2_RALL 1      // the restore loads all of a subtile's entries at once (0: four rounds of 8 per thread)
#endif
#ifndef PJ2_NT
#define PJ2_NT 0        // nontemporal loads of the probe's keys and the restore's answers / rows (A/B)
#endif
#ifndef PJ2_UV
#define PJ2_UV 6
#endif
#ifndef PJ2_BUV
#define PJ2_BUV 4
#endif
constexpr int PJ2_U = PJ2_UV;   // entries per lane in flight in the probe

// one batch of a wave: the runs of subtiles [s0, s0 + 64) in partition p.
// Lane l loads the run bounds of subtile s0 + l; a wave scan of the run
// lengths numbers the batch's entries, and lane l takes entries l, l + 64,
// ... (the run holding entry t: a binary search over the 64 run starts in
// LDS), so the key loads of one run are consecutive lanes.  All PJ2_U key
// loads of a lane are issued here; idx = ~0 marks no entry.
struct Pj2Batch {
	uint32_t tot;
	uint32_t rs, rl, rb;      // PJ2_SRCH: this lane's run (start in the batch, length, index base)
	uint32_t idx[PJ2_U], key[PJ2_U];
};

#ifndef PJ2_DIAG
#define PJ2_DIAG 0      // timing diagnostics only (wrong answers): 1 no table build, 2 no key loads
#endif
#ifndef PJ2_SRCH
#define PJ2_SRCH 1      // entries find their run by a wave max-scan of run marks (0: binary search over LDS)
#endif

// inclusive max-scan over the wave (every value >= -1): Hillis-Steele inside
// the 16-lane rows by DPP row shifts, then the rows' last lanes broadcast
// (row_bcast:15 / :31), no LDS
__device__ __forceinline__ int
wave_max_scan(int x)
{
	x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xf, 0xf, false));   // row_shr:1
	x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xf, 0xf, false));   // row_shr:2
	x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xf, 0xf, false));   // row_shr:4
	x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xf, 0xf, false));   // row_shr:8
	x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xa, 0xf, false));   // row_bcast:15 -> rows 1, 3
	x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xc, 0xf, false));   // row_bcast:31 -> rows 2, 3
	return x;
}

// PJ2_SRCH: the same batch numbering, but entry t's run is the last run that
// starts at or before t: every non-empty run marks its first entry's place
// among the call's 64 PJ2_U entries (a byte in the wave's LDS), each lane
// reads its places and a wave max-scan carries the mark forward; the run
// holding the call's first entry comes from a ballot.  The entry's index is
// the run's base (read from its lane) + t.
__device__ __forceinline__ void
pj2_issue2(const uint32_t *pkey, const uint16_t *o0, const uint16_t *o1, uint32_t nsub, uint32_t s0, uint8_t *slot,
	   uint32_t i0, Pj2Batch &bt, bool scan)
{
	const unsigned lane = __lane_id();
	if (scan) {
		const uint32_t sb = s0 + lane;
		uint32_t b = 0, len = 0;
		if (sb < nsub) {
			b = o0[sb];
			len = o1[sb] - b;
		}
		uint32_t inc = len;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t u = __shfl_up(inc, o);
			if (lane >= (unsigned) o)
				inc += u;
		}
		bt.tot = __shfl(inc, 63);
		bt.rs = inc - len;
		bt.rl = len;
		bt.rb = sb * PJ_SUBROWS + b - bt.rs;
	}
	__builtin_amdgcn_wave_barrier();          // the previous call's reads of slot are done
#pragma unroll
	for (int u = 0; u < PJ2_U; u++)
		slot[u * 64 + lane] = 0xff;
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	if (bt.rl != 0 && bt.rs >= i0 && bt.rs - i0 < 64u * PJ2_U)
		slot[bt.rs - i0] = (uint8_t) lane;
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	const uint64_t before = __ballot(bt.rl != 0 && bt.rs < i0);
	int carry = before ? 63 - __builtin_clzll(before) : 0;
	int mk[PJ2_U];
#pragma unroll
	for (int u = 0; u < PJ2_U; u++) {
		const uint32_t m = slot[u * 64 + lane];
		mk[u] = m == 0xff ? -1 : (int) m;
	}
#pragma unroll
	for (int u = 0; u < PJ2_U; u++) {
		const int r = max(wave_max_scan(mk[u]), carry);
		carry = __builtin_amdgcn_readlane(r, 63);
		const uint32_t t = i0 + u * 64 + lane;
		const uint32_t base = (uint32_t) __shfl((int) bt.rb, r);
		bt.idx[u] = t < bt.tot ? base + t : ~0u;
#if PJ2_DIAG & 2
		bt.key[u] = bt.idx[u];     // timing diagnostic: no key loads
#elif PJ2_NT
		bt.key[u] = t < bt.tot ? __builtin_nontemporal_load(pkey + bt.idx[u]) : 0u;
#else
		bt.key[u] = t < bt.tot ? pkey[bt.idx[u]] : 0u;
#endif
	}
}

__device__ __forceinline__ void
pj2_issue(const uint32_t *pkey, const uint16_t *o0, const uint16_t *o1, uint32_t nsub, uint32_t s0, uint32_t *ws,
	  uint32_t *wb, uint32_t i0, Pj2Batch &bt, bool scan)
{
	const unsigned lane = __lane_id();
	if (scan) {
		const uint32_t sb = s0 + lane;
		uint32_t b = 0, len = 0;
		if (sb < nsub) {
			b = o0[sb];
			len = o1[sb] - b;
		}
		uint32_t inc = len;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t u = __shfl_up(inc, o);
			if (lane >= (unsigned) o)
				inc += u;
		}
		bt.tot = __shfl(inc, 63);
		__builtin_amdgcn_wave_barrier();      // the previous batch's reads of ws / wb are done
		ws[lane] = inc - len;
		wb[lane] = sb * PJ_SUBROWS + b;
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	}
#pragma unroll
	for (int u = 0; u < PJ2_U; u++) {
		const uint32_t t = i0 + u * 64 + lane;
		uint32_t r = 0;
#pragma unroll
		for (uint32_t st = 32; st > 0; st >>= 1)
			r += ws[r + st] <= t ? st : 0;
		bt.idx[u] = t < bt.tot ? wb[r] + (t - ws[r]) : ~0u;
#if PJ2_NT
		bt.key[u] = t < bt.tot ? __builtin_nontemporal_load(pkey + bt.idx[u]) : 0u;
#else
		bt.key[u] = t < bt.tot ? pkey[bt.idx[u]] : 0u;
#endif
	}
}

__device__ __forceinline__ void
pj2_answer(const ulonglong2 *bk, int pbits, uint32_t nbp, const Pj2Batch &bt, uint32_t *pans)
{
#pragma unroll
	for (int u = 0; u < PJ2_U; u++) {
		const uint32_t k = bt.key[u];
		uint32_t bb = gt_home(pj_hash(k), pbits, nbp), m = 0;
		for (;;) {
			const ulonglong2 sl = bk[bb];
			if (sl.x == 0ull)
				break;
			if ((uint32_t) sl.x == k) {
				m = (uint32_t) (sl.x >> 32);
				break;
			}
			if (sl.y == 0ull)
				break;
			if ((uint32_t) sl.y == k) {
				m = (uint32_t) (sl.y >> 32);
				break;
			}
			bb = bb + 1 == nbp ? 0 : bb + 1;
		}
		if (bt.idx[u] != ~0u)
			pans[bt.idx[u]] = m;
	}
}

constexpr int PJ2_BU = PJ2_BUV;  // build entries per thread per round, all loaded before any insert

#ifndef PJ2_TB
#define PJ2_TB 0        // 1: the LDS tables built by their own pass (beside the probe side's cut) and loaded by the
                        // probe -- measured slower (0.89-0.90 against 0.86-0.87 ms: the cut shares the GPU with it)
#endif

// PJ2_TB: partition p's LDS table built as the probe would build it, then
// stored to gtab[p] (2 nbp slots) for the probe to load with plain 16-B
// loads; the build flags (duplicate key, oversized partition) are raised here
__global__ __launch_bounds__(1024) void
k_pj2_tbuild(const uint2 *bent, const uint32_t *bbase, int pbits, uint32_t nbp, unsigned long long *gtab,
	     uint32_t *dupflag)
{
	extern __shared__ __attribute__((aligned(16))) unsigned long long dyn3[];
	unsigned long long *tab = dyn3;
	const uint32_t p = xcd_block(blockIdx.x, gridDim.x), ns = 2 * nbp;
	const unsigned tid = threadIdx.x, lane = __lane_id();
	for (uint32_t i = tid; i < ns; i += blockDim.x)
		tab[i] = 0ull;
	const uint32_t b0 = bbase[p], over = (uint64_t) (bbase[p + 1] - b0) * 10 > (uint64_t) ns * 9;
	const uint32_t b1 = over ? b0 : bbase[p + 1];
	if (over && tid == 0)
		atomicOr(dupflag, 2u);
	bool dup = false;
	uint2 en[PJ2_BUV];
	uint32_t e0 = b0 + tid;
#pragma unroll
	for (int u = 0; u < PJ2_BUV; u++) {
		const uint32_t e = e0 + u * blockDim.x;
		en[u] = e < b1 ? bent[e] : make_uint2(0, 0);
	}
	__syncthreads();                              // the table is zeroed
	while (e0 < b1) {
#pragma unroll
		for (int u = 0; u < PJ2_BUV; u++) {
			if (e0 + u * blockDim.x >= b1)
				continue;
			const unsigned long long v = ((unsigned long long) (en[u].y + 1) << 32) | en[u].x;
			uint32_t h = 2 * gt_home(pj_hash(en[u].x), pbits, nbp);
			for (;;) {
				const unsigned long long o = atomicCAS(&tab[h], 0ull, v);
				if (o == 0ull)
					break;
				if ((uint32_t) o == en[u].x) {
					dup = true;
					break;
				}
				h = h + 1 == ns ? 0 : h + 1;
			}
		}
		e0 += PJ2_BUV * blockDim.x;
#pragma unroll
		for (int u = 0; u < PJ2_BUV; u++) {
			const uint32_t e = e0 + u * blockDim.x;
			en[u] = e < b1 ? bent[e] : make_uint2(0, 0);
		}
	}
	if (__any(dup) && lane == 0)
		atomicOr(dupflag, 1u);
	__syncthreads();
	typedef unsigned long long u2v __attribute__((ext_vector_type(2)));
	u2v *dst = (u2v *) (gtab + (size_t) p * ns);
	for (uint32_t i = tid; i < nbp; i += blockDim.x)
		dst[i] = ((const u2v *) tab)[i];
}

#if PJ2_BC && (PJ2_TB || !PJ2_SRCH)
#error "PJ2_BC needs PJ2_SRCH and not PJ2_TB"
#endif

__global__ __launch_bounds__(1024) void
k_pj2_probe(const uint2 *bent, const uint32_t *bbase, const uint32_t *pkey, const uint16_t *poffT, int pbits,
	    uint32_t nbp, uint32_t nsub, uint32_t *pans, uint32_t *dupflag, const unsigned long long *gtab,
	    const uint32_t *bkey, const uint16_t *brow, const uint16_t *bpoffT, uint32_t nsubB)
{
	extern __shared__ __attribute__((aligned(16))) unsigned long long dyn2[];
	unsigned long long *tab = dyn2;
	uint32_t *wst = (uint32_t *) (dyn2 + 2 * nbp);            // [16][64] run starts in the wave's entry list
	uint32_t *wbs = wst + 16 * 64;                            // [16][64] first index of each run (< 2^32)
	const uint32_t p = xcd_block(blockIdx.x, gridDim.x), ns = 2 * nbp;
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	const uint16_t *o0 = poffT + (size_t) p * nsub, *o1 = poffT + (size_t) (p + 1) * nsub;
	uint32_t *ws = wst + w * 64, *wb = wbs + w * 64;
#if PJ2_SRCH
	// the run marks: 64 PJ2_U bytes per wave in the 16 x 512 B of wst + wbs
	static_assert(PJ2_U <= 8, "64 PJ2_U marks fit a wave's 512 B");
	uint8_t *slot = (uint8_t *) wst + w * 512;
	(void) ws;
	(void) wb;
#endif
#if PJ2_TB
	// the partition's table, built by k_pj2_tbuild
	{
		typedef unsigned long long u2v __attribute__((ext_vector_type(2)));
		const u2v *src = (const u2v *) (gtab + (size_t) p * ns);
		for (uint32_t i = tid; i < nbp; i += blockDim.x)
			((u2v *) tab)[i] = src[i];
	}
#else
	(void) gtab;
	for (uint32_t i = tid; i < ns; i += blockDim.x)
		tab[i] = 0ull;
#endif
#if PJ2_BC
	// the partition's build entries are its run in every build subtile (the
	// build side cut like the probe side, k_pj2_cut): counted first, then
	// inserted a batch of 64 subtiles per wave as the probe takes its runs
	// (pj2_issue2: consecutive lanes load a run's consecutive keys); the row
	// of entry idx is its subtile's first row + brow[idx]
	(void) bent;
	(void) bbase;
	(void) gtab;
	Pj2Batch bt;
	uint32_t s0 = w * 64;
	{
		const uint16_t *q0 = bpoffT + (size_t) p * nsubB, *q1 = bpoffT + (size_t) (p + 1) * nsubB;
		// the waves' counts in their 512-B slot regions past the marks (no
		// static LDS: the dynamic table may take all 160 KB)
		static_assert(64 * PJ2_U + 4 <= 512, "a count word after the marks");
		uint32_t bc = 0;
		for (uint32_t sb = tid; sb < nsubB; sb += blockDim.x)
			bc += (uint32_t) (q1[sb] - q0[sb]);
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			bc += __shfl_xor(bc, o);
		if (lane == 0)
			*(uint32_t *) ((uint8_t *) wst + w * 512 + 64 * PJ2_U) = bc;
		__syncthreads();                          // (also: the table is zeroed)
		uint64_t btot = 0;
		for (int q = 0; q < 16; q++)
			btot += *(const uint32_t *) ((const uint8_t *) wst + q * 512 + 64 * PJ2_U);
		// a build partition above 90 % of the table (the host sized it for
		// the expected largest one) is flagged and not built: its runs are
		// answered "no match" and the host falls back after the restore
		const bool over = btot * 10 > (uint64_t) ns * 9;
		if (over && tid == 0)
			atomicOr(dupflag, 2u);
		bool dup = false;
#if !(PJ2_DIAG & 1)
		if (!over) {
			for (uint32_t sb0 = w * 64; sb0 < nsubB; sb0 += 16 * 64) {
				Pj2Batch bb;
				pj2_issue2(bkey, q0, q1, nsubB, sb0, slot, 0, bb, true);
				for (uint32_t i0 = 0;;) {
					uint32_t rw[PJ2_U];
#pragma unroll
					for (int u = 0; u < PJ2_U; u++)
						rw[u] = bb.idx[u] != ~0u ? brow[bb.idx[u]] : 0u;
#pragma unroll
					for (int u = 0; u < PJ2_U; u++) {
						if (bb.idx[u] == ~0u)
							continue;
						const uint32_t row = (bb.idx[u] & ~(uint32_t) (PJ_SUBROWS - 1)) + rw[u];
						const unsigned long long v = ((unsigned long long) (row + 1) << 32) | bb.key[u];
						uint32_t h = 2 * gt_home(pj_hash(bb.key[u]), pbits, nbp);
						for (;;) {
							const unsigned long long o = atomicCAS(&tab[h], 0ull, v);
							if (o == 0ull)
								break;
							if ((uint32_t) o == bb.key[u]) {
								dup = true;
								break;
							}
							h = h + 1 == ns ? 0 : h + 1;
						}
					}
					i0 += 64 * PJ2_U;
					if (i0 >= bb.tot)
						break;
					pj2_issue2(bkey, q0, q1, nsubB, sb0, slot, i0, bb, false);
				}
			}
		}
#endif
		if (__any(dup) && lane == 0)
			atomicOr(dupflag, 1u);
	}
	// the probe side's first batch, then the table complete
	if (s0 < nsub)
		pj2_issue2(pkey, o0, o1, nsub, s0, slot, 0, bt, true);
	__syncthreads();
#else
	// the first batch's run bounds and key loads go out before the table is
	// built, so their latency hides behind the build
	Pj2Batch bt;
	uint32_t s0 = w * 64;
	if (s0 < nsub) {
#if PJ2_SRCH
		pj2_issue2(pkey, o0, o1, nsub, s0, slot, 0, bt, true);
#else
		pj2_issue(pkey, o0, o1, nsub, s0, ws, wb, 0, bt, true);
#endif
	}
#if PJ2_TB
	(void) bent;
	(void) bbase;
	(void) dupflag;
	__syncthreads();                              // the table is loaded
#else
	// a build partition above 90 % of the table (the host sized it for the
	// expected largest one) is flagged and not built: its runs are answered
	// "no match" and the host falls back after the restore
	// (64-bit: a partition of more than ~429M entries must not wrap past the test)
	const uint32_t b0 = bbase[p], over = (uint64_t) (bbase[p + 1] - b0) * 10 > (uint64_t) ns * 9;
#if PJ2_DIAG & 1
	const uint32_t b1 = b0;          // timing diagnostic: no table (every answer "no match")
#else
	const uint32_t b1 = over ? b0 : bbase[p + 1];
#endif
	if (over && tid == 0)
		atomicOr(dupflag, 2u);
	bool dup = false;
	uint2 en[PJ2_BU];
	uint32_t e0 = b0 + tid;
#pragma unroll
	for (int u = 0; u < PJ2_BU; u++) {
		const uint32_t e = e0 + u * blockDim.x;
		en[u] = e < b1 ? bent[e] : make_uint2(0, 0);
	}
	__syncthreads();                              // the table is zeroed
	while (e0 < b1) {
#pragma unroll
		for (int u = 0; u < PJ2_BU; u++) {
			if (e0 + u * blockDim.x >= b1)
				continue;
			const unsigned long long v = ((unsigned long long) (en[u].y + 1) << 32) | en[u].x;
			uint32_t h = 2 * gt_home(pj_hash(en[u].x), pbits, nbp);
			for (;;) {
				const unsigned long long o = atomicCAS(&tab[h], 0ull, v);
				if (o == 0ull)
					break;
				if ((uint32_t) o == en[u].x) {
					dup = true;
					break;
				}
				h = h + 1 == ns ? 0 : h + 1;
			}
		}
		e0 += PJ2_BU * blockDim.x;
#pragma unroll
		for (int u = 0; u < PJ2_BU; u++) {
			const uint32_t e = e0 + u * blockDim.x;
			en[u] = e < b1 ? bent[e] : make_uint2(0, 0);
		}
	}
	if (__any(dup) && lane == 0)
		atomicOr(dupflag, 1u);
	__syncthreads();
#endif
#endif
	const ulonglong2 *bk = (const ulonglong2 *) tab;     // (an empty table when over)
	// software pipeline: the next chunk's key loads (and, at a batch
	// boundary, the next batch's run bounds) are issued before the current
	// chunk is answered
	uint32_t ci0 = 0;
	while (s0 < nsub) {
		uint32_t ns0 = s0, ni0 = ci0 + 64 * PJ2_U;
		if (ni0 >= bt.tot) {
			ns0 = s0 + 16 * 64;
			ni0 = 0;
		}
		Pj2Batch nx;
		nx.tot = bt.tot;
		nx.rs = bt.rs;
		nx.rl = bt.rl;
		nx.rb = bt.rb;
		if (ns0 < nsub) {
#if PJ2_SRCH
			pj2_issue2(pkey, o0, o1, nsub, ns0, slot, ni0, nx, ni0 == 0);
#else
			pj2_issue(pkey, o0, o1, nsub, ns0, ws, wb, ni0, nx, ni0 == 0);
#endif
		}
		pj2_answer(bk, pbits, nbp, bt, pans);
		bt = nx;
		s0 = ns0;
		ci0 = ni0;
	}
}

__global__ __launch_bounds__(1024) void
k_pj2_restore(const uint16_t *prow, const uint32_t *pans, const uint16_t *poff, uint32_t P, BUN n, uint32_t nsub,
	      Side L, Side R, uint32_t *ticket, uint64_t *status, uint64_t *meta, oid *r1, oid *r2)
{
	__shared__ uint32_t res[PJ_SUBROWS + PJ_SUBROWS / 32];
	__shared__ uint32_t s_sub;
	const unsigned tid = threadIdx.x;
	if (tid == 0)
		s_sub = atomicAdd(ticket, 1u);
	for (uint32_t i = tid; i < PJ_SUBROWS + PJ_SUBROWS / 32; i += blockDim.x)
		res[i] = 0;
	__syncthreads();
	const uint32_t sub = s_sub;
	const BUN a = (BUN) sub * PJ_SUBROWS;
	const uint32_t rows = (uint32_t) min((BUN) PJ_SUBROWS, n - a);
	const uint32_t cnt = poff[(size_t) sub * (P + 1) + P];
#if PJ2_RALL
	// every entry of the subtile loaded at once (the region holds PJ_SUBROWS
	// entries, so whole 16-B pieces past cnt stay inside it): thread tid
	// takes entries 4 (tid + 1024 q) .. + 3, q < 8 -- one latency instead of
	// four dependent rounds
	static_assert(PJ_SUBROWS == 32 * 1024, "32 entries per thread");
	typedef uint32_t u4 __attribute__((ext_vector_type(4)));
	typedef uint32_t u2 __attribute__((ext_vector_type(2)));
	u4 am[8];
	u2 ar[8];
#pragma unroll
	for (int q = 0; q < 8; q++) {
		const uint32_t j = 4 * (tid + 1024 * q);
		am[q] = j < cnt ? __builtin_nontemporal_load((const u4 *) (pans + a + j)) : (u4) {0, 0, 0, 0};
		ar[q] = j < cnt ? __builtin_nontemporal_load((const u2 *) (prow + a + j)) : (u2) {0, 0};
	}
#pragma unroll
	for (int q = 0; q < 8; q++) {
		const uint32_t j = 4 * (tid + 1024 * q);
#pragma unroll
		for (int c = 0; c < 4; c++) {
			const uint32_t m = am[q][c], r = (ar[q][c >> 1] >> (16 * (c & 1))) & 0xffffu;
			if (j + c < cnt && m)
				res[r + (r >> 5)] = m;
		}
	}
#else
	constexpr int U = 8;
	for (uint32_t j0 = tid; j0 < cnt; j0 += U * blockDim.x) {
		uint32_t m[U], r[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t j = j0 + u * blockDim.x;
#if PJ2_NT
			m[u] = j < cnt ? __builtin_nontemporal_load(pans + a + j) : 0u;
			r[u] = j < cnt ? __builtin_nontemporal_load(prow + a + j) : 0u;
#else
			m[u] = j < cnt ? pans[a + j] : 0u;
			r[u] = j < cnt ? prow[a + j] : 0u;
#endif
		}
#pragma unroll
		for (int u = 0; u < U; u++)
			if (m[u])
				res[r[u] + (r[u] >> 5)] = m[u];
	}
#endif
	__syncthreads();
	pj_emit(res, sub, a, rows, nsub, L, R, status, meta, r1, r2);
}

// restore in 75 KB of LDS (PJ2_R2=1): two workgroups per CU, so one's LDS
// and scan phases overlap the other's pair stores.  The answers stay in
// registers (32 entries per thread, as PJ2_RALL loads them); the matched rows
// become a 32K-bit mask by LDS atomics, which the emit's scan reads as its
// run masks; then for each half of the subtile the entries of that half drop
// their answers into a 16K-row stage and the half's pairs are stored in row
// order.
#ifndef PJ2_R2
#define PJ2_R2 0        // measured slower (profiles/r06/join_r2): 1 (answers kept in registers, 28 VGPRs
                        // spilled) 0.945-0.971 ms, 2 (the second half's entries read again) 0.881, 0: 0.851-0.853
#endif
#if PJ2_R2
constexpr uint32_t PJ2_R2H = PJ_SUBROWS / 2;       // rows per stage half

__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void
k_pj2_restore2(const uint16_t *prow, const uint32_t *pans, const uint16_t *poff, uint32_t P, BUN n, uint32_t nsub,
	       Side L, Side R, uint32_t *ticket, uint64_t *status, uint64_t *meta, oid *r1, oid *r2)
{
	__shared__ uint32_t stage[PJ2_R2H + PJ2_R2H / 32];
	__shared__ uint32_t rbase[1024], wsum[16];
	__shared__ uint32_t rmask[1024];
	__shared__ uint64_t s_pre;
	__shared__ uint32_t s_sub;
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	if (tid == 0)
		s_sub = atomicAdd(ticket, 1u);
	rmask[tid] = 0;
	__syncthreads();
	const uint32_t sub = s_sub;
	const BUN a = (BUN) sub * PJ_SUBROWS;
	const uint32_t rows = (uint32_t) min((BUN) PJ_SUBROWS, n - a);
	const uint32_t cnt = poff[(size_t) sub * (P + 1) + P];
	static_assert(PJ_SUBROWS == 32 * 1024, "32 entries per thread");
	typedef uint32_t u4 __attribute__((ext_vector_type(4)));
	typedef uint32_t u2 __attribute__((ext_vector_type(2)));
	u4 am[8];
	u2 ar[8];
#pragma unroll
	for (int q = 0; q < 8; q++) {
		const uint32_t j = 4 * (tid + 1024 * q);
#if PJ2_R2 == 2
		am[q] = j < cnt ? *(const u4 *) (pans + a + j) : (u4) {0, 0, 0, 0};     // read again below: cached
		ar[q] = j < cnt ? *(const u2 *) (prow + a + j) : (u2) {0, 0};
#else
		am[q] = j < cnt ? __builtin_nontemporal_load((const u4 *) (pans + a + j)) : (u4) {0, 0, 0, 0};
		ar[q] = j < cnt ? __builtin_nontemporal_load((const u2 *) (prow + a + j)) : (u2) {0, 0};
#endif
	}
	// the matched rows' bits, and the first half's answers into the stage
#pragma unroll
	for (int q = 0; q < 8; q++) {
		const uint32_t j = 4 * (tid + 1024 * q);
#pragma unroll
		for (int c = 0; c < 4; c++) {
			const uint32_t m = am[q][c], r = (ar[q][c >> 1] >> (16 * (c & 1))) & 0xffffu;
			if (j + c < cnt && m) {
				atomicOr(&rmask[r >> 5], 1u << (r & 31));
#if PJ2_R2 == 2
				if (r < PJ2_R2H)
					stage[r + (r >> 5)] = m;
#endif
			}
		}
	}
	__syncthreads();
	// thread tid's 32 rows [32 tid, 32 tid + 32): count, wave and workgroup
	// scans, the subtile's offset by look-back (as pj_emit_scan)
	const uint32_t r0 = tid * 32;
	const uint32_t msk = r0 >= rows ? 0u : rows - r0 >= 32 ? rmask[tid] : rmask[tid] & ((1u << (rows - r0)) - 1);
	const uint32_t c = __popc(msk);
	uint32_t x = c;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t u = __shfl_up(x, o);
		if (lane >= (unsigned) o)
			x += u;
	}
	if (lane == 63)
		wsum[w] = x;
	__syncthreads();
	uint32_t wpre = 0, tot = 0;
	for (uint32_t q = 0; q < 16; q++) {
		wpre += q < w ? wsum[q] : 0;
		tot += wsum[q];
	}
	rmask[tid] = msk;
	rbase[tid] = wpre + x - c;
	if (w == 0) {
		const uint64_t pre = lookback(status, sub, tot, (uint32_t *) &meta[1]);
		if (lane == 0) {
			s_pre = pre;
			if (sub == nsub - 1)
				meta[0] = pre + tot;
		}
	}
	__syncthreads();
	const uint64_t pre = s_pre;
	for (uint32_t h = 0; h < 2; h++) {
		const uint32_t hb = h * PJ2_R2H;
		if (hb >= rows)
			break;
#if PJ2_R2 == 2
		// the second half's answers: the subtile's entries read again (the
		// first read's registers are not kept through the scan and stores)
		if (h == 1) {
#pragma unroll
			for (int q = 0; q < 8; q++) {
				const uint32_t j = 4 * (tid + 1024 * q);
				am[q] = j < cnt ? *(const u4 *) (pans + a + j) : (u4) {0, 0, 0, 0};
				ar[q] = j < cnt ? *(const u2 *) (prow + a + j) : (u2) {0, 0};
			}
		}
		if (h == 1)
#endif
#pragma unroll
		for (int q = 0; q < 8; q++) {
			const uint32_t j = 4 * (tid + 1024 * q);
#pragma unroll
			for (int c2 = 0; c2 < 4; c2++) {
				const uint32_t m = am[q][c2], r = (ar[q][c2 >> 1] >> (16 * (c2 & 1))) & 0xffffu;
				if (j + c2 < cnt && m && r - hb < PJ2_R2H) {
					const uint32_t rl = r - hb;
					stage[rl + (rl >> 5)] = m;
				}
			}
		}
		__syncthreads();
		const uint32_t he = min(hb + PJ2_R2H, rows);
		for (uint32_t r = hb + tid; r < he; r += blockDim.x) {
			const uint32_t run = r >> 5, bit = r & 31;
			const uint32_t mk = rmask[run];
			if ((mk >> bit) & 1) {
				const uint64_t o = pre + rbase[run] + __popc(mk & ((1u << bit) - 1));
				const uint32_t rl = r - hb;
				r1[o] = oid_of(L, a + r);
				r2[o] = oid_of(R, stage[rl + (rl >> 5)] - 1);
			}
		}
		__syncthreads();
	}
}

#endif

// persistent restore (PJ2_RP=1): one 1024-thread workgroup per CU (the
// 143 KB of LDS allow no second) claims subtiles by ticket and loads the
// next subtile's answers and rows while it writes the current one's pairs,
// so a CU's reads and writes overlap instead of alternating.  The loads take
// the whole 32K-entry region (in bounds: the region holds PJ_SUBROWS entries)
// and the scatter masks entries past the subtile's count.  Claims in ticket
// order keep the look-back deadlock-free: the lowest unpublished subtile's
// owner waits on nothing unpublished.
#ifndef PJ2_RP
#define PJ2_RP 0
#endif

#if PJ2_RP
typedef uint32_t pj_u4 __attribute__((ext_vector_type(4)));
typedef uint32_t pj_u2 __attribute__((ext_vector_type(2)));
struct Pj2Ent {
	pj_u4 am[8];
	pj_u2 ar[8];
	uint32_t cnt;
};

__device__ __forceinline__ void
pj2_rload(const uint16_t *prow, const uint32_t *pans, const uint16_t *poff, uint32_t P, uint32_t sub, Pj2Ent &x)
{
	const BUN a = (BUN) sub * PJ_SUBROWS;
	x.cnt = poff[(size_t) sub * (P + 1) + P];
#pragma unroll
	for (int q = 0; q < 8; q++) {
		const uint32_t j = 4 * (threadIdx.x + 1024 * q);
		x.am[q] = __builtin_nontemporal_load((const pj_u4 *) (pans + a + j));
		x.ar[q] = __builtin_nontemporal_load((const pj_u2 *) (prow + a + j));
	}
}

__device__ __forceinline__ void
pj2_rscatter(const Pj2Ent &x, uint32_t *res)
{
#pragma unroll
	for (int q = 0; q < 8; q++) {
		const uint32_t j = 4 * (threadIdx.x + 1024 * q);
#pragma unroll
		for (int c = 0; c < 4; c++) {
			const uint32_t m = x.am[q][c], r = (x.ar[q][c >> 1] >> (16 * (c & 1))) & 0xffffu;
			if (j + c < x.cnt && m)
				res[r + (r >> 5)] = m;
		}
	}
}

__global__ __launch_bounds__(1024) void
k_pj2_restore_p(const uint16_t *prow, const uint32_t *pans, const uint16_t *poff, uint32_t P, BUN n, uint32_t nsub,
		Side L, Side R, uint32_t *ticket, uint64_t *status, uint64_t *meta, oid *r1, oid *r2)
{
	__shared__ uint32_t res[PJ_SUBROWS + PJ_SUBROWS / 32];
	__shared__ EmitLds e;
	__shared__ uint32_t s_sub;
	const unsigned tid = threadIdx.x;
	if (tid == 0)
		s_sub = atomicAdd(ticket, 1u);
	for (uint32_t i = tid; i < PJ_SUBROWS + PJ_SUBROWS / 32; i += blockDim.x)
		res[i] = 0;
	__syncthreads();
	uint32_t sub = s_sub;
	Pj2Ent x;
	if (sub < nsub)
		pj2_rload(prow, pans, poff, P, sub, x);
	while (sub < nsub) {
		uint32_t nxt = 0;
		if (tid == 0)
			nxt = atomicAdd(ticket, 1u);
		pj2_rscatter(x, res);
		if (tid == 0)
			s_sub = nxt;        // every read of the previous value is behind two barriers
		__syncthreads();
		const BUN a = (BUN) sub * PJ_SUBROWS;
		const uint32_t rows = (uint32_t) min((BUN) PJ_SUBROWS, n - a);
		pj_emit_scan(res, sub, rows, nsub, status, meta, e);
		const uint32_t ns = s_sub;
		if (ns < nsub)
			pj2_rload(prow, pans, poff, P, ns, x);      // in flight during the writes
		pj_emit_write(res, a, rows, L, R, e, r1, r2);
		__syncthreads();
		for (uint32_t i = tid; i < PJ_SUBROWS + PJ_SUBROWS / 32; i += blockDim.x)
			res[i] = 0;
		__syncthreads();
		sub = ns;
	}
}
#endif

// one side cut into partitions: cnt/off matrices, partition bases, entries
struct PjSide {
	uint32_t nsub = 0;
	DevBuf *cnt = nullptr, *off = nullptr, *tot = nullptr, *base = nullptr, *ent = nullptr;
	~PjSide()
	{
		delete cnt;
		delete off;
		delete tot;
		delete base;
		delete ent;
	}
};

int
pj_cut(const Side &S, BUN n, int pbits, bool skipnil, PjSide &o, uint32_t *maxtot_dev, hipStream_t st = nullptr)
{
	if (st == nullptr)
		st = stream();
	const uint32_t P = 1u << pbits;
	o.nsub = (uint32_t) ((n + PJ_SUBROWS - 1) / PJ_SUBROWS);
	const size_t m = (size_t) o.nsub * P * 4 + 64;
	o.cnt = new DevBuf(m);
	o.off = new DevBuf(m);
	o.tot = new DevBuf(P * 4 + 64);
	o.base = new DevBuf(P * 4 + 64);
	o.ent = new DevBuf(n * 8 + 64);
	if (!o.cnt->p || !o.off->p || !o.tot->p || !o.base->p || !o.ent->p)
		return -1;
	const unsigned grid = (o.nsub + PJ_SUBS - 1) / PJ_SUBS;
	hipLaunchKernelGGL(k_pj_hist, dim3(grid), dim3(1024), 0, st, S, n, pbits, skipnil, o.cnt->as<uint32_t>());
	hipLaunchKernelGGL(k_pj_colscan, dim3(P / 64), dim3(1024), 0, st, o.cnt->as<uint32_t>(), o.nsub, P,
			   o.off->as<uint32_t>(), o.tot->as<uint32_t>());
	hipLaunchKernelGGL(k_pj_base, dim3(1), dim3(1024), 0, st, o.tot->as<uint32_t>(), P, o.base->as<uint32_t>(),
			   maxtot_dev);
	hipLaunchKernelGGL(k_pj_scatter, dim3(o.nsub), dim3(1024), 0, st, S, n, pbits, skipnil, o.off->as<uint32_t>(),
			   o.base->as<uint32_t>(), o.ent->as<uint2>());
	return 0;
}

// the join's 48 bytes of meta words and the first and last oid of both
// result columns, stored straight into the thread's pinned host buffer (no
// copy launch)
__global__ void
k_pj_ends(const uint32_t *meta32, const oid *r1, const oid *r2, uint32_t *h)
{
	if (threadIdx.x < 12)
		h[threadIdx.x] = meta32[threadIdx.x];
	if (threadIdx.x == 0) {
		const uint64_t n = ((const uint64_t *) meta32)[4];
		uint64_t *e = (uint64_t *) (h + 12);
		if (n > 0) {
			e[0] = r1[0];
			e[1] = r1[n - 1];
			e[2] = r2[0];
			e[3] = r2[n - 1];
		}
	}
}

// the probe side of join_part with subtile-local runs (k_pj2_*).  The probe
// side's cut is the longer chain (cut, transpose, probe, restore), so it is
// queued first; the build side (Rn, its largest partition in meta32[0], its
// nofit flag in meta32[5], read back after the restore) is cut after it, on
// the side stream (PJ2_SIDE, PJ2_SWAP) forked from the main one before either
int
join_part2(const Side &L, BUN nl, const Side &Rn, BUN nr, int pbits, bool nil_matches, mgdk_bat **ap, mgdk_bat **bp,
	   bool *ukey)
{
	PjSide B;
	hipStream_t st = stream();
	const uint32_t P = 1u << pbits;
	uint32_t *meta32 = (uint32_t *) meta_buf();
	uint64_t *meta = (uint64_t *) meta32 + 4;          // [0] pairs, [1] look-back error
	uint32_t *h = (uint32_t *) pinned(128);
	const uint32_t nsub = (uint32_t) ((nl + PJ_SUBROWS - 1) / PJ_SUBROWS);
	const size_t rsz = (size_t) nsub * PJ_SUBROWS;
	if (nl == 0 || rsz >= ((size_t) 1 << 32))
		return 1;                                   // (entry indexes are 32-bit)
	DevBuf pkey(rsz * 4 + 64), prow(rsz * 2 + 64), pans(rsz * 4 + 64), poff((size_t) nsub * (P + 1) * 2 + 64),
		poffT((size_t) nsub * (P + 1) * 2 + 64);
	if (!pkey.p || !prow.p || !pans.p || !poff.p || !poffT.p)
		return sync_fail();
	const uint32_t nsubB = (uint32_t) ((nr + PJ_SUBROWS - 1) / PJ_SUBROWS);
	const size_t bsz = (size_t) nsubB * PJ_SUBROWS;
	if (bsz >= ((size_t) 1 << 32) - PJ_SUBROWS)
		return 1;                                   // (build rows + 1 are 32-bit)
#if PJ2_BC
	DevBuf bkey(bsz * 4 + 64), brow(bsz * 2 + 64), bpoff((size_t) nsubB * (P + 1) * 2 + 64),
		bpoffT((size_t) nsubB * (P + 1) * 2 + 64);
	if (!bkey.p || !brow.p || !bpoff.p || !bpoffT.p)
		return sync_fail();
#endif
	static const bool cut_attr = hipFuncSetAttribute((const void *) k_pj2_cut,
							 hipFuncAttributeMaxDynamicSharedMemorySize, (int) PJ2_CUT_LDS) == hipSuccess;
	static const bool probe_attr = hipFuncSetAttribute((const void *) k_pj2_probe,
							   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
	(void) hipGetLastError();
	if (!cut_attr || !probe_attr)
		return 1;                                   // the kernels cannot get their LDS: fallback
	// the table is sized for the expected largest build partition (mean + 6
	// sigma) instead of the measured one, so no round trip is needed between
	// the passes: a larger partition, a duplicate build key or a build value
	// without a 4-byte image is flagged on the device, read back once after
	// the restore, and sends the join to the fallback
	const double mean = (double) nr / P;
	const uint32_t est = (uint32_t) (mean + 6.0 * sqrt(mean)) + 1;
	if (est > PJ2_MAXFILL)
		return 1;
	static const int lfpct = getenv("MGDK_PJ_LF") ? atoi(getenv("MGDK_PJ_LF")) : 80;
	uint32_t nbp = (uint32_t) ((uint64_t) est * 100 / (2 * (uint64_t) (lfpct < 40 ? 40 : lfpct > 95 ? 95 : lfpct))) + 1;
	if (2 * nbp <= est)
		nbp = est / 2 + 1;
	nbp = nbp < PJ2_MAXB ? nbp : PJ2_MAXB;             // (est <= PJ2_MAXFILL keeps load <= 4/5)
	// two workgroups per CU when the table fits 80 KiB at <= 90 % load
	constexpr uint32_t NBP2 = (80 * 1024 - 16 * 64 * 8) / 16;
	static const bool occ2 = !getenv("MGDK_PJ2_OCC") || atoi(getenv("MGDK_PJ2_OCC")) != 0;
	if (occ2 && nbp > NBP2 && (uint64_t) est * 10 <= (uint64_t) 2 * NBP2 * 9)
		nbp = NBP2;
	const size_t lds = (size_t) nbp * 16 + 16 * 64 * 8;
#if PJ2_TB
	// the build side's tables, built on st beside the probe side's cut
	static const bool tb_attr = hipFuncSetAttribute((const void *) k_pj2_tbuild,
							hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
	(void) hipGetLastError();
	DevBuf gtab((size_t) P * 2 * nbp * 8 + 64);
	if (!tb_attr || !gtab.p)
		return tb_attr ? -1 : 1;
	const unsigned long long *gtp = gtab.as<unsigned long long>();
#else
	const unsigned long long *gtp = nullptr;
#endif
	// the two sides' cuts depend on nothing the other writes: one runs on the
	// side stream, beside the other, whose few workgroups leave CUs idle
	// (PJ2_SIDE=0: one stream; PJ2_SWAP: the build side is the one on the
	// side stream).  The side stream first waits for what is queued on the
	// main one (the inputs' producers, the meta words' memset).
	hipStream_t cs = st, bs = st;
#if PJ2_SIDE
	if (stream2() != nullptr) {
		if (!side_fork())
			return sync_fail();
#if PJ2_SWAP
		bs = stream2();
#else
		cs = stream2();
#endif
	}
#endif
	// the restore's ticket and look-back words (cleared by the cut)
	const size_t sbytes = (nsub + 8) * sizeof(uint64_t);
	char *sc = (char *) scratch(sbytes);
	if (!sc)
		return sync_fail();
	hipLaunchKernelGGL(k_pj2_cut, dim3(nsub), dim3(1024), PJ2_CUT_LDS, cs, L, nl, pbits, !nil_matches,
			   pkey.as<uint32_t>(), prow.as<uint16_t>(), poff.as<uint16_t>(), (uint64_t *) sc);
	hipLaunchKernelGGL(k_pj2_offt, dim3((nsub + 63) / 64, (P + 1 + 63) / 64), dim3(256), 0, cs, poff.as<uint16_t>(),
			   nsub, P, poffT.as<uint16_t>());
#if PJ2_BC
	// the build side cut into subtile-local runs the same way (the cut leaves
	// the restore's words alone: rzero NULL)
	if (!hip_ok(hipMemsetAsync(meta32, 0, 64, bs), "memset"))
		return sync_fail();
	hipLaunchKernelGGL(k_pj2_cut, dim3(nsubB), dim3(1024), PJ2_CUT_LDS, bs, Rn, nr, pbits, !nil_matches,
			   bkey.as<uint32_t>(), brow.as<uint16_t>(), bpoff.as<uint16_t>(), (uint64_t *) nullptr);
	hipLaunchKernelGGL(k_pj2_offt, dim3((nsubB + 63) / 64, (P + 1 + 63) / 64), dim3(256), 0, bs,
			   bpoff.as<uint16_t>(), nsubB, P, bpoffT.as<uint16_t>());
	if (!hip_ok(hipGetLastError(), "join build cut"))
		return sync_fail();
	const uint2 *bentp = nullptr;
	const uint32_t *bbasep = nullptr;
	const uint32_t *bkeyp = bkey.as<uint32_t>();
	const uint16_t *browp = brow.as<uint16_t>(), *bpoffTp = bpoffT.as<uint16_t>();
#else
	const uint32_t *bkeyp = nullptr;
	const uint16_t *browp = nullptr, *bpoffTp = nullptr;
	// the meta words: the build side's (largest partition, nofit) and the
	// probe's / restore's flags and counts, which run after the side join
	if (!hip_ok(hipMemsetAsync(meta32, 0, 64, bs), "memset") ||
	    pj_cut(Rn, nr, pbits, !nil_matches, B, &meta32[0], bs) < 0)
		return sync_fail();
	const uint2 *bentp = B.ent->as<uint2>();
	const uint32_t *bbasep = B.base->as<uint32_t>();
#endif
#if PJ2_TB
	if (!side_join())
		return sync_fail();
	hipLaunchKernelGGL(k_pj2_tbuild, dim3(P), dim3(1024), (size_t) nbp * 16, st, B.ent->as<uint2>(),
			   B.base->as<uint32_t>(), pbits, nbp, gtab.as<unsigned long long>(), &meta32[2]);
#endif
#if PJ2_SIDE
	if (stream2() != nullptr && !side_join())
		return sync_fail();
#endif
	hipLaunchKernelGGL(k_pj2_probe, dim3(P), dim3(1024), lds, st, bentp, bbasep, pkey.as<uint32_t>(),
			   poffT.as<uint16_t>(), pbits, nbp, nsub, pans.as<uint32_t>(), &meta32[2], gtp,
			   bkeyp, browp, bpoffTp, nsubB);
	mgdk_bat *ra = newbat(0, MGDK_oid, nl), *rb = newbat(0, MGDK_oid, nl);
	if (!ra || !rb) {
		unfix2(ra, rb);
		return sync_fail();
	}
#if PJ2_R2
	hipLaunchKernelGGL(k_pj2_restore2, dim3(nsub), dim3(1024), 0, st, prow.as<uint16_t>(), pans.as<uint32_t>(),
			   poff.as<uint16_t>(), P, nl, nsub, L, Rn, (uint32_t *) sc, (uint64_t *) sc + 8, meta,
			   (oid *) ra->theap, (oid *) rb->theap);
#elif PJ2_RP
	static const unsigned ncu = [] {
		int v = 0, d = 0;
		if (hipGetDevice(&d) != hipSuccess ||
		    hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || v <= 0)
			v = 256;
		(void) hipGetLastError();
		return (unsigned) v;
	}();
	hipLaunchKernelGGL(k_pj2_restore_p, dim3(min(ncu, nsub)), dim3(1024), 0, st, prow.as<uint16_t>(),
			   pans.as<uint32_t>(), poff.as<uint16_t>(), P, nl, nsub, L, Rn, (uint32_t *) sc, (uint64_t *) sc + 8,
			   meta, (oid *) ra->theap, (oid *) rb->theap);
#else
	hipLaunchKernelGGL(k_pj2_restore, dim3(nsub), dim3(1024), 0, st, prow.as<uint16_t>(), pans.as<uint32_t>(),
			   poff.as<uint16_t>(), P, nl, nsub, L, Rn, (uint32_t *) sc, (uint64_t *) sc + 8, meta,
			   (oid *) ra->theap, (oid *) rb->theap);
#endif
	// a failed launch leaves pkey / pans / the results unwritten: fail the call
	if (!hip_ok(hipGetLastError(), "join probe launch")) {
		unfix2(ra, rb);
		return sync_fail();
	}
	// meta32[2]: duplicate build key (1) / oversized partition (2);
	// meta32[5]: build value without a 4-byte image; meta = meta32 + 8:
	// pairs, look-back error, then the results' first / last oids
	hipLaunchKernelGGL(k_pj_ends, dim3(1), dim3(64), 0, st, (const uint32_t *) meta32, (const oid *) ra->theap,
			   (const oid *) rb->theap, h);
	if (!hip_ok(hipGetLastError(), "k_pj_ends") || !sync()) {
		unfix2(ra, rb);
		return -1;
	}
	uint64_t h64[2];
	memcpy(h64, h + 8, 16);
	if (h[2] || h[5]) {
		unfix2(ra, rb);
		return 1;
	}
	if (h64[1] & 1) {
		seterr("HY013!BATjoin: look-back did not complete");
		unfix2(ra, rb);
		return -1;
	}
	ra->count = rb->count = h64[0];
	if (h64[0] > 0) {
		uint64_t e[4];
		memcpy(e, h + 12, 32);
		join_ends = JoinEnds{ra, rb, e[0], e[1], e[2], e[3]};
	}
	*ukey = true;                                       // unique build keys: one match per row
	*ap = ra;
	*bp = rb;
	return 0;
}

// returns 1 when not applicable (caller uses the open-addressing path)
int
join_part(const Side &L, BUN nl, const Side &R, BUN nr, bool nil_matches, mgdk_bat **ap, mgdk_bat **bp, bool *ukey)
{
	const int mode = getenv("MGDK_JOIN_PART") ? atoi(getenv("MGDK_JOIN_PART")) : 1;   // per call (tests)
	const bool w4 = L.w == 4 && R.w == 4, w8 = L.w == 8 && R.w == 8 && L.base && R.base;
	if (mode == 0 || !(w4 || w8) || nr < 65536)
		return 1;
	int pbits = 6;
	while (pbits < PJ_MAXPBITS && ((BUN) 8192 << pbits) < nr)
		pbits++;
	// the expected largest partition (mean + 6 sigma) must fit the LDS table
	while (pbits < PJ_MAXPBITS && (double) nr / (1u << pbits) + 6.0 * sqrt((double) nr / (1u << pbits)) > PJ_MAXFILL)
		pbits++;
	if ((double) nr / (1u << pbits) + 6.0 * sqrt((double) nr / (1u << pbits)) > PJ_MAXFILL)
		return 1;
	// the subtile-local probe side (mode != 3) can take partitions up to
	// PJ2_MAXFILL: MGDK_PJ2_PB = partition bits below the default
	// (halving the partitions doubles the probe's runs)
	const int pbd = mode != 3 && getenv("MGDK_PJ2_PB") ? atoi(getenv("MGDK_PJ2_PB")) : 0;
	for (int k = 0; k < pbd && pbits > 6; k++) {
		const double m = (double) nr / (1u << (pbits - 1));
		if (m + 6.0 * sqrt(m) > PJ2_MAXFILL)
			break;
		pbits--;
	}
	const uint32_t P = 1u << pbits;
	hipStream_t st = stream();
	uint32_t *meta32 = (uint32_t *) meta_buf();
	uint64_t *meta = (uint64_t *) meta32 + 4;          // [0] pairs, [1] look-back error
	uint32_t *h = (uint32_t *) pinned(64);
	// the subtile-local plan (mode != 3) clears the meta words itself, on
	// the stream of the build side's cut, after the probe side's cut is queued
	if (mode == 3 && !hip_ok(hipMemsetAsync(meta32, 0, 64, st), "memset"))
		return -1;
	// both sides are cut before the host looks at the build side's largest
	// partition: one round trip instead of two (an oversized partition, rare,
	// wastes the probe side's cut)
	PjSide B, Pr;
	Side Rn = R;
	Rn.nofit = &meta32[5];
	if (mode != 3)
		return join_part2(L, nl, Rn, nr, pbits, nil_matches, ap, bp, ukey);
	if (pj_cut(Rn, nr, pbits, !nil_matches, B, &meta32[0]) < 0) {
		(void) sync();                              // launched cuts still use the buffers
		return -1;
	}
	if (pj_cut(L, nl, pbits, !nil_matches, Pr, &meta32[1]) < 0) {
		(void) sync();
		return -1;
	}
	if (!hip_ok(hipMemcpyAsync(h, meta32, 32, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	if (h[0] > PJ_MAXFILL || h[5])
		return 1;                                   // oversized partition / build value without a 4-byte image
	// subtile-major offsets of the probe results
	DevBuf offT((size_t) Pr.nsub * P * 4 + 64);
	uint64_t total = 0;
	if (!offT.p ||
	    exclusive_scan(Pr.cnt->as<uint32_t>(), offT.as<uint32_t>(), (BUN) Pr.nsub * P, &total) < 0)
		return sync_fail();
	DevBuf deltaT((size_t) Pr.nsub * P * 4 + 64), flat((size_t) nl * 8 + 64);
	if (!deltaT.p || !flat.p)
		return sync_fail();
	hipLaunchKernelGGL(k_pj_delta, dim3((Pr.nsub + 63) / 64, (P + 63) / 64), dim3(256), 0, st, offT.as<uint32_t>(),
			   Pr.off->as<uint32_t>(), Pr.base->as<uint32_t>(), Pr.nsub, P, deltaT.as<uint32_t>());
	// table: ~80 % load on the largest build partition (an empty slot always
	// remains); LDS = table + the probe's offsets column when it fits
	static const int lfpct = getenv("MGDK_PJ_LF") ? atoi(getenv("MGDK_PJ_LF")) : 80;
	uint32_t nbp = (uint32_t) ((uint64_t) h[0] * 100 / (2 * (uint64_t) (lfpct < 40 ? 40 : lfpct > 95 ? 95 : lfpct))) + 1;
	if (2 * nbp <= h[0])
		nbp = h[0] / 2 + 1;
	nbp = nbp < PJ_SLOTS / 2 ? nbp : PJ_SLOTS / 2;    // (h[0] <= PJ_MAXFILL keeps load < 3/4)
	const bool ldsd = Pr.nsub <= PJ_LDS_SUBS && (size_t) nbp * 16 + (size_t) Pr.nsub * 4 <= 160 * 1024;
	const size_t lds = (size_t) nbp * 16 + (ldsd ? (size_t) Pr.nsub * 4 : 0);
	static const bool lds_attr = hipFuncSetAttribute((const void *) k_pj_probe,
							 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
	(void) lds_attr;
	(void) hipGetLastError();
	hipLaunchKernelGGL(k_pj_probe, dim3(P), dim3(1024), lds, st, B.ent->as<uint2>(), B.base->as<uint32_t>(),
			   Pr.ent->as<uint2>(), Pr.base->as<uint32_t>(), pbits, nbp, deltaT.as<uint32_t>(), Pr.nsub,
			   ldsd, flat.as<uint2>(), &meta32[2]);
	if (!hip_ok(hipMemcpyAsync(h, meta32, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	if (h[2])
		return 1;                                   // duplicate build keys
	mgdk_bat *ra = newbat(0, MGDK_oid, nl), *rb = newbat(0, MGDK_oid, nl);
	const size_t sbytes = (Pr.nsub + 8) * sizeof(uint64_t);
	char *sc = (char *) scratch(sbytes);
	if (!ra || !rb || !sc || !hip_ok(hipMemsetAsync(sc, 0, sbytes, st), "memset")) {
		unfix2(ra, rb);
		return sync_fail();
	}
	hipLaunchKernelGGL(k_pj_restore, dim3(Pr.nsub), dim3(1024), 0, st, flat.as<uint2>(), offT.as<uint32_t>(), P,
			   total, nl, Pr.nsub, L, R, (uint32_t *) sc, (uint64_t *) sc + 8, meta, (oid *) ra->theap,
			   (oid *) rb->theap);
	uint64_t *h64 = (uint64_t *) pinned(64);
	if (!hip_ok(hipMemcpyAsync(h64, meta, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
		unfix2(ra, rb);
		return -1;
	}
	if (h64[1] & 1) {
		seterr("HY013!BATjoin: look-back did not complete");
		unfix2(ra, rb);
		return -1;
	}
	ra->count = rb->count = h64[0];
	*ukey = true;                                       // unique build keys: one match per row
	*ap = ra;
	*bp = rb;
	return 0;
}

// ---------------------------------------------------------------------------
// Global-table path (4-byte keys, unique build keys, build side <= ~20M
// rows): only the build side is cut (the pj_cut passes above).  One
// workgroup per partition builds the partition's table in LDS and stores it
// whole as region p of ONE global table -- P regions of nbp 16-byte buckets
// (2 slots of key image + position + 1), linear probing inside the region,
// no global atomics.  At load <= 3/4 the table of 15M keys is ~170 MB, which
// stays resident in the 256 MB Infinity Cache while the probe streams past
// it (MI355X_MICROARCH.md "Infinity Cache": table + bytes moved between two
// uses of a line <= 256 MiB).  The probe is ONE ordered pass over the left
// side: per row a 4-byte key load and (almost always) one 16-byte bucket
// load served on-die, matches ranked per tile and placed by decoupled
// look-back, so r1 comes out in left order with no probe-side cut, no
// partition-major intermediate and no restore pass.  Duplicate build keys or
// an overfull region are found by the build, after which the probe's result
// is dropped and the caller falls back.
// ---------------------------------------------------------------------------

constexpr uint32_t GT_MAXB = PJ_SLOTS / 2;         // buckets per region (the LDS build table)

// flags[0] |= 1: duplicate build key; flags[1] |= 1: a partition does not
// fit its region
__global__ __launch_bounds__(1024) void
k_gt_build(const uint2 *bent, const uint32_t *bbase, int pbits, uint32_t nbp, ulonglong2 *gtab, uint32_t *flags)
{
	__shared__ unsigned long long tab[PJ_SLOTS];
	const uint32_t p = blockIdx.x, ns = 2 * nbp;
	for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x)
		tab[i] = 0ull;
	__syncthreads();
	const uint32_t b0 = bbase[p], b1 = bbase[p + 1];
	// an empty slot must remain so that every probe ends
	const bool fits = b1 - b0 < ns;
	bool dup = false;
	if (fits)
		for (uint32_t e = b0 + threadIdx.x; e < b1; e += blockDim.x) {
			const uint2 en = bent[e];
			const unsigned long long v = ((unsigned long long) (en.y + 1) << 32) | en.x;
			uint32_t s = 2 * gt_home(pj_hash(en.x), pbits, nbp);
			// every slot passed over is observed with its final content,
			// so of two equal keys the later one always sees the earlier
			for (;;) {
				const unsigned long long o = atomicCAS(&tab[s], 0ull, v);
				if (o == 0ull)
					break;
				if ((uint32_t) o == en.x) {
					dup = true;
					break;
				}
				s = s + 1 == ns ? 0 : s + 1;
			}
		}
	if (__any(dup) && __lane_id() == 0)
		atomicOr(&flags[0], 1u);
	if (!fits && threadIdx.x == 0)
		atomicOr(&flags[1], 1u);
	__syncthreads();
	ulonglong2 *dst = gtab + (size_t) p * nbp;
	for (uint32_t i = threadIdx.x; i < nbp; i += blockDim.x)
		dst[i] = make_ulonglong2(tab[2 * i], tab[2 * i + 1]);
}

struct GtArgs {
	Side l, r;
	BUN n;
	int pbits;
	uint32_t nbp;
	bool nil_matches;
	uint32_t *ticket;
	uint64_t *status;
	uint32_t ntiles;
	uint64_t *meta;       // [0] total pairs, [1] look-back error
	oid *r1, *r2;
};

constexpr int GT_JR = 8;                           // rows per lane in a probe tile

// match position + 1 of key k in its region (0: none); the first bucket is
// already loaded
__device__ __forceinline__ uint32_t
gt_find(const ulonglong2 *t, uint32_t k, ulonglong2 s, uint32_t reg, uint32_t b, uint32_t nbp)
{
	for (uint32_t d = 0;; d++) {
		if (s.x == 0ull)
			return 0;
		if ((uint32_t) s.x == k)
			return (uint32_t) (s.x >> 32);
		if (s.y == 0ull)
			return 0;
		if ((uint32_t) s.y == k)
			return (uint32_t) (s.y >> 32);
		if (d >= nbp)
			return 0;                      // (cannot happen: a region keeps an empty slot)
		b = b + 1 == nbp ? 0 : b + 1;
		s = t[(size_t) reg * nbp + b];
	}
}

template <bool DENSE, int W>
__global__ __launch_bounds__(256) void
k_gt_probe(GtArgs a, const ulonglong2 *t)
{
	constexpr int JR = GT_JR, JTILE = 256 * JR;
	__shared__ uint32_t s_tot[64];     // [r][wave]
	__shared__ uint64_t s_off[64];
	__shared__ uint32_t s_tile;
	__shared__ uint64_t s_pre;
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	if (tid == 0)
		s_tile = atomicAdd(a.ticket, 1u);
	if (JR * 4 < 64 && tid < 64)
		s_tot[tid] = 0;
	__syncthreads();
	const uint32_t tile = s_tile;
	const BUN base = (BUN) tile * JTILE + tid;
	// every load unconditional (clamped row): a load under a branch is
	// waited for before the branch joins
	uint32_t key[JR];
	bool ok[JR];
#pragma unroll
	for (int r = 0; r < JR; r++) {
		const BUN i = base + (BUN) r * 256;
		const BUN ic = i < a.n ? i : a.n - 1;
		if constexpr (W == 4) {
			const int32_t *kb = (const int32_t *) a.l.base;
			key[r] = (uint32_t) (DENSE ? __builtin_nontemporal_load(&kb[a.l.off + ic]) : kb[a.l.oids[ic] - a.l.hseq]);
			ok[r] = i < a.n && (key[r] != 0x80000000u || a.nil_matches);
		} else {
			// 8-byte keys by their 4-byte image; a value without one matches nothing
			const uint64_t *kb = (const uint64_t *) a.l.base;
			const uint64_t v = DENSE ? __builtin_nontemporal_load(&kb[a.l.off + ic]) : kb[a.l.oids[ic] - a.l.hseq];
			const bool isnil = v == (a.l.uns ? (1ull << 63) : (uint64_t) INT64_MIN);
			bool fits;
			key[r] = narrow_key(a.l, v, isnil, fits);
			ok[r] = i < a.n && fits && (!isnil || a.nil_matches);
		}
	}
	uint32_t reg[JR], bk[JR];
	ulonglong2 sv[JR];
#pragma unroll
	for (int r = 0; r < JR; r++) {
		const uint32_t h = pj_hash(key[r]);
		reg[r] = h >> (32 - a.pbits);
		bk[r] = gt_home(h, a.pbits, a.nbp);
		sv[r] = t[(size_t) reg[r] * a.nbp + bk[r]];
	}
	uint32_t m[JR];
#pragma unroll
	for (int r = 0; r < JR; r++)
		m[r] = ok[r] ? gt_find(t, key[r], sv[r], reg[r], bk[r], a.nbp) : 0;
	// ranks: one ballot per row slot r, then a 32-entry scan over (r, wave)
	uint32_t ex[JR];
#pragma unroll
	for (int r = 0; r < JR; r++) {
		const uint64_t bal = __ballot(m[r] != 0);
		ex[r] = __popcll(bal & ((1ull << lane) - 1));
		if (lane == 0)
			s_tot[r * 4 + w] = __popcll(bal);
	}
	__syncthreads();
	if (w == 0) {
		uint64_t v = s_tot[lane];
		const uint64_t own = v;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint64_t u = __shfl_up(v, o);
			if (lane >= (unsigned) o)
				v += u;
		}
		s_off[lane] = v - own;
		const uint64_t agg = __shfl(v, 63);
		const uint64_t pre = lookback(a.status, tile, agg, (uint32_t *) &a.meta[1]);
		if (lane == 0) {
			s_pre = pre;
			if (tile == a.ntiles - 1)
				a.meta[0] = pre + agg;
		}
	}
	__syncthreads();
	const uint64_t pre = s_pre;
#pragma unroll
	for (int r = 0; r < JR; r++) {
		if (m[r] == 0)
			continue;
		const uint64_t pos = pre + s_off[r * 4 + w] + ex[r];
		const BUN i = base + (BUN) r * 256;
		__builtin_nontemporal_store(oid_of(a.l, i), &a.r1[pos]);
		__builtin_nontemporal_store(oid_of(a.r, m[r] - 1), &a.r2[pos]);
	}
}

// returns 1 when not applicable (caller tries the next path)
int
join_gt(const Side &L, BUN nl, const Side &R, BUN nr, bool nil_matches, mgdk_bat **ap, mgdk_bat **bp, bool *ukey)
{
	static const int mode = getenv("MGDK_JOIN_GT") ? atoi(getenv("MGDK_JOIN_GT")) : 1;
	static const int lfpct = getenv("MGDK_JOIN_GT_LF") ? atoi(getenv("MGDK_JOIN_GT_LF")) : 72;
	// the probe's bucket loads pull whole 128-B lines: past ~2M build rows
	// (a ~25 MB table) they cost more than cutting the probe side too
	// (tools/join_sweep.py: 0.18 vs 0.25 ms at 600 K, 0.26 vs 0.27 at 1.5 M,
	// 0.47 vs 0.42 at 4 M build rows); MGDK_JOIN_GT=2 forces the path
	// 4-byte keys, or 8-byte keys by their 4-byte images (the build side's
	// values must all have one: checked while it is cut)
	const bool w4 = L.w == 4 && R.w == 4, w8 = L.w == 8 && R.w == 8 && L.base && R.base;
	if (mode == 0 || !(w4 || w8) || nr < 65536 || nl == 0 || (mode == 1 && nr > 2000000))
		return 1;
	int pbits = 6;
	while (pbits < PJ_MAXPBITS && ((BUN) 8192 << pbits) < nr)
		pbits++;
	const uint32_t P = 1u << pbits;
	// region size from the expected largest partition (mean + 6 sigma): no
	// round trip to read the real one; a partition that does not fit is
	// reported by the build and sends the join down the partitioned path
	const double mean = (double) nr / P;
	const double mx = mean + 6.0 * sqrt(mean) + 64.0;
	uint64_t nbp = (uint64_t) (mx * 100.0 / (2.0 * (lfpct < 40 ? 40 : lfpct > 90 ? 90 : lfpct))) + 1;
	if (nbp > GT_MAXB)
		return 1;
	const uint64_t jtile = 256 * GT_JR;
	const uint64_t ntiles = (nl + jtile - 1) / jtile;
	if (ntiles >= (1ull << 31))
		return 1;
	hipStream_t st = stream();
	uint32_t *meta32 = (uint32_t *) meta_buf();
	uint64_t *meta = (uint64_t *) meta32 + 4;          // [0] pairs, [1] look-back error
	if (!hip_ok(hipMemsetAsync(meta32, 0, 64, st), "memset"))
		return -1;
	PjSide B;
	DevBuf gtab((size_t) P * nbp * 16 + 64);
	mgdk_bat *ra = newbat(0, MGDK_oid, nl), *rb = newbat(0, MGDK_oid, nl);
	const size_t sbytes = (ntiles + 8) * sizeof(uint64_t);
	char *sc = (char *) scratch(sbytes);
	Side Rn = R;
	Rn.nofit = &meta32[2];
	if (!gtab.p || !ra || !rb || !sc || pj_cut(Rn, nr, pbits, !nil_matches, B, &meta32[3]) < 0) {
		(void) sync();                              // kernels may still read B's buffers
		unfix2(ra, rb);
		return -1;
	}
	hipLaunchKernelGGL(k_gt_build, dim3(P), dim3(1024), 0, st, B.ent->as<uint2>(), B.base->as<uint32_t>(), pbits,
			   (uint32_t) nbp, gtab.as<ulonglong2>(), &meta32[0]);
	GtArgs a{};
	a.l = L;
	a.r = R;
	a.n = nl;
	a.pbits = pbits;
	a.nbp = (uint32_t) nbp;
	a.nil_matches = nil_matches;
	a.ticket = (uint32_t *) sc;
	a.status = (uint64_t *) sc + 8;
	a.ntiles = (uint32_t) ntiles;
	a.meta = meta;
	a.r1 = (oid *) ra->theap;
	a.r2 = (oid *) rb->theap;
	if (!hip_ok(hipMemsetAsync(sc, 0, sbytes, st), "memset")) {
		(void) sync();
		unfix2(ra, rb);
		return -1;
	}
	if (L.w == 8) {
		if (L.dense)
			hipLaunchKernelGGL((k_gt_probe<true, 8>), dim3((unsigned) ntiles), dim3(256), 0, st, a, gtab.as<ulonglong2>());
		else
			hipLaunchKernelGGL((k_gt_probe<false, 8>), dim3((unsigned) ntiles), dim3(256), 0, st, a, gtab.as<ulonglong2>());
	} else if (L.dense) {
		hipLaunchKernelGGL((k_gt_probe<true, 4>), dim3((unsigned) ntiles), dim3(256), 0, st, a, gtab.as<ulonglong2>());
	} else {
		hipLaunchKernelGGL((k_gt_probe<false, 4>), dim3((unsigned) ntiles), dim3(256), 0, st, a, gtab.as<ulonglong2>());
	}
	uint32_t *h = (uint32_t *) pinned(64);
	if (!hip_ok(hipMemcpyAsync(h, meta32, 64, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
		unfix2(ra, rb);
		return -1;
	}
	if (h[0] || h[1] || h[2]) {                         // duplicate build keys / region overflow / no 4-byte image
		unfix2(ra, rb);
		return 1;
	}
	const uint64_t *h64 = (const uint64_t *) h + 4;   // = meta
	if (h64[1] & 1) {
		seterr("HY013!BATjoin: look-back did not complete");
		unfix2(ra, rb);
		return -1;
	}
	ra->count = rb->count = h64[0];
	*ukey = true;
	*ap = ra;
	*bp = rb;
	return 0;
}

// ---------------------------------------------------------------------------
// Broadcast path (small unique build side, <= BJ_MAXR rows; 4-byte keys or
// 8-byte keys with 4-byte images): every workgroup builds the whole build
// side's table in its LDS (the build column stays in L2) and then claims
// probe tiles by ticket, answering them from LDS and placing the matches by
// decoupled look-back -- one launch and one host round trip, instead of a
// global-table build (device-scope CAS chains) followed by a probe.  The
// grid is at most two workgroups per CU, so the tables are built a bounded
// number of times however long the probe side is.
// ---------------------------------------------------------------------------

constexpr uint32_t BJ_SLOTS = 8192;           // 64 KiB of LDS: two workgroups per CU
constexpr uint32_t BJ_MAXR = 6144;            // load <= 3/4

template <int W, bool DENSE>
__global__ __launch_bounds__(256) void
k_bj(Side L, BUN nl, Side R, uint32_t nr, bool nil_matches, uint32_t ntiles, uint32_t *ticket, uint64_t *status,
     uint64_t *meta, uint32_t *flags, oid *r1, oid *r2)
{
	constexpr int JR = GT_JR, JTILE = 256 * JR;
	__shared__ unsigned long long tab[BJ_SLOTS];
	__shared__ uint32_t s_tot[64];
	__shared__ uint64_t s_off[64];
	__shared__ uint32_t s_tile;
	__shared__ uint64_t s_pre;
	__shared__ int s_bad;
	const unsigned tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
	for (uint32_t i = tid; i < BJ_SLOTS; i += 256)
		tab[i] = 0ull;
	if (tid == 0)
		s_bad = 0;
	if (tid < 64)
		s_tot[tid] = 0;
	__syncthreads();
	// the build side: 4-byte images, nil only when nil_matches
	bool bad = false;
	for (uint32_t j = tid; j < nr; j += 256) {
		bool isnil, fits = true;
		const uint64_t v = key_of(R, j, isnil);
		const uint32_t k = W == 8 ? narrow_key(R, v, isnil, fits) : (uint32_t) v;
		if (!fits) {
			bad = true;                          // the host falls back
			continue;
		}
		if (isnil && !nil_matches)
			continue;
		const unsigned long long e = ((unsigned long long) (j + 1) << 32) | k;
		uint32_t h = pj_hash(k) >> (32 - 13);
		for (;;) {
			const unsigned long long o = atomicCAS(&tab[h], 0ull, e);
			if (o == 0ull)
				break;
			if ((uint32_t) o == k) {
				bad = true;                  // duplicate key: the general path
				break;
			}
			h = (h + 1) & (BJ_SLOTS - 1);
		}
	}
	if (__any(bad) && lane == 0)
		atomicOr(&s_bad, 1);
	__syncthreads();
	if (s_bad) {
		if (tid == 0)
			atomicOr(flags, 1u);
		// still take (and complete) tickets so the look-back of any tile
		// already claimed by another workgroup finishes
	}
	const bool skip = s_bad != 0;
	for (;;) {
		__syncthreads();
		if (tid == 0)
			s_tile = atomicAdd(ticket, 1u);
		__syncthreads();
		const uint32_t tile = s_tile;
		if (tile >= ntiles)
			break;
		const BUN base = (BUN) tile * JTILE + tid;
		// typed, unconditional loads of the tile's keys (clamped rows)
		uint64_t kv[JR];
#pragma unroll
		for (int r = 0; r < JR; r++) {
			const BUN i = base + (BUN) r * 256, ic = i < nl ? i : nl - 1;
			const BUN p = DENSE ? L.off + ic : L.oids[ic] - L.hseq;
			kv[r] = W == 8 ? ((const uint64_t *) L.base)[p] : (uint64_t) (uint32_t) ((const int32_t *) L.base)[p];
		}
		uint32_t m[JR];
#pragma unroll
		for (int r = 0; r < JR; r++) {
			const BUN i = base + (BUN) r * 256;
			m[r] = 0;
			if (i < nl && !skip) {
				bool fits = true;
				const uint64_t v = kv[r];
				const bool isnil = W == 8 ? v == (L.uns ? (1ull << 63) : (uint64_t) INT64_MIN) : (uint32_t) v == 0x80000000u;
				const uint32_t k = W == 8 ? narrow_key(L, v, isnil, fits) : (uint32_t) v;
				if (fits && (!isnil || nil_matches)) {
					uint32_t h = pj_hash(k) >> (32 - 13);
					for (;;) {
						const unsigned long long o = tab[h];
						if (o == 0ull)
							break;
						if ((uint32_t) o == k) {
							m[r] = (uint32_t) (o >> 32);
							break;
						}
						h = (h + 1) & (BJ_SLOTS - 1);
					}
				}
			}
		}
		uint32_t ex[JR];
#pragma unroll
		for (int r = 0; r < JR; r++) {
			const uint64_t bal = __ballot(m[r] != 0);
			ex[r] = __popcll(bal & ((1ull << lane) - 1));
			if (lane == 0)
				s_tot[r * 4 + w] = __popcll(bal);
		}
		__syncthreads();
		if (w == 0) {
			uint64_t v = s_tot[lane];
			const uint64_t own = v;
#pragma unroll
			for (int o = 1; o < 64; o <<= 1) {
				const uint64_t u = __shfl_up(v, o);
				if (lane >= (unsigned) o)
					v += u;
			}
			s_off[lane] = v - own;
			const uint64_t agg = __shfl(v, 63);
			const uint64_t pre = lookback(status, tile, agg, (uint32_t *) &meta[1]);
			if (lane == 0) {
				s_pre = pre;
				if (tile == ntiles - 1)
					meta[0] = pre + agg;
			}
		}
		__syncthreads();
		const uint64_t pre = s_pre;
#pragma unroll
		for (int r = 0; r < JR; r++) {
			if (m[r] == 0)
				continue;
			const uint64_t pos = pre + s_off[r * 4 + w] + ex[r];
			const BUN i = base + (BUN) r * 256;
			r1[pos] = oid_of(L, i);
			r2[pos] = oid_of(R, m[r] - 1);
		}
	}
}

// returns 1 when not applicable or the build side has duplicates / values
// without a 4-byte image (the caller takes the next path)
int
join_bj(const Side &L, BUN nl, const Side &R, BUN nr, bool nil_matches, mgdk_bat **ap, mgdk_bat **bp, bool *ukey)
{
	static const int mode = getenv("MGDK_JOIN_BJ") ? atoi(getenv("MGDK_JOIN_BJ")) : 1;
	const bool w4 = L.w == 4 && R.w == 4, w8 = L.w == 8 && R.w == 8 && L.base && R.base;
	if (mode == 0 || !(w4 || w8) || nr == 0 || nr > BJ_MAXR || nl == 0)
		return 1;
	const uint64_t jtile = 256 * GT_JR;
	const uint64_t ntiles = (nl + jtile - 1) / jtile;
	if (ntiles >= (1ull << 31))
		return 1;
	hipStream_t st = stream();
	uint32_t *meta32 = (uint32_t *) meta_buf();
	uint64_t *meta = (uint64_t *) meta32 + 4;
	mgdk_bat *ra = newbat(0, MGDK_oid, nl), *rb = newbat(0, MGDK_oid, nl);
	const size_t sbytes = (ntiles + 8) * sizeof(uint64_t);
	char *sc = (char *) scratch(sbytes);
	if (!ra || !rb || !sc || !hip_ok(hipMemsetAsync(meta32, 0, 64, st), "memset") ||
	    !hip_ok(hipMemsetAsync(sc, 0, sbytes, st), "memset")) {
		unfix2(ra, rb);
		return -1;
	}
	const unsigned grid = (unsigned) std::min<uint64_t>(ntiles, 512);
#define BJ(W_, D_) hipLaunchKernelGGL((k_bj<W_, D_>), dim3(grid), dim3(256), 0, st, L, nl, R, (uint32_t) nr, \
				   nil_matches, (uint32_t) ntiles, (uint32_t *) sc, (uint64_t *) sc + 8, meta, &meta32[0], \
				   (oid *) ra->theap, (oid *) rb->theap)
	if (w8) {
		if (L.dense) BJ(8, true); else BJ(8, false);
	} else {
		if (L.dense) BJ(4, true); else BJ(4, false);
	}
#undef BJ
	uint32_t *h = (uint32_t *) pinned(64);
	if (!hip_ok(hipMemcpyAsync(h, meta32, 64, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
		unfix2(ra, rb);
		return -1;
	}
	if (h[0]) {
		unfix2(ra, rb);
		return 1;
	}
	const uint64_t *h64 = (const uint64_t *) h + 4;
	if (h64[1] & 1) {
		seterr("HY013!BATjoin: look-back did not complete");
		unfix2(ra, rb);
		return -1;
	}
	ra->count = rb->count = h64[0];
	*ukey = true;
	*ap = ra;
	*bp = rb;
	return 0;
}

}  // namespace

namespace mgdk {

thread_local JoinEnds join_ends;

// hashjoin (gdk/gdk_join.c:2900-3335) over candidate lists already
// initialised: per l candidate in order, the matches in r in DESCENDING
// position.  The caller (joinalgo.hip) chose this algorithm and sets the
// result properties.  *ukey: the build side had no duplicate key, so no
// probe row has two matches (r1 holds no repeated oid).
int
hash_join(const mgdk_bat *l, const mgdk_bat *r, const Cand &lc, const Cand &rc, bool nil_matches,
	  mgdk_bat **ap, mgdk_bat **bp, bool *ukey)
{
	*ukey = false;
	const BUN nl = lc.n, nr = rc.n;
	if (nr >= ((BUN) 1 << 32) - 1 || nl >= ((BUN) 1 << 32)) {
		seterr("42000!BATjoin: more than 2^32 rows per side");
		return -1;
	}
	Side L{}, R{};
	side_init(L, l, lc);
	side_init(R, r, rc);
	const int w = L.w;
	int rc_ = w == 4 || w == 8 ? join_bj(L, nl, R, nr, nil_matches, ap, bp, ukey) : 1;
	if (rc_ > 0 && (w == 4 || w == 8))
		rc_ = join_gt(L, nl, R, nr, nil_matches, ap, bp, ukey);
	if (rc_ > 0 && (w == 4 || w == 8))
		rc_ = join_part(L, nl, R, nr, nil_matches, ap, bp, ukey);
	if (rc_ > 0)
		rc_ = w == 8 ? join_lp<8>(L, nl, R, nr, nil_matches, ap, bp, ukey)
			     : join_lp<4>(L, nl, R, nr, nil_matches, ap, bp, ukey);
	if (rc_ > 0)
		rc_ = join_csr(L, nl, R, nr, nil_matches, ap, bp);
	return rc_ < 0 ? -1 : 0;
}

}  // namespace mgdk
