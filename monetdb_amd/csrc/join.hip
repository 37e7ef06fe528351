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
				if (d >= a.maxd) {
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
				if (d >= a.maxd)
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

bool
join_type_ok(int t)
{
	t = basetype(t);
	return t == MGDK_bte || t == MGDK_sht || t == MGDK_int || t == MGDK_lng || t == MGDK_oid;
}

void
side_init(Side &s, const mgdk_bat *b, const Cand &c)
{
	s.base = b->theap;
	s.w = b->twidth;
	s.uns = basetype(b->ttype) == MGDK_oid;
	s.dense = c.dense;
	s.off = c.dense ? c.seq - b->hseqbase : 0;
	s.oids = c.oids;
	s.hseq = b->hseqbase;
	s.cseq = c.seq;
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
join_lp(const Side &L, BUN nl, const Side &R, BUN nr, bool nil_matches, mgdk_bat **ap, mgdk_bat **bp)
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
	if (!hip_ok(hipMemcpyAsync(h, meta, 32, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	const uint32_t maxd = (uint32_t) h[2];
	const bool uniq = h[3] == 0;
	if (maxd > DMAX || (!uniq && maxd > DMAX_DUP))
		return 1;

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
		    !hip_ok(hipMemsetAsync(meta, 0, 16, st), "memset")) {
			unfix2(ra, rb);
			return -1;
		}
		if (uniq)
			hipLaunchKernelGGL((k_lp_probe<KW, true>), dim3((unsigned) ntiles), dim3(256), 0, st, a,
					   (const slot_t *) tab.p);
		else
			hipLaunchKernelGGL((k_lp_probe<KW, false>), dim3((unsigned) ntiles), dim3(256), 0, st, a,
					   (const slot_t *) tab.p);
		if (!hip_ok(hipMemcpyAsync(h, meta, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
			unfix2(ra, rb);
			return -1;
		}
		if (h[1] & 1) {
			seterr("HY013!BATjoin: look-back did not complete");
			unfix2(ra, rb);
			return -1;
		}
		const uint64_t nout = h[0];
		if (nout <= ocap) {
			ra->count = rb->count = nout;
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

}  // namespace

extern "C" int
mgdk_BATjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
	     bool nil_matches, mgdk_BUN estimate)
{
	(void) estimate;
	if (l == nullptr || r == nullptr || r1p == nullptr) {
		seterr("BATjoin: NULL argument");
		return -1;
	}
	if (basetype(l->ttype) != basetype(r->ttype)) {
		seterr("42000!BATjoin: type mismatch (%s, %s)", atomname(l->ttype), atomname(r->ttype));
		return -1;
	}
	if (!join_type_ok(l->ttype)) {
		seterr("42000!BATjoin: type %s not supported on the device path", atomname(l->ttype));
		return -1;
	}
	ProfScope prof("join");
	Cand lc, rc;
	if (cand_init(&lc, l, sl) < 0 || cand_init(&rc, r, sr) < 0)
		return -1;
	const BUN nl = lc.n, nr = rc.n;
	if (nr >= ((BUN) 1 << 32) - 1 || nl >= ((BUN) 1 << 32)) {
		seterr("42000!BATjoin: more than 2^32 rows per side");
		return -1;
	}
	Side L{}, R{};
	side_init(L, l, lc);
	side_init(R, r, rc);
	mgdk_bat *a = nullptr, *b = nullptr;
	int rc_ = 0;
	if (nl == 0 || nr == 0) {
		a = newbat(0, MGDK_oid, 0);
		b = newbat(0, MGDK_oid, 0);
		if (!a || !b) {
			unfix2(a, b);
			return -1;
		}
	} else {
		rc_ = l->twidth == 8 ? join_lp<8>(L, nl, R, nr, nil_matches, &a, &b)
				     : join_lp<4>(L, nl, R, nr, nil_matches, &a, &b);
		if (rc_ > 0)
			rc_ = join_csr(L, nl, R, nr, nil_matches, &a, &b);
		if (rc_ < 0)
			return -1;
	}
	const uint64_t nout = a->count;
	a->tsorted = 1;                 // left candidates in order
	a->trevsorted = nout <= 1;
	a->tkey = nout <= 1;
	a->tnonil = b->tnonil = 1;
	b->tsorted = b->trevsorted = b->tkey = nout <= 1;
	*r1p = a;
	if (r2p)
		*r2p = b;
	else
		mgdk_BBPunfix(b);
	return 0;
}
