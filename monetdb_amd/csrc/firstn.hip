// firstn.hip -- BATfirstn on the MI355X (gdk/gdk_firstn.c:1280; SURVEY.md
// §8(f) row 2: the ORDER BY ... LIMIT step after the aggregates).
//
// The reference keeps a binary heap of n candidate oids (:60-97, :212-700)
// and, for the variants that return group ids or distinct groups, adds
// every row equal to the heap's last value (:1023-1280).  On the device the
// n-th best (group, value) pair is found by radix SELECTION (one 256-bin
// histogram pass per 8-bit digit over order-preserving 64-bit rank images,
// first of the prior group ids, then of the values inside the selected
// group), and the result is one ordered compaction of the candidates that
// rank below it (plus the tied ones):
//   * gids requested or distinct: all rows tied with the last value -- the
//     same set as the reference;
//   * plain top-n (gids NULL): the rows strictly better than the last value;
//     when the last value is tied with rows beyond n, the reference's heap
//     is replayed on the device (see "plain first-N" below) so the same
//     tied rows survive; sorted / reverse-sorted / void inputs take the
//     reference's slices (:247-356).
// Group ids are computed exactly as the reference composes them
// (BATproject + BATsort with o/g, :1085-1110, :1223-1268).
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

// rank image: smaller = earlier in the requested order
template <typename T>
__device__ __forceinline__ uint64_t
rankimg(T v, bool asc, bool nilslast)
{
	uint64_t u;
	bool isnil;
	if constexpr (sizeof(T) == 4 && (T) 0.5 != 0) {
		isnil = v != v;
		const float f = v == 0 ? 0.0f : v;
		uint32_t b = __float_as_uint(f);
		b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
		u = (uint64_t) b << 32;
	} else if constexpr (sizeof(T) == 8 && (T) 0.5 != 0) {
		isnil = v != v;
		const double f = v == 0 ? 0.0 : v;
		const uint64_t b = (uint64_t) __double_as_longlong(f);
		u = (b & (1ull << 63)) ? ~b : (b | (1ull << 63));
	} else if constexpr (T(-1) > T(0)) {
		// oid compares as lng (ATOMbasetype, gdk_firstn.c:353): nil smallest
		isnil = (uint64_t) v == ((uint64_t) 1 << 63);
		u = (uint64_t) v ^ (1ull << 63);
	} else {
		isnil = v == NilOf<T>::v();
		u = (uint64_t) (int64_t) v ^ (1ull << 63);
	}
	if (!asc)
		u = ~u;
	// non-nil images lie in [1, 2^64 - 2] after this shift, so a nil placed
	// at either end never ties with a value (e.g. lng_max descending)
	if (asc && nilslast)
		u -= 1;
	else if (!asc && !nilslast)
		u += 1;
	if (isnil)
		u = nilslast ? ~0ull : 0ull;
	return u;
}

template <typename T>
__global__ __launch_bounds__(256) void
k_rank_keys(const T *col, Cand ci, oid hseq, bool asc, bool nilslast, const oid *g, oid gseq, uint64_t *vk,
	    uint64_t *gk)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < ci.n; i += (BUN) gridDim.x * blockDim.x) {
		const oid o = ci.dense ? ci.seq + i : ci.oids[i];
		vk[i] = rankimg<T>(col[o - hseq], asc, nilslast);
		if (gk)
			gk[i] = g ? g[i] : gseq + i;
	}
}

// histogram of digit `shift` over keys whose higher digits equal pval
// (and, for the value stage, whose group key equals gstar)
__global__ __launch_bounds__(256) void
k_rsel_hist(const uint64_t *keys, BUN n, uint64_t pmask, uint64_t pval, int shift, const uint64_t *gk,
	    uint64_t gstar, unsigned long long *hist)
{
	__shared__ uint32_t h[256];
	h[threadIdx.x] = 0;
	__syncthreads();
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint64_t k = keys[i];
		if ((k & pmask) == pval && (!gk || gk[i] == gstar))
			atomicAdd(&h[(k >> shift) & 255], 1u);
	}
	__syncthreads();
	if (h[threadIdx.x])
		atomicAdd(&hist[threadIdx.x], (unsigned long long) h[threadIdx.x]);
}

// 0: after the threshold, 1: strictly before, 2: tied with it
__global__ __launch_bounds__(256) void
k_sel_class(const uint64_t *vk, const uint64_t *gk, BUN n, uint64_t gstar, uint64_t vstar, uint8_t *cls,
	    uint8_t *eq)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint64_t g = gk ? gk[i] : 0;
		const uint64_t v = vk[i];
		uint8_t c = 0;
		if (g < gstar || (g == gstar && v < vstar))
			c = 1;
		else if (g == gstar && v == vstar)
			c = 2;
		cls[i] = c;
		eq[i] = c == 2;
	}
}

__global__ __launch_bounds__(256) void
k_sel_flags(const uint8_t *cls, const uint64_t *eqrank, BUN n, uint64_t take_eq, int8_t *flags)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint8_t c = cls[i];
		flags[i] = c == 1 || (c == 2 && (eqrank == nullptr || eqrank[i] < take_eq));
	}
}


// ---- plain first-N: the reference's heap, reproduced exactly -------------
// BATfirstn without group ids (gdk_firstn.c:211-572, :716-1020) keeps a
// binary heap of n candidates and replaces its root by every later
// candidate that ranks strictly before it; which of the rows tied with the
// n-th value survive depends on the heap's shape.  When the n-th value is
// tied with rows beyond n, the device replays that heap: the initial heap
// (the first n candidates, or for a descending top-n the last n in reverse)
// is built level by level (siftdowns of one level touch disjoint subtrees,
// so they run in parallel in the same result as heapify's sequential loop),
// and only candidates that can still enter it are replayed, in order, by
// one wave.  Which candidates can enter is bounded per 64 Ki-candidate
// block: the root at a block's start is the n-th best of everything before
// it, so once the candidates before the block hold n keys below a splitter
// s, only keys below s - 1 can enter.  Splitters are the threshold, its
// successor and geometric quantiles of a 2048-key sample (ranks n * 2^b),
// so for any input order the replay touches a few times n * log(N / n)
// candidates in expectation.

constexpr int FN_SAMPLE = 2048;
constexpr int FN_NSPL = 63;            // splitters (+1 histogram bin)
constexpr BUN FN_BLOCK = 65536;         // candidates per bound block

__device__ __forceinline__ bool
kless(uint64_t g1, uint64_t v1, uint64_t g2, uint64_t v2)
{
	return g1 < g2 || (g1 == g2 && v1 < v2);
}

struct FnSpl {
	uint64_t g[FN_NSPL], v[FN_NSPL];
	int n;
};

// sorted sample of the candidates' (group, value) keys -> splitters
__global__ __launch_bounds__(1024) void
k_fn_splitters(const uint64_t *vk, const uint64_t *gk, BUN cnt, BUN n, uint64_t tg, uint64_t tv, FnSpl *out)
{
	__shared__ uint64_t sg[FN_SAMPLE], sv[FN_SAMPLE];
	for (int i = threadIdx.x; i < FN_SAMPLE; i += blockDim.x) {
		const BUN p = (BUN) ((unsigned __int128) i * cnt / FN_SAMPLE);
		sg[i] = gk ? gk[p] : 0;
		sv[i] = vk[p];
	}
	__syncthreads();
	// bitonic sort of FN_SAMPLE pairs
	for (int k = 2; k <= FN_SAMPLE; k <<= 1) {
		for (int j = k >> 1; j > 0; j >>= 1) {
			for (int i = threadIdx.x; i < FN_SAMPLE; i += blockDim.x) {
				const int l = i ^ j;
				if (l > i) {
					const bool up = (i & k) == 0;
					const bool gt = kless(sg[l], sv[l], sg[i], sv[i]);
					if (gt == up) {
						uint64_t t = sg[i]; sg[i] = sg[l]; sg[l] = t;
						t = sv[i]; sv[i] = sv[l]; sv[l] = t;
					}
				}
			}
			__syncthreads();
		}
	}
	if (threadIdx.x != 0)
		return;
	uint64_t G[FN_NSPL], V[FN_NSPL];
	int m = 0;
	G[m] = tg; V[m] = tv; m++;
	if (tv != ~0ull) { G[m] = tg; V[m] = tv + 1; m++; }
	else if (tg != ~0ull) { G[m] = tg + 1; V[m] = 0; m++; }
	for (int b = 0; b < 62 && m < FN_NSPL; b++) {
		const unsigned __int128 r = ((unsigned __int128) n << b) * FN_SAMPLE / (cnt ? cnt : 1);
		if (r >= FN_SAMPLE)
			break;
		G[m] = sg[(int) r]; V[m] = sv[(int) r]; m++;
	}
	for (int i = 1; i < m; i++)            // insertion sort
		for (int j = i; j > 0 && kless(G[j], V[j], G[j - 1], V[j - 1]); j--) {
			uint64_t t = G[j]; G[j] = G[j - 1]; G[j - 1] = t;
			t = V[j]; V[j] = V[j - 1]; V[j - 1] = t;
		}
	for (int i = 0; i < m; i++) {
		out->g[i] = G[i];
		out->v[i] = V[i];
	}
	out->n = m;
}

// number of splitters <= key
__device__ __forceinline__ int
fn_bin(const FnSpl &S, uint64_t g, uint64_t v)
{
	int lo = 0, hi = S.n;
	while (lo < hi) {
		const int mid = (lo + hi) >> 1;
		if (kless(g, v, S.g[mid], S.v[mid]))
			hi = mid;
		else
			lo = mid + 1;
	}
	return lo;
}

// per-block histograms over the splitter bins: blocks [0, nbi) cover the
// initial heap [i0, i0 + n), blocks [nbi, ...) the replayed range [s0, s0 + slen)
__global__ __launch_bounds__(256) void
k_fn_hist(const uint64_t *vk, const uint64_t *gk, BUN i0, BUN n, BUN s0, BUN slen, unsigned nbi, const FnSpl *spl,
	  uint32_t *hist)
{
	__shared__ FnSpl S;
	__shared__ uint32_t h[64];
	if (threadIdx.x == 0)
		S = *spl;
	if (threadIdx.x < 64)
		h[threadIdx.x] = 0;
	__syncthreads();
	const unsigned r = blockIdx.x;
	BUN a, e;
	if (r < nbi) {
		a = i0 + (BUN) r * FN_BLOCK;
		e = min(i0 + n, a + FN_BLOCK);
	} else {
		a = s0 + (BUN) (r - nbi) * FN_BLOCK;
		e = min(s0 + slen, a + FN_BLOCK);
	}
	for (BUN i = a + threadIdx.x; i < e; i += blockDim.x)
		atomicAdd(&h[fn_bin(S, gk ? gk[i] : 0, vk[i])], 1u);
	__syncthreads();
	if (threadIdx.x < 64)
		hist[(size_t) r * 64 + threadIdx.x] = h[threadIdx.x];
}

// one wave: running per-bin counts over the blocks in order; block j's bound
// = the first splitter below which the candidates before it hold n keys
__global__ __launch_bounds__(64) void
k_fn_bounds(const uint32_t *hist, unsigned nbi, unsigned nbs, BUN n, const FnSpl *spl, uint8_t *ub)
{
	const int l = threadIdx.x;
	const int ns = spl->n;
	uint64_t run = 0;
	const unsigned rows = nbi + nbs;
	for (unsigned r0 = 0; r0 < rows; r0 += 16) {
		uint32_t pre[16];
#pragma unroll
		for (int k = 0; k < 16; k++)
			pre[k] = r0 + k < rows ? hist[(size_t) (r0 + k) * 64 + l] : 0;
#pragma unroll
		for (int k = 0; k < 16; k++) {
			const unsigned r = r0 + k;
			if (r >= rows)
				break;
			if (r >= nbi) {
				uint64_t sc = run;      // inclusive scan over bins: keys below splitter l
#pragma unroll
				for (int o = 1; o < 64; o <<= 1) {
					const uint64_t t = __shfl_up(sc, o);
					if (l >= o)
						sc += t;
				}
				const uint64_t m = __ballot(l < ns && sc >= n);
				if (l == 0)
					ub[r - nbi] = m ? (uint8_t) __builtin_ctzll(m) : (uint8_t) ns;
			}
			run += pre[k];
		}
	}
}

// may candidate i (in bound block j) still enter the heap?  key < s - 1
__global__ __launch_bounds__(256) void
k_fn_flags(const uint64_t *vk, const uint64_t *gk, BUN s0, BUN slen, const uint8_t *ub, const FnSpl *spl,
	   int8_t *flags)
{
	__shared__ FnSpl S;
	if (threadIdx.x == 0)
		S = *spl;
	__syncthreads();
	for (BUN t = (BUN) blockIdx.x * blockDim.x + threadIdx.x; t < slen; t += (BUN) gridDim.x * blockDim.x) {
		const int b = ub[t / FN_BLOCK];
		bool pass = true;
		if (b < S.n) {
			const uint64_t g = gk ? gk[s0 + t] : 0, v = vk[s0 + t];
			const uint64_t sg = S.g[b], sv = S.v[b];
			const bool pred = (g == sg && v + 1 == sv) || (v == ~0ull && sv == 0 && g + 1 == sg);
			pass = kless(g, v, sg, sv) && !pred;
		}
		flags[t] = pass;
	}
}

struct FnHeap {
	uint64_t *idx, *g, *v;    // slot -> candidate index and its key
	BUN n;
};

// single lane: gdk_firstn.c:71-91 siftdown (max-heap under "ranks before")
__device__ void
fn_siftdown(FnHeap h, BUN pos)
{
	uint64_t pg = h.g[pos], pv = h.v[pos], pi = h.idx[pos];
	BUN c = 2 * pos + 1;
	while (c < h.n) {
		uint64_t cg = h.g[c], cv = h.v[c];
		if (c + 1 < h.n) {
			const uint64_t dg = h.g[c + 1], dv = h.v[c + 1];
			if (!kless(dg, dv, cg, cv)) {
				c++;
				cg = dg;
				cv = dv;
			}
		}
		if (!kless(pg, pv, cg, cv))
			break;
		h.g[pos] = cg;
		h.v[pos] = cv;
		h.idx[pos] = h.idx[c];
		pos = c;
		c = 2 * pos + 1;
	}
	h.g[pos] = pg;
	h.v[pos] = pv;
	h.idx[pos] = pi;
}

__global__ __launch_bounds__(256) void
k_fn_heap_init(FnHeap h, const uint64_t *vk, const uint64_t *gk, BUN cnt, bool reversed)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < h.n; i += (BUN) gridDim.x * blockDim.x) {
		const BUN c = reversed ? cnt - 1 - i : i;
		h.idx[i] = c;
		h.v[i] = vk[c];
		h.g[i] = gk ? gk[c] : 0;
	}
}

// heapify, one level: nodes [lo, hi) have disjoint subtrees
__global__ __launch_bounds__(256) void
k_fn_heapify_level(FnHeap h, BUN lo, BUN hi)
{
	for (BUN i = lo + (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (BUN) gridDim.x * blockDim.x)
		fn_siftdown(h, i);
}

// replay the filtered candidates in order (one wave; lane 0 sifts)
__global__ __launch_bounds__(64) void
k_fn_replay(FnHeap h, const uint64_t *vk, const uint64_t *gk, const oid *cidx, oid cseq, BUN nc)
{
	const int l = threadIdx.x;
	uint64_t rg = h.g[0], rv = h.v[0];
	for (BUN b = 0; b < nc; b += 64) {
		const BUN t = b + l;
		uint64_t c = 0, g = 0, v = 0;
		if (t < nc) {
			c = cidx ? cidx[t] : cseq + t;
			g = gk ? gk[c] : 0;
			v = vk[c];
		}
		uint64_t m = __ballot(t < nc && kless(g, v, rg, rv));
		while (m) {
			const int f = __builtin_ctzll(m);
			const uint64_t fc = __shfl(c, f), fg = __shfl(g, f), fv = __shfl(v, f);
			uint64_t ng = 0, nv = 0;
			if (l == 0) {
				h.idx[0] = fc;
				h.g[0] = fg;
				h.v[0] = fv;
				fn_siftdown(h, 0);
				ng = h.g[0];          // lane 0's own stores: program order
				nv = h.v[0];
			}
			rg = __shfl(ng, 0);
			rv = __shfl(nv, 0);
			m = __ballot(t < nc && l > f && kless(g, v, rg, rv));
		}
	}
}

__global__ __launch_bounds__(256) void
k_fn_mark(FnHeap h, int8_t *flags)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < h.n; i += (BUN) gridDim.x * blockDim.x)
		flags[h.idx[i]] = 1;
}

__global__ __launch_bounds__(256) void
k_fn_slice_flags(int8_t *flags, BUN cnt, BUN a0, BUN a1, BUN b0, BUN b1)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (BUN) gridDim.x * blockDim.x)
		flags[i] = (i >= a0 && i < a1) || (i >= b0 && i < b1);
}

// BATordered / BATordered_rev over the whole of b, and its number of nils
template <typename T>
__global__ __launch_bounds__(256) void
k_fn_props(const T *col, BUN n, uint32_t *out, unsigned long long *nils)
{
	uint32_t f = 0;
	unsigned long long c = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint64_t x = rankimg<T>(col[i], true, false);
		c += x == 0;
		if (i > 0) {
			const uint64_t w = rankimg<T>(col[i - 1], true, false);
			if (w > x)
				f |= 1;          // not sorted
			if (w < x)
				f |= 2;          // not reverse sorted
		}
	}
	f = block_reduce(f, [](uint32_t a, uint32_t b) { return a | b; });
	if (threadIdx.x == 0)
		publish_or(out, f);
	c = block_reduce(c, [](unsigned long long a, unsigned long long b) { return a + b; });
	if (threadIdx.x == 0 && c)
		atomicAdd(nils, c);
}

// radix selection of the k-th smallest (1-based) key; returns the key and
// the rank k' of the wanted element among the keys equal to it
int
rsel(const uint64_t *keys, BUN n, uint64_t k, const uint64_t *gk, uint64_t gstar, uint64_t *val, uint64_t *krem,
     uint64_t *neq = nullptr)
{
	hipStream_t st = stream();
	DevBuf hist(256 * 8);
	unsigned long long *h = (unsigned long long *) pinned(256 * 8);
	if (!hist.p || !h)
		return -1;
	uint64_t pmask = 0, pval = 0;
	for (int shift = 56; shift >= 0; shift -= 8) {
		if (!hip_ok(hipMemsetAsync(hist.p, 0, 256 * 8, st), "memset"))
			return -1;
		hipLaunchKernelGGL(k_rsel_hist, dim3(grid_for(n, 4096, 2048)), dim3(256), 0, st, keys, n, pmask, pval, shift,
				   gk, gstar, hist.as<unsigned long long>());
		if (!hip_ok(hipMemcpyAsync(h, hist.p, 256 * 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			return -1;
		int b = 0;
		for (; b < 256; b++) {
			if (k <= h[b])
				break;
			k -= h[b];
		}
		if (b == 256) {
			seterr("BATfirstn: selection out of range");
			return -1;
		}
		pval |= (uint64_t) b << shift;
		pmask |= (uint64_t) 255 << shift;
		if (neq)
			*neq = h[b];
	}
	*val = pval;
	*krem = k;
	return 0;
}

template <typename T>
void
launch_rank(const mgdk_bat *b, const Cand &ci, bool asc, bool nilslast, const mgdk_bat *g, uint64_t *vk,
	    uint64_t *gk)
{
	hipLaunchKernelGGL((k_rank_keys<T>), dim3(grid_for(ci.n, 1024, 8192)), dim3(256), 0, stream(), (const T *) b->theap,
			   ci, b->hseqbase, asc, nilslast,
			   g && g->ttype != MGDK_void ? (const oid *) g->theap : nullptr, g ? g->tseqbase : 0, vk, gk);
}

bool
firstn_type(int t)
{
	t = basetype(t);
	return t == MGDK_bte || t == MGDK_sht || t == MGDK_int || t == MGDK_lng || t == MGDK_oid || t == MGDK_flt ||
	       t == MGDK_dbl;
}

// candidate positions [0, cnt) selected -> candidate oids
mgdk_bat *
flags_to_cands(const int8_t *flags, const Cand &ci, const mgdk_bat *s)
{
	if (ci.dense)
		return compact_flags(flags, ci.n, ci.seq);
	mgdk_bat *pos = compact_flags(flags, ci.n, s->hseqbase);
	if (pos == nullptr)
		return nullptr;
	mgdk_bat *r = mgdk_BATproject(pos, (mgdk_bat *) s);
	mgdk_BBPunfix(pos);
	return r;
}

// positions (as s-head oids) of the selected candidates (for projecting g)
mgdk_bat *
flags_to_pos(const int8_t *flags, const Cand &ci, const mgdk_bat *s)
{
	return compact_flags(flags, ci.n, s ? s->hseqbase : 0);
}

// rank images of the candidates (+ their prior group ids)
struct Ranked {
	DevBuf vk, gk;
	bool hasg;
	Ranked(BUN cnt, bool g) : vk(cnt * 8 + 8), gk(g ? cnt * 8 + 8 : 8), hasg(g) {}
	const uint64_t *g() const { return hasg ? gk.as<uint64_t>() : nullptr; }
};

int
rank_cands(mgdk_bat *b, const Cand &ci, const mgdk_bat *g, bool asc, bool nilslast, Ranked &r)
{
	if (!r.vk.p || !r.gk.p)
		return -1;
	uint64_t *vk = r.vk.as<uint64_t>(), *gk = g ? r.gk.as<uint64_t>() : nullptr;
	switch (basetype(b->ttype)) {
	case MGDK_bte: launch_rank<int8_t>(b, ci, asc, nilslast, g, vk, gk); break;
	case MGDK_sht: launch_rank<int16_t>(b, ci, asc, nilslast, g, vk, gk); break;
	case MGDK_int: launch_rank<int32_t>(b, ci, asc, nilslast, g, vk, gk); break;
	case MGDK_lng: launch_rank<int64_t>(b, ci, asc, nilslast, g, vk, gk); break;
	case MGDK_oid: launch_rank<uint64_t>(b, ci, asc, nilslast, g, vk, gk); break;
	case MGDK_flt: launch_rank<float>(b, ci, asc, nilslast, g, vk, gk); break;
	default: launch_rank<double>(b, ci, asc, nilslast, g, vk, gk); break;
	}
	return 0;
}

// the n-th smallest (group, value) pair: (gstar, vstar) and the rank krem of
// the n-th row among the rows tied with it
int
find_threshold(const Ranked &r, BUN cnt, BUN n, uint64_t *gstar, uint64_t *vstar, uint64_t *krem,
	       uint64_t *neq = nullptr)
{
	uint64_t k = n;
	*gstar = 0;
	if (r.hasg) {
		uint64_t kg;
		if (rsel(r.g(), cnt, k, nullptr, 0, gstar, &kg) < 0)
			return -1;
		k = kg;             // rank inside the selected group
	}
	return rsel(r.vk.as<uint64_t>(), cnt, k, r.g(), *gstar, vstar, krem, neq);
}

// candidates ranking before (gstar, vstar), plus the tied ones (all, or the
// first take_eq in candidate order)
int
emit_selection(const Ranked &r, const Cand &ci, const mgdk_bat *s, uint64_t gstar, uint64_t vstar, bool all_ties,
	       uint64_t take_eq, mgdk_bat **cands, mgdk_bat **pos)
{
	const BUN cnt = ci.n;
	hipStream_t st = stream();
	DevBuf cls(cnt + 8), eq(cnt + 8), er(all_ties ? 8 : cnt * 8 + 8), fl(cnt + 8);
	if (!cls.p || !eq.p || !er.p || !fl.p)
		return -1;
	const dim3 grd(grid_for(cnt, 1024, 8192)), blk(256);
	hipLaunchKernelGGL(k_sel_class, grd, blk, 0, st, r.vk.as<uint64_t>(), r.g(), cnt, gstar, vstar,
			   cls.as<uint8_t>(), eq.as<uint8_t>());
	const uint64_t *eqrank = nullptr;
	if (!all_ties) {
		uint64_t tot;
		if (exclusive_scan(eq.as<uint8_t>(), er.as<uint64_t>(), cnt, &tot) < 0)
			return -1;
		eqrank = er.as<uint64_t>();
	}
	hipLaunchKernelGGL(k_sel_flags, grd, blk, 0, st, cls.as<uint8_t>(), eqrank, cnt, take_eq, fl.as<int8_t>());
	*cands = flags_to_cands(fl.as<int8_t>(), ci, s);
	if (*cands == nullptr)
		return -1;
	if (pos) {
		*pos = flags_to_pos(fl.as<int8_t>(), ci, s);
		if (*pos == nullptr) {
			mgdk_BBPunfix(*cands);
			*cands = nullptr;
			return -1;
		}
	}
	return 0;
}

mgdk_bat *
all_cands(const Cand &ci, const mgdk_bat *s)
{
	if (ci.dense)
		return mgdk_BATdense(0, ci.seq, ci.n);
	mgdk_bat *d = mgdk_BATdense(0, s->hseqbase, ci.n);
	mgdk_bat *r = d ? mgdk_BATproject(d, (mgdk_bat *) s) : nullptr;
	mgdk_BBPunfix(d);
	return r;
}


// candidates [a0, a1) u [b0, b1) (positions in the candidate list)
mgdk_bat *
slice_cands(const Cand &ci, const mgdk_bat *s, BUN a0, BUN a1, BUN b0, BUN b1)
{
	DevBuf fl(ci.n + 8);
	if (!fl.p)
		return nullptr;
	hipLaunchKernelGGL(k_fn_slice_flags, dim3(grid_for(ci.n, 1024, 8192)), dim3(256), 0, stream(), fl.as<int8_t>(),
			   ci.n, a0, a1, b0, b1);
	return flags_to_cands(fl.as<int8_t>(), ci, s);
}

template <typename T>
void
launch_props(const mgdk_bat *b, uint32_t *out, unsigned long long *nils)
{
	hipLaunchKernelGGL((k_fn_props<T>), dim3(grid_for(b->count, 4096, 4096)), dim3(256), 0, stream(),
			   (const T *) b->theap, b->count, out, nils);
}

// BATordered / BATordered_rev (exact), whether b holds a nil, and the number
// of nils (the leading rows of an ascending column)
int
fn_props(const mgdk_bat *b, bool *sorted, bool *revsorted, bool *hasnil, BUN *nnil)
{
	unsigned long long *m = (unsigned long long *) meta_buf();
	unsigned long long *h = (unsigned long long *) pinned(16);
	if (!hip_ok(hipMemsetAsync(m, 0, 16, stream()), "memset"))
		return -1;
	uint32_t *f = (uint32_t *) m;
	switch (basetype(b->ttype)) {
	case MGDK_bte: launch_props<int8_t>(b, f, m + 1); break;
	case MGDK_sht: launch_props<int16_t>(b, f, m + 1); break;
	case MGDK_int: launch_props<int32_t>(b, f, m + 1); break;
	case MGDK_lng: launch_props<int64_t>(b, f, m + 1); break;
	case MGDK_oid: launch_props<uint64_t>(b, f, m + 1); break;
	case MGDK_flt: launch_props<float>(b, f, m + 1); break;
	default: launch_props<double>(b, f, m + 1); break;
	}
	if (!hip_ok(hipMemcpyAsync(h, m, 16, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return -1;
	const uint32_t bits = (uint32_t) h[0];
	*sorted = !(bits & 1);
	*revsorted = !(bits & 2);
	*nnil = h[1];
	*hasnil = h[1] != 0;
	return 0;
}

// number of candidates with oid < o
__global__ void
k_fn_lower(const oid *oids, BUN n, oid o, BUN *out)
{
	BUN lo = 0, hi = n;
	while (lo < hi) {
		const BUN m = (lo + hi) / 2;
		if (oids[m] < o)
			lo = m + 1;
		else
			hi = m;
	}
	*out = lo;
}

int
cands_below(const Cand &ci, oid o, BUN *pos)
{
	if (ci.dense) {
		*pos = o <= ci.seq ? 0 : (o - ci.seq >= ci.n ? ci.n : o - ci.seq);
		return 0;
	}
	BUN *m = (BUN *) meta_buf(), *h = (BUN *) pinned(8);
	hipLaunchKernelGGL(k_fn_lower, dim3(1), dim3(1), 0, stream(), ci.oids, ci.n, o, m);
	if (!hip_ok(hipMemcpyAsync(h, m, 8, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return -1;
	*pos = *h;
	return 0;
}

// replay of the reference's heap (see the kernels above); cnt > n
mgdk_bat *
heap_replay(const Ranked &r, const Cand &ci, const mgdk_bat *s, BUN n, bool reversed, uint64_t gs, uint64_t vs)
{
	const BUN cnt = ci.n;
	hipStream_t st = stream();
	const uint64_t *vk = r.vk.as<uint64_t>(), *gk = r.g();
	const BUN i0 = reversed ? cnt - n : 0, s0 = reversed ? 0 : n, slen = cnt - n;
	const unsigned nbi = (unsigned) ((n + FN_BLOCK - 1) / FN_BLOCK), nbs = (unsigned) ((slen + FN_BLOCK - 1) / FN_BLOCK);
	DevBuf spl(sizeof(FnSpl)), hist((size_t) (nbi + nbs) * 64 * 4 + 8), ub(nbs + 8), fl(slen + 8);
	DevBuf hidx(n * 8 + 8), hg(n * 8 + 8), hv(n * 8 + 8), out(cnt + 8);
	if (!spl.p || !hist.p || !ub.p || !fl.p || !hidx.p || !hg.p || !hv.p || !out.p)
		return nullptr;
	FnSpl *S = spl.as<FnSpl>();
	hipLaunchKernelGGL(k_fn_splitters, dim3(1), dim3(1024), 0, st, vk, gk, cnt, n, gs, vs, S);
	hipLaunchKernelGGL(k_fn_hist, dim3(nbi + nbs), dim3(256), 0, st, vk, gk, i0, n, s0, slen, nbi, S,
			   hist.as<uint32_t>());
	hipLaunchKernelGGL(k_fn_bounds, dim3(1), dim3(64), 0, st, hist.as<uint32_t>(), nbi, nbs, n, S,
			   ub.as<uint8_t>());
	hipLaunchKernelGGL(k_fn_flags, dim3(grid_for(slen, 1024, 8192)), dim3(256), 0, st, vk, gk, s0, slen,
			   ub.as<uint8_t>(), S, fl.as<int8_t>());
	mgdk_bat *C = compact_flags(fl.as<int8_t>(), slen, s0);
	if (C == nullptr)
		return nullptr;
	FnHeap h{hidx.as<uint64_t>(), hg.as<uint64_t>(), hv.as<uint64_t>(), n};
	hipLaunchKernelGGL(k_fn_heap_init, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, h, vk, gk, cnt, reversed);
	// heapify (gdk_firstn.c:93-97): internal nodes [0, n/2), deepest level first
	const BUN inner = n / 2;
	if (inner > 0) {
		int d = 63 - __builtin_clzll((unsigned long long) inner);   // level of node inner-1 ...
		for (; d >= 0; d--) {
			const BUN lo = ((BUN) 1 << d) - 1, hi = min(((BUN) 1 << (d + 1)) - 1, inner);
			if (lo >= hi)
				continue;
			hipLaunchKernelGGL(k_fn_heapify_level, dim3(grid_for(hi - lo, 256, 8192)), dim3(256), 0, st, h, lo,
					   hi);
		}
	}
	const bool cd = C->ttype == MGDK_void;
	hipLaunchKernelGGL(k_fn_replay, dim3(1), dim3(64), 0, st, h, vk, gk, cd ? nullptr : (const oid *) C->theap,
			   cd ? C->tseqbase : 0, C->count);
	if (!hip_ok(hipMemsetAsync(out.p, 0, cnt, st), "memset")) {
		mgdk_BBPunfix(C);
		return nullptr;
	}
	hipLaunchKernelGGL(k_fn_mark, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, h, out.as<int8_t>());
	mgdk_bat *res = flags_to_cands(out.as<int8_t>(), ci, s);
	mgdk_BBPunfix(C);
	return res;
}

// BATfirstn(&topn, NULL, b, s, g, n, asc, nilslast, false):
// BATfirstn_unique (gdk_firstn.c:211-572) / _with_groups (:716-1020)
mgdk_bat *
firstn_plain(mgdk_bat *b, mgdk_bat *s, mgdk_bat *g, const Cand &ci, BUN n, bool asc, bool nilslast)
{
	const BUN cnt = ci.n;
	if (n >= cnt)
		return all_cands(ci, s);
	if (g == nullptr) {
		if (b->ttype == MGDK_void) {
			// nilslast is irrelevant: all nil or none (:247-277)
			if (asc || b->tseqbase == MGDK_OID_NIL)
				return slice_cands(ci, s, 0, n, 0, 0);
			return slice_cands(ci, s, cnt - n, cnt, 0, 0);
		}
		bool sorted, revsorted, hasnil;
		BUN nnil;
		if (fn_props(b, &sorted, &revsorted, &hasnil, &nnil) < 0)
			return nullptr;
		if (sorted || revsorted) {
			// :278-356; SORTfndlast(b, nil) is the first non-nil row of an
			// ascending column and BATcount(b) of a descending one
			if (nilslast == asc && hasnil) {
				BUN pos = cnt;
				if (sorted && cands_below(ci, b->hseqbase + nnil, &pos) < 0)
					return nullptr;
				if (sorted) {
					if (asc)
						return cnt - pos < n ? slice_cands(ci, s, cnt - n, cnt, 0, 0)
								     : slice_cands(ci, s, pos, pos + n, 0, 0);
					return pos < n ? slice_cands(ci, s, 0, pos, cnt - (n - pos), cnt)
						       : slice_cands(ci, s, 0, n, 0, 0);
				}
				if (asc)
					return pos < n ? slice_cands(ci, s, 0, n, 0, 0) : slice_cands(ci, s, pos - n, pos, 0, 0);
				return cnt - pos < n ? slice_cands(ci, s, 0, n - (cnt - pos), pos, cnt)
						     : slice_cands(ci, s, pos, pos + n, 0, 0);
			}
			if (asc ? sorted : revsorted)
				return slice_cands(ci, s, 0, n, 0, 0);
			return slice_cands(ci, s, cnt - n, cnt, 0, 0);
		}
	} else if (g->ttype == MGDK_void && g->tseqbase != MGDK_OID_NIL) {
		return slice_cands(ci, s, 0, n, 0, 0);     // dense groups decide (:752-768)
	}
	Ranked r(cnt, g != nullptr);
	uint64_t gs, vs, kr, neq = 0;
	if (rank_cands(b, ci, g, asc, nilslast, r) < 0 || find_threshold(r, cnt, n, &gs, &vs, &kr, &neq) < 0)
		return nullptr;
	mgdk_bat *bn = nullptr;
	if (kr == neq) {
		// every row tied with the n-th one is in: the heap's set is determined
		if (emit_selection(r, ci, s, gs, vs, true, 0, &bn, nullptr) < 0)
			return nullptr;
		return bn;
	}
	return heap_replay(r, ci, s, n, g == nullptr && !asc, gs, vs);
}

}  // namespace

extern "C" int
mgdk_BATfirstn(mgdk_bat **topn, mgdk_bat **gids, mgdk_bat *b, mgdk_bat *s, mgdk_bat *g, mgdk_BUN n, bool asc,
	       bool nilslast, bool distinct)
{
	if (topn == nullptr) {
		seterr("BATfirstn: NULL argument");
		return -1;
	}
	*topn = nullptr;
	if (gids)
		*gids = nullptr;
	if (b == nullptr)
		return 0;
	if (!firstn_type(b->ttype) && !(b->ttype == MGDK_void && g == nullptr && gids == nullptr && !distinct)) {
		seterr("42000!BATfirstn: type %s not supported on the device path", atomname(b->ttype));
		return -1;
	}
	if (g != nullptr && (s == nullptr || g->count != s->count)) {
		seterr("BATfirstn: g requires s, aligned with it");
		return -1;
	}
	if (g != nullptr && distinct) {
		seterr("42000!BATfirstn: distinct with groups is not supported on the device path");
		return -1;
	}
	ProfScope prof("firstn");
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return -1;
	if (n == 0 || b->count == 0 || ci.n == 0) {
		*topn = mgdk_BATdense(0, 0, 0);
		if (gids)
			*gids = mgdk_BATdense(0, 0, 0);
		return (*topn && (!gids || *gids)) ? 0 : -1;
	}
	mgdk_bat *bn = nullptr, *pos = nullptr, *su = nullptr;
	int rc = -1;
	if (distinct) {
		// n complete groups of values: the n-th best DISTINCT value is the
		// threshold (found over one representative per value), then every
		// candidate ranking at or before it
		su = mgdk_BATunique(b, s);
		Cand cu;
		if (su == nullptr || cand_init(&cu, b, su) < 0)
			goto out;
		if (n >= cu.n) {
			bn = all_cands(ci, s);
		} else {
			Ranked ru(cu.n, false), ra(ci.n, false);
			uint64_t gs, vs, kr;
			if (rank_cands(b, cu, nullptr, asc, nilslast, ru) < 0 || find_threshold(ru, cu.n, n, &gs, &vs, &kr) < 0 ||
			    rank_cands(b, ci, nullptr, asc, nilslast, ra) < 0 ||
			    emit_selection(ra, ci, s, 0, vs, true, 0, &bn, nullptr) < 0)
				goto out;
		}
	} else if (gids == nullptr) {
		bn = firstn_plain(b, s, g, ci, n, asc, nilslast);
	} else if (n >= ci.n) {
		bn = all_cands(ci, s);
		if (g)
			pos = mgdk_BATdense(0, s->hseqbase, ci.n);
	} else {
		Ranked r(ci.n, g != nullptr);
		uint64_t gs, vs, kr;
		if (rank_cands(b, ci, g, asc, nilslast, r) < 0 || find_threshold(r, ci.n, n, &gs, &vs, &kr) < 0 ||
		    emit_selection(r, ci, s, gs, vs, gids != nullptr, kr, &bn, g ? &pos : nullptr) < 0)
			goto out;
	}
	if (bn == nullptr)
		goto out;
	if (gids) {
		// group ids as the reference composes them (gdk_firstn.c:1085-1110, :1223-1268)
		mgdk_bat *vals = mgdk_BATproject(bn, b), *o4 = nullptr, *g5 = nullptr, *o6 = nullptr, *g7 = nullptr,
			 *o8 = nullptr, *gp = nullptr;
		bool ok = vals != nullptr;
		SortInternal no_oidx;   // the reference sorts these temporaries too
		if (ok && g) {
			gp = mgdk_BATproject(pos, g);
			ok = gp && mgdk_BATsort(nullptr, &o4, &g5, gp, nullptr, nullptr, false, false, false) == 0 &&
			     mgdk_BATsort(nullptr, &o6, &g7, vals, o4, g5, !asc, !asc, false) == 0;
		} else if (ok) {
			ok = mgdk_BATsort(nullptr, &o6, &g7, vals, nullptr, nullptr, !asc, !asc, false) == 0;
		}
		ok = ok && mgdk_BATsort(nullptr, &o8, nullptr, o6, nullptr, nullptr, false, false, false) == 0;
		mgdk_bat *gn = ok ? mgdk_BATproject(o8, g7) : nullptr;
		mgdk_BBPunfix(vals);
		mgdk_BBPunfix(o4);
		mgdk_BBPunfix(g5);
		mgdk_BBPunfix(o6);
		mgdk_BBPunfix(g7);
		mgdk_BBPunfix(o8);
		mgdk_BBPunfix(gp);
		if (gn == nullptr)
			goto out;
		*gids = gn;
	}
	*topn = bn;
	bn = nullptr;
	rc = 0;
out:
	mgdk_BBPunfix(bn);
	mgdk_BBPunfix(pos);
	mgdk_BBPunfix(su);
	return rc;
}
