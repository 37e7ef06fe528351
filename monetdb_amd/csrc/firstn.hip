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
//   * plain top-n (gids NULL): the rows strictly better than the last value
//     plus the FIRST (in candidate order) of the tied rows.  The reference
//     returns the tied rows its heap happened to keep (heap-order
//     dependent; SQL leaves the choice open); on sorted inputs it also
//     returns the first ones.
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
		isnil = (uint64_t) v == ((uint64_t) 1 << 63);
		u = (uint64_t) v;
	} else {
		isnil = v == NilOf<T>::v();
		u = (uint64_t) (int64_t) v ^ (1ull << 63);
	}
	if (!asc)
		u = ~u;
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

// radix selection of the k-th smallest (1-based) key; returns the key and
// the rank k' of the wanted element among the keys equal to it
int
rsel(const uint64_t *keys, BUN n, uint64_t k, const uint64_t *gk, uint64_t gstar, uint64_t *val, uint64_t *krem)
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
find_threshold(const Ranked &r, BUN cnt, BUN n, uint64_t *gstar, uint64_t *vstar, uint64_t *krem)
{
	uint64_t k = n;
	*gstar = 0;
	if (r.hasg) {
		uint64_t kg;
		if (rsel(r.g(), cnt, k, nullptr, 0, gstar, &kg) < 0)
			return -1;
		k = kg;             // rank inside the selected group
	}
	return rsel(r.vk.as<uint64_t>(), cnt, k, r.g(), *gstar, vstar, krem);
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
	if (!firstn_type(b->ttype)) {
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
