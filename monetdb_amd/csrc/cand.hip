// cand.hip -- candidate-list algebra on the MI355X: BATmergecand,
// BATintersectcand, BATdiffcand (gdk/gdk_cand.c:46, :184, :259) and
// BATnegcands (:1296).
//
// A candidate list is a sorted, duplicate-free oid sequence: a dense range
// (void BAT), a materialised oid list, or one of the compressed forms
// (cand_except / cand_mask / msk BATs, materialised first as BATunmask
// would).  The reference walks the two lists with two canditers; here
//   intersect / diff  one flag per candidate of a (is it in b? -- a range
//                     test for a dense b, a binary search otherwise), then
//                     the select path's ordered compaction (a dense result
//                     comes back void, as virtualize() makes it);
//   merge             the candidates of b that a lacks (a diff), then both
//                     sorted lists placed by merge rank: x at its index plus
//                     the number of elements of the other list below it;
//   negcands          [tseq, tseq + nr) minus the deletions inside it, as the
//                     reference builds it: a void BAT whose vheap holds
//                     ccand_t {CAND_NEGOID} and those deletions.
// Results have hseqbase 0 and the properties the reference sets (sorted,
// key, no nils; a dense result virtualised).
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

// a candidate list as the kernels see it: dense [seq, seq + n) or oids
struct CL {
	const oid *o;       // nullptr: dense
	oid seq;
	BUN n;
};

__device__ __forceinline__ oid
cl_at(const CL &c, BUN i)
{
	return c.o ? c.o[i] : c.seq + i;
}

// number of elements of c below v
__device__ __forceinline__ BUN
cl_lower(const CL &c, oid v)
{
	if (c.o == nullptr)
		return v <= c.seq ? 0 : (v - c.seq < c.n ? v - c.seq : c.n);
	BUN lo = 0, hi = c.n;
	while (lo < hi) {
		const BUN m = (lo + hi) >> 1;
		if (c.o[m] < v)
			lo = m + 1;
		else
			hi = m;
	}
	return lo;
}

__device__ __forceinline__ bool
cl_has(const CL &c, oid v)
{
	const BUN i = cl_lower(c, v);
	return i < c.n && cl_at(c, i) == v;
}

// flags[i] = (a_i in b) == keep_in
__global__ __launch_bounds__(256) void
k_cand_member(CL a, CL b, bool keep_in, int8_t *flags)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (BUN) gridDim.x * blockDim.x)
		flags[i] = cl_has(b, cl_at(a, i)) == keep_in;
}

// dst[k] = src[idx_k], idx a compaction result (dense: i0 + k)
__global__ __launch_bounds__(256) void
k_cand_gather(const oid *idx, oid i0, BUN n, const oid *src, oid *dst)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x)
		dst[k] = src[idx ? idx[k] : i0 + k];
}

// every element of x at its merge place: index + elements of y below it
__global__ __launch_bounds__(256) void
k_cand_place(CL x, CL y, oid *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < x.n; i += (BUN) gridDim.x * blockDim.x) {
		const oid v = cl_at(x, i);
		out[i + cl_lower(y, v)] = v;
	}
}

// lower bounds of two values in a sorted oid column (SORTfndfirst)
__global__ void
k_cand_bounds(const oid *o, BUN n, oid v0, oid v1, BUN *out)
{
	const oid v = threadIdx.x == 0 ? v0 : v1;
	BUN lo = 0, hi = n;
	while (lo < hi) {
		const BUN m = (lo + hi) >> 1;
		if (o[m] < v)
			lo = m + 1;
		else
			hi = m;
	}
	out[threadIdx.x] = lo;
}

__global__ __launch_bounds__(256) void
k_cand_iota(oid *dst, oid first, BUN n)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x)
		dst[k] = first + k;
}

// a candidate BAT as a CL; compressed forms materialised into *own (the
// caller releases it)
int
cl_of(const mgdk_bat *b, CL *c, mgdk_bat **own)
{
	*own = nullptr;
	if (b == nullptr) {
		seterr("candidate list is NULL");
		return -1;
	}
	if (is_complex_cand(b)) {
		if ((*own = unmask_cand(b)) == nullptr)
			return -1;
		b = *own;
	}
	if (b->ttype == MGDK_void) {
		*c = CL{nullptr, b->tseqbase, b->count};
		return 0;
	}
	if (b->ttype != MGDK_oid) {
		seterr("candidate list must have type oid");
		return -1;
	}
	*c = CL{(const oid *) b->theap, 0, b->count};
	return 0;
}

}  // namespace

// a sorted, duplicate-free oid BAT of n values: properties, and void when
// dense (virtualize, gdk_select.c:31)
// all candidates as a new candidate list (canditer_slice)
mgdk_bat *
mgdk::cand_slice(const Cand &ci)
{
	if (ci.dense)
		return mgdk_BATdense(0, ci.seq, ci.n);
	mgdk_bat *bn = newbat(0, MGDK_oid, ci.n);
	if (bn == nullptr)
		return nullptr;
	if (!hip_ok(hipMemcpyAsync(bn->theap, ci.oids, ci.n * sizeof(oid), hipMemcpyDeviceToDevice, stream()),
		    "hipMemcpyAsync") || !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	bn->count = ci.n;
	bn->tsorted = bn->tkey = bn->tnonil = 1;
	bn->trevsorted = ci.n <= 1;
	return bn;
}

mgdk_bat *
mgdk::cand_finish(mgdk_bat *bn, BUN n)
{
	bn->count = n;
	bn->tsorted = 1;
	bn->trevsorted = n <= 1;
	bn->tkey = 1;
	bn->tnil = 0;
	bn->tnonil = 1;
	bn->tseqbase = MGDK_OID_NIL;
	if (n == 0) {
		setdense(bn, 0, 0);
		return bn;
	}
	oid *h = (oid *) pinned(16);
	hipStream_t st = stream();
	if (!hip_ok(hipMemcpyAsync(h, bn->theap, 8, hipMemcpyDeviceToHost, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(h + 1, (const oid *) bn->theap + n - 1, 8, hipMemcpyDeviceToHost, st), "memcpy") ||
	    !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[1] - h[0] == n - 1)
		setdense(bn, h[0], n);
	bn->tminpos = 0;
	bn->tmaxpos = n - 1;
	return bn;
}

namespace {

// the candidates of a that are (keep_in) or are not in b, as a new list
mgdk_bat *
member(const CL &a, const CL &b, bool keep_in)
{
	hipStream_t st = stream();
	if (a.n == 0)
		return mgdk_BATdense(0, 0, 0);
	DevBuf f(a.n + 1);
	if (!f.p)
		return nullptr;
	hipLaunchKernelGGL(k_cand_member, dim3(grid_for(a.n, 256 * 8, 8192)), dim3(256), 0, st, a, b, keep_in,
			   f.as<int8_t>());
	// positions (dense a: the oids themselves) of the kept candidates
	mgdk_bat *pos = compact_flags(f.as<int8_t>(), a.n, a.o ? 0 : a.seq);
	if (pos == nullptr || a.o == nullptr)
		return pos;
	const BUN n = pos->count;
	mgdk_bat *bn = newbat(0, MGDK_oid, n);
	if (bn == nullptr) {
		mgdk_BBPunfix(pos);
		return nullptr;
	}
	if (n)
		hipLaunchKernelGGL(k_cand_gather, dim3(grid_for(n, 256 * 8, 8192)), dim3(256), 0, st,
				   pos->ttype == MGDK_void ? nullptr : (const oid *) pos->theap, pos->tseqbase, n, a.o,
				   (oid *) bn->theap);
	mgdk_BBPunfix(pos);
	return cand_finish(bn, n);
}

struct Owned {
	mgdk_bat *a = nullptr, *b = nullptr;
	~Owned()
	{
		mgdk_BBPunfix(a);
		mgdk_BBPunfix(b);
	}
};

}  // namespace

extern "C" mgdk_bat *
mgdk_BATintersectcand(mgdk_bat *a, mgdk_bat *b)
{
	CL ca, cb;
	Owned own;
	if (cl_of(a, &ca, &own.a) < 0 || cl_of(b, &cb, &own.b) < 0)
		return nullptr;
	ProfScope prof("candalgebra");
	if (ca.n == 0 || cb.n == 0)
		return mgdk_BATdense(0, 0, 0);
	if (ca.o == nullptr && cb.o == nullptr) {
		const oid lo = ca.seq > cb.seq ? ca.seq : cb.seq;
		const oid hi = ca.seq + ca.n < cb.seq + cb.n ? ca.seq + ca.n : cb.seq + cb.n;
		return mgdk_BATdense(0, hi > lo ? lo : 0, hi > lo ? hi - lo : 0);
	}
	// flag the candidates of the shorter materialised side (the result is
	// a subset of either)
	if (ca.o == nullptr || (cb.o != nullptr && cb.n < ca.n))
		return member(cb, ca, true);
	return member(ca, cb, true);
}

extern "C" mgdk_bat *
mgdk_BATdiffcand(mgdk_bat *a, mgdk_bat *b)
{
	CL ca, cb;
	Owned own;
	if (cl_of(a, &ca, &own.a) < 0 || cl_of(b, &cb, &own.b) < 0)
		return nullptr;
	ProfScope prof("candalgebra");
	if (ca.n == 0)
		return mgdk_BATdense(0, 0, 0);
	if (cb.n == 0 && ca.o == nullptr)
		return mgdk_BATdense(0, ca.seq, ca.n);
	if (ca.o == nullptr && cb.o == nullptr) {
		// a minus a range: at most two dense pieces
		const oid a0 = ca.seq, a1 = ca.seq + ca.n, b0 = cb.seq, b1 = cb.seq + cb.n;
		if (b1 <= a0 || b0 >= a1)
			return mgdk_BATdense(0, a0, ca.n);
		if (b0 <= a0)
			return b1 >= a1 ? mgdk_BATdense(0, 0, 0) : mgdk_BATdense(0, b1, a1 - b1);
		if (b1 >= a1)
			return mgdk_BATdense(0, a0, b0 - a0);
	}
	return member(ca, cb, false);
}

extern "C" mgdk_bat *
mgdk_BATmergecand(mgdk_bat *a, mgdk_bat *b)
{
	CL ca, cb;
	Owned own;
	if (cl_of(a, &ca, &own.a) < 0 || cl_of(b, &cb, &own.b) < 0)
		return nullptr;
	ProfScope prof("candalgebra");
	hipStream_t st = stream();
	if (ca.n == 0 && cb.n == 0)
		return mgdk_BATdense(0, 0, 0);
	if (ca.o == nullptr && cb.o == nullptr) {
		// overlapping or touching ranges: one range
		const oid a1 = ca.seq + ca.n, b1 = cb.seq + cb.n;
		if (ca.n == 0 || cb.n == 0 || (ca.seq <= b1 && cb.seq <= a1)) {
			const oid lo = ca.n == 0 ? cb.seq : cb.n == 0 ? ca.seq : ca.seq < cb.seq ? ca.seq : cb.seq;
			const oid hi = ca.n == 0 ? b1 : cb.n == 0 ? a1 : a1 > b1 ? a1 : b1;
			return mgdk_BATdense(0, lo, hi - lo);
		}
	}
	// b's candidates that a lacks, then both sorted lists placed by rank
	mgdk_bat *d = member(cb, ca, false);
	if (d == nullptr)
		return nullptr;
	CL cd;
	mgdk_bat *dn = nullptr;
	if (cl_of(d, &cd, &dn) < 0) {
		mgdk_BBPunfix(d);
		return nullptr;
	}
	const BUN n = ca.n + cd.n;
	mgdk_bat *bn = newbat(0, MGDK_oid, n);
	if (bn == nullptr) {
		mgdk_BBPunfix(d);
		return nullptr;
	}
	if (ca.n)
		hipLaunchKernelGGL(k_cand_place, dim3(grid_for(ca.n, 256 * 8, 8192)), dim3(256), 0, st, ca, cd,
				   (oid *) bn->theap);
	if (cd.n)
		hipLaunchKernelGGL(k_cand_place, dim3(grid_for(cd.n, 256 * 8, 8192)), dim3(256), 0, st, cd, ca,
				   (oid *) bn->theap);
	bn = cand_finish(bn, n);
	mgdk_BBPunfix(d);
	return bn;
}

extern "C" mgdk_bat *
mgdk_BATnegcands(mgdk_oid tseq, mgdk_BUN nr, mgdk_bat *odels)
{
	if (odels == nullptr || (odels->ttype != MGDK_oid && odels->ttype != MGDK_void)) {
		seterr("BATnegcands: odels must be an oid list");
		return nullptr;
	}
	ProfScope prof("candalgebra");
	mgdk_bat *bn = mgdk_BATdense(0, tseq, nr);
	if (bn == nullptr || odels->count == 0)
		return bn;
	hipStream_t st = stream();
	// the deletions inside [tseq, tseq + nr): odels[lo, hi) (SORTfndfirst)
	BUN lo, hi;
	if (odels->ttype == MGDK_void) {
		const oid s0 = odels->tseqbase, s1 = s0 + odels->count;
		auto fnd = [&](oid v) -> BUN { return v <= s0 ? 0 : v >= s1 ? odels->count : v - s0; };
		lo = fnd(tseq);
		hi = fnd(tseq + nr);
	} else {
		BUN *hb = (BUN *) pinned(16);
		BUN *db = (BUN *) meta_buf();
		hipLaunchKernelGGL(k_cand_bounds, dim3(1), dim3(2), 0, st, (const oid *) odels->theap, odels->count, tseq,
				   tseq + nr, db);
		if (!hip_ok(hipMemcpyAsync(hb, db, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		lo = hb[0];
		hi = hb[1];
	}
	if (lo == hi)
		return bn;
	if (hi - lo == nr) {
		bn->count = 0;
		return bn;
	}
	const BUN nd = hi - lo;
	Heap *h = heap_new(8 + nd * 8);
	if (h == nullptr || !hip_ok(hipMemsetAsync(h->base, 0, 8, st), "memset")) {   // ccand_t {CAND_NEGOID}
		heap_decref(h);
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	oid *dst = (oid *) ((char *) h->base + 8);
	if (odels->ttype == MGDK_void)
		hipLaunchKernelGGL(k_cand_iota, dim3(grid_for(nd, 256 * 8, 8192)), dim3(256), 0, st, dst,
				   odels->tseqbase + lo, nd);
	else if (!hip_ok(hipMemcpyAsync(dst, (const oid *) odels->theap + lo, nd * 8, hipMemcpyDeviceToDevice, st),
			 "memcpy")) {
		heap_decref(h);
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (!sync()) {
		heap_decref(h);
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	Priv *p = (Priv *) bn->priv;
	heap_decref(p->tvheap);
	p->tvheap = h;
	bn->tvheap = h->base;
	bn->tvheapsize = 8 + nd * 8;
	bn->count = nr - nd;
	bn->trevsorted = bn->count <= 1;
	return bn;
}
