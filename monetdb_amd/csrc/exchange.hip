// exchange.hip -- device-side pieces of the multi-GPU exchange steps
// (SURVEY.md §8 e): hash partitioning of a column into per-rank runs
// (the shuffle of group / join, the mergetable partitioning of
// opt_mergetable.c:1496-1885 done by value instead of by row range), lower
// bounds of (key, position) splitters in a sorted run (sample sort), and
// device-to-device copies between BAT heaps and communication buffers
// (RCCL operates on the buffers; the BATs stay in this library's heaps).
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

__device__ __forceinline__ int64_t
ival(const void *base, int w, bool uns, BUN i, bool &isnil)
{
	switch (w) {
	case 1: { int8_t v = ((const int8_t *) base)[i]; isnil = v == INT8_MIN; return v; }
	case 2: { int16_t v = ((const int16_t *) base)[i]; isnil = v == INT16_MIN; return v; }
	case 4: { int32_t v = ((const int32_t *) base)[i]; isnil = v == INT32_MIN; return v; }
	default: {
		int64_t v = ((const int64_t *) base)[i];
		isnil = uns ? (uint64_t) v == ((uint64_t) 1 << 63) : v == INT64_MIN;
		return v;
	}
	}
}

__device__ __forceinline__ uint64_t
fmix64(uint64_t x)
{
	x ^= x >> 33;
	x *= 0xff51afd7ed558ccdull;
	x ^= x >> 33;
	x *= 0xc4ceb9fe1a85ec53ull;
	return x ^ (x >> 33);
}

// destination part of every row + per-part counts (LDS histogram, one
// atomic per part per workgroup)
__global__ __launch_bounds__(256) void
k_part_dest(const void *base, int w, bool uns, BUN n, uint32_t nparts, uint32_t *dest,
	    unsigned long long *counts)
{
	__shared__ uint32_t h[256];
	h[threadIdx.x] = 0;
	__syncthreads();
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		const int64_t v = ival(base, w, uns, i, isnil);
		// the widened value's hash: equal values meet on one rank whatever
		// their storage width
		const uint32_t d = (uint32_t) __umul64hi(fmix64((uint64_t) v), nparts);
		dest[i] = d;
		atomicAdd(&h[d], 1u);
	}
	__syncthreads();
	if (threadIdx.x < nparts && h[threadIdx.x])
		atomicAdd(&counts[threadIdx.x], (unsigned long long) h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void
k_perm_to_oids(const uint32_t *perm, BUN n, oid hseq, oid *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = hseq + (perm ? perm[i] : (uint32_t) i);
}

__global__ __launch_bounds__(256) void
k_fill_dense(oid *out, BUN n, oid seq)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = seq == MGDK_OID_NIL ? MGDK_OID_NIL : seq + i;
}

// number of rows of the sorted run (k, p) lexicographically below each
// query (qk, qp): keys ascending, positions ascending among equal keys
__global__ __launch_bounds__(256) void
k_lower_bound2(const void *kb, int w, bool uns, const oid *pb, oid pseq, BUN n, const int64_t *qk,
	       const uint64_t *qp, int nq, uint64_t *out)
{
	const int q = blockIdx.x * blockDim.x + threadIdx.x;
	if (q >= nq)
		return;
	BUN lo = 0, hi = n;
	while (lo < hi) {
		const BUN mid = lo + (hi - lo) / 2;
		bool isnil;
		const int64_t k = ival(kb, w, uns, mid, isnil);
		const uint64_t p = pb ? pb[mid] : pseq + mid;
		const bool below = uns ? ((uint64_t) k < (uint64_t) qk[q] || ((uint64_t) k == (uint64_t) qk[q] && p < qp[q]))
				       : (k < qk[q] || (k == qk[q] && p < qp[q]));
		if (below)
			lo = mid + 1;
		else
			hi = mid;
	}
	out[q] = lo;
}

bool
int_type(int tt)
{
	tt = basetype(tt);
	return tt == MGDK_bte || tt == MGDK_sht || tt == MGDK_int || tt == MGDK_lng || tt == MGDK_oid;
}

}  // namespace

extern "C" int
mgdk_BATupload_device(mgdk_bat *b, const void *dev, mgdk_BUN n)
{
	if (b == nullptr || b->ttype == MGDK_void) {
		seterr("cannot upload into a void BAT");
		return -1;
	}
	Priv *p = (Priv *) b->priv;
	const size_t bytes = n * (size_t) b->twidth;
	img8_drop(b);
	if (p->theap == nullptr || p->theap->refs != 1 ||
	    p->theap->size < bytes + ((char *) b->theap - (char *) p->theap->base)) {
		Heap *h = heap_new(bytes ? bytes : 1);
		if (h == nullptr)
			return -1;
		heap_decref(p->theap);
		p->theap = h;
		p->toff = 0;
		b->theap = h->base;
	}
	if (bytes && !hip_ok(hipMemcpyAsync(b->theap, dev, bytes, hipMemcpyDeviceToDevice, stream()), "memcpy D2D"))
		return -1;
	b->count = n;
	// nothing is known about received values
	b->tsorted = b->trevsorted = b->tkey = n <= 1;
	b->tnonil = n == 0;
	b->tnil = 0;
	b->tnosorted = b->tnorevsorted = 0;
	b->tminpos = b->tmaxpos = MGDK_BUN_NONE;
	b->tunique_est = 0;
	return sync_data() ? 0 : -1;
}

extern "C" int
mgdk_BATdownload_device(const mgdk_bat *b, void *dev)
{
	if (b == nullptr) {
		seterr("NULL BAT");
		return -1;
	}
	if (b->count == 0)
		return 0;
	if (b->ttype == MGDK_void)
		hipLaunchKernelGGL(k_fill_dense, dim3(grid_for(b->count, 1024, 4096)), dim3(256), 0, stream(), (oid *) dev,
				   b->count, b->tseqbase);
	else if (!hip_ok(hipMemcpyAsync(dev, b->theap, b->count * (size_t) b->twidth, hipMemcpyDeviceToDevice, stream()),
			 "memcpy D2D"))
		return -1;
	return sync_data() ? 0 : -1;
}

extern "C" int
mgdk_BAThashpartition(mgdk_bat **order, mgdk_bat *b, int nparts, uint64_t *counts)
{
	if (b == nullptr || order == nullptr || counts == nullptr || nparts < 1 || nparts > 256) {
		seterr("BAThashpartition: bad argument");
		return -1;
	}
	if (!int_type(b->ttype) && b->ttype != MGDK_void) {
		seterr("42000!BAThashpartition: type %s not supported", atomname(b->ttype));
		return -1;
	}
	ProfScope prof("hashpartition");
	const BUN n = b->count;
	if (n >= ((BUN) 1 << 32)) {
		seterr("42000!BAThashpartition: more than 2^32 rows");
		return -1;
	}
	hipStream_t st = stream();
	// a dense (void) column partitions like its oid values
	mgdk_bat *mat = nullptr;
	const mgdk_bat *src = b;
	if (b->ttype == MGDK_void) {
		mat = newbat(b->hseqbase, MGDK_oid, n);
		if (mat == nullptr || mgdk_BATdownload_device(b, mat->theap) < 0) {
			mgdk_BBPunfix(mat);
			return -1;
		}
		mat->count = n;
		src = mat;
	}
	DevBuf dst(n * 4 + 4), dst2(n * 4 + 4), v0(n * 4 + 4), v1(n * 4 + 4), cnt(256 * 8);
	mgdk_bat *o = newbat(b->hseqbase, MGDK_oid, n);
	int rc = -1;
	uint32_t *perm = nullptr;
	unsigned long long *hc = (unsigned long long *) pinned(256 * 8);
	if (!dst.p || !dst2.p || !v0.p || !v1.p || !cnt.p || !o || !hc)
		goto out;
	if (!hip_ok(hipMemsetAsync(cnt.p, 0, 256 * 8, st), "memset"))
		goto out;
	if (n)
		hipLaunchKernelGGL(k_part_dest, dim3(grid_for(n, 2048, 4096)), dim3(256), 0, st, src->theap, src->twidth,
				   basetype(src->ttype) == MGDK_oid, n, (uint32_t) nparts, dst.as<uint32_t>(),
				   cnt.as<unsigned long long>());
	if (radix_sort_positions32(dst.as<uint32_t>(), v0.as<uint32_t>(), dst2.as<uint32_t>(), v1.as<uint32_t>(), n, 8,
				   &perm) < 0)
		goto out;
	if (n)
		hipLaunchKernelGGL(k_perm_to_oids, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, perm, n, b->hseqbase,
				   (oid *) o->theap);
	if (!hip_ok(hipMemcpyAsync(hc, cnt.p, 256 * 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		goto out;
	for (int i = 0; i < nparts; i++)
		counts[i] = hc[i];
	o->count = n;
	o->tkey = o->tnonil = 1;
	o->tsorted = o->trevsorted = n <= 1;
	*order = o;
	o = nullptr;
	rc = 0;
out:
	mgdk_BBPunfix(o);
	mgdk_BBPunfix(mat);
	return rc;
}

extern "C" int
mgdk_BATlowerbound2(const mgdk_bat *keys, const mgdk_bat *pos, const int64_t *qk, const uint64_t *qp, int nq,
		    uint64_t *out)
{
	if (keys == nullptr || nq < 0 || (nq > 0 && (!qk || !qp || !out))) {
		seterr("BATlowerbound2: bad argument");
		return -1;
	}
	if (!int_type(keys->ttype)) {
		seterr("42000!BATlowerbound2: type %s not supported", atomname(keys->ttype));
		return -1;
	}
	if (pos && pos->count != keys->count) {
		seterr("BATlowerbound2: keys and positions must be aligned");
		return -1;
	}
	if (nq == 0)
		return 0;
	hipStream_t st = stream();
	DevBuf dq((size_t) nq * 24);
	uint64_t *h = (uint64_t *) pinned((size_t) nq * 8);
	if (!dq.p || !h)
		return -1;
	int64_t *dk = dq.as<int64_t>();
	uint64_t *dp = (uint64_t *) (dk + nq), *dout = dp + nq;
	if (!hip_ok(hipMemcpyAsync(dk, qk, (size_t) nq * 8, hipMemcpyHostToDevice, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(dp, qp, (size_t) nq * 8, hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	hipLaunchKernelGGL(k_lower_bound2, dim3((nq + 255) / 256), dim3(256), 0, st, keys->theap, keys->twidth,
			   basetype(keys->ttype) == MGDK_oid, pos && pos->ttype != MGDK_void ? (const oid *) pos->theap : nullptr,
			   pos ? pos->tseqbase : 0, keys->count, dk, dp, nq, dout);
	if (!hip_ok(hipMemcpyAsync(h, dout, (size_t) nq * 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	for (int i = 0; i < nq; i++)
		out[i] = h[i];
	return 0;
}
