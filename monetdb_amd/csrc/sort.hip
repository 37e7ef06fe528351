// sort.hip -- BATsort on the MI355X (gdk/gdk_batop.c:2342, do_sort :2266-2304).
//
// For integer keys with nilslast == reverse the reference sorts with the
// stable LSD radix sort GDKrsort (gdk/gdk_rsort.c:21); stable float sorts use
// the stable merge sort.  Both produce THE stable permutation, which is what
// this stable LSD radix sort reproduces:
//   key image: order-preserving unsigned 64-bit (sign bit flipped; IEEE
//   floats folded; -0 == +0; nil placed first or last as requested; inverted
//   for descending so ties keep input order);
//   passes: 8-bit digits, only digit positions that are not constant over
//   the input (AND/OR reduction) are sorted;
//   per pass: (1) per-tile digit histogram in LDS, (2) device scan of the
//   digit-major counts, (3) stable scatter: 16 rows of 256 lanes per tile,
//   wave peer groups from 8 bit-sliced ballots, per-wave digit counts in
//   LDS, running per-digit bases -- a lane's destination is
//   tile_base[d] + run[d] + earlier waves' count of d + rank in its wave.
#include <vector>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

constexpr int SITEMS = 16;
constexpr int STILE = 256 * SITEMS;

__global__ __launch_bounds__(256) void
k_rs_hist(const uint64_t *keys, BUN n, int shift, uint32_t *hist, uint32_t nblocks)
{
	__shared__ uint32_t h[256];
	h[threadIdx.x] = 0;
	__syncthreads();
	const BUN base = (BUN) blockIdx.x * STILE;
#pragma unroll
	for (int r = 0; r < SITEMS; r++) {
		BUN i = base + r * 256 + threadIdx.x;
		if (i < n)
			atomicAdd(&h[(keys[i] >> shift) & 255], 1u);
	}
	__syncthreads();
	hist[(BUN) threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(256) void
k_rs_scatter(const uint64_t *keys, const uint32_t *vals, BUN n, int shift, const uint32_t *offs,
	     uint32_t nblocks, uint64_t *keys_out, uint32_t *vals_out)
{
	__shared__ uint32_t run[256], boff[256], wc[4][256];
	const unsigned tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	run[tid] = 0;
	boff[tid] = offs[(BUN) tid * nblocks + blockIdx.x];
	wc[0][tid] = wc[1][tid] = wc[2][tid] = wc[3][tid] = 0;
	__syncthreads();
	const uint64_t lt = lanemask_lt();
	const BUN base = (BUN) blockIdx.x * STILE;
	for (int r = 0; r < SITEMS; r++) {
		const BUN i = base + r * 256 + tid;
		const bool valid = i < n;
		uint64_t k = valid ? keys[i] : 0;
		uint32_t v = valid ? vals[i] : 0;
		uint32_t d = (uint32_t) (k >> shift) & 255;
		uint64_t peer = __ballot(valid);
#pragma unroll
		for (int b = 0; b < 8; b++) {
			uint64_t bal = __ballot((d >> b) & 1);
			peer &= ((d >> b) & 1) ? bal : ~bal;
		}
		const uint32_t rank = (uint32_t) __popcll(peer & lt);
		if (valid && (peer >> lane) == 1)   // highest lane of its peer group
			wc[wave][d] = (uint32_t) __popcll(peer);
		__syncthreads();
		if (valid) {
			uint32_t pos = boff[d] + run[d] + rank;
			for (unsigned w = 0; w < wave; w++)
				pos += wc[w][d];
			keys_out[pos] = k;
			vals_out[pos] = v;
		}
		__syncthreads();
		run[tid] += wc[0][tid] + wc[1][tid] + wc[2][tid] + wc[3][tid];
		wc[0][tid] = wc[1][tid] = wc[2][tid] = wc[3][tid] = 0;
		__syncthreads();
	}
}

__global__ __launch_bounds__(256) void
k_andor(const uint64_t *keys, BUN n, unsigned long long *out)
{
	unsigned long long a = ~0ull, o = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		a &= keys[i];
		o |= keys[i];
	}
	for (int s = 32; s > 0; s >>= 1) {
		a &= __shfl_xor(a, s);
		o |= __shfl_xor(o, s);
	}
	if (__lane_id() == 0) {
		atomicAnd(&out[0], a);
		atomicOr(&out[1], o);
	}
}

// key image of row p
template <typename T>
__device__ __forceinline__ uint64_t
keyimg(T v, bool reverse, bool nilslast)
{
	uint64_t u;
	bool isnil;
	if constexpr (sizeof(T) == 4 && (T) 0.5 != 0) {          // float
		isnil = v != v;
		float f = v == 0 ? 0.0f : v;
		uint32_t b = __float_as_uint(f);
		b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
		u = (uint64_t) b << 32;
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
		u = (uint64_t) (int64_t) v ^ (1ull << 63);
	}
	if (reverse)
		u = ~u;
	if (isnil)
		u = nilslast ? ~0ull : 0ull;
	return u;
}

template <typename T>
__global__ __launch_bounds__(256) void
k_keys(const T *col, BUN n, bool reverse, bool nilslast, uint64_t *keys, uint32_t *idx)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		keys[i] = keyimg<T>(col[i], reverse, nilslast);
		idx[i] = (uint32_t) i;
	}
}

template <typename T>
__global__ __launch_bounds__(256) void
k_gather_sorted(const T *col, const uint32_t *idx, BUN n, oid hseq, T *sorted, oid *order)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		uint32_t j = idx[i];
		if (sorted)
			sorted[i] = col[j];
		if (order)
			order[i] = hseq + j;
	}
}

__global__ __launch_bounds__(256) void
k_newgrp(const uint64_t *keys, BUN n, uint8_t *flag)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		flag[i] = i > 0 && keys[i] != keys[i - 1];
}

__global__ __launch_bounds__(256) void
k_gid(const uint64_t *excl, const uint8_t *flag, BUN n, oid *gid)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		gid[i] = excl[i] + flag[i];
}

template <typename T>
void
launch_keys(const mgdk_bat *b, bool reverse, bool nilslast, uint64_t *keys, uint32_t *idx)
{
	hipLaunchKernelGGL((k_keys<T>), dim3(grid_for(b->count, 1024, 8192)), dim3(256), 0, stream(),
			   (const T *) b->theap, b->count, reverse, nilslast, keys, idx);
}

template <typename T>
void
launch_gather(const mgdk_bat *b, const uint32_t *idx, void *sorted, oid *order)
{
	hipLaunchKernelGGL((k_gather_sorted<T>), dim3(grid_for(b->count, 1024, 8192)), dim3(256), 0, stream(),
			   (const T *) b->theap, idx, b->count, b->hseqbase, (T *) sorted, order);
}

}  // namespace

namespace mgdk {

int
radix_sort_pairs(uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt, BUN n, int bits,
		 uint64_t **keys_out, uint32_t **vals_out)
{
	*keys_out = keys;
	*vals_out = vals;
	if (n <= 1)
		return 0;
	hipStream_t st = stream();
	unsigned long long *ao = (unsigned long long *) meta_buf();
	unsigned long long init[2] = {~0ull, 0ull};
	if (!hip_ok(hipMemcpyAsync(ao, init, 16, hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	hipLaunchKernelGGL(k_andor, dim3(grid_for(n, 4096, 2048)), dim3(256), 0, st, keys, n, ao);
	unsigned long long *h = (unsigned long long *) pinned(16);
	if (!hip_ok(hipMemcpyAsync(h, ao, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	const uint64_t diff = h[0] ^ h[1];
	const uint32_t nblocks = (uint32_t) ((n + STILE - 1) / STILE);
	DevBuf hist((size_t) 256 * nblocks * 4), offs((size_t) 256 * nblocks * 4);
	if (!hist.p || !offs.p)
		return -1;
	uint64_t *kin = keys, *kout = keys_alt;
	uint32_t *vin = vals, *vout = vals_alt;
	for (int shift = 0; shift < bits; shift += 8) {
		if (((diff >> shift) & 255) == 0)
			continue;   // digit constant over all keys: identity pass
		hipLaunchKernelGGL(k_rs_hist, dim3(nblocks), dim3(256), 0, st, kin, n, shift, hist.as<uint32_t>(), nblocks);
		if (exclusive_scan(hist.as<uint32_t>(), offs.as<uint32_t>(), (BUN) 256 * nblocks, nullptr) < 0)
			return -1;
		hipLaunchKernelGGL(k_rs_scatter, dim3(nblocks), dim3(256), 0, st, kin, vin, n, shift, offs.as<uint32_t>(),
				   nblocks, kout, vout);
		std::swap(kin, kout);
		std::swap(vin, vout);
	}
	if (!sync())
		return -1;
	*keys_out = kin;
	*vals_out = vin;
	return 0;
}

}  // namespace mgdk

extern "C" int
mgdk_BATsort(mgdk_bat **sorted, mgdk_bat **order, mgdk_bat **groups, mgdk_bat *b, mgdk_bat *o, mgdk_bat *g,
	     bool reverse, bool nilslast, bool stable)
{
	if (b == nullptr) {
		seterr("b must exist\n");
		return -1;
	}
	if (stable && reverse != nilslast) {
		seterr("stable sort cannot have reverse != nilslast\n");
		return -1;
	}
	if (o != nullptr || g != nullptr) {
		seterr("42000!BATsort: sub-sorting (o/g) is not supported on the device path");
		return -1;
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
		DevBuf k0(n * 8), k1(n * 8), v0(n * 4), v1(n * 4);
		if (!k0.p || !k1.p || !v0.p || !v1.p)
			return -1;
		switch (tt) {
		case MGDK_bte: launch_keys<int8_t>(b, reverse, nilslast, k0.as<uint64_t>(), v0.as<uint32_t>()); break;
		case MGDK_sht: launch_keys<int16_t>(b, reverse, nilslast, k0.as<uint64_t>(), v0.as<uint32_t>()); break;
		case MGDK_int: launch_keys<int32_t>(b, reverse, nilslast, k0.as<uint64_t>(), v0.as<uint32_t>()); break;
		case MGDK_lng: launch_keys<int64_t>(b, reverse, nilslast, k0.as<uint64_t>(), v0.as<uint32_t>()); break;
		case MGDK_oid: launch_keys<uint64_t>(b, reverse, nilslast, k0.as<uint64_t>(), v0.as<uint32_t>()); break;
		case MGDK_flt: launch_keys<float>(b, reverse, nilslast, k0.as<uint64_t>(), v0.as<uint32_t>()); break;
		case MGDK_dbl: launch_keys<double>(b, reverse, nilslast, k0.as<uint64_t>(), v0.as<uint32_t>()); break;
		}
		uint64_t *ks;
		uint32_t *vs;
		if (radix_sort_pairs(k0.as<uint64_t>(), v0.as<uint32_t>(), k1.as<uint64_t>(), v1.as<uint32_t>(), n, 64,
				     &ks, &vs) < 0)
			return -1;
		sn = sorted ? newbat(b->hseqbase, b->ttype, n) : nullptr;
		on = order ? newbat(b->hseqbase, MGDK_oid, n) : nullptr;
		if ((sorted && !sn) || (order && !on))
			goto fail;
		switch (b->twidth) {
		case 1: launch_gather<int8_t>(b, vs, sn ? sn->theap : nullptr, on ? (oid *) on->theap : nullptr); break;
		case 2: launch_gather<int16_t>(b, vs, sn ? sn->theap : nullptr, on ? (oid *) on->theap : nullptr); break;
		case 4: launch_gather<int32_t>(b, vs, sn ? sn->theap : nullptr, on ? (oid *) on->theap : nullptr); break;
		default: launch_gather<int64_t>(b, vs, sn ? sn->theap : nullptr, on ? (oid *) on->theap : nullptr); break;
		}
		if (groups) {
			gn = newbat(b->hseqbase, MGDK_oid, n);
			DevBuf fl(n), ex(n * 8);
			if (!gn || !fl.p || !ex.p)
				goto fail;
			hipLaunchKernelGGL(k_newgrp, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, stream(), ks, n,
					   fl.as<uint8_t>());
			uint64_t tot = 0;
			if (exclusive_scan(fl.as<uint8_t>(), ex.as<uint64_t>(), n, &tot) < 0)
				goto fail;
			hipLaunchKernelGGL(k_gid, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, stream(), ex.as<uint64_t>(),
					   fl.as<uint8_t>(), n, (oid *) gn->theap);
			gn->count = n;
			gn->tsorted = 1;
			gn->trevsorted = tot == 0;
			gn->tkey = tot + 1 == n || n <= 1;
			gn->tnonil = 1;
		}
		if (!sync())
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
			on->tsorted = on->trevsorted = n <= 1;
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
