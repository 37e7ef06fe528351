// prodminmax.hip -- whole-column extremes and products of gdk_aggr.c, and
// BATunmask of gdk_cand.c, on the MI355X:
//   BATmin / BATmax / BATmin_skipnil / BATmax_skipnil (gdk_aggr.c:3570-3844):
//     the value at the column's smallest / largest position as the reference
//     finds it -- a cached tminpos / tmaxpos first, then for an ordered
//     column its end (past the nils), else do_groupmin / do_groupmax over
//     every row (:3247-3485: the FIRST row holding the extreme; without
//     skipnil the first nil); the position is cached in the descriptor as the
//     reference caches it.  The scan is one device pass: each lane keeps its
//     (key, first position) and its first nil, a workgroup reduces them, one
//     workgroup combines the partials.  Keys: the integers as 128-bit
//     images, flt / dbl as the order- and equality-preserving integer image
//     of dbl_cmp (-0.0 == +0.0, so a tie keeps the first row and its bits),
//     str by strcmp over the heap (nil "\200" detected, never compared).
//   BATprod / BATgroupprod (doprod :1340-1548): the reference's recurrence
//     replayed in candidate order per group (rows grouped by the stable
//     counting sort group_rows), all groups at once -- one lane each -- with
//     its three macro shapes kept apart because they treat nils and the
//     "seen" reset differently (AGGR_PROD: a nil before the group's first
//     value is forgotten when that value arrives; AGGR_PROD_HGE marks a group
//     seen on any row; AGGR_PROD_FLOAT as AGGR_PROD with the float overflow
//     test); integer overflow is the exact test of MULI4_WITH_CHECK /
//     HGEMUL_CHECK (|product| <= the type's max).  The whole-column integer
//     BATprod takes a parallel form: the product's magnitude only grows until
//     a zero (a nonzero integer has |v| >= 1), so the reference raises its
//     overflow iff the saturated product of |v| over the rows before the
//     first zero (and before the row that makes the product nil) exceeds the
//     max -- a reduction of (first zero, first nil cut, saturated magnitude,
//     sign parity), exact, instead of one lane's dependent chain.
//   BATunmask (gdk_cand.c:1464): a msk BAT or a cand_mask list as the oid
//     list of its set bits -- or, for a mask list with more than half its
//     bits set, the negative (cand_except) list the reference makes.
#include "mgdk_internal.h"

#include <cfloat>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#pragma clang fp contract(off)

using namespace mgdk;

namespace {

constexpr unsigned long long NOPOS = ~0ull;

// ---- extremes -----------------------------------------------------------

struct MMPart {
	hge key;
	unsigned long long pos;    // first row holding the best key (NOPOS: none)
	unsigned long long nil;    // first nil row (NOPOS: none)
};

// the order-preserving integer image of a float under dbl_cmp (nil excluded)
__device__ __forceinline__ hge
fkey(double d)
{
	if (d == 0)
		return 0;
	long long s;
	__builtin_memcpy(&s, &d, 8);
	return (hge) (s < 0 ? s ^ INT64_MAX : s);
}

template <typename T>
__device__ __forceinline__ hge
mm_key(T v)
{
	return (hge) v;
}
template <>
__device__ __forceinline__ hge
mm_key<float>(float v)
{
	return fkey((double) v);
}
template <>
__device__ __forceinline__ hge
mm_key<double>(double v)
{
	return fkey(v);
}

template <bool DOMAX>
__device__ __forceinline__ bool
mm_better(const MMPart &a, const MMPart &b)   // a before b
{
	if (a.pos == NOPOS)
		return false;
	if (b.pos == NOPOS)
		return true;
	if (a.key != b.key)
		return DOMAX ? a.key > b.key : a.key < b.key;
	return a.pos < b.pos;
}

template <bool DOMAX>
__device__ __forceinline__ MMPart
mm_comb(MMPart a, const MMPart &b)
{
	MMPart r = mm_better<DOMAX>(b, a) ? b : a;
	r.nil = a.nil < b.nil ? a.nil : b.nil;
	return r;
}

template <bool DOMAX>
__device__ MMPart
mm_block_reduce(MMPart x)
{
	__shared__ MMPart sh[16];
	const unsigned lane = __lane_id(), w = threadIdx.x >> 6;
	for (int o = 32; o > 0; o >>= 1) {
		MMPart y;
		y.key = (hge) __shfl_xor((long long) (x.key >> 64), o) << 64 |
			(hge) (unsigned long long) __shfl_xor((long long) x.key, o);
		y.pos = __shfl_xor(x.pos, o);
		y.nil = __shfl_xor(x.nil, o);
		x = mm_comb<DOMAX>(x, y);
	}
	if (lane == 0)
		sh[w] = x;
	__syncthreads();
	if (threadIdx.x == 0)
		for (unsigned k = 1; k < blockDim.x / 64; k++)
			x = mm_comb<DOMAX>(x, sh[k]);
	return x;
}

// each workgroup's partial of rows [0, n); T the value type
template <typename T, bool DOMAX>
__global__ __launch_bounds__(256) void
k_mm_part(const T *v, BUN n, MMPart *part)
{
	MMPart x{0, NOPOS, NOPOS};
	constexpr int U = 8;
	const BUN stride = (BUN) gridDim.x * blockDim.x * U;
	for (BUN i0 = (BUN) blockIdx.x * blockDim.x * U + threadIdx.x; i0 < n; i0 += stride) {
		T y[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x;
			y[u] = v[i < n ? i : 0];
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * blockDim.x;
			if (i >= n)
				continue;
			if (is_nil(y[u])) {
				if (x.nil == NOPOS)
					x.nil = i;
				continue;
			}
			const hge k = mm_key(y[u]);
			if (x.pos == NOPOS || (DOMAX ? k > x.key : k < x.key)) {
				x.key = k;
				x.pos = i;
			}
		}
	}
	x = mm_block_reduce<DOMAX>(x);
	if (threadIdx.x == 0)
		part[blockIdx.x] = x;
}

// str: strcmp of the heap strings (1 / 2-byte offsets past GDK_VAROFFSET)
__device__ __forceinline__ const unsigned char *
str_at(const void *offs, int w, const char *vh, BUN p)
{
	uint64_t o;
	switch (w) {
	case 1: o = (uint64_t) ((const uint8_t *) offs)[p] + 8192; break;
	case 2: o = (uint64_t) ((const uint16_t *) offs)[p] + 8192; break;
	case 4: o = ((const uint32_t *) offs)[p]; break;
	default: o = ((const uint64_t *) offs)[p]; break;
	}
	return (const unsigned char *) vh + o;
}

__device__ __forceinline__ int
dstrcmp(const unsigned char *a, const unsigned char *b)
{
	for (;; a++, b++) {
		if (*a != *b)
			return *a < *b ? -1 : 1;
		if (*a == 0)
			return 0;
	}
}

__device__ __forceinline__ bool
str_nil(const unsigned char *s)
{
	return s[0] == 0x80 && s[1] == 0;
}

template <bool DOMAX>
__global__ __launch_bounds__(256) void
k_mm_str(const void *offs, int w, const char *vh, BUN n, MMPart *part)
{
	MMPart x{0, NOPOS, NOPOS};
	const unsigned char *best = nullptr;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const unsigned char *s = str_at(offs, w, vh, i);
		if (str_nil(s)) {
			if (x.nil == NOPOS)
				x.nil = i;
			continue;
		}
		if (best == nullptr || (DOMAX ? dstrcmp(s, best) > 0 : dstrcmp(s, best) < 0)) {
			best = s;
			x.pos = i;
		}
	}
	// lanes compare their candidates by position through LDS strings: the
	// reduction re-reads the heap (rank keys are positions, compared by
	// the strings they point at)
	__shared__ unsigned long long sp[256], sn[256];
	sp[threadIdx.x] = x.pos;
	sn[threadIdx.x] = x.nil;
	__syncthreads();
	if (threadIdx.x == 0) {
		unsigned long long bp = NOPOS, bn = NOPOS;
		const unsigned char *bs = nullptr;
		for (unsigned t = 0; t < blockDim.x; t++) {
			bn = sn[t] < bn ? sn[t] : bn;
			if (sp[t] == NOPOS)
				continue;
			const unsigned char *s = str_at(offs, w, vh, sp[t]);
			const int c = bs ? dstrcmp(s, bs) : 0;
			if (bs == nullptr || (DOMAX ? c > 0 : c < 0) || (c == 0 && sp[t] < bp)) {
				bs = s;
				bp = sp[t];
			}
		}
		part[blockIdx.x] = MMPart{0, bp, bn};
	}
}

template <bool DOMAX>
__global__ void
k_mm_str_final(const void *offs, int w, const char *vh, const MMPart *part, unsigned np, MMPart *out)
{
	unsigned long long bp = NOPOS, bn = NOPOS;
	const unsigned char *bs = nullptr;
	for (unsigned t = 0; t < np; t++) {
		bn = part[t].nil < bn ? part[t].nil : bn;
		if (part[t].pos == NOPOS)
			continue;
		const unsigned char *s = str_at(offs, w, vh, part[t].pos);
		const int c = bs ? dstrcmp(s, bs) : 0;
		if (bs == nullptr || (DOMAX ? c > 0 : c < 0) || (c == 0 && part[t].pos < bp)) {
			bs = s;
			bp = part[t].pos;
		}
	}
	*out = MMPart{0, bp, bn};
}

template <bool DOMAX>
__global__ __launch_bounds__(256) void
k_mm_final(const MMPart *part, unsigned np, MMPart *out)
{
	MMPart x{0, NOPOS, NOPOS};
	for (unsigned k = threadIdx.x; k < np; k += blockDim.x)
		x = mm_comb<DOMAX>(x, part[k]);
	x = mm_block_reduce<DOMAX>(x);
	if (threadIdx.x == 0)
		*out = x;
}

bool
linear_type(int t)
{
	switch (t) {
	case MGDK_void: case MGDK_bit: case MGDK_bte: case MGDK_sht: case MGDK_int: case MGDK_date: case MGDK_lng:
	case MGDK_oid: case MGDK_daytime: case MGDK_timestamp: case MGDK_hge: case MGDK_flt: case MGDK_dbl:
	case MGDK_str:
		return true;
	}
	return false;
}

// host copy of the bytes at position p (w bytes); str: the string
bool
read_at(const mgdk_bat *b, BUN p, std::string &out)
{
	hipStream_t st = stream();
	char *h = (char *) pinned(64);
	if (b->ttype == MGDK_str) {
		if (!hip_ok(hipMemcpyAsync(h, (const char *) b->theap + p * b->twidth, b->twidth, hipMemcpyDeviceToHost, st),
			    "memcpy") || !sync())
			return false;
		uint64_t o = 0;
		memcpy(&o, h, b->twidth);
		if (b->twidth <= 2)
			o += 8192;
		// strings are NUL terminated: copy in 64-byte steps until the NUL
		out.clear();
		for (;;) {
			const size_t k = b->tvheapsize > o ? (b->tvheapsize - o < 64 ? b->tvheapsize - o : 64) : 0;
			if (k == 0)
				return true;
			if (!hip_ok(hipMemcpyAsync(h, (const char *) b->tvheap + o, k, hipMemcpyDeviceToHost, st), "memcpy") ||
			    !sync())
				return false;
			const void *z = memchr(h, 0, k);
			if (z) {
				out.append(h, (const char *) z - h);
				return true;
			}
			out.append(h, k);
			o += k;
		}
	}
	if (!hip_ok(hipMemcpyAsync(h, (const char *) b->theap + p * b->twidth, b->twidth, hipMemcpyDeviceToHost, st),
		    "memcpy") || !sync())
		return false;
	out.assign(h, b->twidth);
	return true;
}

// the type's nil as bytes (str: "\200")
std::string
nil_bytes(int t, int w)
{
	std::string s(w > 0 ? (size_t) w : 1, '\0');
	switch (basetype(t)) {
	case MGDK_bte: s[0] = (char) 0x80; break;
	case MGDK_sht: { const int16_t v = INT16_MIN; memcpy(&s[0], &v, 2); break; }
	case MGDK_int: { const int32_t v = INT32_MIN; memcpy(&s[0], &v, 4); break; }
	case MGDK_lng: case MGDK_oid: { const int64_t v = INT64_MIN; memcpy(&s[0], &v, 8); break; }
	case MGDK_hge: { const hge v = (hge) ((uhge) 1 << 127); memcpy(&s[0], &v, 16); break; }
	case MGDK_flt: { const float v = __builtin_nanf(""); memcpy(&s[0], &v, 4); break; }
	case MGDK_dbl: { const double v = __builtin_nan(""); memcpy(&s[0], &v, 8); break; }
	case MGDK_str: s = "\x80"; break;
	default: break;
	}
	return s;
}

bool
bytes_nil(int t, const std::string &x)
{
	switch (basetype(t)) {
	case MGDK_flt: { float f; memcpy(&f, x.data(), 4); return f != f; }
	case MGDK_dbl: { double f; memcpy(&f, x.data(), 8); return f != f; }
	case MGDK_str: return x == "\x80";
	default: return x == nil_bytes(t, (int) x.size());
	}
}

// first position of a non-nil value of a sorted column (nils sort first),
// or of the first nil of a reverse-sorted one (nils sort last): binary
// search on the device over the nil predicate
template <typename T>
__global__ void
k_nil_bound(const T *v, BUN n, bool asc, unsigned long long *out)
{
	BUN lo = 0, hi = n;
	while (lo < hi) {
		const BUN m = lo + (hi - lo) / 2;
		const bool nil = is_nil(v[m]);
		if (asc ? nil : !nil)
			lo = m + 1;
		else
			hi = m;
	}
	*out = lo;
}

__global__ void
k_nil_bound_str(const void *offs, int w, const char *vh, BUN n, bool asc, unsigned long long *out)
{
	BUN lo = 0, hi = n;
	while (lo < hi) {
		const BUN m = lo + (hi - lo) / 2;
		const bool nil = str_nil(str_at(offs, w, vh, m));
		if (asc ? nil : !nil)
			lo = m + 1;
		else
			hi = m;
	}
	*out = lo;
}

int
nil_bound(const mgdk_bat *b, bool asc, BUN *res)
{
	DevBuf o(16);
	if (!o.p)
		return -1;
	hipStream_t st = stream();
	unsigned long long *d = o.as<unsigned long long>();
	const BUN n = b->count;
	if (b->ttype == MGDK_str) {
		hipLaunchKernelGGL(k_nil_bound_str, dim3(1), dim3(1), 0, st, (const void *) b->theap, (int) b->twidth,
				   (const char *) b->tvheap, n, asc, d);
	} else {
		switch (basetype(b->ttype)) {
		case MGDK_bte: hipLaunchKernelGGL(k_nil_bound<int8_t>, dim3(1), dim3(1), 0, st, (const int8_t *) b->theap, n, asc, d); break;
		case MGDK_sht: hipLaunchKernelGGL(k_nil_bound<int16_t>, dim3(1), dim3(1), 0, st, (const int16_t *) b->theap, n, asc, d); break;
		case MGDK_int: hipLaunchKernelGGL(k_nil_bound<int32_t>, dim3(1), dim3(1), 0, st, (const int32_t *) b->theap, n, asc, d); break;
		case MGDK_hge: hipLaunchKernelGGL(k_nil_bound<hge>, dim3(1), dim3(1), 0, st, (const hge *) b->theap, n, asc, d); break;
		case MGDK_flt: hipLaunchKernelGGL(k_nil_bound<float>, dim3(1), dim3(1), 0, st, (const float *) b->theap, n, asc, d); break;
		case MGDK_dbl: hipLaunchKernelGGL(k_nil_bound<double>, dim3(1), dim3(1), 0, st, (const double *) b->theap, n, asc, d); break;
		default: hipLaunchKernelGGL(k_nil_bound<int64_t>, dim3(1), dim3(1), 0, st, (const int64_t *) b->theap, n, asc, d); break;
		}
	}
	unsigned long long *h = (unsigned long long *) pinned(16);
	if (!hip_ok(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	*res = h[0];
	return 0;
}

template <bool DOMAX>
int
mm_scan(const mgdk_bat *b, MMPart *res)
{
	hipStream_t st = stream();
	const BUN n = b->count;
	const unsigned np = grid_for(n, 256 * 8, 2048);
	DevBuf part(np * sizeof(MMPart) + 64), out(sizeof(MMPart) + 16);
	if (!part.p || !out.p)
		return -1;
	MMPart *pp = part.as<MMPart>();
	if (b->ttype == MGDK_str) {
		const unsigned g = grid_for(n, 256 * 4, 1024);
		hipLaunchKernelGGL(k_mm_str<DOMAX>, dim3(g), dim3(256), 0, st, (const void *) b->theap, (int) b->twidth,
				   (const char *) b->tvheap, n, pp);
		hipLaunchKernelGGL(k_mm_str_final<DOMAX>, dim3(1), dim3(1), 0, st, (const void *) b->theap, (int) b->twidth,
				   (const char *) b->tvheap, (const MMPart *) pp, g, out.as<MMPart>());
	} else {
#define MMP(T) hipLaunchKernelGGL((k_mm_part<T, DOMAX>), dim3(np), dim3(256), 0, st, (const T *) b->theap, n, pp)
		switch (basetype(b->ttype)) {
		case MGDK_bte: MMP(int8_t); break;
		case MGDK_sht: MMP(int16_t); break;
		case MGDK_int: MMP(int32_t); break;
		case MGDK_hge: MMP(hge); break;
		case MGDK_flt: MMP(float); break;
		case MGDK_dbl: MMP(double); break;
		default: MMP(int64_t); break;
		}
#undef MMP
		hipLaunchKernelGGL(k_mm_final<DOMAX>, dim3(1), dim3(256), 0, st, (const MMPart *) pp, np, out.as<MMPart>());
	}
	MMPart *h = (MMPart *) pinned(64);
	if (!hip_ok(hipMemcpyAsync(h, out.p, sizeof(MMPart), hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	*res = *h;
	return 0;
}

// BATmin_skipnil (gdk_aggr.c:3570) / BATmax_skipnil (:3727)
template <bool DOMAX>
void *
minmax_skipnil(mgdk_bat *b, void *aggr, bool skipnil)
{
	if (b == nullptr) {
		seterr("BAT%s: b must exist", DOMAX ? "max" : "min");
		return nullptr;
	}
	if (!linear_type(b->ttype)) {
		seterr("non-linear type");
		return nullptr;
	}
	if (b->ttype == MGDK_str && aggr != nullptr) {
		seterr("BAT%s: a str result needs aggr == NULL (the value is allocated)", DOMAX ? "max" : "min");
		return nullptr;
	}
	ProfScope prof(DOMAX ? "max" : "min");
	const BUN n = b->count;
	const int w = b->ttype == MGDK_void ? 8 : (int) b->twidth;
	std::string val;
	BUN pos = (BUN) NOPOS;
	const BUN cached = DOMAX ? b->tmaxpos : b->tminpos;
	if (n == 0) {
		val = nil_bytes(b->ttype, w);
	} else if (b->ttype == MGDK_void) {
		// a dense column: ordered, its values the sequence (nil: every value)
		if (b->tseqbase == MGDK_OID_NIL) {
			val = nil_bytes(MGDK_oid, 8);
		} else {
			const oid v = b->tseqbase + (DOMAX ? n - 1 : 0);
			val.assign((const char *) &v, 8);
		}
	} else if (cached != MGDK_BUN_NONE && cached < n) {
		pos = cached;
	} else {
		const bool asc = mgdk_BATordered(b);
		const bool desc = !asc && mgdk_BATordered_rev(b);
		if (asc || desc) {
			if (!DOMAX) {
				if (skipnil && !b->tnonil) {
					BUN q;
					if (nil_bound(b, asc, &q) < 0)
						return nullptr;
					// sorted: the first non-nil (none: nil); reverse sorted:
					// the row before the first nil (none before it: nil)
					pos = asc ? (q == n ? (BUN) NOPOS : q) : (q == 0 ? (BUN) NOPOS : q - 1);
				} else {
					pos = asc ? 0 : n - 1;
				}
			} else {
				pos = asc ? n - 1 : 0;
				if (skipnil && !b->tnonil) {
					std::string x;
					if (!read_at(b, pos, x))
						return nullptr;
					if (bytes_nil(b->ttype, x))
						pos = (BUN) NOPOS;       // no non-nil values
				}
			}
		} else {
			MMPart r;
			if (mm_scan<DOMAX>(b, &r) < 0)
				return nullptr;
			pos = !skipnil && r.nil != NOPOS ? r.nil : r.pos;
		}
		if (pos != (BUN) NOPOS) {
			if (DOMAX)
				b->tmaxpos = pos;
			else
				b->tminpos = pos;
		}
	}
	if (pos != (BUN) NOPOS) {
		if (!read_at(b, pos, val))
			return nullptr;
	} else if (val.empty() && n > 0 && b->ttype != MGDK_void) {
		val = nil_bytes(b->ttype, w);
	}
	if (aggr == nullptr) {
		const size_t sz = b->ttype == MGDK_str ? val.size() + 1 : val.size();
		aggr = malloc(sz ? sz : 1);
		if (aggr == nullptr) {
			seterr("malloc");
			return nullptr;
		}
		memcpy(aggr, val.data(), val.size());
		if (b->ttype == MGDK_str)
			((char *) aggr)[val.size()] = 0;
	} else {
		memcpy(aggr, val.data(), val.size());
	}
	return aggr;
}

// ---- products -----------------------------------------------------------

// the reference's three macro shapes
enum { PK_INT = 0, PK_HGE = 1, PK_FLOAT = 2 };

struct ProdArgs {
	oid off;
	const uint32_t *perm;          // rows grouped by group (nullptr: rows in order)
	const uint64_t *start;         // group k: [start[k], start[k+1]) (nullptr: one group of n)
	BUN ngrp, n;
	bool skip_nils, nil_if_empty;
	void *res;
	uint32_t *flags;               // bit 0 overflow, bit 1 a nil result
};

template <typename T> struct Wider;
template <> struct Wider<int8_t> { typedef int16_t T; };
template <> struct Wider<int16_t> { typedef int32_t T; };
template <> struct Wider<int32_t> { typedef int64_t T; };
template <> struct Wider<int64_t> { typedef hge T; };

template <typename T> __device__ __forceinline__ T tmax();
template <> __device__ __forceinline__ int8_t tmax<int8_t>() { return INT8_MAX; }
template <> __device__ __forceinline__ int16_t tmax<int16_t>() { return INT16_MAX; }
template <> __device__ __forceinline__ int32_t tmax<int32_t>() { return INT32_MAX; }
template <> __device__ __forceinline__ int64_t tmax<int64_t>() { return INT64_MAX; }
template <> __device__ __forceinline__ float tmax<float>() { return FLT_MAX; }
template <> __device__ __forceinline__ double tmax<double>() { return DBL_MAX; }

template <typename T> __device__ __forceinline__ T pnil() { return NilOf<T>::v(); }
template <> __device__ __forceinline__ float pnil<float>() { return __builtin_nanf(""); }
template <> __device__ __forceinline__ double pnil<double>() { return __builtin_nan(""); }

__device__ __forceinline__ float
h2f(hge v)
{
	if (v >= (hge) INT64_MIN && v <= (hge) INT64_MAX)
		return (float) (long long) v;
	const bool neg = v < 0;
	const uhge u = neg ? (uhge) 0 - (uhge) v : (uhge) v;
	const unsigned long long hi = (unsigned long long) (u >> 64);
	const int shift = 64 - __builtin_clzll(hi);
	unsigned long long top = (unsigned long long) (u >> shift);
	if (u & (((uhge) 1 << shift) - 1))
		top |= 1;
	const float f = ldexpf((float) top, shift);
	return neg ? -f : f;
}

// the value as the float operand of AGGR_PROD_FLOAT's arithmetic
template <typename F, typename T>
__device__ __forceinline__ F
as_float(T v)
{
	return (F) v;
}
template <>
__device__ __forceinline__ float
as_float<float, hge>(hge v)
{
	return h2f(v);
}
template <>
__device__ __forceinline__ double
as_float<double, hge>(hge v)
{
	return hge_to_dbl(v);
}

// |a * b| <= max in 128 bits (HGEMUL_CHECK, gdk_calc_private.h:196-230)
__device__ __forceinline__ bool
hge_mul_ok(hge a, hge b, hge *dst)
{
	const bool neg = (a < 0) != (b < 0);
	const uhge x = a < 0 ? (uhge) 0 - (uhge) a : (uhge) a, y = b < 0 ? (uhge) 0 - (uhge) b : (uhge) b;
	const unsigned long long a1 = (unsigned long long) (x >> 64), a2 = (unsigned long long) x;
	const unsigned long long b1 = (unsigned long long) (y >> 64), b2 = (unsigned long long) y;
	if (a1 != 0 && b1 != 0)
		return false;
	uhge c = (uhge) a1 * b2 + (uhge) a2 * b1;
	if (c & (~(uhge) 0 << 63))
		return false;
	c = (c << 64) + (uhge) a2 * b2;
	if (c & ((uhge) 1 << 127))
		return false;
	const uhge mx = ((uhge) 1 << 127) - 1;
	if (c > mx)
		return false;
	*dst = neg ? -(hge) c : (hge) c;
	return true;
}

// one lane per group: doprod's loop over the group's rows in candidate order
template <typename T1, typename T2, int KIND>
__global__ void
k_prod(const T1 *v, ProdArgs a)
{
	const BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= a.ngrp)
		return;
	const BUN j0 = a.start ? a.start[k] : 0, j1 = a.start ? a.start[k + 1] : a.n;
	T2 prod = a.nil_if_empty ? pnil<T2>() : (T2) 1;
	bool seen = false, ovf = false;
	for (BUN j = j0; j < j1 && !ovf; j++) {
		const BUN r = a.perm ? a.perm[j] : j;
		const T1 x = v[a.off + r];
		if (KIND == PK_HGE && a.nil_if_empty && !seen) {
			seen = true;
			prod = 1;
		}
		if (is_nil(x)) {
			if (!a.skip_nils)
				prod = pnil<T2>();
			continue;
		}
		if (KIND != PK_HGE && a.nil_if_empty && !seen) {
			seen = true;
			prod = 1;
		}
		if (is_nil(prod))
			continue;
		if constexpr (KIND == PK_FLOAT) {
			const T2 fx = as_float<T2, T1>(x);
			const T2 ax = fx < 0 ? -fx : fx, ap = prod < 0 ? -prod : prod;
			if (ax > 1 && tmax<T2>() / ax < ap)
				ovf = true;
			else
				prod *= fx;
		} else if constexpr (KIND == PK_HGE) {
			hge d;
			if (!hge_mul_ok((hge) x, (hge) prod, &d))
				ovf = true;
			else
				prod = (T2) d;
		} else {
			typedef typename Wider<T2>::T W;
			const W p = (W) x * (W) prod;
			if (p > (W) tmax<T2>() || p < -(W) tmax<T2>())
				ovf = true;
			else
				prod = (T2) p;
		}
	}
	uint32_t f = (ovf ? 1u : 0u) | (is_nil(prod) ? 2u : 0u);
	((T2 *) a.res)[k] = prod;
	if (f)
		atomicOr(a.flags, f);
}

// the whole-column integer product in parallel (head of this file):
// per workgroup, in row order: the first zero, the first row that makes the
// product nil (a nil with !skip_nils -- AGGR_PROD forgets nils before the
// first value when nil_if_empty), the first non-nil row, and over the rows
// before the first zero the saturated product of |v| and the count of
// negative values; the host combines the partials in order
struct PPart {
	unsigned long long zero, nilrow, first, firstnil;
	uhge mag;                     // saturated at 2^127
	unsigned long long negs;
	unsigned long long any;       // non-nil rows
};

__device__ __forceinline__ uhge
sat_mul(uhge a, uhge b)
{
	const uhge cap = (uhge) 1 << 127;
	if (a == 0 || b == 0)
		return 0;
	if (a >= cap || b >= cap)
		return cap;
	const unsigned long long a1 = (unsigned long long) (a >> 64), b1 = (unsigned long long) (b >> 64);
	if (a1 != 0 && b1 != 0)
		return cap;
	const unsigned long long a2 = (unsigned long long) a, b2 = (unsigned long long) b;
	uhge c = (uhge) a1 * b2 + (uhge) a2 * b1;
	if (c >> 63)
		return cap;
	c = (c << 64);
	const uhge lo = (uhge) a2 * b2;
	if (c > ~(uhge) 0 - lo)
		return cap;
	c += lo;
	return c >= cap ? cap : c;
}

// one workgroup per contiguous chunk of rows, each lane a contiguous run of
// them, so the partials combine in row order
template <typename T>
__global__ __launch_bounds__(256) void
k_prod_part(const T *v, BUN n, BUN chunk, PPart *part)
{
	__shared__ PPart sh[256];
	const BUN b0 = (BUN) blockIdx.x * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
	const BUN per = (b1 - b0 + blockDim.x - 1) / blockDim.x;
	const BUN r0 = b0 + per * threadIdx.x, r1 = r0 + per < b1 ? r0 + per : b1;
	PPart p{NOPOS, NOPOS, NOPOS, NOPOS, 1, 0, 0};
	for (BUN i = r0; i < r1; i++) {
		const T x = v[i];
		if (is_nil(x)) {
			if (p.firstnil == NOPOS)
				p.firstnil = i;
			continue;
		}
		p.any++;
		if (p.first == NOPOS)
			p.first = i;
		if (p.zero != NOPOS)
			continue;
		if (x == 0) {
			p.zero = i;
			continue;
		}
		const hge hx = (hge) x;
		p.mag = sat_mul(p.mag, (uhge) (hx < 0 ? -hx : hx));
		p.negs += hx < 0;
	}
	sh[threadIdx.x] = p;
	__syncthreads();
	if (threadIdx.x == 0) {
		// the lanes' runs in order; the magnitude / sign only while no zero
		// came before (the host cuts at the nil row, which it finds from
		// the firstnil / first fields)
		PPart a = sh[0];
		for (unsigned t = 1; t < blockDim.x; t++) {
			const PPart &q = sh[t];
			if (a.first == NOPOS)
				a.first = q.first;
			if (a.firstnil == NOPOS)
				a.firstnil = q.firstnil;
			a.any += q.any;
			if (a.zero == NOPOS) {
				a.mag = sat_mul(a.mag, q.mag);
				a.negs += q.negs;
				a.zero = q.zero;
			}
		}
		part[blockIdx.x] = a;
	}
}

// the group's rows before the row `cut` only (the whole-column form needs
// the magnitude up to the nil cut when it precedes the first zero: a second
// pass over [0, cut) with the same kernel)

int
prod_type_ok(int tp1, int tp2, int *kind)
{
	auto in = [&](std::initializer_list<int> l) {
		for (int t : l)
			if (t == tp1)
				return true;
		return false;
	};
	bool ok;
	switch (tp2) {
	case MGDK_bte: ok = in({MGDK_bte}); *kind = PK_INT; break;
	case MGDK_sht: ok = in({MGDK_bte, MGDK_sht}); *kind = PK_INT; break;
	case MGDK_int: ok = in({MGDK_bte, MGDK_sht, MGDK_int}); *kind = PK_INT; break;
	case MGDK_lng: ok = in({MGDK_bte, MGDK_sht, MGDK_int, MGDK_lng}); *kind = PK_INT; break;
	case MGDK_hge: ok = in({MGDK_bte, MGDK_sht, MGDK_int, MGDK_lng, MGDK_hge}); *kind = PK_HGE; break;
	case MGDK_flt: ok = in({MGDK_bte, MGDK_sht, MGDK_int, MGDK_lng, MGDK_hge, MGDK_flt}); *kind = PK_FLOAT; break;
	case MGDK_dbl: ok = in({MGDK_bte, MGDK_sht, MGDK_int, MGDK_lng, MGDK_hge, MGDK_flt, MGDK_dbl}); *kind = PK_FLOAT; break;
	default: ok = false; break;
	}
	return ok ? 0 : -1;
}

template <typename T2, int KIND>
void
launch_prod_t2(int tp1, const void *v, const ProdArgs &a, dim3 g, dim3 b)
{
	hipStream_t st = stream();
	switch (tp1) {
	case MGDK_bte: hipLaunchKernelGGL((k_prod<int8_t, T2, KIND>), g, b, 0, st, (const int8_t *) v, a); break;
	case MGDK_sht: hipLaunchKernelGGL((k_prod<int16_t, T2, KIND>), g, b, 0, st, (const int16_t *) v, a); break;
	case MGDK_int: hipLaunchKernelGGL((k_prod<int32_t, T2, KIND>), g, b, 0, st, (const int32_t *) v, a); break;
	case MGDK_lng: hipLaunchKernelGGL((k_prod<int64_t, T2, KIND>), g, b, 0, st, (const int64_t *) v, a); break;
	default:
		if constexpr (KIND != PK_INT) {
			if (tp1 == MGDK_hge)
				hipLaunchKernelGGL((k_prod<hge, T2, KIND>), g, b, 0, st, (const hge *) v, a);
		}
		if constexpr (KIND == PK_FLOAT) {
			if (tp1 == MGDK_flt)
				hipLaunchKernelGGL((k_prod<float, T2, KIND>), g, b, 0, st, (const float *) v, a);
			if constexpr (sizeof(T2) == 8) {
				if (tp1 == MGDK_dbl)
					hipLaunchKernelGGL((k_prod<double, T2, KIND>), g, b, 0, st, (const double *) v, a);
			}
		}
		break;
	}
}

void
launch_prod(int tp1, int tp2, const void *v, const ProdArgs &a)
{
	const dim3 g(grid_for(a.ngrp, 64, 1u << 20)), b(64);
	switch (tp2) {
	case MGDK_bte: launch_prod_t2<int8_t, PK_INT>(tp1, v, a, g, b); break;
	case MGDK_sht: launch_prod_t2<int16_t, PK_INT>(tp1, v, a, g, b); break;
	case MGDK_int: launch_prod_t2<int32_t, PK_INT>(tp1, v, a, g, b); break;
	case MGDK_lng: launch_prod_t2<int64_t, PK_INT>(tp1, v, a, g, b); break;
	case MGDK_hge: launch_prod_t2<hge, PK_HGE>(tp1, v, a, g, b); break;
	case MGDK_flt: launch_prod_t2<float, PK_FLOAT>(tp1, v, a, g, b); break;
	default: launch_prod_t2<double, PK_FLOAT>(tp1, v, a, g, b); break;
	}
}

// the partials of rows [0, n) of v (whole-column integer product)
int
prod_parts(int tp1, const void *v, BUN n, std::vector<PPart> &out)
{
	hipStream_t st = stream();
	const BUN chunk = n < 256 * 64 ? 256 * 64 : (n + 1023) / 1024;
	const unsigned nb = (unsigned) ((n + chunk - 1) / chunk);
	DevBuf part(nb * sizeof(PPart) + 64);
	if (!part.p)
		return -1;
	PPart *pp = part.as<PPart>();
	const dim3 g(nb), b(256);
	switch (tp1) {
	case MGDK_bte: hipLaunchKernelGGL(k_prod_part<int8_t>, g, b, 0, st, (const int8_t *) v, n, chunk, pp); break;
	case MGDK_sht: hipLaunchKernelGGL(k_prod_part<int16_t>, g, b, 0, st, (const int16_t *) v, n, chunk, pp); break;
	case MGDK_int: hipLaunchKernelGGL(k_prod_part<int32_t>, g, b, 0, st, (const int32_t *) v, n, chunk, pp); break;
	case MGDK_lng: hipLaunchKernelGGL(k_prod_part<int64_t>, g, b, 0, st, (const int64_t *) v, n, chunk, pp); break;
	default: hipLaunchKernelGGL(k_prod_part<hge>, g, b, 0, st, (const hge *) v, n, chunk, pp); break;
	}
	out.resize(nb);
	if (!hip_ok(hipMemcpyAsync(out.data(), pp, nb * sizeof(PPart), hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	return 0;
}

// the partials combined in row order
PPart
prod_combine(const std::vector<PPart> &ps)
{
	PPart a{NOPOS, NOPOS, NOPOS, NOPOS, 1, 0, 0};
	bool zero = false;
	for (const PPart &q : ps) {
		if (a.first == NOPOS)
			a.first = q.first;
		if (a.firstnil == NOPOS)
			a.firstnil = q.firstnil;
		a.any += q.any;
		if (!zero) {
			// host saturated multiply
			const uhge cap = (uhge) 1 << 127;
			uhge m;
			if (a.mag == 0 || q.mag == 0)
				m = 0;
			else if (a.mag >= cap || q.mag >= cap)
				m = cap;
			else {
				const unsigned long long a1 = (unsigned long long) (a.mag >> 64), b1 = (unsigned long long) (q.mag >> 64);
				if (a1 && b1) {
					m = cap;
				} else {
					const unsigned long long a2 = (unsigned long long) a.mag, b2 = (unsigned long long) q.mag;
					uhge c = (uhge) a1 * b2 + (uhge) a2 * b1;
					if (c >> 63) {
						m = cap;
					} else {
						c <<= 64;
						const uhge lo = (uhge) a2 * b2;
						m = c > ~(uhge) 0 - lo ? cap : c + lo;
						if (m > cap)
							m = cap;
					}
				}
			}
			a.mag = m;
			a.negs += q.negs;
			if (q.zero != NOPOS) {
				a.zero = q.zero;
				zero = true;
			}
		}
	}
	return a;
}

hge
type_max(int tp2)
{
	switch (tp2) {
	case MGDK_bte: return INT8_MAX;
	case MGDK_sht: return INT16_MAX;
	case MGDK_int: return INT32_MAX;
	case MGDK_lng: return INT64_MAX;
	default: return (hge) (((uhge) 1 << 127) - 1);
	}
}

}  // namespace

extern "C" {

void
mgdk_free(void *p)
{
	free(p);
}

void *
mgdk_BATmin_skipnil(mgdk_bat *b, void *aggr, bool skipnil)
{
	return minmax_skipnil<false>(b, aggr, skipnil);
}

void *
mgdk_BATmax_skipnil(mgdk_bat *b, void *aggr, bool skipnil)
{
	return minmax_skipnil<true>(b, aggr, skipnil);
}

void *
mgdk_BATmin(mgdk_bat *b, void *aggr)
{
	return minmax_skipnil<false>(b, aggr, true);
}

void *
mgdk_BATmax(mgdk_bat *b, void *aggr)
{
	return minmax_skipnil<true>(b, aggr, true);
}

// BATprod (gdk_aggr.c:1650): res of type tp
int
mgdk_BATprod(void *res, int tp, mgdk_bat *b, mgdk_bat *s, bool skip_nils, bool nil_if_empty)
{
	if (b == nullptr || res == nullptr) {
		seterr("BATprod: b must exist");
		return -1;
	}
	int kind;
	const int tp1 = b->ttype;
	if (prod_type_ok(tp1, tp, &kind) < 0) {
		// the init switch rejects the result type first (:1667-1695)
		switch (tp) {
		case MGDK_bte: case MGDK_sht: case MGDK_int: case MGDK_lng: case MGDK_hge: case MGDK_flt: case MGDK_dbl:
			seterr("BATprod: type combination (mul(%s)->%s) not supported.\n", atomname(tp1), atomname(tp));
			break;
		default:
			seterr("type combination (prod(%s)->%s) not supported.\n", atomname(tp1), atomname(tp));
			break;
		}
		return -1;
	}
	ProfScope prof("prod");
	const int w2 = tp == MGDK_bte ? 1 : tp == MGDK_sht ? 2 : tp == MGDK_int || tp == MGDK_flt ? 4 : tp == MGDK_hge ? 16 : 8;
	std::string init = nil_if_empty ? nil_bytes(tp, w2) : std::string();
	if (!nil_if_empty) {
		switch (tp) {
		case MGDK_bte: { const int8_t v = 1; init.assign((const char *) &v, 1); break; }
		case MGDK_sht: { const int16_t v = 1; init.assign((const char *) &v, 2); break; }
		case MGDK_int: { const int32_t v = 1; init.assign((const char *) &v, 4); break; }
		case MGDK_lng: { const int64_t v = 1; init.assign((const char *) &v, 8); break; }
		case MGDK_hge: { const hge v = 1; init.assign((const char *) &v, 16); break; }
		case MGDK_flt: { const float v = 1; init.assign((const char *) &v, 4); break; }
		default: { const double v = 1; init.assign((const char *) &v, 8); break; }
		}
	}
	memcpy(res, init.data(), (size_t) w2);
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return -1;
	if (ci.n == 0)
		return 0;
	// the candidates' values in candidate order
	mgdk_bat *v = b;
	if (!ci.dense && (v = cand_values_at(b, ci)) == nullptr)
		return -1;
	const oid off = ci.dense ? ci.seq - b->hseqbase : 0;
	const void *base = (const char *) v->theap + off * v->twidth;
	hipStream_t st = stream();
	if (kind != PK_FLOAT) {
		// exact parallel form: overflow iff the saturated magnitude of the
		// rows before the first zero and before the nil cut exceeds the max
		std::vector<PPart> ps;
		if (prod_parts(tp1, base, ci.n, ps) < 0)
			return -1;
		PPart a = prod_combine(ps);
		// the row from which the product stays nil: AGGR_PROD_HGE: the first
		// nil; AGGR_PROD with nil_if_empty: the first nil after the first
		// value (earlier nils are forgotten), else the first nil
		unsigned long long cut = NOPOS;
		if (!skip_nils && a.firstnil != NOPOS) {
			if (kind == PK_HGE || !nil_if_empty) {
				cut = a.firstnil;
			} else if (a.first != NOPOS) {
				// the first nil after the first value: from the nil flags of
				// the rows after it (a second look at the partials' rows)
				std::vector<PPart> ps2;
				const BUN from = a.first + 1;
				if (from < ci.n) {
					if (prod_parts(tp1, (const char *) base + from * v->twidth, ci.n - from, ps2) < 0)
						return -1;
					const PPart a2 = prod_combine(ps2);
					if (a2.firstnil != NOPOS)
						cut = from + a2.firstnil;
				}
			}
		}
		uhge mag = a.mag;
		unsigned long long negs = a.negs;
		if (cut != NOPOS && (a.zero == NOPOS || cut < a.zero)) {
			// the magnitude only over the rows before the cut
			std::vector<PPart> ps3;
			if (cut > 0) {
				if (prod_parts(tp1, base, cut, ps3) < 0)
					return -1;
				const PPart a3 = prod_combine(ps3);
				mag = a3.mag;
				negs = a3.negs;
			} else {
				mag = 1;
				negs = 0;
			}
		}
		const hge mx = type_max(tp);
		const bool zero_first = a.zero != NOPOS && (cut == NOPOS || a.zero < cut);
		if (mag > (uhge) mx) {
			seterr("22003!overflow in product aggregate.\n");
			return -1;
		}
		const bool isnil = cut != NOPOS;
		if (!isnil && a.any == 0) {
			// no value: res keeps the initial value (nil_if_empty: nil, else
			// 1) -- except that AGGR_PROD_HGE marks a group seen on any row,
			// a nil one included, and starts it at 1
			if (kind == PK_HGE && nil_if_empty && skip_nils) {
				const hge one = 1;
				memcpy(res, &one, 16);
			}
			return 0;
		}
		if (isnil) {
			const std::string nb = nil_bytes(tp, w2);
			memcpy(res, nb.data(), (size_t) w2);
			return 0;
		}
		const hge r = zero_first ? 0 : ((negs & 1) ? -(hge) mag : (hge) mag);
		switch (tp) {
		case MGDK_bte: { const int8_t x = (int8_t) r; memcpy(res, &x, 1); break; }
		case MGDK_sht: { const int16_t x = (int16_t) r; memcpy(res, &x, 2); break; }
		case MGDK_int: { const int32_t x = (int32_t) r; memcpy(res, &x, 4); break; }
		case MGDK_lng: { const int64_t x = (int64_t) r; memcpy(res, &x, 8); break; }
		default: memcpy(res, &r, 16); break;
		}
		return 0;
	}
	// floats: the reference's rounding order, one lane
	DevBuf out(32), fl(16);
	if (!out.p || !fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 16, st), "memset"))
		return -1;
	ProdArgs pa{};
	pa.off = 0;
	pa.ngrp = 1;
	pa.n = ci.n;
	pa.skip_nils = skip_nils;
	pa.nil_if_empty = nil_if_empty;
	pa.res = out.p;
	pa.flags = fl.as<uint32_t>();
	launch_prod(tp1, tp, base, pa);
	char *h = (char *) pinned(64);
	if (!hip_ok(hipMemcpyAsync(h, out.p, w2, hipMemcpyDeviceToHost, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(h + 32, fl.p, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	uint32_t f;
	memcpy(&f, h + 32, 4);
	if (f & 1) {
		seterr("22003!overflow in product aggregate.\n");
		return -1;
	}
	memcpy(res, h, (size_t) w2);
	return 0;
}

// BATgroupprod (gdk_aggr.c:1575)
mgdk_bat *
mgdk_BATgroupprod(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	if (b == nullptr) {
		seterr("BATgroupprod: b must exist");
		return nullptr;
	}
	if (g == nullptr) {
		seterr("b and g must be aligned\n");
		return nullptr;
	}
	ProfScope prof("groupprod");
	const int tp1 = b->ttype;
	Cand ci0;
	if (cand_init(&ci0, b, s) < 0)
		return nullptr;
	const BUN cnt1 = b->count;
	const oid hseq1 = b->hseqbase;
	mgdk_bat *v1 = b;
	AggrInit a;
	if (group_init(&a, &v1, g, e, s) < 0)
		return nullptr;
	const BUN ng = a.ngrp;
	const int w2 = tp == MGDK_bte ? 1 : tp == MGDK_sht ? 2 : tp == MGDK_int || tp == MGDK_flt ? 4 : tp == MGDK_hge ? 16 : 8;
	if (ci0.n == 0 || ng == 0) {
		const std::string nb = nil_bytes(tp, w2);
		return mgdk_BATconstant(ng == 0 ? 0 : a.min, tp, nb.data(), ng);
	}
	const bool gdense = (g->ttype == MGDK_void && g->tseqbase != MGDK_OID_NIL) ||
			    (g->ttype == MGDK_oid && g->tseqbase != MGDK_OID_NIL);
	if ((e == nullptr || (e->count == ci0.n && e->hseqbase == ci0.seq)) && (gdense || (g->tkey && g->tnonil))) {
		// singleton groups: BATconvert(b, s, tp, 0, 0, 0)
		(void) cnt1;
		(void) hseq1;
		return mgdk_BATconvert(b, s, tp, 0, 0, 0);
	}
	int kind;
	if (prod_type_ok(tp1, tp, &kind) < 0) {
		seterr("BATgroupprod: type combination (mul(%s)->%s) not supported.\n", atomname(tp1), atomname(tp));
		return nullptr;
	}
	GroupRows gr(a.ci.n, ng);
	mgdk_bat *bn = newbat(a.min, tp, ng);
	DevBuf fl(16);
	if (bn == nullptr || !gr.ok() || !fl.p) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (group_rows(a, gr) != 0 || !hip_ok(hipMemsetAsync(fl.p, 0, 16, stream()), "memset")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	ProdArgs pa{};
	pa.off = a.ci.seq - v1->hseqbase;
	pa.perm = gr.perm;
	pa.start = gr.start_p;
	pa.ngrp = ng;
	pa.n = a.ci.n;
	pa.skip_nils = skip_nils;
	pa.nil_if_empty = true;
	pa.res = bn->theap;
	pa.flags = fl.as<uint32_t>();
	launch_prod(tp1, tp, v1->theap, pa);
	uint32_t *h = (uint32_t *) pinned(8);
	if (!hip_ok(hipMemcpyAsync(h, fl.p, 4, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[0] & 1) {
		mgdk_BBPunfix(bn);
		seterr("22003!overflow in product aggregate.\n");
		return nullptr;
	}
	bn->count = ng;
	bn->tkey = bn->tsorted = bn->trevsorted = ng <= 1;
	bn->tnil = (h[0] & 2) != 0;
	bn->tnonil = !bn->tnil;
	return bn;
}

// BATunmask (gdk_cand.c:1464)
mgdk_bat *
mgdk_BATunmask(mgdk_bat *b)
{
	if (b == nullptr) {
		seterr("BATunmask: b must exist");
		return nullptr;
	}
	const bool mcand = b->ttype == MGDK_void && b->tvheap && b->tvheapsize > 8;
	if (b->ttype != MGDK_msk && !mcand) {
		seterr("BATunmask: not a msk BAT or a mask candidate list");
		return nullptr;
	}
	if (mcand) {
		uint64_t *hdr = (uint64_t *) pinned(64);
		if (!hip_ok(hipMemcpyAsync(hdr, b->tvheap, 8, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
			return nullptr;
		if ((*hdr & 1) == 0) {
			seterr("BATunmask: not a msk BAT or a mask candidate list");
			return nullptr;
		}
		const BUN words = (b->tvheapsize - 8) / 4;
		if (b->count > words * 16) {
			// more than half the bits set: the negative list of the unset
			// bits below the last set one (:1493-1535)
			const oid firstbit = (*hdr >> 1) & ((1ull << 48) - 1);
			const oid tseq = b->tseqbase - firstbit;
			mgdk_bat *pos = unmask_cand(b);
			if (pos == nullptr)
				return nullptr;
			// candidates tseq + p for set bits p; the unset bits below the last
			// set bit are [tseq, last] minus the candidates
			BUN nr = 0;
			if (pos->count) {
				oid last;
				if (oid_at(pos, pos->count - 1, &last) < 0) {
					mgdk_BBPunfix(pos);
					return nullptr;
				}
				nr = last - tseq + 1;
			}
			mgdk_bat *all = mgdk_BATdense(0, tseq, nr);
			mgdk_bat *dels = all ? mgdk_BATdiffcand(all, pos) : nullptr;
			mgdk_BBPunfix(all);
			mgdk_BBPunfix(pos);
			if (dels == nullptr)
				return nullptr;
			mgdk_bat *bn = mgdk_BATnegcands(tseq, nr, dels);
			mgdk_BBPunfix(dels);
			if (bn == nullptr)
				return nullptr;
			bn->hseqbase = b->hseqbase;
			return bn;
		}
	}
	mgdk_bat *bn = unmask_cand(b);
	if (bn)
		bn->hseqbase = b->hseqbase;
	return bn;
}

}  // extern "C"
