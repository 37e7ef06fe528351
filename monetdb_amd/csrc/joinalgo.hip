// joinalgo.hip -- BATjoin on the MI355X: the reference's algorithm choice
// (gdk/gdk_join.c:4451-4623), which decides the ORDER of the result pairs
// and their properties, with each algorithm on the device:
//
//   selectjoin      one side holds a single value (gdk_join.c:363-563): a
//                   point BATselect on the other side (select.hip), then
//                   k_sj_expand writes driving candidate x matches;
//   mergejoin_void  the other side is dense (:571-700): a range BATselect on
//                   the driving side, k_mjv_map computes the matches;
//   mergejoin       sorted sides, or one sorted side when binary search beats
//                   a hash (:1023-1335, 1941-2780): k_mj_count finds every
//                   driving row's equal range by binary search over the sorted
//                   side, an exclusive scan places the rows, k_mj_write emits
//                   them (matches ascending);
//   hashjoin        otherwise (:2900-3335): join.hip (matches descending).
// Swapped variants drive from the right side.  The cost model (joincost
// :3586-3689, guess_uniques :3518-3576, count_unique :3337-3516) runs on the
// host over 1000 sampled values gathered on the device; BATordered /
// BATordered_rev (gdk/gdk_batop.c:2002-2262) are one device pass
// (k_order_flags: first descending / ascending / equal neighbour pair) whose
// findings are cached in the input descriptors as the reference caches them.
// The test oracle restates the same choice; the
// sampling rule for BATs of more than 1000 rows: DESIGN.md.
#include <cmath>
#include <vector>

#include "mgdk_internal.h"

using namespace mgdk;

namespace mgdk {
int hash_join(const mgdk_bat *l, const mgdk_bat *r, const Cand &lc, const Cand &rc, bool nil_matches,
	      mgdk_bat **ap, mgdk_bat **bp, bool *ukey);
}

namespace {

// ---- column access: signed 64-bit images, nil (the type minimum) smallest --

struct Col {
	const void *base;   // nullptr: void (dense oids from tseq; nil tseq: all nil)
	int w;
	oid tseq;
	oid hseq;
};

struct CandD {
	bool dense;
	oid seq;
	const oid *oids;
};

__device__ __forceinline__ int64_t
colv(const Col &c, BUN p)
{
	if (c.base == nullptr)
		return c.tseq == MGDK_OID_NIL ? INT64_MIN : (int64_t) (c.tseq + p);
	switch (c.w) {
	case 1: return ((const int8_t *) c.base)[p];
	case 2: return ((const int16_t *) c.base)[p];
	case 4: return ((const int32_t *) c.base)[p];
	default: return ((const int64_t *) c.base)[p];
	}
}

__device__ __forceinline__ oid
cand_at(const CandD &c, BUN i)
{
	return c.dense ? c.seq + i : c.oids[i];
}

Col
col_of(const mgdk_bat *b)
{
	Col c;
	c.base = b->ttype == MGDK_void ? nullptr : b->theap;
	c.w = b->ttype == MGDK_void ? 8 : b->twidth;
	c.tseq = b->tseqbase;
	c.hseq = b->hseqbase;
	return c;
}

CandD
cand_of(const Cand &c)
{
	return CandD{c.dense, c.seq, c.oids};
}

int64_t
nil_image(int tt)
{
	switch (basetype(tt)) {
	case MGDK_bte: return INT8_MIN;
	case MGDK_sht: return INT16_MIN;
	case MGDK_int: return INT32_MIN;
	default: return INT64_MIN;
	}
}

bool
join_type_ok(int t)
{
	t = basetype(t);
	return t == MGDK_void || t == MGDK_bte || t == MGDK_sht || t == MGDK_int || t == MGDK_lng ||
	       t == MGDK_oid;
}

int
atomtype(int t)
{
	return t == MGDK_void ? MGDK_oid : t;
}

// BATtdense: a void or oid column with a sequence base
bool
tdense(const mgdk_bat *b)
{
	return (b->ttype == MGDK_void || b->ttype == MGDK_oid) && b->tseqbase != MGDK_OID_NIL &&
	       !(b->ttype == MGDK_void && b->tvheap);
}

// ---- kernels ------------------------------------------------------------------

constexpr uint64_t NONE = ~0ull;

// first positions p (>= 1) with v[p-1] > v[p], < and ==: the evidence
// BATordered / BATordered_rev record (tnosorted, tnorevsorted, tnokey)
__global__ void __launch_bounds__(256)
k_order_flags(Col c, BUN n, unsigned long long *first)
{
	unsigned long long fd = NONE, fa = NONE, fe = NONE;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN p = (BUN) blockIdx.x * blockDim.x + threadIdx.x + 1; p < n; p += stride) {
		const int64_t x = colv(c, p - 1), y = colv(c, p);
		if (x > y && p < fd)
			fd = p;
		else if (x < y && p < fa)
			fa = p;
		else if (x == y && p < fe)
			fe = p;
	}
	auto mn = [](unsigned long long a, unsigned long long b) { return a < b ? a : b; };
	fd = block_reduce(fd, mn);
	fa = block_reduce(fa, mn);
	fe = block_reduce(fe, mn);
	if (threadIdx.x == 0) {
		if (fd != NONE)
			atomicMin(&first[0], fd);
		if (fa != NONE)
			atomicMin(&first[1], fa);
		if (fe != NONE)
			atomicMin(&first[2], fe);
	}
}

// the same with the value width a template parameter: a lane's 8 rows (and
// their predecessors, mostly the same lines) loaded before any compare, one
// workgroup minimum per flag published only when smaller than the visible
// one (a same-word atomic per workgroup of a large grid serialises)
template <typename T>
__global__ void __launch_bounds__(256)
k_order_flags_t(const T *v, BUN n, unsigned long long *first)
{
	// a wave owns 64 * V * U consecutive values, a lane V consecutive ones
	// per step read with one 16-byte load (the heap is 16-byte aligned: the
	// host checks); a value's predecessor is the one before it in the lane,
	// or the previous lane's last (lane 63 of the previous step for lane 0),
	// so each value is loaded once
	constexpr int V = 16 / (int) sizeof(T), U = 4;
	typedef T vt __attribute__((ext_vector_type(V)));
	const unsigned lane = __lane_id(), w = threadIdx.x >> 6;
	constexpr BUN STEP = 64 * V * U;
	unsigned long long fd = NONE, fa = NONE, fe = NONE;
	for (BUN t0 = ((BUN) blockIdx.x * 4 + w) * STEP; t0 < n; t0 += (BUN) gridDim.x * 4 * STEP) {
		vt y[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN e0 = t0 + ((BUN) u * 64 + lane) * V;
			if (e0 + V <= n) {
				y[u] = __builtin_nontemporal_load((const vt *) (v + e0));
			} else {
#pragma unroll
				for (int k = 0; k < V; k++)
					y[u][k] = v[e0 + k < n ? e0 + k : n - 1];
			}
		}
		T carry = v[t0 ? t0 - 1 : 0];      // the value before the wave's first
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN e0 = t0 + ((BUN) u * 64 + lane) * V;
			const T up = __shfl_up((T) y[u][V - 1], 1);
			T x = lane == 0 ? carry : up;
			carry = __shfl((T) y[u][V - 1], 63);
#pragma unroll
			for (int k = 0; k < V; k++) {
				const BUN p = e0 + k;
				const T yk = y[u][k];
				if (p > 0 && p < n) {
					if (x > yk)
						fd = p < fd ? p : fd;
					else if (x < yk)
						fa = p < fa ? p : fa;
					else
						fe = p < fe ? p : fe;
				}
				x = yk;
			}
		}
		// later rows cannot lower the minima once every lane has all three
		// (wave-uniform: the shuffles need the whole wave)
		if (__all(fd != NONE && fa != NONE && fe != NONE))
			break;
	}
	auto mn = [](unsigned long long a, unsigned long long b) { return a < b ? a : b; };
	fd = block_reduce(fd, mn);
	fa = block_reduce(fa, mn);
	fe = block_reduce(fe, mn);
	if (threadIdx.x == 0) {
		unsigned long long *f[3] = {&first[0], &first[1], &first[2]};
		const unsigned long long val[3] = {fd, fa, fe};
		for (int k = 0; k < 3; k++)
			if (val[k] < __hip_atomic_load(f[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
				atomicMin(f[k], val[k]);
	}
}

// three-way compare of BATordered's scans: BAT_ORDERED for integers,
// BAT_ORDERED_FP for flt / dbl (nil = NaN below every value, two nils equal;
// gdk/gdk_batop.c:1950-1995)
template <typename T>
__device__ __forceinline__ int
ord_cmp(T x, T y)
{
	if constexpr (std::is_floating_point<T>::value) {
		const bool xn = x != x, yn = y != y;
		if (xn || yn)
			return xn ? -(int) !yn : 1;
	}
	return (x > y) - (x < y);
}

// the first-pair positions for the types the vector scan does not cover
// (flt, dbl, hge): one row per lane per step
template <typename T>
__global__ void __launch_bounds__(256)
k_order_flags_g(const T *v, BUN n, unsigned long long *first)
{
	unsigned long long fd = NONE, fa = NONE, fe = NONE;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN p = (BUN) blockIdx.x * blockDim.x + threadIdx.x + 1; p < n; p += stride) {
		const int c = ord_cmp(v[p - 1], v[p]);
		if (c > 0)
			fd = p < fd ? p : fd;
		else if (c < 0)
			fa = p < fa ? p : fa;
		else
			fe = p < fe ? p : fe;
	}
	auto mn = [](unsigned long long a, unsigned long long b) { return a < b ? a : b; };
	fd = block_reduce(fd, mn);
	fa = block_reduce(fa, mn);
	fe = block_reduce(fe, mn);
	if (threadIdx.x == 0) {
		unsigned long long *f[3] = {&first[0], &first[1], &first[2]};
		const unsigned long long val[3] = {fd, fa, fe};
		for (int k = 0; k < 3; k++)
			if (val[k] < __hip_atomic_load(f[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
				atomicMin(f[k], val[k]);
	}
}

// neighbour relations of an oid result column: bit 0 some v[i-1] < v[i],
// bit 1 some >, bit 2 some ==, bit 3 some v[i] != v[i-1] + 1
__global__ void __launch_bounds__(256)
k_oid_adj(const oid *v, BUN n, uint32_t *flags)
{
	uint32_t f = 0;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += stride) {
		const oid x = v[i - 1], y = v[i];
		f |= x < y ? 1u : x > y ? 2u : 4u;
		if (y != x + 1)
			f |= 8u;
	}
	f = block_reduce(f, [](uint32_t a, uint32_t b) { return a | b; });
	if (threadIdx.x == 0)
		publish_or(flags, f);
}

// selectjoin output: driving candidate i repeated m times x the m matches
__global__ void __launch_bounds__(256)
k_sj_expand(CandD dc, Col bn, BUN m, BUN cnt, oid *a, oid *b)
{
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < cnt; k += stride) {
		const BUN i = k / m, j = k - i * m;
		a[k] = cand_at(dc, i);
		b[k] = (oid) colv(bn, j);
	}
}

// mergejoin_void's second column: the driving value mapped into r's head
__global__ void __launch_bounds__(256)
k_mjv_map(Col sel, Col l, BUN n, oid delta, oid *out)
{
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
		const oid o = (oid) colv(sel, k);
		out[k] = (oid) colv(l, o - l.hseq) + delta;
	}
}

// mergejoin: per driving candidate its equal range [lo, lo + cnt) in the
// sorted side's candidate sequence (ascending or descending values).
// meta[0] / meta[1]: smallest / largest driving index starting a matched run
// of equal values; meta[2] bits: 1 some row matches several, 2 a matched run
// holds several driving rows
__global__ void __launch_bounds__(256)
k_mj_count(Col L, CandD lc, BUN nl, Col R, CandD rc, BUN nr, bool rasc, bool nil_matches, int64_t lnil,
	   uint32_t *cnt, uint64_t *lo, unsigned long long *meta)
{
	unsigned long long gmin = NONE, gmax = 0;
	uint32_t f = 0;
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += stride) {
		const int64_t v = colv(L, cand_at(lc, i) - L.hseq);
		BUN a = 0, e = 0;
		if (v != lnil || nil_matches) {
			BUN x = 0, y = nr;
			while (x < y) {              // first index not before v
				const BUN m = (x + y) >> 1;
				const int64_t u = colv(R, cand_at(rc, m) - R.hseq);
				if (rasc ? u < v : u > v)
					x = m + 1;
				else
					y = m;
			}
			a = x;
			y = nr;
			while (x < y) {              // first index after v
				const BUN m = (x + y) >> 1;
				const int64_t u = colv(R, cand_at(rc, m) - R.hseq);
				if (rasc ? u <= v : u >= v)
					x = m + 1;
				else
					y = m;
			}
			e = x;
		}
		const BUN c = e - a;
		cnt[i] = (uint32_t) c;
		lo[i] = a;
		if (c) {
			if (c > 1)
				f |= 1u;
			const bool same = i > 0 && colv(L, cand_at(lc, i - 1) - L.hseq) == v;
			if (same) {
				f |= 2u;
			} else {
				gmin = i < gmin ? i : gmin;
				gmax = i + 1 > gmax ? i + 1 : gmax;
			}
		}
	}
	gmin = block_reduce(gmin, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	gmax = block_reduce(gmax, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	f = block_reduce(f, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0) {
		if (gmin != NONE)
			atomicMin(&meta[0], gmin);
		if (gmax)
			atomicMax(&meta[1], gmax);
		if (f)
			atomicOr((unsigned int *) &meta[2], f);
	}
}

__global__ void __launch_bounds__(256)
k_mj_write(CandD lc, BUN nl, CandD rc, const uint32_t *cnt, const uint64_t *lo, const uint64_t *off,
	   oid *a, oid *b)
{
	const BUN stride = (BUN) gridDim.x * blockDim.x;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += stride) {
		const uint32_t c = cnt[i];
		if (c == 0)
			continue;
		const oid lo_ = cand_at(lc, i);
		const uint64_t o = off[i], s = lo[i];
		for (uint32_t j = 0; j < c; j++) {
			a[o + j] = lo_;
			b[o + j] = cand_at(rc, s + j);
		}
	}
}

// sampled values of a column at the given positions
__global__ void __launch_bounds__(256)
k_gather_vals(Col c, const uint64_t *pos, uint32_t n, int64_t *out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n)
		out[i] = colv(c, pos[i]);
}

// ---- host helpers -------------------------------------------------------------

unsigned
grid256(BUN n)
{
	return grid_for(n, 256 * 8, 4096);
}

// the three first-pair positions of a column (cached per join call)
struct Ord {
	bool have = false;
	BUN desc = 0, asc = 0, eq = 0;   // 0: no such pair
};

int
scan_order(const mgdk_bat *b, Ord &o)
{
	if (o.have)
		return 0;
	unsigned long long *m = (unsigned long long *) meta_buf();
	unsigned long long *h = (unsigned long long *) pinned(64);
	hipStream_t st = stream();
	if (!hip_ok(hipMemsetAsync(m, 0xff, 24, st), "memset"))
		return -1;
	{
		const Col c = col_of(b);
		const dim3 gt(grid_for(b->count, 4 * 64 * 64, 8192));     // 4 waves x 64 lanes x 64 B per step
		if (b->count > 1) {
			const int bt = basetype(b->ttype);
			if (bt == MGDK_flt)
				hipLaunchKernelGGL(k_order_flags_g<float>, dim3(grid256(b->count)), dim3(256), 0, st,
						   (const float *) b->theap, b->count, m);
			else if (bt == MGDK_dbl)
				hipLaunchKernelGGL(k_order_flags_g<double>, dim3(grid256(b->count)), dim3(256), 0, st,
						   (const double *) b->theap, b->count, m);
			else if (bt == MGDK_hge)
				hipLaunchKernelGGL(k_order_flags_g<hge>, dim3(grid256(b->count)), dim3(256), 0, st,
						   (const hge *) b->theap, b->count, m);
			else if (c.base == nullptr || ((uintptr_t) c.base & 15) != 0)
				hipLaunchKernelGGL(k_order_flags, dim3(grid256(b->count)), dim3(256), 0, st, c, b->count, m);
			else if (c.w == 1)
				hipLaunchKernelGGL(k_order_flags_t<int8_t>, gt, dim3(256), 0, st, (const int8_t *) c.base, b->count, m);
			else if (c.w == 2)
				hipLaunchKernelGGL(k_order_flags_t<int16_t>, gt, dim3(256), 0, st, (const int16_t *) c.base, b->count, m);
			else if (c.w == 4)
				hipLaunchKernelGGL(k_order_flags_t<int32_t>, gt, dim3(256), 0, st, (const int32_t *) c.base, b->count, m);
			else
				hipLaunchKernelGGL(k_order_flags_t<int64_t>, gt, dim3(256), 0, st, (const int64_t *) c.base, b->count, m);
		}
	}
	if (!hip_ok(hipMemcpyAsync(h, m, 24, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	o.have = true;
	o.desc = h[0] == NONE ? 0 : h[0];
	o.asc = h[1] == NONE ? 0 : h[1];
	o.eq = h[2] == NONE ? 0 : h[2];
	return 0;
}

// BATordered (gdk/gdk_batop.c:2002-2179): 1 / 0, -1 on error
// integers compare as signed 64-bit images (oid as lng, its nil smallest, as
// BAT_ORDERED(lng) does), flt / dbl as BAT_ORDERED_FP (NaN nil smallest), hge
// as 128-bit integers; str columns are not scanned (reported not ordered
// unless their property says so)
static bool
order_scannable(const mgdk_bat *b)
{
	return b->ttype != MGDK_str && b->ttype != MGDK_msk;
}

int
ordered(mgdk_bat *b, Ord &o)
{
	if (b->ttype == MGDK_void || b->tsorted || b->count == 0)
		return 1;
	if (b->tnosorted > 0 || !order_scannable(b))
		return 0;
	if (scan_order(b, o) < 0)
		return -1;
	if (o.desc) {
		b->tnosorted = o.desc;
		if (o.asc && o.asc < o.desc && !b->trevsorted && b->tnorevsorted == 0)
			b->tnorevsorted = o.asc;
		return 0;
	}
	b->tsorted = 1;
	if (!b->trevsorted && b->tnorevsorted == 0) {
		if (o.asc)
			b->tnorevsorted = o.asc;
		else
			b->trevsorted = 1;
	}
	if (!b->tkey && !o.eq)
		b->tkey = 1;
	return 1;
}

// BATordered_rev (gdk/gdk_batop.c:2181-2262)
int
ordered_rev(mgdk_bat *b, Ord &o)
{
	if (b->count <= 1 || b->trevsorted)
		return 1;
	if (b->ttype == MGDK_void)
		return b->tseqbase == MGDK_OID_NIL;
	if (tdense(b) || b->tnorevsorted > 0 || !order_scannable(b))
		return 0;
	if (scan_order(b, o) < 0)
		return -1;
	if (o.asc) {
		b->tnorevsorted = o.asc;
		return 0;
	}
	b->trevsorted = 1;
	return 1;
}

// neighbour relations of an oid column (bits of k_oid_adj)
int
oid_adj(const mgdk_bat *b, uint32_t *bits)
{
	*bits = 0;
	if (b->count <= 1 || b->ttype == MGDK_void) {
		if (b->ttype == MGDK_void && b->count > 1)
			*bits = 1;   // dense: ascending by one
		return 0;
	}
	uint32_t *m = (uint32_t *) meta_buf();
	uint32_t *h = (uint32_t *) pinned(64);
	hipStream_t st = stream();
	if (!hip_ok(hipMemsetAsync(m, 0, 4, st), "memset"))
		return -1;
	hipLaunchKernelGGL(k_oid_adj, dim3(grid256(b->count)), dim3(256), 0, st, (const oid *) b->theap, b->count, m);
	if (!hip_ok(hipMemcpyAsync(h, m, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	*bits = h[0];
	return 0;
}

// first and last value of an oid column
int
first_last(const mgdk_bat *b, oid *f, oid *l)
{
	*f = *l = 0;
	if (b->count == 0)
		return 0;
	if (b->ttype == MGDK_void) {
		*f = b->tseqbase;
		*l = b->tseqbase + b->count - 1;
		return 0;
	}
	oid *h = (oid *) pinned(64);
	hipStream_t st = stream();
	if (!hip_ok(hipMemcpyAsync(h, b->theap, 8, hipMemcpyDeviceToHost, st), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(h + 1, (const oid *) b->theap + b->count - 1, 8, hipMemcpyDeviceToHost, st),
		    "memcpy") ||
	    !sync())
		return -1;
	*f = h[0];
	*l = h[1];
	return 0;
}

// one value of a column, as its signed image
int
value_at(const mgdk_bat *b, BUN p, int64_t *v)
{
	if (b->ttype == MGDK_void) {
		*v = b->tseqbase == MGDK_OID_NIL ? INT64_MIN : (int64_t) (b->tseqbase + p);
		return 0;
	}
	alignas(8) unsigned char *h = (unsigned char *) pinned(64);
	hipStream_t st = stream();
	if (!hip_ok(hipMemcpyAsync(h, (const char *) b->theap + p * b->twidth, b->twidth, hipMemcpyDeviceToHost, st),
		    "memcpy") ||
	    !sync())
		return -1;
	switch (b->twidth) {
	case 1: *v = *(int8_t *) h; break;
	case 2: *v = *(int16_t *) h; break;
	case 4: *v = *(int32_t *) h; break;
	default: *v = *(int64_t *) h; break;
	}
	return 0;
}

void
out2(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *a, mgdk_bat *b, bool swapped)
{
	if (swapped) {
		mgdk_bat *t = a;
		a = b;
		b = t;
	}
	*r1p = a;
	if (r2p)
		*r2p = b;
	else
		mgdk_BBPunfix(b);
}

void
unfix2(mgdk_bat *a, mgdk_bat *b)
{
	mgdk_BBPunfix(a);
	mgdk_BBPunfix(b);
}

mgdk_bat *
oidcol(BUN n)
{
	mgdk_bat *b = newbat(0, MGDK_oid, n);
	if (b) {
		b->count = n;
		b->tnonil = 1;
		b->tnil = 0;
	}
	return b;
}

// BATsetcount (gdk/gdk_bat.c:2079-2082)
void
setcount_props(mgdk_bat *b)
{
	if (b->count <= 1)
		b->tsorted = b->trevsorted = 1;
}

// virtualize (gdk/gdk_select.c:31-89) of a sorted key oid column
int
virtualize(mgdk_bat *b)
{
	if (b->ttype != MGDK_oid)
		return 0;
	oid f, l;
	if (first_last(b, &f, &l) < 0)
		return -1;
	if (b->count <= 1 || l - f == b->count - 1)
		setdense(b, b->count ? f : 0, b->count);
	return 0;
}

// nomatch (gdk_join.c:301-360): two empty dense BATs
int
nomatch(mgdk_bat **r1p, mgdk_bat **r2p)
{
	mgdk_bat *a = mgdk_BATdense(0, 0, 0), *b = mgdk_BATdense(0, 0, 0);
	if (!a || !b) {
		unfix2(a, b);
		return -1;
	}
	out2(r1p, r2p, a, b, false);
	return 0;
}

// ---- selectjoin (gdk_join.c:363-563) -----------------------------------------

int
selectjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, const Cand &lc, mgdk_bat *sr,
	   bool nil_matches, bool swapped)
{
	const oid o = lc.first;
	int64_t v;
	if (value_at(l, o - l->hseqbase, &v) < 0)
		return -1;
	if (!nil_matches && v == nil_image(l->ttype))
		return nomatch(r1p, r2p);
	alignas(8) unsigned char val[8];
	switch (r->ttype == MGDK_void ? 8 : r->twidth) {
	case 1: *(int8_t *) val = (int8_t) v; break;
	case 2: *(int16_t *) val = (int16_t) v; break;
	case 4: *(int32_t *) val = (int32_t) v; break;
	default: *(int64_t *) val = v; break;
	}
	mgdk_bat *bn = mgdk_BATselect(r, sr, val, nullptr, true, true, false, false);
	if (bn == nullptr)
		return -1;
	const BUN m = bn->count;
	if (m == 0) {
		mgdk_BBPunfix(bn);
		return nomatch(r1p, r2p);
	}
	const BUN cnt = lc.n * m;
	mgdk_bat *a = oidcol(cnt), *b = oidcol(cnt);
	if (!a || !b) {
		unfix2(a, b);
		mgdk_BBPunfix(bn);
		return -1;
	}
	hipLaunchKernelGGL(k_sj_expand, dim3(grid256(cnt)), dim3(256), 0, stream(), cand_of(lc), col_of(bn), m, cnt,
			   (oid *) a->theap, (oid *) b->theap);
	const bool bn_dense = tdense(bn);
	const oid bn_seq = bn->tseqbase;
	mgdk_BBPunfix(bn);
	if (!sync()) {
		unfix2(a, b);
		return -1;
	}
	a->tsorted = 1;
	a->trevsorted = lc.n == 1;
	a->tseqbase = m == 1 && lc.dense ? o : MGDK_OID_NIL;
	a->tkey = m == 1;
	b->tsorted = lc.n == 1 || m == 1;
	b->trevsorted = m == 1;
	b->tseqbase = lc.n == 1 && bn_dense ? bn_seq : MGDK_OID_NIL;
	b->tkey = lc.n == 1;
	setcount_props(a);
	setcount_props(b);
	out2(r1p, r2p, a, b, swapped);
	return 0;
}

// ---- mergejoin_void (gdk_join.c:571-700) ---------------------------------------

int
mergejoin_void(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, const Cand &rc,
	       bool swapped)
{
	oid lo = r->tseqbase, hi = lo + r->count;
	if (rc.seq > r->hseqbase)
		lo += rc.seq - r->hseqbase;
	if (rc.seq + rc.n < r->hseqbase + r->count)
		hi -= r->hseqbase + r->count - rc.seq - rc.n;
	mgdk_bat *a = mgdk_BATselect(l, sl, &lo, &hi, true, false, false, false);
	if (a == nullptr)
		return -1;
	mgdk_bat *b;
	if (a->count == 0) {
		b = mgdk_BATdense(0, 0, 0);
	} else if (tdense(a) && tdense(l)) {
		b = mgdk_BATdense(0, l->tseqbase + a->tseqbase - l->hseqbase + r->hseqbase - r->tseqbase, a->count);
	} else {
		b = oidcol(a->count);
		if (b) {
			hipLaunchKernelGGL(k_mjv_map, dim3(grid256(a->count)), dim3(256), 0, stream(), col_of(a), col_of(l),
					   a->count, r->hseqbase - r->tseqbase, (oid *) b->theap);
			if (!sync()) {
				unfix2(a, b);
				return -1;
			}
			b->tkey = l->tkey;
			b->tsorted = l->tsorted;
			b->trevsorted = l->trevsorted;
			b->tseqbase = MGDK_OID_NIL;
			setcount_props(b);
		}
	}
	if (b == nullptr) {
		mgdk_BBPunfix(a);
		return -1;
	}
	out2(r1p, r2p, a, b, swapped);
	return 0;
}

// ---- mergejoin (gdk_join.c:1941-2780; mergejoin_int / _lng :1023-1335) --------

int
mergejoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, const Cand &lc, const Cand &rc,
	  bool nil_matches, bool swapped)
{
	const int bt = basetype(atomtype(l->ttype));
	const bool special = lc.dense && lc.n == l->count && rc.dense && rc.n == r->count && l->tsorted &&
			     r->tsorted && l->ttype != MGDK_void && (bt == MGDK_int || bt == MGDK_lng || bt == MGDK_oid);
	const bool lsorted = l->tsorted || l->trevsorted;   // lscan > 0
	const BUN nl = lc.n;
	hipStream_t st = stream();
	DevBuf cnt(nl * 4 + 64), lo(nl * 8 + 64), off(nl * 8 + 64);
	unsigned long long *meta = (unsigned long long *) meta_buf();
	unsigned long long *h = (unsigned long long *) pinned(64);
	if (!cnt.p || !lo.p || !off.p || !hip_ok(hipMemsetAsync(meta, 0xff, 8, st), "memset") ||
	    !hip_ok(hipMemsetAsync(meta + 1, 0, 16, st), "memset"))
		return -1;
	hipLaunchKernelGGL(k_mj_count, dim3(grid256(nl)), dim3(256), 0, st, col_of(l), cand_of(lc), nl, col_of(r),
			   cand_of(rc), rc.n, (bool) r->tsorted, nil_matches, nil_image(l->ttype), cnt.as<uint32_t>(),
			   lo.as<uint64_t>(), meta);
	uint64_t total = 0;
	if (exclusive_scan(cnt.as<uint32_t>(), off.as<uint64_t>(), nl, &total) < 0)
		return -1;
	if (!hip_ok(hipMemcpyAsync(h, meta, 24, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	const bool groups_le1 = h[0] == NONE || h[0] + 1 == h[1];
	const bool multi = h[2] & 1, nlmulti = h[2] & 2;
	mgdk_bat *a = oidcol(total), *b = oidcol(total);
	if (!a || !b) {
		unfix2(a, b);
		return -1;
	}
	if (total)
		hipLaunchKernelGGL(k_mj_write, dim3(grid256(nl)), dim3(256), 0, st, cand_of(lc), nl, cand_of(rc),
				   cnt.as<uint32_t>(), lo.as<uint64_t>(), off.as<uint64_t>(), (oid *) a->theap,
				   (oid *) b->theap);
	oid af, al, bf, bl;
	uint32_t adj2 = 0;
	if (!sync() || first_last(a, &af, &al) < 0 || first_last(b, &bf, &bl) < 0 || oid_adj(b, &adj2) < 0) {
		unfix2(a, b);
		return -1;
	}
	const BUN n = total;
	const bool asc2 = adj2 & 1, desc2 = adj2 & 2, eq2 = adj2 & 4, consec2 = !(adj2 & 8);
	// r1 ascends with the driving candidates
	a->tsorted = 1;
	a->trevsorted = n <= 1 || af == al;
	a->tkey = !multi;
	b->tsorted = !desc2;
	if (special) {
		b->trevsorted = !asc2;
		b->tkey = !nlmulti;
		a->tseqbase = n == 0 ? 0 : (a->tkey && al - af == n - 1 ? af : MGDK_OID_NIL);
		b->tseqbase = n == 0 ? 0 : (consec2 ? bf : MGDK_OID_NIL);
		setcount_props(a);
		setcount_props(b);
	} else {
		if (lsorted) {
			b->trevsorted = !asc2;
			b->tkey = !nlmulti;
		} else {
			// l unsorted: flagged reverse sorted only within one run, key
			// only while ascending (or two descending rows of two runs),
			// gdk_join.c:2587-2631
			b->trevsorted = !asc2 && groups_le1;
			b->tkey = (!desc2 && !eq2) || (n == 2 && bf > bl);
		}
		a->tseqbase = b->tseqbase = MGDK_OID_NIL;
		setcount_props(a);
		setcount_props(b);
		if (a->tkey && virtualize(a) < 0) {
			unfix2(a, b);
			return -1;
		}
		if (n <= 1) {
			b->tkey = 1;
			if (virtualize(b) < 0) {
				unfix2(a, b);
				return -1;
			}
		}
	}
	out2(r1p, r2p, a, b, swapped);
	return 0;
}

// ---- hashjoin (gdk_join.c:2900-3335) ------------------------------------------

int
hashjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, const Cand &lc, const Cand &rc,
	 bool nil_matches, bool swapped)
{
	mgdk_bat *a = nullptr, *b = nullptr;
	bool ukey = false;
	join_ends = JoinEnds{};
	if (hash_join(l, r, lc, rc, nil_matches, &a, &b, &ukey) < 0)
		return -1;
	const BUN n = a->count;
	oid af, al, bf, bl;
	uint32_t adj1 = 0;
	// the ends come with the pair count when the partitioned join ran
	const bool ends = join_ends.a == a && join_ends.b == b && n > 0;
	if (ends) {
		af = join_ends.af;
		al = join_ends.al;
		bf = join_ends.bf;
		bl = join_ends.bl;
	}
	join_ends = JoinEnds{};
	// with unique build keys r1 (ascending) cannot repeat an oid: no scan
	if ((!ends && (first_last(a, &af, &al) < 0 || first_last(b, &bf, &bl) < 0)) || (!ukey && oid_adj(a, &adj1) < 0)) {
		unfix2(a, b);
		return -1;
	}
	a->tnonil = b->tnonil = 1;
	a->tnil = b->tnil = 0;
	a->tsorted = 1;
	a->trevsorted = n <= 1 || af == al;
	a->tkey = !(adj1 & 4);
	// r1 keeps a tseqbase while the matched candidates are consecutive
	// (lskipped, gdk_join.c:3206-3230), only for a dense left candidate list
	const bool adense = lc.dense && a->tkey && (n <= 1 || al - af == n - 1);
	b->tsorted = b->trevsorted = 0;
	b->tkey = l->tkey;
	if (n <= 1) {
		a->tsorted = a->trevsorted = a->tkey = 1;
		b->tsorted = b->trevsorted = b->tkey = 1;
	}
	a->tseqbase = n == 0 ? 0 : (n == 1 || adense ? af : MGDK_OID_NIL);
	b->tseqbase = n == 0 ? 0 : (n == 1 ? bf : MGDK_OID_NIL);
	const double ue = l->tunique_est < r->tunique_est ? l->tunique_est : r->tunique_est;
	a->tunique_est = b->tunique_est = ue;
	out2(r1p, r2p, a, b, swapped);
	return 0;
}

// what canditer_init (gdk/gdk_cand.c:407-560) calls a candidate list:
// mask lists keep their own type (no binary search cost, no candidate
// hash), except lists count their exceptions as nvals
struct CandKind {
	bool mask = false;
	BUN nvals = 0;      // except: number of exceptions
	bool except = false;
};

int
cand_kind(const mgdk_bat *s, CandKind *k)
{
	*k = CandKind{};
	// a msk BAT counts as the oid list it unmasks to (runtime.hip unmask_cand)
	if (s == nullptr || !is_complex_cand(s) || s->ttype == MGDK_msk)
		return 0;
	uint64_t *hdr = (uint64_t *) pinned(64);
	if (!hip_ok(hipMemcpyAsync(hdr, s->tvheap, 8, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return -1;
	if (*hdr & 1) {
		k->mask = true;
	} else {
		k->except = true;
		k->nvals = (s->tvheapsize - 8) / 8;
	}
	return 0;
}


// ---- cost model (gdk_join.c:3337-3689) -----------------------------------------

// the BATsample(b, 1000) rows: all up to 1000 (gdk_sample.c:114-117), else
// 1000 evenly spaced (the oracle's rule; the reference samples at random)
uint32_t
sample_positions(BUN cnt, std::vector<uint64_t> &pos)
{
	const BUN n = cnt <= 1000 ? cnt : 1000;
	pos.resize(n);
	for (BUN i = 0; i < n; i++)
		pos[i] = cnt <= 1000 ? i : (uint64_t) ((uhge) i * cnt / 1000);
	return (uint32_t) n;
}

int
gather(const mgdk_bat *b, const std::vector<uint64_t> &pos, std::vector<int64_t> &out)
{
	const uint32_t n = (uint32_t) pos.size();
	out.resize(n);
	if (n == 0)
		return 0;
	if (b->ttype == MGDK_void) {
		for (uint32_t i = 0; i < n; i++)
			out[i] = b->tseqbase == MGDK_OID_NIL ? INT64_MIN : (int64_t) (b->tseqbase + pos[i]);
		return 0;
	}
	hipStream_t st = stream();
	DevBuf dp(n * 8 + 64), dv(n * 8 + 64);
	if (!dp.p || !dv.p ||
	    !hip_ok(hipMemcpyAsync(dp.p, pos.data(), n * 8, hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	hipLaunchKernelGGL(k_gather_vals, dim3((n + 255) / 256), dim3(256), 0, st, col_of(b), dp.as<uint64_t>(), n,
			   dv.as<int64_t>());
	if (!hip_ok(hipMemcpyAsync(out.data(), dv.p, n * 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	return 0;
}

// count_unique (gdk_join.c:3337-3516) over sampled oids s of b
int
count_unique(mgdk_bat *b, Ord &o, const std::vector<uint64_t> &s, BUN *cnt1, BUN *cnt2)
{
	const BUN ns = s.size(), half = ns / 2;
	if (b->tkey || ns <= 1 || tdense(b)) {
		*cnt1 = half;
		*cnt2 = ns;
		return 0;
	}
	if (ordered(b, o) < 0 || ordered_rev(b, o) < 0)
		return -1;
	if ((b->tsorted && b->trevsorted) || (b->ttype == MGDK_void && b->tseqbase == MGDK_OID_NIL)) {
		*cnt1 = *cnt2 = 1;
		return 0;
	}
	std::vector<uint64_t> pos(ns);
	for (BUN i = 0; i < ns; i++)
		pos[i] = s[i] - b->hseqbase;
	std::vector<int64_t> v;
	if (gather(b, pos, v) < 0)
		return -1;
	std::vector<int64_t> seen;
	*cnt1 = 0;
	for (BUN i = 0; i < ns; i++) {
		if (i == half)
			*cnt1 = seen.size();
		bool found = false;
		for (size_t k = 0; k < seen.size() && !found; k++)
			found = seen[k] == v[i];
		if (!found)
			seen.push_back(v[i]);
	}
	*cnt2 = seen.size();
	return 0;
}

// guess_uniques (gdk_join.c:3518-3576); s: the candidate BAT behind c
// (nullptr: all of b)
int
guess_uniques(mgdk_bat *b, Ord &o, const Cand &c, const mgdk_bat *s, double *est)
{
	if (b->tkey) {
		*est = (double) c.n;
		return 0;
	}
	const bool full = s == nullptr || (c.dense && c.n == b->count);
	std::vector<uint64_t> pos, s1;
	if (full) {
		if (b->tunique_est != 0) {
			*est = b->tunique_est;
			return 0;
		}
		sample_positions(b->count, pos);
		s1.resize(pos.size());
		for (size_t i = 0; i < pos.size(); i++)
			s1[i] = b->hseqbase + pos[i];
	} else if (s->ttype == MGDK_void && !s->tvheap) {
		sample_positions(s->count, pos);
		s1.resize(pos.size());
		for (size_t i = 0; i < pos.size(); i++)
			s1[i] = s->tseqbase + pos[i];
	} else if (s->ttype == MGDK_oid) {
		sample_positions(s->count, pos);
		std::vector<int64_t> v;
		if (gather(s, pos, v) < 0)
			return -1;
		s1.assign(v.begin(), v.end());
	} else {
		// a cand_except / cand_mask list: sample its materialised candidates
		sample_positions(c.n, pos);
		s1.resize(pos.size());
		if (c.dense) {
			for (size_t i = 0; i < pos.size(); i++)
				s1[i] = c.seq + pos[i];
		} else {
			std::vector<int64_t> v(pos.size());
			hipStream_t st = stream();
			for (size_t i = 0; i < pos.size(); i++)
				if (!hip_ok(hipMemcpyAsync(&v[i], c.oids + pos[i], 8, hipMemcpyDeviceToHost, st), "memcpy"))
					return -1;
			if (!sync())
				return -1;
			s1.assign(v.begin(), v.end());
		}
	}
	const BUN n2 = s1.size(), n1 = n2 / 2;
	// count_unique iterates the sample as a candidate list of b (clipped)
	std::vector<uint64_t> clipped;
	for (uint64_t x : s1)
		if (x >= b->hseqbase && x < b->hseqbase + b->count)
			clipped.push_back(x);
	BUN cnt1, cnt2;
	if (count_unique(b, o, clipped, &cnt1, &cnt2) < 0)
		return -1;
	const double A = (double) (cnt2 - cnt1) / (n2 - n1);
	double B = cnt1 - n1 * A;
	B += A * c.n;
	if (full && b->tunique_est == 0)
		b->tunique_est = B;
	*est = B;
	return 0;
}

// joincost (gdk_join.c:3586-3689) with no prebuilt hash, transient BATs
int
joincost(mgdk_bat *r, Ord &o, BUN lcount, const Cand &rc, const mgdk_bat *sr, const CandKind &k, double *cost)
{
	const bool rmask = k.mask;
	double rcost = 1;
	if (k.except ? k.nvals > 0 : (!rc.dense && !rmask && rc.n > 0))
		rcost += log2((double) (k.except ? k.nvals : rc.n));
	rcost *= lcount;
	const BUN cnt = r->count;
	if (!tdense(r)) {
		double ue = r->tunique_est;
		if (ue == 0) {
			Cand all{};
			all.dense = true;
			all.seq = r->hseqbase;
			all.n = r->count;
			if (guess_uniques(r, o, all, nullptr, &ue) < 0)
				return -1;
		}
		rcost *= 1.1 * ((double) cnt / ue);
		rcost += cnt * 2.0;
	}
	if (rc.n != cnt && !rmask) {
		double ue = r->tunique_est;
		if (ue == 0 && guess_uniques(r, o, rc, sr, &ue) < 0)
			return -1;
		double rccost = 1.1 * ((double) cnt / ue);
		rccost *= lcount;
		rccost += rc.n * 2.0;
		if (rccost < rcost)
			rcost = rccost;
	}
	*cost = rcost;
	return 0;
}

// flt / dbl join keys as integer images that keep both equality and order
// under the reference's compare (dbl_cmp: -0.0 == +0.0; nil = NaN below
// every value): -0.0 -> +0.0, the sign-magnitude bits turned into two's
// complement order, NaN -> the integer nil (no float maps there).  BATjoin
// over the images takes the reference's algorithm choices and result order
// for the floats (hash path gdk_join.c:2900 with the value's hash, merge
// paths for ordered inputs) and returns the same oids.
template <typename F, typename I, typename U>
__global__ __launch_bounds__(256) void
k_float_image(const F *in, BUN n, I *out)
{
	constexpr U SIGN = (U) 1 << (sizeof(U) * 8 - 1);
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		F v = in[i];
		I r;
		if (v != v) {
			r = (I) SIGN;                // the integer nil
		} else {
			if (v == (F) 0)
				v = (F) 0;              // -0.0 -> +0.0
			U u;
			__builtin_memcpy(&u, &v, sizeof u);
			u = (u & SIGN) ? ~u : (u | SIGN);
			r = (I) (u ^ SIGN);
		}
		out[i] = r;
	}
}

mgdk_bat *
float_image(const mgdk_bat *b)
{
	const bool dbl = basetype(b->ttype) == MGDK_dbl;
	mgdk_bat *m = newbat(b->hseqbase, dbl ? MGDK_lng : MGDK_int, b->count);
	if (m == nullptr)
		return nullptr;
	if (b->count) {
		if (dbl)
			hipLaunchKernelGGL((k_float_image<double, int64_t, uint64_t>), dim3(grid_for(b->count, 1024, 16384)),
					   dim3(256), 0, stream(), (const double *) b->theap, b->count, (int64_t *) m->theap);
		else
			hipLaunchKernelGGL((k_float_image<float, int32_t, uint32_t>), dim3(grid_for(b->count, 1024, 16384)),
					   dim3(256), 0, stream(), (const float *) b->theap, b->count, (int32_t *) m->theap);
	}
	m->count = b->count;
	m->tsorted = b->tsorted;
	m->trevsorted = b->trevsorted;
	m->tkey = b->tkey;
	m->tnonil = b->tnonil;
	m->tnil = b->tnil;
	m->tnosorted = b->tnosorted;
	m->tnorevsorted = b->tnorevsorted;
	m->tseqbase = MGDK_OID_NIL;
	return m;
}

// str join keys: BATjoin compares strings with strCmp (nil first, then
// strcmp's unsigned bytes) and hashes them with strHash; its choices, scans
// and result order only see that order and equality, so a str pair joins
// exactly as the pair of lng columns holding each string's rank among the
// distinct strings of both sides (nil -> lng nil).  The ranks: BATgroup of
// each side (never merges different strings), the groups' representative
// strings of both sides as one str column over the two heaps laid end to
// end (8-byte absolute offsets), its chunked BATsort's group ids.
__device__ __forceinline__ uint64_t
jstr_off(const void *offs, int w, BUN p)
{
	switch (w) {
	case 1: return (uint64_t) ((const uint8_t *) offs)[p] + 8192;      // GDK_VAROFFSET
	case 2: return (uint64_t) ((const uint16_t *) offs)[p] + 8192;
	case 4: return ((const uint32_t *) offs)[p];
	default: return ((const uint64_t *) offs)[p];
	}
}

__device__ __forceinline__ oid
oid_at(const oid *p, oid seq, BUN i)
{
	return p ? p[i] : seq + i;
}

__global__ __launch_bounds__(256) void
k_str_rep_offs(const oid *ext, oid eseq, BUN ne, oid hseq, const void *offs, int w, uint64_t add, uint64_t *out)
{
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < ne; j += (BUN) gridDim.x * blockDim.x)
		out[j] = jstr_off(offs, w, oid_at(ext, eseq, j) - hseq) + add;
}

__global__ __launch_bounds__(256) void
k_str_ranks(const oid *ord, oid oseq, const oid *grp, oid gseq, BUN n, const uint64_t *coffs, const char *vh,
	    int64_t *rank)
{
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (BUN) gridDim.x * blockDim.x) {
		const BUN p = oid_at(ord, oseq, j);
		const uint8_t *s = (const uint8_t *) vh + coffs[p];
		rank[p] = s[0] == 0x80 && s[1] == 0 ? INT64_MIN : (int64_t) oid_at(grp, gseq, j);
	}
}

__global__ __launch_bounds__(256) void
k_str_img(const oid *g, oid gseq, BUN n, const int64_t *rank, BUN base, int64_t *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = rank[base + oid_at(g, gseq, i)];
}

const oid *
oid_col(const mgdk_bat *b, oid *seq)
{
	if (b->ttype == MGDK_void) {
		*seq = b->tseqbase;
		return nullptr;
	}
	*seq = 0;
	return (const oid *) b->theap;
}

mgdk_bat *
str_img(const mgdk_bat *b, const mgdk_bat *g, const int64_t *rank, BUN base)
{
	mgdk_bat *m = newbat(b->hseqbase, MGDK_lng, b->count);
	if (m == nullptr)
		return nullptr;
	oid gs;
	const oid *gp = oid_col(g, &gs);
	if (b->count)
		hipLaunchKernelGGL(k_str_img, dim3(grid_for(b->count, 1024, 16384)), dim3(256), 0, stream(), gp, gs,
				   b->count, rank, base, (int64_t *) m->theap);
	m->count = b->count;
	m->tsorted = b->tsorted;
	m->trevsorted = b->trevsorted;
	m->tkey = b->tkey;
	m->tnonil = b->tnonil;
	m->tnil = b->tnil;
	m->tnosorted = b->tnosorted;
	m->tnorevsorted = b->tnorevsorted;
	m->tseqbase = MGDK_OID_NIL;
	return m;
}

int
str_images(mgdk_bat *l, mgdk_bat *r, mgdk_bat **lip, mgdk_bat **rip)
{
	*lip = *rip = nullptr;
	mgdk_bat *gl = nullptr, *el = nullptr, *gr = nullptr, *er = nullptr, *C = nullptr, *ord = nullptr,
		 *grp = nullptr, *rk = nullptr;
	int rc = -1;
	hipStream_t st = stream();
	if (mgdk_BATgroup(&gl, &el, nullptr, l, nullptr, nullptr, nullptr, nullptr) != 0 ||
	    mgdk_BATgroup(&gr, &er, nullptr, r, nullptr, nullptr, nullptr, nullptr) != 0)
		goto out;
	{
		const BUN nl = el->count, nr = er->count, A = nl + nr;
		const size_t lsz = l->tvheapsize, rsz = r->tvheapsize;
		C = newbat(0, MGDK_lng, A);
		rk = newbat(0, MGDK_lng, A);
		Heap *vh = heap_new(lsz + rsz + 8);
		if (C == nullptr || rk == nullptr || vh == nullptr) {
			heap_decref(vh);
			goto out;
		}
		Priv *p = (Priv *) C->priv;
		heap_decref(p->tvheap);
		p->tvheap = vh;
		C->ttype = MGDK_str;
		C->twidth = 8;
		C->tvheap = vh->base;
		C->tvheapsize = lsz + rsz;
		if ((lsz && !hip_ok(hipMemcpyAsync(vh->base, l->tvheap, lsz, hipMemcpyDeviceToDevice, st), "memcpy")) ||
		    (rsz && !hip_ok(hipMemcpyAsync((char *) vh->base + lsz, r->tvheap, rsz, hipMemcpyDeviceToDevice, st),
				    "memcpy")))
			goto out;
		oid es;
		const oid *ep = oid_col(el, &es);
		if (nl)
			hipLaunchKernelGGL(k_str_rep_offs, dim3(grid_for(nl, 1024, 16384)), dim3(256), 0, st, ep, es, nl,
					   l->hseqbase, (const void *) l->theap, (int) l->twidth, (uint64_t) 0,
					   (uint64_t *) C->theap);
		ep = oid_col(er, &es);
		if (nr)
			hipLaunchKernelGGL(k_str_rep_offs, dim3(grid_for(nr, 1024, 16384)), dim3(256), 0, st, ep, es, nr,
					   r->hseqbase, (const void *) r->theap, (int) r->twidth, (uint64_t) lsz,
					   (uint64_t *) C->theap + nl);
		C->count = A;
		C->tsorted = C->trevsorted = C->tkey = A <= 1;
		C->tnosorted = C->tnorevsorted = 0;
		C->tnonil = l->tnonil && r->tnonil;
		C->tnil = 0;
		if (A) {
			if (mgdk_BATsort(nullptr, &ord, &grp, C, nullptr, nullptr, false, false, false) != 0)
				goto out;
			oid os, gs;
			const oid *op = oid_col(ord, &os), *gp = oid_col(grp, &gs);
			hipLaunchKernelGGL(k_str_ranks, dim3(grid_for(A, 1024, 16384)), dim3(256), 0, st, op, os, gp, gs, A,
					   (const uint64_t *) C->theap, (const char *) C->tvheap, (int64_t *) rk->theap);
		}
		*lip = str_img(l, gl, (const int64_t *) rk->theap, 0);
		*rip = *lip ? str_img(r, gr, (const int64_t *) rk->theap, nl) : nullptr;
		if (*rip == nullptr || !sync())
			goto out;
		rc = 0;
	}
out:
	if (rc != 0) {
		mgdk_BBPunfix(*lip);
		mgdk_BBPunfix(*rip);
		*lip = *rip = nullptr;
	}
	mgdk_BBPunfix(gl);
	mgdk_BBPunfix(el);
	mgdk_BBPunfix(gr);
	mgdk_BBPunfix(er);
	mgdk_BBPunfix(C);
	mgdk_BBPunfix(ord);
	mgdk_BBPunfix(grp);
	mgdk_BBPunfix(rk);
	return rc;
}

// the order the scans found on the images holds for the keys they stand for
void
image_flags_back(mgdk_bat *l, mgdk_bat *r, const mgdk_bat *li, const mgdk_bat *ri)
{
	l->tsorted |= li->tsorted;
	l->trevsorted |= li->trevsorted;
	l->tkey |= li->tkey;
	r->tsorted |= ri->tsorted;
	r->trevsorted |= ri->trevsorted;
	r->tkey |= ri->tkey;
	if (!l->tnosorted)
		l->tnosorted = li->tnosorted;
	if (!l->tnorevsorted)
		l->tnorevsorted = li->tnorevsorted;
	if (!r->tnosorted)
		r->tnosorted = ri->tnosorted;
	if (!r->tnorevsorted)
		r->tnorevsorted = ri->tnorevsorted;
}

}  // namespace

namespace mgdk {

// leftjoin's algorithm choice (gdk/gdk_join.c:4049-4300), for the left-output
// join family (joinkinds.hip): the branch decides the order of several
// matches of a left candidate, which match a semi join with a right output
// keeps, and two quirks (fetchjoin's right-position order, mergejoin's
// skipped nils).  BATordered / BATordered_rev are evaluated in the
// reference's order (their findings cached in l and r as it caches them);
// mergejoin's memory-pressure term (:4185) depends on the host and is taken
// as false.  *equal_order: mergejoin scans l and r the same way
// (:2091-2107).  Returns LJ_* or -1.
int
leftjoin_algo(mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, const Cand &lc, const Cand &rc,
	      bool nil_matches, bool nil_on_miss, bool semi, bool only_misses, bool not_in, bool max_one,
	      bool min_one, bool want_r2, bool *equal_order)
{
	*equal_order = true;
	if (lc.n == 0 || rc.n == 0)
		return LJ_NOMATCH;
	Ord lo, ro;
	int t1, t2;
#define ORD(x) do { if ((x) < 0) return -1; } while (0)
	if (!only_misses && !not_in) {
		if (lc.n == 1)
			return LJ_SELECT;
		ORD(t1 = ordered(l, lo));
		if (t1) {
			ORD(t2 = ordered_rev(l, lo));
			if (t2)
				return LJ_SELECT;
		}
		if (l->ttype == MGDK_void && l->tseqbase == MGDK_OID_NIL)
			return LJ_SELECT;
	}
	CandKind lk, rk;
	if (cand_kind(sl, &lk) < 0 || cand_kind(sr, &rk) < 0)
		return -1;
	const bool ldense = lc.dense && !lk.mask && !lk.except, rdense = rc.dense && !rk.mask && !rk.except;
	if (tdense(r) && rdense)
		return LJ_MJVOID;
	if (tdense(l) && ldense && rdense && !semi && !max_one && !min_one && !nil_matches && !only_misses && !not_in) {
		ORD(t1 = ordered(r, ro));
		if (!t1)
			ORD(t1 = ordered_rev(r, ro));
		if (t1)
			return LJ_FETCH;
	}
	if (tdense(l) && ldense && !want_r2 && (semi || only_misses) && !nil_on_miss && !not_in && !max_one && !min_one)
		return LJ_BITMASK;
	ORD(t1 = ordered(r, ro));
	if (!t1)
		ORD(t1 = ordered_rev(r, ro));
	if (t1) {
		ORD(t2 = ordered(l, lo));
		if (!t2)
			ORD(t2 = ordered_rev(l, lo));
		if (t2 || tdense(r) || lc.n < 1024) {
			if (l->tsorted || l->trevsorted) {
				const bool lv = tdense(l) || l->ttype == MGDK_void, rv = tdense(r) || r->ttype == MGDK_void;
				*equal_order = (l->tsorted && r->tsorted) || (l->trevsorted && r->trevsorted && !lv && !rv);
			}
			return LJ_MERGE;
		}
	}
	if (!nil_on_miss && !only_misses && !not_in && !max_one && !min_one) {
		double lcost, rcost;
		if (joincost(r, ro, lc.n, rc, sr, rk, &rcost) < 0 || joincost(l, lo, rc.n, lc, sl, lk, &lcost) < 0)
			return -1;
		if (semi && !r->tkey)
			lcost += rc.n;                  // BATunique(r)
		lcost += rc.n * log((double) rc.n);     // the sort of the swapped result
		if (lcost < rcost)
			return LJ_SWAP;
	}
	return LJ_HASH;
#undef ORD
}

mgdk_bat *
join_float_image(const mgdk_bat *b)
{
	return float_image(b);
}

int
join_str_images(mgdk_bat *l, mgdk_bat *r, mgdk_bat **lip, mgdk_bat **rip)
{
	return str_images(l, r, lip, rip);
}

void
join_image_flags_back(mgdk_bat *l, mgdk_bat *r, const mgdk_bat *li, const mgdk_bat *ri)
{
	image_flags_back(l, r, li, ri);
}

}  // namespace mgdk

extern "C" int
mgdk_BATjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
	     bool nil_matches, mgdk_BUN estimate)
{
	(void) estimate;
	if (l == nullptr || r == nullptr || r1p == nullptr) {
		seterr("BATjoin: NULL argument");
		return -1;
	}
	*r1p = nullptr;
	if (r2p)
		*r2p = nullptr;
	if (l->ttype == MGDK_msk || r->ttype == MGDK_msk) {
		// msk inputs are joined as the oid lists BATunmask makes of them
		// (gdk_join.c:4500-4517)
		mgdk_bat *lm = l->ttype == MGDK_msk ? unmask_cand(l) : nullptr;
		mgdk_bat *rm = r->ttype == MGDK_msk ? unmask_cand(r) : nullptr;
		int rc = -1;
		if ((l->ttype != MGDK_msk || lm) && (r->ttype != MGDK_msk || rm)) {
			if (lm)
				lm->hseqbase = l->hseqbase;
			if (rm)
				rm->hseqbase = r->hseqbase;
			rc = mgdk_BATjoin(r1p, r2p, lm ? lm : l, rm ? rm : r, sl, sr, nil_matches, estimate);
		}
		mgdk_BBPunfix(lm);
		mgdk_BBPunfix(rm);
		return rc;
	}
	if (basetype(atomtype(l->ttype)) != basetype(atomtype(r->ttype))) {
		seterr("42000!BATjoin: inputs not compatible.");
		return -1;
	}
	if (basetype(l->ttype) == MGDK_flt || basetype(l->ttype) == MGDK_dbl || l->ttype == MGDK_str) {
		mgdk_bat *li = nullptr, *ri = nullptr;
		if (l->ttype == MGDK_str) {
			ProfScope prof("join_str_images");
			if (str_images(l, r, &li, &ri) != 0)
				return -1;
		} else {
			li = float_image(l);
			ri = li ? float_image(r) : nullptr;
		}
		int rc = -1;
		if (li && ri) {
			rc = mgdk_BATjoin(r1p, r2p, li, ri, sl, sr, nil_matches, estimate);
			image_flags_back(l, r, li, ri);
		}
		mgdk_BBPunfix(li);
		mgdk_BBPunfix(ri);
		return rc;
	}
	if (!join_type_ok(l->ttype) || !join_type_ok(r->ttype)) {
		seterr("42000!BATjoin: type %s not supported on the device path", atomname(l->ttype));
		return -1;
	}
	ProfScope prof("join");
	Cand lc, rc;
	if (cand_init(&lc, l, sl) < 0 || cand_init(&rc, r, sr) < 0)
		return -1;
	if (lc.n == 0 || rc.n == 0)
		return nomatch(r1p, r2p);
	Ord lo, ro;
	int t1, t2;
#define ORD(x) do { if ((x) < 0) return -1; } while (0)
	// single value to join: use select (gdk_join.c:4542-4556)
	if (lc.n == 1)
		return selectjoin(r1p, r2p, l, r, lc, sr, nil_matches, false);
	ORD(t1 = ordered(l, lo));
	if (t1) {
		ORD(t2 = ordered_rev(l, lo));
		if (t2)
			return selectjoin(r1p, r2p, l, r, lc, sr, nil_matches, false);
	}
	if (l->ttype == MGDK_void && l->tseqbase == MGDK_OID_NIL)
		return selectjoin(r1p, r2p, l, r, lc, sr, nil_matches, false);
	if (rc.n == 1)
		return selectjoin(r1p, r2p, r, l, rc, sl, nil_matches, true);
	ORD(t1 = ordered(r, ro));
	if (t1) {
		ORD(t2 = ordered_rev(r, ro));
		if (t2)
			return selectjoin(r1p, r2p, r, l, rc, sl, nil_matches, true);
	}
	if (r->ttype == MGDK_void && r->tseqbase == MGDK_OID_NIL)
		return selectjoin(r1p, r2p, r, l, rc, sl, nil_matches, true);
	CandKind lk, rk;
	if (cand_kind(sl, &lk) < 0 || cand_kind(sr, &rk) < 0)
		return -1;
	// dense side (gdk_join.c:4557-4567)
	if (tdense(r) && rc.dense && !rk.mask)
		return mergejoin_void(r1p, r2p, l, r, sl, rc, false);
	if (tdense(l) && lc.dense && !lk.mask)
		return mergejoin_void(r1p, r2p, r, l, sr, lc, true);
	// both sorted (gdk_join.c:4568-4575)
	bool lord, rord;
	ORD(t1 = ordered(l, lo));
	if (!t1)
		ORD(t1 = ordered_rev(l, lo));
	lord = t1;
	if (lord) {
		ORD(t2 = ordered(r, ro));
		if (!t2)
			ORD(t2 = ordered_rev(r, ro));
		if (t2)
			return mergejoin(r1p, r2p, l, r, lc, rc, nil_matches, false);
	}
	// cost model (gdk_join.c:4577-4618)
	double lcost, rcost;
	if (joincost(l, lo, rc.n, lc, sl, lk, &lcost) < 0 || joincost(r, ro, lc.n, rc, sr, rk, &rcost) < 0)
		return -1;
	const bool swap = lcost < rcost;
	const double best = swap ? lcost : rcost;
	ORD(t1 = ordered(r, ro));
	if (!t1)
		ORD(t1 = ordered_rev(r, ro));
	if (t1 && lc.n * (log2((double) rc.n) + 1) < best)
		return mergejoin(r1p, r2p, l, r, lc, rc, nil_matches, false);
	ORD(t1 = ordered(l, lo));
	if (!t1)
		ORD(t1 = ordered_rev(l, lo));
	if (t1 && rc.n * (log2((double) lc.n) + 1) < best)
		return mergejoin(r1p, r2p, r, l, rc, lc, nil_matches, true);
	if (swap)
		return hashjoin(r1p, r2p, r, l, rc, lc, nil_matches, true);
	return hashjoin(r1p, r2p, l, r, lc, rc, nil_matches, false);
#undef ORD
}

extern "C" bool
mgdk_BATordered(mgdk_bat *b)
{
	Ord o;
	return b && ordered(b, o) > 0;
}

extern "C" bool
mgdk_BATordered_rev(mgdk_bat *b)
{
	Ord o;
	return b && ordered_rev(b, o) > 0;
}

// BATguess_uniques (gdk_join.c:3572): the join cost model's distinct-value
// estimate over b's candidates s (NULL: all of b) -- b's count for a key
// column, the cached tunique_est of a full column, else the two-point
// extrapolation over a 1000-row sample (evenly spaced: the reference samples
// at random) that a full column also caches in b
extern "C" mgdk_BUN
mgdk_BATguess_uniques(mgdk_bat *b, mgdk_bat *s)
{
	if (b == nullptr) {
		seterr("BATguess_uniques: b must not be NULL");
		return MGDK_BUN_NONE;
	}
	mgdk_bat *held = nullptr;
	if (s && is_complex_cand(s) && (s = held = unmask_cand(s)) == nullptr)
		return MGDK_BUN_NONE;
	Cand ci;
	Ord o;
	double est = 0;
	const int rc = cand_init(&ci, b, s) < 0 ? -1 : guess_uniques(b, o, ci, s, &est);
	mgdk_BBPunfix(held);
	if (rc < 0)
		return MGDK_BUN_NONE;
	return (mgdk_BUN) est;
}
