// analytic_stats.hip -- windowed statistics and products on the MI355X:
// GDKanalytical_stddev_samp / _stddev_pop / _variance_samp / _variance_pop,
// GDKanalytical_covariance_samp / _pop, GDKanalytical_correlation
// (gdk/gdk_analytic_statistics.c:689-1443) and GDKanalyticalprod
// (gdk/gdk_analytic_func.c:2024-2560).
//
// All of them fold per-row nodes whose arithmetic is order dependent
// (Welford updates; float products; integer products whose overflow check
// depends on where a zero falls), so the device keeps the reference's
// order, per partition, in parallel over partitions and rows:
//   * frames 3 / 4 / 5 (running and whole-partition): one lane per partition
//     folds its rows forward (3, 5) or backward from the end (4) and writes
//     each peer group's (or the partition's) result;
//   * frame 6: every row on its own;
//   * every other frame: the reference's fanout-16 segment tree
//     (gdk/gdk_analytic.h:63-130) for every partition at once -- one launch
//     per level, level L of partition k stored at lvl[L] + (ps >> 4L) + k
//     (analytic_func.hip's layout) -- and one thread per row walking the
//     tree for its frame [s[i], e[i]) exactly as compute_on_segment_tree.
// An inner tree node folds its children as if each were ONE value
// (COMPUTE_LEVELN_*: the child's `delta` stands for the child); that is the
// reference's definition of these frames and is kept as is.
#include <cfloat>
#include <type_traits>

#include "mgdk_internal.h"
#include "segments.h"

#pragma clang fp contract(off)

using namespace mgdk;

namespace {

constexpr int WS_MAX_LEVELS = 17;

struct Cols {
	const void *b1, *b2;
};

template <typename T>
__device__ __forceinline__ double
as_dbl(T v)
{
	return (double) v;
}
template <>
__device__ __forceinline__ double
as_dbl<hge>(hge v)
{
	return hge_to_dbl(v);
}

enum { K_VAR = 0, K_COV = 1, K_COR = 2 };

// stdev_var_deltas / covariance_deltas / correlation_deltas
// (gdk_analytic_statistics.c:794, :1081, :1320); op: K_VAR 0 stddev_samp
// 1 stddev_pop 2 variance_samp 3 variance_pop, K_COV 0 samp 1 pop
template <typename T, int KIND>
struct WNode {
	unsigned long long n;
	double mean1, delta1, m2;
	double mean2, delta2;     // K_COV, K_COR
	double up, down1, down2;  // K_COR
	using Out = double;
	__device__ __forceinline__ void zero()
	{
		n = 0;
		mean1 = delta1 = m2 = mean2 = delta2 = up = down1 = down2 = 0;
	}
	__device__ __forceinline__ void leaf(const Cols &c, BUN i)
	{
		zero();
		const T x = ((const T *) c.b1)[i];
		if (is_nil(x))
			return;
		if (KIND != K_VAR) {
			const T y = ((const T *) c.b2)[i];
			if (is_nil(y))
				return;
			mean2 = delta2 = as_dbl(y);
		}
		n = 1;
		mean1 = delta1 = as_dbl(x);
	}
	// COMPUTE_LEVELN_* (with a leaf: the running frames' row step)
	__device__ __forceinline__ bool fold(const WNode &v)
	{
		if (!v.n)
			return true;
		n++;
		const double nn = (double) n;
		delta1 = v.delta1 - mean1;
		mean1 += delta1 / nn;
		if (KIND == K_VAR) {
			m2 += delta1 * (v.delta1 - mean1);
			return true;
		}
		delta2 = v.delta2 - mean2;
		mean2 += delta2 / nn;
		if (KIND == K_COV) {
			m2 += delta1 * (v.delta2 - mean2);
			return true;
		}
		const double aux = v.delta2 - mean2;
		up += delta1 * aux;
		down1 += delta1 * (v.delta1 - mean1);
		down2 += delta2 * aux;
		return true;
	}
	// FINALIZE_AGGREGATE_* / the running frames' result step: false on
	// overflow (an infinite accumulator)
	__device__ __forceinline__ bool result(int op, double &out, bool &isnil) const
	{
		if (KIND == K_COR) {
			if (__builtin_isinf(up) || __builtin_isinf(down1) || __builtin_isinf(down2))
				return false;
			const double nn = (double) n;
			if (n != 0 && down1 != 0 && down2 != 0) {
				out = (up / nn) / (sqrt(down1 / nn) * sqrt(down2 / nn));
				isnil = false;
			} else {
				out = __builtin_nan("");
				isnil = true;
			}
			return true;
		}
		if (__builtin_isinf(m2))
			return false;
		const unsigned long long sample = KIND == K_VAR ? ((op & 1) == 0) : (op == 0);
		if (n > sample) {
			const double v = m2 / (double) (n - sample);
			out = KIND == K_VAR && op < 2 ? sqrt(v) : v;
			isnil = false;
		} else {
			out = __builtin_nan("");
			isnil = true;
		}
		return true;
	}
};

// the product node: nil = no value yet (PROD_NUM / PROD_FP,
// COMPUTE_LEVEL0_PROD / COMPUTE_LEVELN_PROD_*)
template <typename T2>
__device__ __forceinline__ T2
pnil()
{
	if constexpr (std::is_same<T2, float>::value)
		return __builtin_nanf("");
	else if constexpr (std::is_same<T2, double>::value)
		return __builtin_nan("");
	else
		return NilOf<T2>::v();
}

template <typename T2>
__device__ __forceinline__ T2
pmax()
{
	if constexpr (std::is_same<T2, float>::value)
		return FLT_MAX;
	else if constexpr (std::is_same<T2, double>::value)
		return DBL_MAX;
	else if constexpr (std::is_same<T2, hge>::value)
		return (hge) (((uhge) 1 << 127) - 1);
	else
		return std::numeric_limits<T2>::max();
}

// x * y within [-max, max] of hge (OP_WITH_CHECK with __builtin_mul_overflow
// and the nil excluded): magnitudes as 64-bit limbs
__device__ __forceinline__ bool
mul_hge(hge x, hge y, hge &r)
{
	const bool neg = (x < 0) != (y < 0);
	const uhge a = x < 0 ? (uhge) 0 - (uhge) x : (uhge) x, b = y < 0 ? (uhge) 0 - (uhge) y : (uhge) y;
	const unsigned long long a1 = (unsigned long long) (a >> 64), a0 = (unsigned long long) a;
	const unsigned long long b1 = (unsigned long long) (b >> 64), b0 = (unsigned long long) b;
	if (a1 && b1)
		return false;
	const uhge cross = (uhge) a1 * b0 + (uhge) a0 * b1;
	if (cross >> 63)
		return false;
	const uhge lo = (uhge) a0 * b0;
	const uhge m = (cross << 64) + lo;
	if (m < lo || (m >> 127))
		return false;
	r = neg ? -(hge) m : (hge) m;
	return true;
}

template <typename T1, typename T2>
struct PNode {
	T2 v;
	using Out = T2;
	__device__ __forceinline__ void zero() { v = pnil<T2>(); }
	__device__ __forceinline__ void leaf(const Cols &c, BUN i)
	{
		const T1 x = ((const T1 *) c.b1)[i];
		v = is_nil(x) ? pnil<T2>() : (T2) x;
	}
	__device__ __forceinline__ bool fold(const PNode &c)
	{
		if (is_nil(c.v))
			return true;
		if (is_nil(v)) {
			v = c.v;
			return true;
		}
		if constexpr (std::is_floating_point<T2>::value) {
			const T2 av = v < 0 ? -v : v, ac = c.v < 0 ? -c.v : c.v;
			if (av > 1 && pmax<T2>() / ac < av)
				return false;
			v *= c.v;
			return true;
		} else if constexpr (std::is_same<T2, hge>::value) {
			return mul_hge(c.v, v, v);
		} else {
			// bte..lng: the exact product in 128 bits, within [-max, max]
			const hge p = (hge) c.v * (hge) v;
			if (p > (hge) pmax<T2>() || p < -(hge) pmax<T2>())
				return false;
			v = (T2) p;
			return true;
		}
	}
	__device__ __forceinline__ bool result(int, T2 &out, bool &isnil) const
	{
		out = v;
		isnil = is_nil(v);
		return true;
	}
};

struct WTree {
	void *lvl[WS_MAX_LEVELS];
	int nlev;
};

// flags: bit 0 overflow, bit 1 a nil result
__device__ __forceinline__ void
wflag(uint32_t *flags, uint32_t f)
{
	if (f)
		atomicOr(flags, f);
}

// frames 3 (forward, per peer group), 4 (backward, per peer group), 5 (the
// partition): one lane per partition
template <typename N>
__global__ __launch_bounds__(64) void
k_ws_replay(Cols c, Starts part, const int8_t *o, int frame, int op, typename N::Out *out, uint32_t *flags)
{
	const BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= part.m)
		return;
	const BUN ps = part.at(k), pe = part.end_of(k);
	uint32_t f = 0;
	N acc;
	acc.zero();
	if (frame == 4) {
		if (pe > ps) {
			BUN l = pe - 1;
			for (BUN j = pe - 1;; j--) {
				N x;
				x.leaf(c, j);
				if (!acc.fold(x)) {
					f |= 1;
					break;
				}
				if (o[j] || j == ps) {
					typename N::Out w;
					bool isnil;
					if (!acc.result(op, w, isnil)) {
						f |= 1;
						break;
					}
					f |= isnil ? 2u : 0u;
					for (;; l--) {
						out[l] = w;
						if (l == j)
							break;
					}
					if (j == ps)
						break;
					l = j - 1;
				}
			}
		}
	} else {
		BUN j = ps;
		for (BUN r = ps; r < pe; r++) {
			N x;
			x.leaf(c, r);
			if (!acc.fold(x)) {
				f |= 1;
				break;
			}
			if (r + 1 == pe || (frame == 3 && o[r + 1])) {
				typename N::Out w;
				bool isnil;
				if (!acc.result(op, w, isnil)) {
					f |= 1;
					break;
				}
				f |= isnil ? 2u : 0u;
				for (; j <= r; j++)
					out[j] = w;
			}
		}
	}
	wflag(flags, f);
}

// frame 6 of the products: each row's own value in the result type
template <typename N>
__global__ __launch_bounds__(256) void
k_ws_row(Cols c, BUN n, typename N::Out *out, uint32_t *flags)
{
	uint32_t f = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		N x;
		x.leaf(c, i);
		bool isnil;
		typename N::Out w;
		x.result(0, w, isnil);
		out[i] = w;
		f |= isnil ? 2u : 0u;
	}
	f = block_reduce(f, [](uint32_t a, uint32_t b) { return a | b; });
	if (threadIdx.x == 0)
		wflag(flags, f);
}

__global__ __launch_bounds__(256) void
k_ws_fill(BUN n, double v, double *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = v;
}

__global__ __launch_bounds__(256) void
k_ws_pidx(Starts part, uint32_t *pidx)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < part.n; i += (BUN) gridDim.x * blockDim.x)
		pidx[i] = (uint32_t) part.idx(i);
}

__global__ __launch_bounds__(256) void
k_ws_maxlen(Starts part, unsigned long long *mx)
{
	unsigned long long v = 0;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < part.m; k += (BUN) gridDim.x * blockDim.x)
		v = max(v, (unsigned long long) (part.end_of(k) - part.at(k)));
	v = block_reduce(v, [](unsigned long long x, unsigned long long y) { return x > y ? x : y; });
	if (threadIdx.x == 0 && v)
		atomicMax(mx, v);
}

// populate_segment_tree, level L >= 1: the thread of the first row a node
// covers folds the node's children in order
template <typename N>
__global__ __launch_bounds__(256) void
k_ws_tree_level(Cols c, Starts part, const uint32_t *pidx, WTree t, int L, uint32_t *flags)
{
	const int sh = 4 * L, shc = sh - 4;
	N *outl = (N *) t.lvl[L];
	const N *child = L > 1 ? (const N *) t.lvl[L - 1] : nullptr;
	uint32_t f = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < part.n; i += (BUN) gridDim.x * blockDim.x) {
		const BUN k = pidx[i], ps = part.at(k);
		const BUN rel = i - ps;
		if (rel & (((BUN) 1 << sh) - 1))
			continue;
		const BUN nc = part.end_of(k) - ps;
		const BUN ncl = (nc + ((BUN) 1 << shc) - 1) >> shc;
		const BUN c0 = (rel >> sh) * 16, c1 = min(c0 + 16, ncl);
		N acc;
		acc.zero();
		for (BUN q = c0; q < c1; q++) {
			N x;
			if (L == 1)
				x.leaf(c, ps + q);
			else
				x = child[(ps >> shc) + k + q];
			if (!acc.fold(x))
				f |= 1;
		}
		outl[(ps >> sh) + k + (rel >> sh)] = acc;
	}
	if (f)
		wflag(flags, f);
}

// compute_on_segment_tree (gdk_analytic.h:97-130) for [s[i], e[i])
template <typename N>
__global__ __launch_bounds__(256) void
k_ws_tree_query(Cols c, Starts part, const uint32_t *pidx, WTree t, const oid *S, const oid *E, int op,
		typename N::Out *out, uint32_t *flags)
{
	uint32_t f = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < part.n; i += (BUN) gridDim.x * blockDim.x) {
		const BUN k = pidx[i], ps = part.at(k), nc = part.end_of(k) - ps;
		BUN begin = S[i] > ps ? min((BUN) S[i] - ps, nc) : 0;
		BUN tend = E[i] > ps ? min((BUN) E[i] - ps, nc) : 0;
		N acc;
		acc.zero();
		bool ok = true;
		if (begin < tend) {
			for (int L = 0; L <= t.nlev; L++) {
				const N *lv = L ? (const N *) t.lvl[L] + ((ps >> (4 * L)) + k) : nullptr;
				auto fold_at = [&](BUN pos) {
					N x;
					if (L == 0)
						x.leaf(c, ps + pos);
					else
						x = lv[pos];
					ok &= acc.fold(x);
				};
				BUN pb = begin / 16, pe = tend / 16;
				if (pb == pe) {
					for (BUN pos = begin; pos < tend; pos++)
						fold_at(pos);
					break;
				}
				const BUN gb = pb * 16;
				if (begin != gb) {
					for (BUN pos = begin; pos < gb + 16; pos++)
						fold_at(pos);
					pb++;
				}
				const BUN ge = pe * 16;
				if (tend != ge)
					for (BUN pos = ge; pos < tend; pos++)
						fold_at(pos);
				begin = pb;
				tend = pe;
			}
		}
		typename N::Out w;
		bool isnil = false;
		if (!ok || !acc.result(op, w, isnil)) {
			f |= 1;
			continue;
		}
		out[i] = w;
		f |= isnil ? 2u : 0u;
	}
	f = block_reduce(f, [](uint32_t a, uint32_t b) { return a | b; });
	if (threadIdx.x == 0)
		wflag(flags, f);
}

// one window function over b1 (b2) into r: N the node, op its result
template <typename N>
int
ws_run(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s, mgdk_bat *e, int op,
       int frame_type, bool stat, double row_const)
{
	using Out = typename N::Out;
	const BUN n = b1->count;
	hipStream_t st = stream();
	Cols c{b1->theap, b2 ? b2->theap : nullptr};
	Out *out = (Out *) r->theap;
	DevBuf fl(64);
	if (!fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 64, st), "memset"))
		return -1;
	mgdk_bat *Sp = nullptr;
	int rc = -1;
	if (frame_type == 6) {
		if (stat) {
			// the row alone: 0 (population) or nil, whatever the value
			// (ANALYTICAL_STDEV_VARIANCE_CURRENT_ROW :787, _COVARIANCE_ :1074,
			// _CORRELATION_ :1312)
			hipLaunchKernelGGL(k_ws_fill, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, n, row_const,
					   (double *) out);
			if (row_const != row_const && !hip_ok(hipMemsetAsync(fl.as<char>(), 2, 1, st), "memset"))
				goto out;
		} else {
			hipLaunchKernelGGL((k_ws_row<N>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, c, n, out,
					   fl.as<uint32_t>());
		}
	} else {
		Starts part;
		if (make_starts(p ? (const int8_t *) p->theap : nullptr, n, part, &Sp) < 0)
			goto out;
		if (frame_type >= 3 && frame_type <= 5) {
			hipLaunchKernelGGL((k_ws_replay<N>), dim3((unsigned) ((part.m + 63) / 64)), dim3(64), 0, st, c, part,
					   frame_type == 5 ? (const int8_t *) nullptr : (const int8_t *) o->theap, frame_type,
					   op, out, fl.as<uint32_t>());
		} else {
			if (n >= 0xffffffffull) {
				seterr("42000!analytic: more than 2^32-1 rows on the device path\n");
				goto out;
			}
			unsigned long long *hm = (unsigned long long *) pinned(8);
			DevBuf mx(64), pidx(n * 4 + 4);
			if (!mx.p || !pidx.p || !hip_ok(hipMemsetAsync(mx.p, 0, 8, st), "memset"))
				goto out;
			hipLaunchKernelGGL(k_ws_maxlen, dim3(grid_for(part.m, 1024, 1024)), dim3(256), 0, st, part,
					   mx.as<unsigned long long>());
			hipLaunchKernelGGL(k_ws_pidx, dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, part,
					   pidx.as<uint32_t>());
			if (!hip_ok(hipMemcpyAsync(hm, mx.p, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
				goto out;
			WTree t{};
			int nlev = 1;
			while (nlev < WS_MAX_LEVELS - 1 && ((*hm - 1) >> (4 * nlev)) > 0)
				nlev++;
			t.nlev = nlev;
			size_t tot = 0, offs[WS_MAX_LEVELS] = {0};
			for (int L = 1; L <= nlev; L++) {
				offs[L] = tot;
				tot += ((n >> (4 * L)) + part.m + 1) * sizeof(N);
				tot = (tot + 255) & ~(size_t) 255;
			}
			DevBuf tree(tot);
			if (!tree.p)
				goto out;
			for (int L = 1; L <= nlev; L++)
				t.lvl[L] = tree.as<char>() + offs[L];
			for (int L = 1; L <= nlev; L++)
				hipLaunchKernelGGL((k_ws_tree_level<N>), dim3(grid_for(n, 1024, 8192)), dim3(256), 0, st, c, part,
						   pidx.as<uint32_t>(), t, L, fl.as<uint32_t>());
			hipLaunchKernelGGL((k_ws_tree_query<N>), dim3(grid_for(n, 256, 16384)), dim3(256), 0, st, c, part,
					   pidx.as<uint32_t>(), t, (const oid *) s->theap, (const oid *) e->theap, op, out,
					   fl.as<uint32_t>());
			if (!sync())
				goto out;
		}
	}
	{
		uint32_t *h = (uint32_t *) pinned(16);
		if (!hip_ok(hipMemcpyAsync(h, fl.p, 4, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			goto out;
		if (h[0] & 1) {
			seterr("22003!overflow in calculation.\n");
			goto out;
		}
		r->count = n;
		r->tnil = (h[0] & 2) != 0;
		r->tnonil = (h[0] & 2) == 0;
		r->tsorted = r->trevsorted = r->tkey = n <= 1;
		rc = 0;
	}
out:
	mgdk_BBPunfix(Sp);
	return rc;
}

int
ws_check(const char *fn, mgdk_bat *r, mgdk_bat *o, mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s, mgdk_bat *e,
	 int frame_type, int rtype)
{
	if (r == nullptr || b1 == nullptr) {
		seterr("%s: NULL argument", fn);
		return -1;
	}
	const BUN n = b1->count;
	if (b2 && (b2->count != n || b2->ttype != b1->ttype)) {
		seterr("%s: b1 and b2 must be aligned", fn);
		return -1;
	}
	if (r->ttype != rtype) {
		seterr("%s: r must be a %s BAT", fn, atomname(rtype));
		return -1;
	}
	if (n && r->theap == nullptr) {
		seterr("analytic: result BAT has no heap");
		return -1;
	}
	if ((frame_type == 3 || frame_type == 4) && n && (o == nullptr || o->count < n)) {
		seterr("%s: frames 3 and 4 need the peer bits o", fn);
		return -1;
	}
	if (!(frame_type >= 3 && frame_type <= 6) && n &&
	    (s == nullptr || e == nullptr || s->count < n || e->count < n || basetype(s->ttype) != MGDK_oid ||
	     basetype(e->ttype) != MGDK_oid)) {
		seterr("%s: frame bounds s / e must be oid BATs of the column's length", fn);
		return -1;
	}
	return 0;
}

// GDK_ANALYTICAL_STDEV_VARIANCE / GDK_ANALYTICAL_COVARIANCE /
// GDKanalytical_correlation
int
stat_run(const char *fn, const char *desc, int kind, int op, mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b1,
	 mgdk_bat *b2, mgdk_bat *s, mgdk_bat *e, int tpe, int frame_type)
{
	if (ws_check(fn, r, o, b1, b2, s, e, frame_type, MGDK_dbl) < 0)
		return -1;
	const int bt = tpe;
	if (b1->ttype != tpe) {
		seterr("%s: b must be of type tpe", fn);
		return -1;
	}
	const BUN n = b1->count;
	if (n == 0) {
		r->count = 0;
		r->tnil = 0;
		r->tnonil = 1;
		return 0;
	}
	ProfScope prof("analytic_stats");
	const bool sample = kind == K_VAR ? (op & 1) == 0 : op == 0;
	const double rowc = kind == K_COR || sample ? __builtin_nan("") : 0.0;
#define WS_T(T)                                                                                             \
	(kind == K_VAR   ? ws_run<WNode<T, K_VAR>>(r, p, o, b1, b2, s, e, op, frame_type, true, rowc)           \
	 : kind == K_COV ? ws_run<WNode<T, K_COV>>(r, p, o, b1, b2, s, e, op, frame_type, true, rowc)           \
			 : ws_run<WNode<T, K_COR>>(r, p, o, b1, b2, s, e, op, frame_type, true, rowc))
	switch (bt) {
	case MGDK_bte: return WS_T(int8_t);
	case MGDK_sht: return WS_T(int16_t);
	case MGDK_int: return WS_T(int32_t);
	case MGDK_lng: return WS_T(int64_t);
	case MGDK_hge: return WS_T(hge);
	case MGDK_flt: return WS_T(float);
	case MGDK_dbl: return WS_T(double);
	}
#undef WS_T
	seterr("42000!%s of type %s unsupported.\n", desc, atomname(tpe));
	return -1;
}

}  // namespace

extern "C" {

int
mgdk_GDKanalytical_stddev_samp(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
			       int frame_type)
{
	return stat_run("GDKanalytical_stddev_samp", "standard deviation", K_VAR, 0, r, p, o, b, nullptr, s, e, tpe,
			frame_type);
}

int
mgdk_GDKanalytical_stddev_pop(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
			      int frame_type)
{
	return stat_run("GDKanalytical_stddev_pop", "standard deviation", K_VAR, 1, r, p, o, b, nullptr, s, e, tpe,
			frame_type);
}

int
mgdk_GDKanalytical_variance_samp(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e,
				 int tpe, int frame_type)
{
	return stat_run("GDKanalytical_variance_samp", "variance", K_VAR, 2, r, p, o, b, nullptr, s, e, tpe, frame_type);
}

int
mgdk_GDKanalytical_variance_pop(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tpe,
				int frame_type)
{
	return stat_run("GDKanalytical_variance_pop", "variance", K_VAR, 3, r, p, o, b, nullptr, s, e, tpe, frame_type);
}

int
mgdk_GDKanalytical_covariance_samp(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s,
				   mgdk_bat *e, int tpe, int frame_type)
{
	return stat_run("GDKanalytical_covariance_samp", "covariance", K_COV, 0, r, p, o, b1, b2, s, e, tpe,
			frame_type);
}

int
mgdk_GDKanalytical_covariance_pop(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s,
				  mgdk_bat *e, int tpe, int frame_type)
{
	return stat_run("GDKanalytical_covariance_pop", "covariance", K_COV, 1, r, p, o, b1, b2, s, e, tpe, frame_type);
}

int
mgdk_GDKanalytical_correlation(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s,
			       mgdk_bat *e, int tpe, int frame_type)
{
	return stat_run("GDKanalytical_correlation", "correlation", K_COR, 0, r, p, o, b1, b2, s, e, tpe, frame_type);
}

// GDKanalyticalprod (gdk_analytic_func.c:2479; ANALYTICAL_PROD_BRANCHES :2379)
int
mgdk_GDKanalyticalprod(mgdk_bat *r, mgdk_bat *p, mgdk_bat *o, mgdk_bat *b, mgdk_bat *s, mgdk_bat *e, int tp1,
		       int tp2, int frame_type)
{
	if (r == nullptr || b == nullptr) {
		seterr("GDKanalyticalprod: NULL argument");
		return -1;
	}
	if (b->ttype != tp1) {
		seterr("GDKanalyticalprod: b must be of type tp1");
		return -1;
	}
	if (ws_check("GDKanalyticalprod", r, o, b, nullptr, s, e, frame_type, tp2) < 0)
		return -1;
	if (b->count == 0) {
		r->count = 0;
		r->tnil = 0;
		r->tnonil = 1;
		return 0;
	}
	ProfScope prof("analytic_prod");
#define WP(T1, T2) return ws_run<PNode<T1, T2>>(r, p, o, b, nullptr, s, e, 0, frame_type, false, 0.0)
	switch (tp2) {
	case MGDK_bte:
		if (tp1 == MGDK_bte) WP(int8_t, int8_t);
		break;
	case MGDK_sht:
		if (tp1 == MGDK_bte) WP(int8_t, int16_t);
		if (tp1 == MGDK_sht) WP(int16_t, int16_t);
		break;
	case MGDK_int:
		if (tp1 == MGDK_bte) WP(int8_t, int32_t);
		if (tp1 == MGDK_sht) WP(int16_t, int32_t);
		if (tp1 == MGDK_int) WP(int32_t, int32_t);
		break;
	case MGDK_lng:
		if (tp1 == MGDK_bte) WP(int8_t, int64_t);
		if (tp1 == MGDK_sht) WP(int16_t, int64_t);
		if (tp1 == MGDK_int) WP(int32_t, int64_t);
		if (tp1 == MGDK_lng) WP(int64_t, int64_t);
		break;
	case MGDK_hge:
		if (tp1 == MGDK_bte) WP(int8_t, hge);
		if (tp1 == MGDK_sht) WP(int16_t, hge);
		if (tp1 == MGDK_int) WP(int32_t, hge);
		if (tp1 == MGDK_lng) WP(int64_t, hge);
		if (tp1 == MGDK_hge) WP(hge, hge);
		break;
	case MGDK_flt:
		if (tp1 == MGDK_flt) WP(float, float);
		break;
	case MGDK_dbl:
		if (tp1 == MGDK_flt) WP(float, double);
		if (tp1 == MGDK_dbl) WP(double, double);
		break;
	}
#undef WP
	seterr("42000!type combination (prod(%s)->%s) not supported.\n", atomname(tp1), atomname(tp2));
	return -1;
}

}  // extern "C"
