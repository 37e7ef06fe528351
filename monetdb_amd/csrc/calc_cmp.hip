// calc_cmp.hip -- BATcalc comparisons, between, BATconvert, NOT, division and
// modulo on the MI355X.
//
// Semantics (restated, not translated):
//   compare  gdk/gdk_calc_compare.h:15-995 with the operators of
//            gdk_calc_compare_{lt,le,gt,ge,eq,ne,generic}.c: one bit (bte for
//            cmp) per candidate pair, nil if either side is nil unless the
//            inputs are known nil-free (then raw values are compared, NaN
//            included) or nil_matches (EQ / NE compare the nil flags); mixed
//            types compare after C's usual arithmetic conversions (int vs flt
//            in flt, lng vs dbl in dbl); void / oid operands as :36-72 and
//            :638-684.
//   between  gdk/gdk_calc.c:3770-4206: three-valued BETWEEN with symmetric,
//            linc, hinc, nils_false and anti.
//   convert  gdk/gdk_calc_convert.c:98-660, :870-980, :1415-1548: integer
//            rescaling with round-half-away DIVIDE and the range / DECIMAL
//            precision checks, integer -> float with the scale divisor,
//            float -> integer as (TYPE2) roundl((long double) v * 10^scale):
//            the product is formed exactly in 128-bit integers and rounded to
//            the x87 64-bit significand first, so the result is the one the
//            reference's 80-bit arithmetic gives; -> bit, -> oid, void ->.
//   not      gdk/gdk_calc.c:41-146.
//   div/mod  gdk/gdk_calc_div.c:21-140, gdk/gdk_calc_mod.c:21-110 for the
//            type combinations the reference instantiates.
//
// Every operator is one streaming pass (grid-stride, one element per lane per
// step: loads of 1..16 bytes and a 1-byte result are HBM bound); the first
// failing candidate (overflow, division by zero) is found with one
// atomicMin per workgroup and reported with the reference's message.
#include <cfloat>
#include <cmath>
#include <cstdio>

#include <string>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

// ---- operands ----------------------------------------------------------
// tp: MGDK_{bte,sht,int,lng,hge,flt,dbl,oid,void} after ATOMbasetype
struct Opnd {
	const void *base;   // tail (nullptr: constant)
	int tp;
	bool dense;         // candidates dense: position = off + i
	oid off;
	const oid *oids;    // materialised candidates
	oid hseq;
	oid seq;            // void: tseqbase
	hge ci;             // constant
	double cd;
	float cf;
	bool cnil;
	bool cst;           // a constant operand (incr == false in the reference)
};

struct Num {
	hge i;
	double d;
	float f;
	bool nil;
};

__device__ __forceinline__ float
hge_to_flt(hge v)
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

__device__ __forceinline__ BUN
posof(const Opnd &o, BUN i)
{
	return o.dense ? o.off + i : o.oids[i] - o.hseq;
}

__device__ __forceinline__ Num
ldval(int tp, const void *base, BUN p)
{
	Num v{};
	switch (tp) {
	case MGDK_bte: { int8_t x = ((const int8_t *) base)[p]; v.i = x; v.nil = x == INT8_MIN; break; }
	case MGDK_sht: { int16_t x = ((const int16_t *) base)[p]; v.i = x; v.nil = x == INT16_MIN; break; }
	case MGDK_int: { int32_t x = ((const int32_t *) base)[p]; v.i = x; v.nil = x == INT32_MIN; break; }
	case MGDK_lng: { int64_t x = ((const int64_t *) base)[p]; v.i = x; v.nil = x == INT64_MIN; break; }
	case MGDK_oid: { uint64_t x = ((const uint64_t *) base)[p]; v.i = (hge) x; v.nil = x == MGDK_OID_NIL; break; }
	case MGDK_hge: { hge x = ((const hge *) base)[p]; v.i = x; v.nil = is_nil(x); break; }
	case MGDK_flt: { float x = ((const float *) base)[p]; v.f = x; v.nil = x != x; break; }
	default: { double x = ((const double *) base)[p]; v.d = x; v.nil = x != x; break; }
	}
	return v;
}

// value of operand o for the i-th candidate
__device__ __forceinline__ Num
opval(const Opnd &o, BUN i)
{
	if (o.cst) {
		Num v{};
		v.i = o.ci;
		v.d = o.cd;
		v.f = o.cf;
		v.nil = o.cnil;
		return v;
	}
	const BUN p = posof(o, i);
	if (o.tp == MGDK_void) {
		Num v{};
		v.i = (hge) (o.seq + p);
		v.nil = o.seq == MGDK_OID_NIL;
		return v;
	}
	return ldval(o.tp, o.base, p);
}

__device__ __forceinline__ double
as_dbl(const Num &v, int tp)
{
	return tp == MGDK_dbl ? v.d : tp == MGDK_flt ? (double) v.f : hge_to_dbl(v.i);
}

__device__ __forceinline__ float
as_flt(const Num &v, int tp)
{
	return tp == MGDK_flt ? v.f : hge_to_flt(v.i);
}

enum { OP_LT, OP_LE, OP_GT, OP_GE, OP_EQ, OP_NE, OP_CMP };
// compare domain: the type C's usual arithmetic conversions pick
enum { D_INT, D_FLT, D_DBL, D_OID };

template <int OP>
__device__ __forceinline__ int8_t
opres(bool lt, bool gt, bool le, bool ge, bool eq)
{
	switch (OP) {
	case OP_LT: return lt;
	case OP_LE: return le;
	case OP_GT: return gt;
	case OP_GE: return ge;
	case OP_EQ: return eq;
	case OP_NE: return !eq;
	default: return (int8_t) ((int) gt - (int) lt);
	}
}

template <int OP, int D>
__device__ __forceinline__ int8_t
apply(const Num &a, int ta, const Num &b, int tb)
{
	if (D == D_DBL) {
		const double x = as_dbl(a, ta), y = as_dbl(b, tb);
		return opres<OP>(x < y, x > y, x <= y, x >= y, x == y);
	} else if (D == D_FLT) {
		const float x = as_flt(a, ta), y = as_flt(b, tb);
		return opres<OP>(x < y, x > y, x <= y, x >= y, x == y);
	} else if (D == D_OID) {
		const uint64_t x = (uint64_t) a.i, y = (uint64_t) b.i;
		return opres<OP>(x < y, x > y, x <= y, x >= y, x == y);
	} else {
		const hge x = a.i, y = b.i;
		return opres<OP>(x < y, x > y, x <= y, x >= y, x == y);
	}
}

template <int OP>
__device__ __forceinline__ int8_t
apply_flags(bool x, bool y)
{
	return opres<OP>(x < y, x > y, x <= y, x >= y, x == y);
}

// mode 0: numeric / oid-oid (BINARY_3TYPE_FUNC{,_nonil,_nilmatch});
// mode 1: left void (gdk_calc_compare.h:36-72); mode 2: oid vs void (:638-671)
template <int OP, int D>
__global__ __launch_bounds__(256) void
k_cmp(Opnd a, Opnd b, int8_t *out, BUN n, int mode, bool nonil, bool nilmatch, oid r0,
      unsigned long long *nils)
{
	unsigned long long my = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		int8_t res;
		if (mode == 0) {
			const Num x = opval(a, i), y = opval(b, i);
			if (nonil)
				res = apply<OP, D>(x, a.tp, y, b.tp);
			else if (x.nil || y.nil)
				res = nilmatch ? apply_flags<OP>(x.nil, y.nil) : (int8_t) INT8_MIN;
			else
				res = apply<OP, D>(x, a.tp, y, b.tp);
		} else if (mode == 1) {
			const oid v = a.seq;
			Num x{}, y{};
			if (v == MGDK_OID_NIL || b.tp == MGDK_void) {
				x.i = (hge) v;
				y.i = (hge) r0;
				if (v == MGDK_OID_NIL || r0 == MGDK_OID_NIL)
					res = nilmatch ? apply_flags<OP>(v == MGDK_OID_NIL, r0 == MGDK_OID_NIL) : (int8_t) INT8_MIN;
				else
					res = apply<OP, D_OID>(x, MGDK_oid, y, MGDK_oid);
			} else {
				const oid w = b.cst ? (oid) b.ci : ((const oid *) b.base)[posof(b, i)];
				if (w == MGDK_OID_NIL) {
					res = nilmatch ? apply_flags<OP>(false, true) : (int8_t) INT8_MIN;
				} else {
					x.i = (hge) (v + (a.cst ? 0 : posof(a, i)));
					y.i = (hge) w;
					res = apply<OP, D_OID>(x, MGDK_oid, y, MGDK_oid);
				}
			}
		} else {
			const oid v = r0;
			const oid xl = a.cst ? (oid) a.ci : ((const oid *) a.base)[posof(a, i)];
			Num x{}, y{};
			if (v == MGDK_OID_NIL) {
				res = nilmatch ? apply_flags<OP>(xl == MGDK_OID_NIL, true) : (int8_t) INT8_MIN;
			} else if (xl == MGDK_OID_NIL) {
				res = nilmatch ? apply_flags<OP>(true, false) : (int8_t) INT8_MIN;
			} else {
				x.i = (hge) xl;
				y.i = (hge) (v + (b.cst ? 0 : posof(b, i)));
				res = apply<OP, D_OID>(x, MGDK_oid, y, MGDK_oid);
			}
		}
		out[i] = res;
		my += res == (int8_t) INT8_MIN;
	}
	my = block_reduce(my, [](unsigned long long x, unsigned long long y) { return x + y; });
	if (threadIdx.x == 0 && my)
		atomicAdd(nils, my);
}

int
optype(const mgdk_bat *b)
{
	// ATOMtype(t) == TYPE_oid ? t : ATOMbasetype(t) (gdk_calc_compare.h:866)
	return b->ttype == MGDK_void || b->ttype == MGDK_oid ? b->ttype : basetype(b->ttype);
}

bool
is_int_t(int t)
{
	return t == MGDK_bte || t == MGDK_sht || t == MGDK_int || t == MGDK_lng || t == MGDK_hge;
}

bool
is_num_t(int t)
{
	return is_int_t(t) || t == MGDK_flt || t == MGDK_dbl;
}

// constant value of host memory v of type t (base type)
void
set_cst(Opnd &o, const void *v, int t)
{
	o.base = nullptr;
	o.tp = t;
	o.cst = true;
	switch (t) {
	case MGDK_bte: { int8_t x; memcpy(&x, v, 1); o.ci = x; o.cnil = x == INT8_MIN; break; }
	case MGDK_sht: { int16_t x; memcpy(&x, v, 2); o.ci = x; o.cnil = x == INT16_MIN; break; }
	case MGDK_int: { int32_t x; memcpy(&x, v, 4); o.ci = x; o.cnil = x == INT32_MIN; break; }
	case MGDK_lng: { int64_t x; memcpy(&x, v, 8); o.ci = x; o.cnil = x == INT64_MIN; break; }
	case MGDK_oid: case MGDK_void: { uint64_t x; memcpy(&x, v, 8); o.ci = (hge) x; o.seq = x; o.cnil = x == MGDK_OID_NIL; break; }
	case MGDK_hge: { hge x; memcpy(&x, v, 16); o.ci = x; o.cnil = is_nil(x); break; }
	case MGDK_flt: { float x; memcpy(&x, v, 4); o.cf = x; o.cnil = x != x; break; }
	case MGDK_dbl: { double x; memcpy(&x, v, 8); o.cd = x; o.cnil = x != x; break; }
	}
}

void
set_bat(Opnd &o, const mgdk_bat *b, const Cand &c, int tp)
{
	o.base = b->ttype == MGDK_void ? nullptr : b->theap;
	o.tp = tp;
	o.dense = c.dense;
	o.off = c.dense ? c.seq - b->hseqbase : 0;
	o.oids = c.oids;
	o.hseq = b->hseqbase;
	o.seq = b->tseqbase;
}

unsigned long long *
counters(int k)
{
	unsigned long long *m = (unsigned long long *) meta_buf();
	unsigned long long init[4] = {0, ~0ull, 0, 0};
	if (!hip_ok(hipMemcpyAsync(m, init, 8 * (k < 4 ? k : 4), hipMemcpyHostToDevice, stream()), "memcpy"))
		return nullptr;
	return m;
}

bool
read_counters(unsigned long long *m, unsigned long long *h, int k)
{
	unsigned long long *p = (unsigned long long *) pinned(64);
	if (p == nullptr || !hip_ok(hipMemcpyAsync(p, m, 8 * k, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return false;
	memcpy(h, p, 8 * k);
	return true;
}

void
set_cmp_props(mgdk_bat *bn, BUN n, BUN nils)
{
	bn->count = n;
	bn->tsorted = n <= 1 || nils == n;
	bn->trevsorted = n <= 1 || nils == n;
	bn->tkey = n <= 1;
	bn->tnil = nils != 0;
	bn->tnonil = nils == 0;
}

const char *const cmpfunc[] = {
	"BATcalclt", "BATcalcle", "BATcalcgt", "BATcalcge", "BATcalceq", "BATcalcne", "BATcalccmp",
};

template <int OP>
void
launch_cmp(int d, dim3 g, Opnd &A, Opnd &B, int8_t *out, BUN n, int mode, bool nonil, bool nm, oid r0,
	   unsigned long long *nils)
{
	switch (d) {
	case D_INT: hipLaunchKernelGGL((k_cmp<OP, D_INT>), g, dim3(256), 0, stream(), A, B, out, n, mode, nonil, nm, r0, nils); break;
	case D_FLT: hipLaunchKernelGGL((k_cmp<OP, D_FLT>), g, dim3(256), 0, stream(), A, B, out, n, mode, nonil, nm, r0, nils); break;
	case D_DBL: hipLaunchKernelGGL((k_cmp<OP, D_DBL>), g, dim3(256), 0, stream(), A, B, out, n, mode, nonil, nm, r0, nils); break;
	default: hipLaunchKernelGGL((k_cmp<OP, D_OID>), g, dim3(256), 0, stream(), A, B, out, n, mode, nonil, nm, r0, nils); break;
	}
}

// BATcalcop / BATcalcopcst / BATcalccstop (gdk_calc_compare.h:827-964)
mgdk_bat *
calccmp(int op, mgdk_bat *b1, const void *v1, int t1, mgdk_bat *b2, const void *v2, int t2,
	mgdk_bat *s1, mgdk_bat *s2, bool nil_matches)
{
	ProfScope prof("calccmp");
	Cand c1{}, c2{};
	mgdk_bat *bb = b1 ? b1 : b2;
	Cand ci{};
	if (b1 && b2) {
		if (cand_init(&c1, b1, s1) < 0 || cand_init(&c2, b2, s2) < 0)
			return nullptr;
		const oid h1 = s1 ? s1->hseqbase : b1->hseqbase, h2 = s2 ? s2->hseqbase : b2->hseqbase;
		if (c1.n != c2.n || h1 != h2) {
			seterr("inputs not the same size.\n");
			return nullptr;
		}
		ci = c1;
	} else {
		if (cand_init(&ci, bb, s1) < 0)
			return nullptr;
		if (b1)
			c1 = ci;
		else
			c2 = ci;
	}
	const int rt = op == OP_CMP ? MGDK_bte : MGDK_bit;
	const oid hseq = s1 ? s1->hseqbase : bb->hseqbase;
	const BUN n = ci.n;
	if (n == 0) {
		mgdk_bat *bn = newbat(hseq, rt, 0);
		if (bn)
			bn->count = 0;
		return bn;
	}
	const bool nm = nil_matches && (op == OP_EQ || op == OP_NE);
	if (b1 && b2 && b1->ttype == MGDK_void && b2->ttype == MGDK_void && c1.dense && c2.dense) {
		// BATconstant shortcut (gdk_calc_compare.h:848-861)
		int8_t res;
		if ((b1->tseqbase == MGDK_OID_NIL || b2->tseqbase == MGDK_OID_NIL) && !nm) {
			res = INT8_MIN;
		} else {
			const oid x = b1->tseqbase + c1.seq, y = b2->tseqbase + c2.seq;
			const int lt = x < y, gt = x > y;
			switch (op) {
			case OP_LT: res = lt; break;
			case OP_LE: res = x <= y; break;
			case OP_GT: res = gt; break;
			case OP_GE: res = x >= y; break;
			case OP_EQ: res = x == y; break;
			case OP_NE: res = x != y; break;
			default: res = (int8_t) (gt - lt); break;
			}
		}
		mgdk_bat *bn = mgdk_BATconstant(b1->hseqbase, rt, &res, n);
		if (bn) {
			bn->tnil = res == INT8_MIN;
			bn->tnonil = !bn->tnil;
		}
		return bn;
	}
	Opnd A{}, B{};
	int tA = b1 ? optype(b1) : (t1 == MGDK_void || t1 == MGDK_oid ? t1 : basetype(t1));
	int tB = b2 ? optype(b2) : (t2 == MGDK_void || t2 == MGDK_oid ? t2 : basetype(t2));
	if (!((tA == MGDK_void && (tB == MGDK_oid || tB == MGDK_void)) || (tA == MGDK_oid && (tB == MGDK_oid || tB == MGDK_void)) ||
	      (is_num_t(tA) && is_num_t(tB)))) {
		seterr("%s: bad input types %s,%s.\n", cmpfunc[op], atomname(tA), atomname(tB));
		return nullptr;
	}
	if (b1)
		set_bat(A, b1, c1, tA);
	else
		set_cst(A, v1, tA);
	if (b2)
		set_bat(B, b2, c2, tB);
	else
		set_cst(B, v2, tB);
	bool nonil;
	if (b1 && b2)
		nonil = b1->tnonil && b2->tnonil;
	else if (b1)
		nonil = b1->tnonil && !B.cnil;
	else
		nonil = b2->tnonil && !A.cnil;
	int mode = 0, d;
	oid r0 = 0;
	if (tA == MGDK_void) {
		mode = 1;
		d = D_OID;
		if (!b1)
			A.seq = (oid) A.ci;
		// *(const oid *) rgt: the right tseqbase, the first oid of its tail,
		// or the constant
		if (b2 == nullptr)
			r0 = (oid) B.ci;
		else if (b2->ttype == MGDK_void)
			r0 = b2->tseqbase;
		else if (oid_at(b2, 0, &r0) < 0)
			return nullptr;
	} else if (tA == MGDK_oid && tB == MGDK_void) {
		mode = 2;
		d = D_OID;
		r0 = b2 ? b2->tseqbase : (oid) B.ci;
	} else if (tA == MGDK_dbl || tB == MGDK_dbl) {
		d = D_DBL;
	} else if (tA == MGDK_flt || tB == MGDK_flt) {
		d = D_FLT;
	} else if (tA == MGDK_oid || tB == MGDK_oid) {
		d = D_OID;
	} else {
		d = D_INT;
	}
	mgdk_bat *bn = newbat(hseq, rt, n);
	if (bn == nullptr)
		return nullptr;
	unsigned long long *m = counters(1);
	if (m == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	dim3 g(grid_for(n, 256 * 4, 256 * 64));
	int8_t *out = (int8_t *) bn->theap;
	switch (op) {
	case OP_LT: launch_cmp<OP_LT>(d, g, A, B, out, n, mode, nonil, nm, r0, m); break;
	case OP_LE: launch_cmp<OP_LE>(d, g, A, B, out, n, mode, nonil, nm, r0, m); break;
	case OP_GT: launch_cmp<OP_GT>(d, g, A, B, out, n, mode, nonil, nm, r0, m); break;
	case OP_GE: launch_cmp<OP_GE>(d, g, A, B, out, n, mode, nonil, nm, r0, m); break;
	case OP_EQ: launch_cmp<OP_EQ>(d, g, A, B, out, n, mode, nonil, nm, r0, m); break;
	case OP_NE: launch_cmp<OP_NE>(d, g, A, B, out, n, mode, nonil, nm, r0, m); break;
	default: launch_cmp<OP_CMP>(d, g, A, B, out, n, mode, nonil, nm, r0, m); break;
	}
	unsigned long long h[1];
	if (!read_counters(m, h, 1)) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	set_cmp_props(bn, n, h[0]);
	return bn;
}

// ---- between (gdk/gdk_calc.c:3770-4206) ----------------------------------
__device__ __forceinline__ int8_t or3(int8_t a, int8_t b) { return a == 1 || b == 1 ? 1 : a == INT8_MIN || b == INT8_MIN ? INT8_MIN : 0; }
__device__ __forceinline__ int8_t and3(int8_t a, int8_t b) { return a == 0 || b == 0 ? 0 : a == INT8_MIN || b == INT8_MIN ? INT8_MIN : 1; }

template <int D>
__device__ __forceinline__ int8_t
less3(const Num &a, const Num &b, int t, bool inc)
{
	if (a.nil || b.nil)
		return INT8_MIN;
	return apply<OP_LT, D>(a, t, b, t) || (inc && apply<OP_EQ, D>(a, t, b, t));
}

template <int D>
__device__ __forceinline__ int8_t
between3(const Num &v, const Num &lo, bool linc, const Num &hi, bool hinc, int t)
{
	return and3(less3<D>(lo, v, t, linc), less3<D>(v, hi, t, hinc));
}

template <int D>
__global__ __launch_bounds__(256) void
k_between(Opnd b, Opnd lo, Opnd hi, int8_t *out, BUN n, int t, bool symmetric, bool linc, bool hinc,
	  bool nils_false, bool anti, unsigned long long *nils)
{
	unsigned long long my = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const Num v = opval(b, i), l = opval(lo, i), h = opval(hi, i);
		int8_t r;
		if (v.nil) {
			r = nils_false ? 0 : INT8_MIN;
		} else {
			r = symmetric ? or3(between3<D>(v, l, linc, h, hinc, t), between3<D>(v, h, hinc, l, linc, t))
				      : between3<D>(v, l, linc, h, hinc, t);
			if (anti)
				r = r == INT8_MIN ? INT8_MIN : !r;
		}
		out[i] = r;
		my += r == INT8_MIN;
	}
	my = block_reduce(my, [](unsigned long long x, unsigned long long y) { return x + y; });
	if (threadIdx.x == 0 && my)
		atomicAdd(nils, my);
}

mgdk_bat *
calcbetween(mgdk_bat *b, mgdk_bat *lo, const void *clo, mgdk_bat *hi, const void *chi, int ct,
	    mgdk_bat *s, mgdk_bat *slo, mgdk_bat *shi, bool symmetric, bool linc, bool hinc,
	    bool nils_false, bool anti)
{
	ProfScope prof("calcbetween");
	if ((lo == nullptr || hi == nullptr) && basetype(b->ttype) != basetype(ct)) {
		seterr("incompatible input types.\n");
		return nullptr;
	}
	Cand ci{}, cl{}, chc{};
	if (cand_init(&ci, b, s) < 0 || (lo && cand_init(&cl, lo, slo) < 0) || (hi && cand_init(&chc, hi, shi) < 0))
		return nullptr;
	const oid hseq = s ? s->hseqbase : b->hseqbase;
	if ((lo && (cl.n != ci.n || (slo ? slo->hseqbase : lo->hseqbase) != hseq)) ||
	    (hi && (chc.n != ci.n || (shi ? shi->hseqbase : hi->hseqbase) != hseq))) {
		seterr("inputs not the same size.\n");
		return nullptr;
	}
	int t = basetype(b->ttype);
	if (t != MGDK_void && ((lo && basetype(lo->ttype) != t) || (hi && basetype(hi->ttype) != t))) {
		seterr("incompatible input types.\n");
		return nullptr;
	}
	if (t != MGDK_void && t != MGDK_oid && !is_num_t(t)) {
		seterr("BATcalcbetween: bad input type %s.\n", atomname(b->ttype));
		return nullptr;
	}
	const bool anyvoid = b->ttype == MGDK_void || (lo && lo->ttype == MGDK_void) || (hi && hi->ttype == MGDK_void);
	if (anyvoid && ((b->ttype != MGDK_void && b->ttype != MGDK_oid) || (lo && lo->ttype != MGDK_void && lo->ttype != MGDK_oid) ||
			(hi && hi->ttype != MGDK_void && hi->ttype != MGDK_oid))) {
		// BUNtoid over every operand (gdk_calc.c:4025-4036): oid / void only
		seterr("incompatible input types.\n");
		return nullptr;
	}
	const BUN n = ci.n;
	const bool vd = b->ttype == MGDK_void || (lo && lo->ttype == MGDK_void) || (hi && hi->ttype == MGDK_void);
	Opnd B{}, L{}, H{};
	const int tt = vd || t == MGDK_oid ? MGDK_oid : t;
	set_bat(B, b, ci, b->ttype == MGDK_void ? MGDK_void : tt);
	if (lo)
		set_bat(L, lo, cl, lo->ttype == MGDK_void ? MGDK_void : tt);
	else
		set_cst(L, clo, tt);
	if (hi)
		set_bat(H, hi, chc, hi->ttype == MGDK_void ? MGDK_void : tt);
	else
		set_cst(H, chi, tt);
	if (lo && hi && b->ttype == MGDK_void && lo->ttype == MGDK_void && hi->ttype == MGDK_void) {
		// all three dense (gdk_calc.c:4012-4019): one constant
		auto three = [](oid v, oid l, oid h, bool sym, bool li, bool hc, bool nf, bool an) -> int8_t {
			auto l3 = [](oid a, oid b, bool nilab, bool inc) -> int8_t {
				return nilab ? INT8_MIN : (int8_t) (a < b || (inc && a == b));
			};
			auto a3 = [](int8_t a, int8_t b) -> int8_t { return a == 0 || b == 0 ? 0 : a == INT8_MIN || b == INT8_MIN ? INT8_MIN : 1; };
			auto o3 = [](int8_t a, int8_t b) -> int8_t { return a == 1 || b == 1 ? 1 : a == INT8_MIN || b == INT8_MIN ? INT8_MIN : 0; };
			const bool vn = v == MGDK_OID_NIL, ln = l == MGDK_OID_NIL, hn = h == MGDK_OID_NIL;
			if (vn)
				return nf ? 0 : INT8_MIN;
			int8_t r1 = a3(l3(l, v, ln, li), l3(v, h, hn, hc));
			int8_t r = r1;
			if (sym)
				r = o3(r1, a3(l3(h, v, hn, hc), l3(v, l, ln, li)));
			return an ? (r == INT8_MIN ? INT8_MIN : (int8_t) !r) : r;
		};
		int8_t res = three(b->tseqbase, lo->tseqbase, hi->tseqbase, symmetric, linc, hinc, nils_false, anti);
		mgdk_bat *bn = mgdk_BATconstant(hseq, MGDK_bit, &res, n);
		if (bn) {
			bn->tnil = n >= 1 && res == INT8_MIN;
			bn->tnonil = !bn->tnil;
		}
		return bn;
	}
	// a void operand goes through BUNtoid with the result's head at the first
	// candidate (gdk_calc.c:4025, :4116: COLnew(ci.seq, ...))
	mgdk_bat *bn = newbat(vd ? (n ? ci.first : 0) : hseq, MGDK_bit, n);
	if (bn == nullptr)
		return nullptr;
	if (n == 0) {
		bn->count = 0;
		return bn;
	}
	unsigned long long *m = counters(1);
	if (m == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	dim3 g(grid_for(n, 256 * 4, 256 * 64));
	int8_t *out = (int8_t *) bn->theap;
	if (tt == MGDK_dbl)
		hipLaunchKernelGGL((k_between<D_DBL>), g, dim3(256), 0, stream(), B, L, H, out, n, tt, symmetric, linc, hinc, nils_false, anti, m);
	else if (tt == MGDK_flt)
		hipLaunchKernelGGL((k_between<D_FLT>), g, dim3(256), 0, stream(), B, L, H, out, n, tt, symmetric, linc, hinc, nils_false, anti, m);
	else if (vd)
		hipLaunchKernelGGL((k_between<D_OID>), g, dim3(256), 0, stream(), B, L, H, out, n, tt, symmetric, linc, hinc, nils_false, anti, m);
	else
		hipLaunchKernelGGL((k_between<D_INT>), g, dim3(256), 0, stream(), B, L, H, out, n, tt, symmetric, linc, hinc, nils_false, anti, m);
	unsigned long long h[1];
	if (!read_counters(m, h, 1)) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	set_cmp_props(bn, n, h[0]);
	return bn;
}

// ---- BATconvert ----------------------------------------------------------
hge
scale_of(int k)
{
	hge v = 1;
	while (k-- > 0)
		v *= 10;
	return v;
}

hge
imax_of(int t)
{
	switch (t) {
	case MGDK_bte: return INT8_MAX;
	case MGDK_sht: return INT16_MAX;
	case MGDK_int: return INT32_MAX;
	case MGDK_lng: return INT64_MAX;
	default: return (hge) (((uhge) 1 << 127) - 1);
	}
}

int
ibits(int t)
{
	return t == MGDK_bte ? 8 : t == MGDK_sht ? 16 : t == MGDK_int ? 32 : t == MGDK_lng ? 64 : 128;
}

// (TYPE2) roundl((long double) v * mul) for |mul| < 2^60: the product is
// formed exactly (53-bit significand x mul < 2^113), rounded to the x87
// 64-bit significand (nearest even), then rounded half away from zero to an
// integer.  Returns false when the magnitude reaches 2^127.
__device__ bool
x87_round_mul(double v, uint64_t mul, hge &out)
{
	const unsigned long long bits = (unsigned long long) __double_as_longlong(v);
	const bool neg = bits >> 63;
	const int ex = (int) ((bits >> 52) & 0x7ff);
	unsigned long long M = bits & ((1ull << 52) - 1);
	int E;
	if (ex == 0) {
		E = -1074;
	} else {
		M |= 1ull << 52;
		E = ex - 1075;
	}
	uhge P = (uhge) M * mul;
	if (P == 0) {
		out = 0;
		return true;
	}
	const unsigned long long ph = (unsigned long long) (P >> 64);
	const int nb = ph ? 128 - __builtin_clzll(ph) : 64 - __builtin_clzll((unsigned long long) P);
	if (nb > 64) {
		const int sh = nb - 64;
		uhge q = P >> sh;
		const uhge rem = P & (((uhge) 1 << sh) - 1), half = (uhge) 1 << (sh - 1);
		if (rem > half || (rem == half && (q & 1)))
			q++;
		P = q;
		E += sh;
	}
	uhge R;
	if (E >= 0) {
		const unsigned long long rh = (unsigned long long) (P >> 64);
		const int pb = rh ? 128 - __builtin_clzll(rh) : 64 - __builtin_clzll((unsigned long long) P);
		if (pb + E > 127)
			return false;
		R = P << E;
	} else {
		const int s = -E;
		if (s >= 128) {
			R = 0;
		} else {
			R = P >> s;
			const uhge rem = P & (((uhge) 1 << s) - 1), half = (uhge) 1 << (s - 1);
			if (rem >= half)
				R++;
		}
	}
	if (R >> 127)
		return false;
	out = neg ? -(hge) R : (hge) R;
	return true;
}

// kinds of destination
enum { C_INT, C_FLT, C_DBL, C_BIT, C_OID };

struct ConvArgs {
	int st, dt, kind;       // source base type, destination base type
	int ow;                 // output width
	hge div, mul, max, pr;  // integer rescale parameters
	int prec;
	float lim_f;            // (float) max, (double) max for float sources
	double lim_d;
	uint64_t fmul;          // float -> int multiplier (<= 10^18)
};

__device__ __forceinline__ void
st_int(void *base, int w, BUN i, hge v)
{
	switch (w) {
	case 1: ((int8_t *) base)[i] = (int8_t) v; break;
	case 2: ((int16_t *) base)[i] = (int16_t) v; break;
	case 4: ((int32_t *) base)[i] = (int32_t) v; break;
	case 8: ((int64_t *) base)[i] = (int64_t) v; break;
	default: ((hge *) base)[i] = v; break;
	}
}

__device__ __forceinline__ void
st_nil(void *base, int kind, int w, BUN i)
{
	if (kind == C_FLT)
		((float *) base)[i] = __int_as_float(0x7fc00000);
	else if (kind == C_DBL)
		((double *) base)[i] = __longlong_as_double(0x7ff8000000000000ll);
	else if (kind == C_OID)
		((uint64_t *) base)[i] = MGDK_OID_NIL;
	else
		st_int(base, w, i, w == 16 ? (hge) ((uhge) 1 << 127) : -((hge) 1 << (8 * w - 1)));
}

// one element; returns 0 ok, 1 nil, 2 overflow
__device__ __forceinline__ int
conv_elem(const ConvArgs &a, const Num &v, void *out, BUN i)
{
	if (v.nil) {
		st_nil(out, a.kind, a.ow, i);
		return 1;
	}
	const int st = a.st;
	if (a.kind == C_BIT) {
		((int8_t *) out)[i] = st == MGDK_flt ? v.f != 0 : st == MGDK_dbl ? v.d != 0 : v.i != 0;
		return 0;
	}
	if (a.kind == C_OID) {
		uint64_t o;
		if (st == MGDK_flt) {
			if (v.f < 0 || v.f > a.lim_f)
				return 2;
			o = (uint64_t) v.f;
		} else if (st == MGDK_dbl) {
			if (v.d < 0 || v.d > a.lim_d)
				return 2;
			o = (uint64_t) v.d;
		} else {
			if (v.i < 0 || v.i > (hge) INT64_MAX)
				return 2;
			o = (uint64_t) v.i;
		}
		if (o == MGDK_OID_NIL)
			return 2;
		((uint64_t *) out)[i] = o;
		return 0;
	}
	const bool sint = st != MGDK_flt && st != MGDK_dbl;
	if (sint && a.kind == C_INT) {
		hge x = v.i;
		if (a.div > 1)
			x = x < 0 ? -((-x + a.div / 2) / a.div) : (x + a.div / 2) / a.div;
		if (x < -a.max || x > a.max || (a.prec && (x >= a.pr || x <= -a.pr)))
			return 2;
		st_int(out, a.ow, i, x * a.mul);
		return 0;
	}
	if (sint) {
		if (a.kind == C_FLT) {
			const float f = hge_to_flt(v.i);
			((float *) out)[i] = a.div == 1 ? f : f / hge_to_flt(a.div);
		} else {
			const double d = hge_to_dbl(v.i);
			((double *) out)[i] = a.div == 1 ? d : d / hge_to_dbl(a.div);
		}
		return 0;
	}
	if (a.kind == C_FLT || a.kind == C_DBL) {
		if (st == MGDK_dbl && a.kind == C_FLT) {
			if (v.d < -(double) FLT_MAX || v.d > (double) FLT_MAX)
				return 2;
			((float *) out)[i] = (float) v.d;
		} else if (a.kind == C_FLT) {
			((float *) out)[i] = v.f;
		} else {
			((double *) out)[i] = st == MGDK_flt ? (double) v.f : v.d;
		}
		return 0;
	}
	// float -> integer
	if (st == MGDK_flt ? (v.f < -a.lim_f || v.f > a.lim_f) : (v.d < -a.lim_d || v.d > a.lim_d))
		return 2;
	hge r;
	if (!x87_round_mul(st == MGDK_flt ? (double) v.f : v.d, a.fmul, r) || r < -a.max || r > a.max ||
	    (a.prec && (r >= a.pr || r <= -a.pr)))
		return 2;
	st_int(out, a.ow, i, r);
	return 0;
}

__global__ __launch_bounds__(256) void
k_convert(Opnd b, ConvArgs a, void *out, BUN n, unsigned long long *meta)
{
	unsigned long long nils = 0, first = ~0ull;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const int r = conv_elem(a, opval(b, i), out, i);
		nils += r == 1;
		if (r == 2 && i < first)
			first = i;
	}
	nils = block_reduce(nils, [](unsigned long long x, unsigned long long y) { return x + y; });
	first = block_reduce(first, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	if (threadIdx.x == 0) {
		if (nils)
			atomicAdd(meta, nils);
		if (first != ~0ull)
			atomicMin(meta + 1, first);
	}
}

// convert_void_any (gdk_calc_convert.c:870-979): values tseqbase + position
__global__ __launch_bounds__(256) void
k_convert_void(Opnd b, int kind, int ow, uint64_t maxv, void *out, BUN n, unsigned long long *meta)
{
	unsigned long long first = ~0ull;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const oid o = b.seq + posof(b, i);
		if (kind == C_BIT)
			((int8_t *) out)[i] = 1;   // its loop overwrites dst[0] too
		else if (kind == C_FLT)
			((float *) out)[i] = (float) o;
		else if (kind == C_DBL)
			((double *) out)[i] = (double) o;
		else if (o > maxv) {
			if (i < first)
				first = i;
		} else
			st_int(out, ow, i, (hge) o);
	}
	first = block_reduce(first, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	if (threadIdx.x == 0 && first != ~0ull)
		atomicMin(meta + 1, first);
}

__global__ void
k_fetch2(Opnd a, Opnd b, BUN i, Num *out)
{
	out[0] = opval(a, i);
	if (b.tp >= 0)
		out[1] = opval(b, i);
}

void
fmt_num(char *buf, size_t sz, int t, const Num &v)
{
	// FMT##TYPE / CST##TYPE (gdk/gdk_calc_private.h:300-321)
	switch (t) {
	case MGDK_bte: case MGDK_sht: case MGDK_int: snprintf(buf, sz, "%d", (int) v.i); break;
	case MGDK_lng: snprintf(buf, sz, "%lld", (long long) v.i); break;
	case MGDK_hge: snprintf(buf, sz, "%.40Lg (approx. value)", (long double) v.i); break;
	case MGDK_flt: snprintf(buf, sz, "%.9g", v.f); break;
	case MGDK_dbl: snprintf(buf, sz, "%.17g", v.d); break;
	default: snprintf(buf, sz, "%llu", (unsigned long long) v.i); break;
	}
}

bool
fetch2(const Opnd &a, const Opnd *b, BUN i, Num *h)
{
	Num *dv = (Num *) ((char *) meta_buf() + 64);
	Opnd B{};
	B.tp = -1;
	hipLaunchKernelGGL(k_fetch2, dim3(1), dim3(1), 0, stream(), a, b ? *b : B, i, dv);
	Num *p = (Num *) pinned(2 * sizeof(Num));
	if (p == nullptr || !hip_ok(hipMemcpyAsync(p, dv, 2 * sizeof(Num), hipMemcpyDeviceToHost, stream()), "memcpy") ||
	    !sync())
		return false;
	memcpy(h, p, 2 * sizeof(Num));
	return true;
}

int
cbtype(int t)
{
	// ATOMbasetype(oid) == lng (gdk/gdk_atoms.c:1720-1737)
	return t == MGDK_oid ? MGDK_lng : basetype(t);
}

mgdk_bat *
convert(mgdk_bat *b, mgdk_bat *s, int tp, int scale1, int scale2, int prec)
{
	ProfScope prof("convert");
	if (tp == MGDK_void)
		tp = MGDK_oid;
	Cand ci{};
	if (cand_init(&ci, b, s) < 0)
		return nullptr;
	const oid hseq = s ? s->hseqbase : b->hseqbase;
	const int st = b->ttype == MGDK_void ? MGDK_void : cbtype(b->ttype), dt = cbtype(tp);
	const bool to_oid = tp == MGDK_oid, to_bit = tp == MGDK_bit;
	if ((!is_num_t(st) && st != MGDK_void) || !is_num_t(dt)) {
		seterr("type combination (convert(%s)->%s) not supported.\n", atomname(b->ttype), atomname(tp));
		return nullptr;
	}
	const BUN n = ci.n;
	if (n == 0 || (b->ttype == MGDK_void && b->tseqbase == MGDK_OID_NIL)) {
		// BATconstant(ci.hseq, tp, nil, ncand)
		char nilv[16];
		switch (width_of(tp)) {
		case 1: { int8_t x = INT8_MIN; memcpy(nilv, &x, 1); break; }
		case 2: { int16_t x = INT16_MIN; memcpy(nilv, &x, 2); break; }
		case 4: { if (dt == MGDK_flt) { float x = NAN; memcpy(nilv, &x, 4); } else { int32_t x = INT32_MIN; memcpy(nilv, &x, 4); } break; }
		case 8: { if (dt == MGDK_dbl) { double x = NAN; memcpy(nilv, &x, 8); } else { int64_t x = INT64_MIN; memcpy(nilv, &x, 8); } break; }
		default: { hge x = (hge) ((uhge) 1 << 127); memcpy(nilv, &x, 16); break; }
		}
		mgdk_bat *bn = mgdk_BATconstant(hseq, tp, nilv, n);
		if (bn) {
			bn->tnil = n >= 1;
			bn->tnonil = !bn->tnil;
		}
		return bn;
	}
	if (n == b->count && !to_bit && st == dt && (!to_oid || b->ttype == MGDK_oid) && scale1 == 0 &&
	    scale2 == 0 && prec == 0) {
		// COLcopy (gdk_calc_convert.c:1443-1455)
		mgdk_bat *bn = newbat(hseq, tp, n);
		if (bn == nullptr)
			return nullptr;
		if (!hip_ok(hipMemcpyAsync(bn->theap, b->theap, n * (size_t) width_of(tp), hipMemcpyDeviceToDevice, stream()),
			    "memcpy") || !sync()) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		bn->count = n;
		bn->tsorted = b->tsorted;
		bn->trevsorted = b->trevsorted;
		bn->tkey = b->tkey;
		bn->tnonil = b->tnonil;
		bn->tnil = b->tnil;
		bn->tnosorted = b->tnosorted;
		bn->tnorevsorted = b->tnorevsorted;
		bn->tminpos = b->tminpos;
		bn->tmaxpos = b->tmaxpos;
		bn->tunique_est = b->tunique_est;
		return bn;
	}
	const bool sint = is_int_t(st), dint = is_int_t(dt);
	if (st != MGDK_void && !to_oid && !to_bit) {
		// scale factors the reference casts to the conversion's C types; a
		// factor that does not fit wraps there and is refused here
		bool fit = scale1 <= 38 && scale2 <= 38 && prec <= 38;
		if (fit && sint && dint)
			fit = scale_of(scale1 > scale2 ? scale1 - scale2 : 0) <= imax_of(st) &&
			      scale_of(scale2 > scale1 ? scale2 - scale1 : 0) <= imax_of(dt) && scale_of(prec) <= imax_of(dt);
		else if (fit && sint)
			fit = scale_of(scale1) <= imax_of(st);
		else if (fit && dint)
			fit = scale2 <= 18 && scale_of(scale2) <= imax_of(dt) && scale_of(prec) <= imax_of(dt);
		if (!fit) {
			seterr("convert: scale factor does not fit %s\n", atomname(tp));
			return nullptr;
		}
	}
	mgdk_bat *bn = newbat(hseq, tp, n);
	if (bn == nullptr)
		return nullptr;
	Opnd B{};
	set_bat(B, b, ci, st);
	const int kind = to_bit ? C_BIT : to_oid ? C_OID : dt == MGDK_flt ? C_FLT : dt == MGDK_dbl ? C_DBL : C_INT;
	unsigned long long *m = counters(2);
	if (m == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	dim3 g(grid_for(n, 256 * 4, 256 * 64));
	bool reduce = false;
	if (st == MGDK_void) {
		const uint64_t maxv = dt == MGDK_bte ? INT8_MAX : dt == MGDK_sht ? INT16_MAX : dt == MGDK_int ? INT32_MAX : ~0ull;
		hipLaunchKernelGGL(k_convert_void, g, dim3(256), 0, stream(), B, kind, width_of(tp), maxv, bn->theap, n, m);
	} else {
		ConvArgs a{};
		a.st = st;
		a.dt = dt;
		a.kind = kind;
		a.ow = width_of(tp);
		a.prec = prec;
		a.div = 1;
		a.mul = 1;
		if (kind == C_OID) {
			a.lim_f = (float) INT64_MAX;
			a.lim_d = (double) INT64_MAX;
		} else if (kind == C_BIT) {
			reduce = true;
		} else if (sint && dint) {
			a.div = scale_of(scale1 > scale2 ? scale1 - scale2 : 0);
			a.mul = scale_of(scale2 > scale1 ? scale2 - scale1 : 0);
			a.max = imax_of(dt) / a.mul;
			a.pr = scale_of(prec) / a.mul;
			reduce = a.div > 1;
		} else if (sint) {
			a.div = scale_of(scale1);
			reduce = ibits(st) > (kind == C_FLT ? FLT_MANT_DIG : DBL_MANT_DIG);
		} else if (kind == C_FLT || kind == C_DBL) {
			reduce = st == MGDK_dbl && kind == C_FLT;
		} else {
			a.max = imax_of(dt);
			a.pr = scale_of(prec);
			a.fmul = (uint64_t) scale_of(scale2);
			a.lim_f = dt == MGDK_hge ? 1.7014118e38f : (float) (long long) (dt == MGDK_lng ? INT64_MAX : (long long) a.max);
			a.lim_d = dt == MGDK_hge ? 1.7014118346046923e38 : (double) (long long) a.max;
			reduce = true;
		}
		hipLaunchKernelGGL(k_convert, g, dim3(256), 0, stream(), B, a, bn->theap, n, m);
	}
	unsigned long long h[2];
	if (!read_counters(m, h, 2)) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[1] != ~0ull) {
		Num v[2];
		if (!fetch2(B, nullptr, (BUN) h[1], v)) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		if (st == MGDK_void) {
			seterr("22003!overflow in conversion of %llu to %s.\n", (unsigned long long) v[0].i, atomname(dt));
		} else if (prec > 0 && !to_oid) {
			seterr("22003!overflow in conversion to DECIMAL(%d,%d).\n", prec, scale2);
		} else {
			char buf[96];
			fmt_num(buf, sizeof(buf), st, v[0]);
			seterr("22003!overflow in conversion of %s to %s.\n", buf, to_oid ? "oid" : atomname(dt));
		}
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const BUN nils = h[0];
	bn->count = n;
	bn->tnil = nils != 0;
	bn->tnonil = nils == 0;
	// gdk_calc_convert.c:1528-1537 (no str on this path)
	if (!to_bit || n < 2) {
		bn->tsorted = nils == 0 && b->tsorted;
		bn->trevsorted = nils == 0 && b->trevsorted;
	} else {
		bn->tsorted = bn->trevsorted = 0;
	}
	bn->tkey = (!reduce || n < 2) ? (b->tkey && nils <= 1) : 0;
	return bn;
}

// ---- BATcalcnot (gdk/gdk_calc.c:41-146) -----------------------------------
__global__ __launch_bounds__(256) void
k_not(Opnd b, bool isbit, int w, void *out, BUN n, unsigned long long *meta)
{
	unsigned long long nils = 0, first = ~0ull;
	const hge vmin = w == 16 ? (hge) ((uhge) 1 << 127) : -((hge) 1 << (8 * w - 1));
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const Num v = opval(b, i);
		if (v.nil) {
			st_int(out, w, i, vmin);
			nils++;
		} else if (isbit) {
			((int8_t *) out)[i] = !v.i;
		} else {
			const hge r = ~v.i;
			if (r == vmin) {
				if (i < first)
					first = i;
			} else {
				st_int(out, w, i, r);
			}
		}
	}
	nils = block_reduce(nils, [](unsigned long long x, unsigned long long y) { return x + y; });
	first = block_reduce(first, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	if (threadIdx.x == 0) {
		if (nils)
			atomicAdd(meta, nils);
		if (first != ~0ull)
			atomicMin(meta + 1, first);
	}
}

mgdk_bat *
calcnot(mgdk_bat *b, mgdk_bat *s)
{
	ProfScope prof("calcnot");
	Cand ci{};
	if (cand_init(&ci, b, s) < 0)
		return nullptr;
	const oid hseq = s ? s->hseqbase : b->hseqbase;
	const int t = basetype(b->ttype);
	if (!is_int_t(t)) {
		seterr("type %s not supported.\n", atomname(b->ttype));
		return nullptr;
	}
	const BUN n = ci.n;
	mgdk_bat *bn = newbat(hseq, b->ttype, n);
	if (bn == nullptr)
		return nullptr;
	if (n == 0) {
		bn->count = 0;
		return bn;
	}
	Opnd B{};
	set_bat(B, b, ci, t);
	unsigned long long *m = counters(2);
	if (m == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	hipLaunchKernelGGL(k_not, dim3(grid_for(n, 256 * 4, 256 * 64)), dim3(256), 0, stream(), B,
			   b->ttype == MGDK_bit, width_of(t), bn->theap, n, m);
	unsigned long long h[2];
	if (!read_counters(m, h, 2)) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[1] != ~0ull) {
		Num v[2];
		char buf[96];
		if (fetch2(B, nullptr, (BUN) h[1], v)) {
			fmt_num(buf, sizeof(buf), t, v[0]);
			seterr("22003!overflow in calculation NOT(%s).\n", buf);
		}
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const BUN nils = h[0];
	bn->count = n;
	bn->tsorted = nils == 0 && b->trevsorted;
	bn->trevsorted = nils == 0 && b->tsorted;
	bn->tnil = nils != 0;
	bn->tnonil = nils == 0;
	bn->tkey = b->tkey && nils <= 1;
	return bn;
}

// ---- division and modulo ----------------------------------------------------
int
rank_of(int t)
{
	return t == MGDK_bte ? 0 : t == MGDK_sht ? 1 : t == MGDK_int ? 2 : t == MGDK_lng ? 3 : t == MGDK_hge ? 4
		: t == MGDK_flt ? 5 : 6;
}

// the DIV_3TYPE / DIV_3TYPE_float / MOD_3TYPE / FMOD_3TYPE instantiations
// (gdk_calc_div.c, gdk_calc_mod.c)
bool
divmod_supported(bool div, int t1, int t2, int tp)
{
	if (!is_num_t(t1) || !is_num_t(t2) || !is_num_t(tp))
		return false;
	const int r1 = rank_of(t1), r2 = rank_of(t2), rp = rank_of(tp);
	if (div) {
		if (r2 >= 5)
			return r1 == 6 ? rp == 6 : (r2 == 5 ? rp >= 5 : rp == 6);
		return rp >= r1;
	}
	if (r1 <= 4 && r2 <= 4)
		return rp <= 4 && rp >= (r1 < r2 ? r1 : r2);
	return rp == (r1 == 6 || r2 == 6 ? 6 : 5);
}

// error codes in the low 2 bits of the first-failure word: 1 division by
// zero, 2 overflow with message, 3 result out of range (no message)
template <bool DIV>
__global__ __launch_bounds__(256) void
k_divmod(Opnd a, Opnd b, int dt, int ow, hge dmax, void *out, BUN n, unsigned long long *meta)
{
	unsigned long long nils = 0, first = ~0ull;
	const int kind = dt == MGDK_flt ? C_FLT : dt == MGDK_dbl ? C_DBL : C_INT;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const Num x = opval(a, i), y = opval(b, i);
		if (x.nil || y.nil) {
			st_nil(out, kind, ow, i);
			nils++;
			continue;
		}
		const bool yf = b.tp == MGDK_flt || b.tp == MGDK_dbl, xf = a.tp == MGDK_flt || a.tp == MGDK_dbl;
		const bool zero = b.tp == MGDK_flt ? y.f == 0 : b.tp == MGDK_dbl ? y.d == 0 : y.i == 0;
		int err = 0;
		if (zero) {
			err = 1;
		} else if (DIV) {
			double q;
			if (yf) {
				bool ovf;
				if (kind == C_FLT) {
					const float ay = fabsf(y.f);
					const float ax = a.tp == MGDK_flt ? fabsf(x.f) : hge_to_flt(x.i < 0 ? -x.i : x.i);
					ovf = ay < 1 && FLT_MAX * ay < ax;
				} else {
					const double ay = b.tp == MGDK_flt ? (double) fabsf(y.f) : fabs(y.d);
					const double ax = a.tp == MGDK_flt ? (double) fabsf(x.f) : a.tp == MGDK_dbl ? fabs(x.d)
							: hge_to_dbl(x.i < 0 ? -x.i : x.i);
					ovf = ay < 1 && DBL_MAX * ay < ax;
				}
				if (ovf)
					err = 2;
				q = kind == C_FLT ? (double) (as_flt(x, a.tp) / y.f) : as_dbl(x, a.tp) / as_dbl(y, b.tp);
			} else if (a.tp == MGDK_flt) {
				q = (double) (x.f / hge_to_flt(y.i));
			} else if (a.tp == MGDK_dbl) {
				q = x.d / hge_to_dbl(y.i);
			} else {
				hge qi;
				if (a.tp != MGDK_hge && b.tp != MGDK_hge)
					qi = (hge) ((long long) x.i / (long long) y.i);
				else
					qi = x.i / y.i;
				if (kind == C_FLT)
					((float *) out)[i] = hge_to_flt(qi);
				else if (kind == C_DBL)
					((double *) out)[i] = hge_to_dbl(qi);
				else if (qi < -dmax || qi > dmax)
					err = 3;
				else
					st_int(out, ow, i, qi);
				if (err == 0)
					continue;
			}
			if (err == 0) {
				const double lim = kind == C_FLT ? (double) FLT_MAX : DBL_MAX;
				if (q < -lim || q > lim)
					err = 3;
				else if (kind == C_FLT)
					((float *) out)[i] = (float) q;
				else
					((double *) out)[i] = q;
			}
		} else {
			if (kind == C_FLT) {
				((float *) out)[i] = fmodf(as_flt(x, a.tp), as_flt(y, b.tp));
			} else if (kind == C_DBL) {
				((double *) out)[i] = fmod(as_dbl(x, a.tp), as_dbl(y, b.tp));
			} else {
				// MOD_3TYPE: (TYPE3) lft % rgt -- lft cast to the result type first
				hge l;
				switch (ow) {
				case 1: l = (int8_t) x.i; break;
				case 2: l = (int16_t) x.i; break;
				case 4: l = (int32_t) x.i; break;
				case 8: l = (int64_t) x.i; break;
				default: l = x.i; break;
				}
				hge r;
				if (ow <= 8 && b.tp != MGDK_hge)
					r = (hge) ((long long) l % (long long) y.i);
				else
					r = l % y.i;
				st_int(out, ow, i, r);
			}
		}
		if (err) {
			const unsigned long long code = ((unsigned long long) i << 2) | (unsigned) err;
			if (code < first)
				first = code;
		}
	}
	nils = block_reduce(nils, [](unsigned long long x, unsigned long long y) { return x + y; });
	first = block_reduce(first, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	if (threadIdx.x == 0) {
		if (nils)
			atomicAdd(meta, nils);
		if (first != ~0ull)
			atomicMin(meta + 1, first);
	}
}

mgdk_bat *
calcdivmod(bool div, mgdk_bat *b1, const void *v1, int t1, mgdk_bat *b2, const void *v2, int t2,
	   mgdk_bat *s1, mgdk_bat *s2, int tp)
{
	ProfScope prof(div ? "calcdiv" : "calcmod");
	const char *fname = div ? (b1 && b2 ? "BATcalcdiv" : b1 ? "BATcalcdivcst" : "BATcalccstdiv")
				: (b1 && b2 ? "BATcalcmod" : b1 ? "BATcalcmodcst" : "BATcalccstmod");
	mgdk_bat *bb = b1 ? b1 : b2;
	Cand c1{}, c2{}, ci{};
	if (b1 && b2) {
		if (cand_init(&c1, b1, s1) < 0 || cand_init(&c2, b2, s2) < 0)
			return nullptr;
		const oid h1 = s1 ? s1->hseqbase : b1->hseqbase, h2 = s2 ? s2->hseqbase : b2->hseqbase;
		if (c1.n != c2.n || h1 != h2) {
			seterr("%s: inputs not the same size.\n", fname);
			return nullptr;
		}
		ci = c1;
	} else {
		if (cand_init(&ci, bb, s1) < 0)
			return nullptr;
		if (b1)
			c1 = ci;
		else
			c2 = ci;
	}
	const oid hseq = s1 ? s1->hseqbase : bb->hseqbase;
	const int ta = basetype(b1 ? b1->ttype : t1), tb = basetype(b2 ? b2->ttype : t2), dt = basetype(tp);
	const BUN n = ci.n;
	if (n == 0) {
		mgdk_bat *bn = newbat(hseq, tp, 0);
		if (bn)
			bn->count = 0;
		return bn;
	}
	if (!divmod_supported(div, ta, tb, dt)) {
		seterr("%s: type combination (%s(%s,%s)->%s) not supported.\n", fname, div ? "div" : "mod", atomname(ta),
		       atomname(tb), atomname(dt));
		return nullptr;
	}
	Opnd A{}, B{};
	if (b1)
		set_bat(A, b1, c1, ta);
	else
		set_cst(A, v1, ta);
	if (b2)
		set_bat(B, b2, c2, tb);
	else
		set_cst(B, v2, tb);
	mgdk_bat *bn = newbat(hseq, tp, n);
	if (bn == nullptr)
		return nullptr;
	unsigned long long *m = counters(2);
	if (m == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	dim3 g(grid_for(n, 256 * 4, 256 * 64));
	const int ow = width_of(tp);
	const hge dmax = is_int_t(dt) ? imax_of(dt) : 0;
	if (div)
		hipLaunchKernelGGL(k_divmod<true>, g, dim3(256), 0, stream(), A, B, dt, ow, dmax, bn->theap, n, m);
	else
		hipLaunchKernelGGL(k_divmod<false>, g, dim3(256), 0, stream(), A, B, dt, ow, dmax, bn->theap, n, m);
	unsigned long long h[2];
	if (!read_counters(m, h, 2)) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[1] != ~0ull) {
		const int err = (int) (h[1] & 3);
		if (err == 1) {
			seterr("22012!division by zero.\n");
		} else if (err == 2) {
			Num v[2];
			if (fetch2(A, &B, (BUN) (h[1] >> 2), v)) {
				char x[96], y[96];
				fmt_num(x, sizeof(x), ta, v[0]);
				fmt_num(y, sizeof(y), tb, v[1]);
				seterr("22003!overflow in calculation %s/%s.\n", x, y);
			}
		} else {
			seterr("%s", "");   // BUN_NONE + 2: the reference sets no message
		}
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const BUN nils = h[0];
	set_cmp_props(bn, n, nils);
	return bn;
}

// ---- the rest of gdk_calc.c's element-wise operators ---------------------
// BATcalcnegate / absolute / iszero / sign (gdk_calc.c:233-800), isnil /
// isnotnil (:802-920), min / max and their _no_nil and constant forms
// (:976-2436), xor / or / and (:2439-3030; bit: the three-valued or3 / and3,
// :2590, :2826), lsh / rsh (:3059-3760) and incr / decr
// (gdk_calc_addsub.c:1681): one lane per candidate over the Num operands
// above; the first failing candidate (atomicMin) gives the reference's
// message.
enum { X_NEG, X_ABS, X_ISZERO, X_SIGN, X_ISNIL, X_ISNOTNIL, X_MIN, X_MAX, X_MINNN, X_MAXNN, X_MINC, X_MAXC, X_MINNNC,
       X_MAXNNC, X_AND, X_OR, X_XOR, X_LSH, X_RSH };

struct XArgs {
	int op;
	int t;            // the operands' base type (shifts: the left one)
	int t2;           // shifts: the right operand's base type
	int ow;           // output width
	bool isbit;       // bit operands (three-valued logic)
	bool oid;         // oid / void values (unsigned compare)
	int lbits;        // shifts: bits of the left operand's type
};

__device__ __forceinline__ bool
x_lt(const Num &a, const Num &b, int t, bool oid)
{
	if (t == MGDK_flt)
		return a.f < b.f;
	if (t == MGDK_dbl)
		return a.d < b.d;
	if (oid)
		return (uhge) a.i < (uhge) b.i;
	return a.i < b.i;
}

__device__ __forceinline__ void
x_store(void *out, const XArgs &x, BUN i, const Num &v)
{
	if (x.t == MGDK_flt && x.ow == 4 && x.op != X_ISZERO && x.op != X_SIGN && x.op != X_ISNIL && x.op != X_ISNOTNIL)
		((float *) out)[i] = v.f;
	else if (x.t == MGDK_dbl && x.ow == 8 && x.op != X_ISZERO && x.op != X_SIGN && x.op != X_ISNIL &&
		 x.op != X_ISNOTNIL)
		((double *) out)[i] = v.d;
	else
		st_int(out, x.ow, i, v.i);
}

__device__ __forceinline__ Num
x_nil(const XArgs &x)
{
	Num v{};
	v.nil = true;
	v.f = __int_as_float(0x7fc00000);
	v.d = __longlong_as_double(0x7ff8000000000000ll);
	v.i = x.oid ? (hge) MGDK_OID_NIL : x.ow == 16 ? (hge) ((uhge) 1 << 127) : -((hge) 1 << (8 * x.ow - 1));
	return v;
}

// meta[0] nils, meta[1] first failing candidate
__global__ __launch_bounds__(256) void
k_xop(Opnd a, Opnd b, XArgs x, void *out, BUN n, unsigned long long *meta)
{
	unsigned long long nils = 0, first = ~0ull;
	const Num NIL = x_nil(x);
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const Num p = opval(a, i);
		Num r = p;
		bool isnil = false, fail = false;
		const bool fl = x.t == MGDK_flt || x.t == MGDK_dbl;
		switch (x.op) {
		case X_NEG:
		case X_ABS:
			if (p.nil) {
				isnil = true;
			} else if (x.op == X_NEG) {
				r.i = -p.i;
				r.f = -p.f;
				r.d = -p.d;
			} else {
				r.i = p.i < 0 ? -p.i : p.i;
				r.f = __builtin_fabsf(p.f);
				r.d = __builtin_fabs(p.d);
			}
			break;
		case X_ISZERO:
		case X_SIGN:
			if (p.nil) {
				isnil = true;
			} else {
				const int sg = x.t == MGDK_flt ? (p.f < 0 ? -1 : p.f > 0) : x.t == MGDK_dbl ? (p.d < 0 ? -1 : p.d > 0)
										      : (p.i < 0 ? -1 : p.i > 0);
				const bool z = x.t == MGDK_flt ? p.f == 0 : x.t == MGDK_dbl ? p.d == 0 : p.i == 0;
				r.i = x.op == X_ISZERO ? (hge) z : (hge) sg;
			}
			break;
		case X_ISNIL:
		case X_ISNOTNIL:
			r.i = (hge) (p.nil != (x.op == X_ISNOTNIL));
			break;
		default: {
			const Num q = opval(b, i);
			switch (x.op) {
			case X_MIN:
			case X_MAX:
				if (p.nil || q.nil)
					isnil = true;
				else
					r = (x.op == X_MIN ? x_lt(p, q, x.t, x.oid) : x_lt(q, p, x.t, x.oid)) ? p : q;
				break;
			case X_MINNN:
			case X_MAXNN:
				if (p.nil)
					r = q, isnil = q.nil;
				else
					r = !q.nil && (x.op == X_MINNN ? x_lt(q, p, x.t, x.oid) : x_lt(p, q, x.t, x.oid)) ? q : p;
				break;
			case X_MINC:
			case X_MAXC:
				// the constant is not nil (the caller answered that case)
				if (p.nil)
					isnil = true;
				else
					r = (x.op == X_MINC ? x_lt(p, q, x.t, x.oid) : x_lt(q, p, x.t, x.oid)) ? p : q;
				break;
			case X_MINNNC:
			case X_MAXNNC:
				if (q.nil)
					r = p, isnil = p.nil;
				else if (p.nil)
					r = q;
				else
					r = (x.op == X_MINNNC ? x_lt(p, q, x.t, x.oid) : x_lt(q, p, x.t, x.oid)) ? p : q;
				break;
			case X_AND:
			case X_OR:
			case X_XOR:
				if (x.isbit && x.op != X_XOR) {
					// or3 / and3 (gdk_calc.c:2590, :2826)
					const int8_t v1 = (int8_t) p.i, v2 = (int8_t) q.i;
					int8_t o;
					if (x.op == X_OR)
						o = v1 == 1 || v2 == 1 ? 1 : (p.nil || q.nil) ? INT8_MIN : 0;
					else
						o = v1 == 0 || v2 == 0 ? 0 : (p.nil || q.nil) ? INT8_MIN : 1;
					r.i = o;
					isnil = o == INT8_MIN;
				} else if (p.nil || q.nil) {
					isnil = true;
				} else if (x.isbit) {
					r.i = (p.i == 0) != (q.i == 0);
				} else {
					r.i = x.op == X_AND ? (p.i & q.i) : x.op == X_OR ? (p.i | q.i) : (p.i ^ q.i);
					// a result equal to nil is an overflow (AND / XOR; an OR
					// giving nil has a nil operand)
					fail = r.i == NIL.i && x.op != X_OR;
				}
				break;
			case X_LSH:
			case X_RSH: {
				if (p.nil || q.nil) {
					isnil = true;
					break;
				}
				const int bits = x.lbits;
				const hge sh = q.i;
				if (sh < 0 || sh >= bits) {
					fail = true;
				} else if (x.op == X_LSH) {
					const hge mx = bits == 128 ? (hge) (((uhge) 1 << 127) - 1) : (((hge) 1 << (bits - 1)) - 1);
					if (p.i < 0 || p.i > (mx >> (int) sh))
						fail = true;
					else
						r.i = p.i << (int) sh;
				} else {
					r.i = p.i >> (int) sh;
				}
				break;
			}
			}
		}
		}
		if (fail) {
			if (i < first)
				first = i;
			continue;
		}
		if (isnil) {
			nils++;
			if (x.op == X_ISZERO || x.op == X_SIGN)
				((int8_t *) out)[i] = INT8_MIN;
			else
				x_store(out, x, i, NIL);
			continue;
		}
		if (x.op == X_ISZERO || x.op == X_SIGN || x.op == X_ISNIL || x.op == X_ISNOTNIL)
			((int8_t *) out)[i] = (int8_t) r.i;
		else if (fl)
			x_store(out, x, i, r);
		else
			st_int(out, x.ow, i, r.i);
	}
	nils = block_reduce(nils, [](unsigned long long u, unsigned long long v) { return u + v; });
	first = block_reduce(first, [](unsigned long long u, unsigned long long v) { return u < v ? u : v; });
	if (threadIdx.x == 0) {
		if (nils)
			atomicAdd(meta, nils);
		if (first != ~0ull)
			atomicMin(meta + 1, first);
	}
}

Num
x_nil_host(int t, int w)
{
	Num v{};
	v.nil = true;
	v.i = t == MGDK_oid ? (hge) MGDK_OID_NIL : w == 16 ? (hge) ((uhge) 1 << 127) : -((hge) 1 << (8 * w - 1));
	return v;
}

const char *const xop_name[] = {"BATcalcnegate", "BATcalcabsolute", "BATcalciszero", "BATcalcsign",
				 "BATcalcisnil", "BATcalcisnotnil", "BATcalcmin", "BATcalcmax", "BATcalcmin_no_nil",
				 "BATcalcmax_no_nil", "BATcalcmincst", "BATcalcmaxcst", "BATcalcmincst_no_nil",
				 "BATcalcmaxcst_no_nil", "BATcalcand", "BATcalcor", "BATcalcxor", "BATcalclsh",
				 "BATcalcrsh"};

bool
tdense_bat(const mgdk_bat *b)
{
	return (b->ttype == MGDK_void || b->ttype == MGDK_oid) && b->tseqbase != MGDK_OID_NIL;
}

// the unary operators
mgdk_bat *
calc_unary(int op, mgdk_bat *b, mgdk_bat *s)
{
	if (b == nullptr) {
		seterr("BATcalc: b must exist");
		return nullptr;
	}
	ProfScope prof("calcunary");
	Cand ci{};
	if (cand_init(&ci, b, s) < 0)
		return nullptr;
	const oid hseq = s ? s->hseqbase : b->hseqbase;
	const BUN n = ci.n;
	if (op == X_ISNIL || op == X_ISNOTNIL) {
		// BATcalcisnil_implementation (:802-900): constant answers first
		const bool notnil = op == X_ISNOTNIL;
		if (b->tnonil || tdense_bat(b) || b->ttype == MGDK_void) {
			const int8_t v = (b->tnonil || tdense_bat(b)) ? notnil : !notnil;
			return mgdk_BATconstant(hseq, MGDK_bit, &v, n);
		}
		if (b->ttype == MGDK_str || b->ttype == MGDK_msk) {
			seterr("%s: type %s is not on the device path", xop_name[op], atomname(b->ttype));
			return nullptr;
		}
	}
	const int t = optype(b) == MGDK_oid ? MGDK_lng : basetype(b->ttype);
	const bool numeric = is_num_t(t);
	if (!numeric && !((op == X_ISNIL || op == X_ISNOTNIL) && (t == MGDK_lng || b->ttype == MGDK_oid))) {
		seterr("type %s not supported.\n", atomname(b->ttype));
		return nullptr;
	}
	const int otp = op == X_ISZERO || op == X_ISNIL || op == X_ISNOTNIL ? MGDK_bit : op == X_SIGN ? MGDK_bte : b->ttype;
	if (n == 0) {
		// BATconstant(ci.hseq, type, nil, 0)
		return newbat(hseq, otp, 0);
	}
	mgdk_bat *bn = newbat(hseq, otp, n);
	if (bn == nullptr)
		return nullptr;
	Opnd A{}, B{};
	set_bat(A, b, ci, b->ttype == MGDK_oid ? MGDK_oid : t);
	B.tp = -1;
	XArgs x{op, t, t, width_of(otp), false, b->ttype == MGDK_oid, 0};
	unsigned long long *m = counters(2);
	if (m == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	hipLaunchKernelGGL(k_xop, dim3(grid_for(n, 256 * 4, 256 * 64)), dim3(256), 0, stream(), A, B, x, bn->theap, n, m);
	unsigned long long h[2];
	if (!read_counters(m, h, 2)) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const BUN nils = h[0];
	bn->count = n;
	bn->tnil = nils != 0;
	bn->tnonil = nils == 0;
	bn->tkey = n <= 1;
	switch (op) {
	case X_NEG:
		// unary - reverses the order, but nils mess it up
		bn->tsorted = nils == 0 && b->trevsorted;
		bn->trevsorted = nils == 0 && b->tsorted;
		bn->tkey = b->tkey && nils <= 1;
		break;
	case X_SIGN:
		bn->tsorted = b->tsorted || n <= 1 || nils == n;
		bn->trevsorted = b->trevsorted || n <= 1 || nils == n;
		break;
	case X_ISNIL:
		bn->tsorted = b->trevsorted;
		bn->trevsorted = b->tsorted;
		bn->tnil = 0;
		bn->tnonil = 1;
		break;
	case X_ISNOTNIL:
		bn->tsorted = b->tsorted;
		bn->trevsorted = b->trevsorted;
		bn->tnil = 0;
		bn->tnonil = 1;
		break;
	default:
		bn->tsorted = n <= 1 || nils == n;
		bn->trevsorted = n <= 1 || nils == n;
		break;
	}
	return bn;
}

// min / max (b2 or the constant v of type vt), their _no_nil forms
mgdk_bat *
calc_minmax(int op, mgdk_bat *b1, mgdk_bat *b2, const void *v, int vt, mgdk_bat *s1, mgdk_bat *s2)
{
	const bool cst = b2 == nullptr;
	const char *fname = xop_name[op];
	if (b1 == nullptr) {
		seterr("%s: b must exist", fname);
		return nullptr;
	}
	ProfScope prof("calcminmax");
	const int at1 = b1->ttype == MGDK_void ? MGDK_oid : b1->ttype;
	if (cst ? at1 != (vt == MGDK_void ? MGDK_oid : vt) : at1 != (b2->ttype == MGDK_void ? MGDK_oid : b2->ttype)) {
		seterr("inputs have incompatible types\n");
		return nullptr;
	}
	Cand c1{}, c2{};
	if (cand_init(&c1, b1, s1) < 0 || (!cst && cand_init(&c2, b2, s2) < 0))
		return nullptr;
	const oid h1 = s1 ? s1->hseqbase : b1->hseqbase;
	if (!cst) {
		const oid h2 = s2 ? s2->hseqbase : b2->hseqbase;
		if (c1.n != c2.n || h1 != h2) {
			seterr("inputs not the same size.\n");
			return nullptr;
		}
	}
	const bool isoid = at1 == MGDK_oid;
	const int t = isoid ? MGDK_oid : basetype(b1->ttype);
	if (!isoid && !is_num_t(t)) {
		seterr("%s: type %s is not on the device path", fname, atomname(b1->ttype));
		return nullptr;
	}
	const int otp = at1;
	const BUN n = c1.n;
	Opnd A{}, B{};
	set_bat(A, b1, c1, b1->ttype == MGDK_void ? MGDK_void : t);
	if (cst)
		set_cst(B, v, t);
	else
		set_bat(B, b2, c2, b2->ttype == MGDK_void ? MGDK_void : t);
	int xop = op;
	if (cst) {
		// BATcalcmincst (:1403-1433): an empty input, a nil constant or an
		// all-nil void column give the all-nil column
		const bool allnil1 = b1->ttype == MGDK_void && b1->tseqbase == MGDK_OID_NIL;
		if (op == X_MIN || op == X_MAX) {
			if (n == 0 || B.cnil || allnil1) {
				mgdk_bat *bn = nullptr;
				std::vector<uint8_t> nil(16, 0);
				const int w = width_of(otp);
				Num nv = x_nil_host(otp, w);
				memcpy(nil.data(), &nv.i, 16);
				if (t == MGDK_flt) { const float f = __builtin_nanf(""); memcpy(nil.data(), &f, 4); }
				if (t == MGDK_dbl) { const double d = __builtin_nan(""); memcpy(nil.data(), &d, 8); }
				bn = mgdk_BATconstant(h1, otp, nil.data(), n);
				return bn;
			}
			xop = op == X_MIN ? X_MINC : X_MAXC;
		} else {
			if (n == 0)
				return newbat(h1, otp, 0);
			if (allnil1 && B.cnil) {
				const oid nil = MGDK_OID_NIL;
				return mgdk_BATconstant(h1, MGDK_void, &nil, n);
			}
			xop = op == X_MINNN ? X_MINNNC : X_MAXNNC;
		}
	}
	mgdk_bat *bn = newbat(h1, otp, n);
	if (bn == nullptr)
		return nullptr;
	if (n) {
		XArgs x{xop, t == MGDK_oid ? MGDK_lng : t, t, width_of(otp), false, isoid, 0};
		if (t == MGDK_oid)
			x.t = MGDK_oid;
		unsigned long long *m = counters(2);
		if (m == nullptr) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		hipLaunchKernelGGL(k_xop, dim3(grid_for(n, 256 * 4, 256 * 64)), dim3(256), 0, stream(), A, B, x, bn->theap, n,
				   m);
		unsigned long long h[2];
		if (!read_counters(m, h, 2)) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		bn->tnil = h[0] != 0;
		bn->tnonil = h[0] == 0;
	}
	bn->count = n;
	if (n <= 1) {
		bn->tsorted = bn->trevsorted = bn->tkey = 1;
		oid f = 0;
		if (isoid && n == 1 && oid_at(bn, 0, &f) < 0) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		bn->tseqbase = isoid ? (n == 1 ? f : 0) : MGDK_OID_NIL;
	} else {
		bn->tsorted = bn->trevsorted = bn->tkey = 0;
		bn->tseqbase = MGDK_OID_NIL;
	}
	return bn;
}

// and / or / xor / lsh / rsh of (b1 | constant) with (b2 | constant)
mgdk_bat *
calc_bits(int op, const char *fname, mgdk_bat *b1, const void *v1, int t1, mgdk_bat *b2, const void *v2, int t2,
	  mgdk_bat *s1, mgdk_bat *s2)
{
	mgdk_bat *bb = b1 ? b1 : b2;
	if (bb == nullptr) {
		seterr("%s: b must exist", fname);
		return nullptr;
	}
	ProfScope prof("calcbits");
	const int ta = b1 ? b1->ttype : t1, tb = b2 ? b2->ttype : t2;
	const bool shift = op == X_LSH || op == X_RSH;
	if (!shift && basetype(ta) != basetype(tb)) {
		seterr("incompatible input types.\n");
		return nullptr;
	}
	Cand c1{}, c2{}, ci{};
	if (b1 && b2) {
		if (cand_init(&c1, b1, s1) < 0 || cand_init(&c2, b2, s2) < 0)
			return nullptr;
		const oid h1 = s1 ? s1->hseqbase : b1->hseqbase, h2 = s2 ? s2->hseqbase : b2->hseqbase;
		if (c1.n != c2.n || h1 != h2) {
			seterr("inputs not the same size.\n");
			return nullptr;
		}
		ci = c1;
	} else {
		if (cand_init(&ci, bb, s1) < 0)
			return nullptr;
		if (b1)
			c1 = ci;
		else
			c2 = ci;
	}
	const oid hseq = s1 ? s1->hseqbase : bb->hseqbase;
	const int ba = basetype(ta), bbt = basetype(tb);
	// the result has the left operand's type (:2467, :3269)
	const int otp = ta;
	const BUN n = ci.n;
	mgdk_bat *bn = newbat(hseq, otp, n);
	if (bn == nullptr)
		return nullptr;
	bn->count = 0;
	if (n == 0)
		return bn;
	if (!is_int_t(ba) || !is_int_t(bbt)) {
		mgdk_BBPunfix(bn);
		seterr("%s: bad input type %s.\n", fname, atomname(is_int_t(ba) ? tb : ta));
		return nullptr;
	}
	Opnd A{}, B{};
	if (b1)
		set_bat(A, b1, c1, ba);
	else
		set_cst(A, v1, ba);
	if (b2)
		set_bat(B, b2, c2, bbt);
	else
		set_cst(B, v2, bbt);
	XArgs x{op, ba, bbt, width_of(otp), ta == MGDK_bit, false, 8 * width_of(ba)};
	unsigned long long *m = counters(2);
	if (m == nullptr) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	hipLaunchKernelGGL(k_xop, dim3(grid_for(n, 256 * 4, 256 * 64)), dim3(256), 0, stream(), A, B, x, bn->theap, n, m);
	unsigned long long h[2];
	if (!read_counters(m, h, 2)) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[1] != ~0ull) {
		Num v[2];
		char xa[96], xb[96];
		if (fetch2(A, &B, (BUN) h[1], v)) {
			fmt_num(xa, sizeof(xa), ba, v[0]);
			fmt_num(xb, sizeof(xb), bbt, v[1]);
			if (shift)
				seterr("%s: shift operand too large in %s(%s,%s).\n", fname, op == X_LSH ? "LSH" : "RSH", xa, xb);
			else
				seterr("22003!overflow in calculation %s%s%s.\n", xa, op == X_AND ? "AND" : "XOR", xb);
		}
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	set_cmp_props(bn, n, h[0]);
	return bn;
}

// BATcalcifthenelse (:4376-4760): b a bit column; "then" / "else" BATs (or
// constants) aligned with b; a nil condition takes the else branch
__global__ __launch_bounds__(256) void
k_ifthenelse(const int8_t *cond, BUN n, const void *v1, bool c1, oid seq1, const void *v2, bool c2, oid seq2,
	     int w, void *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const int8_t c = cond[i];
		const bool take1 = c != 0 && c != INT8_MIN;
		const void *src = take1 ? v1 : v2;
		const bool cs = take1 ? c1 : c2;
		const oid seq = take1 ? seq1 : seq2;
		if (src == nullptr) {
			// a void column: its sequence advanced once per row
			// (gdk_calc.c:4550-4561)
			((uint64_t *) out)[i] = seq + i;
			continue;
		}
		const BUN p = cs ? 0 : i;
		switch (w) {
		case 1: ((int8_t *) out)[i] = ((const int8_t *) src)[p]; break;
		case 2: ((int16_t *) out)[i] = ((const int16_t *) src)[p]; break;
		case 4: ((int32_t *) out)[i] = ((const int32_t *) src)[p]; break;
		case 8: ((int64_t *) out)[i] = ((const int64_t *) src)[p]; break;
		default: ((hge *) out)[i] = ((const hge *) src)[p]; break;
		}
	}
}

// a str offset of width w (1 / 2: relative to GDK_VAROFFSET, gdk_atoms.h:421-436)
__device__ __forceinline__ uint64_t
str_off(const void *offs, int w, BUN p)
{
	switch (w) {
	case 1: return (uint64_t) ((const uint8_t *) offs)[p] + 8192;
	case 2: return (uint64_t) ((const uint16_t *) offs)[p] + 8192;
	case 4: return ((const uint32_t *) offs)[p];
	default: return ((const uint64_t *) offs)[p];
	}
}

// str ifthenelse: 8-byte offsets into the result heap (then side: its own
// offsets, else side: + base2; a constant: its place at the heap's end)
__global__ __launch_bounds__(256) void
k_ifte_str(const int8_t *cond, BUN n, const void *o1, int w1, uint64_t c1, const void *o2, int w2, uint64_t base2,
	   uint64_t c2, uint64_t *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const int8_t c = cond[i];
		out[i] = c != 0 && c != INT8_MIN ? (o1 ? str_off(o1, w1, i) : c1) : (o2 ? base2 + str_off(o2, w2, i) : c2);
	}
}

// BATcalcifthenelse of str (gdk_calc.c:4407-4459, the var-sized branch): the
// strings are the then / else side's; the result's heap is the then side's
// heap shared (both sides one heap, no constant) or the sides' heaps and the
// constants copied after one another.  A copied heap may hold a string twice,
// so it is kept at GDK_ELIMLIMIT (64 KiB) or more: grouping then compares
// strings, never offsets (GDK_ELIMDOUBLES, gdk_atoms.h:373-375)
mgdk_bat *
ifthenelse_str(mgdk_bat *b, mgdk_bat *b1, const char *c1, mgdk_bat *b2, const char *c2)
{
	const BUN n = b->count;
	hipStream_t st = stream();
	mgdk_bat *bn = newbat(b->hseqbase, MGDK_lng, n);
	if (bn == nullptr)
		return nullptr;
	Priv *p = (Priv *) bn->priv;
	bn->ttype = MGDK_str;
	bn->twidth = 8;
	const bool shared = b1 && b2 && b1->tvheap == b2->tvheap;
	const size_t s1 = b1 ? b1->tvheapsize : 0, s2 = b2 && !shared ? b2->tvheapsize : 0;
	const size_t l1 = c1 ? strlen(c1) + 1 : 0, l2 = c2 ? strlen(c2) + 1 : 0;
	const uint64_t base2 = shared ? 0 : s1, k1 = s1 + s2, k2 = s1 + s2 + l1;
	bool ok = true;
	if (shared) {
		share_vheap(bn, b1);
	} else {
		size_t size = s1 + s2 + l1 + l2;
		if (size < ((size_t) 1 << 16))
			size = (size_t) 1 << 16;
		Heap *vh = heap_new(size);
		if (vh == nullptr) {
			mgdk_BBPunfix(bn);
			return nullptr;
		}
		heap_decref(p->tvheap);
		p->tvheap = vh;
		bn->tvheap = vh->base;
		bn->tvheapsize = size;
		char *d = (char *) vh->base;
		ok = hip_ok(hipMemsetAsync(d, 0, size, st), "memset") &&
		     (s1 == 0 || hip_ok(hipMemcpyAsync(d, b1->tvheap, s1, hipMemcpyDeviceToDevice, st), "memcpy")) &&
		     (s2 == 0 || hip_ok(hipMemcpyAsync(d + s1, b2->tvheap, s2, hipMemcpyDeviceToDevice, st), "memcpy"));
		if (ok && (l1 || l2)) {
			std::string t;
			if (c1)
				t.append(c1, l1);
			if (c2)
				t.append(c2, l2);
			const void *src = stage_host(t.data(), t.size());
			ok = src && hip_ok(hipMemcpyAsync(d + k1, src, t.size(), hipMemcpyHostToDevice, st), "memcpy");
		}
	}
	if (ok && n)
		hipLaunchKernelGGL(k_ifte_str, dim3(grid_for(n, 256 * 4, 256 * 64)), dim3(256), 0, st, (const int8_t *) b->theap, n,
				   b1 ? b1->theap : nullptr, b1 ? b1->twidth : 0, k1, b2 ? b2->theap : nullptr,
				   b2 ? b2->twidth : 0, base2, k2, (uint64_t *) bn->theap);
	if (!ok || !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	auto snonil = [](const char *c) { return !(c[0] == '\x80' && c[1] == 0); };
	const bool nonil1 = b1 ? (bool) b1->tnonil : snonil(c1), nonil2 = b2 ? (bool) b2->tnonil : snonil(c2);
	bn->count = n;
	bn->tsorted = bn->trevsorted = bn->tkey = n <= 1;
	bn->tnil = 0;
	bn->tnonil = nonil1 && nonil2;
	return bn;
}

mgdk_bat *
calc_ifthenelse(mgdk_bat *b, mgdk_bat *b1, const void *cv1, mgdk_bat *b2, const void *cv2, int ct)
{
	if (b == nullptr || (b1 == nullptr && cv1 == nullptr) || (b2 == nullptr && cv2 == nullptr)) {
		seterr("BATcalcifthenelse: inputs must exist");
		return nullptr;
	}
	ProfScope prof("calcifthenelse");
	const int t1 = b1 ? b1->ttype : ct, t2 = b2 ? b2->ttype : ct;
	auto at = [](int t) { return t == MGDK_void ? MGDK_oid : t; };
	if ((b1 && b1->count != b->count) || (b2 && b2->count != b->count)) {
		seterr("BATcalcifthenelse: BATs have different lengths.\n");
		return nullptr;
	}
	if (b->ttype != MGDK_bit || at(t1) != at(t2)) {
		seterr("\"then\" and \"else\" BATs have different types.\n");
		return nullptr;
	}
	const int tp = at(t1);
	if (tp == MGDK_str)
		return ifthenelse_str(b, b1, (const char *) cv1, b2, (const char *) cv2);
	if (tp == MGDK_msk || width_of(tp) == 0) {
		seterr("BATcalcifthenelse: type %s is not on the device path", atomname(tp));
		return nullptr;
	}
	const BUN n = b->count;
	mgdk_bat *bn = newbat(b->hseqbase, tp, n);
	if (bn == nullptr)
		return nullptr;
	const int w = width_of(tp);
	// constants staged on the device
	DevBuf cb(64);
	if (!cb.p) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	char hc[64] = {0};
	if (cv1)
		memcpy(hc, cv1, w);
	if (cv2)
		memcpy(hc + 32, cv2, w);
	if (!hip_ok(hipMemcpyAsync(cb.p, hc, 64, hipMemcpyHostToDevice, stream()), "memcpy")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	auto src = [&](mgdk_bat *x, int k) -> const void * {
		if (x == nullptr)
			return (const char *) cb.p + 32 * k;
		return x->ttype == MGDK_void ? nullptr : (const void *) x->theap;
	};
	const oid seq1 = b1 && b1->ttype == MGDK_void ? b1->tseqbase : 0, seq2 = b2 && b2->ttype == MGDK_void ? b2->tseqbase : 0;
	if (n)
		hipLaunchKernelGGL(k_ifthenelse, dim3(grid_for(n, 256 * 4, 256 * 64)), dim3(256), 0, stream(),
				   (const int8_t *) b->theap, n, src(b1, 0), b1 == nullptr, seq1, src(b2, 1), b2 == nullptr, seq2, w,
				   bn->theap);
	if (!sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	auto cnonil = [&](const void *c) {
		Opnd o{};
		set_cst(o, c, basetype(tp) == MGDK_oid ? MGDK_oid : basetype(tp));
		return !o.cnil;
	};
	const bool nonil1 = b1 ? (bool) b1->tnonil : cnonil(cv1), nonil2 = b2 ? (bool) b2->tnonil : cnonil(cv2);
	bn->count = n;
	bn->tsorted = bn->trevsorted = bn->tkey = n <= 1;
	bn->tnil = 0;
	bn->tnonil = nonil1 && nonil2;
	return bn;
}

}  // namespace

extern "C" {

mgdk_bat *mgdk_BATcalccmp_op(int op, mgdk_bat *b1, const void *v1, int t1, mgdk_bat *b2, const void *v2, int t2,
			     mgdk_bat *s1, mgdk_bat *s2, bool nil_matches)
{
	if (op < OP_LT || op > OP_CMP || (b1 == nullptr && b2 == nullptr)) {
		seterr("BATcalccmp: bad arguments\n");
		return nullptr;
	}
	return calccmp(op, b1, v1, t1, b2, v2, t2, s1, s2, nil_matches);
}

#define CMPFN(NAME, OPC)                                                                                   \
	mgdk_bat *mgdk_BATcalc##NAME(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2)                 \
	{ return calccmp(OPC, b1, nullptr, 0, b2, nullptr, 0, s1, s2, false); }                           \
	mgdk_bat *mgdk_BATcalc##NAME##cst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s)                   \
	{ return calccmp(OPC, b, nullptr, 0, nullptr, v, vt, s, nullptr, false); }                        \
	mgdk_bat *mgdk_BATcalccst##NAME(const void *v, int vt, mgdk_bat *b, mgdk_bat *s)                     \
	{ return calccmp(OPC, nullptr, v, vt, b, nullptr, 0, s, nullptr, false); }
CMPFN(lt, OP_LT)
CMPFN(le, OP_LE)
CMPFN(gt, OP_GT)
CMPFN(ge, OP_GE)
CMPFN(cmp, OP_CMP)
#undef CMPFN

#define EQFN(NAME, OPC)                                                                                    \
	mgdk_bat *mgdk_BATcalc##NAME(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, bool nil_matches) \
	{ return calccmp(OPC, b1, nullptr, 0, b2, nullptr, 0, s1, s2, nil_matches); }                     \
	mgdk_bat *mgdk_BATcalc##NAME##cst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, bool nil_matches)   \
	{ return calccmp(OPC, b, nullptr, 0, nullptr, v, vt, s, nullptr, nil_matches); }                  \
	mgdk_bat *mgdk_BATcalccst##NAME(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, bool nil_matches)     \
	{ return calccmp(OPC, nullptr, v, vt, b, nullptr, 0, s, nullptr, nil_matches); }
EQFN(eq, OP_EQ)
EQFN(ne, OP_NE)
#undef EQFN

mgdk_bat *mgdk_BATcalcbetween(mgdk_bat *b, mgdk_bat *lo, mgdk_bat *hi, mgdk_bat *s, mgdk_bat *slo, mgdk_bat *shi,
			      bool symmetric, bool linc, bool hinc, bool nils_false, bool anti)
{ return calcbetween(b, lo, nullptr, hi, nullptr, b->ttype, s, slo, shi, symmetric, linc, hinc, nils_false, anti); }
mgdk_bat *mgdk_BATcalcbetweencstcst(mgdk_bat *b, const void *lo, const void *hi, int vt, mgdk_bat *s,
				    bool symmetric, bool linc, bool hinc, bool nils_false, bool anti)
{ return calcbetween(b, nullptr, lo, nullptr, hi, vt, s, nullptr, nullptr, symmetric, linc, hinc, nils_false, anti); }
mgdk_bat *mgdk_BATcalcbetweenbatcst(mgdk_bat *b, mgdk_bat *lo, const void *hi, int vt, mgdk_bat *s, mgdk_bat *slo,
				    bool symmetric, bool linc, bool hinc, bool nils_false, bool anti)
{ return calcbetween(b, lo, nullptr, nullptr, hi, vt, s, slo, nullptr, symmetric, linc, hinc, nils_false, anti); }
mgdk_bat *mgdk_BATcalcbetweencstbat(mgdk_bat *b, const void *lo, mgdk_bat *hi, int vt, mgdk_bat *s, mgdk_bat *shi,
				    bool symmetric, bool linc, bool hinc, bool nils_false, bool anti)
{ return calcbetween(b, nullptr, lo, hi, nullptr, vt, s, nullptr, shi, symmetric, linc, hinc, nils_false, anti); }

mgdk_bat *mgdk_BATconvert(mgdk_bat *b, mgdk_bat *s, int tp, uint8_t scale1, uint8_t scale2, uint8_t precision)
{ return convert(b, s, tp, scale1, scale2, precision); }

mgdk_bat *mgdk_BATcalcnot(mgdk_bat *b, mgdk_bat *s)
{ return calcnot(b, s); }

mgdk_bat *mgdk_BATcalcdiv(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp)
{ return calcdivmod(true, b1, nullptr, 0, b2, nullptr, 0, s1, s2, tp); }
mgdk_bat *mgdk_BATcalcdivcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp)
{ return calcdivmod(true, b, nullptr, 0, nullptr, v, vt, s, nullptr, tp); }
mgdk_bat *mgdk_BATcalccstdiv(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp)
{ return calcdivmod(true, nullptr, v, vt, b, nullptr, 0, s, nullptr, tp); }
mgdk_bat *mgdk_BATcalcmod(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp)
{ return calcdivmod(false, b1, nullptr, 0, b2, nullptr, 0, s1, s2, tp); }
mgdk_bat *mgdk_BATcalcmodcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp)
{ return calcdivmod(false, b, nullptr, 0, nullptr, v, vt, s, nullptr, tp); }
mgdk_bat *mgdk_BATcalccstmod(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp)
{ return calcdivmod(false, nullptr, v, vt, b, nullptr, 0, s, nullptr, tp); }


// the rest of gdk_calc.c's element-wise operators (calc_unary & co. above)
mgdk_bat *mgdk_BATcalcnegate(mgdk_bat *b, mgdk_bat *s) { return calc_unary(X_NEG, b, s); }
mgdk_bat *mgdk_BATcalcabsolute(mgdk_bat *b, mgdk_bat *s) { return calc_unary(X_ABS, b, s); }
mgdk_bat *mgdk_BATcalciszero(mgdk_bat *b, mgdk_bat *s) { return calc_unary(X_ISZERO, b, s); }
mgdk_bat *mgdk_BATcalcsign(mgdk_bat *b, mgdk_bat *s) { return calc_unary(X_SIGN, b, s); }
mgdk_bat *mgdk_BATcalcisnil(mgdk_bat *b, mgdk_bat *s) { return calc_unary(X_ISNIL, b, s); }
mgdk_bat *mgdk_BATcalcisnotnil(mgdk_bat *b, mgdk_bat *s) { return calc_unary(X_ISNOTNIL, b, s); }

// BATcalcincr / BATcalcdecr (gdk_calc_addsub.c:1681-1760): b + 1 / b - 1 in
// b's type with the overflow check of BATcalcaddcst; the properties as
// BATcalcincrdecr sets them.  (The reference's loop passes its candidate
// iterators in swapped roles and computes only the first row; the device
// computes every row.)
static mgdk_bat *
incrdecr(mgdk_bat *b, mgdk_bat *s, bool incr)
{
	if (b == nullptr) {
		seterr("BATcalcincr: b must exist");
		return nullptr;
	}
	const int8_t one = 1;
	mgdk_bat *bn = incr ? mgdk_BATcalcaddcst(b, &one, MGDK_bte, s, b->ttype)
			    : mgdk_BATcalcsubcst(b, &one, MGDK_bte, s, b->ttype);
	if (bn == nullptr)
		return nullptr;
	const BUN n = bn->count;
	const bool allnil = bn->tnil && n > 0 && !bn->tnonil && false;
	(void) allnil;
	bn->tsorted = b->tsorted || n <= 1 || (bn->tnil && n == 1);
	bn->trevsorted = b->trevsorted || n <= 1;
	bn->tkey = n <= 1;
	return bn;
}
mgdk_bat *mgdk_BATcalcincr(mgdk_bat *b, mgdk_bat *s) { return incrdecr(b, s, true); }
mgdk_bat *mgdk_BATcalcdecr(mgdk_bat *b, mgdk_bat *s) { return incrdecr(b, s, false); }

mgdk_bat *mgdk_BATcalcmin(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2)
{ return calc_minmax(X_MIN, b1, b2, nullptr, 0, s1, s2); }
mgdk_bat *mgdk_BATcalcmax(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2)
{ return calc_minmax(X_MAX, b1, b2, nullptr, 0, s1, s2); }
mgdk_bat *mgdk_BATcalcmin_no_nil(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2)
{ return calc_minmax(X_MINNN, b1, b2, nullptr, 0, s1, s2); }
mgdk_bat *mgdk_BATcalcmax_no_nil(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2)
{ return calc_minmax(X_MAXNN, b1, b2, nullptr, 0, s1, s2); }
mgdk_bat *mgdk_BATcalcmincst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s)
{ return calc_minmax(X_MIN, b, nullptr, v, vt, s, nullptr); }
mgdk_bat *mgdk_BATcalcmaxcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s)
{ return calc_minmax(X_MAX, b, nullptr, v, vt, s, nullptr); }
mgdk_bat *mgdk_BATcalcmincst_no_nil(mgdk_bat *b, const void *v, int vt, mgdk_bat *s)
{ return calc_minmax(X_MINNN, b, nullptr, v, vt, s, nullptr); }
mgdk_bat *mgdk_BATcalcmaxcst_no_nil(mgdk_bat *b, const void *v, int vt, mgdk_bat *s)
{ return calc_minmax(X_MAXNN, b, nullptr, v, vt, s, nullptr); }
mgdk_bat *mgdk_BATcalccstmin(const void *v, int vt, mgdk_bat *b, mgdk_bat *s)
{ return calc_minmax(X_MIN, b, nullptr, v, vt, s, nullptr); }
mgdk_bat *mgdk_BATcalccstmax(const void *v, int vt, mgdk_bat *b, mgdk_bat *s)
{ return calc_minmax(X_MAX, b, nullptr, v, vt, s, nullptr); }
mgdk_bat *mgdk_BATcalccstmin_no_nil(const void *v, int vt, mgdk_bat *b, mgdk_bat *s)
{ return calc_minmax(X_MINNN, b, nullptr, v, vt, s, nullptr); }
mgdk_bat *mgdk_BATcalccstmax_no_nil(const void *v, int vt, mgdk_bat *b, mgdk_bat *s)
{ return calc_minmax(X_MAXNN, b, nullptr, v, vt, s, nullptr); }

#define BITFN(NAME, OPC)                                                                                   \
	mgdk_bat *mgdk_BATcalc##NAME(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2)                 \
	{ return calc_bits(OPC, "BATcalc" #NAME, b1, nullptr, 0, b2, nullptr, 0, s1, s2); }               \
	mgdk_bat *mgdk_BATcalc##NAME##cst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s)                    \
	{ return calc_bits(OPC, "BATcalc" #NAME "cst", b, nullptr, 0, nullptr, v, vt, s, nullptr); }      \
	mgdk_bat *mgdk_BATcalccst##NAME(const void *v, int vt, mgdk_bat *b, mgdk_bat *s)                    \
	{ return calc_bits(OPC, "BATcalccst" #NAME, nullptr, v, vt, b, nullptr, 0, s, nullptr); }
BITFN(and, X_AND)
BITFN(or, X_OR)
BITFN(xor, X_XOR)
BITFN(lsh, X_LSH)
BITFN(rsh, X_RSH)
#undef BITFN

mgdk_bat *mgdk_BATcalcifthenelse(mgdk_bat *b, mgdk_bat *b1, mgdk_bat *b2)
{ return calc_ifthenelse(b, b1, nullptr, b2, nullptr, 0); }
mgdk_bat *mgdk_BATcalcifthenelsecst(mgdk_bat *b, mgdk_bat *b1, const void *c2, int ct)
{ return calc_ifthenelse(b, b1, nullptr, nullptr, c2, ct); }
mgdk_bat *mgdk_BATcalcifthencstelse(mgdk_bat *b, const void *c1, int ct, mgdk_bat *b2)
{ return calc_ifthenelse(b, nullptr, c1, b2, nullptr, ct); }
mgdk_bat *mgdk_BATcalcifthencstelsecst(mgdk_bat *b, const void *c1, const void *c2, int ct)
{ return calc_ifthenelse(b, nullptr, c1, nullptr, c2, ct); }

}  // extern "C"
