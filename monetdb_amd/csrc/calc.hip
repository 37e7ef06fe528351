// calc.hip -- BATcalc{add,sub,mul}[cst] for the integer types on the MI355X.
//
// Semantics of gdk/gdk_calc_addsub.c and gdk/gdk_calc_mul.c (MUL_4TYPE /
// MUL_3TYPE_enlarge :23-132, BATcalcmuldivmod :2020-2082): the result has
// one value per candidate pair, nil if either operand is nil, and the
// operation is computed exactly (128-bit here) and checked against the
// result type's range [-max, max] (OP_WITH_CHECK, gdk_calc_private.h:38-46;
// hitting the nil value counts as overflow).  The first overflowing pair in
// candidate order is reported with the reference's message
// "22003!overflow in calculation <a><op><b>.".  Operands are widened from
// 1/2/4/8/16-byte storage; lng*lng->hge (the TPC-H decimal products) can
// never overflow and takes no check.  Streaming, one pass, coalesced.
#include <cstdio>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

struct Operand {
	const void *base;   // tail (NULL for a constant)
	int w;              // storage width
	hge c;              // constant value
	bool cnil;
	bool dense;         // candidates dense: position = seq - hseq + i
	oid off;            // dense: seq - hseq
	const oid *oids;    // materialized candidates
	oid hseq;
};

__device__ __forceinline__ hge
ld(const void *base, int w, BUN p, bool &isnil)
{
	switch (w) {
	case 1: { int8_t v = ((const int8_t *) base)[p]; isnil = v == INT8_MIN; return v; }
	case 2: { int16_t v = ((const int16_t *) base)[p]; isnil = v == INT16_MIN; return v; }
	case 4: { int32_t v = ((const int32_t *) base)[p]; isnil = v == INT32_MIN; return v; }
	case 8: { int64_t v = ((const int64_t *) base)[p]; isnil = v == INT64_MIN; return v; }
	default: { hge v = ((const hge *) base)[p]; isnil = is_nil(v); return v; }
	}
}

__device__ __forceinline__ hge
operand(const Operand &o, BUN i, bool &isnil)
{
	if (o.base == nullptr) {
		isnil = o.cnil;
		return o.c;
	}
	BUN p = o.dense ? o.off + i : o.oids[i] - o.hseq;
	return ld(o.base, o.w, p, isnil);
}

__device__ __host__ __forceinline__ bool
add_ovf(hge a, hge b, hge &r)
{
	r = (hge) ((uhge) a + (uhge) b);
	return ((a < 0) == (b < 0)) && ((r < 0) != (a < 0));
}

__device__ __host__ __forceinline__ bool
sub_ovf(hge a, hge b, hge &r)
{
	r = (hge) ((uhge) a - (uhge) b);
	return ((a < 0) != (b < 0)) && ((r < 0) != (a < 0));
}

__device__ __host__ __forceinline__ bool
mul_ovf(hge a, hge b, hge &r)
{
	const bool neg = (a < 0) != (b < 0);
	const uhge ua = a < 0 ? (uhge) 0 - (uhge) a : (uhge) a;
	const uhge ub = b < 0 ? (uhge) 0 - (uhge) b : (uhge) b;
	const uint64_t ah = (uint64_t) (ua >> 64), al = (uint64_t) ua;
	const uint64_t bh = (uint64_t) (ub >> 64), bl = (uint64_t) ub;
	if (ah && bh)
		return true;
	const uhge lo = (uhge) al * bl;
	const uhge mid = (uhge) ah * bl + (uhge) bh * al;
	if (mid >> 64)
		return true;
	const uhge res = lo + (mid << 64);
	if (res < lo || res >= ((uhge) 1 << 127))
		return true;
	r = neg ? -(hge) res : (hge) res;
	return false;
}

__device__ __forceinline__ void
st(void *base, int w, BUN i, hge v)
{
	switch (w) {
	case 1: ((int8_t *) base)[i] = (int8_t) v; break;
	case 2: ((int16_t *) base)[i] = (int16_t) v; break;
	case 4: ((int32_t *) base)[i] = (int32_t) v; break;
	case 8: ((int64_t *) base)[i] = (int64_t) v; break;
	default: ((hge *) base)[i] = v; break;
	}
}

// OP: 0 add, 1 sub, 2 mul; CHECK: range/overflow check needed.  Each wave
// streams 64 * U consecutive candidates per step (element = chunk base +
// u * 64 + lane), all U operand pairs loaded before any is used.
template <int OP, bool CHECK>
__global__ __launch_bounds__(256) void
k_calc(Operand a, Operand b, void *out, int ow, hge max, BUN n, hge nilv,
       unsigned long long *first_ovf, unsigned long long *nils)
{
	constexpr int U = 8;
	constexpr BUN CH = 64 * U;
	unsigned long long mynils = 0, myovf = ~0ull;
	const unsigned lane = __lane_id();
	const BUN nwaves = (BUN) gridDim.x * (blockDim.x / 64);
	for (BUN ch = (BUN) blockIdx.x * (blockDim.x / 64) + (threadIdx.x / 64); ch * CH < n; ch += nwaves) {
		const BUN i0 = ch * CH + lane;
		hge x[U], y[U];
		bool n1[U], n2[U];
		// loads at a clamped index, unconditionally (a load under a divergent
		// branch is waited for before the branch joins)
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * 64;
			const BUN ic = i < n ? i : n - 1;
			x[u] = operand(a, ic, n1[u]);
			y[u] = operand(b, ic, n2[u]);
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * 64;
			if (i >= n)
				continue;
			if (n1[u] || n2[u]) {
				st(out, ow, i, nilv);
				mynils++;
				continue;
			}
			hge r;
			bool ovf;
			if (OP == 0) ovf = add_ovf(x[u], y[u], r);
			else if (OP == 1) ovf = sub_ovf(x[u], y[u], r);
			else ovf = mul_ovf(x[u], y[u], r);
			if (CHECK && (ovf || r < -max || r > max)) {
				if (i < myovf)
					myovf = i;
				continue;
			}
			st(out, ow, i, r);
		}
	}
	// block reduce then one atomic per workgroup
	mynils = block_reduce(mynils, [](decltype(mynils) x, decltype(mynils) y) { return x + y; });
	myovf = block_reduce(myovf, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	if (threadIdx.x == 0) {
		if (mynils)
			atomicAdd(nils, mynils);
		if (myovf != ~0ull)
			atomicMin(first_ovf, myovf);
	}
}

// Width-generic load without branches: the 16-byte aligned word holding the
// value is loaded and the value shifted out and sign-extended (heaps are at
// least 16-byte aligned and padded, so the word never leaves the heap).  A
// runtime width switch would put each load in its own block, and the
// compiler waits for every such load before the block joins.
__device__ __forceinline__ hge
ld_any(const void *base, int w, BUN p, bool &isnil)
{
	const uintptr_t a = (uintptr_t) base + (uintptr_t) p * (uintptr_t) w;
	const uint4 q = *(const uint4 *) (a & ~(uintptr_t) 15);
	const unsigned sh = (unsigned) (a & 15) * 8;
	uhge x = ((uhge) (((unsigned long long) q.w << 32) | q.z) << 64) | (((unsigned long long) q.y << 32) | q.x);
	x >>= sh;
	const unsigned bits = 8u * (unsigned) w;
	const unsigned up = 128u - bits;
	const hge v = up ? ((hge) (x << up) >> up) : (hge) x;
	const hge nilv = up ? -((hge) 1 << (bits - 1)) : (hge) ((uhge) 1 << 127);
	isnil = v == nilv;
	return v;
}

// typed load for the common 8- and 16-byte operands (one 8- or 16-byte load
// per value instead of ld_any's 16-byte word), ld_any for the others (W = 0)
template <int W>
__device__ __forceinline__ hge
ld_t(const void *base, int w, BUN p, bool &isnil)
{
	if constexpr (W == 8) {
		const int64_t x = ((const int64_t *) base)[p];
		isnil = x == INT64_MIN;
		return x;
	} else if constexpr (W == 16) {
		const hge x = ((const hge *) base)[p];
		isnil = x == (hge) ((uhge) 1 << 127);
		return x;
	} else {
		return ld_any(base, w, p, isnil);
	}
}

// fast path: dense candidates (or constants: CA / CB), branch-free loads
template <int OP, bool CHECK, bool CA, bool CB, int WA, int WB>
__global__ __launch_bounds__(256) void
k_calc_d(Operand a, Operand b, void *out, int ow, hge max, BUN n, hge nilv,
	 unsigned long long *first_ovf, unsigned long long *nils)
{
	constexpr int U = 8;
	constexpr BUN CH = 64 * U;
	unsigned long long mynils = 0, myovf = ~0ull;
	const unsigned lane = __lane_id();
	const BUN nwaves = (BUN) gridDim.x * (blockDim.x / 64);
	for (BUN ch = (BUN) blockIdx.x * (blockDim.x / 64) + (threadIdx.x / 64); ch * CH < n; ch += nwaves) {
		const BUN i0 = ch * CH + lane;
		hge x[U], y[U];
		bool n1[U], n2[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * 64;
			const BUN ic = i < n ? i : n - 1;
			if (CA) { x[u] = a.c; n1[u] = a.cnil; } else x[u] = ld_t<WA>(a.base, a.w, a.off + ic, n1[u]);
			if (CB) { y[u] = b.c; n2[u] = b.cnil; } else y[u] = ld_t<WB>(b.base, b.w, b.off + ic, n2[u]);
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * 64;
			if (i >= n)
				continue;
			if (n1[u] || n2[u]) {
				st(out, ow, i, nilv);
				mynils++;
				continue;
			}
			hge r;
			bool ovf;
			if (OP == 0) ovf = add_ovf(x[u], y[u], r);
			else if (OP == 1) ovf = sub_ovf(x[u], y[u], r);
			else ovf = mul_ovf(x[u], y[u], r);
			if (CHECK && (ovf || r < -max || r > max)) {
				if (i < myovf)
					myovf = i;
				continue;
			}
			st(out, ow, i, r);
		}
	}
	mynils = block_reduce(mynils, [](decltype(mynils) x, decltype(mynils) y) { return x + y; });
	myovf = block_reduce(myovf, [](unsigned long long x, unsigned long long y) { return x < y ? x : y; });
	if (threadIdx.x == 0) {
		if (mynils)
			atomicAdd(nils, mynils);
		if (myovf != ~0ull)
			atomicMin(first_ovf, myovf);
	}
}

__global__ void
k_operands_at(Operand a, Operand b, BUN i, hge *out)
{
	bool n1, n2;
	out[0] = operand(a, i, n1);
	out[1] = operand(b, i, n2);
}

bool
is_int_type(int t)
{
	t = basetype(t);
	return t == MGDK_bte || t == MGDK_sht || t == MGDK_int || t == MGDK_lng || t == MGDK_hge;
}

hge
type_max(int t)
{
	switch (basetype(t)) {
	case MGDK_bte: return INT8_MAX;
	case MGDK_sht: return INT16_MAX;
	case MGDK_int: return INT32_MAX;
	case MGDK_lng: return INT64_MAX;
	default: return (hge) (((uhge) 1 << 127) - 1);
	}
}

void
fmtval(char *buf, size_t sz, int t, hge v)
{
	switch (basetype(t)) {
	case MGDK_bte: case MGDK_sht: case MGDK_int: snprintf(buf, sz, "%d", (int) v); break;
	case MGDK_lng: snprintf(buf, sz, "%lld", (long long) v); break;
	default: snprintf(buf, sz, "%.40Lg (approx. value)", (long double) v); break;
	}
}

hge
cst_value(const void *v, int vt, bool &isnil)
{
	switch (basetype(vt)) {
	case MGDK_bte: { int8_t x = *(const int8_t *) v; isnil = x == INT8_MIN; return x; }
	case MGDK_sht: { int16_t x = *(const int16_t *) v; isnil = x == INT16_MIN; return x; }
	case MGDK_int: { int32_t x = *(const int32_t *) v; isnil = x == INT32_MIN; return x; }
	case MGDK_lng: { int64_t x = *(const int64_t *) v; isnil = x == INT64_MIN; return x; }
	default: { hge x; memcpy(&x, v, 16); isnil = is_nil(x); return x; }
	}
}

// b1/b2 may be NULL when the constant (v1/v2) is used
mgdk_bat *
calc(int op, mgdk_bat *b1, const void *v1, int t1, mgdk_bat *b2, const void *v2, int t2,
     mgdk_bat *s1, mgdk_bat *s2, int tp)
{
	static const char *opname[] = {"+", "-", "*"};
	static const char *fname[] = {"BATcalcadd", "BATcalcsub", "BATcalcmul"};
	if (b1)
		t1 = b1->ttype;
	if (b2)
		t2 = b2->ttype;
	if (!is_int_type(t1) || !is_int_type(t2) || !is_int_type(tp)) {
		seterr("%s: type combination %s(%s,%s)->%s) not supported.\n", fname[op],
		       op == 0 ? "add" : op == 1 ? "sub" : "mul", atomname(t1), atomname(t2), atomname(tp));
		return nullptr;
	}
	ProfScope prof("calc");
	Cand c1{}, c2{};
	mgdk_bat *bb = b1 ? b1 : b2;
	if (b1 && cand_init(&c1, b1, s1) < 0)
		return nullptr;
	if (b2 && cand_init(&c2, b2, b1 ? s2 : s1) < 0)
		return nullptr;
	oid hseq1 = b1 ? (s1 ? s1->hseqbase : b1->hseqbase) : 0;
	oid hseq2 = b2 ? ((b1 ? s2 : s1) ? (b1 ? s2 : s1)->hseqbase : b2->hseqbase) : 0;
	if (b1 && b2 && (c1.n != c2.n || hseq1 != hseq2)) {
		seterr("%s: inputs not the same size.\n", fname[op]);
		return nullptr;
	}
	const Cand &ci = b1 ? c1 : c2;
	const BUN n = ci.n;
	mgdk_bat *bn = newbat(b1 ? hseq1 : hseq2, tp, n);
	if (bn == nullptr)
		return nullptr;
	if (n == 0) {
		bn->count = 0;
		return bn;
	}
	Operand A{}, B{};
	auto setop = [](Operand &o, mgdk_bat *b, const Cand &c, const void *v, int vt) {
		if (b) {
			o.base = b->theap;
			o.w = b->twidth;
			o.dense = c.dense;
			o.off = c.dense ? c.seq - b->hseqbase : 0;
			o.oids = c.oids;
			o.hseq = b->hseqbase;
		} else {
			o.base = nullptr;
			o.c = cst_value(v, vt, o.cnil);
		}
	};
	setop(A, b1, c1, v1, t1);
	setop(B, b2, c2, v2, t2);
	const int ow = width_of(tp);
	const hge max = type_max(tp);
	// lng*lng (or narrower) into hge cannot overflow (MUL_3TYPE_enlarge's
	// couldoverflow == false); neither can narrow add/sub into hge
	const int w1 = width_of(t1), w2 = width_of(t2);
	bool check = true;
	if (basetype(tp) == MGDK_hge && w1 <= 8 && w2 <= 8)
		check = false;
	unsigned long long *m = (unsigned long long *) meta_buf();
	unsigned long long init[2] = {~0ull, 0ull};
	if (!hip_ok(hipMemcpyAsync(m, init, 16, hipMemcpyHostToDevice, stream()), "memcpy")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	hge nilv = (hge) ((uhge) 1 << 127);
	switch (ow) {
	case 1: nilv = INT8_MIN; break;
	case 2: nilv = INT16_MIN; break;
	case 4: nilv = INT32_MIN; break;
	case 8: nilv = INT64_MIN; break;
	}
	dim3 g(grid_for(n, 256 * 8, 256 * 16)), blk(256);
	const bool fast = (A.base == nullptr || A.dense) && (B.base == nullptr || B.dense);
	// operand widths with a typed loader (8 / 16 bytes), 0: generic
	const int wa = A.base && (A.w == 8 || A.w == 16) ? A.w : 0;
	const int wb = B.base && (B.w == 8 || B.w == 16) ? B.w : 0;
#define LAUNCHD(OPC, CHK, CA_, CB_, WA_, WB_) hipLaunchKernelGGL((k_calc_d<OPC, CHK, CA_, CB_, WA_, WB_>), g, blk, 0, stream(), A, B, bn->theap, ow, max, n, nilv, m, m + 1)
#define LW(OPC, CHK, CA_, CB_, WA_) do { if (wb == 8) LAUNCHD(OPC, CHK, CA_, CB_, WA_, 8); \
		else if (wb == 16) LAUNCHD(OPC, CHK, CA_, CB_, WA_, 16); else LAUNCHD(OPC, CHK, CA_, CB_, WA_, 0); } while (0)
#define LAUNCH(OPC, CHK) do { if (!fast) hipLaunchKernelGGL((k_calc<OPC, CHK>), g, blk, 0, stream(), A, B, bn->theap, ow, max, n, nilv, m, m + 1); \
		else if (A.base == nullptr) LW(OPC, CHK, true, false, 0); \
		else if (B.base == nullptr) { if (wa == 8) LAUNCHD(OPC, CHK, false, true, 8, 0); \
			else if (wa == 16) LAUNCHD(OPC, CHK, false, true, 16, 0); else LAUNCHD(OPC, CHK, false, true, 0, 0); } \
		else if (wa == 8) LW(OPC, CHK, false, false, 8); \
		else if (wa == 16) LW(OPC, CHK, false, false, 16); \
		else LW(OPC, CHK, false, false, 0); } while (0)
	if (op == 0) { if (check) LAUNCH(0, true); else LAUNCH(0, false); }
	else if (op == 1) { if (check) LAUNCH(1, true); else LAUNCH(1, false); }
	else { if (check) LAUNCH(2, true); else LAUNCH(2, false); }
#undef LAUNCH
#undef LW
#undef LAUNCHD
	unsigned long long *h = (unsigned long long *) pinned(64);
	if (h == nullptr || !hip_ok(hipMemcpyAsync(h, m, 16, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[0] != ~0ull) {
		hge *dv = (hge *) (m + 4);
		hipLaunchKernelGGL(k_operands_at, dim3(1), dim3(1), 0, stream(), A, B, (BUN) h[0], dv);
		hge vals[2] = {0, 0};
		if (hip_ok(hipMemcpyAsync(h + 2, dv, 32, hipMemcpyDeviceToHost, stream()), "memcpy") && sync())
			memcpy(vals, h + 2, 32);
		char a[64], b[64];
		fmtval(a, sizeof(a), t1, vals[0]);
		fmtval(b, sizeof(b), t2, vals[1]);
		seterr("22003!overflow in calculation %s%s%s.\n", a, opname[op], b);
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const BUN nils = h[1];
	bn->count = n;
	// result order (gdk_calc_addsub.c:1528-1531, 1590-1593, 1649-1652,
	// 3208-3209, 3262-3265, 3318-3321; gdk_calc_mul.c:2068-2069, 2133-2138,
	// 2194-2199): a constant operand keeps the BAT's order (a negative
	// multiplier or cst - b reverses it), two sorted BATs add to a sorted
	// result, anything else is unordered; only without nils
	bool srt = false, rev = false;
	if (nils == 0) {
		if (b1 && b2) {
			if (op == 0) {
				srt = b1->tsorted && b2->tsorted;
				rev = b1->trevsorted && b2->trevsorted;
			}
		} else {
			int sign = 1;
			if (op == 2) {
				bool cn;
				const hge c = cst_value(b1 ? v2 : v1, b1 ? t2 : t1, cn);
				sign = c > 0 ? 1 : c < 0 ? -1 : 0;
			} else if (op == 1 && !b1) {
				sign = -1;
			}
			srt = (sign >= 0 && bb->tsorted) || (sign <= 0 && bb->trevsorted);
			rev = (sign >= 0 && bb->trevsorted) || (sign <= 0 && bb->tsorted);
		}
	}
	bn->tsorted = srt || n <= 1 || nils == n;
	bn->trevsorted = rev || n <= 1 || nils == n;
	bn->tkey = n <= 1;
	bn->tnil = nils != 0;
	bn->tnonil = nils == 0;
	return bn;
}

}  // namespace

extern "C" {

mgdk_bat *mgdk_BATcalcadd(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp)
{ return calc(0, b1, nullptr, 0, b2, nullptr, 0, s1, s2, tp); }
mgdk_bat *mgdk_BATcalcsub(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp)
{ return calc(1, b1, nullptr, 0, b2, nullptr, 0, s1, s2, tp); }
mgdk_bat *mgdk_BATcalcmul(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *s1, mgdk_bat *s2, int tp)
{ return calc(2, b1, nullptr, 0, b2, nullptr, 0, s1, s2, tp); }
mgdk_bat *mgdk_BATcalcaddcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp)
{ return calc(0, b, nullptr, 0, nullptr, v, vt, s, nullptr, tp); }
mgdk_bat *mgdk_BATcalcsubcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp)
{ return calc(1, b, nullptr, 0, nullptr, v, vt, s, nullptr, tp); }
mgdk_bat *mgdk_BATcalcmulcst(mgdk_bat *b, const void *v, int vt, mgdk_bat *s, int tp)
{ return calc(2, b, nullptr, 0, nullptr, v, vt, s, nullptr, tp); }
mgdk_bat *mgdk_BATcalccstadd(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp)
{ return calc(0, nullptr, v, vt, b, nullptr, 0, s, nullptr, tp); }
mgdk_bat *mgdk_BATcalccstsub(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp)
{ return calc(1, nullptr, v, vt, b, nullptr, 0, s, nullptr, tp); }
mgdk_bat *mgdk_BATcalccstmul(const void *v, int vt, mgdk_bat *b, mgdk_bat *s, int tp)
{ return calc(2, nullptr, v, vt, b, nullptr, 0, s, nullptr, tp); }

}  // extern "C"
