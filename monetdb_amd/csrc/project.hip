// project.hip -- BATproject on the MI355X (gdk/gdk_project.c:590-857).
//
// out[i] = r[l[i] - r.hseqbase].  A dense l that lies inside r is a
// zero-copy slice view (BATslice, gdk_project.c:623-645); otherwise a
// gather kernel reads the oid list with 16-byte loads (two oids per lane)
// and gathers the values (1/2/4/8/16 B).  A nil oid gives nil, an oid
// outside r is the reference's "does not match always" error.  str columns
// gather their heap offsets and share the string heap (the "stringtrick",
// gdk_project.c:681-718).
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void
k_project(const oid *__restrict__ l, BUN n, const T *__restrict__ r, oid rseq, BUN rcnt, T nilv,
	  T *__restrict__ out, uint32_t *__restrict__ flags)
{
	const BUN stride = (BUN) gridDim.x * blockDim.x * 2;
	uint32_t bad = 0, nil = 0;
	for (BUN i = ((BUN) blockIdx.x * blockDim.x + threadIdx.x) * 2; i < n; i += stride) {
		oid o0 = l[i];
		oid o1 = i + 1 < n ? l[i + 1] : rseq;
		T v0, v1;
		if (o0 == MGDK_OID_NIL) { v0 = nilv; nil = 1; }
		else if (o0 - rseq >= rcnt) { v0 = nilv; bad = 1; }
		else v0 = r[o0 - rseq];
		if (o1 == MGDK_OID_NIL) { v1 = nilv; nil = 1; }
		else if (o1 - rseq >= rcnt) { v1 = nilv; bad = 1; }
		else v1 = r[o1 - rseq];
		out[i] = v0;
		if (i + 1 < n)
			out[i + 1] = v1;
	}
	bad = block_reduce(bad, [](uint32_t x, uint32_t y) { return x | y; });
	nil = block_reduce(nil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0) {
		publish_or(&flags[0], bad);
		publish_or(&flags[1], nil);
	}
}

// r is a dense oid column: values are r.tseqbase + (o - rseq)
__global__ __launch_bounds__(256) void
k_project_void(const oid *__restrict__ l, BUN n, oid rseq, BUN rcnt, oid rtseq,
	       oid *__restrict__ out, uint32_t *__restrict__ flags)
{
	uint32_t bad = 0, nil = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		oid o = l[i];
		if (o == MGDK_OID_NIL) { out[i] = MGDK_OID_NIL; nil = 1; }
		else if (o - rseq >= rcnt) { out[i] = MGDK_OID_NIL; bad = 1; }
		else out[i] = rtseq == MGDK_OID_NIL ? MGDK_OID_NIL : rtseq + (o - rseq);
	}
	bad = block_reduce(bad, [](uint32_t x, uint32_t y) { return x | y; });
	nil = block_reduce(nil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0) {
		publish_or(&flags[0], bad);
		publish_or(&flags[1], nil);
	}
}

template <typename T>
static void
launch(const oid *l, BUN n, const void *r, oid rseq, BUN rcnt, const void *nilp, void *out,
       uint32_t *flags)
{
	T nilv;
	memcpy(&nilv, nilp, sizeof(T));
	unsigned g = grid_for(n, 512, 256 * 16);
	hipLaunchKernelGGL((k_project<T>), dim3(g), dim3(256), 0, stream(), l, n, (const T *) r, rseq, rcnt,
			   nilv, (T *) out, flags);
}

}  // namespace

extern "C" mgdk_bat *
mgdk_BATproject(mgdk_bat *l, mgdk_bat *r)
{
	if (l == nullptr || r == nullptr) {
		seterr("BATproject: NULL argument");
		return nullptr;
	}
	if (l->ttype != MGDK_void && l->ttype != MGDK_oid) {
		seterr("BATproject: left must be oid");
		return nullptr;
	}
	ProfScope prof("project");
	const BUN n = l->count;
	const int rt = r->ttype;
	if (l->ttype == MGDK_void && n > 0) {
		if (l->tseqbase == MGDK_OID_NIL) {
			// all-nil left: BATconstant of nil (gdk_project.c:650-670)
			alignas(16) unsigned char nilv[16] = {0};
			switch (basetype(rt)) {
			case MGDK_bte: *(int8_t *) nilv = INT8_MIN; break;
			case MGDK_sht: *(int16_t *) nilv = INT16_MIN; break;
			case MGDK_int: *(int32_t *) nilv = INT32_MIN; break;
			case MGDK_lng: *(int64_t *) nilv = INT64_MIN; break;
			case MGDK_oid: case MGDK_void: *(uint64_t *) nilv = MGDK_OID_NIL; break;
			case MGDK_hge: nilv[15] = 0x80; break;
			default:
				seterr("42000!BATproject: nil projection of %s unsupported", atomname(rt));
				return nullptr;
			}
			return mgdk_BATconstant(l->hseqbase, rt == MGDK_void ? MGDK_oid : rt, nilv, n);
		}
		oid lo = l->tseqbase, hi = l->tseqbase + n;
		if (lo >= r->hseqbase && hi <= r->hseqbase + r->count) {
			mgdk_bat *bn = mgdk_BATslice(r, lo - r->hseqbase, hi - r->hseqbase);
			if (bn)
				bn->hseqbase = l->hseqbase;
			return bn;
		}
		seterr("does not match always\n");
		return nullptr;
	}
	if (n == 0) {
		mgdk_bat *bn = newbat(l->hseqbase, rt == MGDK_oid ? MGDK_void : rt, 0);
		if (bn && rt == MGDK_str)
			share_vheap(bn, r);
		return bn;
	}
	// l is a materialised oid list
	const int ot = rt == MGDK_void ? MGDK_oid : rt;
	const int alloc_t = rt != MGDK_str ? ot
		: r->twidth == 1 ? MGDK_bte : r->twidth == 2 ? MGDK_sht : r->twidth == 4 ? MGDK_int : MGDK_lng;
	mgdk_bat *bn = newbat(l->hseqbase, alloc_t, n);
	if (bn == nullptr)
		return nullptr;
	if (rt == MGDK_str) {
		bn->ttype = MGDK_str;   // offsets of the shared string heap
		share_vheap(bn, r);
	}
	uint32_t *flags = (uint32_t *) meta_buf();
	if (!hip_ok(hipMemsetAsync(flags, 0, 16, stream()), "memset")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const oid *lo = (const oid *) l->theap;
	alignas(16) unsigned char nilv[16] = {0};
	if (rt == MGDK_void) {
		hipLaunchKernelGGL(k_project_void, dim3(grid_for(n, 256, 256 * 16)), dim3(256), 0, stream(), lo, n,
				   r->hseqbase, r->count, r->tseqbase, (oid *) bn->theap, flags);
	} else {
		switch (rt == MGDK_str ? -r->twidth : basetype(rt)) {
		case MGDK_bte: *(int8_t *) nilv = INT8_MIN; launch<int8_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case MGDK_sht: *(int16_t *) nilv = INT16_MIN; launch<int16_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case MGDK_int: *(int32_t *) nilv = INT32_MIN; launch<int32_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case MGDK_flt: { float f = __builtin_nanf(""); memcpy(nilv, &f, 4); launch<int32_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break; }
		case MGDK_lng: *(int64_t *) nilv = INT64_MIN; launch<int64_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case MGDK_oid: *(uint64_t *) nilv = MGDK_OID_NIL; launch<int64_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case MGDK_dbl: { double d = __builtin_nan(""); memcpy(nilv, &d, 8); launch<int64_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break; }
		case MGDK_hge: nilv[15] = 0x80; launch<hge>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case -1: launch<uint8_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case -2: launch<uint16_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case -4: launch<uint32_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		case -8: launch<uint64_t>(lo, n, r->theap, r->hseqbase, r->count, nilv, bn->theap, flags); break;
		default:
			seterr("42000!BATproject: type %s not supported on the device path", atomname(rt));
			mgdk_BBPunfix(bn);
			return nullptr;
		}
	}
	uint32_t *h = (uint32_t *) pinned(16);
	if (h == nullptr || !hip_ok(hipMemcpyAsync(h, flags, 8, hipMemcpyDeviceToHost, stream()), "memcpy") ||
	    !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[0]) {
		seterr("does not match always\n");
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (h[1] && rt == MGDK_str) {
		seterr("42000!BATproject: nil oid into a str column unsupported on the device path");
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	bn->count = n;
	bn->tnil = h[1] != 0;
	bn->tnonil = l->tnonil && r->tnonil && !h[1];
	bn->tsorted = n <= 1 || (l->tsorted && r->tsorted) || (l->trevsorted && r->trevsorted) || r->count <= 1;
	bn->trevsorted = n <= 1 || (l->tsorted && r->trevsorted) || (l->trevsorted && r->tsorted) || r->count <= 1;
	bn->tkey = n <= 1 || (l->tkey && r->tkey);
	return bn;
}
