// dict.hip -- dictionary- and frame-of-reference-compressed column inputs on
// the MI355X (sql/backends/monet5/dict.c, for.c).
//
// A DICT column is a code column o (bte / sht / int, read UNSIGNED as an
// index) plus a dictionary BAT u of the distinct values (dict.c:110-226);
// a FOR column is a bte / sht offset column plus one minimum (for.c:119).
// Selections run on the codes: the predicate is evaluated once on the
// (small) dictionary with the GDK select semantics of the value type --
// exactly dict.c's general path BATselect(lv, ...) (:1006, :898) -- giving
// a code -> qualifies map; every candidate row then costs one 1- or 2-byte
// code read and a map lookup, and the qualifying rows are compacted in
// order.  That is the semijoin the reference computes with BATintersect,
// and on sorted dictionaries the same rows as its code-range fast path.
// Decompression is a gather through the dictionary (dict.c:352-445) or an
// add of the minimum (for.c:30-80).
#include <climits>
#include <cstring>
#include <type_traits>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

template <typename C>
__device__ __forceinline__ uint32_t
code_at(const void *o, BUN i)
{
	typedef typename std::conditional<sizeof(C) == 1, uint8_t,
					  typename std::conditional<sizeof(C) == 2, uint16_t, uint32_t>::type>::type U;
	return ((const U *) o)[i];
}

template <typename C, typename V>
__global__ __launch_bounds__(256) void
k_dict_decompress(const void *o, BUN n, const V *u, BUN nu, V nil, V *out, uint32_t *bad)
{
	uint32_t b = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint32_t c = code_at<C>(o, i);
		if (c < nu) {
			out[i] = u[c];
		} else {
			out[i] = nil;
			b = 1;
		}
	}
	b = block_reduce(b, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(bad, b);
}

// flags of the candidates whose code qualifies
template <typename C>
__global__ __launch_bounds__(256) void
k_dict_flags(const void *o, Cand ci, oid hseq, const uint8_t *map, BUN nmap, int8_t *flags)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < ci.n; i += (BUN) gridDim.x * blockDim.x) {
		const oid p = (ci.dense ? ci.seq + i : ci.oids[i]) - hseq;
		const uint32_t c = code_at<C>(o, p);
		flags[i] = c < nmap && map[c];
	}
}

__global__ __launch_bounds__(256) void
k_map_from_oids(const oid *sel, oid seq, BUN n, oid base, uint8_t *map)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		map[(sel ? sel[i] : seq + i) - base] = 1;
}

template <typename T, typename O>
__global__ __launch_bounds__(256) void
k_for_decompress(const T *o, BUN n, int64_t minval, O *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = (O) (minval + (int64_t) o[i]);
}

template <typename T>
__global__ __launch_bounds__(256) void
k_for_compress(const int64_t *b, BUN n, int64_t minval, T *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = (T) (b[i] - minval);
}

__global__ __launch_bounds__(256) void
k_minmax_lng(const int64_t *b, BUN n, unsigned long long *mm, uint32_t *nil)
{
	long long mn = LLONG_MAX, mx = LLONG_MIN + 1;
	uint32_t hasnil = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const int64_t v = b[i];
		if (v == INT64_MIN) {
			hasnil = 1;
			continue;
		}
		mn = v < mn ? v : mn;
		mx = v > mx ? v : mx;
	}
	mn = block_reduce(mn, [](long long x, long long y) { return x < y ? x : y; });
	mx = block_reduce(mx, [](long long x, long long y) { return x > y ? x : y; });
	hasnil = block_reduce(hasnil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0) {
		atomicMin((long long *) &mm[0], mn);
		atomicMax((long long *) &mm[1], mx);
		publish_or(nil, hasnil);
	}
}

template <typename C>
__global__ __launch_bounds__(256) void
k_codes_from_oids(const oid *r2, oid seq, BUN n, C *out)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = (C) (r2 ? r2[i] : seq + i);
}

bool
code_type(int t)
{
	return t == MGDK_bte || t == MGDK_sht || t == MGDK_int;
}

// the qualifying codes of a selection on the dictionary -> candidate list
mgdk_bat *
dict_select_codes(mgdk_bat *lo, mgdk_bat *lc, mgdk_bat *lv, mgdk_bat *sel)
{
	hipStream_t st = stream();
	const BUN nu = lv->count;
	Cand ci;
	if (cand_init(&ci, lo, lc) < 0)
		return nullptr;
	DevBuf map(nu + 8), fl(ci.n + 8);
	if (!map.p || !fl.p || !hip_ok(hipMemsetAsync(map.p, 0, nu + 8, st), "memset"))
		return nullptr;
	if (sel->count)
		hipLaunchKernelGGL(k_map_from_oids, dim3(grid_for(sel->count, 1024, 4096)), dim3(256), 0, st,
				   sel->ttype == MGDK_void ? nullptr : (const oid *) sel->theap, sel->tseqbase, sel->count,
				   lv->hseqbase, map.as<uint8_t>());
	if (ci.n) {
		const dim3 g(grid_for(ci.n, 2048, 8192)), blk(256);
		switch (lo->twidth) {
		case 1: hipLaunchKernelGGL((k_dict_flags<int8_t>), g, blk, 0, st, lo->theap, ci, lo->hseqbase, map.as<uint8_t>(), nu, fl.as<int8_t>()); break;
		case 2: hipLaunchKernelGGL((k_dict_flags<int16_t>), g, blk, 0, st, lo->theap, ci, lo->hseqbase, map.as<uint8_t>(), nu, fl.as<int8_t>()); break;
		default: hipLaunchKernelGGL((k_dict_flags<int32_t>), g, blk, 0, st, lo->theap, ci, lo->hseqbase, map.as<uint8_t>(), nu, fl.as<int8_t>()); break;
		}
	}
	if (ci.dense)
		return compact_flags(fl.as<int8_t>(), ci.n, ci.seq);
	mgdk_bat *pos = compact_flags(fl.as<int8_t>(), ci.n, lc->hseqbase);
	if (pos == nullptr)
		return nullptr;
	mgdk_bat *r = mgdk_BATproject(pos, lc);
	mgdk_BBPunfix(pos);
	return r;
}

int
check_dict(mgdk_bat *lo, mgdk_bat *lv)
{
	if (lo == nullptr || lv == nullptr) {
		seterr("dict: NULL argument");
		return -1;
	}
	if (!code_type(lo->ttype)) {
		seterr("dict: codes must be bte, sht or int (got %s)", atomname(lo->ttype));
		return -1;
	}
	return 0;
}

}  // namespace

// dict.c:352 DICTdecompress_: b[i] = u[(unsigned) o[i]]
extern "C" mgdk_bat *
mgdk_DICTdecompress(mgdk_bat *o, mgdk_bat *u)
{
	if (check_dict(o, u) < 0)
		return nullptr;
	const int w = u->twidth;
	if (u->ttype == MGDK_void || u->ttype == MGDK_str || !(w == 1 || w == 2 || w == 4 || w == 8 || w == 16)) {
		seterr("42000!DICTdecompress: dictionary type %s not supported on the device path", atomname(u->ttype));
		return nullptr;
	}
	ProfScope prof("dictdecompress");
	const BUN n = o->count;
	mgdk_bat *b = newbat(o->hseqbase, u->ttype, n);
	DevBuf bad(16);
	if (b == nullptr || !bad.p || !hip_ok(hipMemsetAsync(bad.p, 0, 16, stream()), "memset")) {
		mgdk_BBPunfix(b);
		return nullptr;
	}
	if (n) {
		const dim3 g(grid_for(n, 2048, 8192)), blk(256);
		hipStream_t st = stream();
#define DEC(C, V, NILV) hipLaunchKernelGGL((k_dict_decompress<C, V>), g, blk, 0, st, o->theap, n, (const V *) u->theap, \
					   u->count, (V) (NILV), (V *) b->theap, bad.as<uint32_t>())
#define DECW(C) switch (w) { \
		case 1: DEC(C, int8_t, INT8_MIN); break; \
		case 2: DEC(C, int16_t, INT16_MIN); break; \
		case 4: DEC(C, int32_t, INT32_MIN); break; \
		case 8: DEC(C, int64_t, INT64_MIN); break; \
		default: DEC(C, hge, NilOf<hge>::v()); break; }
		switch (o->twidth) {
		case 1: DECW(int8_t); break;
		case 2: DECW(int16_t); break;
		default: DECW(int32_t); break;
		}
#undef DECW
#undef DEC
	}
	uint32_t *h = (uint32_t *) pinned(16);
	if (!h || !hip_ok(hipMemcpyAsync(h, bad.p, 4, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync()) {
		mgdk_BBPunfix(b);
		return nullptr;
	}
	if (h[0]) {
		seterr("DICTdecompress: code out of the dictionary's range");
		mgdk_BBPunfix(b);
		return nullptr;
	}
	b->count = n;
	// BATnegateprops: nothing is known
	b->tsorted = b->trevsorted = b->tkey = n <= 1;
	b->tnonil = 0;
	b->tnil = 0;
	return b;
}

// dict.c:926 DICTselect (after its nil normalisation :965-977)
extern "C" mgdk_bat *
mgdk_DICTselect(mgdk_bat *lo, mgdk_bat *lc, mgdk_bat *lv, const void *l, const void *h, bool li, bool hi, bool anti)
{
	if (check_dict(lo, lv) < 0)
		return nullptr;
	ProfScope prof("dictselect");
	// "here we don't need open ended parts with nil"
	const int w = lv->twidth;
	char lbuf[16], hbuf[16], nilb[16];
	memset(nilb, 0, sizeof(nilb));
	switch (basetype(lv->ttype)) {
	case MGDK_bte: *(int8_t *) nilb = INT8_MIN; break;
	case MGDK_sht: *(int16_t *) nilb = INT16_MIN; break;
	case MGDK_int: *(int32_t *) nilb = INT32_MIN; break;
	case MGDK_lng: *(int64_t *) nilb = INT64_MIN; break;
	case MGDK_oid: *(uint64_t *) nilb = MGDK_OID_NIL; break;
	case MGDK_hge: nilb[15] = (char) 0x80; break;
	case MGDK_flt: { float f = __builtin_nanf(""); memcpy(nilb, &f, 4); break; }
	case MGDK_dbl: { double d = __builtin_nan(""); memcpy(nilb, &d, 8); break; }
	default:
		seterr("42000!DICTselect: dictionary type %s not supported on the device path", atomname(lv->ttype));
		return nullptr;
	}
	auto isnil = [&](const char *v) {
		if (basetype(lv->ttype) == MGDK_flt) { float f; memcpy(&f, v, 4); return f != f; }
		if (basetype(lv->ttype) == MGDK_dbl) { double d; memcpy(&d, v, 8); return d != d; }
		return memcmp(v, nilb, w) == 0;
	};
	memcpy(lbuf, l, w);
	memcpy(hbuf, h ? h : l, w);
	if (!anti) {
		if (li && isnil(lbuf)) {
			memcpy(lbuf, hbuf, w);
			li = false;
		}
		if (hi && isnil(hbuf)) {
			memcpy(hbuf, lbuf, w);
			hi = false;
		}
		if (memcmp(lbuf, hbuf, w) == 0 && isnil(hbuf))
			anti = true;
	}
	mgdk_bat *sel = mgdk_BATselect(lv, nullptr, lbuf, hbuf, li, hi, anti, false);
	if (sel == nullptr)
		return nullptr;
	mgdk_bat *r = dict_select_codes(lo, lc, lv, sel);
	mgdk_BBPunfix(sel);
	return r;
}

// dict.c:788 DICTthetaselect
extern "C" mgdk_bat *
mgdk_DICTthetaselect(mgdk_bat *lo, mgdk_bat *lc, mgdk_bat *lv, const void *v, const char *op)
{
	if (check_dict(lo, lv) < 0)
		return nullptr;
	ProfScope prof("dictselect");
	mgdk_bat *sel = mgdk_BATthetaselect(lv, nullptr, v, op);
	if (sel == nullptr)
		return nullptr;
	mgdk_bat *r = dict_select_codes(lo, lc, lv, sel);
	mgdk_BBPunfix(sel);
	return r;
}

// dict.c:110 DICTcompress_intern: u = the distinct values (first-occurrence
// order, or sorted when `ordered`), o = each row's index in u, as the
// smallest code type that holds |u| (smallest_type) or count(b)
extern "C" int
mgdk_DICTcompress(mgdk_bat **O, mgdk_bat **U, mgdk_bat *b, bool ordered, bool smallest_type)
{
	if (b == nullptr || O == nullptr || U == nullptr) {
		seterr("dict.compress: NULL argument");
		return -1;
	}
	const int bt = basetype(b->ttype);
	if (!(bt == MGDK_bte || bt == MGDK_sht || bt == MGDK_int || bt == MGDK_lng || bt == MGDK_oid)) {
		seterr("42000!DICTcompress: type %s not supported on the device path", atomname(b->ttype));
		return -1;
	}
	mgdk_bat *u = mgdk_BATunique(b, nullptr), *uv = nullptr, *us = nullptr, *r1 = nullptr, *r2 = nullptr,
		 *o = nullptr;
	int rc = -1;
	if (u == nullptr)
		return -1;
	{
		const BUN cnt = u->count;
		if (cnt >= (BUN) INT32_MAX) {
			seterr("3F000!dict compress: too many values");
			goto out;
		}
		int tt = cnt < 256 ? MGDK_bte : cnt < 65536 ? MGDK_sht : MGDK_int;
		if (!smallest_type) {
			const BUN c2 = b->count;
			tt = c2 < 256 ? MGDK_bte : c2 < 65536 ? MGDK_sht : MGDK_int;
		}
		uv = mgdk_BATproject(u, b);
		if (uv == nullptr)
			goto out;
		uv->tkey = 1;
		if (ordered) {
			if (mgdk_BATsort(&us, nullptr, nullptr, uv, nullptr, nullptr, false, false, false) < 0)
				goto out;
			mgdk_BBPunfix(uv);
			uv = us;
			us = nullptr;
			uv->tkey = 1;
		}
		// every row's position in uv: an equi-join where nil meets nil
		// (the reference's HASHloop finds nil too)
		if (mgdk_BATjoin(&r1, &r2, b, uv, nullptr, nullptr, true, 0) < 0)
			goto out;
		if (r1->count != b->count) {
			seterr("dict.compress: lookup lost rows");
			goto out;
		}
		o = newbat(b->hseqbase, tt, b->count);
		if (o == nullptr)
			goto out;
		if (b->count) {
			const dim3 g(grid_for(b->count, 1024, 8192)), blk(256);
			const oid *r2p = r2->ttype == MGDK_void ? nullptr : (const oid *) r2->theap;
			switch (tt) {
			case MGDK_bte: hipLaunchKernelGGL((k_codes_from_oids<int8_t>), g, blk, 0, stream(), r2p, r2->tseqbase, b->count, (int8_t *) o->theap); break;
			case MGDK_sht: hipLaunchKernelGGL((k_codes_from_oids<int16_t>), g, blk, 0, stream(), r2p, r2->tseqbase, b->count, (int16_t *) o->theap); break;
			default: hipLaunchKernelGGL((k_codes_from_oids<int32_t>), g, blk, 0, stream(), r2p, r2->tseqbase, b->count, (int32_t *) o->theap); break;
			}
			if (!sync())
				goto out;
		}
		o->count = b->count;
		o->tsorted = uv->tsorted && b->tsorted;
		o->trevsorted = 0;
		o->tkey = b->tkey;
		o->tnonil = 0;
		o->tnil = 0;
		*O = o;
		*U = uv;
		o = nullptr;
		uv = nullptr;
		rc = 0;
	}
out:
	mgdk_BBPunfix(u);
	mgdk_BBPunfix(uv);
	mgdk_BBPunfix(us);
	mgdk_BBPunfix(r1);
	mgdk_BBPunfix(r2);
	mgdk_BBPunfix(o);
	return rc;
}

// for.c:148 FORcompress_intern (lng columns): offsets from the minimum as
// bte when the spread is < 63, else sht; nils and spreads > 32767 refused
extern "C" mgdk_bat *
mgdk_FORcompress(mgdk_bat *b, int64_t *minval)
{
	if (b == nullptr || minval == nullptr) {
		seterr("for.compress: NULL argument");
		return nullptr;
	}
	if (b->ttype != MGDK_lng) {
		seterr("3F000!for compress: type %s not yet implemented", atomname(b->ttype));
		return nullptr;
	}
	const BUN n = b->count;
	if (n == 0) {
		seterr("42000!for compress: cannot compute range of values on empty columns");
		return nullptr;
	}
	hipStream_t st = stream();
	DevBuf mm(32);
	long long init[2] = {LLONG_MAX, LLONG_MIN + 1};
	if (!mm.p || !hip_ok(hipMemcpyAsync(mm.p, init, 16, hipMemcpyHostToDevice, st), "memcpy") ||
	    !hip_ok(hipMemsetAsync((char *) mm.p + 16, 0, 4, st), "memset"))
		return nullptr;
	hipLaunchKernelGGL(k_minmax_lng, dim3(grid_for(n, 4096, 2048)), dim3(256), 0, st, (const int64_t *) b->theap, n,
			   mm.as<unsigned long long>(), (uint32_t *) ((char *) mm.p + 16));
	long long *h = (long long *) pinned(32);
	if (!h || !hip_ok(hipMemcpyAsync(h, mm.p, 24, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return nullptr;
	if (((uint32_t *) (h + 2))[0]) {
		seterr("3F000!for compress: for 'for' compression column's cannot have NULL's");
		return nullptr;
	}
	const long long mn = h[0], mx = h[1];
	if (mx - mn > INT16_MAX) {
		seterr("3F000!for compress: too large value spread for 'for' compression");
		return nullptr;
	}
	const int tt = (mx - mn) < INT8_MAX / 2 ? MGDK_bte : MGDK_sht;
	mgdk_bat *o = newbat(b->hseqbase, tt, n);
	if (o == nullptr)
		return nullptr;
	const dim3 g(grid_for(n, 1024, 8192)), blk(256);
	if (tt == MGDK_bte)
		hipLaunchKernelGGL((k_for_compress<int8_t>), g, blk, 0, st, (const int64_t *) b->theap, n, (int64_t) mn, (int8_t *) o->theap);
	else
		hipLaunchKernelGGL((k_for_compress<int16_t>), g, blk, 0, st, (const int64_t *) b->theap, n, (int64_t) mn, (int16_t *) o->theap);
	if (!sync()) {
		mgdk_BBPunfix(o);
		return nullptr;
	}
	o->count = n;
	o->tsorted = o->trevsorted = o->tkey = n <= 1;
	o->tnonil = 0;
	o->tnil = 0;
	*minval = mn;
	return o;
}

// for.c:30 FORdecompress_: b[i] = minval + o[i] (type lng or int)
extern "C" mgdk_bat *
mgdk_FORdecompress(mgdk_bat *o, int64_t minval, int tp)
{
	if (o == nullptr || !(o->ttype == MGDK_bte || o->ttype == MGDK_sht) || !(tp == MGDK_lng || tp == MGDK_int)) {
		seterr("for.decompress: offsets must be bte/sht and the type lng or int");
		return nullptr;
	}
	ProfScope prof("fordecompress");
	const BUN n = o->count;
	mgdk_bat *b = newbat(o->hseqbase, tp, n);
	if (b == nullptr)
		return nullptr;
	if (n) {
		const dim3 g(grid_for(n, 2048, 8192)), blk(256);
		hipStream_t st = stream();
		if (o->ttype == MGDK_bte && tp == MGDK_lng)
			hipLaunchKernelGGL((k_for_decompress<int8_t, int64_t>), g, blk, 0, st, (const int8_t *) o->theap, n, minval, (int64_t *) b->theap);
		else if (o->ttype == MGDK_bte)
			hipLaunchKernelGGL((k_for_decompress<int8_t, int32_t>), g, blk, 0, st, (const int8_t *) o->theap, n, minval, (int32_t *) b->theap);
		else if (tp == MGDK_lng)
			hipLaunchKernelGGL((k_for_decompress<int16_t, int64_t>), g, blk, 0, st, (const int16_t *) o->theap, n, minval, (int64_t *) b->theap);
		else
			hipLaunchKernelGGL((k_for_decompress<int16_t, int32_t>), g, blk, 0, st, (const int16_t *) o->theap, n, minval, (int32_t *) b->theap);
		if (!sync()) {
			mgdk_BBPunfix(b);
			return nullptr;
		}
	}
	b->count = n;
	b->tsorted = b->trevsorted = b->tkey = n <= 1;   // BATnegateprops
	b->tnonil = 0;
	b->tnil = 0;
	return b;
}
