// project.hip -- BATproject on the MI355X (gdk/gdk_project.c:590-857).
//
// out[i] = r[l[i] - r.hseqbase].  A dense l that lies inside r is a
// zero-copy slice view (BATslice, gdk_project.c:623-645); otherwise a
// gather kernel reads the oid list with 16-byte loads (two oids per lane)
// and gathers the values (1/2/4/8/16 B).  A nil oid gives nil, an oid
// outside r is the reference's "does not match always" error.  str columns
// gather their heap offsets and share the string heap (the "stringtrick",
// gdk_project.c:681-718).
#include <type_traits>
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

// each wave streams 64 * U consecutive oids per step (element = chunk base
// + u * 64 + lane): U oid loads in flight, then U independent gathers
template <typename T>
__global__ __launch_bounds__(256) void
k_project(const oid *__restrict__ l, BUN n, const T *__restrict__ r, oid rseq, BUN rcnt, T nilv,
	  T *__restrict__ out, uint32_t *__restrict__ flags)
{
	constexpr int U = 16;
	constexpr BUN CH = 64 * U;
	uint32_t bad = 0, nil = 0;
	const unsigned lane = __lane_id();
	const BUN nwaves = (BUN) gridDim.x * (blockDim.x / 64);
	for (BUN ch = (BUN) blockIdx.x * (blockDim.x / 64) + (threadIdx.x / 64); ch * CH < n; ch += nwaves) {
		const BUN i0 = ch * CH + lane;
		oid o[U];
		// unconditional loads at clamped indices, masked afterwards (a load
		// under a divergent branch is waited for before the branch joins)
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * 64;
			o[u] = l[i < n ? i : n - 1];
		}
		T v[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const bool isnil = o[u] == MGDK_OID_NIL, out_of = !isnil && o[u] - rseq >= rcnt;
			const BUN p = (isnil || out_of) ? 0 : o[u] - rseq;
			v[u] = r[p];     // r has >= 1 readable element (the host passes a dummy for empty r)
			if (isnil || out_of)
				v[u] = nilv;
			nil |= isnil;
			bad |= out_of;
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN i = i0 + (BUN) u * 64;
			if (i < n)
				out[i] = v[u];
		}
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
	if (rcnt == 0)
		r = meta_buf();   // every non-nil oid is out of range; the gather still reads r[0]
	unsigned g = grid_for(n, 256 * 8, 256 * 16);
	hipLaunchKernelGGL((k_project<T>), dim3(g), dim3(256), 0, stream(), l, n, (const T *) r, rseq, rcnt,
			   nilv, (T *) out, flags);
}

// l carries its select scan's bitmap (Priv::smap): one workgroup per scan
// tile streams the projected column over the tile's candidate slots in row
// order (row = slot base + u * 256 + lane: every load covers 256 consecutive
// values), and each hit goes to the tile's hit prefix + its rank among the
// tile's set bits (LDS prefix of the word popcounts).  Reads the column once
// plus n/8 bytes of bitmap instead of 8-byte oids and a gather.
constexpr uint32_t PB_MAXW = 512;     // bitmap words per tile at most (select's sel_wpt)

// the tile's bitmap words in LDS with their exclusive popcount prefix
// (thread tid owns words tid and tid + 256)
__device__ __forceinline__ void
pb_prefix(const uint32_t *__restrict__ bits, uint64_t t, uint32_t wpt, uint32_t *s_w, uint32_t *s_pre,
	  uint32_t *s_wave)
{
	const unsigned tid = threadIdx.x, lane = __lane_id(), wave = tid >> 6;
	uint32_t w0 = 0, w1 = 0;
	if (tid < wpt)
		w0 = bits[t * wpt + tid];
	if (tid + 256 < wpt)
		w1 = bits[t * wpt + tid + 256];
	const uint32_t c0 = __popc(w0), c1 = __popc(w1);
	uint32_t x = c0;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t y = __shfl_up(x, o);
		if ((int) lane >= o)
			x += y;
	}
	if (lane == 63)
		s_wave[wave] = x;
	__syncthreads();
	uint32_t ex = x - c0, tot0 = 0;
	for (unsigned q = 0; q < 4; q++) {
		ex += q < wave ? s_wave[q] : 0;
		tot0 += s_wave[q];
	}
	__syncthreads();
	uint32_t x1 = c1;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t y = __shfl_up(x1, o);
		if ((int) lane >= o)
			x1 += y;
	}
	if (lane == 63)
		s_wave[wave] = x1;
	__syncthreads();
	uint32_t ex1 = tot0 + x1 - c1;
	for (unsigned q = 0; q < wave; q++)
		ex1 += s_wave[q];
	if (tid < wpt) {
		s_w[tid] = w0;
		s_pre[tid] = ex;
	}
	if (tid + 256 < wpt) {
		s_w[tid + 256] = w1;
		s_pre[tid + 256] = ex1;
	}
	__syncthreads();
}

template <typename T>
__global__ __launch_bounds__(256) void
k_project_bits(const uint32_t *__restrict__ bits, const uint64_t *__restrict__ pre, uint32_t wpt, uint64_t nslots,
	       int64_t rowbase, BUN rcnt, const T *__restrict__ r, T *__restrict__ out)
{
	__shared__ uint32_t s_w[PB_MAXW], s_pre[PB_MAXW];
	__shared__ uint32_t s_wave[4];
	const unsigned tid = threadIdx.x;
	const uint64_t t = blockIdx.x;
	pb_prefix(bits, t, wpt, s_w, s_pre, s_wave);
	const uint64_t obase = pre[t];
	const uint64_t s0 = t * (uint64_t) wpt * 32;
	const uint32_t tslots = wpt * 32;
	constexpr int U = 16;
	for (uint32_t r0 = 0; r0 < tslots; r0 += 256 * U) {
		T v[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint64_t j = s0 + r0 + (uint32_t) u * 256 + tid;
			int64_t row = rowbase + (int64_t) j;
			row = row < 0 ? 0 : row >= (int64_t) rcnt ? (int64_t) rcnt - 1 : row;   // clamped, masked below
			v[u] = r[row];
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t sl = r0 + (uint32_t) u * 256 + tid;
			if (sl >= tslots || s0 + sl >= nslots)
				continue;
			const uint32_t wv = s_w[sl >> 5], bit = sl & 31;
			if ((wv >> bit) & 1)
				out[obase + s_pre[sl >> 5] + __popc(wv & ((1u << bit) - 1))] = v[u];
		}
	}
}

// vector form (1/2/4/8-byte values, the tile's first row a multiple of
// V = 16 / sizeof(T)): a lane loads V consecutive values with one 16-byte
// nontemporal load, so each wave load instruction covers 1 KiB of the
// column; the chunk's hits are compacted into LDS at their rank and stored
// from there by consecutive lanes (per-lane runs of V values written
// straight to HBM are partial lines: 2x slower).  Rows past the last whole
// vector of r (< V of them, last tile only) are read by single loads after
// the main loop.
template <typename T>
__global__ __launch_bounds__(256) void
k_project_bits_v(const uint32_t *__restrict__ bits, const uint64_t *__restrict__ pre, uint32_t wpt,
		 uint64_t nslots, int64_t rowbase, BUN rcnt, const T *__restrict__ r, T *__restrict__ out,
		 const void *zero)
{
	constexpr int V = 16 / sizeof(T), U = 8;
	constexpr uint32_t CH = 256 * V * U;                 // slots per chunk
	typedef uint32_t vec_t __attribute__((ext_vector_type(4)));
	__shared__ uint32_t s_w[PB_MAXW], s_pre[PB_MAXW];
	__shared__ uint32_t s_wave[4];
	__shared__ T stage[CH];
	const unsigned tid = threadIdx.x;
	const uint64_t t = blockIdx.x;
	pb_prefix(bits, t, wpt, s_w, s_pre, s_wave);
	const uint64_t obase = pre[t];
	const uint64_t s0 = t * (uint64_t) wpt * 32;
	const uint32_t tslots = wpt * 32;
	const int64_t nvec = (int64_t) (rcnt / V);           // whole vectors of r
	const vec_t *rv = (const vec_t *) r;
	// lanes without a hit in their V slots load from the zero region: a
	// column line is fetched only when it holds a hit (sparse lists)
	const vec_t *z = (const vec_t *) zero + (((uint64_t) t * 256 + tid) & (ZERO_REGION / 16 - 1));
	for (uint32_t r0 = 0; r0 < tslots; r0 += CH) {
		vec_t v[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t sl = r0 + ((uint32_t) u * 256 + tid) * V;
			int64_t vi = (rowbase + (int64_t) (s0 + sl)) / V;
			vi = vi < 0 ? 0 : vi >= nvec ? nvec - 1 : vi;      // clamped, masked below
			const uint32_t hit = sl < tslots ? (s_w[sl >> 5] >> (sl & 31)) & ((1u << V) - 1) : 0u;
			v[u] = __builtin_nontemporal_load(hit ? rv + vi : z);
		}
		// the chunk's hits are the output range [c0, c1) of the tile
		const uint32_t c0 = s_pre[r0 >> 5];
		const uint32_t re = min(r0 + CH, tslots);
		const uint32_t c1 = re < tslots ? s_pre[re >> 5] : s_pre[(tslots >> 5) - 1] + __popc(s_w[(tslots >> 5) - 1]);
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t sl = r0 + ((uint32_t) u * 256 + tid) * V;
			if (sl >= tslots)
				continue;
			const int64_t row0 = rowbase + (int64_t) (s0 + sl);
			const uint32_t wv = s_w[sl >> 5], b0 = sl & 31;
			uint32_t msk = (wv >> b0) & ((1u << V) - 1);
			// slots past nslots or rows past the whole vectors are not here
			const int64_t lim = min((int64_t) (nslots - (s0 + sl)), nvec * V - row0);
			if (lim < V)
				msk &= lim <= 0 ? 0u : ((1u << lim) - 1);
			uint32_t o = s_pre[sl >> 5] + __popc(wv & ((1u << b0) - 1)) - c0;
			T e[V];
			__builtin_memcpy(e, &v[u], 16);
#pragma unroll
			for (int q = 0; q < V; q++)
				if ((msk >> q) & 1)
					stage[o++] = e[q];
		}
		__syncthreads();
		// the hits the lane masks dropped (past nslots / the whole vectors)
		// leave their stage places unwritten; those places are not stored
		const uint32_t nst = c1 - c0;
		uint32_t valid = nst;
		{
			const int64_t lastrow = nvec * V - 1 - rowbase - (int64_t) s0;   // last slot with a whole-vector row
			const int64_t lastsl = min(lastrow, (int64_t) (nslots - s0) - 1);
			if (lastsl < (int64_t) re - 1) {
				if (lastsl < (int64_t) r0)
					valid = 0;
				else {
					const uint32_t ls = (uint32_t) lastsl, wv = s_w[ls >> 5], bit = ls & 31;
					valid = s_pre[ls >> 5] + __popc(wv & (bit == 31 ? ~0u : ((2u << bit) - 1))) - c0;
				}
			}
		}
		T *dst = out + obase + c0;
		if constexpr (sizeof(T) < 4) {
			// 1- and 2-byte values leave as 4-byte words (a store per value
			// wrote 64 B per wave instruction): the unaligned head and the
			// tail by single stores, every word wholly inside this chunk's
			// output range
			constexpr uint32_t E = 4 / sizeof(T);
			typedef typename std::conditional<sizeof(T) == 1, uint8_t, uint16_t>::type U;
			const uint32_t mis = (uint32_t) (((uintptr_t) dst & 3) / sizeof(T));
			const uint32_t head = mis ? min(valid, E - mis) : 0u;
			if (tid < head)
				dst[tid] = stage[tid];
			const uint32_t nw = (valid - head) / E;
			uint32_t *dw = (uint32_t *) (dst + head);
			for (uint32_t j = tid; j < nw; j += 256) {
				uint32_t wv = 0;
#pragma unroll
				for (uint32_t e = 0; e < E; e++)
					wv |= (uint32_t) (U) stage[head + j * E + e] << (8 * sizeof(T) * e);
				dw[j] = wv;
			}
			const uint32_t done = head + nw * E;
			if (tid < valid - done)
				dst[done + tid] = stage[done + tid];
		} else {
			for (uint32_t j = tid; j < valid; j += 256)
				dst[j] = stage[j];
		}
		__syncthreads();
	}
	// rows of r after its last whole vector
	const int64_t tail0 = nvec * V;
	if (tail0 < (int64_t) rcnt && tid < V) {
		const int64_t row = tail0 + tid;
		const int64_t sl64 = row - rowbase - (int64_t) s0;
		if (row < (int64_t) rcnt && sl64 >= 0 && sl64 < (int64_t) tslots && s0 + (uint64_t) sl64 < nslots) {
			const uint32_t sl = (uint32_t) sl64, wv = s_w[sl >> 5], bit = sl & 31;
			if ((wv >> bit) & 1)
				out[obase + s_pre[sl >> 5] + __popc(wv & ((1u << bit) - 1))] = r[row];
		}
	}
}

template <typename T>
static void
launch_bits(const SelMap &m, const mgdk_bat *r, void *out)
{
	const int64_t rowbase = m.base - (int64_t) r->hseqbase;
	constexpr int V = 16 / sizeof(T);
	const void *zero = zero_region();
	if (V > 1 && zero && rowbase % V == 0 && ((uintptr_t) r->theap & 15) == 0 && r->count >= (BUN) V)
		hipLaunchKernelGGL((k_project_bits_v<T>), dim3((unsigned) m.ntiles), dim3(256), 0, stream(), m.bits,
				   m.pre, m.wpt, m.nslots, rowbase, r->count, (const T *) r->theap, (T *) out, zero);
	else
		hipLaunchKernelGGL((k_project_bits<T>), dim3((unsigned) m.ntiles), dim3(256), 0, stream(), m.bits,
				   m.pre, m.wpt, m.nslots, rowbase, r->count, (const T *) r->theap, (T *) out);
}


// ---- BATproject2 / BATprojectchain (gdk/gdk_project.c:590, :879) --------
//
// One fused gather: every output row follows its oid through the chain of
// oid columns (no intermediate is materialised) and then reads the value
// from the last column -- or, for BATproject2, from whichever of r1 / r2
// (r2 following r1 in head oids) holds it.

constexpr int CHAIN_MAX = 8;

struct ColRef {
	const void *t;       // NULL: dense (void) column, value = tseq + (o - hlo)
	oid hlo;
	BUN cnt;
	oid tseq;
};

struct Chain {
	ColRef l0;           // the first (oid) column, read by position
	ColRef lv[CHAIN_MAX];
	int nl;              // intermediate oid columns
	ColRef f[2];         // final value column(s)
	int nf;
};

template <typename T>
__device__ __forceinline__ T
colval(const ColRef &c, oid off)
{
	if (c.t == nullptr)
		return (T) (c.tseq == MGDK_OID_NIL ? MGDK_OID_NIL : c.tseq + off);
	return ((const T *) c.t)[off];
}

template <typename T>
__global__ __launch_bounds__(256) void
k_project_chain(Chain c, BUN n, T nilv, T *out, uint32_t *flags)
{
	uint32_t bad = 0, nil = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		oid o = colval<oid>(c.l0, i);
		bool isnil = false;
		for (int k = 0; k < c.nl && !isnil; k++) {
			if (o == MGDK_OID_NIL) {
				isnil = true;
				break;
			}
			if (o < c.lv[k].hlo || o - c.lv[k].hlo >= c.lv[k].cnt) {
				bad = 1;
				isnil = true;
				break;
			}
			o = colval<oid>(c.lv[k], o - c.lv[k].hlo);
		}
		T v = nilv;
		if (!isnil && o == MGDK_OID_NIL)
			isnil = true;
		if (!isnil) {
			if (o >= c.f[0].hlo && o - c.f[0].hlo < c.f[0].cnt)
				v = colval<T>(c.f[0], o - c.f[0].hlo);
			else if (c.nf > 1 && o >= c.f[1].hlo && o - c.f[1].hlo < c.f[1].cnt)
				v = colval<T>(c.f[1], o - c.f[1].hlo);
			else
				bad = 1;
		}
		nil |= isnil;
		out[i] = v;
	}
	bad = block_reduce(bad, [](uint32_t x, uint32_t y) { return x | y; });
	nil = block_reduce(nil, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0) {
		publish_or(&flags[0], bad);
		publish_or(&flags[1], nil);
	}
}

ColRef
colref(const mgdk_bat *b)
{
	ColRef c;
	c.t = b->ttype == MGDK_void ? nullptr : b->theap;
	c.hlo = b->hseqbase;
	c.cnt = b->count;
	c.tseq = b->tseqbase;
	return c;
}

// run the fused gather; the value type comes from fin[0]
mgdk_bat *
run_chain(Chain &c, BUN n, oid hseq, const mgdk_bat *fin0, const mgdk_bat *fin1, bool *nil_seen)
{
	const int rt = fin0->ttype;
	const int ot = rt == MGDK_void ? MGDK_oid : rt;
	const int w = rt == MGDK_void ? 8 : fin0->twidth;
	if (fin1 && ((fin1->ttype == MGDK_void ? 8 : fin1->twidth) != w ||
		     (rt == MGDK_str && fin1->tvheap != fin0->tvheap) ||
		     (basetype(fin1->ttype == MGDK_void ? MGDK_oid : fin1->ttype) != basetype(ot)))) {
		seterr("42000!BATproject2: r1 and r2 must have the same type (and, for str, share their heap) on the "
		       "device path");
		return nullptr;
	}
	const int alloc_t = rt != MGDK_str ? ot : w == 1 ? MGDK_bte : w == 2 ? MGDK_sht : w == 4 ? MGDK_int : MGDK_lng;
	mgdk_bat *bn = newbat(hseq, alloc_t, n);
	if (bn == nullptr)
		return nullptr;
	if (rt == MGDK_str) {
		bn->ttype = MGDK_str;
		share_vheap(bn, fin0);
	}
	uint32_t *flags = (uint32_t *) meta_buf();
	if (!hip_ok(hipMemsetAsync(flags, 0, 16, stream()), "memset")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const dim3 g(grid_for(n, 1024, 256 * 16)), blk(256);
	hipStream_t st = stream();
	alignas(16) unsigned char nilv[16] = {0};
	const int bt = rt == MGDK_str ? -w : basetype(ot);
	switch (bt) {
	case MGDK_bte: *(int8_t *) nilv = INT8_MIN; hipLaunchKernelGGL((k_project_chain<int8_t>), g, blk, 0, st, c, n, *(int8_t *) nilv, (int8_t *) bn->theap, flags); break;
	case MGDK_sht: *(int16_t *) nilv = INT16_MIN; hipLaunchKernelGGL((k_project_chain<int16_t>), g, blk, 0, st, c, n, *(int16_t *) nilv, (int16_t *) bn->theap, flags); break;
	case MGDK_int: *(int32_t *) nilv = INT32_MIN; hipLaunchKernelGGL((k_project_chain<int32_t>), g, blk, 0, st, c, n, *(int32_t *) nilv, (int32_t *) bn->theap, flags); break;
	case MGDK_flt: { const float f = __builtin_nanf(""); uint32_t u; memcpy(&u, &f, 4); hipLaunchKernelGGL((k_project_chain<uint32_t>), g, blk, 0, st, c, n, u, (uint32_t *) bn->theap, flags); break; }
	case MGDK_lng: hipLaunchKernelGGL((k_project_chain<int64_t>), g, blk, 0, st, c, n, (int64_t) INT64_MIN, (int64_t *) bn->theap, flags); break;
	case MGDK_oid: hipLaunchKernelGGL((k_project_chain<uint64_t>), g, blk, 0, st, c, n, (uint64_t) MGDK_OID_NIL, (uint64_t *) bn->theap, flags); break;
	case MGDK_dbl: { const double d = __builtin_nan(""); uint64_t u; memcpy(&u, &d, 8); hipLaunchKernelGGL((k_project_chain<uint64_t>), g, blk, 0, st, c, n, u, (uint64_t *) bn->theap, flags); break; }
	case MGDK_hge: hipLaunchKernelGGL((k_project_chain<hge>), g, blk, 0, st, c, n, NilOf<hge>::v(), (hge *) bn->theap, flags); break;
	case -1: hipLaunchKernelGGL((k_project_chain<uint8_t>), g, blk, 0, st, c, n, (uint8_t) 0, (uint8_t *) bn->theap, flags); break;
	case -2: hipLaunchKernelGGL((k_project_chain<uint16_t>), g, blk, 0, st, c, n, (uint16_t) 0, (uint16_t *) bn->theap, flags); break;
	case -4: hipLaunchKernelGGL((k_project_chain<uint32_t>), g, blk, 0, st, c, n, (uint32_t) 0, (uint32_t *) bn->theap, flags); break;
	case -8: hipLaunchKernelGGL((k_project_chain<uint64_t>), g, blk, 0, st, c, n, (uint64_t) 0, (uint64_t *) bn->theap, flags); break;
	default:
		seterr("42000!BATproject: type %s not supported on the device path", atomname(rt));
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	uint32_t *h = (uint32_t *) pinned(16);
	if (h == nullptr || !hip_ok(hipMemcpyAsync(h, flags, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
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
	*nil_seen = h[1] != 0;
	return bn;
}

// l as a ColRef (complex candidate lists materialised into *tmp)
int
left_ref(mgdk_bat *l, ColRef &c, mgdk_bat **tmp)
{
	*tmp = nullptr;
	if (is_complex_cand(l)) {
		mgdk_bat *m = unmask_cand(l);
		if (m == nullptr)
			return -1;
		*tmp = m;
		c = colref(m);
		c.hlo = l->hseqbase;
		return 0;
	}
	c = colref(l);
	return 0;
}

}  // namespace

extern "C" mgdk_bat *
mgdk_BATproject(mgdk_bat *l, mgdk_bat *r)
{
	if (l == nullptr || r == nullptr) {
		seterr("BATproject: NULL argument");
		return nullptr;
	}
	if (l->ttype != MGDK_void && l->ttype != MGDK_oid && l->ttype != MGDK_msk) {
		seterr("BATproject: left must be oid");
		return nullptr;
	}
	if (is_complex_cand(l)) {
		// candidate list with exceptions, a bitmask, or a msk BAT
		// (gdk_project.c:645-660: BATunmask)
		mgdk_bat *m = unmask_cand(l);
		if (m == nullptr)
			return nullptr;
		m->hseqbase = l->hseqbase;
		mgdk_bat *bn = mgdk_BATproject(m, r);
		mgdk_BBPunfix(m);
		return bn;
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
	SelMap sm;
	// a select result with its bitmap, all of whose oids lie in r (no nil,
	// no "does not match"): stream r in row order
	const bool bits = rt != MGDK_void && smap_get(l, &sm) && sm.wpt <= PB_MAXW && sm.lo >= r->hseqbase &&
			  sm.hi - r->hseqbase < r->count && r->count > 0;
	if (bits) {
		switch (rt == MGDK_str ? r->twidth : width_of(rt)) {
		case 1: launch_bits<uint8_t>(sm, r, bn->theap); break;
		case 2: launch_bits<uint16_t>(sm, r, bn->theap); break;
		case 4: launch_bits<uint32_t>(sm, r, bn->theap); break;
		case 8: launch_bits<uint64_t>(sm, r, bn->theap); break;
		default: launch_bits<hge>(sm, r, bn->theap); break;
		}
	} else if (rt == MGDK_void) {
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
extern "C" mgdk_bat *
mgdk_BATproject2(mgdk_bat *l, mgdk_bat *r1, mgdk_bat *r2)
{
	if (l == nullptr || r1 == nullptr) {
		seterr("BATproject2: NULL argument");
		return nullptr;
	}
	if (r2 == nullptr)
		return mgdk_BATproject(l, r1);
	if (r1->hseqbase + r1->count != r2->hseqbase) {
		seterr("BATproject2: r2 must follow r1");
		return nullptr;
	}
	if (r1->count == 0)        // gdk_project.c:613-620
		return mgdk_BATproject(l, r2);
	if (l->ttype == MGDK_void && !is_complex_cand(l) && l->count > 0 && l->tseqbase != MGDK_OID_NIL) {
		// dense l: a slice of r1 or r2 when it lies inside one of them (:622-645)
		const oid lo = l->tseqbase, hi = l->tseqbase + l->count;
		if ((lo >= r1->hseqbase && hi <= r1->hseqbase + r1->count) || lo >= r2->hseqbase)
			return mgdk_BATproject(l, lo >= r2->hseqbase ? r2 : r1);
		if (lo < r1->hseqbase || hi > r2->hseqbase + r2->count) {
			seterr("does not match always\n");
			return nullptr;
		}
	}
	if (l->ttype != MGDK_void && l->ttype != MGDK_oid && l->ttype != MGDK_msk) {
		seterr("BATproject2: left must be oid");
		return nullptr;
	}
	ProfScope prof("project2");
	Chain c{};
	mgdk_bat *tmp;
	if (left_ref(l, c.l0, &tmp) < 0)
		return nullptr;
	const BUN n = tmp ? tmp->count : l->count;
	c.nl = 0;
	c.f[0] = colref(r1);
	c.f[1] = colref(r2);
	c.nf = 2;
	bool nils = false;
	mgdk_bat *bn = run_chain(c, n, l->hseqbase, r1, r2, &nils);
	mgdk_BBPunfix(tmp);
	if (bn) {
		bn->tnonil = !nils && l->tnonil && r1->tnonil && r2->tnonil;
		bn->tsorted = bn->trevsorted = bn->tkey = n <= 1;
	}
	return bn;
}

// BATprojectchain (gdk_project.c:879-1164): bats is NULL-terminated
extern "C" mgdk_bat *
mgdk_BATprojectchain(mgdk_bat **bats)
{
	int n = 0;
	while (bats && bats[n])
		n++;
	if (n == 0) {
		seterr("must have BAT arguments\n");
		return nullptr;
	}
	mgdk_bat *b = bats[n - 1];
	if (n == 1)
		return mgdk_BATslice(b, 0, b->count);
	// drop identity steps (dense, hseqbase == tseqbase == next hseqbase, same count)
	mgdk_bat *keep[64];
	int k = 0;
	for (int i = 0; i < n; i++) {
		mgdk_bat *x = bats[i];
		if (i + 1 < n && x->ttype == MGDK_void && !is_complex_cand(x) && x->tseqbase != MGDK_OID_NIL &&
		    x->hseqbase == x->tseqbase && x->tseqbase == bats[i + 1]->hseqbase && x->count == bats[i + 1]->count)
			continue;
		if (k == 64 || k - 1 > CHAIN_MAX) {
			seterr("42000!BATprojectchain: chains longer than %d not supported on the device path", CHAIN_MAX + 2);
			return nullptr;
		}
		keep[k++] = x;
	}
	if (k == 1)
		return mgdk_BATslice(keep[0], 0, keep[0]->count);
	if (k == 2)
		return mgdk_BATproject(keep[0], keep[1]);
	bool allnil = false, issorted = true, nonil = true;
	for (int i = 0; i < k; i++) {
		allnil |= keep[i]->ttype == MGDK_void && !is_complex_cand(keep[i]) && keep[i]->tseqbase == MGDK_OID_NIL;
		issorted &= keep[i]->tsorted != 0;
		if (i + 1 < k)
			nonil &= keep[i]->tnonil != 0;
	}
	ProfScope prof("projectchain");
	Chain c{};
	mgdk_bat *tmp[CHAIN_MAX + 1] = {nullptr};
	int ntmp = 0;
	auto cleanup = [&]() {
		for (int i = 0; i < ntmp; i++)
			mgdk_BBPunfix(tmp[i]);
	};
	if (left_ref(keep[0], c.l0, &tmp[ntmp]) < 0)
		return nullptr;
	const BUN cnt = tmp[ntmp] ? tmp[ntmp]->count : keep[0]->count;
	ntmp += tmp[ntmp] != nullptr;
	if (allnil || cnt == 0) {
		cleanup();
		alignas(16) unsigned char nilv[16] = {0};
		const int rt = b->ttype;
		switch (basetype(rt)) {
		case MGDK_bte: *(int8_t *) nilv = INT8_MIN; break;
		case MGDK_sht: *(int16_t *) nilv = INT16_MIN; break;
		case MGDK_int: *(int32_t *) nilv = INT32_MIN; break;
		case MGDK_lng: *(int64_t *) nilv = INT64_MIN; break;
		case MGDK_oid: case MGDK_void: *(uint64_t *) nilv = MGDK_OID_NIL; break;
		case MGDK_hge: nilv[15] = 0x80; break;
		case MGDK_flt: { const float f = __builtin_nanf(""); memcpy(nilv, &f, 4); break; }
		case MGDK_dbl: { const double d = __builtin_nan(""); memcpy(nilv, &d, 8); break; }
		default:
			seterr("42000!BATprojectchain: nil projection of %s unsupported", atomname(rt));
			return nullptr;
		}
		return mgdk_BATconstant(keep[0]->hseqbase, rt == MGDK_oid ? MGDK_void : rt, nilv, cnt);
	}
	c.nl = 0;
	for (int i = 1; i + 1 < k; i++) {
		if (keep[i]->ttype != MGDK_void && keep[i]->ttype != MGDK_oid && keep[i]->ttype != MGDK_msk) {
			cleanup();
			seterr("BATprojectchain: all but the last BAT must be oid");
			return nullptr;
		}
		if (left_ref(keep[i], c.lv[c.nl], &tmp[ntmp]) < 0) {
			cleanup();
			return nullptr;
		}
		if (tmp[ntmp]) {
			c.lv[c.nl].cnt = tmp[ntmp]->count;
			ntmp++;
		}
		c.nl++;
	}
	c.f[0] = colref(b);
	c.nf = 1;
	bool nils = false;
	mgdk_bat *bn = run_chain(c, cnt, keep[0]->hseqbase, b, nullptr, &nils);
	cleanup();
	if (bn) {
		// gdk_project.c:1141-1146
		bn->tsorted = cnt <= 1 || issorted;
		bn->trevsorted = cnt <= 1;
		bn->tnonil = nonil && b->tnonil && !nils;
		bn->tkey = cnt <= 1;
	}
	return bn;
}
