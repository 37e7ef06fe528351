// join.hip -- the hash path of BATjoin on the MI355X
// (gdk/gdk_join.c:4451 BATjoin -> :2900 hashjoin, probe loop HASHJOIN
// :2781-2895; hash build gdk/gdk_hash.c:658-704).
//
// GDK's result order: r1 follows the left candidates in order; the matches
// of one left row come in DESCENDING right position, because the chains of
// the right-side hash are built by prepending.  The device reproduces that
// order without chains:
//   build  bucket id per right candidate, stable LSD radix sort of
//          (bucket, candidate index) pairs (sort.hip) + bucket counts and a
//          device scan -> a CSR table whose buckets list right candidates in
//          ascending position; the right key images are gathered into the
//          same order so a probe reads its bucket sequentially;
//   probe  pass 1 counts the matches of every left candidate, a device scan
//          gives every left row its output offset, pass 2 walks its bucket
//          backwards (descending right position) and writes (l oid, r oid).
// nil never matches unless nil_matches.  Integer key types (bte..lng, date,
// oid).
#include <vector>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

struct Side {
	const void *base;
	int w;
	bool uns;          // oid: unsigned
	bool dense;
	oid off;           // dense: position of candidate 0
	const oid *oids;   // materialized candidates
	oid hseq;
	oid cseq;          // dense: oid of candidate 0
};

__device__ __forceinline__ uint64_t
key_of(const Side &s, BUN i, bool &isnil)
{
	BUN p = s.dense ? s.off + i : s.oids[i] - s.hseq;
	switch (s.w) {
	case 1: { int8_t v = ((const int8_t *) s.base)[p]; isnil = v == INT8_MIN; return (uint64_t) (int64_t) v; }
	case 2: { int16_t v = ((const int16_t *) s.base)[p]; isnil = v == INT16_MIN; return (uint64_t) (int64_t) v; }
	case 4: { int32_t v = ((const int32_t *) s.base)[p]; isnil = v == INT32_MIN; return (uint64_t) (int64_t) v; }
	default: {
		uint64_t v = ((const uint64_t *) s.base)[p];
		isnil = s.uns ? v == ((uint64_t) 1 << 63) : (int64_t) v == INT64_MIN;
		return v;
	}
	}
}

__device__ __forceinline__ oid
oid_of(const Side &s, BUN i)
{
	return s.dense ? s.cseq + i : s.oids[i];
}

__device__ __forceinline__ uint64_t
hash64(uint64_t x)
{
	x ^= x >> 33;
	x *= 0xff51afd7ed558ccdull;
	x ^= x >> 33;
	x *= 0xc4ceb9fe1a85ec53ull;
	return x ^ (x >> 33);
}

__global__ __launch_bounds__(256) void
k_build_keys(Side r, BUN n, uint64_t mask, uint64_t *bucket, uint32_t *idx, uint32_t *cnt)
{
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		uint64_t k = key_of(r, j, isnil);
		uint64_t b = hash64(k) & mask;
		bucket[j] = b;
		idx[j] = (uint32_t) j;
		atomicAdd(&cnt[b], 1u);
	}
}

__global__ __launch_bounds__(256) void
k_build_gather(Side r, BUN n, const uint32_t *sidx, uint64_t *skey, uint8_t *snil)
{
	for (BUN e = (BUN) blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		skey[e] = key_of(r, sidx[e], isnil);
		snil[e] = isnil;
	}
}

template <bool WRITE>
__global__ __launch_bounds__(256) void
k_probe(Side l, BUN n, uint64_t mask, const uint64_t *boff, const uint64_t *skey, const uint8_t *snil,
	const uint32_t *sidx, Side r, bool nil_matches, uint32_t *cnt, const uint64_t *ooff, oid *r1, oid *r2)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		uint64_t k = key_of(l, i, isnil);
		uint32_t c = 0;
		if (!isnil || nil_matches) {
			uint64_t b = hash64(k) & mask;
			const uint64_t e0 = boff[b], e1 = boff[b + 1];
			if (WRITE) {
				uint64_t pos = ooff[i];
				const oid lo = oid_of(l, i);
				for (uint64_t e = e1; e > e0; e--) {
					if (skey[e - 1] == k && (bool) snil[e - 1] == isnil) {
						r1[pos] = lo;
						r2[pos] = oid_of(r, sidx[e - 1]);
						pos++;
					}
				}
			} else {
				for (uint64_t e = e0; e < e1; e++)
					c += skey[e] == k && (bool) snil[e] == isnil;
			}
		}
		if (!WRITE)
			cnt[i] = c;
	}
}

bool
join_type_ok(int t)
{
	t = basetype(t);
	return t == MGDK_bte || t == MGDK_sht || t == MGDK_int || t == MGDK_lng || t == MGDK_oid;
}

void
side_init(Side &s, const mgdk_bat *b, const Cand &c)
{
	s.base = b->theap;
	s.w = b->twidth;
	s.uns = basetype(b->ttype) == MGDK_oid;
	s.dense = c.dense;
	s.off = c.dense ? c.seq - b->hseqbase : 0;
	s.oids = c.oids;
	s.hseq = b->hseqbase;
	s.cseq = c.seq;
}

}  // namespace

extern "C" int
mgdk_BATjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
	     bool nil_matches, mgdk_BUN estimate)
{
	(void) estimate;
	if (l == nullptr || r == nullptr || r1p == nullptr) {
		seterr("BATjoin: NULL argument");
		return -1;
	}
	if (basetype(l->ttype) != basetype(r->ttype)) {
		seterr("42000!BATjoin: type mismatch (%s, %s)", atomname(l->ttype), atomname(r->ttype));
		return -1;
	}
	if (!join_type_ok(l->ttype)) {
		seterr("42000!BATjoin: type %s not supported on the device path", atomname(l->ttype));
		return -1;
	}
	ProfScope prof("join");
	Cand lc, rc;
	if (cand_init(&lc, l, sl) < 0 || cand_init(&rc, r, sr) < 0)
		return -1;
	const BUN nl = lc.n, nr = rc.n;
	if (nr >= ((BUN) 1 << 32) || nl >= ((BUN) 1 << 32)) {
		seterr("42000!BATjoin: more than 2^32 rows per side");
		return -1;
	}
	hipStream_t st = stream();
	Side L{}, R{};
	side_init(L, l, lc);
	side_init(R, r, rc);
	// build
	uint64_t B = 1;
	int bits = 0;
	while (B < nr) {
		B <<= 1;
		bits++;
	}
	if (bits < 8) {
		bits = 8;
		B = 256;
	}
	const uint64_t mask = B - 1;
	DevBuf bk(nr * 8 + 8), bk2(nr * 8 + 8), bi(nr * 4 + 4), bi2(nr * 4 + 4), bcnt(B * 4), boff((B + 1) * 8);
	DevBuf skey(nr * 8 + 8), snil(nr + 8), lcnt(nl * 4 + 4), ooff(nl * 8 + 8);
	if (!bk.p || !bk2.p || !bi.p || !bi2.p || !bcnt.p || !boff.p || !skey.p || !snil.p || !lcnt.p || !ooff.p)
		return -1;
	if (!hip_ok(hipMemsetAsync(bcnt.p, 0, B * 4, st), "memset"))
		return -1;
	if (nr)
		hipLaunchKernelGGL(k_build_keys, dim3(grid_for(nr, 1024, 8192)), dim3(256), 0, st, R, nr, mask,
				   bk.as<uint64_t>(), bi.as<uint32_t>(), bcnt.as<uint32_t>());
	uint64_t *sk;
	uint32_t *si;
	if (radix_sort_pairs(bk.as<uint64_t>(), bi.as<uint32_t>(), bk2.as<uint64_t>(), bi2.as<uint32_t>(), nr, bits,
			     &sk, &si) < 0)
		return -1;
	uint64_t tot = 0;
	if (exclusive_scan(bcnt.as<uint32_t>(), boff.as<uint64_t>(), B, &tot) < 0)
		return -1;
	if (!hip_ok(hipMemcpyAsync(boff.as<uint64_t>() + B, &tot, 8, hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	if (nr)
		hipLaunchKernelGGL(k_build_gather, dim3(grid_for(nr, 1024, 8192)), dim3(256), 0, st, R, nr, si,
				   skey.as<uint64_t>(), snil.as<uint8_t>());
	// probe: count, scan, write
	if (nl)
		hipLaunchKernelGGL((k_probe<false>), dim3(grid_for(nl, 1024, 8192)), dim3(256), 0, st, L, nl, mask,
				   boff.as<uint64_t>(), skey.as<uint64_t>(), snil.as<uint8_t>(), si, R, nil_matches,
				   lcnt.as<uint32_t>(), nullptr, nullptr, nullptr);
	uint64_t nout = 0;
	if (exclusive_scan(lcnt.as<uint32_t>(), ooff.as<uint64_t>(), nl, &nout) < 0)
		return -1;
	mgdk_bat *a = newbat(0, MGDK_oid, nout), *b = newbat(0, MGDK_oid, nout);
	if (!a || !b) {
		mgdk_BBPunfix(a);
		mgdk_BBPunfix(b);
		return -1;
	}
	if (nl && nout)
		hipLaunchKernelGGL((k_probe<true>), dim3(grid_for(nl, 1024, 8192)), dim3(256), 0, st, L, nl, mask,
				   boff.as<uint64_t>(), skey.as<uint64_t>(), snil.as<uint8_t>(), si, R, nil_matches,
				   nullptr, ooff.as<uint64_t>(), (oid *) a->theap, (oid *) b->theap);
	if (!sync()) {
		mgdk_BBPunfix(a);
		mgdk_BBPunfix(b);
		return -1;
	}
	a->count = b->count = nout;
	a->tsorted = 1;                 // left candidates in order
	a->trevsorted = nout <= 1;
	a->tkey = nout <= 1;
	a->tnonil = b->tnonil = 1;
	b->tsorted = b->trevsorted = b->tkey = nout <= 1;
	*r1p = a;
	if (r2p)
		*r2p = b;
	else
		mgdk_BBPunfix(b);
	return 0;
}
