// joinkinds.hip -- the left-output join family of gdk_join.c on the MI355X:
// BATintersect / BATsemijoin's candidate output (semi), BATdiff (anti, with
// SQL NOT IN semantics), BATleftjoin and BATouterjoin (gdk_join.c:4320-4407,
// all through leftjoin :4049).
//
// What these return does not depend on which of leftjoin's algorithms runs
// (selectjoin, mergejoin_void, fetchjoin, bitmaskjoin, mergejoin, hashjoin):
// it is the left candidates, in order, with or without a match among the
// right candidates (and, for left / outer joins, that match).  So the device
// runs one plan for all of them:
//   the right candidates' values as sign-extended 64-bit images with their
//   oids, sorted by value (BATsort, stable: ties by oid);
//   per left candidate one binary search: its match count (capped at 2) and
//   first match;
//   flags -> the select path's ordered compaction -> the left oids (and the
//   matches) of the kept candidates.
// The reference's nil rules are kept: a nil matches only with nil_matches
// (gdk_join.c:3127, :2338); NOT IN drops nil left values and gives nothing
// when a right candidate is nil (:3027-3060, :2038), except on the dense-
// right path mergejoin_void (:4096-4101), which has no not_in argument;
// empty sides give nomatch (:301-360); max_one / match_one raise "more than
// one match" (:2760).  A left / outer join where a left candidate matches
// twice is refused loudly: the order of several matches depends on the
// algorithm, which this plan does not replay.
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

struct JSide {
	const void *base;   // nullptr: void
	int w;
	oid tseq;           // void: value of position 0 (nil: all nil)
	oid hseq;
	bool dense;         // candidates dense: seq + i, else oids[i]
	oid seq;
	const oid *oids;
	BUN n;
};

__device__ __forceinline__ oid
js_oid(const JSide &s, BUN i)
{
	return s.dense ? s.seq + i : s.oids[i];
}

// sign-extended image of the value at position p; *isnil
__device__ __forceinline__ int64_t
js_val(const JSide &s, BUN p, bool &isnil)
{
	if (s.base == nullptr) {
		isnil = s.tseq == MGDK_OID_NIL;
		return isnil ? INT64_MIN : (int64_t) (s.tseq + p);
	}
	switch (s.w) {
	case 1: { const int8_t v = ((const int8_t *) s.base)[p]; isnil = v == INT8_MIN; return v; }
	case 2: { const int16_t v = ((const int16_t *) s.base)[p]; isnil = v == INT16_MIN; return v; }
	case 4: { const int32_t v = ((const int32_t *) s.base)[p]; isnil = v == INT32_MIN; return v; }
	default: { const int64_t v = ((const int64_t *) s.base)[p]; isnil = v == INT64_MIN; return v; }
	}
}

__global__ __launch_bounds__(256) void
k_jk_rvals(JSide r, int64_t *rv, oid *ro, uint32_t *anynil)
{
	bool nil_seen = false;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < r.n; i += (BUN) gridDim.x * blockDim.x) {
		const oid o = js_oid(r, i);
		bool isnil;
		rv[i] = js_val(r, o - r.hseq, isnil);
		ro[i] = o;
		nil_seen |= isnil;
	}
	if (__any(nil_seen) && __lane_id() == 0)
		atomicOr(anynil, 1u);
}

__global__ __launch_bounds__(256) void
k_jk_gather(const oid *order, BUN n, const oid *ro, oid *dst)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		dst[i] = ro[order[i]];
}

// mode 0 semi, 1 anti, 2 left, 3 outer; flags[i] = keep the candidate;
// match[i] = its first match (nil: none); err |= 1: two matches, 2: a miss
__global__ __launch_bounds__(256) void
k_jk_probe(JSide l, const int64_t *rv, const oid *ro, BUN nr, bool nil_matches, bool not_in, int mode,
	   int8_t *flags, oid *match, uint32_t *err)
{
	bool two = false, miss = false;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < l.n; i += (BUN) gridDim.x * blockDim.x) {
		const oid lo = js_oid(l, i);
		bool isnil;
		const int64_t v = js_val(l, lo - l.hseq, isnil);
		BUN cnt = 0, at = 0;
		bool skip = false;
		if (isnil && (!nil_matches || not_in)) {
			skip = not_in;
		} else {
			BUN a = 0, b = nr;
			while (a < b) {
				const BUN m = (a + b) >> 1;
				if (rv[m] < v)
					a = m + 1;
				else
					b = m;
			}
			at = a;
			cnt = (a < nr && rv[a] == v) + (a + 1 < nr && rv[a + 1] == v);
		}
		two |= cnt > 1;
		miss |= cnt == 0;
		int8_t keep;
		switch (mode) {
		case 0: keep = cnt > 0; break;
		case 1: keep = cnt == 0 && !skip; break;
		case 2: keep = cnt > 0; break;
		default: keep = 1; break;
		}
		flags[i] = keep;
		if (match)
			match[i] = cnt ? ro[at] : MGDK_OID_NIL;
	}
	const uint32_t f = (__any(two) ? 1u : 0u) | (__any(miss) ? 2u : 0u);
	if (f && __lane_id() == 0)
		atomicOr(err, f);
}

__global__ __launch_bounds__(256) void
k_jk_pick(const oid *idx, oid i0, BUN n, JSide l, const oid *match, oid *r1, oid *r2)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		const BUN i = idx ? idx[k] : i0 + k;
		if (r1)
			r1[k] = js_oid(l, i);
		if (r2)
			r2[k] = match[i];
	}
}

struct Held {
	std::vector<mgdk_bat *> v;
	~Held()
	{
		for (mgdk_bat *b : v)
			mgdk_BBPunfix(b);
	}
	mgdk_bat *keep(mgdk_bat *b)
	{
		if (b)
			v.push_back(b);
		return b;
	}
};

bool
jk_type_ok(int t)
{
	switch (t) {
	case MGDK_void: case MGDK_bte: case MGDK_sht: case MGDK_int: case MGDK_date: case MGDK_lng:
	case MGDK_oid: case MGDK_daytime: case MGDK_timestamp:
		return true;
	}
	return false;
}

int
atomtype(int t)
{
	return t == MGDK_void ? MGDK_oid : basetype(t);
}

// b (msk / mask forms unmasked, as leftjoin does) and its candidates as a JSide
int
jside(const char *fn, mgdk_bat *b, mgdk_bat *s, JSide *j, Held &held, mgdk_bat **bout)
{
	if (b->ttype == MGDK_msk || is_complex_cand(b)) {
		if ((b = held.keep(unmask_cand(b))) == nullptr)
			return -1;
	}
	if (s && is_complex_cand(s) && (s = held.keep(unmask_cand(s))) == nullptr)
		return -1;
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return -1;
	*j = JSide{b->ttype == MGDK_void ? nullptr : b->theap, b->twidth, b->tseqbase, b->hseqbase, ci.dense, ci.seq,
		   ci.oids, ci.n};
	*bout = b;
	(void) fn;
	return 0;
}

// the shared plan; mode as k_jk_probe.  r1 (and r2) out
int
jk_run(const char *fn, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, bool nil_matches, bool not_in,
       bool max_one, int mode, mgdk_bat **r1p, mgdk_bat **r2p)
{
	*r1p = nullptr;
	if (r2p)
		*r2p = nullptr;
	if (l == nullptr || r == nullptr) {
		seterr("%s: inputs must not be NULL", fn);
		return -1;
	}
	Held held;
	JSide L, R;
	mgdk_bat *lb, *rb;
	if (jside(fn, l, sl, &L, held, &lb) < 0 || jside(fn, r, sr, &R, held, &rb) < 0)
		return -1;
	if (atomtype(lb->ttype) != atomtype(rb->ttype)) {
		seterr("%s: inputs not compatible.", fn);
		return -1;
	}
	if (!jk_type_ok(lb->ttype) || !jk_type_ok(rb->ttype)) {
		seterr("%s: type %s is not on the device path", fn, atomname(lb->ttype));
		return -1;
	}
	ProfScope prof("joinkinds");
	hipStream_t st = stream();
	const bool want_r2 = mode >= 2;
	// nomatch (gdk_join.c:301-360): semi / left -> empty; anti / outer -> every
	// left candidate (outer: with nil matches)
	if (L.n == 0 || R.n == 0) {
		const bool all = mode == 1 || mode == 3;
		const BUN n = all ? L.n : 0;
		if (mode <= 1 && L.dense) {
			*r1p = mgdk_BATdense(0, n ? L.seq : 0, n);
			return *r1p ? 0 : -1;
		}
		mgdk_bat *a = newbat(0, MGDK_oid, n), *b = want_r2 ? newbat(0, MGDK_oid, n) : nullptr;
		if (a == nullptr || (want_r2 && b == nullptr)) {
			mgdk_BBPunfix(a);
			mgdk_BBPunfix(b);
			return -1;
		}
		if (n)
			hipLaunchKernelGGL(k_jk_pick, dim3(grid_for(n, 256 * 8, 8192)), dim3(256), 0, st, nullptr, 0, n, L,
					   (const oid *) nullptr, (oid *) a->theap, (oid *) nullptr);
		if (b && n) {
			const oid nil = MGDK_OID_NIL;
			mgdk_bat *c = mgdk_BATconstant(0, MGDK_oid, &nil, n);
			if (c == nullptr || !hip_ok(hipMemcpyAsync(b->theap, c->theap, n * 8, hipMemcpyDeviceToDevice, st),
						   "memcpy")) {
				mgdk_BBPunfix(c);
				mgdk_BBPunfix(a);
				mgdk_BBPunfix(b);
				return -1;
			}
			(void) sync();
			mgdk_BBPunfix(c);
		}
		if (!sync()) {
			mgdk_BBPunfix(a);
			mgdk_BBPunfix(b);
			return -1;
		}
		a->count = n;
		a->tsorted = a->tkey = a->tnonil = 1;
		a->trevsorted = n <= 1;
		if (b) {
			b->count = n;
			b->tnil = n > 0;
			b->tnonil = n == 0;
			b->tsorted = b->trevsorted = 1;
			b->tkey = n <= 1;
		}
		*r1p = a;
		if (r2p)
			*r2p = b;
		else
			mgdk_BBPunfix(b);
		return 0;
	}
	// the dense-right path (mergejoin_void) has no not_in
	const bool rtdense = rb->ttype == MGDK_void ? rb->tseqbase != MGDK_OID_NIL
						    : (rb->ttype == MGDK_oid && rb->tseqbase != MGDK_OID_NIL);
	if (rtdense && R.dense)
		not_in = false;
	// right candidates' images sorted, with their oids
	mgdk_bat *rvb = held.keep(newbat(0, MGDK_lng, R.n));
	// flags in a buffer of their own: BATsort below uses meta_buf()
	DevBuf ro(R.n * 8 + 8), so(R.n * 8 + 8), fl(L.n + 8), mt(want_r2 ? L.n * 8 + 8 : 8), mb(16);
	uint32_t *meta = mb.as<uint32_t>();
	uint32_t *h = (uint32_t *) pinned(16);
	if (rvb == nullptr || !ro.p || !so.p || !fl.p || !mt.p || !mb.p || !hip_ok(hipMemsetAsync(meta, 0, 8, st), "memset"))
		return -1;
	hipLaunchKernelGGL(k_jk_rvals, dim3(grid_for(R.n, 256 * 8, 8192)), dim3(256), 0, st, R,
			   (int64_t *) rvb->theap, ro.as<oid>(), meta);
	rvb->count = R.n;
	rvb->tsorted = rvb->trevsorted = rvb->tkey = 0;
	rvb->tnonil = 0;
	mgdk_bat *sv = nullptr, *sord = nullptr;
	if (mgdk_BATsort(&sv, &sord, nullptr, rvb, nullptr, nullptr, false, false, true) != 0)
		return -1;
	held.keep(sv);
	held.keep(sord);
	// sorted right oids
	{
		const oid *ord = sord->ttype == MGDK_void ? nullptr : (const oid *) sord->theap;
		if (ord)
			hipLaunchKernelGGL(k_jk_gather, dim3(grid_for(R.n, 256 * 8, 8192)), dim3(256), 0, st, ord, R.n,
					   (const oid *) ro.p, so.as<oid>());
		else if (!hip_ok(hipMemcpyAsync(so.p, ro.p, R.n * 8, hipMemcpyDeviceToDevice, st), "memcpy"))
			return -1;
	}
	const int64_t *rvs = sv->ttype == MGDK_void ? nullptr : (const int64_t *) sv->theap;
	if (rvs == nullptr) {
		seterr("%s: sorted right values", fn);
		return -1;
	}
	hipLaunchKernelGGL(k_jk_probe, dim3(grid_for(L.n, 256 * 8, 8192)), dim3(256), 0, st, L, rvs, so.as<oid>(), R.n,
			   nil_matches, not_in, mode, fl.as<int8_t>(), want_r2 ? mt.as<oid>() : (oid *) nullptr, meta + 1);
	if (!hip_ok(hipMemcpyAsync(h, meta, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	// copies: compact_flags below reuses the pinned buffer
	const uint32_t rnil = h[0], perr = h[1];
	if ((perr & 1) && max_one) {
		seterr("more than one match");
		return -1;
	}
	if ((perr & 1) && mode >= 2) {
		seterr("%s: a left row with several matches is not on the device path", fn);
		return -1;
	}
	if (not_in && rnil) {
		// NOT IN a set holding a nil: nothing qualifies
		*r1p = mgdk_BATdense(0, 0, 0);
		return *r1p ? 0 : -1;
	}
	// the kept candidates
	mgdk_bat *pos = held.keep(compact_flags(fl.as<int8_t>(), L.n, 0));
	if (pos == nullptr)
		return -1;
	const BUN n = pos->count;
	const oid *idx = pos->ttype == MGDK_void ? nullptr : (const oid *) pos->theap;
	const oid i0 = pos->ttype == MGDK_void ? pos->tseqbase : 0;
	if (mode <= 1 && L.dense) {
		// dense candidates: the positions are the oids shifted
		mgdk_bat *a = newbat(0, MGDK_oid, n);
		if (a == nullptr)
			return -1;
		if (n)
			hipLaunchKernelGGL(k_jk_pick, dim3(grid_for(n, 256 * 8, 8192)), dim3(256), 0, st, idx, i0, n, L,
					   (const oid *) nullptr, (oid *) a->theap, (oid *) nullptr);
		if (!sync()) {
			mgdk_BBPunfix(a);
			return -1;
		}
		a->count = n;
		a->tsorted = a->tkey = a->tnonil = 1;
		a->trevsorted = n <= 1;
		*r1p = cand_finish(a, n);
		return *r1p ? 0 : -1;
	}
	mgdk_bat *a = newbat(0, MGDK_oid, n), *b = want_r2 ? newbat(0, MGDK_oid, n) : nullptr;
	if (a == nullptr || (want_r2 && b == nullptr)) {
		mgdk_BBPunfix(a);
		mgdk_BBPunfix(b);
		return -1;
	}
	if (n)
		hipLaunchKernelGGL(k_jk_pick, dim3(grid_for(n, 256 * 8, 8192)), dim3(256), 0, st, idx, i0, n, L,
				   want_r2 ? mt.as<const oid>() : (const oid *) nullptr, (oid *) a->theap,
				   b ? (oid *) b->theap : (oid *) nullptr);
	if (!sync()) {
		mgdk_BBPunfix(a);
		mgdk_BBPunfix(b);
		return -1;
	}
	a->count = n;
	a->tsorted = a->tkey = a->tnonil = 1;
	a->trevsorted = n <= 1;
	if (mode <= 1) {
		*r1p = cand_finish(a, n);
		return *r1p ? 0 : -1;
	}
	b->count = n;
	b->tsorted = b->trevsorted = n <= 1;
	b->tkey = n <= 1;
	// an outer join's miss leaves a nil match (k_jk_probe: meta bit 2)
	const bool anynil = mode == 3 && (perr & 2) != 0;
	b->tnil = anynil;
	b->tnonil = !anynil;
	*r1p = a;
	*r2p = b;
	return 0;
}

}  // namespace

extern "C" mgdk_bat *
mgdk_BATintersect(mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, bool nil_matches, bool max_one,
		  mgdk_BUN estimate)
{
	(void) estimate;
	mgdk_bat *a;
	return jk_run("BATintersect", l, r, sl, sr, nil_matches, false, max_one, 0, &a, nullptr) < 0 ? nullptr : a;
}

extern "C" mgdk_bat *
mgdk_BATdiff(mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, bool nil_matches, bool not_in,
	     mgdk_BUN estimate)
{
	(void) estimate;
	mgdk_bat *a;
	return jk_run("BATdiff", l, r, sl, sr, nil_matches, not_in, false, 1, &a, nullptr) < 0 ? nullptr : a;
}

extern "C" int
mgdk_BATsemijoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		 bool nil_matches, bool max_one, mgdk_BUN estimate)
{
	(void) estimate;
	if (r2p != nullptr) {
		*r2p = nullptr;
		seterr("BATsemijoin: the right output (which match of several) is not on the device path");
		return -1;
	}
	return jk_run("BATsemijoin", l, r, sl, sr, nil_matches, false, max_one, 0, r1p, nullptr);
}

extern "C" int
mgdk_BATleftjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		 bool nil_matches, mgdk_BUN estimate)
{
	(void) estimate;
	return jk_run("BATleftjoin", l, r, sl, sr, nil_matches, false, false, 2, r1p, r2p);
}

extern "C" int
mgdk_BATouterjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
		  bool nil_matches, bool match_one, mgdk_BUN estimate)
{
	(void) estimate;
	return jk_run("BATouterjoin", l, r, sl, sr, nil_matches, false, match_one, 3, r1p, r2p);
}
