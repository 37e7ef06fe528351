// joinkinds.hip -- the left-output join family of gdk_join.c on the MI355X:
// BATintersect / BATsemijoin's candidate output (semi), BATdiff (anti, with
// SQL NOT IN semantics), BATleftjoin and BATouterjoin (gdk_join.c:4320-4407,
// all through leftjoin :4049), and BATmarkjoin (:4367).
//
// A left candidate's matches do not depend on which of leftjoin's algorithms
// runs (selectjoin, mergejoin_void, fetchjoin, bitmaskjoin, mergejoin,
// hashjoin, the swapped hashjoin); their order, which one a semi join with a
// right output keeps, and two quirks do.  So the device runs one plan and
// asks the reference's algorithm choice (joinalgo.hip leftjoin_algo) only
// when the answer depends on it:
//   the right candidates' values as sign-extended 64-bit images with their
//   candidate indexes, sorted by value (BATsort, stable: ties by index);
//   per left candidate two binary searches: its match range and count;
//   one match per candidate (or only the left output): flags -> the select
//   path's ordered compaction -> the left oids (and the matches);
//   several matches with a right output: per candidate its row count, an
//   exclusive scan, and each candidate writes its rows in the algorithm's
//   order -- ascending (selectjoin, mergejoin), descending (hashjoin: the
//   hash chains), the first / last match for semi (selectjoin, the swapped
//   hash join's BATunique; hashjoin, mergejoin in equal order), the swapped
//   hash join's pairs in hashjoin(r, l) order put through the GDKqsort
//   replay (qsort.hip) as the reference sorts them (gdk_join.c:4236);
//   fetchjoin (dense l): the rows in right position order, i.e. the left
//   candidates descending when r is reverse sorted, and no rows for misses
//   (the reference reaches it without checking nil_on_miss, :4156-4168).
// The reference's nil rules are kept: a nil matches only with nil_matches
// (gdk_join.c:3127, :2338); NOT IN drops nil left values and gives nothing
// when a right candidate is nil (:3027-3060, :2038), except on the dense-
// right path mergejoin_void (:4096-4101), which has no not_in; mergejoin
// over an ordered l skips l's nils before its scan, so BATdiff does not list
// them there (:2093-2100); empty sides give nomatch (:301-360); max_one /
// match_one raise "more than one match" (:2760), selectjoin's min_one "not
// enough matches" (:399-404).  flt / dbl / str keys join as BATjoin's order-
// and equality-preserving integer images (joinalgo.hip).
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
k_jk_iota(BUN n, oid *dst)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		dst[i] = i;
}

__global__ __launch_bounds__(256) void
k_jk_gather(const oid *order, BUN n, const oid *ro, oid *dst)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		dst[i] = ro[order[i]];
}

// mode 0 semi, 1 anti, 2 left, 3 outer, 4 mark; flags[i] = keep the
// candidate; match[i] = its first match (nil: none); mark[i] (mode 4): TRUE on
// a match, on a miss nil when the left value or a right candidate (*rnil) is
// nil, else FALSE (gdk_join.c:3026-3076, :3127-3133); lob[i] / cnt[i]: its
// match range in the sorted right images (optional).  err bits: 1 two
// matches, 2 a miss, 4 a nil mark, 8 a nil left value, 16 a miss of a left
// value that can match, 32 a count of 2^32 or more
__global__ __launch_bounds__(256) void
k_jk_probe(JSide l, const int64_t *rv, const oid *ro, BUN nr, bool nil_matches, bool not_in, int mode,
	   int8_t *flags, oid *match, int8_t *mark, const uint32_t *rnil, uint64_t *lob, uint32_t *cntb, uint32_t *err)
{
	uint32_t f = 0;
	const bool rhasnil = mark && *rnil != 0;
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
			BUN c = a, d = nr;
			while (c < d) {
				const BUN m = (c + d) >> 1;
				if (rv[m] <= v)
					c = m + 1;
				else
					d = m;
			}
			cnt = c - a;
			f |= cnt == 0 ? 16u : 0u;
		}
		f |= (cnt > 1 ? 1u : 0u) | (cnt == 0 ? 2u : 0u) | (isnil ? 8u : 0u) | (cnt >> 32 ? 32u : 0u);
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
		if (mark) {
			const int8_t m = cnt ? 1 : (isnil || rhasnil) ? INT8_MIN : 0;
			mark[i] = m;
			f |= m == INT8_MIN ? 4u : 0u;
		}
		if (lob) {
			lob[i] = at;
			cntb[i] = (uint32_t) (cnt >> 32 ? 0xffffffffu : cnt);
		}
	}
	for (int o = 32; o > 0; o >>= 1)
		f |= __shfl_xor(f, o);
	if (f && __lane_id() == 0)
		atomicOr(err, f);
}

// mergejoin over an ordered l skips l's nil values (gdk_join.c:2093-2100):
// BATdiff's flags of nil left values cleared
__global__ __launch_bounds__(256) void
k_jk_dropnil(JSide l, int8_t *flags)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < l.n; i += (BUN) gridDim.x * blockDim.x) {
		bool isnil;
		(void) js_val(l, js_oid(l, i) - l.hseq, isnil);
		if (isnil)
			flags[i] = 0;
	}
}

// the rows each left candidate puts out when it may have several matches:
// semi one per match found, left one per match, outer / mark one per match
// or one nil row (fetchjoin: no nil rows)
__global__ __launch_bounds__(256) void
k_jk_ocnt(BUN n, const uint32_t *cnt, int mode, bool fetch, uint32_t *ocnt)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const uint32_t c = cnt[i];
		ocnt[i] = mode == 0 ? (c > 0) : (mode == 2 || fetch) ? c : (c > 0 ? c : 1u);
	}
}

// the order a left candidate's matches leave in (see the head of this file)
enum { JK_ASC = 0, JK_DESC = 1, JK_FIRST = 2, JK_LAST = 3 };

// each left candidate writes its rows at its offset (rev: the candidates'
// blocks in reverse order, fetchjoin over a reverse-sorted r); sidx: the
// right candidate index of each sorted image; mk: the probe's per-candidate
// mark (for a miss); pairs (optional): (right index << 32 | ~left index)
// keys of the swapped hash join instead of the result columns
__global__ __launch_bounds__(256) void
k_jk_emit(JSide L, JSide R, const uint64_t *lob, const uint32_t *cnt, const uint32_t *ocnt, const uint64_t *off,
	  uint64_t tot, bool rev, int kind, const oid *sidx, const int8_t *mk, oid *r1, oid *r2, int8_t *r3,
	  int64_t *pairs)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < L.n; i += (BUN) gridDim.x * blockDim.x) {
		const uint32_t q = ocnt[i], c = cnt[i];
		if (q == 0)
			continue;
		const uint64_t o = rev ? tot - off[i] - q : off[i];
		const oid lo = js_oid(L, i);
		if (c == 0) {
			r1[o] = lo;
			if (r2)
				r2[o] = MGDK_OID_NIL;
			if (r3)
				r3[o] = mk[i];
			continue;
		}
		const uint64_t a = lob[i];
		for (uint32_t k = 0; k < q; k++) {
			const uint64_t p = kind == JK_ASC ? a + k : kind == JK_DESC ? a + c - 1 - k
					   : kind == JK_FIRST ? a : a + c - 1;
			const oid ri = sidx[p];
			if (pairs) {
				pairs[o + k] = (int64_t) ((ri << 32) | (0xffffffffull - i));
				continue;
			}
			r1[o + k] = lo;
			if (r2)
				r2[o + k] = js_oid(R, ri);
			if (r3)
				r3[o + k] = 1;
		}
	}
}

// the swapped hash join's sorted pair keys -> GDKqsort replay input
// (rank = left candidate index, payload = right candidate index)
__global__ __launch_bounds__(256) void
k_jk_swkeys(const int64_t *keys, uint64_t n, uint32_t *rank, uint64_t *pay)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		const uint64_t x = (uint64_t) keys[k];
		rank[k] = 0xffffffffu - (uint32_t) x;
		pay[k] = x >> 32;
	}
}

__global__ __launch_bounds__(256) void
k_jk_swout(const uint32_t *rank, const uint64_t *pay, uint64_t n, JSide L, JSide R, oid *r1, oid *r2)
{
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		r1[k] = js_oid(L, rank[k]);
		if (r2)
			r2[k] = js_oid(R, pay[k]);
	}
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
jside(const char *fn, mgdk_bat *b, mgdk_bat *s, JSide *j, Held &held, mgdk_bat **bout, Cand *cout = nullptr)
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
	if (cout)
		*cout = ci;
	(void) fn;
	return 0;
}

// a result column released to the caller or, on an error return, freed
struct Own {
	mgdk_bat *b = nullptr;
	~Own() { mgdk_BBPunfix(b); }
	mgdk_bat *release()
	{
		mgdk_bat *x = b;
		b = nullptr;
		return x;
	}
};

// the shared plan; mode as k_jk_probe.  r1 (and r2, and for mode 4 the
// mark column r3) out; semi (mode 0) with r2p: BATsemijoin's right output
int
jk_run(const char *fn, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, bool nil_matches, bool not_in,
       bool max_one, int mode, mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat **r3p = nullptr, bool min_one = false)
{
	*r1p = nullptr;
	if (r2p)
		*r2p = nullptr;
	if (r3p)
		*r3p = nullptr;
	if (l == nullptr || r == nullptr) {
		seterr("%s: inputs must not be NULL", fn);
		return -1;
	}
	// flt / dbl / str keys: BATjoin's integer images keep equality, order
	// and nil, so every choice and result below is the keys' own
	{
		const int lt = basetype(l->ttype), rt = basetype(r->ttype);
		if ((lt == MGDK_flt || lt == MGDK_dbl || l->ttype == MGDK_str) && lt == rt && l->ttype == r->ttype) {
			mgdk_bat *li = nullptr, *ri = nullptr;
			if (l->ttype == MGDK_str) {
				if (join_str_images(l, r, &li, &ri) != 0)
					return -1;
			} else {
				li = join_float_image(l);
				ri = li ? join_float_image(r) : nullptr;
			}
			int rc = -1;
			if (li && ri) {
				rc = jk_run(fn, li, ri, sl, sr, nil_matches, not_in, max_one, mode, r1p, r2p, r3p, min_one);
				join_image_flags_back(l, r, li, ri);
			}
			mgdk_BBPunfix(li);
			mgdk_BBPunfix(ri);
			return rc;
		}
	}
	Held held;
	JSide L, R;
	Cand LC, RC;
	mgdk_bat *lb, *rb;
	if (jside(fn, l, sl, &L, held, &lb, &LC) < 0 || jside(fn, r, sr, &R, held, &rb, &RC) < 0)
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
	const bool want_r2 = mode == 4 || mode == 0 ? r2p != nullptr : mode >= 2;
	const bool nil_on_miss = mode >= 3;
	const bool semi = mode == 0 || (mode == 4 && r2p == nullptr);
	Own mk;
	// nomatch (gdk_join.c:301-360): semi / left -> empty; anti / outer / mark
	// -> every left candidate (outer, mark: with nil matches; mark: FALSE,
	// leftjoin :4144 passes defmark 0)
	if (L.n == 0 || R.n == 0) {
		const bool all = mode == 1 || mode >= 3;
		const BUN n = all ? L.n : 0;
		if (mode == 4) {
			const int8_t f = 0;
			if ((mk.b = mgdk_BATconstant(0, MGDK_bit, &f, n)) == nullptr)
				return -1;
		}
		if (mode <= 1 && L.dense && !want_r2) {
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
		*r1p = mode == 0 ? cand_finish(a, n) : a;
		if (r2p)
			*r2p = b;
		else
			mgdk_BBPunfix(b);
		if (r3p)
			*r3p = mk.release();
		return *r1p ? 0 : -1;
	}
	if (mode == 4 && (mk.b = newbat(0, MGDK_bit, L.n)) == nullptr)
		return -1;
	// the dense-right path (mergejoin_void) has no not_in
	const bool rtdense = rb->ttype == MGDK_void ? rb->tseqbase != MGDK_OID_NIL
						    : (rb->ttype == MGDK_oid && rb->tseqbase != MGDK_OID_NIL);
	if (rtdense && R.dense)
		not_in = false;
	// right candidates' images sorted, with their candidate indexes (the
	// sort's order) and oids
	mgdk_bat *rvb = held.keep(newbat(0, MGDK_lng, R.n));
	// flags in a buffer of their own: BATsort below uses meta_buf()
	DevBuf ro(R.n * 8 + 8), so(R.n * 8 + 8), fl(L.n + 8), mt(want_r2 ? L.n * 8 + 8 : 8), mb(16);
	DevBuf lob(L.n * 8 + 8), cnt(L.n * 4 + 8);
	uint32_t *meta = mb.as<uint32_t>();
	uint32_t *h = (uint32_t *) pinned(16);
	if (rvb == nullptr || !ro.p || !so.p || !fl.p || !mt.p || !mb.p || !lob.p || !cnt.p ||
	    !hip_ok(hipMemsetAsync(meta, 0, 8, st), "memset"))
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
	// sorted right oids; the sort's order = the candidate indexes
	const oid *ord = sord->ttype == MGDK_void ? nullptr : (const oid *) sord->theap;
	DevBuf sidxb(ord ? 8 : R.n * 8 + 8);
	if (ord)
		hipLaunchKernelGGL(k_jk_gather, dim3(grid_for(R.n, 256 * 8, 8192)), dim3(256), 0, st, ord, R.n,
				   (const oid *) ro.p, so.as<oid>());
	else if (!sidxb.p || !hip_ok(hipMemcpyAsync(so.p, ro.p, R.n * 8, hipMemcpyDeviceToDevice, st), "memcpy"))
		return -1;
	const int64_t *rvs = sv->ttype == MGDK_void ? nullptr : (const int64_t *) sv->theap;
	if (rvs == nullptr) {
		seterr("%s: sorted right values", fn);
		return -1;
	}
	hipLaunchKernelGGL(k_jk_probe, dim3(grid_for(L.n, 256 * 8, 8192)), dim3(256), 0, st, L, rvs, so.as<oid>(), R.n,
			   nil_matches, not_in, mode, fl.as<int8_t>(), want_r2 ? mt.as<oid>() : (oid *) nullptr,
			   mk.b ? (int8_t *) mk.b->theap : (int8_t *) nullptr, (const uint32_t *) meta, lob.as<uint64_t>(),
			   cnt.as<uint32_t>(), meta + 1);
	if (!hip_ok(hipMemcpyAsync(h, meta, 8, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
		return -1;
	// copies: compact_flags below reuses the pinned buffer
	const uint32_t rnil = h[0], perr = h[1];
	if ((perr & 1) && max_one) {
		seterr("more than one match");
		return -1;
	}
	if (not_in && rnil) {
		// NOT IN a set holding a nil: nothing qualifies
		*r1p = mgdk_BATdense(0, 0, 0);
		return *r1p ? 0 : -1;
	}
	// the reference's algorithm choice, where the answer depends on it
	int algo = -1;
	bool eqo = true;
	const bool ltdense = lb->ttype == MGDK_void ? lb->tseqbase != MGDK_OID_NIL
						    : (lb->ttype == MGDK_oid && lb->tseqbase != MGDK_OID_NIL);
	const bool multi = (perr & 1) && want_r2;
	const bool need = multi || (mode == 1 && !not_in && !nil_matches && (perr & 8)) ||
			  (mode >= 2 && want_r2 && ltdense && !nil_matches) || (min_one && (perr & 16));
	if (need) {
		algo = leftjoin_algo(lb, rb, sl, sr, LC, RC,
				     nil_matches, nil_on_miss, semi, mode == 1, not_in, max_one, min_one, want_r2, &eqo);
		if (algo < 0)
			return -1;
	}
	if (min_one && (perr & 16) && algo == LJ_SELECT) {
		seterr("not enough matches");
		return -1;
	}
	if (mode == 1 && algo == LJ_MERGE && (lb->tsorted || lb->trevsorted))
		hipLaunchKernelGGL(k_jk_dropnil, dim3(grid_for(L.n, 256 * 8, 8192)), dim3(256), 0, st, L, fl.as<int8_t>());
	if (multi || algo == LJ_FETCH) {
		if (perr & 32) {
			seterr("%s: a left value with 2^32 or more matches is not on the device path", fn);
			return -1;
		}
		const bool fetch = algo == LJ_FETCH;
		const bool rev = fetch && !rb->tsorted;
		DevBuf ocnt(L.n * 4 + 8), off(L.n * 8 + 8);
		if (!ocnt.p || !off.p)
			return -1;
		hipLaunchKernelGGL(k_jk_ocnt, dim3(grid_for(L.n, 256 * 8, 8192)), dim3(256), 0, st, L.n,
				   cnt.as<const uint32_t>(), mode, fetch, ocnt.as<uint32_t>());
		uint64_t tot = 0;
		if (exclusive_scan(ocnt.as<const uint32_t>(), off.as<uint64_t>(), L.n, &tot) != 0)
			return -1;
		int kind = JK_ASC;
		if (semi)
			kind = algo == LJ_HASH || (algo == LJ_MERGE && eqo) ? JK_LAST : JK_FIRST;
		else if (algo == LJ_HASH)
			kind = JK_DESC;
		const oid *sidx = ord ? ord : nullptr;
		if (sidx == nullptr) {
			// the right images were already in order: index i is i
			hipLaunchKernelGGL(k_jk_iota, dim3(grid_for(R.n, 256 * 8, 8192)), dim3(256), 0, st, R.n,
					   sidxb.as<oid>());
			sidx = sidxb.as<const oid>();
		}
		Own A, B;
		if ((A.b = newbat(0, MGDK_oid, tot)) == nullptr || (want_r2 && (B.b = newbat(0, MGDK_oid, tot)) == nullptr))
			return -1;
		Own M;
		if (mode == 4 && (M.b = newbat(0, MGDK_bit, tot)) == nullptr)
			return -1;
		const bool swap = algo == LJ_SWAP && !semi;
		if (swap) {
			// hashjoin(r, l)'s pairs -- right candidates in order, each
			// one's left matches descending -- then GDKqsort on the left
			// oids (gdk_join.c:4203-4251)
			if (R.n >= ((BUN) 1 << 31) || L.n >= ((BUN) 1 << 32) || tot >= ((uint64_t) 1 << 32)) {
				seterr("%s: swapped hash join of more than 2^31 rows is not on the device path", fn);
				return -1;
			}
			mgdk_bat *pk = held.keep(newbat(0, MGDK_lng, tot));
			if (pk == nullptr)
				return -1;
			if (tot)
				hipLaunchKernelGGL(k_jk_emit, dim3(grid_for(L.n, 256 * 4, 8192)), dim3(256), 0, st, L, R,
						   lob.as<const uint64_t>(), cnt.as<const uint32_t>(), ocnt.as<const uint32_t>(),
						   off.as<const uint64_t>(), tot, false, (int) JK_ASC, sidx, (const int8_t *) nullptr,
						   (oid *) nullptr, (oid *) nullptr, (int8_t *) nullptr, (int64_t *) pk->theap);
			pk->count = tot;
			pk->tsorted = pk->trevsorted = pk->tkey = tot <= 1;
			pk->tnonil = 1;
			mgdk_bat *ps = nullptr;
			if (tot > 1) {
				if (mgdk_BATsort(&ps, nullptr, nullptr, pk, nullptr, nullptr, false, false, false) != 0)
					return -1;
				held.keep(ps);
			}
			DevBuf rank(tot * 4 + 8), pay(tot * 8 + 8);
			if (!rank.p || !pay.p)
				return -1;
			if (tot)
				hipLaunchKernelGGL(k_jk_swkeys, dim3(grid_for(tot, 256 * 8, 8192)), dim3(256), 0, st,
						   (const int64_t *) (ps ? ps->theap : pk->theap), tot, rank.as<uint32_t>(),
						   pay.as<uint64_t>());
			if (tot > 1) {
				std::vector<std::pair<uint64_t, uint32_t>> segs{{0, (uint32_t) tot}};
				if (qsort_replay(rank.as<uint32_t>(), pay.as<uint64_t>(), tot, segs) < 0)
					return -1;
			}
			if (tot)
				hipLaunchKernelGGL(k_jk_swout, dim3(grid_for(tot, 256 * 8, 8192)), dim3(256), 0, st,
						   rank.as<const uint32_t>(), pay.as<const uint64_t>(), tot, L, R, (oid *) A.b->theap,
						   B.b ? (oid *) B.b->theap : (oid *) nullptr);
		} else if (tot) {
			hipLaunchKernelGGL(k_jk_emit, dim3(grid_for(L.n, 256 * 4, 8192)), dim3(256), 0, st, L, R,
					   lob.as<const uint64_t>(), cnt.as<const uint32_t>(), ocnt.as<const uint32_t>(),
					   off.as<const uint64_t>(), tot, rev, kind, sidx,
					   mk.b ? (const int8_t *) mk.b->theap : (const int8_t *) nullptr, (oid *) A.b->theap,
					   B.b ? (oid *) B.b->theap : (oid *) nullptr, M.b ? (int8_t *) M.b->theap : (int8_t *) nullptr,
					   (int64_t *) nullptr);
		}
		if (!sync())
			return -1;
		mgdk_bat *a = A.release();
		a->count = tot;
		const bool onekey = semi || !(perr & 1);
		a->tsorted = !rev || tot <= 1;
		a->trevsorted = rev || tot <= 1;
		a->tkey = onekey || tot <= 1;
		a->tnonil = 1;
		a->tnil = 0;
		const bool misses = nil_on_miss && !fetch && (perr & 2);
		if (B.b) {
			B.b->count = tot;
			B.b->tsorted = B.b->trevsorted = B.b->tkey = tot <= 1;
			B.b->tnil = misses;
			B.b->tnonil = !misses;
		}
		if (M.b) {
			M.b->count = tot;
			M.b->tnil = misses && (perr & 4);
			M.b->tnonil = !M.b->tnil;
			M.b->tsorted = M.b->trevsorted = M.b->tkey = tot <= 1;
		}
		*r1p = semi ? cand_finish(a, tot) : a;
		if (*r1p == nullptr)
			return -1;
		if (r2p)
			*r2p = B.release();
		if (r3p)
			*r3p = M.release();
		return 0;
	}
	// the kept candidates
	mgdk_bat *pos = held.keep(compact_flags(fl.as<int8_t>(), L.n, 0));
	if (pos == nullptr)
		return -1;
	const BUN n = pos->count;
	const oid *idx = pos->ttype == MGDK_void ? nullptr : (const oid *) pos->theap;
	const oid i0 = pos->ttype == MGDK_void ? pos->tseqbase : 0;
	if (mode <= 1 && L.dense && !want_r2) {
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
		if (b) {
			// BATsemijoin's right output: one match per kept candidate
			b->count = n;
			b->tsorted = b->trevsorted = b->tkey = n <= 1;
			b->tnil = 0;
			b->tnonil = 1;
		}
		*r1p = cand_finish(a, n);
		if (*r1p == nullptr) {
			mgdk_BBPunfix(b);
			return -1;
		}
		if (r2p)
			*r2p = b;
		return 0;
	}
	if (mode == 4) {
		// every left candidate is kept: the marks are in candidate order
		mk.b->count = n;
		mk.b->tnil = (perr & 4) != 0;
		mk.b->tnonil = !mk.b->tnil;
		mk.b->tsorted = mk.b->trevsorted = n <= 1;
		mk.b->tkey = n <= 1;
		*r3p = mk.release();
	}
	if (!want_r2) {
		*r1p = a;
		return 0;
	}
	b->count = n;
	b->tsorted = b->trevsorted = n <= 1;
	b->tkey = n <= 1;
	// an outer join's miss leaves a nil match (k_jk_probe: meta bit 2)
	const bool anynil = mode >= 3 && (perr & 2) != 0;
	b->tnil = anynil;
	b->tnonil = !anynil;
	*r1p = a;
	*r2p = b;
	return 0;
}

// ---- BATthetajoin / BATbandjoin (gdk_join.c:3699 thetajoin, :4626) -----
// The reference runs nested loops: the pairs in left-candidate order, each
// left candidate's matches in right-candidate order.  On the device the
// right candidates' values are sorted once (their candidate index along);
// a left value's matches are one range of that order (two for <>), found by
// binary search -- the predicate is monotone in the right value -- then the
// counts give the offsets, each left candidate writes its (left, right)
// index pairs, and a sort of the pairs restores the right-candidate order
// inside each left candidate (skipped when the right side is already in
// value order).  bandjoin over flt / dbl evaluates the reference's
// floating-point expression (and its overflow rules) pair by pair instead:
// a brute-force nested loop, right values streamed through LDS.

#pragma clang fp contract(off)

// signed 64-bit key ordered as ATOMcompare: nil the smallest (and equal to
// itself), -0.0 == +0.0 for flt / dbl
__device__ __forceinline__ int64_t
th_key(const JSide &s, int fk, BUN p)
{
	if (fk == 0) {
		bool isnil;
		const int64_t v = js_val(s, p, isnil);
		return isnil ? INT64_MIN : v;
	}
	double d = fk == 1 ? (double) ((const float *) s.base)[p] : ((const double *) s.base)[p];
	if (d != d)
		return INT64_MIN;
	if (d == 0)
		d = 0;
	uint64_t b = (uint64_t) __double_as_longlong(d);
	b = (b >> 63) ? ~b : (b | (1ull << 63));
	return (int64_t) (b ^ (1ull << 63));
}

__global__ __launch_bounds__(256) void
k_th_rkeys(JSide r, int fk, int64_t *key)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < r.n; i += (BUN) gridDim.x * blockDim.x)
		key[i] = th_key(r, fk, js_oid(r, i) - r.hseq);
}

// first index in [a, b) with v[i] >= x (ge) or v[i] > x (!ge)
__device__ __forceinline__ BUN
th_bound(const int64_t *v, BUN a, BUN b, int64_t x, bool gt)
{
	while (a < b) {
		const BUN m = a + (b - a) / 2;
		if (gt ? v[m] <= x : v[m] < x)
			a = m + 1;
		else
			b = m;
	}
	return a;
}

struct ThArgs {
	int mode;          // 0 theta, 1 band (integers)
	int mask;          // theta: MASK_EQ 1 | MASK_LT 2 | MASK_GT 4
	bool nil_matches;
	hge c1, c2;        // band
	bool linc, hinc;
};

// per left candidate: its ranges [r0, r1) and [r2, r3) of the sorted right
// values and their total
__global__ __launch_bounds__(256) void
k_th_ranges(JSide L, int fk, const int64_t *sk, BUN nr, ThArgs t, uint32_t *rg, uint32_t *cnt)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < L.n; i += (BUN) gridDim.x * blockDim.x) {
		const int64_t x = th_key(L, fk, js_oid(L, i) - L.hseq);
		const BUN nnil = th_bound(sk, 0, nr, INT64_MIN, true);
		BUN a = 0, b = 0, c = 0, d = 0;
		if (t.mode == 0) {
			if (x != INT64_MIN || t.nil_matches) {
				// the right values below / equal to / above x are three
				// consecutive parts; vl op vr keeps some of them: GT the
				// part below, EQ the equal one, LT the part above
				const BUN s0 = t.nil_matches ? 0 : nnil;
				const BUN lo = th_bound(sk, s0, nr, x, false), hi = th_bound(sk, s0, nr, x, true);
				const BUN pa[3] = {s0, lo, hi}, pb[3] = {lo, hi, nr};
				const bool inc[3] = {(t.mask & 4) != 0, (t.mask & 1) != 0, (t.mask & 2) != 0};
				int nrg = 0;
				BUN ra[2] = {0, 0}, rb[2] = {0, 0};
				for (int q = 0; q < 3; q++) {
					if (!inc[q] || pa[q] == pb[q])
						continue;
					if (nrg && rb[nrg - 1] == pa[q])
						rb[nrg - 1] = pb[q];
					else {
						ra[nrg] = pa[q];
						rb[nrg] = pb[q];
						nrg++;
					}
				}
				a = ra[0];
				b = rb[0];
				c = ra[1];
				d = rb[1];
			}
		} else if (x != INT64_MIN) {
			// band: vr - c1 <= vl <= vr + c2 (exact): vl - c2 <= vr <= vl + c1
			const hge lo = (hge) x - t.c2, hi = (hge) x + t.c1;
			const int64_t lo64 = lo < (hge) INT64_MIN ? INT64_MIN : (int64_t) lo;
			const int64_t hi64 = hi > (hge) INT64_MAX ? INT64_MAX : (int64_t) hi;
			if (hi >= (hge) INT64_MIN && lo <= (hge) INT64_MAX) {
				a = lo < (hge) INT64_MIN ? nnil : th_bound(sk, nnil, nr, lo64, !t.hinc);
				b = hi > (hge) INT64_MAX ? nr : th_bound(sk, nnil, nr, hi64, t.linc);
				if (b < a)
					b = a;
			}
		}
		rg[4 * i] = (uint32_t) a;
		rg[4 * i + 1] = (uint32_t) b;
		rg[4 * i + 2] = (uint32_t) c;
		rg[4 * i + 3] = (uint32_t) d;
		cnt[i] = (uint32_t) ((b - a) + (d - c));
	}
}

// the pairs of each left candidate: key (left index << rb) | right index
// (sorted order's payload), or straight into r1 / r2 when the right side
// is in value order
__global__ __launch_bounds__(256) void
k_th_emit(JSide L, JSide R, const uint32_t *rg, const uint64_t *off, const oid *sidx, int rb, int64_t *keys,
	  oid *r1, oid *r2)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < L.n; i += (BUN) gridDim.x * blockDim.x) {
		BUN o = off[i];
		const oid lo = js_oid(L, i);
		for (int q = 0; q < 2; q++) {
			const BUN a = rg[4 * i + 2 * q], b = rg[4 * i + 2 * q + 1];
			for (BUN k = a; k < b; k++, o++) {
				const BUN ri = sidx ? sidx[k] : k;
				if (keys) {
					keys[o] = (int64_t) (((uint64_t) i << rb) | ri);
				} else {
					r1[o] = lo;
					r2[o] = js_oid(R, ri);
				}
			}
		}
	}
}

__global__ __launch_bounds__(256) void
k_th_decode(const int64_t *keys, BUN n, int rb, JSide L, JSide R, oid *r1, oid *r2)
{
	const uint64_t m = ((uint64_t) 1 << rb) - 1;
	for (BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (BUN) gridDim.x * blockDim.x) {
		const uint64_t x = (uint64_t) keys[k];
		r1[k] = js_oid(L, x >> rb);
		r2[k] = js_oid(R, x & m);
	}
}

// bandjoin's pair test for flt (in dbl) and dbl (SUBF / ADDF_WITH_CHECK),
// gdk_join.c:4923-4966
template <typename T>
__device__ __forceinline__ bool
band_fp(T vl, T vr, T c1, T c2, bool linc, bool hinc)
{
	if constexpr (sizeof(T) == 4) {
		double v1 = (double) vr, v2 = v1;
		v1 -= c1;
		if (vl <= v1 && (!linc || vl != v1))
			return false;
		v2 += c2;
		if (vl >= v2 && (!hinc || vl != v2))
			return false;
		return true;
	} else {
		const double mx = 1.7976931348623157e308;
		bool skip1 = false;
		double v1 = 0, v2 = 0;
		if (c1 < 1 ? mx + c1 < vr : -mx + c1 > vr) {
			if (c1 < 0)
				return false;
			skip1 = true;
		} else {
			v1 = vr - c1;
		}
		if (!skip1 && vl <= v1 && (!linc || vl != v1))
			return false;
		if (c2 < 1 ? -mx - c2 > vr : mx - c2 < vr) {
			if (c2 > 0)
				return false;
			return true;
		}
		v2 = vr + c2;
		if (vl >= v2 && (!hinc || vl != v2))
			return false;
		return true;
	}
}

// brute force over the right candidates (streamed through LDS, 1024 at a
// time): pass 0 counts per left candidate, pass 1 writes the pairs in
// right-candidate order
template <typename T>
__global__ __launch_bounds__(256) void
k_band_fp(JSide L, JSide R, T c1, T c2, bool linc, bool hinc, int pass, uint32_t *cnt, const uint64_t *off,
	  oid *r1, oid *r2)
{
	__shared__ T sv[1024];
	__shared__ oid so[1024];
	__shared__ uint8_t sn[1024];
	const BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	const bool live = i < L.n;
	oid lo = 0;
	T vl = 0;
	bool lnil = true;
	if (live) {
		lo = js_oid(L, i);
		vl = ((const T *) L.base)[lo - L.hseq];
		lnil = vl != vl;
	}
	uint32_t c = 0;
	BUN o = pass && live ? off[i] : 0;
	for (BUN c0 = 0; c0 < R.n; c0 += 1024) {
		__syncthreads();
		for (unsigned q = threadIdx.x; q < 1024; q += blockDim.x) {
			const BUN k = c0 + q;
			if (k < R.n) {
				const oid ro = js_oid(R, k);
				const T v = ((const T *) R.base)[ro - R.hseq];
				sv[q] = v;
				so[q] = ro;
				sn[q] = v != v;
			}
		}
		__syncthreads();
		if (!live || lnil)
			continue;
		const unsigned m = (unsigned) min((BUN) 1024, R.n - c0);
		for (unsigned q = 0; q < m; q++) {
			if (sn[q] || !band_fp<T>(vl, sv[q], c1, c2, linc, hinc))
				continue;
			if (pass) {
				r1[o] = lo;
				r2[o] = so[q];
				o++;
			} else {
				c++;
			}
		}
	}
	if (live && !pass)
		cnt[i] = c;
}

int
th_fk(int t)
{
	return t == MGDK_flt ? 1 : t == MGDK_dbl ? 2 : 0;
}

bool
th_type_ok(int t)
{
	return jk_type_ok(t) || t == MGDK_flt || t == MGDK_dbl;
}

// the shared driver: mode 0 theta (mask), 1 band (c1, c2 as the column's
// type, already checked non-nil and non-empty)
int
th_run(const char *fn, mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, ThArgs t,
       const void *c1, const void *c2)
{
	*r1p = nullptr;
	if (r2p)
		*r2p = nullptr;
	Held held;
	JSide L, R;
	mgdk_bat *lb, *rb;
	if (jside(fn, l, sl, &L, held, &lb) < 0 || jside(fn, r, sr, &R, held, &rb) < 0)
		return -1;
	const int tt = atomtype(lb->ttype);
	if (tt != atomtype(rb->ttype)) {
		seterr("%s: inputs not compatible.\n", fn);
		return -1;
	}
	if (!th_type_ok(lb->ttype) || !th_type_ok(rb->ttype)) {
		seterr("%s: type %s is not on the device path", fn, atomname(lb->ttype));
		return -1;
	}
	// void with a nil sequence: every value nil (thetajoin :3738-3763)
	const bool lallnil = lb->ttype == MGDK_void && lb->tseqbase == MGDK_OID_NIL;
	const bool rallnil = rb->ttype == MGDK_void && rb->tseqbase == MGDK_OID_NIL;
	ProfScope prof("thetajoin");
	hipStream_t st = stream();
	auto result = [&](BUN n, mgdk_bat **a, mgdk_bat **b) -> bool {
		*a = newbat(0, MGDK_oid, n);
		*b = newbat(0, MGDK_oid, n);
		if (*a == nullptr || *b == nullptr) {
			mgdk_BBPunfix(*a);
			mgdk_BBPunfix(*b);
			return false;
		}
		return true;
	};
	auto finish = [&](mgdk_bat *a, mgdk_bat *b, BUN n, bool onekey) {
		a->count = b->count = n;
		a->tsorted = a->tnonil = b->tnonil = 1;
		a->tkey = onekey || n <= 1;
		a->trevsorted = n <= 1;
		b->tsorted = b->trevsorted = b->tkey = n <= 1;
		*r1p = a;
		if (r2p)
			*r2p = b;
		else
			mgdk_BBPunfix(b);
	};
	if (L.n == 0 || R.n == 0 || ((lallnil || rallnil) && (t.mode == 1 || !t.nil_matches))) {
		mgdk_bat *a, *b;
		if (!result(0, &a, &b))
			return -1;
		finish(a, b, 0, true);
		return 0;
	}
	const int fk = th_fk(tt);
	if (t.mode == 1 && fk) {
		// bandjoin over flt / dbl: the reference's expression pair by pair
		DevBuf cnt(L.n * 4 + 4), off(L.n * 8 + 8);
		if (!cnt.p || !off.p)
			return -1;
		const dim3 g((unsigned) ((L.n + 255) / 256));
		if (fk == 1)
			hipLaunchKernelGGL(k_band_fp<float>, g, dim3(256), 0, st, L, R, *(const float *) c1,
					   *(const float *) c2, t.linc, t.hinc, 0, cnt.as<uint32_t>(), (const uint64_t *) nullptr,
					   (oid *) nullptr, (oid *) nullptr);
		else
			hipLaunchKernelGGL(k_band_fp<double>, g, dim3(256), 0, st, L, R, *(const double *) c1,
					   *(const double *) c2, t.linc, t.hinc, 0, cnt.as<uint32_t>(), (const uint64_t *) nullptr,
					   (oid *) nullptr, (oid *) nullptr);
		uint64_t tot = 0;
		if (exclusive_scan(cnt.as<uint32_t>(), off.as<uint64_t>(), L.n, &tot) != 0)
			return -1;
		mgdk_bat *a, *b;
		if (!result(tot, &a, &b))
			return -1;
		if (tot) {
			if (fk == 1)
				hipLaunchKernelGGL(k_band_fp<float>, g, dim3(256), 0, st, L, R, *(const float *) c1,
						   *(const float *) c2, t.linc, t.hinc, 1, (uint32_t *) nullptr,
						   off.as<uint64_t>(), (oid *) a->theap, (oid *) b->theap);
			else
				hipLaunchKernelGGL(k_band_fp<double>, g, dim3(256), 0, st, L, R, *(const double *) c1,
						   *(const double *) c2, t.linc, t.hinc, 1, (uint32_t *) nullptr,
						   off.as<uint64_t>(), (oid *) a->theap, (oid *) b->theap);
		}
		if (!sync()) {
			mgdk_BBPunfix(a);
			mgdk_BBPunfix(b);
			return -1;
		}
		finish(a, b, tot, tot <= L.n && false);
		return 0;
	}
	if (R.n >= 0xffffffffull || L.n >= 0xffffffffull) {
		seterr("%s: more than 2^32-1 candidates on the device path", fn);
		return -1;
	}
	// the right values sorted, their candidate index along
	mgdk_bat *kb = held.keep(newbat(0, MGDK_lng, R.n));
	if (kb == nullptr)
		return -1;
	hipLaunchKernelGGL(k_th_rkeys, dim3(grid_for(R.n, 256 * 8, 8192)), dim3(256), 0, st, R, fk, (int64_t *) kb->theap);
	kb->count = R.n;
	kb->tsorted = kb->trevsorted = kb->tkey = 0;
	kb->tnonil = 0;
	mgdk_bat *sv = nullptr, *so = nullptr;
	if (mgdk_BATsort(&sv, &so, nullptr, kb, nullptr, nullptr, false, false, true) != 0)
		return -1;
	held.keep(sv);
	held.keep(so);
	const oid *sidx = so->ttype == MGDK_void ? nullptr : (const oid *) so->theap;
	DevBuf rg(L.n * 16 + 16), cnt(L.n * 4 + 4), off(L.n * 8 + 8);
	if (!rg.p || !cnt.p || !off.p)
		return -1;
	hipLaunchKernelGGL(k_th_ranges, dim3(grid_for(L.n, 256 * 4, 8192)), dim3(256), 0, st, L, fk,
			   (const int64_t *) sv->theap, R.n, t, rg.as<uint32_t>(), cnt.as<uint32_t>());
	uint64_t tot = 0;
	if (exclusive_scan(cnt.as<uint32_t>(), off.as<uint64_t>(), L.n, &tot) != 0)
		return -1;
	int rbits = 1;
	while (rbits < 63 && (R.n >> rbits))
		rbits++;
	if (sidx && (L.n >> (63 - rbits))) {
		seterr("%s: result too large for the device path", fn);
		return -1;
	}
	mgdk_bat *a, *b;
	if (!result(tot, &a, &b))
		return -1;
	if (tot) {
		if (sidx == nullptr) {
			hipLaunchKernelGGL(k_th_emit, dim3(grid_for(L.n, 256 * 4, 8192)), dim3(256), 0, st, L, R,
					   (const uint32_t *) rg.p, off.as<uint64_t>(), (const oid *) nullptr, rbits,
					   (int64_t *) nullptr, (oid *) a->theap, (oid *) b->theap);
		} else {
			mgdk_bat *pk = held.keep(newbat(0, MGDK_lng, tot));
			if (pk == nullptr) {
				mgdk_BBPunfix(a);
				mgdk_BBPunfix(b);
				return -1;
			}
			hipLaunchKernelGGL(k_th_emit, dim3(grid_for(L.n, 256 * 4, 8192)), dim3(256), 0, st, L, R,
					   (const uint32_t *) rg.p, off.as<uint64_t>(), sidx, rbits, (int64_t *) pk->theap,
					   (oid *) nullptr, (oid *) nullptr);
			pk->count = tot;
			pk->tsorted = pk->trevsorted = pk->tkey = 0;
			pk->tnonil = 1;
			mgdk_bat *ps = nullptr;
			if (mgdk_BATsort(&ps, nullptr, nullptr, pk, nullptr, nullptr, false, false, false) != 0) {
				mgdk_BBPunfix(a);
				mgdk_BBPunfix(b);
				return -1;
			}
			held.keep(ps);
			hipLaunchKernelGGL(k_th_decode, dim3(grid_for(tot, 256 * 8, 16384)), dim3(256), 0, st,
					   (const int64_t *) ps->theap, tot, rbits, L, R, (oid *) a->theap, (oid *) b->theap);
		}
	}
	if (!sync()) {
		mgdk_BBPunfix(a);
		mgdk_BBPunfix(b);
		return -1;
	}
	finish(a, b, tot, false);
	return 0;
}

// bandjoin's trivial cases (gdk_join.c:4667-4729): a nil bound, -c1 > c2,
// or -c1 == c2 with an open end
template <typename T>
bool
band_empty(const void *c1p, const void *c2p, bool linc, bool hinc)
{
	const T c1 = *(const T *) c1p, c2 = *(const T *) c2p;
	if (is_nil(c1) || is_nil(c2))
		return true;
	return -c1 > c2 || ((!hinc || !linc) && -c1 == c2);
}

// ---- BATrangejoin (gdk_join.c:5422, rangejoin :5067) ---------------------
// Not anti, not symmetric, l sorted or reverse sorted: per right candidate
// (one lane each) the l positions of [rl, rh] by binary search
// (SORTfndfirst / SORTfndlast), mapped to the left candidates in between;
// right-major output placed by a scan of the counts.  Otherwise the nested
// loop (left-major, BETWEEN's three-valued logic), brute force with the
// right bounds streamed through LDS.  The result properties are the
// reference's extra scan over the result (k_oid_props).

// first position p of l (asc: value >= v / > v with last; desc: <= v / < v)
__device__ __forceinline__ BUN
rj_fnd(const JSide &l, int fk, BUN cnt, bool rev, int64_t v, bool last)
{
	BUN a = 0, b = cnt;
	while (a < b) {
		const BUN m = a + (b - a) / 2;
		const int64_t x = th_key(l, fk, m);
		const bool before = rev ? (last ? x >= v : x > v) : (last ? x <= v : x < v);
		if (before)
			a = m + 1;
		else
			b = m;
	}
	return a;
}

// index of the first candidate >= o (canditer_search(.., next = true))
__device__ __forceinline__ BUN
cand_lower(const JSide &c, oid o)
{
	if (c.dense)
		return o <= c.seq ? 0 : (o - c.seq < c.n ? o - c.seq : c.n);
	BUN a = 0, b = c.n;
	while (a < b) {
		const BUN m = a + (b - a) / 2;
		if (c.oids[m] < o)
			a = m + 1;
		else
			b = m;
	}
	return a;
}

__global__ __launch_bounds__(256) void
k_rj_sorted(JSide L, BUN lcnt, JSide RL, JSide RH, int fk, bool rev, bool linc, bool hinc, uint32_t *rg,
	    uint32_t *cnt)
{
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < RL.n; j += (BUN) gridDim.x * blockDim.x) {
		const oid ro = js_oid(RL, j);
		const int64_t vlo = th_key(RL, fk, ro - RL.hseq), vhi = th_key(RH, fk, ro - RH.hseq);
		BUN cl = 0, ch = 0;
		if (vlo != INT64_MIN && vhi != INT64_MIN) {
			BUN low, high;
			if (!rev) {
				low = rj_fnd(L, fk, lcnt, false, vlo, !linc);
				high = rj_fnd(L, fk, lcnt, false, vhi, hinc);
			} else {
				low = rj_fnd(L, fk, lcnt, true, vhi, !hinc);
				high = rj_fnd(L, fk, lcnt, true, vlo, linc);
			}
			if (high > low) {
				cl = cand_lower(L, low + L.hseq);
				ch = cand_lower(L, high + L.hseq);
			}
		}
		rg[2 * j] = (uint32_t) cl;
		rg[2 * j + 1] = (uint32_t) (ch > cl ? ch : cl);
		cnt[j] = (uint32_t) (ch > cl ? ch - cl : 0);
	}
}

__global__ __launch_bounds__(256) void
k_rj_sorted_emit(JSide L, JSide RL, const uint32_t *rg, const uint64_t *off, oid *r1, oid *r2)
{
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < RL.n; j += (BUN) gridDim.x * blockDim.x) {
		const oid ro = js_oid(RL, j);
		BUN o = off[j];
		for (BUN q = rg[2 * j]; q < rg[2 * j + 1]; q++, o++) {
			r1[o] = js_oid(L, q);
			r2[o] = ro;
		}
	}
}

// l unsorted with an order index (gdk_join.c:5137-5273): the bounds are
// found on the index (ORDERfndfirst / ORDERfndlast, gdk_search.c:423) and
// the index entries in between that are left candidates are emitted in the
// index's order.  The reference searches the index with offset 0
// (vals[ord[i]]), right only for hseqbase 0; positions here are ord[i] -
// hseqbase.
__device__ __forceinline__ BUN
rj_ofnd(const JSide &l, int fk, const oid *ord, BUN cnt, int64_t v, bool last)
{
	BUN a = 0, b = cnt;
	while (a < b) {
		const BUN m = a + (b - a) / 2;
		const int64_t x = th_key(l, fk, ord[m] - l.hseq);
		if (last ? x <= v : x < v)
			a = m + 1;
		else
			b = m;
	}
	return a;
}

__device__ __forceinline__ bool
js_contains(const JSide &c, oid o)
{
	if (c.dense)
		return o >= c.seq && o - c.seq < c.n;
	BUN a = 0, b = c.n;
	while (a < b) {
		const BUN m = a + (b - a) / 2;
		if (c.oids[m] < o)
			a = m + 1;
		else
			b = m;
	}
	return a < c.n && c.oids[a] == o;
}

// pass 0: per right candidate the index range and the number of left
// candidates in it; pass 1: write them
__global__ __launch_bounds__(256) void
k_rj_oidx(JSide L, BUN lcnt, const oid *ord, JSide RL, JSide RH, int fk, bool linc, bool hinc, int pass,
	  uint32_t *rg, uint32_t *cnt, const uint64_t *off, oid *r1, oid *r2)
{
	for (BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x; j < RL.n; j += (BUN) gridDim.x * blockDim.x) {
		const oid ro = js_oid(RL, j);
		if (pass) {
			BUN o = off[j];
			for (BUN q = rg[2 * j]; q < rg[2 * j + 1]; q++) {
				const oid lo = ord[q];
				if (js_contains(L, lo)) {
					r1[o] = lo;
					r2[o] = ro;
					o++;
				}
			}
			continue;
		}
		const int64_t vlo = th_key(RL, fk, ro - RL.hseq), vhi = th_key(RH, fk, ro - RH.hseq);
		BUN low = 0, high = 0;
		uint32_t c = 0;
		if (vlo != INT64_MIN && vhi != INT64_MIN) {
			low = rj_ofnd(L, fk, ord, lcnt, vlo, !linc);
			high = rj_ofnd(L, fk, ord, lcnt, vhi, hinc);
			for (BUN q = low; q < high; q++)
				c += js_contains(L, ord[q]);
		}
		rg[2 * j] = (uint32_t) low;
		rg[2 * j + 1] = (uint32_t) (high > low ? high : low);
		cnt[j] = c;
	}
}

// BETWEEN (gdk_join.c:5040-5064): 1 true, 0 false, -1 nil
__device__ __forceinline__ int
rj_between3(int64_t v, int64_t lo, bool linc, int64_t hi, bool hinc)
{
	const int g = lo == INT64_MIN ? -1 : (lo < v || (linc && v == lo));
	const int l = hi == INT64_MIN ? -1 : (v < hi || (hinc && v == hi));
	if (g == 0 || l == 0)
		return 0;
	return g < 0 || l < 0 ? -1 : 1;
}

// the nested loop: pass 0 counts per left candidate, pass 1 writes
__global__ __launch_bounds__(256) void
k_rj_nested(JSide L, JSide RL, JSide RH, int fk, bool linc, bool hinc, bool anti, bool symmetric, int pass,
	    uint32_t *cnt, const uint64_t *off, oid *r1, oid *r2)
{
	__shared__ int64_t slo[1024], shi[1024];
	__shared__ oid so[1024];
	const BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	const bool live = i < L.n;
	oid lo = 0;
	int64_t v = INT64_MIN;
	if (live) {
		lo = js_oid(L, i);
		v = th_key(L, fk, lo - L.hseq);
	}
	const bool vn = v == INT64_MIN && L.base != nullptr;
	uint32_t c = 0;
	BUN o = pass && live ? off[i] : 0;
	for (BUN c0 = 0; c0 < RL.n; c0 += 1024) {
		__syncthreads();
		for (unsigned q = threadIdx.x; q < 1024; q += blockDim.x) {
			const BUN k = c0 + q;
			if (k < RL.n) {
				const oid ro = js_oid(RL, k);
				slo[q] = th_key(RL, fk, ro - RL.hseq);
				shi[q] = th_key(RH, fk, ro - RH.hseq);
				so[q] = ro;
			}
		}
		__syncthreads();
		if (!live || vn)
			continue;
		const unsigned m = (unsigned) min((BUN) 1024, RL.n - c0);
		for (unsigned q = 0; q < m; q++) {
			int r = rj_between3(v, slo[q], linc, shi[q], hinc);
			if (symmetric) {
				const int r2v = rj_between3(v, shi[q], hinc, slo[q], linc);
				r = r == 1 || r2v == 1 ? 1 : (r < 0 || r2v < 0 ? -1 : 0);
			}
			if (anti)
				r = r < 0 ? -1 : !r;
			if (r != 1)
				continue;
			if (pass) {
				r1[o] = lo;
				r2[o] = so[q];
				o++;
			} else {
				c++;
			}
		}
	}
	if (live && !pass)
		cnt[i] = c;
}

// the reference's property scan of an oid result: bit 0 equal neighbours,
// 1 an ascent, 2 a descent, 3 an ascent by more than one
__global__ __launch_bounds__(256) void
k_oid_props(const oid *d, BUN n, uint32_t *flags)
{
	uint32_t f = 0;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += (BUN) gridDim.x * blockDim.x) {
		const oid a = d[i - 1], b = d[i];
		if (a == b)
			f |= 1;
		else if (a < b)
			f |= 2 | (a + 1 != b ? 8u : 0u);
		else
			f |= 4;
	}
	f = block_reduce(f, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0 && f)
		atomicOr(flags, f);
}

// r's properties from k_oid_props' bits (gdk_join.c:5351-5410)
void
rj_props(mgdk_bat *r, uint32_t f, oid first)
{
	r->tkey = !(f & 1) && !(f & 4);
	r->tsorted = !(f & 4);
	r->trevsorted = !(f & 2);
	r->tnil = 0;
	r->tnonil = 1;
	r->tseqbase = (!(f & 1) && !(f & 4) && !(f & 8)) ? (r->count ? first : 0) : MGDK_OID_NIL;
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
	return jk_run("BATsemijoin", l, r, sl, sr, nil_matches, false, max_one, 0, r1p, r2p);
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
	return jk_run("BATouterjoin", l, r, sl, sr, nil_matches, false, match_one, 3, r1p, r2p, nullptr, match_one);
}

// BATmarkjoin (gdk_join.c:4367): leftjoin with nil_on_miss, semi when r2p is
// NULL
extern "C" int
mgdk_BATmarkjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat **r3p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl,
		 mgdk_bat *sr, mgdk_BUN estimate)
{
	(void) estimate;
	if (r3p == nullptr) {
		seterr("BATmarkjoin: the mark output must not be NULL");
		return -1;
	}
	return jk_run("BATmarkjoin", l, r, sl, sr, false, false, false, 4, r1p, r2p, r3p);
}

// BATthetajoin (gdk_join.c:4409): op JOIN_EQ 0 (BATjoin), JOIN_LT -1,
// JOIN_LE -2, JOIN_GT 1, JOIN_GE 2, JOIN_NE -3
extern "C" int
mgdk_BATthetajoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, int op,
		  bool nil_matches, mgdk_BUN estimate)
{
	ThArgs t{};
	switch (op) {
	case 0:
		return mgdk_BATjoin(r1p, r2p, l, r, sl, sr, nil_matches, estimate);
	case -3: t.mask = 2 | 4; break;
	case -1: t.mask = 2; break;
	case -2: t.mask = 2 | 1; break;
	case 1: t.mask = 4; break;
	case 2: t.mask = 4 | 1; break;
	default:
		seterr("unknown operator %d.\n", op);
		return -1;
	}
	if (l == nullptr || r == nullptr) {
		seterr("BATthetajoin: inputs must not be NULL");
		return -1;
	}
	t.mode = 0;
	t.nil_matches = nil_matches;
	return th_run("BATthetajoin", r1p, r2p, l, r, sl, sr, t, nullptr, nullptr);
}

// BATbandjoin (gdk_join.c:4626): l within [r - c1, r + c2] (linc / hinc
// include the ends); c1, c2 point at values of the columns' type
extern "C" int
mgdk_BATbandjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, const void *c1,
		 const void *c2, bool linc, bool hinc, mgdk_BUN estimate)
{
	(void) estimate;
	*r1p = nullptr;
	if (r2p)
		*r2p = nullptr;
	if (l == nullptr || r == nullptr || c1 == nullptr || c2 == nullptr) {
		seterr("BATbandjoin: inputs must not be NULL");
		return -1;
	}
	if (atomtype(l->ttype) != atomtype(r->ttype)) {
		seterr("BATbandjoin: inputs not compatible.\n");
		return -1;
	}
	const int bt = basetype(l->ttype);
	bool empty;
	ThArgs t{};
	t.mode = 1;
	t.linc = linc;
	t.hinc = hinc;
	switch (bt) {
	case MGDK_bte: empty = band_empty<int8_t>(c1, c2, linc, hinc); t.c1 = *(const int8_t *) c1; t.c2 = *(const int8_t *) c2; break;
	case MGDK_sht: empty = band_empty<int16_t>(c1, c2, linc, hinc); t.c1 = *(const int16_t *) c1; t.c2 = *(const int16_t *) c2; break;
	case MGDK_int: empty = band_empty<int32_t>(c1, c2, linc, hinc); t.c1 = *(const int32_t *) c1; t.c2 = *(const int32_t *) c2; break;
	case MGDK_lng: empty = band_empty<int64_t>(c1, c2, linc, hinc); t.c1 = *(const int64_t *) c1; t.c2 = *(const int64_t *) c2; break;
	case MGDK_flt: empty = band_empty<float>(c1, c2, linc, hinc); break;
	case MGDK_dbl: empty = band_empty<double>(c1, c2, linc, hinc); break;
	default:
		seterr("unsupported type\n");
		return -1;
	}
	if (empty) {
		mgdk_bat *a = newbat(0, MGDK_oid, 0), *b = newbat(0, MGDK_oid, 0);
		if (a == nullptr || b == nullptr) {
			mgdk_BBPunfix(a);
			mgdk_BBPunfix(b);
			return -1;
		}
		a->tsorted = a->trevsorted = a->tkey = a->tnonil = 1;
		b->tsorted = b->trevsorted = b->tkey = b->tnonil = 1;
		*r1p = a;
		if (r2p)
			*r2p = b;
		else
			mgdk_BBPunfix(b);
		return 0;
	}
	return th_run("BATbandjoin", r1p, r2p, l, r, sl, sr, t, c1, c2);
}

// BATrangejoin (gdk_join.c:5422): l within [rl, rh] of each right candidate
extern "C" int
mgdk_BATrangejoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *rl, mgdk_bat *rh, mgdk_bat *sl, mgdk_bat *sr,
		  bool linc, bool hinc, bool anti, bool symmetric, mgdk_BUN estimate)
{
	(void) estimate;
	*r1p = nullptr;
	if (r2p)
		*r2p = nullptr;
	if (l == nullptr || rl == nullptr || rh == nullptr) {
		seterr("BATrangejoin: inputs must not be NULL");
		return -1;
	}
	if (atomtype(l->ttype) != atomtype(rl->ttype) || atomtype(l->ttype) != atomtype(rh->ttype)) {
		seterr("BATrangejoin: inputs not compatible.\n");
		return -1;
	}
	if (rl->count != rh->count || rl->hseqbase != rh->hseqbase) {
		seterr("BATrangejoin: right inputs not aligned.\n");
		return -1;
	}
	Held held;
	JSide L, RL, RH;
	mgdk_bat *lb, *rlb, *rhb;
	if (jside("BATrangejoin", l, sl, &L, held, &lb) < 0 || jside("BATrangejoin", rl, sr, &RL, held, &rlb) < 0 ||
	    jside("BATrangejoin", rh, sr, &RH, held, &rhb) < 0)
		return -1;
	if (!th_type_ok(lb->ttype) || !th_type_ok(rlb->ttype) || !th_type_ok(rhb->ttype)) {
		seterr("BATrangejoin: type %s is not on the device path", atomname(lb->ttype));
		return -1;
	}
	const bool lnilall = lb->ttype == MGDK_void && lb->tseqbase == MGDK_OID_NIL;
	const bool rlnil = rlb->ttype == MGDK_void && rlb->tseqbase == MGDK_OID_NIL;
	const bool rhnil = rhb->ttype == MGDK_void && rhb->tseqbase == MGDK_OID_NIL;
	hipStream_t st = stream();
	ProfScope prof("rangejoin");
	const int fk = th_fk(atomtype(lb->ttype));
	mgdk_bat *a = nullptr, *b = nullptr;
	uint64_t tot = 0;
	auto alloc = [&](BUN n) {
		a = newbat(0, MGDK_oid, n);
		b = newbat(0, MGDK_oid, n);
		if (a == nullptr || b == nullptr) {
			mgdk_BBPunfix(a);
			mgdk_BBPunfix(b);
			return false;
		}
		return true;
	};
	if (L.n == 0 || RL.n == 0 || lnilall || (rlnil && rhnil) || ((rlnil || rhnil) && !anti)) {
		if (!alloc(0))
			return -1;
	} else if (rlnil || rhnil) {
		// anti with a nil bound column: thetajoin l > rh (or l < rl), :5448-5460
		ThArgs t{};
		t.mode = 0;
		t.mask = rlnil ? 4 : 2;
		t.nil_matches = false;
		return th_run("BATrangejoin", r1p, r2p, l, rlnil ? rh : rl, sl, sr, t, nullptr, nullptr);
	} else if (RL.n >= 0xffffffffull || L.n >= 0xffffffffull) {
		seterr("BATrangejoin: more than 2^32-1 candidates on the device path");
		return -1;
	} else {
		// the reference computes both orders first (:5071-5075)
		bool asc = false, desc = false;
		if (!anti && !symmetric) {
			asc = mgdk_BATordered(lb);
			desc = mgdk_BATordered_rev(lb);
		}
		// an unsorted l's order index (gdk_join.c:5137-5156)
		size_t ooff = 0;
		Heap *oh = !anti && !symmetric && !asc && !desc && lb == l && lb->count < 0xffffffffull ?
			oidx_get(l, nullptr, OIDX_OWN, &ooff) : nullptr;
		if (oh) {
			DevBuf rg(RL.n * 8 + 8), cnt(RL.n * 4 + 4), off(RL.n * 8 + 8);
			const dim3 grd(grid_for(RL.n, 256 * 4, 8192));
			const oid *ord = (const oid *) ((const char *) oh->base + ooff);
			bool okk = rg.p && cnt.p && off.p;
			if (okk) {
				hipLaunchKernelGGL(k_rj_oidx, grd, dim3(256), 0, st, L, lb->count, ord, RL, RH, fk, linc, hinc, 0,
						   rg.as<uint32_t>(), cnt.as<uint32_t>(), (const uint64_t *) nullptr, (oid *) nullptr,
						   (oid *) nullptr);
				okk = exclusive_scan(cnt.as<uint32_t>(), off.as<uint64_t>(), RL.n, &tot) == 0 && alloc(tot);
			}
			if (okk && tot)
				hipLaunchKernelGGL(k_rj_oidx, grd, dim3(256), 0, st, L, lb->count, ord, RL, RH, fk, linc, hinc, 1,
						   rg.as<uint32_t>(), cnt.as<uint32_t>(), off.as<uint64_t>(), (oid *) a->theap,
						   (oid *) b->theap);
			// the index stays referenced until the stream has drained
			const bool drained = sync_data();
			heap_decref(oh);
			if (!okk || !drained) {
				if (okk) {
					mgdk_BBPunfix(a);
					mgdk_BBPunfix(b);
				}
				return -1;
			}
		} else if (asc || desc) {
			DevBuf rg(RL.n * 8 + 8), cnt(RL.n * 4 + 4), off(RL.n * 8 + 8);
			if (!rg.p || !cnt.p || !off.p)
				return -1;
			hipLaunchKernelGGL(k_rj_sorted, dim3(grid_for(RL.n, 256 * 4, 8192)), dim3(256), 0, st, L, lb->count, RL,
					   RH, fk, !asc, linc, hinc, rg.as<uint32_t>(), cnt.as<uint32_t>());
			if (exclusive_scan(cnt.as<uint32_t>(), off.as<uint64_t>(), RL.n, &tot) != 0 || !alloc(tot))
				return -1;
			if (tot)
				hipLaunchKernelGGL(k_rj_sorted_emit, dim3(grid_for(RL.n, 256 * 4, 8192)), dim3(256), 0, st, L, RL,
						   (const uint32_t *) rg.p, off.as<uint64_t>(), (oid *) a->theap, (oid *) b->theap);
		} else {
			DevBuf cnt(L.n * 4 + 4), off(L.n * 8 + 8);
			if (!cnt.p || !off.p)
				return -1;
			const dim3 g((unsigned) ((L.n + 255) / 256));
			hipLaunchKernelGGL(k_rj_nested, g, dim3(256), 0, st, L, RL, RH, fk, linc, hinc, anti, symmetric, 0,
					   cnt.as<uint32_t>(), (const uint64_t *) nullptr, (oid *) nullptr, (oid *) nullptr);
			if (exclusive_scan(cnt.as<uint32_t>(), off.as<uint64_t>(), L.n, &tot) != 0 || !alloc(tot))
				return -1;
			if (tot)
				hipLaunchKernelGGL(k_rj_nested, g, dim3(256), 0, st, L, RL, RH, fk, linc, hinc, anti, symmetric,
						   1, (uint32_t *) nullptr, off.as<uint64_t>(), (oid *) a->theap, (oid *) b->theap);
		}
	}
	DevBuf fl(16);
	uint32_t *h = (uint32_t *) pinned(32);
	if (!fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 16, st), "memset")) {
		mgdk_BBPunfix(a);
		mgdk_BBPunfix(b);
		return -1;
	}
	if (tot > 1) {
		hipLaunchKernelGGL(k_oid_props, dim3(grid_for(tot, 256 * 8, 4096)), dim3(256), 0, st, (const oid *) a->theap,
				   tot, fl.as<uint32_t>());
		hipLaunchKernelGGL(k_oid_props, dim3(grid_for(tot, 256 * 8, 4096)), dim3(256), 0, st, (const oid *) b->theap,
				   tot, fl.as<uint32_t>() + 1);
	}
	bool ok = hip_ok(hipMemcpyAsync(h, fl.p, 8, hipMemcpyDeviceToHost, st), "memcpy");
	if (ok && tot)
		ok = hip_ok(hipMemcpyAsync(h + 2, a->theap, 8, hipMemcpyDeviceToHost, st), "memcpy") &&
		     hip_ok(hipMemcpyAsync(h + 4, b->theap, 8, hipMemcpyDeviceToHost, st), "memcpy");
	if (!ok || !sync()) {
		mgdk_BBPunfix(a);
		mgdk_BBPunfix(b);
		return -1;
	}
	oid f1 = 0, f2 = 0;
	memcpy(&f1, h + 2, 8);
	memcpy(&f2, h + 4, 8);
	a->count = b->count = tot;
	rj_props(a, h[0], f1);
	rj_props(b, h[1], f2);
	*r1p = a;
	if (r2p)
		*r2p = b;
	else
		mgdk_BBPunfix(b);
	return 0;
}

// ---- cross products (gdk/gdk_cross.c) ---------------------------------------

namespace {

__device__ __forceinline__ oid
cross_oid(bool dense, oid seq, const oid *oids, BUN i)
{
	return dense ? seq + i : oids[i];
}

// pair p = i * n2 + j of the l-major product: r1[p] = left candidate i,
// r2[p] = right candidate j (BATcrossci's two loops, gdk_cross.c:95-118).
// 32-bit index arithmetic when the product fits
template <typename I>
__global__ void
k_cross(oid *__restrict__ r1, oid *__restrict__ r2, bool d1, oid s1, const oid *o1, bool d2, oid s2, const oid *o2,
	I n2, I total)
{
	for (I p = blockIdx.x * (I) blockDim.x + threadIdx.x; p < total; p += (I) gridDim.x * blockDim.x) {
		const I i = p / n2, j = p - i * n2;
		r1[p] = cross_oid(d1, s1, o1, i);
		if (r2)
			r2[p] = cross_oid(d2, s2, o2, j);
	}
}

// a void column of n nil oids (BATtseqbase(bn, oid_nil), gdk_bat.c:2167)
mgdk_bat *
nil_void(BUN n)
{
	mgdk_bat *b = mgdk_BATdense(0, 0, 0);
	if (b == nullptr)
		return nullptr;
	b->tseqbase = MGDK_OID_NIL;
	b->count = n;
	b->tsorted = b->trevsorted = 1;
	b->tkey = n <= 1;
	b->tnonil = n == 0;
	b->tnil = n > 0;
	return b;
}

// BATcrossci (gdk_cross.c:22): the special cases return candidate slices and
// constants, the general case the l-major pairs
int
crossci(const Cand &c1, const Cand &c2, mgdk_bat **r1p, mgdk_bat **r2p)
{
	Own a, b;
	if (c1.n == 0 || c2.n == 0) {
		a.b = mgdk_BATdense(0, 0, 0);
		if (a.b == nullptr || (r2p && (b.b = mgdk_BATdense(0, 0, 0)) == nullptr))
			return -1;
	} else if (c2.n == 1) {
		if ((a.b = cand_slice(c1)) == nullptr)
			return -1;
		if (r2p) {
			const oid v = c2.first;
			b.b = c1.n == 1 ? cand_slice(c2) : mgdk_BATconstant(0, MGDK_oid, &v, c1.n);
			if (b.b == nullptr)
				return -1;
		}
	} else if (c1.n == 1) {
		const oid v = c1.first;
		if ((a.b = mgdk_BATconstant(0, MGDK_oid, &v, c2.n)) == nullptr ||
		    (r2p && (b.b = cand_slice(c2)) == nullptr))
			return -1;
	} else {
		if (c1.n > (BUN) MGDK_BUN_NONE / c2.n) {
			seterr("BATsubcross: result too large");
			return -1;
		}
		const BUN total = c1.n * c2.n;
		if ((a.b = newbat(0, MGDK_oid, total)) == nullptr || (r2p && (b.b = newbat(0, MGDK_oid, total)) == nullptr))
			return -1;
		ProfScope prof("crossproduct");
		oid *p1 = (oid *) a.b->theap, *p2 = r2p ? (oid *) b.b->theap : nullptr;
		const unsigned grid = grid_for(total, BLOCK * 8, 256u * 64u);
		if (total <= 0xffffffffu)
			hipLaunchKernelGGL((k_cross<uint32_t>), dim3(grid), dim3(BLOCK), 0, stream(), p1, p2, c1.dense, c1.seq,
					   c1.oids, c2.dense, c2.seq, c2.oids, (uint32_t) c2.n, (uint32_t) total);
		else
			hipLaunchKernelGGL((k_cross<uint64_t>), dim3(grid), dim3(BLOCK), 0, stream(), p1, p2, c1.dense, c1.seq,
					   c1.oids, c2.dense, c2.seq, c2.oids, (uint64_t) c2.n, (uint64_t) total);
		if (!hip_ok(hipGetLastError(), "k_cross") || !sync())
			return -1;
		a.b->count = total;
		a.b->tsorted = a.b->tnonil = 1;
		a.b->tnil = 0;
		a.b->trevsorted = 0;     // c1.n > 1
		a.b->tkey = 0;           // c2.n > 1
		if (r2p) {
			b.b->count = total;
			b.b->tnonil = 1;
			b.b->tnil = b.b->tsorted = b.b->trevsorted = b.b->tkey = 0;
		}
	}
	*r1p = a.release();
	if (r2p)
		*r2p = b.release();
	return 0;
}

// the candidates of b (complex lists unmasked first, as the joins do)
int
cross_cands(mgdk_bat *b, mgdk_bat *s, Cand *ci, Held &held)
{
	if (b == nullptr) {
		seterr("BATsubcross: inputs must not be NULL");
		return -1;
	}
	if (s && is_complex_cand(s) && (s = held.keep(unmask_cand(s))) == nullptr)
		return -1;
	return cand_init(ci, b, s);
}

}  // namespace

// BATsubcross (gdk_cross.c:138): every (left, right) candidate pair, left-major;
// max_one: at most one right candidate when there is a left one
extern "C" int
mgdk_BATsubcross(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, bool max_one)
{
	*r1p = nullptr;
	if (r2p)
		*r2p = nullptr;
	Held held;
	Cand c1, c2;
	if (cross_cands(l, sl, &c1, held) < 0 || cross_cands(r, sr, &c2, held) < 0)
		return -1;
	if (max_one && c1.n > 0 && c2.n > 1) {
		seterr("more than one match");
		return -1;
	}
	return crossci(c1, c2, r1p, r2p);
}

// BAToutercross (gdk_cross.c:153): the left outer form; no right candidate
// pairs every left one with nil
extern "C" int
mgdk_BAToutercross(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr, bool max_one)
{
	*r1p = nullptr;
	if (r2p)
		*r2p = nullptr;
	Held held;
	Cand c1, c2;
	if (cross_cands(l, sl, &c1, held) < 0 || cross_cands(r, sr, &c2, held) < 0)
		return -1;
	if (max_one && c1.n > 0 && c2.n > 1) {
		seterr("more than one match");
		return -1;
	}
	if (c1.n == 0 || c2.n == 0) {
		Own a, b;
		a.b = c1.n == 0 ? nil_void(0) : cand_slice(c1);
		if (a.b == nullptr || (r2p && (b.b = nil_void(c1.n)) == nullptr))
			return -1;
		*r1p = a.release();
		if (r2p)
			*r2p = b.release();
		return 0;
	}
	return crossci(c1, c2, r1p, r2p);
}
