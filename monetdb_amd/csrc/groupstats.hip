// groupstats.hip -- the statistics of gdk_aggr.c on the MI355X:
//   BATgroupstdev_sample / _population, BATgroupvariance_sample /
//   _population (dogroupstdev, gdk_aggr.c:4612-4806), BATgroupcovariance_
//   sample / _population (dogroupcovariance :4851-5011), BATgroupcorrelation
//   (:5057-5202); the whole-column BATcalcstdev_* / BATcalcvariance_*
//   (calcvariance :4276-4380), BATcalccovariance_* (calccovariance
//   :4404-4476) and BATcalccorrelation (:4503-4559); the quantiles
//   BATgroupmedian / BATgroupquantile and their _avg forms
//   (doBATgroupquantile :3881-4252).
//
// The moments are Welford updates (AGGR_STDEV :4561, AGGR_COVARIANCE :4808,
// AGGR_CORRELATION :5013 and the _SINGLE loops): each step's rounding
// depends on every earlier step, so a result is a function of the values in
// CANDIDATE ORDER.  The device keeps that order: the rows are grouped by a
// stable counting sort (group_rows, aggr.hip) and one lane replays one
// group's recurrence -- all groups at once -- with the reference's operations
// in the reference's order and no contraction into fused multiply-adds (the
// pragma below), so the results are the reference's bit for bit.  A group is
// a chain of dependent divisions: the device wins with many groups; a single
// group (the BATcalc* forms) runs at one lane's speed.
//
// The quantiles follow the reference's plan: sort g, sub-sort b within the
// groups (mgdk_BATsort, both on the device); one lane per run of equal group
// ids then picks its quantile position -- or interpolates (the _avg forms).
#include "mgdk_internal.h"

#include <cmath>
#include <string>

#pragma clang fp contract(off)

using namespace mgdk;

namespace {

template <typename T>
__device__ __forceinline__ double
to_dbl(T v)
{
	return (double) v;
}
template <>
__device__ __forceinline__ double
to_dbl<hge>(hge v)
{
	return hge_to_dbl(v);
}

enum { ST_VAR = 0, ST_COV = 1, ST_COR = 2 };
constexpr unsigned long long CNT_NONE = ~0ull;

// flags: bit 0 overflow ("22003!overflow in calculation."), bit 1 a nil result
// the reference counts (nils / nils2 of dogroupstdev and its kin)
struct MomArgs {
	oid off;               // position of candidate 0 in the value columns
	const uint32_t *perm;  // group_rows: NULL identity
	const uint64_t *start; // group_rows: NULL one group (every row, ids range-checked)
	const oid *gids;       // NULL: dense g (gseq + row)
	oid gseq, gmin;
	BUN ngrp, n;
	bool all;              // whole column (BATcalc*): every row, nils skipped
	bool skip_nils, issample, variance;
	double *res;
	double *avg;           // BATcalc{stdev,variance}: the mean (or NULL)
	uint32_t *flags;
};

// one lane per group: AGGR_STDEV / AGGR_COVARIANCE / AGGR_CORRELATION over
// the group's rows in candidate order, then the result step of the same
// macro (grouped) or of calcvariance / calccovariance / BATcalccorrelation
// (all); the whole-column loops stop at the first infinite accumulator
template <typename T, int KIND>
__global__ void
k_moments(const T *v1, const T *v2, MomArgs a)
{
	const BUN k = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= a.ngrp)
		return;
	const BUN j0 = a.start ? a.start[k] : 0, j1 = a.start ? a.start[k + 1] : a.n;
	unsigned long long cnt = 0;
	double mean1 = 0, mean2 = 0, m2 = 0, up = 0, down1 = 0, down2 = 0;
	bool ovf = false;
	constexpr int U = 4;
	for (BUN j = j0; j < j1 && cnt != CNT_NONE && !ovf; j += U) {
		T x[U], y[U];
		bool ok[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const BUN jj = j + u;
			ok[u] = jj < j1;
			BUN r = 0;
			if (ok[u]) {
				r = a.perm ? a.perm[jj] : jj;
				if (!a.start && !a.all) {
					const oid g = a.gids ? a.gids[r] : a.gseq + r;
					ok[u] = g >= a.gmin && g - a.gmin < a.ngrp;
				}
			}
			if (ok[u]) {
				x[u] = v1[a.off + r];
				if (KIND != ST_VAR)
					y[u] = v2[a.off + r];
			}
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			if (!ok[u] || cnt == CNT_NONE || ovf)
				continue;
			if (is_nil(x[u]) || (KIND != ST_VAR && is_nil(y[u]))) {
				if (!a.skip_nils && !a.all)
					cnt = CNT_NONE;
				continue;
			}
			cnt++;
			const double n = (double) cnt;
			const double xd = to_dbl(x[u]);
			const double delta1 = xd - mean1;
			mean1 += delta1 / n;
			if (KIND == ST_VAR) {
				m2 += delta1 * (xd - mean1);
				ovf = a.all && __builtin_isinf(m2);
			} else {
				const double yd = to_dbl(y[u]);
				const double delta2 = yd - mean2;
				mean2 += delta2 / n;
				if (KIND == ST_COV) {
					m2 += delta1 * (yd - mean2);
					ovf = a.all && __builtin_isinf(m2);
				} else {
					const double aux = yd - mean2;
					up += delta1 * aux;
					down1 += delta1 * (xd - mean1);
					down2 += delta2 * aux;
					ovf = a.all && (__builtin_isinf(up) || __builtin_isinf(down1) ||
							__builtin_isinf(down2));
				}
			}
		}
	}
	const double nil = __builtin_nan("");
	double res;
	bool isnil = false;
	if (ovf) {
		res = nil;
	} else if (a.all) {
		// calcvariance / calccovariance (n <= issample -> nil),
		// BATcalccorrelation (n != 0 && down1 != 0 && down2 != 0)
		const unsigned long long ss = a.issample ? 1 : 0;
		if (KIND == ST_COR) {
			const double n = (double) cnt;
			res = (cnt != 0 && down1 != 0 && down2 != 0) ? (up / n) / (sqrt(down1 / n) * sqrt(down2 / n)) : nil;
		} else if (cnt <= ss) {
			res = nil;
			mean1 = nil;
		} else {
			res = m2 / (double) (cnt - ss);
			if (KIND == ST_VAR && !a.variance)
				res = sqrt(res);
		}
	} else if (KIND == ST_COR) {
		if (cnt <= 1 || cnt == CNT_NONE || down1 == 0 || down2 == 0) {
			res = nil;
			isnil = true;
		} else if (__builtin_isinf(up) || __builtin_isinf(down1) || __builtin_isinf(down2)) {
			res = nil;
			ovf = true;
		} else {
			const double n = (double) cnt;
			res = (up / n) / (sqrt(down1 / n) * sqrt(down2 / n));
		}
	} else if (cnt == 0 || cnt == CNT_NONE) {
		res = nil;
		mean1 = nil;
		isnil = true;
	} else if (cnt == 1) {
		res = a.issample ? nil : 0.0;
		isnil = a.issample;
	} else if (__builtin_isinf(m2)) {
		res = nil;
		ovf = true;
	} else {
		res = m2 / (double) (cnt - (a.issample ? 1 : 0));
		if (KIND == ST_VAR && !a.variance)
			res = sqrt(res);
	}
	a.res[k] = res;
	if (a.avg)
		a.avg[k] = mean1;
	const uint32_t f = (ovf ? 1u : 0u) | (isnil ? 2u : 0u);
	if (f)
		atomicOr(a.flags, f);
}

template <int KIND>
void
launch_moments(int tt, const void *v1, const void *v2, const MomArgs &a)
{
	const dim3 grid((unsigned) ((a.ngrp + 63) / 64)), blk(64);
	hipStream_t st = stream();
	switch (tt) {
	case MGDK_bte:
		hipLaunchKernelGGL((k_moments<int8_t, KIND>), grid, blk, 0, st, (const int8_t *) v1, (const int8_t *) v2, a);
		break;
	case MGDK_sht:
		hipLaunchKernelGGL((k_moments<int16_t, KIND>), grid, blk, 0, st, (const int16_t *) v1, (const int16_t *) v2, a);
		break;
	case MGDK_int:
		hipLaunchKernelGGL((k_moments<int32_t, KIND>), grid, blk, 0, st, (const int32_t *) v1, (const int32_t *) v2, a);
		break;
	case MGDK_lng:
		hipLaunchKernelGGL((k_moments<int64_t, KIND>), grid, blk, 0, st, (const int64_t *) v1, (const int64_t *) v2, a);
		break;
	case MGDK_hge:
		hipLaunchKernelGGL((k_moments<hge, KIND>), grid, blk, 0, st, (const hge *) v1, (const hge *) v2, a);
		break;
	case MGDK_flt:
		hipLaunchKernelGGL((k_moments<float, KIND>), grid, blk, 0, st, (const float *) v1, (const float *) v2, a);
		break;
	default:
		hipLaunchKernelGGL((k_moments<double, KIND>), grid, blk, 0, st, (const double *) v1, (const double *) v2, a);
		break;
	}
}

bool
moment_type(int tt)
{
	switch (tt) {
	case MGDK_bte: case MGDK_sht: case MGDK_int: case MGDK_lng: case MGDK_hge: case MGDK_flt: case MGDK_dbl:
		return true;
	}
	return false;
}

bool
tdense(const mgdk_bat *b)
{
	return (b->ttype == MGDK_void || basetype(b->ttype) == MGDK_oid) && b->tseqbase != MGDK_OID_NIL;
}

struct Fixed {
	std::vector<mgdk_bat *> v;
	~Fixed()
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

// the error of a failed step, prefixed with the operator's name as the
// reference's GDKerror("%s: %s\n", func, err) does
void
prefix_err(const char *fn)
{
	std::string m = mgdk_GDKerrbuf();
	seterr("%s: %s", fn, m.c_str());
}

mgdk_bat *
const_dbl(oid hseq, double v, BUN n)
{
	return mgdk_BATconstant(hseq, MGDK_dbl, &v, n);
}

// dogroupstdev / dogroupcovariance / BATgroupcorrelation
mgdk_bat *
group_moments(const char *fn, int kind, mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s,
	      bool skip_nils, bool issample, bool variance)
{
	const bool prefixed = kind != ST_COR;
	if (b1 == nullptr || (kind != ST_VAR && b2 == nullptr)) {
		if (prefixed)
			seterr("%s: b must exist\n", fn);
		else
			seterr("b must exist\n");
		return nullptr;
	}
	if (kind != ST_VAR && (b1->count != b2->count || b1->ttype != b2->ttype || tdense(b1) != tdense(b2))) {
		seterr("%s: b1 and b2 must be aligned\n", fn);
		return nullptr;
	}
	if (g == nullptr) {
		if (kind == ST_VAR)
			seterr("%s: b and g must be aligned\n", fn);
		else if (kind == ST_COV)
			seterr("%s: b1, b2 and g must be aligned\n", fn);
		else
			seterr("b1, b2 and g must be aligned\n");
		return nullptr;
	}
	ProfScope prof("groupstats");
	// what the trivial cases read, before group_init replaces b1
	const BUN cnt1 = b1->count;
	const oid hseq1 = b1->hseqbase, hseq2 = b2 ? b2->hseqbase : 0;
	const bool nonil1 = b1->tnonil, nonil2 = b2 ? b2->tnonil : true;
	Cand ci0;
	if (cand_init(&ci0, b1, s) < 0) {
		if (prefixed)
			prefix_err(fn);
		return nullptr;
	}
	mgdk_bat *v1 = b1;
	AggrInit a;
	if (group_init(&a, &v1, g, e, s) < 0) {
		if (prefixed)
			prefix_err(fn);
		return nullptr;
	}
	const BUN ng = a.ngrp;
	if (cnt1 == 0 || ng == 0)
		return const_dbl(ng == 0 ? 0 : a.min, __builtin_nan(""), ng);
	const bool singles = tdense(g) || (g->tkey && g->tnonil);
	if (kind == ST_VAR) {
		if ((e == nullptr || (e->count == ci0.n && e->hseqbase == hseq1)) && singles && (issample || nonil1))
			return const_dbl(a.min, issample ? __builtin_nan("") : 0.0, ng);
	} else if ((e == nullptr || (e->count == cnt1 && (e->hseqbase == hseq1 || e->hseqbase == hseq2))) && singles) {
		if (kind == ST_COR)
			return const_dbl(a.min, __builtin_nan(""), ng);
		if (issample || (nonil1 && nonil2))
			return const_dbl(a.min, issample ? __builtin_nan("") : 0.0, ng);
	}
	if (!moment_type(b1->ttype)) {
		if (prefixed)
			seterr("%s: type (%s) not supported.\n", fn, atomname(b1->ttype));
		else
			seterr("type (%s) not supported.\n", atomname(b1->ttype));
		return nullptr;
	}
	// b2 at the same positions as b1 (the reference indexes both by the
	// candidate's position in b1)
	Fixed fx;
	mgdk_bat *v2 = b2;
	if (b2 && !ci0.dense) {
		mgdk_bat *view = fx.keep(mgdk_BATslice(b2, 0, b2->count));
		if (view == nullptr)
			return nullptr;
		view->hseqbase = hseq1;
		if ((v2 = cand_values_at(view, ci0)) == nullptr)
			return nullptr;
	}
	GroupRows gr(a.ci.n, ng);
	mgdk_bat *bn = newbat(a.min, MGDK_dbl, ng);
	DevBuf fl(16);
	if (bn == nullptr || !gr.ok() || !fl.p) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	if (group_rows(a, gr) != 0 || !hip_ok(hipMemsetAsync(fl.p, 0, 16, stream()), "memset")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	MomArgs m{};
	m.off = a.ci.seq - v1->hseqbase;
	m.perm = gr.perm;
	m.start = gr.start_p;
	m.gids = a.gids;
	m.gseq = a.gseq;
	m.gmin = a.min;
	m.ngrp = ng;
	m.n = a.ci.n;
	m.all = false;
	m.skip_nils = skip_nils;
	m.issample = issample;
	m.variance = variance;
	m.res = (double *) bn->theap;
	m.avg = nullptr;
	m.flags = fl.as<uint32_t>();
	const void *p2 = v2 ? v2->theap : nullptr;
	if (kind == ST_VAR)
		launch_moments<ST_VAR>(v1->ttype, v1->theap, nullptr, m);
	else if (kind == ST_COV)
		launch_moments<ST_COV>(v1->ttype, v1->theap, p2, m);
	else
		launch_moments<ST_COR>(v1->ttype, v1->theap, p2, m);
	uint32_t *h = (uint32_t *) pinned(8);
	if (!hip_ok(hipMemcpyAsync(h, fl.p, 4, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const uint32_t f = h[0];
	if (f & 1) {
		mgdk_BBPunfix(bn);
		seterr("22003!overflow in calculation.\n");
		return nullptr;
	}
	bn->count = ng;
	bn->tkey = bn->tsorted = bn->trevsorted = ng <= 1;
	bn->tnil = (f & 2) != 0;
	bn->tnonil = (f & 2) == 0;
	return bn;
}

// ---- the parallel form of the whole-column moments (fp_parallel_min) ----
// Block b folds the rows [b * tile, (b + 1) * tile) -- lane l the rows
// l, l + 256, ... of it, each lane a Welford recurrence as AGGR_STDEV /
// AGGR_COVARIANCE / AGGR_CORRELATION step it -- then the lanes and the
// blocks are combined in order by the pairwise update of Chan, Golub and
// LeVeque (n = na + nb, d = mean_b - mean_a: mean = mean_a + d nb / n,
// M2 = M2a + M2b + d^2 na nb / n, the co-moments alike).  Only the rounding
// differs from the sequential fold (DESIGN.md states the bound).
struct MomState {
	double n, mean1, mean2, m2, down1, down2;   // m2: the co-moment (up) for ST_COR
};

template <int KIND>
__device__ __forceinline__ MomState
mom_comb(const MomState &a, const MomState &b)
{
	if (a.n == 0)
		return b;
	if (b.n == 0)
		return a;
	MomState r;
	r.n = a.n + b.n;
	const double f = b.n / r.n, d1 = b.mean1 - a.mean1, w = a.n * f;
	r.mean1 = a.mean1 + d1 * f;
	r.mean2 = r.down1 = r.down2 = 0;
	if (KIND == ST_VAR) {
		r.m2 = a.m2 + b.m2 + d1 * d1 * w;
	} else {
		const double d2 = b.mean2 - a.mean2;
		r.mean2 = a.mean2 + d2 * f;
		r.m2 = a.m2 + b.m2 + d1 * d2 * w;
		if (KIND == ST_COR) {
			r.down1 = a.down1 + b.down1 + d1 * d1 * w;
			r.down2 = a.down2 + b.down2 + d2 * d2 * w;
		}
	}
	return r;
}

template <int KIND>
__device__ __forceinline__ bool
mom_inf(const MomState &s)
{
	return __builtin_isinf(s.m2) || (KIND == ST_COR && (__builtin_isinf(s.down1) || __builtin_isinf(s.down2)));
}

template <typename T, int KIND>
__global__ __launch_bounds__(256) void
k_mom_par(const T *v1, const T *v2, BUN n, BUN tile, MomState *part, uint32_t *flags)
{
	__shared__ MomState lds[256];
	const BUN b0 = (BUN) blockIdx.x * tile, b1 = min(n, b0 + tile);
	MomState s{0, 0, 0, 0, 0, 0};
	unsigned long long cnt = 0;
	for (BUN r = b0 + threadIdx.x; r < b1; r += 256) {
		const T x = v1[r];
		T y{};
		if (KIND != ST_VAR)
			y = v2[r];
		if (is_nil(x) || (KIND != ST_VAR && is_nil(y)))
			continue;
		const double nn = (double) ++cnt;
		const double xd = to_dbl(x);
		const double delta1 = xd - s.mean1;
		s.mean1 += delta1 / nn;
		if (KIND == ST_VAR) {
			s.m2 += delta1 * (xd - s.mean1);
		} else {
			const double yd = to_dbl(y);
			const double delta2 = yd - s.mean2;
			s.mean2 += delta2 / nn;
			if (KIND == ST_COV) {
				s.m2 += delta1 * (yd - s.mean2);
			} else {
				const double aux = yd - s.mean2;
				s.m2 += delta1 * aux;
				s.down1 += delta1 * (xd - s.mean1);
				s.down2 += delta2 * aux;
			}
		}
	}
	s.n = (double) cnt;
	const bool inf = mom_inf<KIND>(s);
	if (inf)
		atomicOr(flags, 1u);
	s = block_tree(s, [](const MomState &a, const MomState &b) { return mom_comb<KIND>(a, b); }, lds);
	if (threadIdx.x == 0)
		part[blockIdx.x] = s;
}

// the blocks' states combined in block order (thread t: a contiguous run of
// them, then the tree) and the result step of calcvariance /
// calccovariance / BATcalccorrelation
template <int KIND>
__global__ __launch_bounds__(256) void
k_mom_fin(const MomState *part, unsigned nb, bool issample, bool variance, double *res, double *avg,
	  uint32_t *flags)
{
	__shared__ MomState lds[256];
	const unsigned per = (nb + 255) / 256, p0 = threadIdx.x * per, p1 = min(nb, p0 + per);
	MomState s{0, 0, 0, 0, 0, 0};
	for (unsigned p = p0; p < p1; p++)
		s = mom_comb<KIND>(s, part[p]);
	s = block_tree(s, [](const MomState &a, const MomState &b) { return mom_comb<KIND>(a, b); }, lds);
	if (threadIdx.x != 0)
		return;
	const double nil = __builtin_nan("");
	const unsigned long long cnt = (unsigned long long) s.n;
	double r, mean1 = s.mean1;
	if (mom_inf<KIND>(s) || (*flags & 1)) {
		r = nil;
		atomicOr(flags, 1u);
	} else if (KIND == ST_COR) {
		const double nn = s.n;
		r = (cnt != 0 && s.down1 != 0 && s.down2 != 0) ? (s.m2 / nn) / (sqrt(s.down1 / nn) * sqrt(s.down2 / nn)) : nil;
	} else if (cnt <= (issample ? 1ull : 0ull)) {
		r = nil;
		mean1 = nil;
	} else {
		r = s.m2 / (double) (cnt - (issample ? 1 : 0));
		if (KIND == ST_VAR && !variance)
			r = sqrt(r);
	}
	*res = r;
	*avg = cnt ? mean1 : nil;
}

template <int KIND>
void
launch_mom_par(int tt, const void *v1, const void *v2, BUN n, MomState *part, unsigned nb, BUN tile,
	       uint32_t *flags)
{
	const dim3 grid(nb), blk(256);
	hipStream_t st = stream();
	switch (tt) {
	case MGDK_bte: hipLaunchKernelGGL((k_mom_par<int8_t, KIND>), grid, blk, 0, st, (const int8_t *) v1, (const int8_t *) v2, n, tile, part, flags); break;
	case MGDK_sht: hipLaunchKernelGGL((k_mom_par<int16_t, KIND>), grid, blk, 0, st, (const int16_t *) v1, (const int16_t *) v2, n, tile, part, flags); break;
	case MGDK_int: hipLaunchKernelGGL((k_mom_par<int32_t, KIND>), grid, blk, 0, st, (const int32_t *) v1, (const int32_t *) v2, n, tile, part, flags); break;
	case MGDK_lng: hipLaunchKernelGGL((k_mom_par<int64_t, KIND>), grid, blk, 0, st, (const int64_t *) v1, (const int64_t *) v2, n, tile, part, flags); break;
	case MGDK_hge: hipLaunchKernelGGL((k_mom_par<hge, KIND>), grid, blk, 0, st, (const hge *) v1, (const hge *) v2, n, tile, part, flags); break;
	case MGDK_flt: hipLaunchKernelGGL((k_mom_par<float, KIND>), grid, blk, 0, st, (const float *) v1, (const float *) v2, n, tile, part, flags); break;
	default: hipLaunchKernelGGL((k_mom_par<double, KIND>), grid, blk, 0, st, (const double *) v1, (const double *) v2, n, tile, part, flags); break;
	}
}

// calcvariance / calccovariance / BATcalccorrelation over the whole column
double
calc_moments(int kind, double *avgp, mgdk_bat *b1, mgdk_bat *b2, bool issample, bool variance)
{
	const double nil = __builtin_nan("");
	if (avgp)
		*avgp = nil;
	if (b1 == nullptr || (kind != ST_VAR && b2 == nullptr)) {
		seterr("b must exist\n");
		return nil;
	}
	if (!moment_type(b1->ttype)) {
		seterr("type (%s) not supported.\n", atomname(b1->ttype));
		return nil;
	}
	if (kind != ST_VAR && (b1->count != b2->count || b1->ttype != b2->ttype)) {
		seterr("b1 and b2 must be aligned\n");
		return nil;
	}
	ProfScope prof("calcstats");
	DevBuf out(32), fl(16);
	if (!out.p || !fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 16, stream()), "memset"))
		return nil;
	MomArgs m{};
	m.off = 0;
	m.ngrp = 1;
	m.n = b1->count;
	m.all = true;
	m.skip_nils = true;
	m.issample = issample;
	m.variance = variance;
	m.res = out.as<double>();
	m.avg = out.as<double>() + 1;
	m.flags = fl.as<uint32_t>();
	const BUN n = b1->count;
	if (n >= fp_parallel_min() && n > 0) {
		// the parallel form: ~16 rows per lane, at most 2048 blocks
		unsigned nb = (unsigned) min((BUN) 2048, (n + 4095) / 4096);
		const BUN tile = (n + nb - 1) / nb;
		nb = (unsigned) ((n + tile - 1) / tile);
		DevBuf part((size_t) nb * sizeof(MomState));
		if (!part.p)
			return nil;
		MomState *pp = part.as<MomState>();
		const void *p2 = kind != ST_VAR ? b2->theap : nullptr;
		if (kind == ST_VAR) {
			launch_mom_par<ST_VAR>(b1->ttype, b1->theap, p2, n, pp, nb, tile, m.flags);
			hipLaunchKernelGGL((k_mom_fin<ST_VAR>), dim3(1), dim3(256), 0, stream(), pp, nb, issample, variance,
					   m.res, m.avg, m.flags);
		} else if (kind == ST_COV) {
			launch_mom_par<ST_COV>(b1->ttype, b1->theap, p2, n, pp, nb, tile, m.flags);
			hipLaunchKernelGGL((k_mom_fin<ST_COV>), dim3(1), dim3(256), 0, stream(), pp, nb, issample, variance,
					   m.res, m.avg, m.flags);
		} else {
			launch_mom_par<ST_COR>(b1->ttype, b1->theap, p2, n, pp, nb, tile, m.flags);
			hipLaunchKernelGGL((k_mom_fin<ST_COR>), dim3(1), dim3(256), 0, stream(), pp, nb, issample, variance,
					   m.res, m.avg, m.flags);
		}
		if (!sync())
			return nil;
	} else if (kind == ST_VAR)
		launch_moments<ST_VAR>(b1->ttype, b1->theap, nullptr, m);
	else if (kind == ST_COV)
		launch_moments<ST_COV>(b1->ttype, b1->theap, b2->theap, m);
	else
		launch_moments<ST_COR>(b1->ttype, b1->theap, b2->theap, m);
	double *h = (double *) pinned(24);
	if (!hip_ok(hipMemcpyAsync(h, out.p, 16, hipMemcpyDeviceToHost, stream()), "memcpy") ||
	    !hip_ok(hipMemcpyAsync(h + 2, fl.p, 4, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync())
		return nil;
	uint32_t f;
	memcpy(&f, h + 2, 4);
	if (f & 1) {
		seterr("22003!overflow in calculation.\n");
		return nil;
	}
	if (avgp)
		*avgp = h[1];
	return h[0];
}

// ---- quantiles ---------------------------------------------------------

template <typename T>
__device__ __forceinline__ bool
q_nil(const T *v, BUN i)
{
	return is_nil(v[i]);
}

template <typename T> __device__ __forceinline__ T qnil() { return NilOf<T>::v(); }
template <> __device__ __forceinline__ float qnil<float>() { return __builtin_nanf(""); }
template <> __device__ __forceinline__ double qnil<double>() { return __builtin_nan(""); }

__global__ __launch_bounds__(256) void
k_copy_bytes(const uint8_t *src, uint8_t *dst, size_t n)
{
	for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x)
		dst[i] = src[i];
}

// one lane per output group j: the run [starts[j], starts[j+1]) of the
// sorted (g, b) rows (the last run ends at n); j >= k (fewer runs than
// groups): nil, as the reference pads its result (gdk_aggr.c:4073-4077).
// average: DO_QUANTILE_AVG (:3860) interpolating in dbl; else the value at
// r + p - (BUN) (p + 0.5 - f) (:4060-4068)
template <typename T>
__global__ void
k_quantile(const T *sv, const oid *starts, oid s0, BUN k, BUN n, BUN ng, double q, bool skip_nils, bool average,
	   T *out, double *dout, uint32_t *flags)
{
	const BUN j = (BUN) blockIdx.x * blockDim.x + threadIdx.x;
	if (j >= ng)
		return;
	bool isnil = false;
	if (j >= k) {
		isnil = true;
	} else {
		BUN r = starts ? starts[j] : s0 + j;
		const BUN p = j + 1 < k ? (starts ? starts[j + 1] : s0 + j + 1) : n;
		if (skip_nils) {
			// nils sort first: the first non-nil of the run
			BUN lo = r, hi = p;
			while (lo < hi) {
				const BUN m = lo + (hi - lo) / 2;
				if (q_nil(sv, m))
					lo = m + 1;
				else
					hi = m;
			}
			r = lo;
		}
		if (r == p) {
			isnil = true;
		} else if (average) {
			const double f = (double) (p - r - 1) * q;
			const double lo = floor(f), hi = ceil(f);
			const T low = sv[r + (BUN) hi], high = sv[r + (BUN) lo];
			if (is_nil(low) || is_nil(high)) {
				isnil = true;
			} else {
				dout[j] = (f - lo) * to_dbl(low) + (lo + 1 - f) * to_dbl(high);
			}
		} else {
			const double f = (double) (p - r - 1) * q;
			const BUN qi = r + p - (BUN) ((double) p + 0.5 - f);
			const T v = sv[qi];
			out[j] = v;
			isnil = is_nil(v);
			if (isnil)
				atomicOr(flags, 2u);
			return;
		}
	}
	if (isnil) {
		if (average)
			dout[j] = __builtin_nan("");
		else
			out[j] = qnil<T>();
		atomicOr(flags, 2u);
	}
}

template <typename T>
__global__ void
k_run_starts(const T *g, BUN n, int8_t *fl)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		fl[i] = i == 0 || g[i] != g[i - 1];
}

// an element of b's tail as the kernels type it
int
qkind(int tt)
{
	switch (tt) {
	case MGDK_bte: case MGDK_bit: return 1;
	case MGDK_sht: return 2;
	case MGDK_int: case MGDK_date: return 4;
	case MGDK_lng: case MGDK_oid: case MGDK_daytime: case MGDK_timestamp: return 8;
	case MGDK_hge: return 16;
	case MGDK_flt: return -4;
	case MGDK_dbl: return -8;
	}
	return 0;
}

void
launch_quantile(int tt, const void *sv, const oid *starts, oid s0, BUN k, BUN n, BUN ng, double q, bool skip_nils,
		bool average, void *out, double *dout, uint32_t *flags)
{
	const dim3 grid((unsigned) ((ng + 255) / 256)), blk(256);
	hipStream_t st = stream();
#define QL(T) hipLaunchKernelGGL(k_quantile<T>, grid, blk, 0, st, (const T *) sv, starts, s0, k, n, ng, q, skip_nils, \
				 average, (T *) out, dout, flags)
	switch (qkind(tt)) {
	case 1: QL(int8_t); break;
	case 2: QL(int16_t); break;
	case 4: QL(int32_t); break;
	case 8: QL(int64_t); break;
	case 16: QL(hge); break;
	case -4: QL(float); break;
	default: QL(double); break;
	}
#undef QL
}

// doBATgroupquantile (gdk_aggr.c:3881)
mgdk_bat *
group_quantile(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, double quantile, bool skip_nils,
	       bool average)
{
	if (b == nullptr) {
		seterr("b must exist\n");
		return nullptr;
	}
	if (average) {
		switch (basetype(b->ttype)) {
		case MGDK_bte: case MGDK_sht: case MGDK_int: case MGDK_lng: case MGDK_hge: case MGDK_flt: case MGDK_dbl:
			break;
		default:
			seterr("incompatible type\n");
			return nullptr;
		}
	}
	// BATgroupaggrinit (:65): g optional here (one group)
	Cand ci;
	if (cand_init(&ci, b, s) < 0)
		return nullptr;
	oid min = 0;
	BUN ngrp = 1;
	mgdk_bat *vals = b;      // b at the candidates, head at the first one
	AggrInit a;
	if (g) {
		if (group_init(&a, &vals, g, e, s) < 0)
			return nullptr;
		min = a.min;
		ngrp = a.ngrp;
	}
	if (tp != b->ttype) {
		seterr("type of b and tp differ\n");
		return nullptr;
	}
	const int qk = qkind(b->ttype);
	if (qk == 0) {
		seterr("%s: type %s is not on the device path\n", average ? "BATgroupquantile_avg" : "BATgroupquantile",
		       atomname(b->ttype));
		return nullptr;
	}
	if (quantile < 0 || quantile > 1) {
		seterr("cannot determine quantile for p=%f (p has to be in [0,1])\n", quantile);
		return nullptr;
	}
	const int rt = average ? MGDK_dbl : tp;
	if (b->count == 0 || ngrp == 0 || std::isnan(quantile)) {
		mgdk_bat *bn;
		if (average) {
			bn = const_dbl(ngrp == 0 ? 0 : min, __builtin_nan(""), ngrp);
		} else {
			hge nilv;
			switch (qk) {
			case 1: { int8_t v = INT8_MIN; memcpy(&nilv, &v, 1); break; }
			case 2: { int16_t v = INT16_MIN; memcpy(&nilv, &v, 2); break; }
			case 4: { int32_t v = INT32_MIN; memcpy(&nilv, &v, 4); break; }
			case 8: { int64_t v = INT64_MIN; memcpy(&nilv, &v, 8); break; }
			case 16: nilv = NilOf<hge>::v(); break;
			case -4: { float v = __builtin_nanf(""); memcpy(&nilv, &v, 4); break; }
			default: { double v = __builtin_nan(""); memcpy(&nilv, &v, 8); break; }
			}
			bn = mgdk_BATconstant(ngrp == 0 ? 0 : min, tp, &nilv, ngrp);
		}
		return bn;
	}
	ProfScope prof("groupquantile");
	Fixed fx;
	// vals from voff on: b's values at the candidates (group_init gathered a
	// materialised list, then a.ci is dense over the gathered column)
	const BUN n = ci.n;
	oid voff;
	if (g) {
		voff = a.ci.seq - vals->hseqbase;
	} else if (!ci.dense) {
		if ((vals = cand_values_at(b, ci)) == nullptr)
			return nullptr;
		voff = 0;
	} else {
		voff = ci.seq - b->hseqbase;
	}
	if (g) {
		// BATproject(s, g) (:3953): g is aligned with the candidates, so a list
		// with gaps reaches past g's end
		if (!ci.dense && n && ci.last - ci.first + 1 != n) {
			seterr("BATproject: does not match always\n");
			return nullptr;
		}
		if (tdense(g)) {
			// singleton groups: a copy of b's values (as dbl for the averages)
			mgdk_bat *cv = vals;
			if (voff != 0 || n != vals->count)
				cv = fx.keep(mgdk_BATslice(vals, voff, voff + n));
			if (cv == nullptr)
				return nullptr;
			mgdk_bat *bn;
			if (average) {
				bn = mgdk_BATconvert(cv, nullptr, MGDK_dbl, 0, 0, 0);
			} else {
				bn = newbat(0, tp, n);
				if (bn) {
					const size_t bytes = (size_t) n * width_of(tp);
					if (bytes)
						hipLaunchKernelGGL(k_copy_bytes, dim3(grid_for(bytes, 256 * 16, 8192)), dim3(256), 0,
								   stream(), (const uint8_t *) cv->theap, (uint8_t *) bn->theap, bytes);
					if (!sync()) {
						mgdk_BBPunfix(bn);
						return nullptr;
					}
					bn->count = n;
					bn->tsorted = cv->tsorted;
					bn->trevsorted = cv->trevsorted;
					bn->tkey = cv->tkey;
					bn->tnonil = cv->tnonil;
					bn->tnil = cv->tnil;
				}
			}
			if (bn == nullptr)
				return nullptr;
			bn->hseqbase = g->tseqbase;
			return bn;
		}
	}
	// the values (at the candidates) as a column of their own
	mgdk_bat *bv = vals;
	if (voff != 0 || n != vals->count)
		bv = fx.keep(mgdk_BATslice(vals, voff, voff + n));
	if (bv == nullptr)
		return nullptr;
	mgdk_bat *sv = nullptr, *gs = nullptr, *go = nullptr;
	if (g) {
		mgdk_bat *gp = g;
		if (mgdk_BATsort(&gs, &go, nullptr, gp, nullptr, nullptr, false, false, false) != 0)
			return nullptr;
		fx.keep(gs);
		fx.keep(go);
		if (mgdk_BATsort(&sv, nullptr, nullptr, bv, go, gs, false, false, false) != 0)
			return nullptr;
	} else {
		// with the order, as the reference asks for it (gdk_aggr.c:4121): a
		// column that is not a view keeps it as its order index
		mgdk_bat *so = nullptr;
		if (mgdk_BATsort(&sv, &so, nullptr, bv, nullptr, nullptr, false, false, false) != 0)
			return nullptr;
		mgdk_BBPunfix(so);
	}
	fx.keep(sv);
	// runs of equal group ids
	BUN k = 1;
	const oid *starts = nullptr;
	oid s0 = 0;
	if (g) {
		if (gs->ttype == MGDK_void) {
			k = n;           // distinct ids: one row each
		} else {
			DevBuf rf(n + 8);
			if (!rf.p)
				return nullptr;
			hipLaunchKernelGGL(k_run_starts<uint64_t>, dim3(grid_for(n, 2048, 8192)), dim3(256), 0, stream(),
					   (const uint64_t *) gs->theap, n, rf.as<int8_t>());
			mgdk_bat *ps = fx.keep(compact_flags(rf.as<int8_t>(), n, 0));
			if (ps == nullptr)
				return nullptr;
			k = ps->count;
			if (ps->ttype == MGDK_void)
				s0 = ps->tseqbase;
			else
				starts = (const oid *) ps->theap;
		}
		if (k > ngrp) {
			seterr("%s: more group ids than groups\n", average ? "BATgroupquantile_avg" : "BATgroupquantile");
			return nullptr;
		}
	}
	mgdk_bat *bn = newbat(g ? min : 0, rt, ngrp);
	DevBuf fl(16);
	if (bn == nullptr || !fl.p || !hip_ok(hipMemsetAsync(fl.p, 0, 16, stream()), "memset")) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	launch_quantile(sv->ttype == MGDK_void ? MGDK_oid : sv->ttype, sv->theap, starts, s0, k, n, ngrp, quantile,
			skip_nils, average, average ? nullptr : bn->theap, average ? (double *) bn->theap : nullptr,
			fl.as<uint32_t>());
	uint32_t *h = (uint32_t *) pinned(8);
	if (!hip_ok(hipMemcpyAsync(h, fl.p, 4, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync()) {
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	bn->count = ngrp;
	bn->tkey = bn->tsorted = bn->trevsorted = ngrp <= 1;
	bn->tnil = (h[0] & 2) != 0;
	bn->tnonil = (h[0] & 2) == 0;
	return bn;
}

}  // namespace

extern "C" {

mgdk_bat *
mgdk_BATgroupstdev_sample(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	(void) tp;
	return group_moments("BATgroupstdev_sample", ST_VAR, b, nullptr, g, e, s, skip_nils, true, false);
}

mgdk_bat *
mgdk_BATgroupstdev_population(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	(void) tp;
	return group_moments("BATgroupstdev_population", ST_VAR, b, nullptr, g, e, s, skip_nils, false, false);
}

mgdk_bat *
mgdk_BATgroupvariance_sample(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	(void) tp;
	return group_moments("BATgroupvariance_sample", ST_VAR, b, nullptr, g, e, s, skip_nils, true, true);
}

mgdk_bat *
mgdk_BATgroupvariance_population(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	(void) tp;
	return group_moments("BATgroupvariance_population", ST_VAR, b, nullptr, g, e, s, skip_nils, false, true);
}

mgdk_bat *
mgdk_BATgroupcovariance_sample(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp,
			       bool skip_nils)
{
	(void) tp;
	return group_moments("BATgroupcovariance_sample", ST_COV, b1, b2, g, e, s, skip_nils, true, false);
}

mgdk_bat *
mgdk_BATgroupcovariance_population(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp,
				   bool skip_nils)
{
	(void) tp;
	return group_moments("BATgroupcovariance_population", ST_COV, b1, b2, g, e, s, skip_nils, false, false);
}

mgdk_bat *
mgdk_BATgroupcorrelation(mgdk_bat *b1, mgdk_bat *b2, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	(void) tp;
	return group_moments("BATgroupcorrelation", ST_COR, b1, b2, g, e, s, skip_nils, false, false);
}

double
mgdk_BATcalcstdev_population(double *avgp, mgdk_bat *b)
{
	return calc_moments(ST_VAR, avgp, b, nullptr, false, false);
}

double
mgdk_BATcalcstdev_sample(double *avgp, mgdk_bat *b)
{
	return calc_moments(ST_VAR, avgp, b, nullptr, true, false);
}

double
mgdk_BATcalcvariance_population(double *avgp, mgdk_bat *b)
{
	return calc_moments(ST_VAR, avgp, b, nullptr, false, true);
}

double
mgdk_BATcalcvariance_sample(double *avgp, mgdk_bat *b)
{
	return calc_moments(ST_VAR, avgp, b, nullptr, true, true);
}

double
mgdk_BATcalccovariance_population(mgdk_bat *b1, mgdk_bat *b2)
{
	return calc_moments(ST_COV, nullptr, b1, b2, false, false);
}

double
mgdk_BATcalccovariance_sample(mgdk_bat *b1, mgdk_bat *b2)
{
	return calc_moments(ST_COV, nullptr, b1, b2, true, false);
}

double
mgdk_BATcalccorrelation(mgdk_bat *b1, mgdk_bat *b2)
{
	return calc_moments(ST_COR, nullptr, b1, b2, false, false);
}

mgdk_bat *
mgdk_BATgroupmedian(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	return group_quantile(b, g, e, s, tp, 0.5, skip_nils, false);
}

mgdk_bat *
mgdk_BATgroupquantile(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, double quantile, bool skip_nils)
{
	return group_quantile(b, g, e, s, tp, quantile, skip_nils, false);
}

mgdk_bat *
mgdk_BATgroupmedian_avg(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, bool skip_nils)
{
	return group_quantile(b, g, e, s, tp, 0.5, skip_nils, true);
}

mgdk_bat *
mgdk_BATgroupquantile_avg(mgdk_bat *b, mgdk_bat *g, mgdk_bat *e, mgdk_bat *s, int tp, double quantile,
			  bool skip_nils)
{
	return group_quantile(b, g, e, s, tp, quantile, skip_nils, true);
}

}  // extern "C"
