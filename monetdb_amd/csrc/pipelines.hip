// pipelines.hip -- the op-at-a-time TPC-H Q1 / Q6 MAL plans composed from
// the device GDK operators, exactly as the reference's MAL interpreter
// calls them (algebra.select x2, thetaselect,
// projection x2, batcalc.*, aggr.sum; §3.3 Q1: thetaselect, projection x6,
// group.group, group.subgroup, batcalc.- + * + *, aggr.subsum x4 (+ disc),
// aggr.subcount, aggr.subavg x3).  Used as the exact fallback of the fused kernels and as
// the "drop-in" timing of the GDK boundary.
#include <cstring>
#include <vector>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {
struct Bats {
	std::vector<mgdk_bat *> v;
	mgdk_bat *add(mgdk_bat *b) { v.push_back(b); return b; }
	~Bats() { for (mgdk_bat *b : v) mgdk_BBPunfix(b); }
};
// the plan's result columns read back with one wait (the result export of
// the MAL plan), through the thread's pinned buffer
struct Readback {
	std::vector<std::pair<const mgdk_bat *, void *>> v;
	void add(const mgdk_bat *b, void *host) { v.emplace_back(b, host); }
	int run()
	{
		size_t tot = 16;
		for (auto &x : v)
			if (x.first->ttype != MGDK_void)
				tot += (x.first->count * (size_t) x.first->twidth + 15) & ~(size_t) 15;
		char *h = (char *) pinned(tot);
		if (h == nullptr)
			return -1;
		size_t o = 0;
		for (auto &x : v) {
			const mgdk_bat *b = x.first;
			const size_t bytes = b->count * (size_t) b->twidth;
			if (b->ttype == MGDK_void || bytes == 0)
				continue;
			if (!hip_ok(hipMemcpyAsync(h + o, b->theap, bytes, hipMemcpyDeviceToHost, stream()), "memcpy"))
				return -1;
			o += (bytes + 15) & ~(size_t) 15;
		}
		if (!sync())
			return -1;
		o = 0;
		for (auto &x : v) {
			const mgdk_bat *b = x.first;
			if (b->ttype == MGDK_void) {
				if (mgdk_BATdownload(b, x.second) < 0)
					return -1;
				continue;
			}
			const size_t bytes = b->count * (size_t) b->twidth;
			memcpy(x.second, h + o, bytes);
			o += (bytes + 15) & ~(size_t) 15;
		}
		return 0;
	}
};
}  // namespace

namespace mgdk {

int
q1_opatatime(mgdk_bat *shipdate, mgdk_bat *rf, mgdk_bat *ls, mgdk_bat *qty, mgdk_bat *price,
	     mgdk_bat *disc, mgdk_bat *tax, int32_t dmax, mgdk_q1row *rows, int maxgroups, int *ngroups)
{
	ProfScope prof("q1_opatatime");
	Bats t;
	mgdk_bat *c1 = t.add(mgdk_BATthetaselect(shipdate, nullptr, &dmax, "<="));
	if (!c1)
		return -1;
	mgdk_bat *prf = t.add(mgdk_BATproject(c1, rf));
	mgdk_bat *pls = t.add(mgdk_BATproject(c1, ls));
	mgdk_bat *pq = t.add(mgdk_BATproject(c1, qty));
	mgdk_bat *pp = t.add(mgdk_BATproject(c1, price));
	mgdk_bat *pd = t.add(mgdk_BATproject(c1, disc));
	mgdk_bat *pt = t.add(mgdk_BATproject(c1, tax));
	if (!prf || !pls || !pq || !pp || !pd || !pt)
		return -1;
	mgdk_bat *g1, *e1, *h1, *g2, *e2, *h2;
	if (mgdk_BATgroup(&g1, &e1, &h1, prf, nullptr, nullptr, nullptr, nullptr) < 0)
		return -1;
	t.add(g1), t.add(e1), t.add(h1);
	if (mgdk_BATgroup(&g2, &e2, &h2, pls, nullptr, g1, e1, h1) < 0)
		return -1;
	t.add(g2), t.add(e2), t.add(h2);
	int64_t hundred = 100;
	mgdk_bat *omd = t.add(mgdk_BATcalccstsub(&hundred, MGDK_lng, pd, nullptr, MGDK_lng));
	mgdk_bat *dp = omd ? t.add(mgdk_BATcalcmul(pp, omd, nullptr, nullptr, MGDK_hge)) : nullptr;
	mgdk_bat *opt = t.add(mgdk_BATcalccstadd(&hundred, MGDK_lng, pt, nullptr, MGDK_lng));
	mgdk_bat *ch = (dp && opt) ? t.add(mgdk_BATcalcmul(dp, opt, nullptr, nullptr, MGDK_hge)) : nullptr;
	if (!ch)
		return -1;
	mgdk_bat *s1 = t.add(mgdk_BATgroupsum(pq, g2, e2, nullptr, MGDK_hge, true));
	mgdk_bat *s2 = t.add(mgdk_BATgroupsum(pp, g2, e2, nullptr, MGDK_hge, true));
	mgdk_bat *s3 = t.add(mgdk_BATgroupsum(dp, g2, e2, nullptr, MGDK_hge, true));
	mgdk_bat *s4 = t.add(mgdk_BATgroupsum(ch, g2, e2, nullptr, MGDK_hge, true));
	mgdk_bat *s5 = t.add(mgdk_BATgroupsum(pd, g2, e2, nullptr, MGDK_hge, true));
	mgdk_bat *cn = t.add(mgdk_BATgroupcount(pq, g2, e2, nullptr, MGDK_lng, false));
	// aggr.subavg (3 outputs) of quantity, extendedprice, discount
	mgdk_bat *av[3], *rm[3], *ac[3];
	mgdk_bat *avin[3] = {pq, pp, pd};
	for (int k = 0; k < 3; k++) {
		if (mgdk_BATgroupavg3(&av[k], &rm[k], &ac[k], avin[k], g2, e2, nullptr, true) < 0)
			return -1;
		t.add(av[k]), t.add(rm[k]), t.add(ac[k]);
	}
	// extents are positions in the projected (filtered) columns
	mgdk_bat *krf = t.add(mgdk_BATproject(e2, prf));
	mgdk_bat *kls = t.add(mgdk_BATproject(e2, pls));
	mgdk_bat *krow = t.add(mgdk_BATproject(e2, c1));   // lineitem oid of each group's first row
	if (!s1 || !s2 || !s3 || !s4 || !s5 || !cn || !krf || !kls || !krow)
		return -1;
	// ORDER BY l_returnflag, l_linestatus: algebra.sort on the first key,
	// the subsort of the second within its groups, every output column
	// projected through the final order (the plan's leftfetchjoins)
	{
		mgdk_bat *sa, *oa, *ga, *sb, *ob, *gb;
		SortInternal no_oidx;   // the plan's sorts of projected temporaries
		if (mgdk_BATsort(&sa, &oa, &ga, krf, nullptr, nullptr, false, false, false) < 0)
			return -1;
		t.add(sa), t.add(oa), t.add(ga);
		if (mgdk_BATsort(&sb, &ob, &gb, kls, oa, ga, false, false, false) < 0)
			return -1;
		t.add(sb), t.add(ob);
		if (gb)
			t.add(gb);
		mgdk_bat **outs[] = {&s1, &s2, &s3, &s4, &s5, &cn, &krf, &kls, &krow,
				     &av[0], &av[1], &av[2], &rm[0], &rm[1], &rm[2]};
		for (mgdk_bat **o : outs)
			if (!(*o = t.add(mgdk_BATproject(ob, *o))))
				return -1;
	}
	const BUN ng = e2->count;
	if ((int) ng > maxgroups) {
		seterr("q1: more groups (%llu) than room for results", (unsigned long long) ng);
		return -1;
	}
	std::vector<hge> v1(ng), v2(ng), v3(ng), v4(ng), v5(ng);
	std::vector<int64_t> vc(ng);
	std::vector<oid> ve(ng);
	std::vector<uint8_t> vr(ng), vl(ng);
	std::vector<int64_t> va[3], vrm[3];
	Readback rb;
	for (int k = 0; k < 3; k++) {
		va[k].resize(ng);
		vrm[k].resize(ng);
		rb.add(av[k], va[k].data());
		rb.add(rm[k], vrm[k].data());
	}
	rb.add(s1, v1.data()), rb.add(s2, v2.data()), rb.add(s3, v3.data()), rb.add(s4, v4.data());
	rb.add(s5, v5.data()), rb.add(cn, vc.data()), rb.add(krow, ve.data()), rb.add(krf, vr.data());
	rb.add(kls, vl.data());
	if (rb.run() < 0)
		return -1;
	for (BUN k = 0; k < ng; k++) {
		mgdk_q1row &r = rows[k];
		memset(&r, 0, sizeof(r));
		r.returnflag = vr[k];
		r.linestatus = vl[k];
		memcpy(r.sum_qty, &v1[k], 16);
		memcpy(r.sum_base_price, &v2[k], 16);
		memcpy(r.sum_disc_price, &v3[k], 16);
		memcpy(r.sum_charge, &v4[k], 16);
		memcpy(r.sum_disc, &v5[k], 16);
		r.count_order = vc[k];
		r.first_row = ve[k];
		r.avg_qty = va[0][k], r.rem_qty = vrm[0][k];
		r.avg_price = va[1][k], r.rem_price = vrm[1][k];
		r.avg_disc = va[2][k], r.rem_disc = vrm[2][k];
	}
	*ngroups = (int) ng;
	return 0;
}

int
q6_opatatime(mgdk_bat *shipdate, mgdk_bat *discount, mgdk_bat *quantity, mgdk_bat *price, int32_t d0,
	     int32_t d1, int64_t dlo, int64_t dhi, int64_t qmax, void *revenue)
{
	Bats t;
	mgdk_bat *c1 = t.add(mgdk_BATselect(shipdate, nullptr, &d0, &d1, true, false, false, false));
	mgdk_bat *c2 = c1 ? t.add(mgdk_BATselect(discount, c1, &dlo, &dhi, true, true, false, false)) : nullptr;
	mgdk_bat *c3 = c2 ? t.add(mgdk_BATthetaselect(quantity, c2, &qmax, "<")) : nullptr;
	mgdk_bat *p1 = c3 ? t.add(mgdk_BATproject(c3, price)) : nullptr;
	mgdk_bat *p2 = c3 ? t.add(mgdk_BATproject(c3, discount)) : nullptr;
	mgdk_bat *m = (p1 && p2) ? t.add(mgdk_BATcalcmul(p1, p2, nullptr, nullptr, MGDK_hge)) : nullptr;
	if (!m)
		return -1;
	if (m->count == 0) {
		memset(revenue, 0, 16);
		return 0;
	}
	return mgdk_BATsum(revenue, MGDK_hge, m, nullptr, true, true);
}

}  // namespace mgdk

extern "C" {

// op-at-a-time variants exported for timing the GDK-boundary path
int mgdk_q6_opatatime(mgdk_bat *shipdate, mgdk_bat *discount, mgdk_bat *quantity, mgdk_bat *price,
		      int32_t d0, int32_t d1, int64_t dlo, int64_t dhi, int64_t qmax, void *revenue)
{
	return q6_opatatime(shipdate, discount, quantity, price, d0, d1, dlo, dhi, qmax, revenue);
}

int mgdk_q1_opatatime(mgdk_bat *shipdate, mgdk_bat *rf, mgdk_bat *ls, mgdk_bat *qty, mgdk_bat *price,
		      mgdk_bat *disc, mgdk_bat *tax, int32_t dmax, mgdk_q1row *rows, int maxgroups, int *ngroups)
{
	return q1_opatatime(shipdate, rf, ls, qty, price, disc, tax, dmax, rows, maxgroups, ngroups);
}

}  // extern "C"
