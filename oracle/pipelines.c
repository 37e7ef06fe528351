/*
 * pipelines.c -- TPC-H Q6 / Q1 column pipelines over the oracle operators,
 * op-at-a-time like MonetDB's MAL plans, with
 * mitosis-style row-range slicing across threads (opt_mitosis.c:150-230;
 * partial aggregates re-aggregated as in opt_mergetable.c:1496-1670).
 * TEST INFRASTRUCTURE ONLY: this is the CPU comparator and the parity
 * reference for the product's pipelines.
 */
#include "gdk_oracle.h"

#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void ora_seterr(const char *fmt, ...);
static char shared_err[1024];

static ora_bat
view(int type, void *base, uint64_t row0, uint64_t n)
{
	ora_bat b;
	memset(&b, 0, sizeof(b));
	b.type = type;
	b.width = type == ORA_int || type == ORA_date ? 4 : type == ORA_str ? 1 : 8;
	b.count = n;
	b.hseqbase = row0;
	b.tseqbase = ORA_OID_NIL;
	b.base = (char *) base + row0 * b.width;
	b.nonil = 1;
	return b;
}

/* Q6: select(shipdate in [1994-01-01,1995-01-01)) -> select(discount in
 * [5,7], C1) -> thetaselect(quantity < 2400, C2) -> project price and
 * discount -> batcalc.* lng*lng->hge -> aggr.sum (hge) */
static int
q6_slice(const ora_lineitem *li, uint64_t row0, uint64_t n, ora_hge *res)
{
	ora_bat sd = view(ORA_date, li->shipdate, row0, n);
	ora_bat di = view(ORA_lng, li->discount, row0, n);
	ora_bat qt = view(ORA_lng, li->quantity, row0, n);
	ora_bat pr = view(ORA_lng, li->extendedprice, row0, n);
	int32_t d0 = ora_mkdate(1994, 1, 1), d1 = ora_mkdate(1995, 1, 1);
	int64_t lo = 5, hi = 7, q = 2400;
	int rc = -1;
	ora_bat *c1 = NULL, *c2 = NULL, *c3 = NULL, *p1 = NULL, *p2 = NULL, *m = NULL;
	if ((c1 = ora_select(&sd, NULL, &d0, &d1, true, false, false, false)) == NULL)
		goto out;
	if ((c2 = ora_select(&di, c1, &lo, &hi, true, true, false, false)) == NULL)
		goto out;
	if ((c3 = ora_thetaselect(&qt, c2, &q, "<")) == NULL)
		goto out;
	if ((p1 = ora_project(c3, &pr)) == NULL || (p2 = ora_project(c3, &di)) == NULL)
		goto out;
	if ((m = ora_calc('*', p1, NULL, 0, p2, NULL, 0, NULL, ORA_hge)) == NULL)
		goto out;
	if (m->count == 0) {
		*res = 0;
		rc = 0;
		goto out;
	}
	rc = ora_sum(res, ORA_hge, m, NULL, true, true);
out:
	ora_free(c1); ora_free(c2); ora_free(c3); ora_free(p1); ora_free(p2); ora_free(m);
	return rc;
}

int
ora_q6(const ora_lineitem *li, int nthreads, ora_hge *revenue)
{
	if (nthreads < 1)
		nthreads = 1;
	uint64_t n = li->n;
	ora_hge tot = 0;
	int err = 0;
#pragma omp parallel for num_threads(nthreads) reduction(+:tot) reduction(|:err) schedule(static, 1)
	for (int t = 0; t < nthreads; t++) {
		uint64_t a = n * (uint64_t) t / (uint64_t) nthreads;
		uint64_t b = n * (uint64_t) (t + 1) / (uint64_t) nthreads;
		ora_hge r = 0;
		if (q6_slice(li, a, b - a, &r) < 0) {
			err |= 1;
#pragma omp critical
			snprintf(shared_err, sizeof(shared_err), "%s", ora_errbuf());
		}
		tot += r;
	}
	*revenue = tot;
	if (err)
		ora_seterr("%s", shared_err);
	return err ? -1 : 0;
}

/* Q1 per slice: thetaselect(shipdate <= 1998-09-02) -> project 6 columns
 * -> group(returnflag) -> subgroup(linestatus) -> batcalc (100-disc),
 * price*(100-disc) -> hge, (100+tax), disc_price*(100+tax) -> hge ->
 * subsum x4 (hge), subcount, and the avg3 inputs (exact sums + counts). */
typedef struct {
	uint8_t rf, ls;
	ora_hge sum_qty, sum_price, sum_disc_price, sum_charge, sum_disc;
	int64_t cnt;
	int64_t nn_qty, nn_price, nn_disc;   /* non-nil counts: aggr.subavg skips nils */
} q1acc;

static int
q1_slice(const ora_lineitem *li, uint64_t row0, uint64_t n, q1acc *acc, int *nacc)
{
	ora_bat sd = view(ORA_date, li->shipdate, row0, n);
	ora_bat rf = view(ORA_str, li->returnflag, row0, n);
	ora_bat ls = view(ORA_str, li->linestatus, row0, n);
	ora_bat qt = view(ORA_lng, li->quantity, row0, n);
	ora_bat pr = view(ORA_lng, li->extendedprice, row0, n);
	ora_bat di = view(ORA_lng, li->discount, row0, n);
	ora_bat tx = view(ORA_lng, li->tax, row0, n);
	char heap[8192 + 24] = {0};
	rf.vheap = ls.vheap = heap;
	rf.vheapsize = ls.vheapsize = sizeof(heap);
	int32_t dmax = ora_mkdate(1998, 9, 2);
	int64_t hundred = 100;
	int rc = -1;
	ora_bat *c1 = NULL, *prf = NULL, *pls = NULL, *pq = NULL, *pp = NULL, *pd = NULL, *pt = NULL;
	ora_bat *g1 = NULL, *e1 = NULL, *h1 = NULL, *g2 = NULL, *e2 = NULL, *h2 = NULL;
	ora_bat *omd = NULL, *dp = NULL, *opt = NULL, *ch = NULL;
	ora_bat *s1 = NULL, *s2 = NULL, *s3 = NULL, *s4 = NULL, *s5 = NULL, *cn = NULL;
	ora_bat *nq = NULL, *np = NULL, *nd = NULL;
	ora_bat *krf = NULL, *kls = NULL;
	*nacc = 0;
	if ((c1 = ora_thetaselect(&sd, NULL, &dmax, "<=")) == NULL)
		goto out;
	if (c1->count == 0) {
		rc = 0;
		goto out;
	}
	if (!(prf = ora_project(c1, &rf)) || !(pls = ora_project(c1, &ls)) ||
	    !(pq = ora_project(c1, &qt)) || !(pp = ora_project(c1, &pr)) ||
	    !(pd = ora_project(c1, &di)) || !(pt = ora_project(c1, &tx)))
		goto out;
	if (ora_group(&g1, &e1, &h1, prf, NULL, NULL) < 0)
		goto out;
	if (ora_group(&g2, &e2, &h2, pls, NULL, g1) < 0)
		goto out;
	if (!(omd = ora_calc('-', NULL, &hundred, ORA_lng, pd, NULL, 0, NULL, ORA_lng)) ||
	    !(dp = ora_calc('*', pp, NULL, 0, omd, NULL, 0, NULL, ORA_hge)) ||
	    !(opt = ora_calc('+', NULL, &hundred, ORA_lng, pt, NULL, 0, NULL, ORA_lng)) ||
	    !(ch = ora_calc('*', dp, NULL, 0, opt, NULL, 0, NULL, ORA_hge)))
		goto out;
	if (!(s1 = ora_groupsum(pq, g2, e2, NULL, ORA_hge, true)) ||
	    !(s2 = ora_groupsum(pp, g2, e2, NULL, ORA_hge, true)) ||
	    !(s3 = ora_groupsum(dp, g2, e2, NULL, ORA_hge, true)) ||
	    !(s4 = ora_groupsum(ch, g2, e2, NULL, ORA_hge, true)) ||
	    !(s5 = ora_groupsum(pd, g2, e2, NULL, ORA_hge, true)) ||
	    !(cn = ora_groupcount(pq, g2, e2, NULL, false)) ||
	    !(nq = ora_groupcount(pq, g2, e2, NULL, true)) ||
	    !(np = ora_groupcount(pp, g2, e2, NULL, true)) ||
	    !(nd = ora_groupcount(pd, g2, e2, NULL, true)))
		goto out;
	if (!(krf = ora_project(e2, prf)) || !(kls = ora_project(e2, pls)))
		goto out;
	for (uint64_t k = 0; k < e2->count; k++) {
		q1acc *a = &acc[k];
		a->rf = ((uint8_t *) krf->base)[k];
		a->ls = ((uint8_t *) kls->base)[k];
		a->sum_qty = ((ora_hge *) s1->base)[k];
		a->sum_price = ((ora_hge *) s2->base)[k];
		a->sum_disc_price = ((ora_hge *) s3->base)[k];
		a->sum_charge = ((ora_hge *) s4->base)[k];
		a->sum_disc = ((ora_hge *) s5->base)[k];
		a->cnt = ((int64_t *) cn->base)[k];
		a->nn_qty = ((int64_t *) nq->base)[k];
		a->nn_price = ((int64_t *) np->base)[k];
		a->nn_disc = ((int64_t *) nd->base)[k];
	}
	*nacc = (int) e2->count;
	rc = 0;
out:
	ora_free(c1); ora_free(prf); ora_free(pls); ora_free(pq); ora_free(pp); ora_free(pd); ora_free(pt);
	ora_free(g1); ora_free(e1); ora_free(h1); ora_free(g2); ora_free(e2); ora_free(h2);
	ora_free(omd); ora_free(dp); ora_free(opt); ora_free(ch);
	ora_free(s1); ora_free(s2); ora_free(s3); ora_free(s4); ora_free(s5); ora_free(cn);
	ora_free(nq); ora_free(np); ora_free(nd);
	ora_free(krf); ora_free(kls);
	return rc;
}

/* avg3 of an exact sum: floor division then round half away from zero
 * (gdk/gdk_aggr.c:2070-2095, BATgroupavg3combine :2634 gives the same for
 * combined partials since the sums are exact) */
static void
avg_round(ora_hge s, int64_t n, int64_t *avg, int64_t *rem)
{
	ora_hge q = s / n, r = s % n;
	if (r < 0) {
		q -= 1;
		r += n;
	}
	if (r > 0) {
		if (q < 0) {
			if (2 * r > n) { q++; r -= n; }
		} else if (2 * r >= n) {
			q++;
			r -= n;
		}
	}
	*avg = (int64_t) q;
	*rem = (int64_t) r;
}

int
ora_q1(const ora_lineitem *li, int nthreads, ora_q1row *rows, int *nrows)
{
	if (nthreads < 1)
		nthreads = 1;
	q1acc *part = calloc((size_t) nthreads * 16, sizeof(q1acc));
	int *np = calloc((size_t) nthreads, sizeof(int));
	int err = 0;
#pragma omp parallel for num_threads(nthreads) reduction(|:err) schedule(static, 1)
	for (int t = 0; t < nthreads; t++) {
		uint64_t a = li->n * (uint64_t) t / (uint64_t) nthreads;
		uint64_t b = li->n * (uint64_t) (t + 1) / (uint64_t) nthreads;
		if (q1_slice(li, a, b - a, part + (size_t) t * 16, &np[t]) < 0) {
			err |= 1;
#pragma omp critical
			snprintf(shared_err, sizeof(shared_err), "%s", ora_errbuf());
		}
	}
	/* mergetable: re-group the packed partials by key (first occurrence
	 * over slices in order), re-aggregate */
	q1acc fin[16];
	int nf = 0;
	for (int t = 0; t < nthreads && !err; t++) {
		for (int k = 0; k < np[t]; k++) {
			q1acc *a = &part[(size_t) t * 16 + k];
			int f;
			for (f = 0; f < nf; f++)
				if (fin[f].rf == a->rf && fin[f].ls == a->ls)
					break;
			if (f == nf) {
				memset(&fin[nf], 0, sizeof(q1acc));
				fin[nf].rf = a->rf;
				fin[nf].ls = a->ls;
				nf++;
			}
			fin[f].sum_qty += a->sum_qty;
			fin[f].sum_price += a->sum_price;
			fin[f].sum_disc_price += a->sum_disc_price;
			fin[f].sum_charge += a->sum_charge;
			fin[f].sum_disc += a->sum_disc;
			fin[f].cnt += a->cnt;
			fin[f].nn_qty += a->nn_qty;
			fin[f].nn_price += a->nn_price;
			fin[f].nn_disc += a->nn_disc;
		}
	}
	free(part);
	free(np);
	if (err) {
		ora_seterr("%s", shared_err);
		return -1;
	}
	/* ORDER BY l_returnflag, l_linestatus: heap offsets are assigned in
	 * alphabetical order (A<N<R, F<O) */
	for (int i = 0; i < nf; i++)
		for (int j = i + 1; j < nf; j++)
			if (fin[j].rf < fin[i].rf || (fin[j].rf == fin[i].rf && fin[j].ls < fin[i].ls)) {
				q1acc tmp = fin[i];
				fin[i] = fin[j];
				fin[j] = tmp;
			}
	for (int i = 0; i < nf; i++) {
		ora_q1row *r = &rows[i];
		memset(r, 0, sizeof(*r));
		r->returnflag = fin[i].rf;
		r->linestatus = fin[i].ls;
		r->sum_qty = fin[i].sum_qty;
		r->sum_base_price = fin[i].sum_price;
		r->sum_disc_price = fin[i].sum_disc_price;
		r->sum_charge = fin[i].sum_charge;
		r->count_order = fin[i].cnt;
		/* BATgroupavg3 over the non-nil values (gdk_aggr.c:1996-2095); a
		 * group of nils only is nil (not reached by the tests) */
		if (fin[i].nn_qty)
			avg_round(fin[i].sum_qty, fin[i].nn_qty, &r->avg_qty, &r->rem_qty);
		if (fin[i].nn_price)
			avg_round(fin[i].sum_price, fin[i].nn_price, &r->avg_price, &r->rem_price);
		if (fin[i].nn_disc)
			avg_round(fin[i].sum_disc, fin[i].nn_disc, &r->avg_disc, &r->rem_disc);
	}
	*nrows = nf;
	return 0;
}
