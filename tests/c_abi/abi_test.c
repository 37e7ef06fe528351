/*
 * abi_test.c -- a C99 caller of libmgdk.so through include/mgdk.h only, the
 * way a GDK adaptor calls it: no Python, no C++.
 *
 *   select:  s = BATthetaselect(b, NULL, &v, "<")        (gdk_select.c:2103)
 *   project: p = BATproject(s, c)                         (gdk_project.c:857)
 *   sum:     BATsum(&res, TYPE_lng, p, NULL, true, true)  (gdk_aggr.c:1018)
 *   error:   BATcalcmulcst overflow -> NULL + "22003!overflow in calculation ..."
 *            in GDKerrbuf (gdk_calc_mul.c, gdk.h:1947), then GDKclrerr
 *
 * Inputs are generated here, uploaded, the results downloaded and checked
 * against plain C loops.  Exit 0 = every check passed; the last stdout line
 * is "abi ok".
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mgdk.h"

#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
	fprintf(stderr, __VA_ARGS__); fprintf(stderr, " [%s]\n", mgdk_GDKerrbuf()); return 1; } } while (0)

int
main(void)
{
	const mgdk_BUN n = 1000003;
	int32_t *a = malloc(n * sizeof(int32_t));
	int64_t *c = malloc(n * sizeof(int64_t));
	uint64_t x = 88172645463325252ULL;
	for (mgdk_BUN i = 0; i < n; i++) {
		x ^= x << 13; x ^= x >> 7; x ^= x << 17;      /* xorshift64 */
		a[i] = (int32_t) (x % 1000);
		c[i] = (int64_t) (x >> 20) % 100000 - 50000;
	}
	CHECK(mgdk_init(0) == 0, "mgdk_init");
	mgdk_bat *b = mgdk_COLnew(0, MGDK_int, n), *v = mgdk_COLnew(0, MGDK_lng, n);
	CHECK(b && v, "COLnew");
	CHECK(mgdk_BATupload(b, a, n) == 0 && mgdk_BATupload(v, c, n) == 0, "upload");
	b->tnonil = v->tnonil = 1;
	b->tsorted = b->trevsorted = b->tkey = 0;
	v->tsorted = v->trevsorted = v->tkey = 0;

	/* select a < 100, project c, sum */
	int32_t thr = 100;
	mgdk_bat *s = mgdk_BATthetaselect(b, NULL, &thr, "<");
	CHECK(s != NULL, "BATthetaselect");
	mgdk_BUN want_hits = 0;
	int64_t want_sum = 0;
	for (mgdk_BUN i = 0; i < n; i++)
		if (a[i] < thr) {
			want_hits++;
			want_sum += c[i];
		}
	CHECK(s->count == want_hits, "hits %" PRIu64 " != %" PRIu64, (uint64_t) s->count, (uint64_t) want_hits);
	CHECK(s->ttype == MGDK_oid || s->ttype == MGDK_void, "select result type %d", s->ttype);
	mgdk_oid *oids = malloc((s->count + 1) * sizeof(mgdk_oid));
	CHECK(mgdk_BATdownload(s, oids) == 0, "download oids");
	for (mgdk_BUN i = 0, k = 0; i < n; i++)
		if (a[i] < thr) {
			CHECK(oids[k] == i, "oid %" PRIu64 " at %" PRIu64, (uint64_t) oids[k], (uint64_t) k);
			k++;
		}
	mgdk_bat *p = mgdk_BATproject(s, v);
	CHECK(p != NULL && p->count == want_hits && p->ttype == MGDK_lng, "BATproject");
	int64_t got = 0;
	CHECK(mgdk_BATsum(&got, MGDK_lng, p, NULL, true, true) == 0, "BATsum");
	CHECK(got == want_sum, "sum %" PRId64 " != %" PRId64, got, want_sum);

	/* forced overflow: lng * 2^62 -> NULL and the reference's message */
	mgdk_GDKclrerr();
	int64_t big = (int64_t) 1 << 62;
	mgdk_bat *o = mgdk_BATcalcmulcst(v, &big, MGDK_lng, NULL, MGDK_lng);
	CHECK(o == NULL, "overflow not reported");
	CHECK(strncmp(mgdk_GDKerrbuf(), "22003!overflow in calculation", 29) == 0, "message '%s'", mgdk_GDKerrbuf());
	mgdk_GDKclrerr();
	CHECK(mgdk_GDKerrbuf()[0] == 0, "GDKclrerr");
	/* the library still works after the error */
	mgdk_bat *s2 = mgdk_BATthetaselect(b, NULL, &thr, ">=");
	CHECK(s2 != NULL && s2->count == n - want_hits, "select after error");

	mgdk_BBPunfix(s2);
	mgdk_BBPunfix(p);
	mgdk_BBPunfix(s);
	mgdk_BBPunfix(v);
	mgdk_BBPunfix(b);
	free(oids);
	free(a);
	free(c);
	printf("hits %" PRIu64 " sum %" PRId64 "\nabi ok\n", (uint64_t) want_hits, want_sum);
	return 0;
}
