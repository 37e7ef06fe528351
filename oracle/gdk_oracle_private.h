/*
 * gdk_oracle_private.h -- helpers shared by the oracle's translation units.
 * TEST INFRASTRUCTURE ONLY (see gdk_oracle.h).
 */
#ifndef GDK_ORACLE_PRIVATE_H
#define GDK_ORACLE_PRIVATE_H

#include "gdk_oracle.h"

/* a candidate iterator (gdk/gdk_cand.c:407 canditer_init) restated as an
 * explicit dense (seq, n) range or a clipped sorted oid array */
typedef struct {
	bool dense;
	ora_oid seq;          /* dense: first candidate */
	const ora_oid *oids;  /* materialized: first candidate */
	uint64_t n;
} ora_ci;

static inline ora_oid
ci_get(const ora_ci *ci, uint64_t i)
{
	return ci->dense ? ci->seq + i : ci->oids[i];
}

int ora_ci_init(ora_ci *ci, const ora_bat *b, const ora_bat *s);
void ora_seterr(const char *fmt, ...);
int ora_width(int type);
ora_bat *ora_dense(ora_oid hseq, ora_oid tseq, uint64_t cnt);

#endif
