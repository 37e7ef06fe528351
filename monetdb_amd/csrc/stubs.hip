// stubs.hip -- entry points whose device kernels are not built yet; they
// fail loudly with a GDK error (never a silent CPU fallback).
#include "mgdk_internal.h"

using namespace mgdk;

extern "C" {

int
mgdk_BATjoin(mgdk_bat **r1p, mgdk_bat **r2p, mgdk_bat *l, mgdk_bat *r, mgdk_bat *sl, mgdk_bat *sr,
	     bool nil_matches, mgdk_BUN estimate)
{
	(void) r1p; (void) r2p; (void) l; (void) r; (void) sl; (void) sr; (void) nil_matches; (void) estimate;
	seterr("42000!BATjoin: device hash join not built yet");
	return -1;
}

int
mgdk_BATsort(mgdk_bat **sorted, mgdk_bat **order, mgdk_bat **groups, mgdk_bat *b, mgdk_bat *o, mgdk_bat *g,
	     bool reverse, bool nilslast, bool stable)
{
	(void) sorted; (void) order; (void) groups; (void) b; (void) o; (void) g; (void) reverse; (void) nilslast; (void) stable;
	seterr("42000!BATsort: device sort not built yet");
	return -1;
}

int
mgdk_GDKanalyticalwindowbounds(mgdk_bat *r, mgdk_bat *b, mgdk_bat *p, mgdk_bat *l, const void *bound, int tp1,
			       int tp2, int unit, bool preceding, mgdk_oid first_half)
{
	(void) r; (void) b; (void) p; (void) l; (void) bound; (void) tp1; (void) tp2; (void) unit; (void) preceding; (void) first_half;
	seterr("42000!GDKanalyticalwindowbounds: device kernel not built yet");
	return -1;
}

}  // extern "C"
