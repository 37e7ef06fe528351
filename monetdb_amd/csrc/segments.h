// segments.h -- sorted lists of segment (partition / peer-group) starts
// from a bit column, shared by the window kernels (analytic_func.hip,
// analytic_win.hip): the reference walks its np / op arrays row by row
// (gdk/gdk_analytic_func.c); the device finds a row's segment by binary
// search over the compacted starts.
#pragma once

#include "mgdk_internal.h"

namespace mgdk {

// sorted list of segment starts (row 0 always first)
struct Starts {
	const oid *L;        // NULL: dense Lseq + k
	oid Lseq;
	BUN m;               // entries, including a virtual row 0 when lead
	bool lead;
	BUN n;
	__device__ __forceinline__ oid at(BUN k) const
	{
		if (lead) {
			if (k == 0)
				return 0;
			k--;
		}
		return L ? L[k] : Lseq + k;
	}
	// index of the segment holding row i
	__device__ __forceinline__ BUN idx(BUN i) const
	{
		BUN lo = 0, hi = m;
		while (hi - lo > 1) {
			const BUN mid = (lo + hi) / 2;
			if (at(mid) <= i)
				lo = mid;
			else
				hi = mid;
		}
		return lo;
	}
	__device__ __forceinline__ BUN end_of(BUN k) const { return k + 1 < m ? at(k + 1) : n; }
	// [start, end) of the segment holding row i
	__device__ __forceinline__ void seg(BUN i, BUN &s, BUN &e) const
	{
		BUN lo = 0, hi = m;
		while (hi - lo > 1) {
			const BUN mid = (lo + hi) / 2;
			if (at(mid) <= i)
				lo = mid;
			else
				hi = mid;
		}
		s = at(lo);
		e = lo + 1 < m ? at(lo + 1) : n;
	}
};

// starts list from flags (nonzero = start); row 0 is always a start.
// *keep owns the compacted list (unfix it after the kernels that read it)
int make_starts(const int8_t *flags, BUN n, Starts &st, mgdk_bat **keep);

}  // namespace mgdk
