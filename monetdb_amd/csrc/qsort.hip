// qsort.hip -- GDKqsort's permutation on the MI355X (gdk/gdk_qsort.c,
// gdk/gdk_qsort_impl.h:61-204: Bentley & McIlroy's three-way quicksort with
// INSERTSORT = 60 and the "no swap: insertion sort below 1024" shortcut).
//
// An unstable BATsort returns the values in order but equal values in the
// order the quicksort's swaps leave them (do_sort, gdk_batop.c:2266-2304).
// The device reproduces that permutation exactly.  Every decision of the
// algorithm is a comparison, so it runs on each row's dense RANK in the
// requested order (equal values = equal ranks, computed by the stable sort
// that precedes the replay); the payload is the row's oid.
//
// Segments (the runs the reference sorts separately) are replayed
//   - below 60 rows: insertion sort = a stable sort of the current
//     arrangement (batched: one radix sort of (segment start, rank));
//   - 60 .. SEQMAX rows: one thread runs the reference's loop on its
//     segment;
//   - above SEQMAX rows: one partition step per level for all such segments
//     at once (below), their two sub-segments going to the next level.
//
// One partition step in parallel.  After the pivot moves to position 0 the
// reference scans from the left (stopping at a value greater than the
// pivot) and from the right (stopping at a smaller one) and swaps the pair.
// The k-th greater value from the left meets the k-th smaller one from the
// right, so with g_k / l_k their positions there are S = #{k : g_k < l_k}
// swaps and the scans cross at B = min(g_{S+1}, l_S).  Left of B every
// position is seen once by the left scan: a smaller value (or the smaller
// value swapped in for g_k) is appended to the run [a, b) of smaller values,
// and an equal value, swapped to a, moves the run's FIRST element to its end
// -- a queue: append = push, equal = pop + push.  The queue ends ordered by
// each element's last push, i.e. it is the window [R, R + P) of a log in
// which push j stores its element and the r-th effective rotation stores a
// copy of log entry r; the copies are resolved by pointer jumping.  The
// right side is the mirror image.  The two block swaps that move the equal
// values to the middle are index maps.
#include <vector>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

constexpr uint32_t INSERTSORT = 60;
constexpr uint32_t SEQMAX = 160;

struct Seg {
	uint64_t start;
	uint32_t len;
	uint32_t _pad;
};

// ---- sequential replay (one thread per segment) ---------------------------
struct QS {
	uint32_t *r;
	uint64_t *p;
	__device__ bool lt(uint32_t i, uint32_t j) const { return r[i] < r[j]; }
	__device__ void swap(uint32_t i, uint32_t j) const
	{
		const uint32_t a = r[i];
		r[i] = r[j];
		r[j] = a;
		const uint64_t b = p[i];
		p[i] = p[j];
		p[j] = b;
	}
	__device__ uint32_t med3(uint32_t a, uint32_t b, uint32_t c) const
	{
		return lt(a, b) ? (lt(b, c) ? b : (lt(a, c) ? c : a)) : (lt(c, b) ? b : (lt(a, c) ? a : c));
	}
	__device__ void insertion(uint32_t n) const
	{
		for (uint32_t b = 1; b < n; b++)
			for (uint32_t a = b; a > 0 && lt(a, a - 1); a--)
				swap(a, a - 1);
	}
};

// gdk_qsort_impl.h:61-204 with the recursion on the smaller part as an
// explicit stack (its depth is at most log2 of the segment length)
__global__ __launch_bounds__(64) void
k_qs_seq(const Seg *segs, uint32_t nseg, uint32_t *rank, uint64_t *pay)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= nseg)
		return;
	struct Frame { uint32_t off, n; } stk[40];
	int top = 0;
	stk[top++] = {0, segs[k].len};
	uint32_t *const r0 = rank + segs[k].start;
	uint64_t *const p0 = pay + segs[k].start;
	while (top > 0) {
		Frame f = stk[--top];
		uint32_t off = f.off, n = f.n;
		for (;;) {
			QS q{r0 + off, p0 + off};
			if (n < INSERTSORT) {
				q.insertion(n);
				break;
			}
			uint32_t b = n >> 1, a = 0, c = n - 1;
			const uint32_t d0 = n >> 3;
			a = q.med3(a, a + d0, a + 2 * d0);
			b = q.med3(b - d0, b, b + d0);
			c = q.med3(c - 2 * d0, c - d0, c);
			b = q.med3(a, b, c);
			if (b != 0)
				q.swap(0, b);
			a = b = 1;
			c = n - 1;
			uint32_t d = n - 1;
			bool swap_cnt = false;
			for (;;) {
				while (b <= c && !q.lt(0, b)) {
					if (q.r[b] == q.r[0]) {
						swap_cnt = true;
						q.swap(a, b);
						a++;
					}
					b++;
				}
				while (b <= c && !q.lt(c, 0)) {
					if (q.r[0] == q.r[c]) {
						swap_cnt = true;
						q.swap(c, d);
						d--;
					}
					c--;
				}
				if (b > c)
					break;
				q.swap(b, c);
				swap_cnt = true;
				b++;
				c--;
			}
			if (!swap_cnt && n < 1024) {
				q.insertion(n);
				break;
			}
			uint32_t rr = a < b - a ? a : b - a;
			for (uint32_t z = 0; z < rr; z++)
				q.swap(z, b - rr + z);
			rr = d - c < n - d - 1 ? d - c : n - d - 1;
			for (uint32_t z = 0; z < rr; z++)
				q.swap(b + z, n - rr + z);
			const uint32_t nl = b - a, ng = d - c;
			if (nl < ng) {
				if (nl > 1)
					stk[top++] = {off, nl};
				if (ng <= 1)
					break;
				off += n - ng;
				n = ng;
			} else {
				if (ng > 1)
					stk[top++] = {off + n - ng, ng};
				if (nl <= 1)
					break;
				n = nl;
			}
		}
	}
}

// ---- segment classification ---------------------------------------------
// lists: 0 big (> SEQMAX), 1 sequential, 2 stable (insertion sort)
__global__ __launch_bounds__(256) void
k_qs_classify(const Seg *in, uint32_t n, Seg *big, Seg *seq, Seg *stab, uint32_t *cnt, uint32_t cap_big,
	      uint32_t cap_seq, uint32_t cap_stab)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const Seg s = in[i];
	if (s.len <= 1)
		return;
	if (s.len > SEQMAX) {
		const uint32_t k = atomicAdd(&cnt[0], 1u);
		if (k < cap_big)
			big[k] = s;
	} else if (s.len >= INSERTSORT) {
		const uint32_t k = atomicAdd(&cnt[1], 1u);
		if (k < cap_seq)
			seq[k] = s;
	} else {
		const uint32_t k = atomicAdd(&cnt[2], 1u);
		if (k < cap_stab)
			stab[k] = s;
	}
}

// ---- parallel partition step ---------------------------------------------
struct Part {
	uint64_t start;
	uint32_t n, pivot;
	uint64_t foff;            // flat offset of the segment
	uint64_t lo, go;          // global offsets of its smaller / greater lists
	uint32_t nl, ng;          // smaller / greater values (excluding the pivot)
	uint32_t S, B;            // swaps, crossing point
	uint32_t a, PL, RL;       // left: equal run incl. pivot, pushes, effective rotations
	uint32_t PR, RR, ER;      // right: pushes, effective rotations, equal values
	uint32_t firstpush, lastpush;
	uint64_t logL, logR;      // offsets of the two logs
	uint32_t mode;            // 0 partition, 1 stable (no swap below 1024 rows)
	uint32_t _pad;
};

__device__ __forceinline__ uint32_t
seg_of(const uint64_t *foff, uint32_t S, uint64_t f)
{
	uint32_t lo = 0, hi = S;           // last k with foff[k] <= f
	while (hi - lo > 1) {
		const uint32_t m = (lo + hi) >> 1;
		if (foff[m] <= f)
			lo = m;
		else
			hi = m;
	}
	return lo;
}

// pivot (median of three medians of three) moved to position 0
__global__ __launch_bounds__(64) void
k_qs_pivot(const Seg *big, uint32_t S, uint32_t *rank, uint64_t *pay, Part *part, const uint64_t *foff)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= S)
		return;
	const Seg s = big[k];
	QS q{rank + s.start, pay + s.start};
	const uint32_t n = s.len, d0 = n >> 3;
	uint32_t a = q.med3(0, d0, 2 * d0);
	uint32_t b = q.med3((n >> 1) - d0, n >> 1, (n >> 1) + d0);
	uint32_t c = q.med3(n - 1 - 2 * d0, n - 1 - d0, n - 1);
	b = q.med3(a, b, c);
	if (b != 0)
		q.swap(0, b);
	Part P{};
	P.start = s.start;
	P.n = n;
	P.pivot = q.r[0];
	P.foff = foff[k];
	part[k] = P;
}

__global__ __launch_bounds__(256) void
k_qs_flags(const Part *part, const uint64_t *foff, uint32_t S, uint64_t F, const uint32_t *rank, uint32_t *fseg,
	   uint8_t *fl, uint8_t *fg)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t f = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; f < F; f += stride) {
		const uint32_t k = seg_of(foff, S, f);
		fseg[f] = k;
		const uint32_t p = (uint32_t) (f - part[k].foff);
		const uint32_t r = rank[part[k].start + p];
		fl[f] = p > 0 && r < part[k].pivot;
		fg[f] = p > 0 && r > part[k].pivot;
	}
}

__global__ __launch_bounds__(256) void
k_qs_lists(const Part *part, uint64_t F, const uint32_t *fseg, const uint8_t *fl, const uint8_t *fg,
	   const uint64_t *exl, const uint64_t *exg, uint32_t *lpos, uint32_t *gpos)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t f = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; f < F; f += stride) {
		const Part &P = part[fseg[f]];
		const uint32_t p = (uint32_t) (f - P.foff);
		if (fg[f])
			gpos[exg[f]] = p;                                   // k-th greater from the left
		if (fl[f])
			lpos[P.lo + (P.nl - 1 - (exl[f] - P.lo))] = p;      // k-th smaller from the right
	}
}

// totals per segment (the flat scans at its first / next segment's first element)
__global__ __launch_bounds__(64) void
k_qs_totals(Part *part, uint32_t S, const uint64_t *exl, const uint64_t *exg, uint64_t totl, uint64_t totg)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= S)
		return;
	Part &P = part[k];
	P.lo = exl[P.foff];
	P.go = exg[P.foff];
	const uint64_t el = k + 1 < S ? exl[part[k + 1].foff] : totl;
	const uint64_t eg = k + 1 < S ? exg[part[k + 1].foff] : totg;
	P.nl = (uint32_t) (el - P.lo);
	P.ng = (uint32_t) (eg - P.go);
}

// S, B and the sizes of the two queues and logs; logs sized per segment
__global__ __launch_bounds__(64) void
k_qs_cross(Part *part, uint32_t S, const uint32_t *lpos, const uint32_t *gpos, uint32_t *logsz)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= S)
		return;
	Part &P = part[k];
	const uint32_t n = P.n, nl = P.nl, ng = P.ng;
	const uint32_t *G = gpos + P.go, *L = lpos + P.lo;
	// S = number of k with G[k-1] < L[k-1] (a prefix)
	uint32_t lo = 0, hi = nl < ng ? nl : ng;
	while (lo < hi) {
		const uint32_t m = (lo + hi + 1) >> 1;
		if (G[m - 1] < L[m - 1])
			lo = m;
		else
			hi = m - 1;
	}
	const uint32_t sw = lo;
	const uint32_t gnext = sw < ng ? G[sw] : 0xffffffffu;
	const uint32_t lS = sw > 0 ? L[sw - 1] : n;
	const uint32_t B = gnext < lS ? gnext : lS;
	P.S = sw;
	P.B = B;
	const uint32_t nE = n - 1 - nl - ng;
	if (sw == 0 && nE == 0 && n < 1024) {
		P.mode = 1;
		logsz[2 * k] = logsz[2 * k + 1] = 0;
		return;
	}
	P.mode = 0;
	// first / last position holding a smaller or greater value
	const uint32_t fL = nl ? L[nl - 1] : 0xffffffffu, fG = ng ? G[0] : 0xffffffffu;
	const uint32_t lL = nl ? L[0] : 0, lG = ng ? G[ng - 1] : 0;
	P.firstpush = fL < fG ? fL : fG;
	P.lastpush = nl + ng ? (lL > lG ? lL : lG) : 0;
	// the region sizes need the scans at B (k_qs_sizes)
	logsz[2 * k] = logsz[2 * k + 1] = 0;
}

// counts of the left region from the flat scans: X_before(p) = ex[foff + p] - base
__global__ __launch_bounds__(64) void
k_qs_sizes(Part *part, uint32_t S, const uint64_t *exl, const uint64_t *exg, uint64_t F, uint64_t totl,
	   uint64_t totg, uint32_t *logsz)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= S)
		return;
	Part &P = part[k];
	if (P.mode != 0)
		return;
	const uint32_t n = P.n, B = P.B;
	const uint64_t fB = P.foff + B;
	const uint64_t lB = fB < F ? exl[fB] : totl, gB = fB < F ? exg[fB] : totg;
	// B <= n; at B == n the next segment's first element (or the end) holds
	// the totals, which is what fB indexes
	const uint32_t Lb = (uint32_t) (lB - P.lo), Gb = (uint32_t) (gB - P.go);
	P.PL = Lb + Gb;
	const uint32_t EL = (B - 1) - P.PL;
	P.a = 1 + EL;
	P.RL = (P.PL > 0 && P.firstpush < B) ? EL - (P.firstpush - 1) : 0;
	P.PR = P.nl + P.ng - P.PL;
	P.ER = (n - B) - P.PR;
	P.RR = (P.PR > 0 && P.lastpush >= B) ? (P.lastpush - B) - (P.PR - 1) : 0;
	logsz[2 * k] = P.PL + P.RL;
	logsz[2 * k + 1] = P.PR + P.RR;
}

__global__ __launch_bounds__(64) void
k_qs_logoff(Part *part, uint32_t S, const uint64_t *logoff)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= S)
		return;
	part[k].logL = logoff[2 * k];
	part[k].logR = logoff[2 * k + 1];
}

// log entries: >= 0 an element (segment position), < 0 a copy of entry -e-1
__global__ __launch_bounds__(256) void
k_qs_log(const Part *part, uint64_t F, const uint32_t *fseg, const uint8_t *fl, const uint8_t *fg,
	 const uint64_t *exl, const uint64_t *exg, const uint32_t *lpos, const uint32_t *gpos, int64_t *log,
	 uint32_t *logseg)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t f = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; f < F; f += stride) {
		const uint32_t k = fseg[f];
		const Part &P = part[k];
		if (P.mode != 0)
			continue;
		const uint32_t p = (uint32_t) (f - P.foff);
		if (p == 0)
			continue;
		const bool isl = fl[f], isg = fg[f];
		const uint32_t Lb = (uint32_t) (exl[f] - P.lo), Gb = (uint32_t) (exg[f] - P.go);  // in [1, p)
		if (p < P.B) {
			const uint32_t Eb = (p - 1) - Lb - Gb;
			const uint32_t effb = p > P.firstpush && P.firstpush != 0xffffffffu ? Eb - (P.firstpush - 1) : 0;
			const uint64_t idx = P.logL + Lb + Gb + effb;
			if (isl) {
				log[idx] = p;
				logseg[idx] = k;
			} else if (isg) {
				log[idx] = lpos[P.lo + Gb];     // the Gb-th smaller value from the right
				logseg[idx] = k;
			} else if (p > P.firstpush && P.firstpush != 0xffffffffu) {
				log[idx] = -(int64_t) (P.logL + effb) - 1;
				logseg[idx] = k;
			}
		} else {
			// right region, scanned from n - 1 down: counts in (p, n)
			const uint32_t La = P.nl - Lb - isl, Ga = P.ng - Gb - isg;
			const uint32_t pa = La + Ga;
			const uint32_t Ea = (P.n - 1 - p) - pa;
			const uint32_t effa = p < P.lastpush ? Ea - (P.n - 1 - P.lastpush) : 0;
			const uint64_t idx = P.logR + pa + effa;
			if (isg) {
				log[idx] = p;
				logseg[idx] = k | 0x80000000u;
			} else if (isl) {
				log[idx] = gpos[P.go + La];     // the La-th greater value from the left
				logseg[idx] = k | 0x80000000u;
			} else if (p < P.lastpush) {
				log[idx] = -(int64_t) (P.logR + effa) - 1;
				logseg[idx] = k | 0x80000000u;
			}
		}
	}
}

__global__ __launch_bounds__(256) void
k_qs_jump(int64_t *log, uint64_t nlog, uint32_t *changed)
{
	uint32_t ch = 0;
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t j = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; j < nlog; j += stride) {
		const int64_t e = log[j];
		if (e < 0) {
			const int64_t e2 = __hip_atomic_load(&log[-e - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			log[j] = e2;
			ch |= e2 < 0;
		}
	}
	ch = block_reduce(ch, [](uint32_t x, uint32_t y) { return x | y; });
	if (threadIdx.x == 0)
		publish_or(changed, ch);
}

// the block swaps of gdk_qsort_impl.h:161-166 as a map of positions
__device__ __forceinline__ uint32_t
qs_final(const Part &P, uint32_t q)
{
	const uint32_t B = P.B, n = P.n;
	const uint32_t r1 = P.a < P.PL ? P.a : P.PL;
	const uint32_t r2 = P.PR < P.ER ? P.PR : P.ER;
	if (q < r1)
		return B - r1 + q;
	if (q >= B - r1 && q < B)
		return q - (B - r1);
	if (q >= B && q < B + r2)
		return n - r2 + (q - B);
	if (q >= n - r2)
		return B + (q - (n - r2));
	return q;
}

// pivot and equal values: placed by their position
__global__ __launch_bounds__(256) void
k_qs_place_eq(const Part *part, uint64_t F, const uint32_t *fseg, const uint8_t *fl, const uint8_t *fg,
	      const uint64_t *exl, const uint64_t *exg, const uint32_t *rank, const uint64_t *pay, uint32_t *nrank,
	      uint64_t *npay)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t f = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; f < F; f += stride) {
		const Part &P = part[fseg[f]];
		const uint32_t p = (uint32_t) (f - P.foff);
		if (P.mode != 0) {
			nrank[f] = rank[P.start + p];       // unchanged (stable-sorted later)
			npay[f] = pay[P.start + p];
			continue;
		}
		if (fl[f] || fg[f])
			continue;
		uint32_t q;
		if (p == 0) {
			q = 0;
		} else {
			const uint32_t Lb = (uint32_t) (exl[f] - P.lo), Gb = (uint32_t) (exg[f] - P.go);
			if (p < P.B) {
				q = 1 + (p - 1) - Lb - Gb;
			} else {
				const uint32_t pa = (P.nl - Lb) + (P.ng - Gb);
				const uint32_t Ea = (P.n - 1 - p) - pa;
				q = P.n - 1 - Ea;
			}
		}
		const uint64_t d = P.foff + qs_final(P, q);
		nrank[d] = rank[P.start + p];
		npay[d] = pay[P.start + p];
	}
}

// pushed values: placed by their queue slot
__global__ __launch_bounds__(256) void
k_qs_place_q(const Part *part, uint64_t nlog, const int64_t *log, const uint32_t *logseg, const uint32_t *rank,
	     const uint64_t *pay, uint32_t *nrank, uint64_t *npay)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t j = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; j < nlog; j += stride) {
		const uint32_t ks = logseg[j];
		const bool right = (ks & 0x80000000u) != 0;
		const Part &P = part[ks & 0x7fffffffu];
		uint32_t q;
		if (!right) {
			if (j < P.logL + P.RL)
				continue;                       // popped entries
			q = P.a + (uint32_t) (j - P.logL - P.RL);
		} else {
			if (j < P.logR + P.RR)
				continue;
			const uint32_t t = (uint32_t) (j - P.logR - P.RR);
			q = P.B + (P.PR - 1 - t);
		}
		const uint32_t e = (uint32_t) log[j];
		const uint64_t d = P.foff + qs_final(P, q);
		nrank[d] = rank[P.start + e];
		npay[d] = pay[P.start + e];
	}
}

__global__ __launch_bounds__(256) void
k_qs_back(const Part *part, const uint64_t *foff, uint32_t S, uint64_t F, const uint32_t *nrank,
	  const uint64_t *npay, uint32_t *rank, uint64_t *pay)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t f = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; f < F; f += stride) {
		const Part &P = part[seg_of(foff, S, f)];
		const uint64_t i = P.start + (f - P.foff);
		rank[i] = nrank[f];
		pay[i] = npay[f];
	}
}

// the next level's segments: the smaller and greater parts; stable ones
__global__ __launch_bounds__(64) void
k_qs_children(const Part *part, uint32_t S, Seg *out, uint32_t *cnt, Seg *stab, uint32_t *stabcnt)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= S)
		return;
	const Part &P = part[k];
	if (P.mode == 1) {
		stab[atomicAdd(stabcnt, 1u)] = Seg{P.start, P.n, 0};
		return;
	}
	const uint32_t nlt = P.B - P.a, ngt = P.PR;
	if (nlt > 1)
		out[atomicAdd(cnt, 1u)] = Seg{P.start, nlt, 0};
	if (ngt > 1)
		out[atomicAdd(cnt, 1u)] = Seg{P.start + P.n - ngt, ngt, 0};
}

// ---- stable sort of short segments (insertion sort) ---------------------
__global__ __launch_bounds__(256) void
k_qs_mark(const Seg *segs, uint32_t nseg, uint8_t *mark)
{
	const uint32_t k = blockIdx.x;
	if (k >= nseg)
		return;
	const Seg s = segs[k];
	for (uint32_t i = threadIdx.x; i < s.len; i += blockDim.x)
		mark[s.start + i] = 1 + (i == 0);       // 2: first row of a segment
}

__global__ __launch_bounds__(256) void
k_qs_stkeys(BUN n, const uint8_t *mark, const uint64_t *ex, const uint32_t *rank, uint64_t *key, uint32_t *pos,
	    uint64_t *segid_scan)
{
	// key = (segment number << 32) | rank; the segment number is the count
	// of segment starts up to here (segid_scan: inclusive count of marks==2)
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
		if (!mark[i])
			continue;
		const uint64_t j = ex[i];
		key[j] = (segid_scan[i] << 32) | rank[i];
		pos[j] = (uint32_t) i;
	}
}

__global__ __launch_bounds__(256) void
k_qs_stgather(uint64_t m, const uint32_t *slot, const uint32_t *src, const uint32_t *rank, const uint64_t *pay,
	      uint32_t *trank, uint64_t *tpay)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t j = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
		trank[j] = rank[src[j]];
		tpay[j] = pay[src[j]];
	}
}

__global__ __launch_bounds__(256) void
k_qs_stscatter(uint64_t m, const uint32_t *slot, const uint32_t *trank, const uint64_t *tpay, uint32_t *rank,
	       uint64_t *pay)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t j = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
		rank[slot[j]] = trank[j];
		pay[slot[j]] = tpay[j];
	}
}

__global__ __launch_bounds__(256) void
k_qs_startflags(BUN n, const uint8_t *mark, uint8_t *st)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
		st[i] = mark[i] == 2;
}

__global__ __launch_bounds__(256) void
k_qs_ismark(BUN n, const uint8_t *mark, uint8_t *m1)
{
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
		m1[i] = mark[i] != 0;
}

__global__ __launch_bounds__(256) void
k_qs_segid(BUN n, const uint8_t *st, uint64_t *ex)
{
	// inclusive = exclusive + own flag, minus 1: the segment number
	const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
	for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
		ex[i] = ex[i] + st[i] - 1;
}

int
stable_segments(uint32_t *rank, uint64_t *pay, BUN n, const Seg *segs, uint32_t nseg)
{
	if (nseg == 0)
		return 0;
	hipStream_t st = stream();
	DevBuf mark(n), m1(n), sflag(n), ex(n * 8), sid(n * 8);
	if (!mark.p || !m1.p || !sflag.p || !ex.p || !sid.p)
		return -1;
	if (!hip_ok(hipMemsetAsync(mark.p, 0, n, st), "memset"))
		return -1;
	hipLaunchKernelGGL(k_qs_mark, dim3(nseg), dim3(64), 0, st, segs, nseg, mark.as<uint8_t>());
	const dim3 grd(grid_for(n, 1024, 8192)), blk(256);
	hipLaunchKernelGGL(k_qs_ismark, grd, blk, 0, st, n, mark.as<uint8_t>(), m1.as<uint8_t>());
	hipLaunchKernelGGL(k_qs_startflags, grd, blk, 0, st, n, mark.as<uint8_t>(), sflag.as<uint8_t>());
	uint64_t m = 0, ns = 0;
	if (exclusive_scan(m1.as<uint8_t>(), ex.as<uint64_t>(), n, &m) < 0 ||
	    exclusive_scan(sflag.as<uint8_t>(), sid.as<uint64_t>(), n, &ns) < 0)
		return -1;
	hipLaunchKernelGGL(k_qs_segid, grd, blk, 0, st, n, sflag.as<uint8_t>(), sid.as<uint64_t>());
	DevBuf k0(m * 8), k1(m * 8), v0(m * 4), v1(m * 4), slot(m * 4), tr(m * 4), tp(m * 8);
	if (!k0.p || !k1.p || !v0.p || !v1.p || !slot.p || !tr.p || !tp.p)
		return -1;
	hipLaunchKernelGGL(k_qs_stkeys, grd, blk, 0, st, n, mark.as<uint8_t>(), ex.as<uint64_t>(), rank,
			   k0.as<uint64_t>(), v0.as<uint32_t>(), sid.as<uint64_t>());
	// slots = the positions in order (v0 before sorting)
	if (!hip_ok(hipMemcpyAsync(slot.p, v0.p, m * 4, hipMemcpyDeviceToDevice, st), "memcpy"))
		return -1;
	uint64_t *ko;
	uint32_t *vo;
	if (radix_sort_pairs(k0.as<uint64_t>(), v0.as<uint32_t>(), k1.as<uint64_t>(), v1.as<uint32_t>(), m, 64, &ko,
			     &vo) < 0)
		return -1;
	const dim3 g2(grid_for(m, 1024, 8192));
	hipLaunchKernelGGL(k_qs_stgather, g2, blk, 0, st, m, slot.as<uint32_t>(), vo, rank, pay, tr.as<uint32_t>(),
			   tp.as<uint64_t>());
	hipLaunchKernelGGL(k_qs_stscatter, g2, blk, 0, st, m, slot.as<uint32_t>(), tr.as<uint32_t>(), tp.as<uint64_t>(),
			   rank, pay);
	return sync() ? 0 : -1;
}

}  // namespace

namespace mgdk {

// GDKqsort of every segment of (rank, pay); segs: host list of (start, len)
int
qsort_replay(uint32_t *rank, uint64_t *pay, BUN n, const std::vector<std::pair<uint64_t, uint32_t>> &segs0)
{
	hipStream_t st = stream();
	if (segs0.empty() || n == 0)
		return 0;
	const uint32_t cap = (uint32_t) (n / 2 + 2);   // segments hold >= 2 rows
	DevBuf cur(cap * sizeof(Seg)), big(cap * sizeof(Seg)), seq(cap * sizeof(Seg)), stab(cap * sizeof(Seg));
	DevBuf cnt(64);
	if (!cur.p || !big.p || !seq.p || !stab.p || !cnt.p)
		return -1;
	std::vector<Seg> hs;
	for (auto &s : segs0)
		if (s.second > 1)
			hs.push_back(Seg{s.first, s.second, 0});
	uint32_t ncur = (uint32_t) hs.size();
	if (ncur == 0)
		return 0;
	if (!hip_ok(hipMemcpyAsync(cur.p, hs.data(), ncur * sizeof(Seg), hipMemcpyHostToDevice, st), "memcpy"))
		return -1;
	uint32_t hc[4];
	// small device -> host reads through the thread's pinned buffer
	auto rd = [&](const void *dev, size_t bytes) {
		void *h = pinned(64);
		if (h == nullptr || !hip_ok(hipMemcpyAsync(h, dev, bytes, hipMemcpyDeviceToHost, st), "memcpy") || !sync())
			return false;
		memcpy(hc, h, bytes);
		return true;
	};
	uint32_t nseq = 0, nstab = 0;
	for (int level = 0; ncur > 0; level++) {
		// classify the current segments (seq / stab lists grow across levels)
		uint32_t init[4] = {0, nseq, nstab, 0};
		if (!hip_ok(hipMemcpyAsync(cnt.p, init, 16, hipMemcpyHostToDevice, st), "memcpy"))
			return -1;
		hipLaunchKernelGGL(k_qs_classify, dim3(grid_for(ncur, 256)), dim3(256), 0, st, cur.as<Seg>(), ncur,
				   big.as<Seg>(), seq.as<Seg>(), stab.as<Seg>(), cnt.as<uint32_t>(), cap, cap, cap);
		if (!rd(cnt.p, 16))
			return -1;
		const uint32_t S = hc[0];
		nseq = hc[1];
		nstab = hc[2];
		if (S == 0)
			break;
		// flat offsets of the big segments
		std::vector<Seg> hb(S);
		if (!hip_ok(hipMemcpyAsync(hb.data(), big.p, S * sizeof(Seg), hipMemcpyDeviceToHost, st), "memcpy") ||
		    !sync())
			return -1;
		std::vector<uint64_t> hfoff(S);
		uint64_t F = 0;
		for (uint32_t k = 0; k < S; k++) {
			hfoff[k] = F;
			F += hb[k].len;
		}
		DevBuf foff(S * 8), part(S * sizeof(Part)), fseg(F * 4), fl(F), fg(F), exl(F * 8), exg(F * 8);
		DevBuf lpos(F * 4), gpos(F * 4), logsz(S * 8), logoff(S * 16), nr(F * 4), np(F * 8), flag(16);
		if (!foff.p || !part.p || !fseg.p || !fl.p || !fg.p || !exl.p || !exg.p || !lpos.p || !gpos.p ||
		    !logsz.p || !logoff.p || !nr.p || !np.p || !flag.p)
			return -1;
		if (!hip_ok(hipMemcpyAsync(foff.p, hfoff.data(), S * 8, hipMemcpyHostToDevice, st), "memcpy"))
			return -1;
		const dim3 gs(grid_for(S, 64)), bs(64), gf(grid_for(F, 1024, 8192)), bf(256);
		Part *pt = part.as<Part>();
		hipLaunchKernelGGL(k_qs_pivot, gs, bs, 0, st, big.as<Seg>(), S, rank, pay, pt, foff.as<uint64_t>());
		hipLaunchKernelGGL(k_qs_flags, gf, bf, 0, st, pt, foff.as<uint64_t>(), S, F, rank, fseg.as<uint32_t>(),
				   fl.as<uint8_t>(), fg.as<uint8_t>());
		uint64_t totl = 0, totg = 0;
		if (exclusive_scan(fl.as<uint8_t>(), exl.as<uint64_t>(), F, &totl) < 0 ||
		    exclusive_scan(fg.as<uint8_t>(), exg.as<uint64_t>(), F, &totg) < 0)
			return -1;
		hipLaunchKernelGGL(k_qs_totals, gs, bs, 0, st, pt, S, exl.as<uint64_t>(), exg.as<uint64_t>(), totl, totg);
		hipLaunchKernelGGL(k_qs_lists, gf, bf, 0, st, pt, F, fseg.as<uint32_t>(), fl.as<uint8_t>(), fg.as<uint8_t>(),
				   exl.as<uint64_t>(), exg.as<uint64_t>(), lpos.as<uint32_t>(), gpos.as<uint32_t>());
		hipLaunchKernelGGL(k_qs_cross, gs, bs, 0, st, pt, S, lpos.as<uint32_t>(), gpos.as<uint32_t>(),
				   logsz.as<uint32_t>());
		hipLaunchKernelGGL(k_qs_sizes, gs, bs, 0, st, pt, S, exl.as<uint64_t>(), exg.as<uint64_t>(), F, totl, totg,
				   logsz.as<uint32_t>());
		uint64_t nlog = 0;
		if (exclusive_scan(logsz.as<uint32_t>(), logoff.as<uint64_t>(), 2 * (BUN) S, &nlog) < 0)
			return -1;
		hipLaunchKernelGGL(k_qs_logoff, gs, bs, 0, st, pt, S, logoff.as<uint64_t>());
		DevBuf log(nlog * 8 + 8), logseg(nlog * 4 + 4);
		if (!log.p || !logseg.p)
			return -1;
		hipLaunchKernelGGL(k_qs_log, gf, bf, 0, st, pt, F, fseg.as<uint32_t>(), fl.as<uint8_t>(), fg.as<uint8_t>(),
				   exl.as<uint64_t>(), exg.as<uint64_t>(), lpos.as<uint32_t>(), gpos.as<uint32_t>(),
				   log.as<int64_t>(), logseg.as<uint32_t>());
		// resolve the copies
		for (int round = 0; nlog > 0; round++) {
			if (round > 64) {
				seterr("42000!BATsort: quicksort replay did not converge");
				return -1;
			}
			if (!hip_ok(hipMemsetAsync(flag.p, 0, 4, st), "memset"))
				return -1;
			hipLaunchKernelGGL(k_qs_jump, dim3(grid_for(nlog, 1024, 8192)), bf, 0, st, log.as<int64_t>(), nlog,
					   flag.as<uint32_t>());
			if (!rd(flag.p, 4))
				return -1;
			if (hc[0] == 0)
				break;
		}
		hipLaunchKernelGGL(k_qs_place_eq, gf, bf, 0, st, pt, F, fseg.as<uint32_t>(), fl.as<uint8_t>(),
				   fg.as<uint8_t>(), exl.as<uint64_t>(), exg.as<uint64_t>(), rank, pay, nr.as<uint32_t>(),
				   np.as<uint64_t>());
		if (nlog)
			hipLaunchKernelGGL(k_qs_place_q, dim3(grid_for(nlog, 1024, 8192)), bf, 0, st, pt, nlog,
					   log.as<int64_t>(), logseg.as<uint32_t>(), rank, pay, nr.as<uint32_t>(),
					   np.as<uint64_t>());
		hipLaunchKernelGGL(k_qs_back, gf, bf, 0, st, pt, foff.as<uint64_t>(), S, F, nr.as<uint32_t>(),
				   np.as<uint64_t>(), rank, pay);
		// next level: children of the big segments (stable ones appended)
		uint32_t init2[4] = {0, nstab, 0, 0};
		if (!hip_ok(hipMemcpyAsync(cnt.p, init2, 16, hipMemcpyHostToDevice, st), "memcpy"))
			return -1;
		hipLaunchKernelGGL(k_qs_children, gs, bs, 0, st, pt, S, cur.as<Seg>(), cnt.as<uint32_t>(), stab.as<Seg>(),
				   cnt.as<uint32_t>() + 1);
		if (!rd(cnt.p, 16))
			return -1;
		ncur = hc[0];
		nstab = hc[1];
	}
	if (nseq)
		hipLaunchKernelGGL(k_qs_seq, dim3(grid_for(nseq, 64)), dim3(64), 0, st, seq.as<Seg>(), nseq, rank, pay);
	if (stable_segments(rank, pay, n, stab.as<Seg>(), nstab) < 0)
		return -1;
	return sync() ? 0 : -1;
}

}  // namespace mgdk
