// runtime.hip -- HBM heap allocator, per-thread streams, error buffer, BAT
// descriptors and candidate-list plumbing for libmgdk.so.
//
// Mirrors the GDK runtime conventions the operators rely on:
//   GDKerror / GDKerrbuf thread-local messages   gdk/gdk.h:1710,1947
//   HEAPalloc / GDKmalloc + memory accounting     gdk/gdk_heap.c:141-225, gdk/gdk_utils.c:1636,1752
//   COLnew / BATdense / BATslice / BBPunfix       gdk/gdk_bat.c:292,298, gdk/gdk_batop.c:1825, gdk/gdk_bbp.c:3149
//   canditer_init clipping                         gdk/gdk_cand.c:407
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <ctime>

#include "mgdk_internal.h"

namespace mgdk {

static thread_local char errbuf[2048];
static int g_device = 0;

void
seterr(const char *fmt, ...)
{
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(errbuf, sizeof(errbuf), fmt, ap);
	va_end(ap);
}

bool
hip_ok(hipError_t e, const char *what)
{
	if (e == hipSuccess)
		return true;
	seterr("HY013!HIP error %s in %s", hipGetErrorString(e), what);
	return false;
}

// ---- streams ----------------------------------------------------------------
struct ThreadCtx {
	hipStream_t s = nullptr;
	hipStream_t s2 = nullptr;       // a side stream for independent passes of one operator
	hipEvent_t ev2 = nullptr, ev1 = nullptr;
	void *scratch = nullptr;
	size_t scratch_size = 0;
	void *pinned = nullptr;
	size_t pinned_size = 0;
	std::vector<void *> pinned_retired;   // outgrown pinned buffers (see pinned())
	void *meta = nullptr;
	void *stage = nullptr;          // pinned upload arena, reclaimed at sync()
	size_t stage_size = 0, stage_used = 0;
	~ThreadCtx() {
		if (stage)
			(void) hipHostFree(stage);
		if (meta)
			dfree(meta);
		if (scratch)
			dfree(scratch);
		if (pinned)
			(void) hipHostFree(pinned);
		for (void *q : pinned_retired)
			(void) hipHostFree(q);
		if (ev2)
			(void) hipEventDestroy(ev2);
		if (ev1)
			(void) hipEventDestroy(ev1);
		if (s2)
			(void) hipStreamDestroy(s2);
		if (s)
			(void) hipStreamDestroy(s);
	}
};
static thread_local ThreadCtx tctx;

hipStream_t
stream()
{
	if (tctx.s == nullptr) {
		(void) hipSetDevice(g_device);
		if (hipStreamCreateWithFlags(&tctx.s, hipStreamNonBlocking) != hipSuccess)
			tctx.s = nullptr;
	}
	return tctx.s;
}

// the thread's side stream; side_join() makes the main stream wait for what
// was queued on it (so a sync of the main stream covers both)
hipStream_t
stream2()
{
	if (tctx.s2 == nullptr) {
		(void) hipSetDevice(g_device);
		// MGDK_S2_PRIO=1: the side stream at the device's greatest priority
		// (its kernels' workgroups dispatched ahead of the main stream's)
		static const int prio = getenv("MGDK_S2_PRIO") ? atoi(getenv("MGDK_S2_PRIO")) : 0;
		int lo = 0, hi = 0;
		if (prio != 0 && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess && hi != lo) {
			if (hipStreamCreateWithPriority(&tctx.s2, hipStreamNonBlocking, hi) != hipSuccess)
				tctx.s2 = nullptr;
		} else if (hipStreamCreateWithFlags(&tctx.s2, hipStreamNonBlocking) != hipSuccess) {
			tctx.s2 = nullptr;
		}
		(void) hipGetLastError();
	}
	return tctx.s2;
}

bool
side_fork()
{
	if (tctx.s2 == nullptr)
		return true;
	if (tctx.ev1 == nullptr && hipEventCreateWithFlags(&tctx.ev1, hipEventDisableTiming) != hipSuccess) {
		tctx.ev1 = nullptr;
		return hip_ok(hipStreamSynchronize(stream()), "main stream sync");
	}
	return hip_ok(hipEventRecord(tctx.ev1, stream()), "main stream event") &&
	       hip_ok(hipStreamWaitEvent(tctx.s2, tctx.ev1, 0), "main stream wait");
}

bool
side_join()
{
	if (tctx.s2 == nullptr)
		return true;
	if (tctx.ev2 == nullptr && hipEventCreateWithFlags(&tctx.ev2, hipEventDisableTiming) != hipSuccess) {
		tctx.ev2 = nullptr;
		return hip_ok(hipStreamSynchronize(tctx.s2), "side stream sync");
	}
	return hip_ok(hipEventRecord(tctx.ev2, tctx.s2), "side stream event") &&
	       hip_ok(hipStreamWaitEvent(stream(), tctx.ev2, 0), "side stream wait");
}

// The calling thread's query context (MT_thread_set_qry_ctx,
// gdk/gdk_system.h:187-210): the reference tests it every
// CHECK_QRY_TIMEOUT_STEP iterations of its loops (TIMEOUT_LOOP, gdk.h:2420-
// 2462); a device operator tests it whenever it waits for its stream, i.e.
// between its launches, and fails the same way (GDK_FAIL / NULL with the
// TIMEOUT_MESSAGE text, gdk.h:2321-2346).
static thread_local mgdk_qryctx *qry_ctx;

static bool
qry_timed_out()
{
	mgdk_qryctx *qc = qry_ctx;
	if (qc == nullptr)
		return false;
	if (qc->endtime >= 0 && qc->endtime && mgdk_usec() > qc->endtime)
		qc->endtime = MGDK_QRY_TIMEOUT;
	switch (qc->endtime) {
	case MGDK_QRY_TIMEOUT: seterr("Timeout was reached!\n"); return true;
	case MGDK_QRY_INTERRUPT: seterr("Query interrupted!\n"); return true;
	case MGDK_QRY_DISCONNECT: seterr("Client is disconnected!\n"); return true;
	default: return false;
	}
}

// stream drain of a data transfer (upload / download / a host read of one
// value): the reference tests the query context only inside operator loops,
// so a client can still read back or clean up after a timeout
bool
sync_data()
{
	hipError_t e = hipStreamSynchronize(stream());
	tctx.stage_used = 0;                // every staged upload has been read
	if (e != hipSuccess)
		return hip_ok(e, "hipStreamSynchronize");
	return hip_ok(hipGetLastError(), "kernel launch");
}

// stream drain between an operator's launches: also tests the query context
bool
sync()
{
	return sync_data() && !qry_timed_out();
}

// ---- caching HBM allocator ---------------------------------------------------
// Sizes are rounded to a class (power of two up to 64 MiB, then 64 MiB
// multiples) and freed blocks are kept per class.  Every operator
// synchronises its stream before returning, so a cached block is never in
// use by an in-flight kernel when it is handed out again.
static std::mutex alloc_mu;
static std::map<size_t, std::vector<void *>> free_lists;
static std::map<void *, size_t> live;
static uint64_t cur_bytes = 0, cached_bytes = 0;

static size_t
size_class(size_t n)
{
	if (n < 256)
		return 256;
	const size_t big = (size_t) 64 << 20;
	if (n >= big)
		return (n + big - 1) / big * big;
	size_t c = 256;
	while (c < n)
		c <<= 1;
	return c;
}

void *
dalloc(size_t bytes)
{
	size_t c = size_class(bytes);
	{
		std::lock_guard<std::mutex> g(alloc_mu);
		auto it = free_lists.find(c);
		if (it != free_lists.end() && !it->second.empty()) {
			void *p = it->second.back();
			it->second.pop_back();
			live[p] = c;
			cur_bytes += c;
			cached_bytes -= c;
			return p;
		}
	}
	(void) hipSetDevice(g_device);
	void *p = nullptr;
	hipError_t e = hipMalloc(&p, c);
	if (e != hipSuccess) {
		mgdk_mem_release_cache();
		e = hipMalloc(&p, c);
	}
	if (e != hipSuccess) {
		seterr("HY013!Could not allocate space (%zu bytes in HBM)", c);
		return nullptr;
	}
	std::lock_guard<std::mutex> g(alloc_mu);
	live[p] = c;
	cur_bytes += c;
	return p;
}

void
dfree(void *p)
{
	if (p == nullptr)
		return;
	// A block goes back to the shared cache only once the freeing thread's
	// stream is idle: operators synchronise before they return, so this
	// costs one query on the normal path, and an error path that leaves
	// kernels in flight (reading or writing the block) drains them here
	// before another thread can be handed the block.
	if (tctx.s && hipStreamQuery(tctx.s) == hipErrorNotReady)
		(void) hipStreamSynchronize(tctx.s);
	std::lock_guard<std::mutex> g(alloc_mu);
	auto it = live.find(p);
	if (it == live.end())
		return;
	size_t c = it->second;
	live.erase(it);
	cur_bytes -= c;
	cached_bytes += c;
	free_lists[c].push_back(p);
}

void *
scratch(size_t bytes)
{
	if (tctx.scratch_size < bytes) {
		if (tctx.scratch)
			dfree(tctx.scratch);
		size_t n = bytes < ((size_t) 1 << 20) ? ((size_t) 1 << 20) : bytes;
		tctx.scratch = dalloc(n);
		tctx.scratch_size = tctx.scratch ? n : 0;
	}
	return tctx.scratch;
}

void *
meta_buf()
{
	if (tctx.meta == nullptr)
		tctx.meta = dalloc(4096);
	return tctx.meta;
}

void *
pinned(size_t bytes)
{
	if (tctx.pinned_size < bytes) {
		// an outgrown buffer is retired, not freed: a caller may hold it
		// across a nested operator that asks for more (it stays valid until
		// the thread ends; sizes at least double, so the retired buffers
		// together are never larger than the live one)
		if (tctx.pinned)
			tctx.pinned_retired.push_back(tctx.pinned);
		size_t n = bytes < (1u << 20) ? (size_t) 1 << 20 : bytes;
		if (n < 2 * tctx.pinned_size)
			n = 2 * tctx.pinned_size;
		if (hipHostMalloc(&tctx.pinned, n, hipHostMallocDefault) != hipSuccess) {
			tctx.pinned = nullptr;
			tctx.pinned_size = 0;
			seterr("HY013!Could not allocate pinned host memory");
			return nullptr;
		}
		tctx.pinned_size = n;
	}
	return tctx.pinned;
}

// Pinned staging for host->device copies that are not waited for one by
// one: an operator stages its small result columns, queues their copies and
// waits once.  The arena is reclaimed at the thread's next sync(); a request
// that does not fit waits for the queued copies first.
void *
stage_host(const void *src, size_t bytes)
{
	const size_t need = (bytes + 255) & ~(size_t) 255;
	if (tctx.stage_used + need > tctx.stage_size) {
		if (tctx.stage_used && !sync_data())
			return nullptr;
		if (need > tctx.stage_size) {
			if (tctx.stage)
				(void) hipHostFree(tctx.stage);
			size_t n = need < ((size_t) 1 << 20) ? ((size_t) 1 << 20) : need;
			if (hipHostMalloc(&tctx.stage, n, hipHostMallocDefault) != hipSuccess) {
				tctx.stage = nullptr;
				tctx.stage_size = 0;
				seterr("HY013!Could not allocate pinned host memory");
				return nullptr;
			}
			tctx.stage_size = n;
		}
	}
	char *d = (char *) tctx.stage + tctx.stage_used;
	tctx.stage_used += need;
	memcpy(d, src, bytes);
	return d;
}

const void *
zero_region()
{
	// created on first use; a failed allocation is retried by the next call
	static std::mutex mu;
	static void *volatile z = nullptr;
	if (z != nullptr)
		return z;
	std::lock_guard<std::mutex> g(mu);
	if (z == nullptr) {
		void *p = dalloc(ZERO_REGION);
		if (p && hipMemset(p, 0, ZERO_REGION) == hipSuccess && hipDeviceSynchronize() == hipSuccess)
			z = p;
		else
			dfree(p);
	}
	if (z == nullptr)
		seterr("HY013!could not allocate the zero region");
	return z;
}

// ---- profiling ---------------------------------------------------------------
static std::mutex prof_mu;
static std::map<std::string, std::pair<double, uint64_t>> prof;
static bool prof_on = false;

ProfScope::ProfScope(const char *n) : name(n), on(prof_on)
{
	if (on) {
		(void) hipEventCreate(&e0);
		(void) hipEventCreate(&e1);
		(void) hipEventRecord(e0, stream());
	}
}

ProfScope::~ProfScope()
{
	if (!on)
		return;
	(void) hipEventRecord(e1, stream());
	(void) hipEventSynchronize(e1);
	float ms = 0;
	(void) hipEventElapsedTime(&ms, e0, e1);
	(void) hipEventDestroy(e0);
	(void) hipEventDestroy(e1);
	std::lock_guard<std::mutex> g(prof_mu);
	auto &x = prof[name];
	x.first += ms;
	x.second += 1;
}

// ---- BATs ----------------------------------------------------------------------
int
width_of(int tt)
{
	switch (tt) {
	case MGDK_void: return 0;
	case MGDK_bit: case MGDK_bte: return 1;
	case MGDK_sht: return 2;
	case MGDK_int: case MGDK_date: case MGDK_flt: return 4;
	case MGDK_oid: case MGDK_lng: case MGDK_dbl: case MGDK_daytime: case MGDK_timestamp: return 8;
	case MGDK_hge: return 16;
	case MGDK_str: return 1;
	default: return -1;
	}
}

int
basetype(int tt)
{
	return tt == MGDK_date ? MGDK_int : tt == MGDK_bit ? MGDK_bte :
	       tt == MGDK_daytime || tt == MGDK_timestamp ? MGDK_lng : tt;
}

const char *
atomname(int tt)
{
	switch (tt) {
	case MGDK_void: return "void";
	case MGDK_bit: return "bit";
	case MGDK_bte: return "bte";
	case MGDK_sht: return "sht";
	case MGDK_int: return "int";
	case MGDK_oid: return "oid";
	case MGDK_flt: return "flt";
	case MGDK_dbl: return "dbl";
	case MGDK_lng: return "lng";
	case MGDK_hge: return "hge";
	case MGDK_date: return "date";
	case MGDK_daytime: return "daytime";
	case MGDK_timestamp: return "timestamp";
	case MGDK_str: return "str";
	}
	return "any";
}

Heap *
heap_new(size_t bytes)
{
	Heap *h = new Heap;
	h->size = bytes;
	h->refs = 1;
	h->base = bytes ? dalloc(bytes) : nullptr;
	if (bytes && h->base == nullptr) {
		delete h;
		return nullptr;
	}
	return h;
}

void
heap_decref(Heap *h)
{
	if (h == nullptr)
		return;
	if (__atomic_sub_fetch(&h->refs, 1, __ATOMIC_ACQ_REL) == 0) {
		dfree(h->base);
		delete h;
	}
}

size_t
tail_bytes(const mgdk_bat *b, BUN n)
{
	return b->ttype == MGDK_msk ? (size_t) ((n + 31) / 32) * 4 : n * (size_t) b->twidth;
}

mgdk_bat *
newbat(oid hseq, int tt, BUN cap)
{
	int w = tt == MGDK_msk ? 0 : width_of(tt);
	if (w < 0) {
		seterr("42000!type %d not supported", tt);
		return nullptr;
	}
	mgdk_bat *b = (mgdk_bat *) calloc(1, sizeof(mgdk_bat));
	Priv *p = new Priv{};
	b->priv = p;
	b->ttype = tt;
	b->twidth = w;
	b->hseqbase = hseq;
	b->tseqbase = tt == MGDK_void ? 0 : MGDK_OID_NIL;
	b->tsorted = b->trevsorted = b->tkey = 1;
	b->tnonil = 1;
	b->tminpos = b->tmaxpos = MGDK_BUN_NONE;
	if (tt == MGDK_msk) {
		// bits packed into 32-bit words (gdk_atoms.c msk); count = bits
		b->twidth = 4;
		b->tseqbase = MGDK_OID_NIL;
		p->theap = heap_new(((cap ? cap : 1) + 31) / 32 * 4);
		if (p->theap == nullptr) {
			delete p;
			free(b);
			return nullptr;
		}
		b->theap = p->theap->base;
	} else if (w > 0) {
		p->theap = heap_new((cap ? cap : 1) * (size_t) w);
		if (p->theap == nullptr) {
			delete p;
			free(b);
			return nullptr;
		}
		b->theap = p->theap->base;
	}
	return b;
}

const uint8_t *
img8_get(const mgdk_bat *b)
{
	const Priv *p = (const Priv *) b->priv;
	if (p == nullptr || p->img8 == nullptr || b->ttype != MGDK_oid || p->img8_n != b->count)
		return nullptr;
	return (const uint8_t *) p->img8->base;
}

uint8_t *
img8_new(mgdk_bat *b)
{
	Priv *p = (Priv *) b->priv;
	img8_drop(b);
	p->img8 = heap_new(b->count ? b->count : 1);
	if (p->img8 == nullptr)
		return nullptr;
	p->img8_n = b->count;
	return (uint8_t *) p->img8->base;
}

static void oidx_leave(Priv *p);

void
img8_drop(mgdk_bat *b)
{
	Priv *p = (Priv *) b->priv;
	if (p && p->img8) {
		heap_decref(p->img8);
		p->img8 = nullptr;
		p->img8_n = 0;
	}
	if (p && p->smap) {
		heap_decref(p->smap);
		p->smap = nullptr;
		p->smap_n = 0;
	}
	if (p && (p->oidx || p->poidx)) {
		oidx_leave(p);
		p->view = false;   // a written view holds a tail of its own
	}
}

// ---- order index slots (gdk_orderidx.c) -----------------------------------
static std::mutex oidx_mu;

static void
slot_decref(OidxSlot *s)
{
	if (s && --s->refs == 0) {
		heap_decref(s->idx);
		delete s;
	}
}

static void
oidx_leave(Priv *p)
{
	std::lock_guard<std::mutex> g(oidx_mu);
	slot_decref(p->oidx);
	slot_decref(p->poidx);
	p->oidx = p->poidx = nullptr;
}

Heap *
oidx_get(const mgdk_bat *b, bool *stable, int which, size_t *off)
{
	const Priv *p = (const Priv *) b->priv;
	if (p == nullptr || b->ttype == MGDK_void)
		return nullptr;
	std::lock_guard<std::mutex> g(oidx_mu);
	const OidxSlot *s = (which & OIDX_OWN) && p->oidx && p->oidx->idx && p->oidx->n == b->count ? p->oidx :
		(which & OIDX_PARENT) && p->poidx && p->poidx->idx && p->poidx->n == b->count ? p->poidx : nullptr;
	if (s == nullptr)
		return nullptr;
	__atomic_add_fetch(&s->idx->refs, 1, __ATOMIC_ACQ_REL);
	if (stable)
		*stable = s->stable;
	if (off)
		*off = s->off;
	return s->idx;
}

int
oidx_put(mgdk_bat *b, const mgdk_bat *order, bool stable)
{
	Priv *p = (Priv *) b->priv;
	Heap *h = nullptr;
	size_t off = 0;
	if (order->ttype == MGDK_void || ((const Priv *) order->priv)->theap == nullptr) {
		// a dense order materialised (BATorderidx never keeps one)
		h = heap_new(b->count * sizeof(oid) + 8);
		if (h == nullptr)
			return -1;
		std::vector<oid> seq(b->count);
		for (BUN i = 0; i < b->count; i++)
			seq[i] = order->tseqbase + i;
		if (b->count && !(hip_ok(hipMemcpyAsync(h->base, seq.data(), b->count * sizeof(oid), hipMemcpyHostToDevice,
							 stream()), "orderidx copy") && sync_data())) {
			heap_decref(h);
			return -1;
		}
	} else {
		h = ((const Priv *) order->priv)->theap;
		off = (size_t) ((const char *) order->theap - (const char *) h->base);
		__atomic_add_fetch(&h->refs, 1, __ATOMIC_ACQ_REL);
	}
	std::lock_guard<std::mutex> g(oidx_mu);
	if (p->oidx == nullptr)
		p->oidx = new OidxSlot{1, nullptr, 0, 0, false};
	if (p->oidx->idx && p->oidx->n == b->count) {
		heap_decref(h);   // it has one (another thread was first)
		return 0;
	}
	heap_decref(p->oidx->idx);
	p->oidx->idx = h;
	p->oidx->off = off;
	p->oidx->n = b->count;
	p->oidx->stable = stable;
	return 0;
}

mgdk_bat *
oidx_bat(Heap *h, size_t off, oid hseq, BUN n)
{
	mgdk_bat *o = (mgdk_bat *) calloc(1, sizeof(mgdk_bat));
	Priv *p = new Priv{};
	o->priv = p;
	o->ttype = MGDK_oid;
	o->twidth = 8;
	o->hseqbase = hseq;
	o->tseqbase = MGDK_OID_NIL;
	o->tminpos = o->tmaxpos = MGDK_BUN_NONE;
	__atomic_add_fetch(&h->refs, 1, __ATOMIC_ACQ_REL);
	p->theap = h;
	p->toff = off;
	o->theap = (char *) h->base + off;
	o->count = n;
	o->tkey = o->tnonil = 1;
	o->tnil = 0;
	o->tsorted = o->trevsorted = n <= 1;
	return o;
}

bool
is_view(const mgdk_bat *b)
{
	const Priv *p = (const Priv *) b->priv;
	return p && p->view;
}

// v, a view over all of b, sees b's index (the slot is created empty when b
// has none, so one b gets later is seen too)
void
oidx_share(mgdk_bat *v, const mgdk_bat *b)
{
	Priv *vp = (Priv *) v->priv, *bp = (Priv *) b->priv;
	std::lock_guard<std::mutex> g(oidx_mu);
	if (bp->oidx == nullptr)
		bp->oidx = new OidxSlot{1, nullptr, 0, 0, false};
	bp->oidx->refs++;
	vp->poidx = bp->oidx;
}

bool
smap_get(const mgdk_bat *b, SelMap *m)
{
	const Priv *p = (const Priv *) b->priv;
	if (p == nullptr || p->smap == nullptr || b->ttype != MGDK_oid || p->smap_n != b->count)
		return false;
	m->pre = (const uint64_t *) p->smap->base;
	m->bits = (const uint32_t *) ((const char *) p->smap->base + p->smap_bits_off);
	m->wpt = p->smap_wpt;
	m->ntiles = p->smap_ntiles;
	m->nslots = p->smap_nslots;
	m->base = p->smap_base;
	m->lo = p->smap_lo;
	m->hi = p->smap_hi;
	return true;
}

void
smap_set(mgdk_bat *b, Heap *h, const SelMap &m)
{
	Priv *p = (Priv *) b->priv;
	img8_drop(b);
	__atomic_add_fetch(&h->refs, 1, __ATOMIC_ACQ_REL);
	p->smap = h;
	p->smap_n = b->count;
	p->smap_wpt = m.wpt;
	p->smap_ntiles = m.ntiles;
	p->smap_nslots = m.nslots;
	p->smap_base = m.base;
	p->smap_bits_off = (size_t) ((const char *) m.bits - (const char *) h->base);
	p->smap_lo = m.lo;
	p->smap_hi = m.hi;
}

void
setdense(mgdk_bat *b, oid tseq, BUN cnt)
{
	Priv *p = (Priv *) b->priv;
	img8_drop(b);
	heap_decref(p->theap);
	p->theap = nullptr;
	b->theap = nullptr;
	b->ttype = MGDK_void;
	b->twidth = 0;
	b->tseqbase = tseq;
	b->count = cnt;
	b->tsorted = b->tkey = b->tnonil = 1;
	b->tnil = 0;
	b->trevsorted = cnt <= 1;
}

void
share_vheap(mgdk_bat *dst, const mgdk_bat *src)
{
	Priv *d = (Priv *) dst->priv, *s = (Priv *) src->priv;
	if (s->tvheap)
		__atomic_add_fetch(&s->tvheap->refs, 1, __ATOMIC_ACQ_REL);
	heap_decref(d->tvheap);
	d->tvheap = s->tvheap;
	dst->tvheap = src->tvheap;
	dst->tvheapsize = src->tvheapsize;
}

// ---- candidate lists -------------------------------------------------------------
__global__ void
k_lower_bounds(const oid *a, BUN n, oid lo, oid hi, BUN *out)
{
	// out[0] = lower_bound(a, lo), out[1] = lower_bound(a, hi),
	// out[2] = a[p], out[3] = a[q-1]
	BUN p = 0, e = n;
	while (p < e) {
		BUN m = (p + e) / 2;
		if (a[m] < lo) p = m + 1; else e = m;
	}
	BUN q = p;
	e = n;
	while (q < e) {
		BUN m = (q + e) / 2;
		if (a[m] < hi) q = m + 1; else e = m;
	}
	out[0] = p;
	out[1] = q;
	out[2] = q > p ? a[p] : 0;
	out[3] = q > p ? a[q - 1] : 0;
}

// complex candidate lists (gdk/gdk_cand.h:23-38): a void BAT whose vheap
// holds a ccand_t header {type:1, firstbit:48} and then either the
// excluded oids (CAND_NEGOID, cand_except) or 32-bit mask words
// (CAND_MSK, cand_mask).  cand_init (gdk_cand.c:455-490) materialises them
// on the device into an ordered oid list (one flag pass + the ordered
// compaction); the lists stay alive in a small per-thread ring until later
// cand_init calls of the same thread replace them (operators synchronise
// before returning, so a list is never replaced while a kernel reads it).
__global__ void
k_cand_negoid(int8_t *flags, BUN R)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (BUN) gridDim.x * blockDim.x)
		flags[i] = 1;
}

__global__ void
k_cand_negoid_clear(int8_t *flags, BUN R, oid seq, const oid *exc, BUN nexc)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < nexc; i += (BUN) gridDim.x * blockDim.x) {
		const oid x = exc[i];
		if (x >= seq && x - seq < R)
			flags[x - seq] = 0;
	}
}

__global__ void
k_cand_mask(int8_t *flags, BUN nbits, const uint32_t *mask)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < nbits; i += (BUN) gridDim.x * blockDim.x)
		flags[i] = (int8_t) ((mask[i >> 5] >> (i & 31)) & 1);
}

static thread_local mgdk_bat *cand_ring[4];
static thread_local unsigned cand_ring_next;

mgdk_bat *
unmask_cand(const mgdk_bat *s)
{
	if (s->ttype == MGDK_msk) {
		// a bit BAT: candidate hseqbase + i for every set bit i < count,
		// the positive list BATunmask makes of it (gdk_cand.c:1464-1490,
		// :1560-1600); the reference's canditer_init has no working branch
		// for a msk-typed s (gdk_cand.c:468-473 asserts), and its callers
		// (BATjoin gdk_join.c:4500-4517, BATproject2 gdk_project.c:652-660)
		// unmask msk BATs first -- so the device takes every msk s that way
		const BUN R = s->count;
		DevBuf f(R + 1);
		if (!f.p)
			return nullptr;
		hipLaunchKernelGGL(k_cand_mask, dim3(grid_for(R, 1024, 8192)), dim3(256), 0, stream(), f.as<int8_t>(),
				   R, (const uint32_t *) s->theap);
		return compact_flags(f.as<int8_t>(), R, s->hseqbase);
	}
	uint64_t *hdr = (uint64_t *) pinned(64);
	if (hdr == nullptr ||
	    !hip_ok(hipMemcpyAsync(hdr, s->tvheap, 8, hipMemcpyDeviceToHost, stream()), "hipMemcpyAsync") || !sync())
		return nullptr;
	const bool msk = (*hdr & 1) != 0;
	const oid firstbit = (*hdr >> 1) & ((1ull << 48) - 1);
	const char *payload = (const char *) s->tvheap + 8;
	const BUN bytes = s->tvheapsize - 8;
	hipStream_t st = stream();
	BUN R;
	oid seq;
	if (msk) {
		// ci->seq = tseqbase - firstbit, bit i = candidate seq + i
		seq = s->tseqbase - firstbit;
		R = bytes / 4 * 32;
		DevBuf f(R + 1);
		if (!f.p)
			return nullptr;
		hipLaunchKernelGGL(k_cand_mask, dim3(grid_for(R, 1024, 8192)), dim3(256), 0, st, f.as<int8_t>(), R,
				   (const uint32_t *) payload);
		return compact_flags(f.as<int8_t>(), R, seq);
	}
	// candidates [tseqbase, tseqbase + count + nexc) minus the exceptions
	const BUN nexc = bytes / 8;
	seq = s->tseqbase;
	R = s->count + nexc;
	DevBuf f(R + 1);
	if (!f.p)
		return nullptr;
	hipLaunchKernelGGL(k_cand_negoid, dim3(grid_for(R, 1024, 8192)), dim3(256), 0, st, f.as<int8_t>(), R);
	if (nexc)
		hipLaunchKernelGGL(k_cand_negoid_clear, dim3(grid_for(nexc, 1024, 8192)), dim3(256), 0, st,
				   f.as<int8_t>(), R, seq, (const oid *) payload, nexc);
	return compact_flags(f.as<int8_t>(), R, seq);
}

// BATmaskedcands (gdk_cand.c:1366-1460): the words of the cand_mask list --
// masked's bits (or their complement), rows past masked's end selected, the
// bits past nr cleared -- with the number of set bits (meta[0]) and the
// lowest set bit (meta[1], a minimum kept as ~max of the complement)
__global__ __launch_bounds__(256) void
k_masked_words(uint32_t *r, const uint32_t *src, BUN bcount, BUN nr, bool selected, unsigned long long *meta)
{
	const BUN nmask = (nr + 31) / 32, nsrc = (bcount + 31) / 32;
	const uint32_t rest = (uint32_t) (bcount & 31);
	unsigned long long ones = 0, lowest = ~0ull;
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < nmask; i += (BUN) gridDim.x * blockDim.x) {
		uint32_t w;
		if (i < nsrc) {
			w = selected ? src[i] : ~src[i];
			if (nr > bcount && rest > 0 && i == nsrc - 1)
				w |= ~0u << rest;
		} else {
			w = ~0u;
		}
		if (i == nmask - 1 && (nr & 31))
			w &= (1u << (nr & 31)) - 1;
		r[i] = w;
		ones += __popc(w);
		if (w && lowest == ~0ull)
			lowest = i * 32 + __ffs(w) - 1;
	}
	ones = block_reduce(ones, [](unsigned long long a, unsigned long long b) { return a + b; });
	lowest = block_reduce(lowest, [](unsigned long long a, unsigned long long b) { return a < b ? a : b; });
	if (threadIdx.x == 0) {
		if (ones)
			atomicAdd(&meta[0], ones);
		publish_max(&meta[1], ~lowest);
	}
}

__global__ void
k_cand_search(const oid *oids, BUN n, oid o, unsigned long long *out)
{
	BUN lo = 0, hi = n;
	while (lo < hi) {
		const BUN m = (lo + hi) >> 1;
		if (oids[m] < o)
			lo = m + 1;
		else
			hi = m;
	}
	*out = lo;
}

BUN
cand_index(const Cand &ci, oid o)
{
	if (ci.dense)
		return o - ci.seq;
	unsigned long long *m = (unsigned long long *) meta_buf();
	unsigned long long *h = (unsigned long long *) pinned(64);
	hipLaunchKernelGGL(k_cand_search, dim3(1), dim3(1), 0, stream(), ci.oids, ci.n, o, m);
	if (!hip_ok(hipMemcpyAsync(h, m, 8, hipMemcpyDeviceToHost, stream()), "memcpy") || !sync_data())
		return ~(BUN) 0;
	return h[0];
}

int
oid_at(const mgdk_bat *b, BUN p, oid *v)
{
	if (b->ttype == MGDK_void) {
		*v = b->tseqbase == MGDK_OID_NIL ? MGDK_OID_NIL : b->tseqbase + p;
		return 0;
	}
	oid *h = (oid *) pinned(64);
	if (!hip_ok(hipMemcpyAsync(h, (const oid *) b->theap + p, 8, hipMemcpyDeviceToHost, stream()), "memcpy") ||
	    !sync_data())
		return -1;
	*v = h[0];
	return 0;
}

int
cand_init(Cand *ci, const mgdk_bat *b, const mgdk_bat *s)
{
	oid lo = b ? b->hseqbase : 0;
	oid hi = b ? b->hseqbase + b->count : ~(oid) 0;
	*ci = Cand{};
	ci->dense = true;
	if (s == nullptr) {
		ci->seq = lo;
		ci->n = b ? b->count : 0;
		ci->first = lo;
		ci->last = lo + ci->n - 1;
		return 0;
	}
	if (s->count == 0 || (b && b->count == 0))
		return 0;
	if (is_complex_cand(s)) {
		mgdk_bat *m = unmask_cand(s);
		if (m == nullptr)
			return -1;
		mgdk_BBPunfix(cand_ring[cand_ring_next & 3]);
		cand_ring[cand_ring_next++ & 3] = m;
		return cand_init(ci, b, m);
	}
	if (s->ttype == MGDK_void) {
		if (s->tseqbase == MGDK_OID_NIL) {
			seterr("candidate list with nil seqbase");
			return -1;
		}
		oid a = s->tseqbase, e = s->tseqbase + s->count;
		if (a < lo) a = lo;
		if (e > hi) e = hi;
		if (a < e) {
			ci->seq = a;
			ci->n = e - a;
			ci->first = a;
			ci->last = e - 1;
		}
		return 0;
	}
	if (s->ttype != MGDK_oid) {
		seterr("candidate list must have type oid");
		return -1;
	}
	BUN *meta = (BUN *) meta_buf();
	if (meta == nullptr)
		return -1;
	hipLaunchKernelGGL(k_lower_bounds, dim3(1), dim3(1), 0, stream(),
			   (const oid *) s->theap, s->count, lo, hi, meta);
	BUN *h = (BUN *) pinned(64);
	if (h == nullptr)
		return -1;
	if (!hip_ok(hipMemcpyAsync(h, meta, 4 * sizeof(BUN), hipMemcpyDeviceToHost, stream()),
		    "hipMemcpyAsync") || !sync())
		return -1;
	BUN p = h[0], q = h[1];
	if (p >= q)
		return 0;
	ci->n = q - p;
	ci->first = h[2];
	ci->last = h[3];
	if (ci->last - ci->first == ci->n - 1) {
		ci->seq = ci->first;
	} else {
		ci->dense = false;
		ci->oids = (const oid *) s->theap + p;
		ci->src = s;
	}
	return 0;
}

}  // namespace mgdk

using namespace mgdk;

extern "C" {

int
mgdk_init(int device)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
		seterr("HY013!no HIP device available");
		return -1;
	}
	if (device < 0 || device >= n) {
		seterr("HY013!device %d out of range (%d devices)", device, n);
		return -1;
	}
	g_device = device;
	if (!hip_ok(hipSetDevice(device), "hipSetDevice"))
		return -1;
	return stream() ? 0 : -1;
}

int64_t
mgdk_usec(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_REALTIME, &ts);
	return (int64_t) ts.tv_sec * 1000000 + ts.tv_nsec / 1000;
}

void
mgdk_thread_set_qry_ctx(mgdk_qryctx *ctx)
{
	qry_ctx = ctx;
}

mgdk_qryctx *
mgdk_thread_get_qry_ctx(void)
{
	return qry_ctx;
}

const char *
mgdk_GDKerrbuf(void)
{
	return errbuf;
}

void
mgdk_GDKclrerr(void)
{
	errbuf[0] = 0;
}

int
mgdk_sync(void)
{
	return sync_data() ? 0 : -1;
}

void *
mgdk_stream(void)
{
	return (void *) stream();
}

uint64_t
mgdk_mem_cursize(void)
{
	std::lock_guard<std::mutex> g(alloc_mu);
	return cur_bytes;
}

void
mgdk_mem_release_cache(void)
{
	std::lock_guard<std::mutex> g(alloc_mu);
	for (auto &kv : free_lists)
		for (void *p : kv.second)
			(void) hipFree(p);
	free_lists.clear();
	cached_bytes = 0;
}

void
mgdk_prof_enable(int on)
{
	prof_on = on != 0;
}

int
mgdk_prof_get(const char *kernel, double *total_ms, uint64_t *launches)
{
	std::lock_guard<std::mutex> g(prof_mu);
	auto it = prof.find(kernel);
	if (it == prof.end()) {
		*total_ms = 0;
		*launches = 0;
		return -1;
	}
	*total_ms = it->second.first;
	*launches = it->second.second;
	return 0;
}

void
mgdk_prof_reset(void)
{
	std::lock_guard<std::mutex> g(prof_mu);
	prof.clear();
}

mgdk_bat *
mgdk_COLnew(mgdk_oid hseq, int tt, mgdk_BUN cap)
{
	return newbat(hseq, tt, cap);
}

mgdk_bat *
mgdk_BATdense(mgdk_oid hseq, mgdk_oid tseq, mgdk_BUN cnt)
{
	mgdk_bat *b = newbat(hseq, MGDK_void, 0);
	if (b)
		setdense(b, tseq, cnt);
	return b;
}

__global__ void
k_fill(char *dst, const char *val, int w, BUN n)
{
	for (BUN i = blockIdx.x * (BUN) blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		for (int k = 0; k < w; k++)
			dst[i * w + k] = val[k];
}

mgdk_bat *
mgdk_BATconstant(mgdk_oid hseq, int tt, const void *val, mgdk_BUN cnt)
{
	mgdk_bat *b = newbat(hseq, tt, cnt);
	if (b == nullptr)
		return nullptr;
	int w = b->twidth;
	if (w > 0 && cnt > 0) {
		char *dv = (char *) meta_buf();
		if (!hip_ok(hipMemcpyAsync(dv, val, w, hipMemcpyHostToDevice, stream()), "memcpy")) {
			mgdk_BBPunfix(b);
			return nullptr;
		}
		hipLaunchKernelGGL(k_fill, dim3(grid_for(cnt, 1024, 4096)), dim3(256), 0, stream(),
				   (char *) b->theap, dv, w, cnt);
		if (!sync()) {
			mgdk_BBPunfix(b);
			return nullptr;
		}
	}
	b->count = cnt;
	b->tsorted = b->trevsorted = 1;
	b->tkey = cnt <= 1;
	// gdk_batop.c:2916-2920: tnil when the value is the type's nil
	bool isnil = false;
	if (val != nullptr && w > 0) {
		const int bt = basetype(tt);
		if (bt == MGDK_flt) {
			float f;
			memcpy(&f, val, 4);
			isnil = f != f;
		} else if (bt == MGDK_dbl) {
			double d;
			memcpy(&d, val, 8);
			isnil = d != d;
		} else if (bt != MGDK_str) {
			unsigned char buf[16];
			memcpy(buf, val, w);
			isnil = buf[w - 1] == 0x80;   // little endian: the minimum has only the top bit set
			for (int k = 0; k < w - 1 && isnil; k++)
				isnil = buf[k] == 0;
		}
	}
	b->tnil = cnt >= 1 && isnil;
	b->tnonil = !b->tnil;
	return b;
}

mgdk_bat *
mgdk_BATslice(mgdk_bat *b, mgdk_BUN lo, mgdk_BUN hi)
{
	if (hi > b->count)
		hi = b->count;
	if (lo > hi)
		lo = hi;
	if (b->ttype == MGDK_msk && (lo & 31)) {
		seterr("42000!BATslice: a msk view must start at a multiple of 32 rows");
		return nullptr;
	}
	mgdk_bat *v = (mgdk_bat *) calloc(1, sizeof(mgdk_bat));
	Priv *p = new Priv{}, *bp = (Priv *) b->priv;
	*v = *b;
	v->priv = p;
	v->hseqbase = b->hseqbase + lo;
	v->count = hi - lo;
	if (b->ttype == MGDK_void) {
		if (b->tseqbase != MGDK_OID_NIL)
			v->tseqbase = b->tseqbase + lo;
	} else {
		p->theap = bp->theap;
		if (p->theap)
			__atomic_add_fetch(&p->theap->refs, 1, __ATOMIC_ACQ_REL);
		v->theap = (char *) b->theap + tail_bytes(b, lo);
	}
	if (bp->tvheap) {
		p->tvheap = bp->tvheap;
		__atomic_add_fetch(&p->tvheap->refs, 1, __ATOMIC_ACQ_REL);
	}
	p->view = true;
	if (lo == 0 && hi == b->count && b->ttype != MGDK_void)
		oidx_share(v, b);
	// what is known of the parent's order holds for a slice, positions do not
	v->tnosorted = v->tnorevsorted = 0;
	v->tminpos = v->tmaxpos = MGDK_BUN_NONE;
	v->tunique_est = 0;
	if (v->count <= 1)
		v->tsorted = v->trevsorted = v->tkey = 1;
	return v;
}

void
mgdk_BBPunfix(mgdk_bat *b)
{
	if (b == nullptr)
		return;
	Priv *p = (Priv *) b->priv;
	if (p) {
		heap_decref(p->theap);
		heap_decref(p->tvheap);
		heap_decref(p->img8);
		heap_decref(p->smap);
		oidx_leave(p);
		delete p;
	}
	free(b);
}

int
mgdk_BATupload(mgdk_bat *b, const void *host, mgdk_BUN n)
{
	if (b->ttype == MGDK_void) {
		seterr("cannot upload into a void BAT");
		return -1;
	}
	Priv *p = (Priv *) b->priv;
	size_t bytes = tail_bytes(b, n);
	img8_drop(b);
	// a heap shared with views (refs > 1) is never written in place
	if (p->theap == nullptr || p->theap->refs != 1 ||
	    p->theap->size < bytes + ((char *) b->theap - (char *) p->theap->base)) {
		Heap *h = heap_new(bytes ? bytes : 1);
		if (h == nullptr)
			return -1;
		heap_decref(p->theap);
		p->theap = h;
		b->theap = h->base;
	}
	const void *src = bytes && bytes <= ((size_t) 16 << 20) ? stage_host(host, bytes) : host;
	if (bytes && (src == nullptr ||
		      !hip_ok(hipMemcpyAsync(b->theap, src, bytes, hipMemcpyHostToDevice, stream()), "hipMemcpyAsync H2D")))
		return -1;
	b->count = n;
	// the new values carry no known positions or estimates
	b->tnosorted = b->tnorevsorted = 0;
	b->tminpos = b->tmaxpos = MGDK_BUN_NONE;
	b->tunique_est = 0;
	return sync_data() ? 0 : -1;
}

int
mgdk_BATdownload(const mgdk_bat *b, void *host)
{
	if (b->ttype == MGDK_void) {
		oid *o = (oid *) host;
		for (BUN i = 0; i < b->count; i++)
			o[i] = b->tseqbase == MGDK_OID_NIL ? MGDK_OID_NIL : b->tseqbase + i;
		return 0;
	}
	size_t bytes = tail_bytes(b, b->count);
	if (bytes && !hip_ok(hipMemcpyAsync(host, b->theap, bytes, hipMemcpyDeviceToHost, stream()),
			     "hipMemcpyAsync D2H"))
		return -1;
	return sync_data() ? 0 : -1;
}

mgdk_bat *
mgdk_BATmaskedcands(oid hseq, BUN nr, mgdk_bat *masked, bool selected)
{
	if (masked == nullptr || masked->ttype != MGDK_msk) {
		seterr("BATmaskedcands: masked must be a msk BAT");
		return nullptr;
	}
	mgdk_bat *bn = newbat(hseq, MGDK_void, 0);
	if (bn == nullptr)
		return nullptr;
	bn->tseqbase = hseq;
	bn->count = 0;
	if (masked->count == 0 || nr == 0)
		return bn;
	const BUN nmask = (nr + 31) / 32;
	Heap *h = heap_new(8 + nmask * 4);
	unsigned long long *meta = (unsigned long long *) meta_buf();
	unsigned long long *hm = (unsigned long long *) pinned(64);
	hipStream_t st = stream();
	if (h == nullptr || meta == nullptr || hm == nullptr || !hip_ok(hipMemsetAsync(meta, 0, 16, st), "memset")) {
		heap_decref(h);
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	hipLaunchKernelGGL(k_masked_words, dim3(grid_for(nmask, 256 * 8, 2048)), dim3(256), 0, st,
			   (uint32_t *) ((char *) h->base + 8), (const uint32_t *) masked->theap, masked->count, nr,
			   selected, meta);
	if (!hip_ok(hipMemcpyAsync(hm, meta, 16, hipMemcpyDeviceToHost, st), "memcpy") || !sync()) {
		heap_decref(h);
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	const BUN cnt = hm[0];
	if (cnt == 0) {                 // no point having a mask if it's empty
		heap_decref(h);
		return bn;
	}
	const unsigned long long firstbit = ~hm[1];
	// ccand_t {type = CAND_MSK (bit 0), firstbit (bits 1..48)} (gdk_cand.h:23-38)
	hm[2] = 1ull | (firstbit << 1);
	if (!hip_ok(hipMemcpyAsync(h->base, &hm[2], 8, hipMemcpyHostToDevice, st), "memcpy") || !sync()) {
		heap_decref(h);
		mgdk_BBPunfix(bn);
		return nullptr;
	}
	Priv *p = (Priv *) bn->priv;
	p->tvheap = h;
	bn->tvheap = h->base;
	bn->tvheapsize = 8 + nmask * 4;
	bn->tseqbase = hseq + firstbit;
	bn->count = cnt;
	bn->trevsorted = cnt <= 1;
	return bn;
}

int
mgdk_BATsetvheap(mgdk_bat *b, const void *host, uint64_t size)
{
	Priv *p = (Priv *) b->priv;
	Heap *h = heap_new(size ? size : 1);
	if (h == nullptr)
		return -1;
	if (size && !hip_ok(hipMemcpyAsync(h->base, host, size, hipMemcpyHostToDevice, stream()), "vheap")) {
		heap_decref(h);
		return -1;
	}
	heap_decref(p->tvheap);
	p->tvheap = h;
	b->tvheap = h->base;
	b->tvheapsize = size;
	return sync_data() ? 0 : -1;
}

int
mgdk_BATdownload_vheap(const mgdk_bat *b, void *host)
{
	if (b->tvheap == nullptr)
		return 0;
	if (!hip_ok(hipMemcpyAsync(host, b->tvheap, b->tvheapsize, hipMemcpyDeviceToHost, stream()), "vheap"))
		return -1;
	return sync_data() ? 0 : -1;
}

}  // extern "C"

// BATappend (gdk/gdk_batop.c:1011 -> BATappend2 :674): append the candidates
// s of n to b in place.  Fixed-width tails only (str would need heap
// merging); a void b stays void while n continues its sequence.  The tail
// heap grows geometrically; a heap shared with views is copied first.
__global__ void
k_fill_seq(oid *out, BUN n, oid seq)
{
	for (BUN i = (BUN) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (BUN) gridDim.x * blockDim.x)
		out[i] = seq == MGDK_OID_NIL ? MGDK_OID_NIL : seq + i;
}

// atomcmp of two values of base type bt (host), nil smallest as in GDK
static int
atom_cmp(int bt, const void *x, const void *y)
{
#define CMP3(T) { T a, c; memcpy(&a, x, sizeof(T)); memcpy(&c, y, sizeof(T)); return (a > c) - (a < c); }
	switch (bt) {
	case MGDK_bte: CMP3(int8_t)
	case MGDK_sht: CMP3(int16_t)
	case MGDK_int: CMP3(int32_t)
	case MGDK_lng: CMP3(int64_t)
	case MGDK_hge: CMP3(hge)
	case MGDK_oid: {
		oid a, c;
		memcpy(&a, x, 8);
		memcpy(&c, y, 8);
		// oid_nil compares smallest (gdk_atoms.c oidCmp via lngCmp on the
		// signed image)
		return ((int64_t) a > (int64_t) c) - ((int64_t) a < (int64_t) c);
	}
	case MGDK_flt: {
		float a, c;
		memcpy(&a, x, 4);
		memcpy(&c, y, 4);
		return a != a ? -(c == c) : c != c ? 1 : (a > c) - (a < c);
	}
	case MGDK_dbl: {
		double a, c;
		memcpy(&a, x, 8);
		memcpy(&c, y, 8);
		return a != a ? -(c == c) : c != c ? 1 : (a > c) - (a < c);
	}
	default: CMP3(int64_t)
	}
#undef CMP3
}

// value at position p of a fixed-width column (host read; void: its oid)
static bool
value_at(const mgdk_bat *b, BUN p, void *out)
{
	if (b->ttype == MGDK_void) {
		oid v = b->tseqbase == MGDK_OID_NIL ? MGDK_OID_NIL : b->tseqbase + p;
		memcpy(out, &v, 8);
		return true;
	}
	void *h = pinned(16);
	return h && hip_ok(hipMemcpyAsync(h, (const char *) b->theap + p * (size_t) b->twidth, b->twidth,
					  hipMemcpyDeviceToHost, stream()), "memcpy") && sync_data() &&
	       memcpy(out, h, b->twidth);
}

extern "C" int
mgdk_BATappend(mgdk_bat *b, mgdk_bat *n, mgdk_bat *s, bool force)
{
	(void) force;
	if (b == nullptr || n == nullptr) {
		seterr("BATappend: NULL argument");
		return -1;
	}
	mgdk_bat *src = n, *proj = nullptr;
	if (s) {
		proj = mgdk_BATproject(s, n);
		if (proj == nullptr)
			return -1;
		src = proj;
	}
	const BUN cnt = src->count;
	int rc = -1;
	Heap *old_heap = nullptr;
	if (cnt == 0) {
		rc = 0;
		goto out;
	}
	if (b->ttype == MGDK_str || src->ttype == MGDK_str) {
		seterr("42000!BATappend: str tails are not supported on the device path");
		goto out;
	}
	{
		const int bt = basetype(b->ttype == MGDK_void ? MGDK_oid : b->ttype);
		const int nt = basetype(src->ttype == MGDK_void ? MGDK_oid : src->ttype);
		if (b->count > 0 && bt != nt) {
			seterr("Incompatible operands (%s vs. %s).\n", atomname(b->ttype), atomname(src->ttype));
			goto out;
		}
		if (b->count == 0 && b->ttype != src->ttype && b->ttype != MGDK_void && bt != nt) {
			seterr("Incompatible operands (%s vs. %s).\n", atomname(b->ttype), atomname(src->ttype));
			goto out;
		}
	}
	// the extremes' positions and the distinct-value estimate
	// (gdk_batop.c:762-792): kept when the appended part's extreme is known
	// and no candidate list renumbers it, else unknown
	{
		const int vt = basetype(b->ttype == MGDK_void ? MGDK_oid : b->ttype);
		const BUN bc = b->count;
		char x[16], y[16];
		BUN *pos[2] = {&b->tmaxpos, &b->tminpos};
		const BUN npos[2] = {n->tmaxpos, n->tminpos};
		for (int k = 0; k < 2; k++) {
			if (bc != 0 && *pos[k] == MGDK_BUN_NONE)
				continue;
			if (npos[k] == MGDK_BUN_NONE) {
				*pos[k] = MGDK_BUN_NONE;
				continue;
			}
			int c = -1;
			if (bc != 0) {
				if (!value_at(b, *pos[k], x) || !value_at(n, npos[k], y))
					goto out;
				c = atom_cmp(vt, x, y);
				if (k == 1)
					c = -c;
			}
			if (c < 0)
				*pos[k] = s == nullptr ? bc + npos[k] : MGDK_BUN_NONE;
		}
		if (cnt > bc / 1000)   // GDK_UNIQUE_ESTIMATE_KEEP_FRACTION, gdk_private.h:439
			b->tunique_est = 0;
	}
	// void + continuing dense sequence stays void
	if (b->ttype == MGDK_void && src->ttype == MGDK_void &&
	    (b->count == 0 || (b->tseqbase != MGDK_OID_NIL && src->tseqbase == b->tseqbase + b->count))) {
		if (b->count == 0)
			b->tseqbase = src->tseqbase;
		b->count += cnt;
		b->trevsorted = b->count <= 1;
		rc = 0;
		goto out;
	}
	{
		Priv *p = (Priv *) b->priv;
		hipStream_t st = stream();
		img8_drop(b);
		const int tt = b->ttype == MGDK_void ? MGDK_oid : b->ttype;
		const size_t w = (size_t) width_of(tt);
		const BUN total = b->count + cnt;
		const size_t used_off = p->theap ? (size_t) ((char *) b->theap - (char *) p->theap->base) : 0;
		const bool fits = b->ttype != MGDK_void && p->theap && p->theap->refs == 1 &&
				  p->theap->size >= used_off + total * w;
		if (!fits) {
			size_t cap = total * w;
			if (p->theap && b->ttype != MGDK_void)
				cap = cap < 2 * b->count * w ? 2 * b->count * w : cap;
			Heap *h = heap_new(cap);
			if (h == nullptr)
				goto out;
			if (b->count) {
				if (b->ttype == MGDK_void)
					hipLaunchKernelGGL(k_fill_seq, dim3(grid_for(b->count, 1024, 4096)), dim3(256), 0, st,
							   (oid *) h->base, b->count, b->tseqbase);
				else if (!hip_ok(hipMemcpyAsync(h->base, b->theap, b->count * w, hipMemcpyDeviceToDevice, st),
						 "memcpy D2D")) {
					heap_decref(h);
					goto out;
				}
			}
			// the old heap is still being read by the copy just queued:
			// release it only after the stream has drained (below)
			old_heap = p->theap;
			p->theap = h;
			b->theap = h->base;
			if (b->ttype == MGDK_void) {
				b->ttype = MGDK_oid;
				b->twidth = 8;
				b->tseqbase = MGDK_OID_NIL;
			}
		}
		char *dst = (char *) b->theap + b->count * w;
		if (src->ttype == MGDK_void)
			hipLaunchKernelGGL(k_fill_seq, dim3(grid_for(cnt, 1024, 4096)), dim3(256), 0, st, (oid *) dst, cnt,
					   src->tseqbase);
		else if (!hip_ok(hipMemcpyAsync(dst, src->theap, cnt * w, hipMemcpyDeviceToDevice, st), "memcpy D2D"))
			goto out;
		if (!sync())
			goto out;
		heap_decref(old_heap);
		old_heap = nullptr;
		const bool wasempty = b->count == 0;
		b->count = total;
		// properties the append cannot vouch for are cleared (BATappend2
		// keeps them only after comparing the boundary values)
		b->tnonil = (wasempty || b->tnonil) && src->tnonil;
		b->tnil = (!wasempty && b->tnil) || src->tnil;
		b->tsorted = wasempty ? src->tsorted : total <= 1;
		b->trevsorted = wasempty ? src->trevsorted : total <= 1;
		b->tkey = wasempty ? src->tkey : total <= 1;
		rc = 0;
	}
out:
	if (old_heap) {
		(void) hipStreamSynchronize(stream());   // error path: drain before release
		heap_decref(old_heap);
	}
	mgdk_BBPunfix(proj);
	return rc;
}

// ---- order-dependent float folds: where the parallel form starts ---------
static std::atomic<uint64_t> g_fp_par_min{(uint64_t) 1 << 20};

namespace mgdk {
BUN
fp_parallel_min()
{
	return (BUN) g_fp_par_min.load(std::memory_order_relaxed);
}
}  // namespace mgdk

extern "C" mgdk_BUN
mgdk_set_fp_parallel_min(mgdk_BUN rows)
{
	return (mgdk_BUN) g_fp_par_min.exchange((uint64_t) rows);
}
