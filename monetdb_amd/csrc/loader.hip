// loader.hip -- persistent BAT heaps from a MonetDB dbfarm into HBM
// (HEAPload gdk/gdk_heap.c:729, BATsave
// gdk/gdk_storage.c:785, the BBP.dir catalogue gdk/gdk_bbp.c:595-714).
//
// BBP.dir (version GDKLIBRARY 061050, gdk_bbp.c:2154-2194, :2110-2151):
//   BBP.dir, GDKversion <v>
//   <sizeof size_t> <sizeof oid> <sizeof hge>
//   BBPsize=<n>
//   BBPinfo=<logno>
//   per BAT: <id> <name> <restricted<<1> <count> <hseqbase>
//            <type> <width> <var> <props> <nokey0> <nokey1> <nosorted>
//            <norevsorted> <tseqbase> <free> <minpos> <maxpos> [<vheap free>]
//            [<options>]
// The physical file of BAT id is its octal name under 2-digit octal
// subdirectories (BBPgetfilename :386, BBPsubdir_recursive :363); the tail
// is <name>.tail (str: .tail1/.tail2/.tail4 by offset width, settailname
// gdk_bat.c:194), the string heap <name>.theap.
// The tail is streamed through two pinned staging buffers with
// asynchronous copies, so the read of chunk k+1 overlaps the copy of k.
#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mgdk_internal.h"

using namespace mgdk;

namespace {

struct TypeName {
	const char *name;
	int tt;
};

const TypeName TYPES[] = {
	{"void", MGDK_void}, {"bit", MGDK_bit}, {"bte", MGDK_bte}, {"sht", MGDK_sht}, {"int", MGDK_int},
	{"oid", MGDK_oid}, {"flt", MGDK_flt}, {"dbl", MGDK_dbl}, {"lng", MGDK_lng}, {"hge", MGDK_hge},
	{"date", MGDK_date}, {"str", MGDK_str}, {"msk", MGDK_msk},
};

int
type_of(const char *name)
{
	for (const TypeName &t : TYPES)
		if (strcmp(t.name, name) == 0)
			return t.tt;
	return -1;
}

// BBPgetfilename (gdk_bbp.c:363-396)
void
physical_name(int64_t id, char *s, size_t len)
{
	char tmp[64];
	char *p = tmp;
	if (id >= 0100) {
		// subdirectories from the most significant pair of octal digits
		int64_t v = id >> 6;
		char dirs[32][3];
		int nd = 0;
		while (true) {
			const int64_t d = v & 077;
			dirs[nd][0] = (char) ('0' + (d >> 3));
			dirs[nd][1] = (char) ('0' + (d & 7));
			dirs[nd][2] = 0;
			nd++;
			if (v < 0100)
				break;
			v >>= 6;
		}
		for (int k = nd - 1; k >= 0; k--) {
			*p++ = dirs[k][0];
			*p++ = dirs[k][1];
			*p++ = '/';
		}
	}
	snprintf(p, sizeof(tmp) - (size_t) (p - tmp), "%" PRIo64, id);
	snprintf(s, len, "%s", tmp);
}

}  // namespace

extern "C" int
mgdk_BBPreaddir(const char *path, mgdk_bbpentry *out, int maxn, int *nout)
{
	if (path == nullptr || nout == nullptr) {
		seterr("BBPreaddir: NULL argument");
		return -1;
	}
	FILE *fp = fopen(path, "r");
	if (fp == nullptr) {
		seterr("BBPreaddir: cannot open %s: %s", path, strerror(errno));
		return -1;
	}
	char buf[4096];
	unsigned version = 0;
	int rc = -1, n = 0, lineno = 0;
	int szsize = 0, szoid = 0, szhge = 0;
	if (!fgets(buf, sizeof(buf), fp) || sscanf(buf, "BBP.dir, GDKversion %u", &version) != 1) {
		seterr("BBPreaddir: %s is not a BBP.dir", path);
		goto out;
	}
	// gdk_bbp.c:990-998 refuses newer versions; older ones (which the
	// reference upgrades in place) use other line formats than the one parsed here
	if (version != 061050U) {
		seterr("BBPreaddir: incompatible BBP version: expected 0%o, got 0%o (%s)", 061050U, version,
		       version > 061050U ? "newer" : "too old");
		goto out;
	}
	if (!fgets(buf, sizeof(buf), fp) || sscanf(buf, "%d %d %d", &szsize, &szoid, &szhge) != 3 || szoid != 8) {
		seterr("BBPreaddir: incompatible BBP.dir sizes line");
		goto out;
	}
	lineno = 2;
	while (fgets(buf, sizeof(buf), fp)) {
		lineno++;
		if (strncmp(buf, "BBPsize=", 8) == 0 || strncmp(buf, "BBPinfo=", 8) == 0)
			continue;
		char *nl = strpbrk(buf, "\r\n");
		if (nl)
			*nl = 0;
		mgdk_bbpentry e;
		memset(&e, 0, sizeof(e));
		unsigned restricted = 0, props = 0, width = 0, var = 0;
		uint64_t count, hseq, nokey0, nokey1, nosorted, norevsorted, tseq, freeb, minpos, maxpos;
		int nread = 0;
		if (sscanf(buf, "%" SCNd64 " %128s %u %" SCNu64 " %" SCNu64 "%n", &e.batid, e.name, &restricted, &count,
			   &hseq, &nread) < 5) {
			seterr("BBPreaddir: invalid format on line %d", lineno);
			goto out;
		}
		int n2 = 0;
		if (sscanf(buf + nread,
			   " %32s %u %u %u %" SCNu64 " %" SCNu64 " %" SCNu64 " %" SCNu64 " %" SCNu64 " %" SCNu64
			   " %" SCNu64 " %" SCNu64 "%n",
			   e.type, &width, &var, &props, &nokey0, &nokey1, &nosorted, &norevsorted, &tseq, &freeb, &minpos,
			   &maxpos, &n2) < 12) {
			seterr("BBPreaddir: invalid heap entry on line %d", lineno);
			goto out;
		}
		nread += n2;
		e.tt = type_of(e.type);
		e.width = (int32_t) width;
		e.var = (int32_t) (var & ~2u);
		e.props = props;
		e.count = count;
		e.hseqbase = hseq;
		e.tseqbase = (props & 0x0200) == 0 || tseq >= MGDK_OID_NIL ? MGDK_OID_NIL : tseq;
		e.free = freeb;
		if (e.var && e.tt != MGDK_void) {
			uint64_t vfree = 0;
			int n3 = 0;
			if (sscanf(buf + nread, " %" SCNu64 "%n", &vfree, &n3) < 1) {
				seterr("BBPreaddir: invalid var heap entry on line %d", lineno);
				goto out;
			}
			nread += n3;
			e.vfree = vfree;
		}
		char phys[64];
		physical_name(e.batid, phys, sizeof(phys));
		const char *ext = ".tail";
		if (e.tt == MGDK_str)
			ext = width <= 1 ? ".tail1" : width == 2 ? ".tail2" : width == 4 ? ".tail4" : ".tail";
		snprintf(e.tail, sizeof(e.tail), "%s%s", phys, ext);
		if (e.var && e.tt != MGDK_void)
			snprintf(e.theap, sizeof(e.theap), "%s.theap", phys);
		if (out && n < maxn)
			out[n] = e;
		n++;
	}
	*nout = n;
	rc = 0;
out:
	fclose(fp);
	return rc;
}

// HEAPload (gdk_heap.c:729) into HBM: the tail file of e under bat_dir
extern "C" mgdk_bat *
mgdk_BATload(const char *bat_dir, const mgdk_bbpentry *e)
{
	if (bat_dir == nullptr || e == nullptr) {
		seterr("BATload: NULL argument");
		return nullptr;
	}
	if (e->tt < 0 || e->tt == MGDK_msk) {
		seterr("42000!BATload: type %s not supported on the device path", e->type);
		return nullptr;
	}
	if (e->tt == MGDK_void) {
		mgdk_bat *b = mgdk_BATdense(e->hseqbase, e->tseqbase, e->count);
		return b;
	}
	const int w = e->tt == MGDK_str ? e->width : width_of(e->tt);
	if (w <= 0 || (e->tt != MGDK_str && w != e->width)) {
		seterr("BATload: width %d does not match type %s", e->width, e->type);
		return nullptr;
	}
	ProfScope prof("batload");
	char path[1024];
	snprintf(path, sizeof(path), "%s/%s", bat_dir, e->tail);
	const size_t bytes = (size_t) e->count * (size_t) w;
	// HEAPsave writes no file for an empty heap (gdk_heap.c:871-884) and
	// HEAPload creates an empty one (:826-831): nothing to read then
	FILE *fp = bytes ? fopen(path, "rb") : nullptr;
	if (bytes && fp == nullptr) {
		seterr("BATload: cannot open %s: %s", path, strerror(errno));
		return nullptr;
	}
	// str: the tail holds heap offsets of e->width bytes
	mgdk_bat *b = newbat(e->hseqbase, e->tt, e->tt == MGDK_str ? e->count * (BUN) w : e->count);
	if (b == nullptr) {
		if (fp)
			fclose(fp);
		return nullptr;
	}
	b->twidth = w;
	const size_t CH = (size_t) 64 << 20;
	hipStream_t st = stream();
	char *stage = nullptr;
	if (bytes && !hip_ok(hipHostMalloc((void **) &stage, 2 * CH, hipHostMallocDefault), "hipHostMalloc"))
		stage = nullptr;
	hipEvent_t ev[2];
	bool okev = hip_ok(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming), "event") &&
		    hip_ok(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming), "event");
	bool ok = (bytes == 0 || stage != nullptr) && okev;
	bool used[2] = {false, false};
	size_t off = 0;
	int k = 0;
	while (ok && off < bytes) {
		const size_t len = bytes - off < CH ? bytes - off : CH;
		if (used[k] && !hip_ok(hipEventSynchronize(ev[k]), "event sync")) {
			ok = false;
			break;
		}
		char *buf = stage + (size_t) k * CH;
		if (fread(buf, 1, len, fp) != len) {
			seterr("BATload: %s is shorter than %zu bytes", path, bytes);
			ok = false;
			break;
		}
		ok = hip_ok(hipMemcpyAsync((char *) b->theap + off, buf, len, hipMemcpyHostToDevice, st), "memcpy H2D") &&
		     hip_ok(hipEventRecord(ev[k], st), "event");
		used[k] = true;
		off += len;
		k ^= 1;
	}
	if (fp)
		fclose(fp);
	ok = ok && sync();
	if (okev) {
		(void) hipEventDestroy(ev[0]);
		(void) hipEventDestroy(ev[1]);
	}
	if (stage)
		(void) hipHostFree(stage);
	if (ok && e->tt == MGDK_str && e->theap[0] && e->vfree == 0) {
		ok = mgdk_BATsetvheap(b, nullptr, 0) == 0;
	} else if (ok && e->tt == MGDK_str && e->theap[0]) {
		snprintf(path, sizeof(path), "%s/%s", bat_dir, e->theap);
		FILE *vf = fopen(path, "rb");
		std::vector<char> vh(e->vfree ? e->vfree : 1);
		if (vf == nullptr || (e->vfree && fread(vh.data(), 1, e->vfree, vf) != e->vfree)) {
			seterr("BATload: cannot read string heap %s", path);
			ok = false;
		}
		if (vf)
			fclose(vf);
		ok = ok && mgdk_BATsetvheap(b, vh.data(), e->vfree) == 0;
	}
	if (!ok) {
		mgdk_BBPunfix(b);
		return nullptr;
	}
	b->count = e->count;
	b->tsorted = (e->props & 0x0001) != 0;
	b->trevsorted = (e->props & 0x0080) != 0;
	b->tkey = (e->props & 0x0100) != 0;
	b->tnonil = (e->props & 0x0400) != 0;
	b->tnil = (e->props & 0x0800) != 0;
	return b;
}
