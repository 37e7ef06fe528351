// Probe-pass shape probe (tuning aid only, not part of the library): 60M
// (key, row) entries grouped by region, each looked up with ONE 16-byte
// bucket load in its region of a 150 MB bucketed table, (match, row) stored.
//   mode 0: stream only (no lookup) -- the ceiling
//   mode 1: regions dealt to XCDs (region r on XCD r % 8, regions in order):
//           a region's 1.17 MB of table stays in that XCD's L2
//   mode 2: the same entries, plain workgroup order (regions spread over
//           all XCDs: table lines served from the Infinity Cache)
//   mode 3: every lookup in a random region (whole table, Infinity Cache)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int U = 8, T = 256, CHUNK = U * T;
typedef unsigned v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix(uint32_t k) { return k * 0x9E3779B1u; }

template <int MODE>
__global__ __launch_bounds__(T) void
k_probe(const uint2 *ent, size_t n, const ulonglong2 *tab, uint32_t nreg, uint32_t nbp, uint32_t cpr, uint2 *out)
{
	uint32_t chunk;
	if (MODE == 1) {
		const uint32_t x = blockIdx.x & 7, k = blockIdx.x >> 3;
		const uint32_t per = nreg / 8;          // regions per XCD
		const uint32_t r = x + 8 * (k / cpr);
		chunk = r * cpr + k % cpr;
		if (k / cpr >= per)
			return;
	} else {
		chunk = blockIdx.x;
	}
	const size_t e0 = (size_t) chunk * CHUNK + threadIdx.x;
	v2u en[U];
#pragma unroll
	for (int u = 0; u < U; u++) {
		const size_t e = e0 + (size_t) u * T;
		en[u] = __builtin_nontemporal_load((const v2u *) ent + (e < n ? e : 0));
	}
	if (MODE != 0) {
		const uint32_t reg = chunk / cpr;
		ulonglong2 s[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t h = mix(en[u].x);
			const uint32_t rr = MODE == 3 ? (h >> 7) % nreg : reg;
			s[u] = tab[(size_t) rr * nbp + __umulhi(h, nbp)];
		}
#pragma unroll
		for (int u = 0; u < U; u++)
			en[u].x = (uint32_t) s[u].x == en[u].x ? (uint32_t) (s[u].x >> 32) : (uint32_t) s[u].y;
	} else {
#pragma unroll
		for (int u = 0; u < U; u++)
			en[u].x ^= 0x5bd1e995u;
	}
#pragma unroll
	for (int u = 0; u < U; u++) {
		const size_t e = e0 + (size_t) u * T;
		if (e < n)
			__builtin_nontemporal_store(en[u], (v2u *) out + e);
	}
}

int
main(int argc, char **argv)
{
	const uint32_t nreg = 128, cpr = 229;
	const size_t n = (size_t) nreg * cpr * CHUNK;     // 60.0M entries
	const uint32_t nbp = argc > 1 ? atoi(argv[1]) : 73216;   // buckets per region (1.17 MB)
	std::vector<uint2> h(n);
	uint32_t x = 12345;
	for (size_t i = 0; i < n; i++) {
		x ^= x << 13; x ^= x >> 17; x ^= x << 5;
		h[i] = make_uint2(x, (uint32_t) i);
	}
	uint2 *ent, *out;
	ulonglong2 *tab;
	CK(hipMalloc(&ent, n * 8));
	CK(hipMalloc(&out, n * 8));
	CK(hipMalloc(&tab, (size_t) nreg * nbp * 16));
	CK(hipMemcpy(ent, h.data(), n * 8, hipMemcpyHostToDevice));
	CK(hipMemset(tab, 0x11, (size_t) nreg * nbp * 16));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	const uint32_t grid = nreg * cpr;
	for (int mode = 0; mode < 4; mode++) {
		float best = 1e9;
		for (int rep = 0; rep < 6; rep++) {
			CK(hipEventRecord(a));
			switch (mode) {
			case 0: hipLaunchKernelGGL(k_probe<0>, dim3(grid), dim3(T), 0, 0, ent, n, tab, nreg, nbp, cpr, out); break;
			case 1: hipLaunchKernelGGL(k_probe<1>, dim3(grid), dim3(T), 0, 0, ent, n, tab, nreg, nbp, cpr, out); break;
			case 2: hipLaunchKernelGGL(k_probe<2>, dim3(grid), dim3(T), 0, 0, ent, n, tab, nreg, nbp, cpr, out); break;
			default: hipLaunchKernelGGL(k_probe<3>, dim3(grid), dim3(T), 0, 0, ent, n, tab, nreg, nbp, cpr, out); break;
			}
			CK(hipEventRecord(b));
			CK(hipEventSynchronize(b));
			float ms;
			CK(hipEventElapsedTime(&ms, a, b));
			if (rep > 0 && ms < best)
				best = ms;
		}
		printf("mode %d: %.4f ms  (%.2f TB/s of entry bytes in+out)\n", mode, best, n * 16 / best / 1e9);
	}
	return 0;
}
