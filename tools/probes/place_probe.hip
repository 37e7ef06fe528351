// Placement-shape probe (tuning aid only, not part of the library): what does
// it cost the hash join's probe pass to drop each answer straight at its
// row instead of writing (match, row) entries for a restore pass?
// 60M (key, row) entries cut into P partitions (rows ascending inside a
// partition, as the partitioned join's subtile-major runs leave them); one
// 1024-thread workgroup per partition streams its entries and stores:
//   mode 0: (answer, row) 8 B at the entry's own place (today's probe output)
//   mode 1: the 4-B answer at out4[row] (scattered, plain stores)
//   mode 2: the same with nontemporal stores
//   mode 3: the 8-B answer at out8[row] (plain)
// then the finishing stream (read out4, write r1 / r2 as 8-B oids) is timed
// separately (mode 9).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int U = 8, T = 1024;
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t k) { return k * 0x9E3779B1u; }

template <int MODE>
__global__ __launch_bounds__(T) void
k_place(const uint2 *ent, const uint32_t *pbase, uint2 *out, uint32_t *out4, uint64_t *out8)
{
	const uint32_t p = blockIdx.x;
	const uint32_t q0 = pbase[p], q1 = pbase[p + 1];
	for (uint32_t e0 = q0 + threadIdx.x; e0 < q1; e0 += U * T) {
		uint2 en[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t e = e0 + u * T;
			{ const v2u t = __builtin_nontemporal_load((const v2u *) ent + (e < q1 ? e : q0)); en[u] = make_uint2(t.x, t.y); }
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t e = e0 + u * T;
			if (e >= q1)
				continue;
			const uint32_t a = mix(en[u].x) >> 8;
			if (MODE == 0)
				__builtin_nontemporal_store((v2u) {a, en[u].y}, (v2u *) out + e);
			else if (MODE == 1)
				out4[en[u].y] = a;
			else if (MODE == 2)
				__builtin_nontemporal_store(a, out4 + en[u].y);
			else
				out8[en[u].y] = a;
		}
	}
}

__global__ __launch_bounds__(256) void
k_finish(const uint32_t *out4, size_t n, uint64_t *r1, uint64_t *r2)
{
	const size_t i0 = ((size_t) blockIdx.x * 256 + threadIdx.x) * 4;
	if (i0 + 4 > n)
		return;
	const v4u m = __builtin_nontemporal_load((const v4u *) (out4 + i0));
	typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
	__builtin_nontemporal_store((u2) {i0, i0 + 1}, (u2 *) (r1 + i0));
	__builtin_nontemporal_store((u2) {i0 + 2, i0 + 3}, (u2 *) (r1 + i0 + 2));
	__builtin_nontemporal_store((u2) {m.x, m.y}, (u2 *) (r2 + i0));
	__builtin_nontemporal_store((u2) {m.z, m.w}, (u2 *) (r2 + i0 + 2));
}

int
main(int argc, char **argv)
{
	const size_t n = 60000000;
	const uint32_t P = argc > 1 ? atoi(argv[1]) : 2048;
	std::vector<uint32_t> part(n), cnt(P + 1, 0);
	uint32_t x = 12345;
	for (size_t i = 0; i < n; i++) {
		x ^= x << 13; x ^= x >> 17; x ^= x << 5;
		part[i] = x % P;
		cnt[part[i] + 1]++;
	}
	for (uint32_t p = 0; p < P; p++)
		cnt[p + 1] += cnt[p];
	std::vector<uint32_t> cur(cnt.begin(), cnt.end() - 1);
	std::vector<uint2> h(n);
	for (size_t i = 0; i < n; i++) {
		x ^= x << 13; x ^= x >> 17; x ^= x << 5;
		h[cur[part[i]]++] = make_uint2(x, (uint32_t) i);
	}
	uint2 *ent, *out;
	uint32_t *pb, *out4;
	uint64_t *out8, *r1, *r2;
	CK(hipMalloc(&ent, n * 8));
	CK(hipMalloc(&out, n * 8));
	CK(hipMalloc(&out4, n * 4));
	CK(hipMalloc(&out8, n * 8));
	CK(hipMalloc(&r1, n * 8));
	CK(hipMalloc(&r2, n * 8));
	CK(hipMalloc(&pb, (P + 1) * 4));
	CK(hipMemcpy(ent, h.data(), n * 8, hipMemcpyHostToDevice));
	CK(hipMemcpy(pb, cnt.data(), (P + 1) * 4, hipMemcpyHostToDevice));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	for (int mode : {0, 1, 2, 3, 9}) {
		float best = 1e9;
		for (int rep = 0; rep < 6; rep++) {
			CK(hipEventRecord(a));
			switch (mode) {
			case 0: hipLaunchKernelGGL(k_place<0>, dim3(P), dim3(T), 0, 0, ent, pb, out, out4, out8); break;
			case 1: hipLaunchKernelGGL(k_place<1>, dim3(P), dim3(T), 0, 0, ent, pb, out, out4, out8); break;
			case 2: hipLaunchKernelGGL(k_place<2>, dim3(P), dim3(T), 0, 0, ent, pb, out, out4, out8); break;
			case 3: hipLaunchKernelGGL(k_place<3>, dim3(P), dim3(T), 0, 0, ent, pb, out, out4, out8); break;
			default: hipLaunchKernelGGL(k_finish, dim3((n / 4 + 255) / 256), dim3(256), 0, 0, out4, n, r1, r2); break;
			}
			CK(hipEventRecord(b));
			CK(hipEventSynchronize(b));
			float ms;
			CK(hipEventElapsedTime(&ms, a, b));
			if (rep > 0 && ms < best)
				best = ms;
		}
		printf("P %u mode %d: %.4f ms\n", P, mode, best);
	}
	return 0;
}
