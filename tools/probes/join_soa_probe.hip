// Join plan shape probe (tuning aid only, not part of the library): the
// probe side of a partitioned hash join with subtile-local partitioning and
// split key / row arrays, timed pass by pass on 60M shuffled 4-byte keys.
//   K1 scatter  per 32 Ki-row subtile: keys counting-sorted by partition in
//               LDS, stored contiguously in the subtile's own region (4-B
//               keys, 2-B local rows in a second array) + the subtile's
//               partition offsets (P + 1 uint16)
//   K2 probe    one workgroup per partition: an LDS table lookup per key of
//               its run in every subtile, the 4-B answer stored at the key's
//               own index (runs of ~S / P entries)
//   K3 restore  per subtile: answers dropped into an LDS row array through
//               the local rows, then r1 (row oid) / r2 (answer) stored as
//               8-B oids, contiguous
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint32_t S = 32768;           // rows per subtile
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned long long v2ul __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t part_of(uint32_t k, int pbits) { return (k * 0x9E3779B1u) >> (32 - pbits); }

__global__ __launch_bounds__(1024) void
k1_scatter(const uint32_t *key, size_t n, int pbits, uint32_t *okey, uint16_t *orow, uint16_t *off)
{
	extern __shared__ uint32_t sm[];
	const uint32_t P = 1u << pbits;
	uint32_t *hist = sm, *start = sm + P, *stk = sm + 2 * P;     // stk: S keys
	uint16_t *str = (uint16_t *) stk;                              // S rows, after the keys left
	__shared__ uint32_t wsum[16];
	const size_t a = (size_t) blockIdx.x * S;
	const unsigned tid = threadIdx.x;
	for (uint32_t p = tid; p < P; p += 1024)
		hist[p] = 0;
	__syncthreads();
	uint32_t k[32], rk[32];
	const v4u *src = (const v4u *) (key + a);
#pragma unroll
	for (int q = 0; q < 8; q++) {
		const v4u v = __builtin_nontemporal_load(src + q * 1024 + tid);
		k[4 * q] = v.x; k[4 * q + 1] = v.y; k[4 * q + 2] = v.z; k[4 * q + 3] = v.w;
	}
#pragma unroll
	for (int q = 0; q < 32; q++)
		rk[q] = atomicAdd(&hist[part_of(k[q], pbits)], 1u);
	__syncthreads();
	// exclusive scan of hist (P <= 4096)
	const uint32_t per = (P + 1023) / 1024;
	uint32_t loc[4], t = 0;
	for (uint32_t q = 0; q < per; q++) {
		const uint32_t p = tid * per + q;
		loc[q] = p < P ? hist[p] : 0;
		t += loc[q];
	}
	uint32_t x = t;
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t u = __shfl_up(x, o);
		if (__lane_id() >= (unsigned) o)
			x += u;
	}
	if (__lane_id() == 63)
		wsum[tid >> 6] = x;
	__syncthreads();
	uint32_t pre = x - t;
	for (uint32_t w = 0; w < (tid >> 6); w++)
		pre += wsum[w];
	for (uint32_t q = 0; q < per; q++) {
		const uint32_t p = tid * per + q;
		if (p < P) {
			start[p] = pre;
			off[(size_t) blockIdx.x * (P + 1) + p] = (uint16_t) pre;
		}
		pre += loc[q];
	}
	if (tid == 0)
		off[(size_t) blockIdx.x * (P + 1) + P] = (uint16_t) 0;   // S wraps to 0 in uint16: end = S
	__syncthreads();
#pragma unroll
	for (int q = 0; q < 32; q++) {
		rk[q] += start[part_of(k[q], pbits)];
		stk[rk[q]] = k[q];
	}
	__syncthreads();
	v4u *dk = (v4u *) (okey + a);
#pragma unroll
	for (int q = 0; q < 8; q++)
		__builtin_nontemporal_store(((v4u *) stk)[q * 1024 + tid], dk + q * 1024 + tid);
	__syncthreads();
#pragma unroll
	for (int q = 0; q < 32; q++)
		str[rk[q]] = (uint16_t) ((q >> 2) * 4096 + tid * 4 + (q & 3));
	__syncthreads();
	v4u *dr = (v4u *) (orow + a);
#pragma unroll
	for (int q = 0; q < 4; q++)
		__builtin_nontemporal_store(((v4u *) str)[q * 1024 + tid], dr + q * 1024 + tid);
}

// transpose of the offsets: offT[p][s] = start of (s, p) run, offT[P][s] = S
__global__ __launch_bounds__(256) void
k_off_t(const uint16_t *off, uint32_t nsub, uint32_t P, uint16_t *offT)
{
	__shared__ uint16_t t[64][65];
	const uint32_t s0 = blockIdx.x * 64, p0 = blockIdx.y * 64;
	for (uint32_t k = threadIdx.x; k < 64 * 64; k += 256) {
		const uint32_t r = k / 64, c = k % 64;
		if (s0 + r < nsub && p0 + c <= P)
			t[r][c] = off[(size_t) (s0 + r) * (P + 1) + p0 + c];
	}
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < 64 * 64; k += 256) {
		const uint32_t r = k / 64, c = k % 64;
		if (s0 + c < nsub && p0 + r <= P)
			offT[(size_t) (p0 + r) * nsub + s0 + c] = t[c][r];
	}
}

// one workgroup per partition; lane-per-run gathers (a lane walks its
// subtiles' runs, 4 keys per 16-B load where aligned)
template <int MODE>
__global__ __launch_bounds__(256) void
k2_probe(const uint32_t *okey, const uint16_t *offT, uint32_t nsub, uint32_t P, uint32_t *ans)
{
	__shared__ uint32_t tab[16384];
	const uint32_t p = blockIdx.x;
	for (uint32_t i = threadIdx.x; i < 16384; i += 256)
		tab[i] = i * 2654435761u;
	__syncthreads();
	const uint16_t *o0 = offT + (size_t) p * nsub, *o1 = offT + (size_t) (p + 1) * nsub;
	if (MODE == 0) {
		// lane per run
		for (uint32_t s = threadIdx.x; s < nsub; s += 256) {
			const uint32_t b = o0[s], e = p + 1 == P ? S : o1[s];
			const size_t base = (size_t) s * S;
			for (uint32_t j = b; j < e; j++) {
				const uint32_t k = okey[base + j];
				ans[base + j] = tab[(k * 0x85ebca6bu) >> 18] ^ k;
			}
		}
	} else {
		// wave per run group: 64 lanes cover a run's entries (runs ~16: 4
		// runs per wave instruction, lanes split 16 / run)
		const unsigned lane = __lane_id(), w = threadIdx.x >> 6;
		for (uint32_t s0 = w * 4; s0 < nsub; s0 += 16) {
			const uint32_t s = s0 + lane / 16, q = lane % 16;
			if (s >= nsub)
				continue;
			const uint32_t b = o0[s], e = p + 1 == P ? S : o1[s];
			const size_t base = (size_t) s * S;
			for (uint32_t j = b + q; j < e; j += 16) {
				const uint32_t k = okey[base + j];
				ans[base + j] = tab[(k * 0x85ebca6bu) >> 18] ^ k;
			}
		}
	}
}

__global__ __launch_bounds__(1024) void
k3_restore(const uint16_t *orow, const uint32_t *ans, size_t n, unsigned long long *r1, unsigned long long *r2)
{
	extern __shared__ uint32_t m[];     // S answers by local row
	const size_t a = (size_t) blockIdx.x * S;
	const unsigned tid = threadIdx.x;
	const v4u *sa = (const v4u *) (ans + a);
	const uint2 *sr = (const uint2 *) (orow + a);
	v4u aa[8];
	uint2 rr[8];
#pragma unroll
	for (int q = 0; q < 8; q++) {
		aa[q] = __builtin_nontemporal_load(sa + q * 1024 + tid);
		rr[q] = sr[q * 1024 + tid];
	}
#pragma unroll
	for (int q = 0; q < 8; q++) {
		m[rr[q].x & 0xffff] = aa[q].x;
		m[rr[q].x >> 16] = aa[q].y;
		m[rr[q].y & 0xffff] = aa[q].z;
		m[rr[q].y >> 16] = aa[q].w;
	}
	__syncthreads();
	v2ul *d1 = (v2ul *) (r1 + a), *d2 = (v2ul *) (r2 + a);
#pragma unroll 4
	for (int q = 0; q < 16; q++) {
		const uint32_t i = q * 2048 + tid * 2;
		__builtin_nontemporal_store((v2ul) {a + i, a + i + 1}, d1 + q * 1024 + tid);
		__builtin_nontemporal_store((v2ul) {m[i], m[i + 1]}, d2 + q * 1024 + tid);
	}
}

int
main(int argc, char **argv)
{
	const int pbits = argc > 1 ? atoi(argv[1]) : 11;
	const uint32_t P = 1u << pbits;
	const uint32_t nsub = 1831;
	const size_t n = (size_t) nsub * S;     // 60.0M
	std::vector<uint32_t> h(n);
	uint32_t x = 12345;
	for (size_t i = 0; i < n; i++) {
		x ^= x << 13; x ^= x >> 17; x ^= x << 5;
		h[i] = x;
	}
	uint32_t *key, *okey, *ans;
	uint16_t *orow, *off, *offT;
	unsigned long long *r1, *r2;
	CK(hipMalloc(&key, n * 4));
	CK(hipMalloc(&okey, n * 4));
	CK(hipMalloc(&ans, n * 4));
	CK(hipMalloc(&orow, n * 2));
	CK(hipMalloc(&off, (size_t) nsub * (P + 1) * 2));
	CK(hipMalloc(&offT, (size_t) nsub * (P + 1) * 2));
	CK(hipMalloc(&r1, n * 8));
	CK(hipMalloc(&r2, n * 8));
	CK(hipMemcpy(key, h.data(), n * 4, hipMemcpyHostToDevice));
	const size_t lds1 = (2 * P + S) * 4;
	CK(hipFuncSetAttribute((const void *) k1_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds1));
	CK(hipFuncSetAttribute((const void *) k3_restore, hipFuncAttributeMaxDynamicSharedMemorySize, (int) (S * 4)));
	hipEvent_t ev[6];
	for (auto &e : ev)
		CK(hipEventCreate(&e));
	float best[5] = {1e9, 1e9, 1e9, 1e9, 1e9};
	for (int rep = 0; rep < 6; rep++) {
		CK(hipEventRecord(ev[0]));
		hipLaunchKernelGGL(k1_scatter, dim3(nsub), dim3(1024), lds1, 0, key, n, pbits, okey, orow, off);
		CK(hipEventRecord(ev[1]));
		hipLaunchKernelGGL(k_off_t, dim3((nsub + 63) / 64, (P + 1 + 63) / 64), dim3(256), 0, 0, off, nsub, P, offT);
		CK(hipEventRecord(ev[2]));
		hipLaunchKernelGGL(k2_probe<0>, dim3(P), dim3(256), 0, 0, okey, offT, nsub, P, ans);
		CK(hipEventRecord(ev[3]));
		hipLaunchKernelGGL(k2_probe<1>, dim3(P), dim3(256), 0, 0, okey, offT, nsub, P, ans);
		CK(hipEventRecord(ev[4]));
		hipLaunchKernelGGL(k3_restore, dim3(nsub), dim3(1024), S * 4, 0, orow, ans, n, r1, r2);
		CK(hipEventRecord(ev[5]));
		CK(hipEventSynchronize(ev[5]));
		for (int k = 0; k < 5; k++) {
			float ms;
			CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
			if (rep > 0 && ms < best[k])
				best[k] = ms;
		}
	}
	printf("P %u: scatter %.4f  offT %.4f  probe(lane/run) %.4f  probe(16 lanes/run) %.4f  restore %.4f ms\n", P,
	       best[0], best[1], best[2], best[3], best[4]);
	return 0;
}
