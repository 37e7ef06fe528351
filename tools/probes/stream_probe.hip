// HBM read-stream probe: register loads (nt / default) vs LDS-DMA
// (global_load_lds_dwordx4) rings, over a 16 GiB buffer.  Tuning aid only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_reg(const u4 *p, size_t n16, unsigned *out)
{
	unsigned acc = 0;
	const size_t stride = (size_t) gridDim.x * blockDim.x;
	size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
	for (; i + (U - 1) * stride < n16; i += U * stride) {
		u4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			v[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
		for (int u = 0; u < U; u++)
			acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

// each wave streams its own contiguous 1 KiB pieces through S LDS slots
template <int S, int AUX, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_glds(const u4 *p, size_t npieces, unsigned *out)
{
	__shared__ u4 ring[WPB][S][64];
	const int w = threadIdx.x / 64, lane = threadIdx.x % 64;
	const size_t nw = (size_t) gridDim.x * WPB;
	const size_t wid = (size_t) blockIdx.x * WPB + w;
	unsigned acc = 0;
	size_t k = wid;
	// prologue: S pieces in flight
	int issued = 0;
	for (int s = 0; s < S; s++) {
		size_t piece = wid + (size_t) s * nw;
		if (piece < npieces) {
			__builtin_amdgcn_global_load_lds((const void *) (p + piece * 64 + lane), (__attribute__((address_space(3))) void *) &ring[w][s][0], 16, 0, AUX);
			issued++;
		}
	}
	int slot = 0;
	for (; k < npieces; k += nw) {
		// oldest piece done when at most S-1 remain in flight
		__builtin_amdgcn_s_waitcnt(0x3f70 | ((S - 1) & 0xf) | (((S - 1) >> 4) << 14));
		u4 v = ring[w][slot][lane];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
		size_t nxt = k + (size_t) S * nw;
		if (nxt < npieces)
			__builtin_amdgcn_global_load_lds((const void *) (p + nxt * 64 + lane), (__attribute__((address_space(3))) void *) &ring[w][slot][0], 16, 0, AUX);
		else
			__builtin_amdgcn_s_waitcnt(0x3f70);   // drain: keep the count exact
		slot = slot + 1 == S ? 0 : slot + 1;
	}
	(void) issued;
	if (acc == 0x12345678u)
		out[0] = acc;
}

static float timeit(void (*launch)(const u4 *, size_t, unsigned *), const u4 *p, size_t n, unsigned *o)
{
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	launch(p, n, o);
	hipDeviceSynchronize();
	std::vector<float> t;
	for (int r = 0; r < 5; r++) {
		hipEventRecord(a);
		launch(p, n, o);
		hipEventRecord(b);
		hipEventSynchronize(b);
		float ms;
		hipEventElapsedTime(&ms, a, b);
		t.push_back(ms);
	}
	float best = t[0];
	for (float x : t) best = x < best ? x : best;
	return best;
}

#define REG(U, NT, BPC) [](const u4 *p, size_t n, unsigned *o) { hipLaunchKernelGGL((k_reg<U, NT>), dim3(256 * BPC), dim3(256), 0, 0, p, n / 16, o); }
#define GLDS(S, AUX, WPB, BPC) [](const u4 *p, size_t n, unsigned *o) { hipLaunchKernelGGL((k_glds<S, AUX, WPB>), dim3(256 * BPC), dim3(64 * WPB), 0, 0, p, n / 1024, o); }

int main(int argc, char **argv)
{
	const size_t bytes = argc > 1 ? (size_t) atoll(argv[1]) : (size_t) 16 << 30;
	u4 *p;
	unsigned *o;
	if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) {
		printf("alloc failed\n");
		return 1;
	}
	hipMemset(p, 1, bytes);
	struct V { const char *name; void (*f)(const u4 *, size_t, unsigned *); };
	V vs[] = {
		{"reg U2 nt bpc16", REG(2, true, 16)},
		{"reg U4 nt bpc8", REG(4, true, 8)},
		{"reg U2 def bpc16", REG(2, false, 16)},
		{"reg U4 def bpc16", REG(4, false, 16)},
		{"glds S4 nt wpb4 bpc4", GLDS(4, 2, 4, 4)},
		{"glds S8 nt wpb4 bpc2", GLDS(8, 2, 4, 2)},
		{"glds S8 nt wpb4 bpc4", GLDS(8, 2, 4, 4)},
		{"glds S8 def wpb4 bpc4", GLDS(8, 0, 4, 4)},
		{"glds S16 nt wpb4 bpc2", GLDS(16, 2, 4, 2)},
		{"glds S16 nt wpb1 bpc8", GLDS(16, 2, 1, 8)},
		{"glds S4 nt wpb4 bpc8", GLDS(4, 2, 4, 8)},
	};
	for (auto &v : vs) {
		float ms = timeit(v.f, p, bytes, o);
		printf("%-24s %8.3f ms  %6.3f TB/s\n", v.name, ms, bytes / ms / 1e9);
	}
	return 0;
}
