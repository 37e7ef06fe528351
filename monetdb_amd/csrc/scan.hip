// scan.hip -- device-wide exclusive prefix sum (decoupled look-back), used by
// the radix sort, the hash join and the window bounds.
//
// Tile = 256 lanes x 16 consecutive items; a lane scans its 16 items
// serially, the block scans the 256 lane totals in LDS (wave scans via
// __shfl_up), and tiles chain through 8-byte {flag, value} granules polled
// with agent-scope relaxed atomics; tiles are numbered by a ticket so that
// every predecessor is resident (same protocol as k_select).
#include "mgdk_internal.h"

using namespace mgdk;

namespace {

constexpr uint64_t ST_AGG = 1ull << 62, ST_PRE = 2ull << 62, ST_VAL = (1ull << 62) - 1;
constexpr int ITEMS = 64;

__device__ uint64_t
lookback64(uint64_t *status, uint32_t tile, uint64_t agg, uint32_t *err)
{
	const unsigned lane = __lane_id();
	if (tile == 0) {
		if (lane == 0)
			__hip_atomic_store(&status[0], ST_PRE | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		return 0;
	}
	if (lane == 0)
		__hip_atomic_store(&status[tile], ST_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	uint64_t excl = 0;
	int64_t base = (int64_t) tile - 1;
	for (;;) {
		int64_t idx = base - (int64_t) lane;
		uint64_t s = ST_PRE;
		if (idx >= 0) {
			uint32_t spins = 0;
			for (;;) {
				s = __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				if ((s >> 62) != 0)
					break;
				if (++spins > (1u << 26)) {
					atomicOr(err, 1u);
					s = ST_PRE;
					break;
				}
				__builtin_amdgcn_s_sleep(1);
			}
		}
		uint64_t pmask = __ballot((s >> 62) == 2);
		int first = pmask ? __ffsll((long long) pmask) - 1 : 64;
		uint64_t v = ((int) lane <= first) ? (s & ST_VAL) : 0;
		for (int o = 32; o > 0; o >>= 1)
			v += __shfl_xor(v, o);
		excl += v;
		if (pmask)
			break;
		base -= 64;
	}
	if (lane == 0)
		__hip_atomic_store(&status[tile], ST_PRE | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	return excl;
}

// a lane sums its ITEMS consecutive inputs with 16-byte loads (pass 1), the
// tile is scanned, then the lane re-reads them (cache-resident) and writes
// its outputs (pass 2); 64 items per lane keeps tile tickets to one per
// 16 Ki items (a single ticket counter sustains ~88 atomics/us)
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void
k_scan(const TI *in, TO *out, BUN n, uint64_t *status, uint32_t *ticket, uint32_t ntiles,
       uint64_t *total, uint32_t *err)
{
	constexpr int VI = 16 / sizeof(TI);
	typedef TI vec_t __attribute__((ext_vector_type(VI)));
	__shared__ uint32_t s_tile;
	__shared__ uint64_t s_wave[4];
	__shared__ uint64_t s_prefix;
	const unsigned tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	if (tid == 0)
		s_tile = atomicAdd(ticket, 1u);
	__syncthreads();
	const uint32_t tile = s_tile;
	const BUN base = ((BUN) tile * 256 + tid) * ITEMS;
	const bool fullv = base + ITEMS <= n;
	uint64_t sum = 0;
	if (fullv) {
#pragma unroll
		for (int k = 0; k < ITEMS; k += VI) {
			vec_t x = *(const vec_t *) (in + base + k);
#pragma unroll
			for (int q = 0; q < VI; q++)
				sum += (uint64_t) x[q];
		}
	} else {
		for (int k = 0; k < ITEMS; k++)
			if (base + k < n)
				sum += (uint64_t) in[base + k];
	}
	// inclusive wave scan of lane sums
	uint64_t x = sum;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		uint64_t y = __shfl_up(x, o);
		if ((int) lane >= o)
			x += y;
	}
	if (lane == 63)
		s_wave[wave] = x;
	__syncthreads();
	uint64_t wpre = 0, agg = 0;
	for (int w = 0; w < 4; w++) {
		if (w < (int) wave)
			wpre += s_wave[w];
		agg += s_wave[w];
	}
	if (wave == 0) {
		uint64_t p = lookback64(status, tile, agg, err);
		if (lane == 0) {
			s_prefix = p;
			if (tile == ntiles - 1)
				*total = p + agg;
		}
	}
	__syncthreads();
	uint64_t run = s_prefix + wpre + x - sum;
	if (fullv) {
#pragma unroll
		for (int k = 0; k < ITEMS; k += VI) {
			vec_t xv = *(const vec_t *) (in + base + k);
#pragma unroll
			for (int q = 0; q < VI; q++) {
				out[base + k + q] = (TO) run;
				run += (uint64_t) xv[q];
			}
		}
	} else {
		for (int k = 0; k < ITEMS; k++) {
			if (base + k < n) {
				out[base + k] = (TO) run;
				run += (uint64_t) in[base + k];
			}
		}
	}
}

template <typename TI, typename TO>
int
scan_launch(const TI *in, TO *out, BUN n, uint64_t *ws)
{
	const uint64_t per = 256 * ITEMS;
	const uint64_t ntiles = (n + per - 1) / per;
	uint32_t *ticket = (uint32_t *) ws;
	uint64_t *status = ws + 8;
	hipStream_t s = stream();
	if (!hip_ok(hipMemsetAsync(ws, 0, (ntiles + 16) * 8, s), "memset"))
		return -1;
	hipLaunchKernelGGL((k_scan<TI, TO>), dim3((unsigned) ntiles), dim3(256), 0, s, in, out, n, status, ticket,
			   (uint32_t) ntiles, ws + 2, (uint32_t *) (ws + 3));
	return 0;
}

template <typename TI, typename TO>
int
scan_impl(const TI *in, TO *out, BUN n, uint64_t *total_host)
{
	if (n == 0) {
		if (total_host)
			*total_host = 0;
		return 0;
	}
	const uint64_t per = 256 * ITEMS;
	const uint64_t ntiles = (n + per - 1) / per;
	DevBuf st((ntiles + 16) * 8);
	if (!st.p)
		return -1;
	uint32_t *ticket = (uint32_t *) st.p;
	uint64_t *status = st.as<uint64_t>() + 8;
	uint64_t *total = st.as<uint64_t>() + 2;
	uint32_t *err = (uint32_t *) (st.as<uint64_t>() + 3);
	hipStream_t s = stream();
	if (!hip_ok(hipMemsetAsync(st.p, 0, (ntiles + 16) * 8, s), "memset"))
		return -1;
	hipLaunchKernelGGL((k_scan<TI, TO>), dim3((unsigned) ntiles), dim3(256), 0, s, in, out, n, status, ticket,
			   (uint32_t) ntiles, total, err);
	uint64_t *h = (uint64_t *) pinned(16);
	if (!hip_ok(hipMemcpyAsync(h, total, 16, hipMemcpyDeviceToHost, s), "memcpy") || !sync())
		return -1;
	if ((uint32_t) h[1]) {
		seterr("HY013!scan: look-back did not complete");
		return -1;
	}
	if (total_host)
		*total_host = h[0];
	return 0;
}

}  // namespace

namespace mgdk {

BUN
scan_ws_words(BUN n)
{
	return (n + 256 * ITEMS - 1) / (256 * ITEMS) + 16;
}

int
exclusive_scan_nosync(const uint32_t *in, uint64_t *out, BUN n, uint64_t *ws)
{
	if (n == 0)
		return hip_ok(hipMemsetAsync(ws, 0, 32, stream()), "memset") ? 0 : -1;
	return scan_launch<uint32_t, uint64_t>(in, out, n, ws);
}

int
exclusive_scan(const uint32_t *in, uint32_t *out, BUN n, uint64_t *total)
{
	return scan_impl<uint32_t, uint32_t>(in, out, n, total);
}

int
exclusive_scan(const uint32_t *in, uint64_t *out, BUN n, uint64_t *total)
{
	return scan_impl<uint32_t, uint64_t>(in, out, n, total);
}

int
exclusive_scan(const uint8_t *in, uint64_t *out, BUN n, uint64_t *total)
{
	return scan_impl<uint8_t, uint64_t>(in, out, n, total);
}

}  // namespace mgdk
