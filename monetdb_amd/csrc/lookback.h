// lookback.h -- decoupled look-back for single-pass ordered compaction
// (select.hip, join.hip).  Per-tile 8-byte status granules {flag:2, count:62}
// written and polled with agent-scope relaxed atomics
// (MI355X_MICROARCH.md "Valid forms", R2 granule hand-off); tiles are
// numbered in dispatch order by an atomic ticket so every predecessor is
// already resident when a tile polls it.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mgdk_lb {

constexpr uint64_t ST_AGG = 1ull << 62, ST_PRE = 2ull << 62, ST_VAL = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t
lb_load(uint64_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void
lb_store(uint64_t *p, uint64_t v)
{
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Executed by one full wave; returns the exclusive prefix of `tile`.
// status[] must be zero before the launch.  A predecessor that never
// publishes (cannot happen with ticketed tiles) sets *err instead of hanging.
__device__ inline uint64_t
lookback(uint64_t *status, uint32_t tile, uint64_t agg, uint32_t *err, uint32_t maxspins = 1u << 26)
{
	const unsigned lane = __lane_id();
	if (tile == 0) {
		if (lane == 0)
			lb_store(&status[0], ST_PRE | agg);
		return 0;
	}
	if (lane == 0)
		lb_store(&status[tile], ST_AGG | agg);
	uint64_t excl = 0;
	int64_t base = (int64_t) tile - 1;
	for (;;) {
		int64_t idx = base - (int64_t) lane;
		uint64_t s = ST_PRE;
		if (idx >= 0) {
			uint32_t spins = 0;
			for (;;) {
				s = lb_load(&status[idx]);
				if ((s >> 62) != 0)
					break;
				if (++spins > maxspins) {
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
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			v += __shfl_xor(v, o);
		excl += v;
		if (pmask)
			break;
		base -= 64;
	}
	if (lane == 0)
		lb_store(&status[tile], ST_PRE | (excl + agg));
	return excl;
}


// XCD-grouped tile claims (sort.hip's claim_tile): the tiles are dealt to
// the XCDs in groups of xg consecutive tiles; each XCD claims its own tiles
// in order through its ticket xtk[xcd] and takes another XCD's when its own
// are gone.  A tile's predecessor may then be unclaimed while the tile
// waits on it (and stay so while the dispatcher has no room for the
// workgroup that would claim it), so a look-back over such claims must not
// wait for an unclaimed predecessor: xcd_claimed tells.
__device__ __forceinline__ uint32_t
claim_xcd_tile(uint32_t *xtk, uint32_t ntiles, uint32_t xg)
{
	const uint32_t x = (uint32_t) __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;   // HW_REG_XCC_ID
	for (uint32_t k = 0; k < 8; k++) {
		const uint32_t y = (x + k) & 7;
		const uint32_t j = atomicAdd(&xtk[y], 1u);
		const uint32_t t = (j / xg) * 8 * xg + y * xg + j % xg;
		if (t < ntiles)
			return t;
	}
	return ~0u;
}

// tile t has been claimed (every claim of it is an atomicAdd on its owner's
// ticket that passed it)
__device__ __forceinline__ bool
xcd_claimed(const uint32_t *xtk, uint64_t t, uint32_t xg)
{
	const uint32_t y = (uint32_t) (t / xg) & 7;
	const uint32_t j = (uint32_t) (t / (8 * (uint64_t) xg)) * xg + (uint32_t) (t % xg);
	return __hip_atomic_load(&xtk[y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > j;
}

}  // namespace mgdk_lb
