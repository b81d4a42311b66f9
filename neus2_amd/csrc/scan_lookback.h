// Single-pass decoupled look-back scan pieces (scan.hip's generic exclusive scan and the fused scans of march.hip).
//
// A launch scans 4096-element tiles (256 threads x 16 consecutive elements), tile = blockIdx.x. Each tile publishes an
// 8-byte {flag, tag, value} word with an agent-scope atomic store (the data is the flag: no fence pairs); its first
// wave reads up to 64 predecessors' words per pass, relaxed, until every word of the window carries this launch's tag,
// and sums back to the nearest inclusive prefix. Forward progress rests on in-order workgroup dispatch: the blocks of a
// launch are dispatched in blockIdx order, so every predecessor of a spinning tile has been dispatched (it is running or
// done) and none waits for the spinning tile's slot. (Residency is not the argument: SCAN_MAX_TILES blocks need not all
// fit at once.) The spin is bounded anyway: a give-up counts in ScanState::fail, which the training step reads back and
// raises as an error (testbed.cpp health_raise), so a wrong scan never passes silently. The tag is a per-state launch counter kept on the host (scan_next_tag), so a word left by
// an earlier launch never matches and the state needs no per-call memset: it is zeroed once after allocation
// (scan_temp_reset). Every shared word is a global-address-space agent-scope access (sc1).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace neus {

constexpr uint32_t SCAN_TILE = 4096, SCAN_THREADS = 256, SCAN_ITEMS = SCAN_TILE / SCAN_THREADS, SCAN_MAX_TILES = 4096;
struct ScanState {
	unsigned long long status[2][SCAN_MAX_TILES];  // two independent sums per launch; [63:62] flag (1 aggregate, 2 inclusive), [61:32] tag, [31:0] value
	uint32_t fail;                                 // bounded-wait give-ups
	uint32_t pad_[3];
};
constexpr size_t SCAN_STATE_BYTES = (sizeof(ScanState) + 255) / 256 * 256;

typedef __attribute__((address_space(1))) unsigned long long scan_gu64;
typedef __attribute__((address_space(1))) uint32_t scan_gu32;
__device__ __forceinline__ unsigned long long scan_ld(const unsigned long long* p) {
	return __hip_atomic_load((scan_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void scan_st(unsigned long long* p, unsigned long long v) {
	__hip_atomic_store((scan_gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct ScanTile { uint32_t tile; unsigned long long tag; };
// tag: the launch's scan_next_tag value (1 .. 2^30 - 1)
__device__ __forceinline__ ScanTile scan_tile(uint32_t tag) { return ScanTile{blockIdx.x, (unsigned long long)tag << 32}; }

// wave 0 only: publishes the tile's aggregate, looks back, publishes the inclusive prefix; returns the tile's exclusive
// prefix (every lane)
__device__ __forceinline__ uint32_t scan_lookback(ScanState* st, int which, const ScanTile& t, uint32_t agg) {
	constexpr unsigned long long AGG = 1ull << 62, INCL = 2ull << 62;
	unsigned long long* status = st->status[which];
	const uint32_t lane = threadIdx.x & 63;
	if (t.tile == 0) {
		if (lane == 0) scan_st(&status[0], INCL | t.tag | agg);
		return 0u;
	}
	if (lane == 0) scan_st(&status[t.tile], AGG | t.tag | agg);
	uint32_t excl = 0;
	int64_t j = (int64_t)t.tile - 1;  // the window's nearest predecessor (lane 0)
	uint32_t spins = 0;
	for (;;) {
		const int64_t idx = j - (int64_t)lane;
		unsigned long long x = 0;
		for (;;) {
			x = idx >= 0 ? scan_ld(&status[idx]) : (INCL | t.tag);
			const bool ready = (x & (0x3fffffffull << 32)) == t.tag && (x >> 62) != 0;
			if (__all(ready)) break;
			if (++spins > (1u << 22)) {  // bounded: a corrupted state gives a wrong scan and a fail count, not a hang
				if (lane == 0) __hip_atomic_fetch_add((scan_gu32*)&st->fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				x = INCL | t.tag;
				break;
			}
			__builtin_amdgcn_s_sleep(1);
		}
		const unsigned long long inc_mask = __ballot((x >> 62) == 2);
		const uint32_t val = (uint32_t)x;
		uint32_t s = val;
		if (inc_mask) {
			const int p = __builtin_ctzll(inc_mask);  // the nearest inclusive prefix
			s = (int)lane <= p ? val : 0u;
		}
#pragma unroll
		for (int off = 32; off > 0; off >>= 1) s += (uint32_t)__shfl_xor((int)s, off);
		excl += s;
		if (inc_mask) break;
		j -= 64;
	}
	if (lane == 0) scan_st(&status[t.tile], INCL | t.tag | (uint32_t)(excl + agg));
	return excl;
}

// block-wide: thread sum -> the thread's exclusive prefix inside the tile (return) and the tile total (agg)
__device__ __forceinline__ uint32_t scan_block(uint32_t tsum, uint32_t* s_wsum /* SCAN_THREADS / 64 words */, uint32_t& agg) {
	const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	uint32_t incl = tsum;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) { const uint32_t y = (uint32_t)__shfl_up((int)incl, d); if ((int)lane >= d) incl += y; }
	if (lane == 63) s_wsum[wv] = incl;
	__syncthreads();
	uint32_t wbefore = 0;
	agg = 0;
#pragma unroll
	for (int w = 0; w < (int)(SCAN_THREADS / 64); ++w) { if (w < (int)wv) wbefore += s_wsum[w]; agg += s_wsum[w]; }
	return wbefore + incl - tsum;
}

// 16 consecutive u32 of this thread (zeros past n); vec: 16-B aligned buffer
__device__ __forceinline__ void scan_load16(const uint32_t* in, size_t b0, uint32_t n, bool vec, uint32_t (&v)[SCAN_ITEMS]) {
	if (vec && b0 + SCAN_ITEMS <= n) {
		const uint4* p = (const uint4*)(in + b0);
#pragma unroll
		for (int q = 0; q < (int)SCAN_ITEMS / 4; ++q) { const uint4 u = p[q]; v[4 * q] = u.x; v[4 * q + 1] = u.y; v[4 * q + 2] = u.z; v[4 * q + 3] = u.w; }
	} else {
#pragma unroll
		for (int k = 0; k < (int)SCAN_ITEMS; ++k) v[k] = b0 + k < n ? in[b0 + k] : 0u;
	}
}
__device__ __forceinline__ void scan_store16(uint32_t* out, size_t b0, uint32_t n, bool vec, const uint32_t (&v)[SCAN_ITEMS]) {
	if (vec && b0 + SCAN_ITEMS <= n) {
		uint4* p = (uint4*)(out + b0);
#pragma unroll
		for (int q = 0; q < (int)SCAN_ITEMS / 4; ++q) p[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
	} else {
#pragma unroll
		for (int k = 0; k < (int)SCAN_ITEMS; ++k) if (b0 + k < n) out[b0 + k] = v[k];
	}
}

} // namespace neus
