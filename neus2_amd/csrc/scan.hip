// Device-wide exclusive scans / sums for the deterministic ray / sample / record compaction (replacing the reference's
// atomicAdd appends, testbed_nerf.cu:1421-1428, 1682).
//
// Exclusive scan: ONE launch, single pass with decoupled look-back (scan_lookback.h) over 4096-element tiles (the
// step's scans are 2^18 ray counts and the scatter's ~1M bucket x block counts: 64 and ~260 tiles), instead of
// rocPRIM's init + scan pair. The state lives at the start of the caller's temp buffer and is zeroed once after its
// allocation (scan_temp_reset). Larger inputs (> 16M elements: marching cubes at high resolution) and the float sums
// go through hipCUB behind the state.
#include "kernels.h"
#include "scan_lookback.h"
#include <hipcub/hipcub.hpp>
#include <mutex>
#include <stdexcept>
#include <unordered_map>

namespace neus {

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_lookback(const uint32_t* in, uint32_t* out, uint32_t n, ScanState* __restrict__ st, uint32_t vec,
                                                                uint32_t tag, uint32_t tile_base) {
	__shared__ uint32_t s_prefix, s_wsum[SCAN_THREADS / 64];
	ScanTile tl = scan_tile(tag);
	tl.tile += tile_base;  // 0 (tests: 1, the first tile never runs)
	const size_t b0 = (size_t)tl.tile * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
	uint32_t v[SCAN_ITEMS];
	scan_load16(in, b0, n, vec != 0, v);
	uint32_t tsum = 0;
#pragma unroll
	for (int k = 0; k < (int)SCAN_ITEMS; ++k) tsum += v[k];
	uint32_t agg;
	const uint32_t texcl = scan_block(tsum, s_wsum, agg);
	if (threadIdx.x < 64) {
		const uint32_t pre = scan_lookback(st, 0, tl, agg);
		if (threadIdx.x == 0) s_prefix = pre;
	}
	__syncthreads();
	uint32_t run = s_prefix + texcl;
#pragma unroll
	for (int k = 0; k < (int)SCAN_ITEMS; ++k) { const uint32_t x = v[k]; v[k] = run; run += x; }
	scan_store16(out, b0, n, vec != 0, v);
}

size_t scan_temp_bytes(uint32_t n) {
	size_t a = 0, b = 0;
	(void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
	(void)hipcub::DeviceReduce::Sum(nullptr, b, (const float*)nullptr, (float*)nullptr, (int)n);
	return SCAN_STATE_BYTES + (a > b ? a : b);
}
// launches so far per state (the tag of the next one is this + 1, modulo the 30-bit tag range, never 0)
static std::mutex g_tag_mu;
static std::unordered_map<const void*, uint32_t> g_tags;
void scan_temp_reset(hipStream_t s, void* temp) {
	if (!temp) return;
	(void)hipMemsetAsync(temp, 0, SCAN_STATE_BYTES, s);
	std::lock_guard<std::mutex> g(g_tag_mu);
	g_tags[temp] = 0;
}
uint32_t scan_next_tag(void* temp) {
	std::lock_guard<std::mutex> g(g_tag_mu);
	uint32_t& c = g_tags[temp];
	c = c % 0x3fffffffu + 1u;
	return c;
}
uint32_t scan_failures(void* temp) {
	uint32_t f = 0;
	if (temp) (void)hipMemcpy(&f, (const char*)temp + offsetof(ScanState, fail), 4, hipMemcpyDeviceToHost);
	return f;
}
void scan_temp_release(void* temp) {
	std::lock_guard<std::mutex> g(g_tag_mu);
	g_tags.erase(temp);
}
void debug_scan_skip_first_tile(hipStream_t s, void* temp, const uint32_t* in, uint32_t* out, uint32_t n) {
	const uint32_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
	if (tiles < 2 || tiles > SCAN_MAX_TILES) throw std::runtime_error("debug_scan_skip_first_tile: needs 2 .. SCAN_MAX_TILES tiles");
	k_scan_lookback<<<tiles - 1, SCAN_THREADS, 0, s>>>(in, out, n, (ScanState*)temp, 0u, scan_next_tag(temp), 1u);
}
void launch_exclusive_scan(hipStream_t s, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n) {
	if (n == 0) return;
	const uint32_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
	if (tiles <= SCAN_MAX_TILES) {
		const uint32_t vec = ((((uintptr_t)in) | ((uintptr_t)out)) & 15u) == 0 ? 1u : 0u;
		dbg_lds_gate(s);
		k_scan_lookback<<<tiles, SCAN_THREADS, 0, s>>>(in, out, n, (ScanState*)temp, vec, scan_next_tag(temp), 0u);
		return;
	}
	size_t tb = temp_bytes - SCAN_STATE_BYTES;
	(void)hipcub::DeviceScan::ExclusiveSum((char*)temp + SCAN_STATE_BYTES, tb, in, out, (int)n, s);
}
void launch_sum_f32(hipStream_t s, void* temp, size_t temp_bytes, const float* in, float* out, uint32_t n) {
	dbg_lds_gate(s);
	size_t tb = temp_bytes - SCAN_STATE_BYTES;
	(void)hipcub::DeviceReduce::Sum((char*)temp + SCAN_STATE_BYTES, tb, in, out, (int)n, s);
}

} // namespace neus
