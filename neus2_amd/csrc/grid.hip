// Multiresolution hash-grid encoding for gfx950.
//
//   k_grid_encode  : forward (enc, optional dy/dx) — restates kernel_grid (grid.h:174-369)
//   k_scatter_hist / k_scatter_bin / k_scatter_accum : fused first-order (kernel_grid_backward,
//                    grid.h:371-500) and second-order (kernel_grid_backward_input_backward_grid,
//                    grid.h:880-1007) parameter gradients, binned by destination bucket and summed
//                    in int64 fixed point (deterministic; see the scatter section below) instead of
//                    the reference's two kernels x 8 corner fp16x2 atomics.
//
// k_grid_encode launch shape: blockIdx.y = level (level-major, like the reference): resident blocks work on
// one or two levels at a time, so the hashed level (2^19 x 4 B = 2 MiB) stays in the XCD's
// 4 MiB L2 while the blocks of that level run. Samples are grid-strided and the active count is
// read from device memory, so the host never syncs and the launch is graph-capturable.
#include "kernels.h"
#include "grid_common.h"
#include <algorithm>
#include <vector>

namespace neus {

__device__ __forceinline__ uint32_t load_n(const uint32_t* n_ptr, uint32_t n_fixed) { return n_ptr ? *n_ptr : n_fixed; }

// enc: [L][ld] packed half2 (features 2l, 2l+1); dydx: [L*6][ld] f32 (feature f, dim d at row 6l+3f+d)
// With a rollover (EncodeRollover: the training batch), records i >= n_in = min(compacted, n_elements) are the
// reference's fill_rollover_and_rescale copies (my_tcnn common_device.h:515-535): every level reads record i % n_in,
// and the level-0 blocks write the copies (coordinates, and dL/doutput scaled by n_in / n_elements) for the kernels
// after this one (k_rollover's work, without its launch).
__global__ void __launch_bounds__(256) k_grid_encode(
	const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
	const float* __restrict__ coords, uint32_t coord_stride,
	const GridLevels gl, uint32_t valid_level,
	const half_t* __restrict__ grid, uint32_t* __restrict__ enc, float* __restrict__ dydx, EncodeRollover ro) {
	const uint32_t n = load_n(n_ptr, n_fixed);
	const uint32_t l = blockIdx.y;
	const half_t* gp = grid + (size_t)gl.offset[l] * 2;
	const uint32_t n_in = ro.n_in_ptr ? min(*ro.n_in_ptr, ro.n_elements) : 0xffffffffu;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const uint32_t src = i < n_in ? i : i % n_in;  // (n_in > 0 whenever n > 0: n_train is 0 without records)
		if (l == 0 && i != src) {
			// rows i >= n_in are written, rows src < n_in read: the const input view and ro.coords never meet on an element
			for (uint32_t k = 0; k < coord_stride; ++k) ro.coords[(size_t)i * coord_stride + k] = coords[(size_t)src * coord_stride + k];
#pragma unroll
			for (int k = 0; k < OUT_W; ++k) {
				const float r = (float)ro.dL_dout[(size_t)src * OUT_W + k];
				ro.dL_dout[(size_t)i * OUT_W + k] = (half_t)(r * n_in / ro.n_elements);
			}
		}
		if (l > valid_level) {
			enc[(size_t)l * ld + i] = 0u;
			if (dydx) {
#pragma unroll
				for (int k = 0; k < 6; ++k) dydx[(size_t)(6 * l + k) * ld + i] = 0.0f;
			}
			continue;
		}
		const float* c = coords + (size_t)src * coord_stride;
		LevelSetup s = level_setup(gl, l, c[0], c[1], c[2]);
		h2 v[8];
		gather_corners(s, gp, v);
		const h2 out = interp_features(s, v);
		enc[(size_t)l * ld + i] = *(const uint32_t*)&out;
		if (dydx) {
			float gr[2][3];
			interp_dydx(s, v, gr);
#pragma unroll
			for (int f = 0; f < 2; ++f)
#pragma unroll
				for (int d = 0; d < 3; ++d) dydx[(size_t)(6 * l + 3 * f + d) * ld + i] = gr[f][d];
		}
	}
}

__device__ __forceinline__ void atomic_add_f32(float* p, float v) {
	__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Runs of consecutive lanes with the same grid entry (consecutive samples of one ray share
// coarse-level cells) are summed with a segmented shuffle scan; returns true on the lane that
// carries the run's sum (the last lane of the run). All 64 lanes must call this; `ok` masks lanes
// without a sample.
__device__ __forceinline__ bool wave_run_sum(uint32_t e, float& a0, float& a1, bool ok) {
	const uint32_t lane = threadIdx.x & 63;
	if (!ok) { e = 0xffffffffu; a0 = a1 = 0.f; }
	const uint32_t e_prev = dpp_u32<DPP_WAVE_SHR1>(~e, e);  // lane 0 keeps ~e: a head
	const uint64_t heads = __ballot(e_prev != e);
	if (heads == ~0ull) return ok;  // no run longer than one lane
	// run start: the highest head at or below this lane (lane 0 is always one)
	const uint32_t rs = 63u - (uint32_t)__clzll(heads & ((2ull << lane) - 1ull));
	// segmented sums: Kogge-Stone within rows of 16 lanes, then across rows (a run reaching back past its row's
	// start); a step no lane of the wave needs is skipped (fine levels: runs of 2-3 lanes)
	const uint32_t r0 = lane & ~15u;
#define NEUS_SEG_STEP(CTRL, MASK, COND)                                                                  \
	{                                                                                                    \
		const bool c = (COND);                                                                           \
		if (__ballot(c)) {                                                                               \
			const float t0 = dpp_f32<CTRL, MASK>(0.f, a0), t1 = dpp_f32<CTRL, MASK>(0.f, a1);             \
			a0 = c ? a0 + t0 : a0;                                                                       \
			a1 = c ? a1 + t1 : a1;                                                                       \
		}                                                                                                \
	}
	NEUS_SEG_STEP(DPP_ROW_SHR + 1, 0xf, lane - r0 >= 1u && lane - 1u >= rs)
	NEUS_SEG_STEP(DPP_ROW_SHR + 2, 0xf, lane - r0 >= 2u && lane - 2u >= rs)
	NEUS_SEG_STEP(DPP_ROW_SHR + 4, 0xf, lane - r0 >= 4u && lane - 4u >= rs)
	NEUS_SEG_STEP(DPP_ROW_SHR + 8, 0xf, lane - r0 >= 8u && lane - 8u >= rs)
	NEUS_SEG_STEP(DPP_BCAST15, 0xa, (r0 == 16u || r0 == 48u) && rs < r0)  // rows 1, 3 += the previous row's last lane
	NEUS_SEG_STEP(DPP_BCAST31, 0xc, lane >= 32u && rs < 32u)              // rows 2, 3 += lane 31
#undef NEUS_SEG_STEP
	const bool tail = lane == 63u || ((heads >> (lane + 1u)) & 1ull);
	return ok && tail;
}

// Slot of this lane's record in its bucket's per-block counter, with one LDS atomic per distinct
// bucket of the wave (lanes of one bucket get consecutive slots).
__device__ __forceinline__ uint32_t wave_bucket_slot(uint32_t* hist, uint32_t bkt, bool active) {
	const uint32_t lane = threadIdx.x & 63;
	uint64_t todo = __ballot(active);
	uint32_t res = 0;
	while (todo) {
		const int leader = __ffsll((unsigned long long)todo) - 1;
		const uint32_t lb = wave_lane_value(bkt, leader);
		const uint64_t m = __ballot(active && bkt == lb);
		uint32_t base = 0;
		if ((int)lane == leader) base = atomicAdd(&hist[lb], (uint32_t)__popcll(m));
		base = wave_lane_value(base, leader);
		if (active && bkt == lb) res = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
		todo &= ~m;
	}
	return res;
}

// ---------------------------------------------------------------- hash-grid gradient scatter
// Fused first-order (kernel_grid_backward, grid.h:371-500) and second-order
// (kernel_grid_backward_input_backward_grid, grid.h:880-1007) gradient of every corner of every level.
// The reference adds each corner with an fp16x2 global atomic at a random address; on MI355X float
// atomics run at the memory side and a wave-instruction whose 64 lanes hit 64 random addresses runs
// ~17x below the atomic byte rate, and float LDS atomics run at ~1/3 lane per clock per CU (integer
// LDS atomics ~13, scripts/micro/lds_atomics.hip). So the contributions are binned by destination and
// summed in integer fixed point:
//   k_scatter_hist    per-block histogram of contributions over 4096-entry buckets
//   exclusive scan    bucket-major [bucket][block] -> each block's slot range in each bucket
//   k_scatter_bin     recompute the contributions; per wave and level, stage them in LDS, reserve one
//                     contiguous run per bucket and write the records into their runs
//   records           (entry, fp16x2 contribution): the reference adds each corner's contribution as an
//                     fp16x2 atomic operand (grid.h:371-500), i.e. rounded to half; so is the record
//   k_scatter_accum   one workgroup per bucket: sum its records in LDS as int64 fixed point (2^-32,
//                     order-independent, so the gradient is bitwise deterministic) and store the
//                     bucket's fp32 gradient (plain stores: the workgroup owns its entries)
// Both bin passes evaluate the identical contribution sequence, so the slot counts always match.
//
// Record format (round 6). At the bench shape the loss scale is 128 / R = 2^-11 (testbed_nerf.cu:1765), so most corner
// contributions of the hashed levels are far below fp16's smallest normal (2^-14): an unscaled fp16 record quantises
// them to multiples of 2^-24, which put the fine levels' gradient 0.04-0.25 rel-L2 away from the exact sum. Each
// record now carries its own power-of-two scale: k in [0, 31] (5 bits above the 11-bit entry of rec_i) is the largest
// shift with max(|a0|, |a1|) * 2^k < 2^15, and rec_g = fp16(a * 2^k) - an 11-bit significand for every contribution
// above 2^-45. The accumulation adds round(v * 2^(SB_FIX_BITS - k)) in int64 (2^-38 fixed point: exact for the pair's
// larger value, |per-entry sum| < 2^25), still order-independent, so the gradient stays bitwise deterministic.
constexpr int SB_FIX_BITS = 38;
static_assert(SB_SHIFT <= 11, "the record's scale exponent needs the 5 bits of rec_i above the entry");
#ifndef NEUS_REC_SCALE
#define NEUS_REC_SCALE 1  // development: 0 keeps every record unscaled (k = 0: the round-5 records, for A/B timing)
#endif
__device__ __forceinline__ uint32_t rec_scale_exp(float a0, float a1) {
	if (!NEUS_REC_SCALE) return 0u;
	const uint32_t m = max(__float_as_uint(a0) & 0x7fffffffu, __float_as_uint(a1) & 0x7fffffffu);  // |larger| (finite: ordered as uint)
	const int ex = (int)(m >> 23) - 127;                                                         // floor(log2 |larger|); 0 -> -127
	return (uint32_t)min(max(14 - ex, 0), 31);
}
__device__ __forceinline__ uint32_t rec_value(float a0, float a1, uint32_t k) {
	const float s = __uint_as_float((127u + k) << 23);  // 2^k, exact
	return __builtin_bit_cast(uint32_t, (h2){(half_t)(a0 * s), (half_t)(a1 * s)});
}
__device__ __forceinline__ unsigned long long rec_fix(float v, uint32_t k) {  // fp16 record value of scale k -> int64 multiple of 2^-38
	const float s = __uint_as_float((127u + (uint32_t)SB_FIX_BITS - k) << 23);
	return (unsigned long long)__float2ll_rn(fminf(fmaxf(v, -65504.0f), 65504.0f) * s);
}
__device__ __forceinline__ float fix_to_float(unsigned long long v) { return (float)((double)(long long)v * (1.0 / 274877906944.0)); }  // 2^-38

// Contribution of corner idx of level l for one sample (first + second order, both features).
struct ScatterLevel { LevelSetup s; float dl0, dl1, g0, g1, vin[3]; uint32_t off; };
__device__ __forceinline__ void corner_contribution(const ScatterLevel& L, uint32_t idx, uint32_t& gidx, float& a0, float& a1) {
	// first order: w_corner; second order: sum_d (+/-) scale v_d prod_{other} w_other
	float wc = 1.f;
#pragma unroll
	for (int d = 0; d < 3; ++d) wc *= (idx & (1u << d)) ? L.s.pos[d] : 1.f - L.s.pos[d];
	float w2 = 0.f;
#pragma unroll
	for (int gd = 0; gd < 3; ++gd) {
		float t = L.vin[gd];
#pragma unroll
		for (int d = 0; d < 3; ++d) if (d != gd) t *= (idx & (1u << d)) ? L.s.pos[d] : 1.f - L.s.pos[d];
		w2 += (idx & (1u << gd)) ? t : -t;
	}
	a0 = L.dl0 * wc + L.g0 * w2;
	a1 = L.dl1 * wc + L.g1 * w2;
	const uint32_t gx = L.s.g[0] + (idx & 1), gy = L.s.g[1] + ((idx >> 1) & 1), gz = L.s.g[2] + ((idx >> 2) & 1);
	gidx = L.off + grid_index(L.s.hsize, L.s.res, gx, gy, gz);
}
__device__ __forceinline__ ScatterLevel scatter_level_ab(const GridLevels& gl, uint32_t l, float x, float y, float z, uint32_t a, uint32_t b2,
                                                         const float4 vv) {
	ScatterLevel L;
	L.s = level_setup(gl, l, x, y, z);
	const h2 d1 = *(const h2*)&a, g2 = *(const h2*)&b2;
	L.dl0 = (float)d1[0]; L.dl1 = (float)d1[1]; L.g0 = (float)g2[0]; L.g1 = (float)g2[1];
	L.vin[0] = L.s.scale * vv.x; L.vin[1] = L.s.scale * vv.y; L.vin[2] = L.s.scale * vv.z;
	L.off = gl.offset[l];
	return L;
}
__device__ __forceinline__ ScatterLevel scatter_level(const GridLevels& gl, uint32_t l, float x, float y, float z, uint32_t ic, uint32_t ld,
                                                      const uint32_t* __restrict__ dLdenc, const uint32_t* __restrict__ g, const float4 vv) {
	ScatterLevel L;
	L.s = level_setup(gl, l, x, y, z);
	const uint32_t a = dLdenc[(size_t)l * ld + ic], b2 = g[(size_t)l * ld + ic];
	const h2 d1 = *(const h2*)&a, g2 = *(const h2*)&b2;
	L.dl0 = (float)d1[0]; L.dl1 = (float)d1[1]; L.g0 = (float)g2[0]; L.g1 = (float)g2[1];
	L.vin[0] = L.s.scale * vv.x; L.vin[1] = L.s.scale * vv.y; L.vin[2] = L.s.scale * vv.z;
	L.off = gl.offset[l];
	return L;
}

// Slot order of the blocks inside a bucket: blocks dispatched to the same XCD (blockIdx mod 8) are made
// adjacent, so the short per-block runs that share a 128-B line of the record arrays are written through
// one L2 (consecutive blockIdx land on different XCDs). A bijection on [0, n); the sum per bucket and
// the bucket boundaries are unchanged, and k_scatter_accum is order-independent.
__device__ __forceinline__ uint32_t xcd_slot(uint32_t blk, uint32_t n) {
	const uint32_t q = n >> 3, r = n & 7, x = blk & 7, y = blk >> 3;
	return x * q + min(x, r) + y;
}

__global__ void __launch_bounds__(256) k_scatter_hist(const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
                                                      const float* __restrict__ coords, uint32_t coord_stride, const GridLevels gl,
                                                      uint32_t valid_level, const uint32_t* __restrict__ dLdenc, const uint32_t* __restrict__ g,
                                                      const float4* __restrict__ v4, ScatterWork w) {
	__shared__ uint32_t hist[SB_MAX_BUCKETS];
	for (uint32_t b = threadIdx.x; b < w.n_buckets; b += blockDim.x) hist[b] = 0;
	__syncthreads();
	const uint32_t n = load_n(n_ptr, n_fixed);
	const uint32_t blk = blockIdx.x, i = blk * blockDim.x + threadIdx.x;
	const bool ok = i < n;
	const uint32_t ic = ok ? i : 0;
	const float* c = coords + (size_t)ic * coord_stride;
	const float x = c[0], y = c[1], z = c[2];
	const float4 vv = v4[ic];
	for (uint32_t l = 0; l < gl.n_levels && l <= valid_level; ++l) {
		const ScatterLevel L = scatter_level(gl, l, x, y, z, ic, ld, dLdenc, g, vv);
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			uint32_t gidx; float a0, a1;
			corner_contribution(L, idx, gidx, a0, a1);
			const bool emit = wave_run_sum(gidx, a0, a1, ok);
			const uint32_t bkt = gidx >> SB_SHIFT;
			// levels spanning a few buckets: one LDS add per (wave, bucket) instead of up to 64 on one counter
			if (L.s.hsize <= 4 * SB_SIZE) (void)wave_bucket_slot(hist, bkt, emit);
			else if (emit) atomicAdd(&hist[bkt], 1u);
		}
	}
	__syncthreads();
	for (uint32_t b = threadIdx.x; b < w.n_active; b += blockDim.x) w.counts[(size_t)b * w.n_blocks + xcd_slot(blk, w.n_blocks)] = hist[b];
	if (blk == 0 && threadIdx.x == 0) w.counts[(size_t)w.n_active * w.n_blocks] = 0u;  // the scan's extra element: offs[end] = total
}

// Per wave and level: each lane keeps its 8 records in registers while their buckets are counted (as
// k_scatter_hist); each non-empty bucket then reserves its run with one LDS atomic on the block's cursor
// for that bucket, the wave scans its bucket counts, and the records are counting-sorted by bucket into a
// per-wave LDS stage. The stage is written out in order, so consecutive lanes store consecutive slots of
// one bucket's run (coalesced segments instead of one scattered 2-B + 4-B store pair per lane). The
// block's cursors cover only the current level's buckets (one barrier group per level).
constexpr int SB_WSTAGE = 64 * 8;
__global__ void __launch_bounds__(256) k_scatter_bin(const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
                                                     const float* __restrict__ coords, uint32_t coord_stride, const GridLevels gl,
                                                     uint32_t valid_level, const uint32_t* __restrict__ dLdenc, const uint32_t* __restrict__ g,
                                                     const float4* __restrict__ v4, ScatterWork w) {
	__shared__ uint32_t cursor[SB_LEVEL_BUCKETS];                // next global slot of this block in the level's buckets
	__shared__ uint32_t carry_b, carry_v;                        // a bucket shared with the previous level
	__shared__ uint32_t wcnt[4][SB_LEVEL_BUCKETS], wbase[4][SB_LEVEL_BUCKETS], wloff[4][SB_LEVEL_BUCKETS];
	__shared__ uint32_t st_g[4][SB_WSTAGE];                       // sorted stage: fp16x2 contribution
	__shared__ uint32_t st_e[4][SB_WSTAGE];                       // sorted stage: entry in bucket | level-local bucket << 16
	const uint32_t blk = blockIdx.x, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
	const uint32_t n = load_n(n_ptr, n_fixed);
	const uint32_t i = blk * blockDim.x + threadIdx.x;
	const bool ok = i < n;
	const uint32_t ic = ok ? i : 0;
	const float* c = coords + (size_t)ic * coord_stride;
	const float x = c[0], y = c[1], z = c[2];
	const float4 vv = v4[ic];
	uint32_t* cnt = wcnt[wv];
	uint32_t* bas = wbase[wv];
	uint32_t* loff = wloff[wv];
	uint32_t* sg = st_g[wv];
	uint32_t* se = st_e[wv];
	if (threadIdx.x == 0) { carry_b = ~0u; carry_v = 0; }
	for (uint32_t l = 0; l < gl.n_levels && l <= valid_level; ++l) {
		const uint32_t b_first = gl.offset[l] >> SB_SHIFT, nlb = ((gl.offset[l + 1] - 1) >> SB_SHIFT) - b_first + 1;
		__syncthreads();  // previous level's cursors are final (carry_b / carry_v written), its stage drained
		for (uint32_t k = threadIdx.x; k < nlb; k += blockDim.x) {
			const uint32_t b = b_first + k;
			cursor[k] = b == carry_b ? carry_v : w.offs[(size_t)b * w.n_blocks + xcd_slot(blk, w.n_blocks)];
		}
		for (uint32_t k = lane; k < nlb; k += 64) cnt[k] = 0;
		__builtin_amdgcn_wave_barrier();
		const ScatterLevel L = scatter_level(gl, l, x, y, z, ic, ld, dLdenc, g, vv);
		uint32_t re[8], rg[8];
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			uint32_t gidx; float a0, a1;
			corner_contribution(L, idx, gidx, a0, a1);
			const bool emit = wave_run_sum(gidx, a0, a1, ok);
			if (emit) atomicAdd(&cnt[(gidx >> SB_SHIFT) - b_first], 1u);
			const uint32_t kx = rec_scale_exp(a0, a1);
			re[idx] = emit ? gidx | kx << 24 : ~0u;  // entries < 2^24 (SB_MAX_BUCKETS)
			rg[idx] = rec_value(a0, a1, kx);
		}
		__syncthreads();  // cursors loaded, bucket counts complete
		// per bucket: the run reserved on the block cursor and the wave-local offset (exclusive scan of the counts)
		uint32_t total = 0;
		for (uint32_t k0 = 0; k0 < nlb; k0 += 64) {
			const uint32_t k = k0 + lane;
			const uint32_t v = k < nlb ? cnt[k] : 0u;
			const uint32_t incl = wave_incl_sum(v);
			if (k < nlb) { bas[k] = v ? atomicAdd(&cursor[k], v) : 0u; loff[k] = total + incl - v; cnt[k] = 0; }
			total += wave_lane_value(incl, 63);
		}
		__syncthreads();  // offsets visible, counters cleared
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			const uint32_t ek = re[idx];
			if (ek != ~0u) {
				const uint32_t e = ek & 0xffffffu;
				const uint32_t lb = (e >> SB_SHIFT) - b_first;
				const uint32_t pos = loff[lb] + atomicAdd(&cnt[lb], 1u);
				se[pos] = (e & (SB_SIZE - 1)) | (ek >> 24) << SB_SHIFT | (lb << 16);
				sg[pos] = rg[idx];
			}
		}
		__syncthreads();  // stage complete
		for (uint32_t r = lane; r < total; r += 64) {
			const uint32_t u = se[r], lb = u >> 16;
			const uint32_t gp = bas[lb] + (r - loff[lb]);
			w.rec_i[gp] = (uint16_t)(u & 0xffffu);
			w.rec_g[gp] = __builtin_bit_cast(h2, sg[r]);
		}
		__syncthreads();  // all reservations of this level done
		if (threadIdx.x == 0) { carry_b = b_first + nlb - 1; carry_v = cursor[nlb - 1]; }
	}
}

// ---------------------------------------------------------------- wide-block binning (default)
// The same records, slots and buckets as k_scatter_hist / k_scatter_bin, with one BS-thread workgroup per BS = 512
// (default) or 1024 samples instead of 256: a (block, bucket) run of a hashed level holds ~32-64 records instead of ~16, so the
// sorted stage leaves the workgroup as whole 128-B lines (the 256-sample runs were written in 32-64 B pieces), the
// histogram has 2-4x fewer (bucket, block) counters to scan, and the per-level barriers are paid once per BS samples.
// The wave groups (64 consecutive samples) and their run sums are unchanged, so the records - and the int64 sums -
// are bitwise those of the 256-sample path.
template <int BS>
__global__ void __launch_bounds__(BS) k_scatter_hist_w(const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
                                                         const float* __restrict__ coords, uint32_t coord_stride, const GridLevels gl,
                                                         uint32_t valid_level, const uint32_t* __restrict__ dLdenc, const uint32_t* __restrict__ g,
                                                         const float4* __restrict__ v4, ScatterWork w) {
	__shared__ uint32_t hist[SB_MAX_BUCKETS];
	for (uint32_t b = threadIdx.x; b < w.n_active; b += blockDim.x) hist[b] = 0;
	__syncthreads();
	const uint32_t n = load_n(n_ptr, n_fixed);
	const uint32_t blk = blockIdx.x, i = blk * blockDim.x + threadIdx.x;
	const bool ok = i < n;
	const uint32_t ic = ok ? i : 0;
	const float* c = coords + (size_t)ic * coord_stride;
	const float x = c[0], y = c[1], z = c[2];
	const float4 vv = v4[ic];
	for (uint32_t l = 0; l < gl.n_levels && l <= valid_level; ++l) {
		const ScatterLevel L = scatter_level(gl, l, x, y, z, ic, ld, dLdenc, g, vv);
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			uint32_t gidx; float a0, a1;
			corner_contribution(L, idx, gidx, a0, a1);
			const bool emit = wave_run_sum(gidx, a0, a1, ok);
			const uint32_t bkt = gidx >> SB_SHIFT;
			if (L.s.hsize <= 4 * SB_SIZE) (void)wave_bucket_slot(hist, bkt, emit);
			else if (emit) atomicAdd(&hist[bkt], 1u);
		}
	}
	__syncthreads();
	for (uint32_t b = threadIdx.x; b < w.n_active; b += blockDim.x) w.counts[(size_t)b * w.n_chunks + xcd_slot(blk, w.n_chunks)] = hist[b];
	if (blk == 0 && threadIdx.x == 0) w.counts[(size_t)w.n_active * w.n_chunks] = 0u;  // the scan's extra element: offs[end] = total
}

template <int BS>
__global__ void __launch_bounds__(BS) k_scatter_bin_w(const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
                                                        const float* __restrict__ coords, uint32_t coord_stride, const GridLevels gl,
                                                        uint32_t valid_level, const uint32_t* __restrict__ dLdenc, const uint32_t* __restrict__ g,
                                                        const float4* __restrict__ v4, ScatterWork w) {
	__shared__ uint32_t cnt[SB_LEVEL_BUCKETS], cursor[SB_LEVEL_BUCKETS], base[SB_LEVEL_BUCKETS + 1];
	__shared__ uint32_t carry_b, carry_v;  // a bucket shared with the previous level: the block's next slot in it
	__shared__ uint16_t st_i[BS * 8];
	__shared__ uint32_t st_g[BS * 8];
	__shared__ uint16_t st_b[BS * 8];      // level-local bucket of each staged record (up to 257 per level at 2048-entry buckets)
	const uint32_t blk = blockIdx.x, lane = threadIdx.x & 63;
	const uint32_t n = load_n(n_ptr, n_fixed);
	const uint32_t i = blk * blockDim.x + threadIdx.x;
	const bool ok = i < n;
	const uint32_t ic = ok ? i : 0;
	const float* c = coords + (size_t)ic * coord_stride;
	const float x = c[0], y = c[1], z = c[2];
	const float4 vv = v4[ic];
	const uint32_t slot_blk = xcd_slot(blk, w.n_chunks);
	if (threadIdx.x == 0) { carry_b = ~0u; carry_v = 0; }
	for (uint32_t l = 0; l < gl.n_levels && l <= valid_level; ++l) {
		const uint32_t b_first = gl.offset[l] >> SB_SHIFT, nlb = ((gl.offset[l + 1] - 1) >> SB_SHIFT) - b_first + 1;
		const bool few = gl.offset[l + 1] - gl.offset[l] <= 4 * SB_SIZE;
		__syncthreads();  // the previous level's stage is written out, carry_b / carry_v final
		for (uint32_t k = threadIdx.x; k < nlb; k += blockDim.x) {
			const uint32_t b = b_first + k;
			cnt[k] = 0;
			cursor[k] = b == carry_b ? carry_v : w.offs[(size_t)b * w.n_chunks + slot_blk];
		}
		__syncthreads();
		const ScatterLevel L = scatter_level(gl, l, x, y, z, ic, ld, dLdenc, g, vv);
		uint32_t re[8], rs[8], rg[8];
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			uint32_t gidx; float a0, a1;
			corner_contribution(L, idx, gidx, a0, a1);
			const bool emit = wave_run_sum(gidx, a0, a1, ok);
			const uint32_t lb = (gidx >> SB_SHIFT) - b_first;
			uint32_t sl = 0;
			if (few) sl = wave_bucket_slot(cnt, lb, emit);
			else if (emit) sl = atomicAdd(&cnt[lb], 1u);
			const uint32_t kx = rec_scale_exp(a0, a1);
			re[idx] = emit ? gidx | kx << 24 : ~0u;  // entries < 2^24 (SB_MAX_BUCKETS)
			rs[idx] = sl;
			rg[idx] = rec_value(a0, a1, kx);
		}
		__syncthreads();  // bucket counts complete
		if (threadIdx.x < 64) {  // exclusive scan of the counts (one wave)
			uint32_t total = 0;
			for (uint32_t k0 = 0; k0 < nlb; k0 += 64) {
				const uint32_t k = k0 + lane;
				const uint32_t v = k < nlb ? cnt[k] : 0u;
				const uint32_t incl = wave_incl_sum(v);
				if (k < nlb) base[k] = total + incl - v;
				total += wave_lane_value(incl, 63);
			}
			if (lane == 0) base[nlb] = total;
		}
		__syncthreads();
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			const uint32_t ek = re[idx];
			if (ek != ~0u) {
				const uint32_t e = ek & 0xffffffu;
				const uint32_t lb = (e >> SB_SHIFT) - b_first;
				const uint32_t pos = base[lb] + rs[idx];
				st_i[pos] = (uint16_t)((e & (SB_SIZE - 1)) | (ek >> 24) << SB_SHIFT);
				st_g[pos] = rg[idx];
				st_b[pos] = (uint16_t)lb;
			}
		}
		__syncthreads();  // stage complete: consecutive threads store consecutive slots of a bucket's run
		const uint32_t total = base[nlb];
		for (uint32_t r = threadIdx.x; r < total; r += blockDim.x) {
			const uint32_t lb = st_b[r];
			const uint32_t gp = cursor[lb] + (r - base[lb]);
			w.rec_i[gp] = st_i[r];
			w.rec_g[gp] = __builtin_bit_cast(h2, st_g[r]);
		}
		if (threadIdx.x == 0) { carry_b = b_first + nlb - 1; carry_v = cursor[nlb - 1] + cnt[nlb - 1]; }
	}
}

// ---------------------------------------------------------------- per-block record regions (default)
// The same records as the binned paths, without the histogram pass and the device-wide slot scan: each BS-sample
// workgroup counting-sorts its records of a level by level-local bucket (4096 entries of that level) in LDS and writes
// them out as ONE contiguous region [level][block] (BS x 8 slots), whole 128-B lines, plus the bucket start offsets of
// the region (rtab [level][block][bucket], u16). The accumulation of bucket (l, k) then reads the k-th segment of every
// block's level-l region (~32 records each on a hashed level): the region reads are the only extra cost, against the
// histogram pass, the ~1M-entry scan and the runs of 16-64 records the binned path writes to scattered slots. Records,
// their int64 sums and so the gradient are bitwise the binned paths' (the sum per entry is order-independent).
constexpr uint32_t RT_STRIDE = SB_LEVEL_BUCKETS + 1;
template <int BS>
__global__ void __launch_bounds__(BS) k_scatter_bin_r(const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
                                                        const float* __restrict__ coords, uint32_t coord_stride, const GridLevels gl,
                                                        uint32_t valid_level, const uint32_t* __restrict__ dLdenc, const uint32_t* __restrict__ g,
                                                        const float4* __restrict__ v4, ScatterWork w) {
	__shared__ uint32_t cnt[SB_LEVEL_BUCKETS], base[SB_LEVEL_BUCKETS + 1];
	__shared__ uint16_t st_i[BS * 8];
	__shared__ uint32_t st_g[BS * 8];
	const uint32_t blk = blockIdx.x, lane = threadIdx.x & 63;
	const uint32_t n = load_n(n_ptr, n_fixed);
	const uint32_t i = blk * blockDim.x + threadIdx.x;
	const bool ok = i < n;
	const uint32_t ic = ok ? i : 0;
	const float* c = coords + (size_t)ic * coord_stride;
	const float x = c[0], y = c[1], z = c[2];
	const float4 vv = v4[ic];
	const uint32_t n_lv = min(gl.n_levels, valid_level + 1);
	// the level's two per-sample operands, loaded one level ahead (the level loop's barriers would otherwise expose
	// their latency once per level); workgroup (chunk, y) bins levels y, y + gridDim.y, ... of its chunk
	const uint32_t lstep = gridDim.y;
	uint32_t a_cur = dLdenc[(size_t)blockIdx.y * ld + ic], g_cur = g[(size_t)blockIdx.y * ld + ic];
	for (uint32_t l = blockIdx.y; l < n_lv; l += lstep) {
		const uint32_t ln = min(l + lstep, n_lv - 1);
		const uint32_t a_next = dLdenc[(size_t)ln * ld + ic], g_next = g[(size_t)ln * ld + ic];
		const uint32_t off = gl.offset[l], size = gl.offset[l + 1] - off;
		const uint32_t nlb = (size + SB_SIZE - 1) >> SB_SHIFT;
		const bool few = size <= 4 * SB_SIZE;
		for (uint32_t k = threadIdx.x; k < nlb; k += blockDim.x) cnt[k] = 0;
		__syncthreads();
		const ScatterLevel L = scatter_level_ab(gl, l, x, y, z, a_cur, g_cur, vv);
		a_cur = a_next; g_cur = g_next;
		uint32_t re[8], rs[8], rg[8];
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			uint32_t gidx; float a0, a1;
			corner_contribution(L, idx, gidx, a0, a1);
			const bool emit = wave_run_sum(gidx, a0, a1, ok);
			const uint32_t e = gidx - off, lb = e >> SB_SHIFT;
			uint32_t sl = 0;
			if (few) sl = wave_bucket_slot(cnt, lb, emit);
			else if (emit) sl = atomicAdd(&cnt[lb], 1u);
			const uint32_t kx = rec_scale_exp(a0, a1);
			re[idx] = emit ? e | kx << 24 : ~0u;  // level-local entries < 2^19
			rs[idx] = sl;
			rg[idx] = rec_value(a0, a1, kx);
		}
		__syncthreads();  // bucket counts complete
		if (threadIdx.x < 64) {  // exclusive scan of the counts (one wave)
			uint32_t total = 0;
			for (uint32_t k0 = 0; k0 < nlb; k0 += 64) {
				const uint32_t k = k0 + lane;
				const uint32_t v = k < nlb ? cnt[k] : 0u;
				const uint32_t incl = wave_incl_sum(v);
				if (k < nlb) base[k] = total + incl - v;
				total += wave_lane_value(incl, 63);
			}
			if (lane == 0) base[nlb] = total;
		}
		__syncthreads();
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			const uint32_t ek = re[idx];
			if (ek != ~0u) {
				const uint32_t e = ek & 0xffffffu;
				const uint32_t pos = base[e >> SB_SHIFT] + rs[idx];
				st_i[pos] = (uint16_t)((e & (SB_SIZE - 1)) | (ek >> 24) << SB_SHIFT);
				st_g[pos] = rg[idx];
			}
		}
		__syncthreads();  // stage complete: the region is written out contiguously
		const size_t region = ((size_t)l * w.n_chunks + blk) * (BS * 8);
		const uint32_t total = base[nlb];
		for (uint32_t r = threadIdx.x; r < total; r += blockDim.x) {
			w.rec_i[region + r] = st_i[r];
			w.rec_g[region + r] = __builtin_bit_cast(h2, st_g[r]);
		}
		uint16_t* tab = w.rtab + ((size_t)l * w.n_chunks + blk) * RT_STRIDE;
		for (uint32_t k = threadIdx.x; k <= nlb; k += blockDim.x) tab[k] = (uint16_t)base[k];
		__syncthreads();  // LDS reused by the next level
	}
}

// One workgroup per level-local bucket (l, k), or `parts` workgroups over slices of the blocks for the heavy buckets
// of the small dense levels (int64 sums meeting in a split slot, as k_scatter_accum). A wave takes 64 of the slice's
// blocks at a time (blocks wv, wv + 4, ... of the slice: every wave gets a share of a short slice): their segment
// lengths, a wave scan, and the concatenated segments read lane-contiguously, SC_U batches of 64 records in flight
// (the owner of each record by binary search over the 64 segment starts in LDS).
constexpr int SC_U = 8;
#ifndef NEUS_SC_WAVES
#define NEUS_SC_WAVES 4
#endif
constexpr int SC_WAVES = NEUS_SC_WAVES;  // (8 waves per workgroup measured slower: 93 -> 103 us at the bench state)
__global__ void __launch_bounds__(64 * SC_WAVES) k_scatter_accum_r(ScatterWork w, const GridLevels gl, float* __restrict__ grads, uint32_t bs8,
                                                                   uint32_t job0, uint32_t n_jobs, uint32_t xg) {
	__shared__ unsigned long long acc[2 * SB_SIZE];
	__shared__ uint32_t s_pre[SC_WAVES][65], s_src[SC_WAVES][64];
	__shared__ uint32_t s_last;
	// Workgroup -> job: groups of xg consecutive jobs (adjacent buckets of a level, whose record segments share 128-B
	// lines of every block's region) go to one XCD (workgroups are dispatched to the XCDs round-robin: XCD = blockIdx
	// mod 8), so a shared line is fetched into one L2 instead of two; xg = 1 is list order. (An XCD-contiguous mapping,
	// each XCD an eighth of the list, measured 93 -> 169 us at the bench state.)
	const uint32_t bx = blockIdx.x & 7u, bk = blockIdx.x >> 3;
	const uint32_t jl = ((bk / xg) * 8u + bx) * xg + bk % xg;
	if (jl >= n_jobs) return;
	const uint4 job = w.jobs2[job0 + jl];
	const uint32_t l = job.x, kb = job.y, part = job.z & 0xffffu, parts = job.z >> 16, slot = job.w;
	const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
	for (uint32_t k = threadIdx.x; k < 2 * SB_SIZE; k += blockDim.x) acc[k] = 0ull;
	__syncthreads();
	const uint32_t nb = w.n_chunks;
	const uint32_t b0 = (uint32_t)((uint64_t)nb * part / parts), b1 = (uint32_t)((uint64_t)nb * (part + 1) / parts);
	uint32_t* pre = s_pre[wv];
	uint32_t* src = s_src[wv];
	for (uint32_t it = 0; b0 + wv + SC_WAVES * 64 * it < b1; ++it) {
		const uint32_t b = b0 + wv + SC_WAVES * (64 * it + lane);
		uint32_t s0 = 0, len = 0;
		if (b < b1) {
			const uint16_t* tab = w.rtab + ((size_t)l * nb + b) * RT_STRIDE;
			s0 = tab[kb];
			len = (uint32_t)tab[kb + 1] - s0;
		}
		const uint32_t incl = wave_incl_sum(len);
		const uint32_t total = wave_lane_value(incl, 63);
		__builtin_amdgcn_wave_barrier();
		pre[lane] = incl - len;
		src[lane] = (uint32_t)(((size_t)l * nb + (b < b1 ? b : 0u)) * bs8) + s0;  // u32: < 2^32 records
		__builtin_amdgcn_wave_barrier();
		for (uint32_t r0 = 0; r0 < total; r0 += 64 * SC_U) {
			uint32_t q[SC_U];
#pragma unroll
			for (int u = 0; u < SC_U; ++u) {
				const uint32_t r = min(r0 + 64u * u + lane, total - 1u);
				uint32_t o = 0;
#pragma unroll
				for (uint32_t step = 32; step > 0; step >>= 1) if (pre[o + step] <= r) o += step;
				q[u] = src[o] + (r - pre[o]);
			}
			uint32_t ev[SC_U], gv[SC_U];
#pragma unroll
			for (int u = 0; u < SC_U; ++u) { ev[u] = w.rec_i[q[u]]; gv[u] = __builtin_bit_cast(uint32_t, w.rec_g[q[u]]); }
#pragma unroll
			for (int u = 0; u < SC_U; ++u) {
				if (r0 + 64u * u + lane < total) {
					const h2 g2 = __builtin_bit_cast(h2, gv[u]);
					const uint32_t e = ev[u] & (SB_SIZE - 1), kx = ev[u] >> SB_SHIFT;
					atomicAdd(&acc[e], rec_fix((float)g2[0], kx));
					atomicAdd(&acc[SB_SIZE + e], rec_fix((float)g2[1], kx));
				}
			}
		}
		__builtin_amdgcn_wave_barrier();
	}
	__syncthreads();
	const uint32_t off = gl.offset[l], size = gl.offset[l + 1] - off;
	const uint32_t e0 = off + kb * SB_SIZE, ne = min(SB_SIZE, size - kb * SB_SIZE);
	if (parts == 1) {
		for (uint32_t k = threadIdx.x; k < 2 * ne; k += blockDim.x)
			grads[2 * (size_t)e0 + k] = fix_to_float(acc[(k & 1) * SB_SIZE + (k >> 1)]);
		return;
	}
	unsigned long long* H = w.split + (size_t)slot * 2 * SB_SIZE;
	for (uint32_t k = threadIdx.x; k < 2 * SB_SIZE; k += blockDim.x) {
		const unsigned long long v = acc[k];
		if (v) atomicAdd(&H[k], v);
	}
	__threadfence();
	__syncthreads();
	if (threadIdx.x == 0) s_last = atomicAdd(&w.split_done[slot], 1u) == parts - 1 ? 1u : 0u;
	__syncthreads();
	if (!s_last) return;
	__threadfence();
	for (uint32_t k = threadIdx.x; k < 2 * ne; k += blockDim.x) {
		const unsigned long long v = atomicExch(&H[(k & 1) * SB_SIZE + (k >> 1)], 0ull);
		grads[2 * (size_t)e0 + k] = fix_to_float(v);
	}
	if (threadIdx.x == 0) atomicExch(&w.split_done[slot], 0u);
}

// One workgroup per bucket, or `parts` workgroups for a bucket of a small dense level (one 4096-entry bucket can hold a
// whole level's records): each part sums an equal slice of the bucket's records in LDS and adds its nonzero int64 sums
// to the bucket's split slot with 64-bit integer atomics (exact, so the total is order-independent and bitwise the
// one-workgroup sum); the last part to finish reads the slot back (exchanging it with zero for the next use) and
// stores the fp32 gradient.
__global__ void __launch_bounds__(256) k_scatter_accum(ScatterWork w, float* __restrict__ grads, uint32_t n_entries) {
	__shared__ unsigned long long acc[2 * SB_SIZE];  // feature planes, int64 fixed point (2^-38)
	__shared__ uint32_t s_last;
	const uint4 job = w.jobs[blockIdx.x];
	const uint32_t b = job.x, part = job.y, parts = job.z, slot = job.w;
	for (uint32_t k = threadIdx.x; k < 2 * SB_SIZE; k += blockDim.x) acc[k] = 0ull;
	__syncthreads();
	uint32_t c0 = w.offs[(size_t)b * w.n_blocks], c1 = w.offs[(size_t)(b + 1) * w.n_blocks];
	if (parts > 1) {
		const uint32_t len = c1 - c0;
		c1 = c0 + (uint32_t)((uint64_t)len * (part + 1) / parts);
		c0 = c0 + (uint32_t)((uint64_t)len * part / parts);
	}
	auto add = [&](uint32_t ek, float v0, float v1) {  // ek: entry | scale exponent << SB_SHIFT
		const uint32_t e = ek & (SB_SIZE - 1), kx = ek >> SB_SHIFT;
		atomicAdd(&acc[e], rec_fix(v0, kx));
		atomicAdd(&acc[SB_SIZE + e], rec_fix(v1, kx));
	};
	// unaligned head and tail one per thread, the 8-aligned middle as groups of 8 per thread
	const uint32_t a0 = min(c1, (c0 + 7u) & ~7u), a1 = max(a0, c1 & ~7u);
	auto one = [&](uint32_t r) { const h2 gv = w.rec_g[r]; add(w.rec_i[r], (float)gv[0], (float)gv[1]); };
	for (uint32_t r = c0 + threadIdx.x; r < a0; r += blockDim.x) one(r);
	for (uint32_t r = a1 + threadIdx.x; r < c1; r += blockDim.x) one(r);
	for (uint32_t gq = a0 / 8 + threadIdx.x; gq < a1 / 8; gq += blockDim.x) {
		const uint4 ei = *(const uint4*)(w.rec_i + 8 * (size_t)gq);
		const uint4* gp = (const uint4*)(w.rec_g + 8 * (size_t)gq);
		const uint4 u0 = gp[0], u1 = gp[1];
		const uint32_t ew[4] = {ei.x, ei.y, ei.z, ei.w}, gw[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
		for (int k = 0; k < 8; ++k) {
			const h2 gv = __builtin_bit_cast(h2, gw[k]);
			add((ew[k >> 1] >> (16 * (k & 1))) & 0xffffu, (float)gv[0], (float)gv[1]);
		}
	}
	__syncthreads();
	// the bucket owns entries [b * SB_SIZE, +SB_SIZE): plain stores of the interleaved fp32 pairs
	const uint32_t e0 = b << SB_SHIFT;
	const uint32_t ne = min(SB_SIZE, n_entries - e0);
	if (parts == 1) {
		for (uint32_t k = threadIdx.x; k < 2 * ne; k += blockDim.x)
			grads[2 * (size_t)e0 + k] = fix_to_float(acc[(k & 1) * SB_SIZE + (k >> 1)]);
		return;
	}
	unsigned long long* H = w.split + (size_t)slot * 2 * SB_SIZE;
	for (uint32_t k = threadIdx.x; k < 2 * SB_SIZE; k += blockDim.x) {
		const unsigned long long v = acc[k];
		if (v) atomicAdd(&H[k], v);
	}
	__threadfence();
	__syncthreads();
	if (threadIdx.x == 0) s_last = atomicAdd(&w.split_done[slot], 1u) == parts - 1 ? 1u : 0u;
	__syncthreads();
	if (!s_last) return;
	__threadfence();
	for (uint32_t k = threadIdx.x; k < 2 * ne; k += blockDim.x) {
		const unsigned long long v = atomicExch(&H[(k & 1) * SB_SIZE + (k >> 1)], 0ull);
		grads[2 * (size_t)e0 + k] = fix_to_float(v);
	}
	if (threadIdx.x == 0) atomicExch(&w.split_done[slot], 0u);
}

// ---------------------------------------------------------------- operator-module helpers (neus_module_*)
// dL/dx of the encoding (GridEncoding::backward's dL_dinput, kernel_grid_backward_input, grid.h:503-565):
// dL_dx[i][d] = sum over levels / features of dL_dy[f][i] * dy_dx[f][d][i]; dL_dy is [L][ld] half2.
__global__ void __launch_bounds__(256) k_enc_input_grad(uint32_t n, uint32_t ld, uint32_t L, const uint32_t* __restrict__ dLdy,
                                                        const float* __restrict__ dydx, float* __restrict__ dLdx, uint32_t stride) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	float acc[3] = {0.f, 0.f, 0.f};
	for (uint32_t l = 0; l < L; ++l) {
		const uint32_t a = dLdy[(size_t)l * ld + i];
		const h2 g = *(const h2*)&a;
#pragma unroll
		for (int f = 0; f < 2; ++f)
#pragma unroll
			for (int d = 0; d < 3; ++d) acc[d] += (float)g[f] * dydx[(size_t)(6 * l + 3 * f + d) * ld + i];
	}
#pragma unroll
	for (int d = 0; d < 3; ++d) dLdx[(size_t)i * stride + d] = acc[d];
}
// dL/d(dL_dy) of backward_backward_input (kernel_grid_backward_input_backward_dLdoutput, grid.h:1092-1120):
// out[f][i] = sum_d dL_ddLdx[i][d] * dy_dx[f][d][i], written as [L][ld] half2; and dL_ddLdx packed as float4
// for the fused scatter's second-order term.
__global__ void __launch_bounds__(256) k_enc_ddLdoutput(uint32_t n, uint32_t ld, uint32_t L, const float* __restrict__ ddx,
                                                        const float* __restrict__ dydx, uint32_t* __restrict__ out, float4* __restrict__ v4) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const float v[3] = {ddx[3 * (size_t)i], ddx[3 * (size_t)i + 1], ddx[3 * (size_t)i + 2]};
	v4[i] = make_float4(v[0], v[1], v[2], 0.f);
	if (!out) return;
	for (uint32_t l = 0; l < L; ++l) {
		h2 o;
#pragma unroll
		for (int f = 0; f < 2; ++f) {
			float a = 0.f;
#pragma unroll
			for (int d = 0; d < 3; ++d) a += v[d] * dydx[(size_t)(6 * l + 3 * f + d) * ld + i];
			o[f] = (half_t)a;
		}
		out[(size_t)l * ld + i] = *(const uint32_t*)&o;
	}
}

// Encoding output layouts of the operator module (tcnn GPUMatrix layouts): paired [L][n] half2 (this build's kernels)
// <-> AoS [n][2L] (column-major: the cpp::Module view, cpp_api.cu:58-70) or SoA [2L][n] (GridEncoding's preferred
// layout, grid.h:2357-2359). One thread per (sample, level).
__global__ void __launch_bounds__(256) k_enc_relayout(uint32_t n, uint32_t L, const uint32_t* __restrict__ paired, half_t* __restrict__ dst,
                                                      uint32_t layout, uint32_t to_paired, uint32_t* __restrict__ paired_out, const half_t* __restrict__ src) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n * L) return;
	const uint32_t l = t / n, i = t % n;
	const size_t a0 = layout == ENC_LAYOUT_AOS ? (size_t)i * 2 * L + 2 * l : (size_t)(2 * l) * n + i;
	const size_t a1 = layout == ENC_LAYOUT_AOS ? a0 + 1 : a0 + n;
	if (to_paired) {
		h2 v = {src[a0], src[a1]};
		paired_out[(size_t)l * n + i] = *(const uint32_t*)&v;
	} else {
		const uint32_t u = paired[(size_t)l * n + i];
		const h2 v = *(const h2*)&u;
		dst[a0] = v[0];
		dst[a1] = v[1];
	}
}
// paired [L][n] half2 <-> sample rows [n][ld] fp16 with the features in columns [0, 2L) and the columns [2L, ld) zero: the
// FullyFusedMLP input of a HashGrid-encoded network (GridEncoding pads its output with zeros, grid.h:1540-1550). One
// thread per (sample, column pair).
__global__ void __launch_bounds__(256) k_enc_rows(uint32_t n, uint32_t L, uint32_t ld, const uint32_t* __restrict__ paired, half_t* __restrict__ rows,
                                                  uint32_t to_paired, uint32_t* __restrict__ paired_out, const half_t* __restrict__ src) {
	const uint32_t half_ld = ld / 2;
	const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= (uint64_t)n * half_ld) return;
	const uint32_t i = (uint32_t)(t / half_ld), c = (uint32_t)(t % half_ld);
	if (to_paired) {
		if (c < L) paired_out[(size_t)c * n + i] = *(const uint32_t*)(src + (size_t)i * ld + 2 * c);
	} else {
		const uint32_t u = c < L ? paired[(size_t)c * n + i] : 0u;
		*(uint32_t*)(rows + (size_t)i * ld + 2 * c) = u;
	}
}
// fp32 parameter gradients -> the caller's fp16 buffer (tcnn's param-precision gradients, trainer.h:72-109): Overwrite
// stores the rounded value, Accumulate adds into the fp16 value in fp32 and rounds once
__global__ void __launch_bounds__(256) k_grad_to_half(uint32_t n, const float* __restrict__ g, half_t* __restrict__ out, uint32_t accumulate) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	out[i] = (half_t)(accumulate ? (float)out[i] + g[i] : g[i]);
}

// ---------------------------------------------------------------- host launchers
void launch_enc_to_layout(hipStream_t s, uint32_t n, uint32_t L, const uint32_t* paired, half_t* dst, uint32_t layout) {
	if (n) k_enc_relayout<<<(n * L + 255) / 256, 256, 0, s>>>(n, L, paired, dst, layout, 0u, nullptr, nullptr);
}
void launch_enc_from_layout(hipStream_t s, uint32_t n, uint32_t L, const half_t* src, uint32_t layout, uint32_t* paired) {
	if (n) k_enc_relayout<<<(n * L + 255) / 256, 256, 0, s>>>(n, L, nullptr, nullptr, layout, 1u, paired, src);
}
void launch_enc_to_rows(hipStream_t s, uint32_t n, uint32_t L, const uint32_t* paired, half_t* rows, uint32_t ld) {
	if (ld % 2 || ld < 2 * L) throw std::runtime_error("launch_enc_to_rows: ld must be even and >= 2 L");
	const uint64_t m = (uint64_t)n * (ld / 2);
	if (m) k_enc_rows<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(n, L, ld, paired, rows, 0u, nullptr, nullptr);
}
void launch_enc_from_rows(hipStream_t s, uint32_t n, uint32_t L, const half_t* rows, uint32_t ld, uint32_t* paired) {
	if (ld % 2 || ld < 2 * L) throw std::runtime_error("launch_enc_from_rows: ld must be even and >= 2 L");
	const uint64_t m = (uint64_t)n * (ld / 2);
	if (m) k_enc_rows<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(n, L, ld, nullptr, nullptr, 1u, paired, rows);
}
void launch_grad_to_half(hipStream_t s, uint32_t n, const float* g, half_t* out, bool accumulate) {
	if (n) k_grad_to_half<<<(n + 255) / 256, 256, 0, s>>>(n, g, out, accumulate ? 1u : 0u);
}
void launch_enc_input_grad(hipStream_t s, uint32_t n, uint32_t ld, uint32_t L, const half_t* dLdy, const float* dydx, float* dLdx, uint32_t stride) {
	if (n) k_enc_input_grad<<<(n + 255) / 256, 256, 0, s>>>(n, ld, L, (const uint32_t*)dLdy, dydx, dLdx, stride);
}
void launch_enc_ddLdoutput(hipStream_t s, uint32_t n, uint32_t ld, uint32_t L, const float* ddx, const float* dydx, half_t* out, float4* v4) {
	if (n) k_enc_ddLdoutput<<<(n + 255) / 256, 256, 0, s>>>(n, ld, L, ddx, dydx, (uint32_t*)out, v4);
}
void launch_grid_encode(hipStream_t s, const uint32_t* n_ptr, uint32_t n_fixed, uint32_t ld, const float* coords, uint32_t coord_stride,
                        const GridLevels& gl, uint32_t valid_level, const half_t* grid, uint32_t* enc, float* dydx, uint32_t grid_x,
                        const EncodeRollover* ro) {
	if (!grid_x) return;
	const EncodeRollover r = ro ? *ro : EncodeRollover{nullptr, 0u, nullptr, nullptr};
	dbg_lds_gate(s);
	k_grid_encode<<<dim3(grid_x, gl.n_levels), 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, grid, enc, dydx, r);
}
size_t scatter_records_capacity(uint32_t n_cap, uint32_t n_levels) { return (size_t)n_cap * n_levels * 8; }
std::vector<uint32_t> scatter_accum_jobs(const GridLevels& gl, uint32_t n_buckets, uint32_t& n_split) {
	// parts of a bucket ~ its records relative to a hashed level's bucket: 32 x 4096 / (entries of the smallest level
	// overlapping it), clamped to [1, 32] (level 0 at 16^3: 32 parts; 23^3: 10; 33^3: 3; 48^3 and up: 1)
	std::vector<uint32_t> jobs;
	n_split = 0;
	for (uint32_t b = 0; b < n_buckets; ++b) {
		uint32_t smin = 0xffffffffu;
		for (uint32_t l = 0; l < gl.n_levels; ++l)
			if (gl.offset[l] < (b + 1) * SB_SIZE && gl.offset[l + 1] > b * SB_SIZE) smin = std::min(smin, gl.offset[l + 1] - gl.offset[l]);
		const uint32_t parts = smin == 0xffffffffu ? 1u : std::max(1u, std::min(32u, (uint32_t)((32ull * SB_SIZE) / std::max(1u, smin))));
		const uint32_t slot = parts > 1 ? n_split++ : 0u;
		for (uint32_t p = 0; p < parts; ++p) { jobs.push_back(b); jobs.push_back(p); jobs.push_back(parts); jobs.push_back(slot); }
	}
	return jobs;
}
std::vector<uint32_t> scatter_region_jobs(const GridLevels& gl, uint32_t& n_split, std::vector<uint32_t>& jobs_before_level) {
	// level-local buckets; parts as scatter_accum_jobs: 32 x 4096 / the level's entries, clamped to [1, 32]
	std::vector<uint32_t> jobs;
	n_split = 0;
	jobs_before_level.assign(gl.n_levels + 1, 0u);
	for (uint32_t l = 0; l < gl.n_levels; ++l) {
		const uint32_t size = gl.offset[l + 1] - gl.offset[l], nlb = (size + SB_SIZE - 1) / SB_SIZE;
		if (nlb > SB_LEVEL_BUCKETS) throw std::runtime_error("hash-grid level table too large for the scatter's per-level buckets");
		const uint32_t parts = std::max(1u, std::min(32u, (uint32_t)((32ull * SB_SIZE) / std::max(1u, size))));
		for (uint32_t k = 0; k < nlb; ++k) {
			const uint32_t slot = parts > 1 ? n_split++ : 0u;
			for (uint32_t p = 0; p < parts; ++p) { jobs.push_back(l); jobs.push_back(k); jobs.push_back(p | (parts << 16)); jobs.push_back(slot); }
		}
		jobs_before_level[l + 1] = (uint32_t)(jobs.size() / 4);
	}
	return jobs;
}
uint32_t scatter_n_buckets(const GridLevels& gl) {
	for (uint32_t l = 0; l < gl.n_levels; ++l)
		if (((gl.offset[l + 1] - 1) >> SB_SHIFT) - (gl.offset[l] >> SB_SHIFT) + 1 > SB_LEVEL_BUCKETS)
			throw std::runtime_error("hash-grid level table too large for the scatter's per-level buckets");
	return (gl.offset[gl.n_levels] + SB_SIZE - 1) >> SB_SHIFT;
}
// the accumulation grid: n jobs rounded up to whole rounds of 8 XCD groups (the remap's domain)
static inline uint32_t accum_blocks(uint32_t n, uint32_t xg) { return (n + 8 * xg - 1) / (8 * xg) * (8 * xg); }
void launch_grid_scatter(hipStream_t s, const uint32_t* n_ptr, uint32_t n_fixed, uint32_t ld, const float* coords, uint32_t coord_stride,
                         const GridLevels& gl, uint32_t valid_level, const half_t* dLdenc, const half_t* g, const float4* v, float* grads,
                         const ScatterWork& w, void* scan_tmp, size_t scan_tmp_bytes, const ScatterSplit* split) {
	if (w.mode == 2) {
		// the grid spans the workspace's sample capacity (w.n_chunks x w.chunk >= n)
		// one workgroup per (chunk, level) by default: ~14x the workgroups of a level loop, so the phases (corner
		// contributions, bucket count, scan, stage, region write) of different workgroups overlap on a CU
		const uint32_t n_lv = std::min(gl.n_levels, valid_level + 1);
		const dim3 grid(w.n_chunks, w.level_groups ? std::min(w.level_groups, n_lv) : n_lv);
		dbg_lds_gate(s);
		if (w.chunk == 1024)
			k_scatter_bin_r<1024><<<grid, 1024, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc,
			                                            (const uint32_t*)g, v, w);
		else if (w.chunk == 256)
			k_scatter_bin_r<256><<<grid, 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc,
			                                          (const uint32_t*)g, v, w);
		else
			k_scatter_bin_r<512><<<grid, 512, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc,
			                                          (const uint32_t*)g, v, w);
		const uint32_t n_act = std::min(valid_level + 1, gl.n_levels);
		if (!split) {
			const uint32_t nj = std::min(w.n_jobs2, w.jobs2_before[n_act]);
			dbg_lds_gate(s);
			if (nj) k_scatter_accum_r<<<accum_blocks(nj, w.xcd_group), 64 * SC_WAVES, 0, s>>>(w, gl, grads, w.chunk * 8, 0u, nj, w.xcd_group);
			return;
		}
		uint32_t lo = 0;
		for (uint32_t gi = 0; gi < split->n_groups && lo < n_act; ++gi) {
			const uint32_t hi = gi + 1 == split->n_groups ? n_act : std::min(split->level_end[gi], n_act);
			if (hi <= lo) continue;
			const uint32_t j0 = std::min(w.n_jobs2, w.jobs2_before[lo]), j1 = std::min(w.n_jobs2, w.jobs2_before[hi]);
			dbg_lds_gate(s);
			if (j1 > j0)
				k_scatter_accum_r<<<accum_blocks(j1 - j0, w.xcd_group), 64 * SC_WAVES, 0, s>>>(w, gl, grads, w.chunk * 8, j0, j1 - j0, w.xcd_group);
			if (split->done) split->done(lo, hi);
			lo = hi;
		}
		return;
	}
	if (w.mode == 0) {
		// the grid spans the workspace's sample capacity (w.n_chunks x w.chunk >= n)
		const size_t nb = (size_t)w.n_active * w.n_chunks;
		if (w.chunk == 1024)
			k_scatter_hist_w<1024><<<w.n_chunks, 1024, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc,
			                                                   (const uint32_t*)g, v, w);
		else
			k_scatter_hist_w<512><<<w.n_chunks, 512, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc,
			                                                 (const uint32_t*)g, v, w);
		launch_exclusive_scan(s, scan_tmp, scan_tmp_bytes, w.counts, w.offs, (uint32_t)nb + 1);
		if (w.chunk == 1024)
			k_scatter_bin_w<1024><<<w.n_chunks, 1024, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc,
			                                                  (const uint32_t*)g, v, w);
		else
			k_scatter_bin_w<512><<<w.n_chunks, 512, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc,
			                                                (const uint32_t*)g, v, w);
		ScatterWork wa = w;
		wa.n_blocks = w.n_chunks;  // bucket b's records start at offs[b * n_chunks]
		k_scatter_accum<<<w.n_jobs, 256, 0, s>>>(wa, grads, gl.offset[gl.n_levels]);
		return;
	}
	// the grid always spans the workspace's sample capacity (w.n_blocks x 256 >= n, checked by the host)
	const uint32_t nblk = w.n_blocks;
	const size_t nb = (size_t)w.n_active * w.n_blocks;  // buckets past n_active get no records (scatter_work_for)
	k_scatter_hist<<<nblk, 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc, (const uint32_t*)g, v, w);
	launch_exclusive_scan(s, scan_tmp, scan_tmp_bytes, w.counts, w.offs, (uint32_t)nb + 1);
	k_scatter_bin<<<nblk, 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc, (const uint32_t*)g, v, w);
	// every bucket (also one without records: its entries' gradient is zero) is written by its workgroup
	k_scatter_accum<<<w.n_jobs, 256, 0, s>>>(w, grads, gl.offset[gl.n_levels]);
}

} // namespace neus
