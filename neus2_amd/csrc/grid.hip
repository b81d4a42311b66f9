// Multiresolution hash-grid encoding for gfx950.
//
//   k_grid_encode  : forward (enc, optional dy/dx) — restates kernel_grid (grid.h:174-369)
//   k_grid_scatter : fused first-order (kernel_grid_backward, grid.h:371-500) and second-order
//                    (kernel_grid_backward_input_backward_grid, grid.h:880-1007) parameter
//                    gradients: ONE pass, one fp32 RMW per corner-feature instead of the
//                    reference's two kernels x 24 corner atomics.
//
// Launch shape: blockIdx.y = level (level-major, like the reference): resident blocks work on
// one or two levels at a time, so the hashed level (2^19 x 4 B = 2 MiB) stays in the XCD's
// 4 MiB L2 while the blocks of that level run. Samples are grid-strided and the active count is
// read from device memory, so the host never syncs and the launch is graph-capturable.
#include "kernels.h"
#include "grid_common.h"
#include <algorithm>

namespace neus {

__device__ __forceinline__ uint32_t load_n(const uint32_t* n_ptr, uint32_t n_fixed) { return n_ptr ? *n_ptr : n_fixed; }

// enc: [L][ld] packed half2 (features 2l, 2l+1); dydx: [L*6][ld] f32 (feature f, dim d at row 6l+3f+d)
__global__ void __launch_bounds__(256) k_grid_encode(
	const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
	const float* __restrict__ coords, uint32_t coord_stride,
	const GridLevels gl, uint32_t valid_level,
	const half_t* __restrict__ grid, uint32_t* __restrict__ enc, float* __restrict__ dydx) {
	const uint32_t n = load_n(n_ptr, n_fixed);
	const uint32_t l = blockIdx.y;
	const half_t* gp = grid + (size_t)gl.offset[l] * 2;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		if (l > valid_level) {
			enc[(size_t)l * ld + i] = 0u;
			if (dydx) {
#pragma unroll
				for (int k = 0; k < 6; ++k) dydx[(size_t)(6 * l + k) * ld + i] = 0.0f;
			}
			continue;
		}
		const float* c = coords + (size_t)i * coord_stride;
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
	const int lane = threadIdx.x & 63;
	if (!ok) { e = 0xffffffffu; a0 = a1 = 0.f; }
	const uint32_t e_prev = __shfl_up(e, 1);
	const bool head = lane == 0 || e_prev != e;
	if (__ballot(!head) != 0) {  // at least one run longer than one lane
		int rs = head ? lane : 0;
#pragma unroll
		for (int off = 1; off < 64; off <<= 1) { const int t = __shfl_up(rs, off); if (lane >= off) rs = max(rs, t); }
#pragma unroll
		for (int off = 1; off < 64; off <<= 1) {
			const float t0 = __shfl_up(a0, off), t1 = __shfl_up(a1, off);
			if (lane - off >= rs) { a0 += t0; a1 += t1; }
		}
		const uint32_t e_next = __shfl_down(e, 1);
		const bool tail = lane == 63 || e_next != e;
		return ok && tail;
	}
	return ok;
}

// ---------------------------------------------------------------- hash-grid gradient scatter
// Fused first-order (kernel_grid_backward, grid.h:371-500) and second-order
// (kernel_grid_backward_input_backward_grid, grid.h:880-1007) gradient of every corner of every level.
// The reference adds each corner with an fp16x2 global atomic at a random address; on MI355X float
// atomics run at the memory side and a wave-instruction whose 64 lanes hit 64 random addresses runs
// ~17x below the atomic byte rate. Here the contributions are instead binned by destination:
//   k_scatter_bin<0>  per-block histogram of contributions over 8192-entry buckets (LDS atomics)
//   exclusive scan    bucket-major [bucket][block] -> each block's slot range in each bucket
//   k_scatter_bin<1>  recompute the contributions and write them to their bucket's slots
//   k_scatter_accum   one workgroup per 64K-record chunk: accumulate in LDS (fp32), then add the
//                     touched part of the bucket to the fp32 gradient with contiguous atomics
// Both bin passes evaluate the identical contribution sequence, so the slot counts always match.
template <int PASS>
__global__ void __launch_bounds__(256) k_scatter_bin(const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
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
		const LevelSetup s = level_setup(gl, l, x, y, z);
		const uint32_t a = dLdenc[(size_t)l * ld + ic], b2 = g[(size_t)l * ld + ic];
		const h2 d1 = *(const h2*)&a, g2 = *(const h2*)&b2;
		const float dl0 = (float)d1[0], dl1 = (float)d1[1], g0 = (float)g2[0], g1 = (float)g2[1];
		const float vin[3] = {s.scale * vv.x, s.scale * vv.y, s.scale * vv.z};
		const uint32_t off = gl.offset[l];
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			// first order: w_corner; second order: sum_d (+/-) scale v_d prod_{other} w_other
			float wc = 1.f;
#pragma unroll
			for (int d = 0; d < 3; ++d) wc *= (idx & (1u << d)) ? s.pos[d] : 1.f - s.pos[d];
			float w2 = 0.f;
#pragma unroll
			for (int gd = 0; gd < 3; ++gd) {
				float t = vin[gd];
#pragma unroll
				for (int d = 0; d < 3; ++d) if (d != gd) t *= (idx & (1u << d)) ? s.pos[d] : 1.f - s.pos[d];
				w2 += (idx & (1u << gd)) ? t : -t;
			}
			float a0 = dl0 * wc + g0 * w2;
			float a1 = dl1 * wc + g1 * w2;
			const uint32_t gx = s.g[0] + (idx & 1), gy = s.g[1] + ((idx >> 1) & 1), gz = s.g[2] + ((idx >> 2) & 1);
			const uint32_t gidx = off + grid_index(s.hsize, s.res, gx, gy, gz);
			if (wave_run_sum(gidx, a0, a1, ok)) {
				const uint32_t bkt = gidx >> SB_SHIFT;
				if (PASS == 0) {
					atomicAdd(&hist[bkt], 1u);
				} else {
					const uint32_t pos = w.offs[(size_t)bkt * w.n_blocks + blk] + atomicAdd(&hist[bkt], 1u);
					w.rec_i[pos] = (uint16_t)(gidx & (SB_SIZE - 1));
					w.rec_g[pos] = make_float2(a0, a1);
				}
			}
		}
	}
	if (PASS == 0) {
		__syncthreads();
		for (uint32_t b = threadIdx.x; b < w.n_buckets; b += blockDim.x) w.counts[(size_t)b * w.n_blocks + blk] = hist[b];
	}
}

__global__ void __launch_bounds__(256) k_scatter_accum(ScatterWork w, float* __restrict__ grads, uint32_t n_entries) {
	__shared__ float acc[2 * SB_SIZE];
	const size_t nb = (size_t)w.n_buckets * w.n_blocks;
	const uint32_t total = w.offs[nb];
	uint32_t c0 = blockIdx.x * SB_CHUNK;
	if (c0 >= total) return;
	const uint32_t c1 = min(total, c0 + SB_CHUNK);
	// bucket holding record c0: the last b with start(b) <= c0, start(b) = offs[b * n_blocks]
	uint32_t lo = 0, hi = w.n_buckets - 1;
	while (lo < hi) {
		const uint32_t mid = (lo + hi + 1) / 2;
		if (w.offs[(size_t)mid * w.n_blocks] <= c0) lo = mid; else hi = mid - 1;
	}
	uint32_t b = lo;
	while (c0 < c1) {
		const uint32_t bend = b + 1 < w.n_buckets ? min(c1, w.offs[(size_t)(b + 1) * w.n_blocks]) : c1;
		for (uint32_t k = threadIdx.x; k < 2 * SB_SIZE; k += blockDim.x) acc[k] = 0.f;
		__syncthreads();
		for (uint32_t r = c0 + threadIdx.x; r < bend; r += blockDim.x) {
			const uint32_t e = w.rec_i[r];
			const float2 gv = w.rec_g[r];
			atomicAdd(&acc[2 * e], gv.x);
			atomicAdd(&acc[2 * e + 1], gv.y);
		}
		__syncthreads();
		const uint32_t e0 = b << SB_SHIFT;
		const uint32_t ne = min(SB_SIZE, n_entries - e0);
		for (uint32_t k = threadIdx.x; k < 2 * ne; k += blockDim.x) {
			const float vsum = acc[k];
			if (vsum != 0.f) atomic_add_f32(grads + 2 * (size_t)e0 + k, vsum);
		}
		__syncthreads();
		c0 = bend;
		++b;
	}
}

// ---------------------------------------------------------------- host launchers
void launch_grid_encode(hipStream_t s, const uint32_t* n_ptr, uint32_t n_fixed, uint32_t ld, const float* coords, uint32_t coord_stride,
                        const GridLevels& gl, uint32_t valid_level, const half_t* grid, uint32_t* enc, float* dydx, uint32_t grid_x) {
	if (!grid_x) return;
	k_grid_encode<<<dim3(grid_x, gl.n_levels), 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, grid, enc, dydx);
}
size_t scatter_records_capacity(uint32_t n_cap, uint32_t n_levels) { return (size_t)n_cap * n_levels * 8; }
uint32_t scatter_n_buckets(const GridLevels& gl) { return (gl.offset[gl.n_levels] + SB_SIZE - 1) >> SB_SHIFT; }
void launch_grid_scatter(hipStream_t s, const uint32_t* n_ptr, uint32_t n_fixed, uint32_t ld, const float* coords, uint32_t coord_stride,
                         const GridLevels& gl, uint32_t valid_level, const half_t* dLdenc, const half_t* g, const float4* v, float* grads,
                         const ScatterWork& w, void* scan_tmp, size_t scan_tmp_bytes) {
	// the grid always spans the workspace's sample capacity (w.n_blocks x 256 >= n, checked by the host)
	const uint32_t nblk = w.n_blocks, n_cap = nblk * 256;
	const size_t nb = (size_t)w.n_buckets * w.n_blocks;
	k_scatter_bin<0><<<nblk, 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc, (const uint32_t*)g, v, w);
	(void)hipMemsetAsync(w.counts + nb, 0, 4, s);
	launch_exclusive_scan(s, scan_tmp, scan_tmp_bytes, w.counts, w.offs, (uint32_t)nb + 1);
	k_scatter_bin<1><<<nblk, 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc, (const uint32_t*)g, v, w);
	const uint32_t n_chunks = (uint32_t)((scatter_records_capacity(n_cap, gl.n_levels) + SB_CHUNK - 1) / SB_CHUNK);
	k_scatter_accum<<<n_chunks, 256, 0, s>>>(w, grads, gl.offset[gl.n_levels]);
}

} // namespace neus
