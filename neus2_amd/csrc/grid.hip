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

// Wave-aggregated atomic add of (a0, a1) to gg[2e], gg[2e+1]: consecutive lanes with the same entry
// (consecutive samples of one ray share coarse-level cells) are first summed with a segmented
// shuffle scan, and only the last lane of each run issues the two fp32 atomics. All 64 lanes must
// call this; `ok` masks lanes without a sample.
__device__ __forceinline__ void wave_aggregated_add(float* gg, uint32_t e, float a0, float a1, bool ok) {
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
		if (!tail) return;
	}
	if (!ok) return;
	atomic_add_f32(gg + 2 * (size_t)e, a0);
	atomic_add_f32(gg + 2 * (size_t)e + 1, a1);
}

// grads: fp32 grid gradient (grid part of the parameter gradient vector).
// dLdenc, g: [L][ld] packed half2; v: [ld] float4 (dL/d grad_sdf, w unused).
// Every lane of a wave stays in the loop (wave-wide shuffles), lanes past n are masked.
__global__ void __launch_bounds__(256) k_grid_scatter(
	const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, uint32_t ld,
	const float* __restrict__ coords, uint32_t coord_stride,
	const GridLevels gl, uint32_t valid_level,
	const uint32_t* __restrict__ dLdenc, const uint32_t* __restrict__ g, const float4* __restrict__ v4,
	float* __restrict__ grads) {
	const uint32_t n = load_n(n_ptr, n_fixed);
	const uint32_t l = blockIdx.y;
	if (l > valid_level) return;
	float* gg = grads + (size_t)gl.offset[l] * 2;
	for (uint32_t b0 = blockIdx.x * blockDim.x; b0 < n; b0 += gridDim.x * blockDim.x) {
		const uint32_t i = b0 + threadIdx.x;
		const bool ok = i < n;
		const uint32_t ic = ok ? i : 0;
		const float* c = coords + (size_t)ic * coord_stride;
		LevelSetup s = level_setup(gl, l, c[0], c[1], c[2]);
		uint32_t a = dLdenc[(size_t)l * ld + ic], b = g[(size_t)l * ld + ic];
		const h2 d1 = *(h2*)&a, g2 = *(h2*)&b;
		const float dl0 = (float)d1[0], dl1 = (float)d1[1], g0 = (float)g2[0], g1 = (float)g2[1];
		const float4 vv = v4[ic];
		const float vin[3] = {s.scale * vv.x, s.scale * vv.y, s.scale * vv.z};
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			// first order: w_corner
			float w = 1.f;
#pragma unroll
			for (int d = 0; d < 3; ++d) w *= (idx & (1u << d)) ? s.pos[d] : 1.f - s.pos[d];
			// second order: sum_d (+/-) scale v_d prod_{other} w_other
			float w2 = 0.f;
#pragma unroll
			for (int gd = 0; gd < 3; ++gd) {
				float t = vin[gd];
#pragma unroll
				for (int d = 0; d < 3; ++d) if (d != gd) t *= (idx & (1u << d)) ? s.pos[d] : 1.f - s.pos[d];
				w2 += (idx & (1u << gd)) ? t : -t;
			}
			const float a0 = dl0 * w + g0 * w2;
			const float a1 = dl1 * w + g1 * w2;
			const uint32_t gx = s.g[0] + (idx & 1), gy = s.g[1] + ((idx >> 1) & 1), gz = s.g[2] + ((idx >> 2) & 1);
			const uint32_t e = grid_index(s.hsize, s.res, gx, gy, gz);
			wave_aggregated_add(gg, e, a0, a1, ok);
		}
	}
}

// ---------------------------------------------------------------- host launchers
void launch_grid_encode(hipStream_t s, const uint32_t* n_ptr, uint32_t n_fixed, uint32_t ld, const float* coords, uint32_t coord_stride,
                        const GridLevels& gl, uint32_t valid_level, const half_t* grid, uint32_t* enc, float* dydx, uint32_t grid_x) {
	if (!grid_x) return;
	k_grid_encode<<<dim3(grid_x, gl.n_levels), 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, grid, enc, dydx);
}
void launch_grid_scatter(hipStream_t s, const uint32_t* n_ptr, uint32_t n_fixed, uint32_t ld, const float* coords, uint32_t coord_stride,
                         const GridLevels& gl, uint32_t valid_level, const half_t* dLdenc, const half_t* g, const float4* v, float* grads, uint32_t grid_x) {
	if (!grid_x) return;
	k_grid_scatter<<<dim3(grid_x, gl.n_levels), 256, 0, s>>>(n_ptr, n_fixed, ld, coords, coord_stride, gl, valid_level, (const uint32_t*)dLdenc, (const uint32_t*)g, v, grads);
}

} // namespace neus
