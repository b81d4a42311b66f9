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
#include <algorithm>

namespace neus {

struct LevelSetup { float pos[3]; uint32_t g[3]; float scale; uint32_t hsize, res; };

__device__ __forceinline__ LevelSetup level_setup(const GridLevels& gl, uint32_t l, float x, float y, float z) {
	LevelSetup s;
	s.scale = gl.scale[l]; s.res = gl.res[l]; s.hsize = gl.offset[l + 1] - gl.offset[l];
	const float in[3] = {x, y, z};
#pragma unroll
	for (int d = 0; d < 3; ++d) {
		// pos_fract (common_device.h:404-434), linear interpolation. `input * scale + 0.5f` is one
		// expression that nvcc (--fmad=true, the default) emits as a single FFMA: fused here too.
		float p = __builtin_fmaf(in[d], s.scale, 0.5f);
		float fl = floorf(p);
		s.g[d] = (uint32_t)(int)fl;
		s.pos[d] = p - fl;
	}
	return s;
}

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
		// 8 corner gathers (half2 each), issued together
		h2 v[8];
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			const uint32_t gx = s.g[0] + (idx & 1), gy = s.g[1] + ((idx >> 1) & 1), gz = s.g[2] + ((idx >> 2) & 1);
			const uint32_t e = grid_index(s.hsize, s.res, gx, gy, gz);
			v[idx] = *(const h2*)(gp + 2 * (size_t)e);
		}
		// fp16 accumulation of fp16-rounded terms, as the reference (result[f] += (T)(weight * data))
		half_t r0 = (half_t)0.f, r1 = (half_t)0.f;
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			float w = 1.f;
#pragma unroll
			for (int d = 0; d < 3; ++d) w *= (idx & (1u << d)) ? s.pos[d] : 1.f - s.pos[d];
			r0 = (half_t)((float)r0 + (float)(half_t)(w * (float)v[idx][0]));
			r1 = (half_t)((float)r1 + (float)(half_t)(w * (float)v[idx][1]));
		}
		h2 out; out[0] = r0; out[1] = r1;
		enc[(size_t)l * ld + i] = *(uint32_t*)&out;
		if (dydx) {
			float gr[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
#pragma unroll
			for (int gd = 0; gd < 3; ++gd) {
#pragma unroll
				for (uint32_t idx = 0; idx < 4; ++idx) {
					float w = s.scale;
					uint32_t cl = 0;
#pragma unroll
					for (int ngd = 0; ngd < 2; ++ngd) {
						const int d = ngd >= gd ? ngd + 1 : ngd;
						if (idx & (1u << ngd)) { w *= s.pos[d]; cl |= 1u << d; } else { w *= 1.f - s.pos[d]; }
					}
					const uint32_t cr = cl | (1u << gd);
					gr[0][gd] = __builtin_fmaf(w, (float)v[cr][0] - (float)v[cl][0], gr[0][gd]);
					gr[1][gd] = __builtin_fmaf(w, (float)v[cr][1] - (float)v[cl][1], gr[1][gd]);
				}
			}
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

// grads: fp32 grid gradient (grid part of the parameter gradient vector).
// dLdenc, g: [L][ld] packed half2; v: [ld] float4 (dL/d grad_sdf, w unused).
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
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const float* c = coords + (size_t)i * coord_stride;
		LevelSetup s = level_setup(gl, l, c[0], c[1], c[2]);
		uint32_t a = dLdenc[(size_t)l * ld + i], b = g[(size_t)l * ld + i];
		const h2 d1 = *(h2*)&a, g2 = *(h2*)&b;
		const float dl0 = (float)d1[0], dl1 = (float)d1[1], g0 = (float)g2[0], g1 = (float)g2[1];
		const float4 vv = v4[i];
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
			atomic_add_f32(gg + 2 * (size_t)e, a0);
			atomic_add_f32(gg + 2 * (size_t)e + 1, a1);
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
