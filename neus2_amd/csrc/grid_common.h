// One hash-grid level for one position: shared by the stand-alone encode kernel (grid.hip) and the
// fused encode+MLP kernels (mlp.hip), so both produce bit-identical features and dy/dx.
// Restates kernel_grid (my_tcnn grid.h:174-369) for N_POS_DIMS = 3, 2 features, linear interpolation.
#pragma once
#include "common.h"

namespace neus {

struct LevelSetup { float pos[3]; uint32_t g[3]; float scale; uint32_t hsize, res; };

__device__ __forceinline__ LevelSetup level_setup(float scale, uint32_t res, uint32_t hsize, float x, float y, float z) {
	LevelSetup s;
	s.scale = scale; s.res = res; s.hsize = hsize;
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
__device__ __forceinline__ LevelSetup level_setup(const GridLevels& gl, uint32_t l, float x, float y, float z) {
	return level_setup(gl.scale[l], gl.res[l], gl.offset[l + 1] - gl.offset[l], x, y, z);
}

// 8 corner gathers (half2 each) of one level, issued together. gp points at the level's table.
__device__ __forceinline__ void gather_corners(const LevelSetup& s, const half_t* __restrict__ gp, h2 v[8]) {
#pragma unroll
	for (uint32_t idx = 0; idx < 8; ++idx) {
		const uint32_t gx = s.g[0] + (idx & 1), gy = s.g[1] + ((idx >> 1) & 1), gz = s.g[2] + ((idx >> 2) & 1);
		const uint32_t e = grid_index(s.hsize, s.res, gx, gy, gz);
		v[idx] = *(const h2*)(gp + 2 * (size_t)e);
	}
}

// Features: fp16 accumulation of fp16-rounded terms, as the reference (result[f] += (T)(weight * data)).
__device__ __forceinline__ h2 interp_features(const LevelSetup& s, const h2 v[8]) {
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
	return out;
}

// d(feature f)/d(x_d): grads += weight * (right - left) * pos_derivative(=1), one FFMA per term
// under nvcc --fmad=true (grid.h:330-362).
__device__ __forceinline__ void interp_dydx(const LevelSetup& s, const h2 v[8], float gr[2][3]) {
#pragma unroll
	for (int f = 0; f < 2; ++f)
#pragma unroll
		for (int d = 0; d < 3; ++d) gr[f][d] = 0.f;
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
}

} // namespace neus
