// The HashGrid encoding in fp32 (tcnn create_encoding(..., EPrecision::Fp32), cpp_api.cu:174-180 -> GridEncoding<float>):
// float table, float features, float gradients. The fp16 encoding of the training step (grid.hip) is untouched; this is
// the operator-API variant a caller asks for with requested_precision = fp32.
//   k_grid_f32_forward : kernel_grid (grid.h:174-369) with T = float: result[f] += weight * value in fp32, dy/dx kept
//                        for dL_dinput / second order
//   k_grid_f32_backward: kernel_grid_backward (grid.h:371-500; float atomicAdd per feature, as GRAD_T = float)
//   k_grid_f32_input_grad: dL_dinput = sum over the 2L features, in feature order, of dL_dy . dy/dx (kernel_grid_
//                        backward_input, grid.h:804-830: one thread per sample, so the sum is run-to-run deterministic)
//   k_grid_f32_bbi     : kernel_grid_backward_input_backward_grid (grid.h:880-1007) and dL_ddLdoutput = dy/dx .
//                        dL_ddLdinput (kernel_grid_backward_input_backward_dLdoutput)
// One thread per (sample, level) (blockIdx.y = level, as the reference's launch): a level's table stays in the XCD's L2
// while its blocks run. Output / dL_doutput layouts: AoS [n][2L] (cpp::Module's column-major view) or SoA [2L][n].
#include "kernels.h"
#include "grid_common.h"

namespace neus {

namespace {

__device__ __forceinline__ size_t enc_addr(uint32_t layout, uint32_t n, uint32_t L, uint32_t i, uint32_t col) {
	return layout == ENC_LAYOUT_AOS ? (size_t)i * 2 * L + col : (size_t)col * n + i;
}

__device__ __forceinline__ void gather_f32(const LevelSetup& s, const float* __restrict__ gp, float v[8][2], uint32_t e[8]) {
#pragma unroll
	for (uint32_t idx = 0; idx < 8; ++idx) {
		const uint32_t gx = s.g[0] + (idx & 1), gy = s.g[1] + ((idx >> 1) & 1), gz = s.g[2] + ((idx >> 2) & 1);
		e[idx] = grid_index(s.hsize, s.res, gx, gy, gz);
		const float2 t = *(const float2*)(gp + 2 * (size_t)e[idx]);
		v[idx][0] = t.x; v[idx][1] = t.y;
	}
}

__device__ __forceinline__ float corner_weight(const LevelSetup& s, uint32_t idx) {
	float w = 1.f;
#pragma unroll
	for (int d = 0; d < 3; ++d) w *= (idx & (1u << d)) ? s.pos[d] : 1.f - s.pos[d];
	return w;
}

// d(feature f)/d(x_d) (grid.h:330-362, pos_derivative = 1 for linear interpolation)
__device__ __forceinline__ void dydx_f32(const LevelSetup& s, const float v[8][2], float gr[2][3]) {
#pragma unroll
	for (int gd = 0; gd < 3; ++gd) {
		gr[0][gd] = gr[1][gd] = 0.f;
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
			gr[0][gd] = __builtin_fmaf(w, v[cr][0] - v[cl][0], gr[0][gd]);
			gr[1][gd] = __builtin_fmaf(w, v[cr][1] - v[cl][1], gr[1][gd]);
		}
	}
}

__global__ void __launch_bounds__(256) k_grid_f32_forward(uint32_t n, const GridLevels gl, uint32_t valid_level, const float* __restrict__ coords,
                                                          const float* __restrict__ table, float* __restrict__ out, uint32_t layout,
                                                          float* __restrict__ dydx) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, l = blockIdx.y, L = gl.n_levels;
	if (i >= n) return;
	float f0 = 0.f, f1 = 0.f, gr[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
	if (l <= valid_level) {
		const LevelSetup s = level_setup(gl, l, coords[(size_t)i * 3], coords[(size_t)i * 3 + 1], coords[(size_t)i * 3 + 2]);
		float v[8][2];
		uint32_t e[8];
		gather_f32(s, table + (size_t)gl.offset[l] * 2, v, e);
#pragma unroll
		for (uint32_t idx = 0; idx < 8; ++idx) {
			const float w = corner_weight(s, idx);
			f0 += w * v[idx][0];
			f1 += w * v[idx][1];
		}
		if (dydx) dydx_f32(s, v, gr);
	}
	out[enc_addr(layout, n, L, i, 2 * l)] = f0;
	out[enc_addr(layout, n, L, i, 2 * l + 1)] = f1;
	if (dydx) {
#pragma unroll
		for (int f = 0; f < 2; ++f)
#pragma unroll
			for (int d = 0; d < 3; ++d) dydx[(size_t)(6 * l + 3 * f + d) * n + i] = gr[f][d];
	}
}

__global__ void __launch_bounds__(256) k_grid_f32_backward(uint32_t n, const GridLevels gl, uint32_t valid_level, const float* __restrict__ coords,
                                                           const float* __restrict__ dLdy, uint32_t layout, float* __restrict__ grads) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, l = blockIdx.y, L = gl.n_levels;
	if (i >= n || l > valid_level) return;
	const float g0 = dLdy[enc_addr(layout, n, L, i, 2 * l)], g1 = dLdy[enc_addr(layout, n, L, i, 2 * l + 1)];
	const LevelSetup s = level_setup(gl, l, coords[(size_t)i * 3], coords[(size_t)i * 3 + 1], coords[(size_t)i * 3 + 2]);
	float* gp = grads + (size_t)gl.offset[l] * 2;
#pragma unroll
	for (uint32_t idx = 0; idx < 8; ++idx) {
		const uint32_t e = grid_index(s.hsize, s.res, s.g[0] + (idx & 1), s.g[1] + ((idx >> 1) & 1), s.g[2] + ((idx >> 2) & 1));
		const float w = corner_weight(s, idx);
		atomicAdd(gp + 2 * (size_t)e, w * g0);
		atomicAdd(gp + 2 * (size_t)e + 1, w * g1);
	}
}

// dL/dx[i][d] = sum over features k = 2l + f, in k order, of dL_dy[k][i] * dy_dx[k][d][i] (result[dim] += ..., nvcc
// contracted to an FMA); the features of levels past valid_level have dy/dx = 0 (the forward wrote zeros)
__global__ void __launch_bounds__(256) k_grid_f32_input_grad(uint32_t n, uint32_t L, const float* __restrict__ dLdy, uint32_t layout,
                                                             const float* __restrict__ dydx, float* __restrict__ dLdx) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	float r[3] = {0.f, 0.f, 0.f};
	for (uint32_t k = 0; k < 2 * L; ++k) {
		const float g = dLdy[enc_addr(layout, n, L, i, k)];
#pragma unroll
		for (int d = 0; d < 3; ++d) r[d] = __builtin_fmaf(g, dydx[(size_t)(3 * k + d) * n + i], r[d]);
	}
#pragma unroll
	for (int d = 0; d < 3; ++d) dLdx[(size_t)i * 3 + d] = r[d];
}

__global__ void __launch_bounds__(256) k_grid_f32_bbi(uint32_t n, const GridLevels gl, uint32_t valid_level, const float* __restrict__ coords,
                                                      const float* __restrict__ ddx, const float* __restrict__ dLdy, uint32_t layout,
                                                      float* __restrict__ grads, const float* __restrict__ dydx, float* __restrict__ ddLdy) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, l = blockIdx.y, L = gl.n_levels;
	if (i >= n) return;
	const float v0 = ddx[(size_t)i * 3], v1 = ddx[(size_t)i * 3 + 1], v2 = ddx[(size_t)i * 3 + 2];
	if (ddLdy) {
#pragma unroll
		for (int f = 0; f < 2; ++f) {
			const float* r = dydx + (size_t)(6 * l + 3 * f) * n + i;
			ddLdy[enc_addr(layout, n, L, i, 2 * l + f)] = l <= valid_level ? r[0] * v0 + r[(size_t)n] * v1 + r[(size_t)2 * n] * v2 : 0.f;
		}
	}
	if (!grads || l > valid_level) return;
	const LevelSetup s = level_setup(gl, l, coords[(size_t)i * 3], coords[(size_t)i * 3 + 1], coords[(size_t)i * 3 + 2]);
	const float g0 = dLdy[enc_addr(layout, n, L, i, 2 * l)], g1 = dLdy[enc_addr(layout, n, L, i, 2 * l + 1)];
	float* gp = grads + (size_t)gl.offset[l] * 2;
	const float vv[3] = {v0, v1, v2};
#pragma unroll
	for (int gd = 0; gd < 3; ++gd) {
		const float gin = s.scale * vv[gd];
#pragma unroll
		for (uint32_t idx = 0; idx < 4; ++idx) {
			float w = gin;
			uint32_t c[3];
#pragma unroll
			for (int ngd = 0; ngd < 2; ++ngd) {
				const int d = ngd >= gd ? ngd + 1 : ngd;
				if (idx & (1u << ngd)) { w *= s.pos[d]; c[d] = s.g[d] + 1; } else { w *= 1.f - s.pos[d]; c[d] = s.g[d]; }
			}
			c[gd] = s.g[gd];
			const uint32_t el = grid_index(s.hsize, s.res, c[0], c[1], c[2]);
			c[gd] = s.g[gd] + 1;
			const uint32_t er = grid_index(s.hsize, s.res, c[0], c[1], c[2]);
			atomicAdd(gp + 2 * (size_t)el, -w * g0);
			atomicAdd(gp + 2 * (size_t)el + 1, -w * g1);
			atomicAdd(gp + 2 * (size_t)er, w * g0);
			atomicAdd(gp + 2 * (size_t)er + 1, w * g1);
		}
	}
}

void check_layout(uint32_t layout) {
	if (layout != ENC_LAYOUT_AOS && layout != ENC_LAYOUT_SOA) throw std::runtime_error("fp32 HashGrid: output layout AoS or SoA");
}

}  // namespace

void launch_grid_f32_forward(hipStream_t s, uint32_t n, const GridLevels& gl, uint32_t valid_level, const float* coords, const float* table,
                             float* out, uint32_t layout, float* dydx) {
	check_layout(layout);
	if (n) k_grid_f32_forward<<<dim3((n + 255) / 256, gl.n_levels), 256, 0, s>>>(n, gl, valid_level, coords, table, out, layout, dydx);
}
void launch_grid_f32_backward(hipStream_t s, uint32_t n, const GridLevels& gl, uint32_t valid_level, const float* coords, const float* dLdy,
                              uint32_t layout, float* grads, const float* dydx, float* dLdx) {
	check_layout(layout);
	if (dLdx && !dydx) throw std::runtime_error("fp32 HashGrid backward: dL_dinput needs the forward's dy/dx");
	if (!n) return;
	if (grads) k_grid_f32_backward<<<dim3((n + 255) / 256, gl.n_levels), 256, 0, s>>>(n, gl, valid_level, coords, dLdy, layout, grads);
	if (dLdx) k_grid_f32_input_grad<<<(n + 255) / 256, 256, 0, s>>>(n, gl.n_levels, dLdy, layout, dydx, dLdx);
}
void launch_grid_f32_bbi(hipStream_t s, uint32_t n, const GridLevels& gl, uint32_t valid_level, const float* coords, const float* ddx,
                         const float* dLdy, uint32_t layout, float* grads, const float* dydx, float* ddLdy) {
	check_layout(layout);
	if (n) k_grid_f32_bbi<<<dim3((n + 255) / 256, gl.n_levels), 256, 0, s>>>(n, gl, valid_level, coords, ddx, dLdy, layout, grads, dydx, ddLdy);
}

}  // namespace neus
