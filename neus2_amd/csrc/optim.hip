// Optimizer and occupancy-grid kernels for gfx950.
//
//   k_adam_ema       : Ema(ExponentialDecay(Adam)) step (adam.h:51-160, ema.h:45-110,
//                      exponential_decay.h:61-80) fused with the fp16 weight cast and the EMA
//                      (inference-weight) update: one streaming pass over the P parameters.
//   k_transpose_w    : fp16 transposed copies of the MLP matrices for the MFMA backward.
//   k_grid_samples   : generate_grid_samples_nerf_nonuniform (testbed_nerf.cu:640-669)
//   k_splat_max      : splat_grid_samples_nerf_max_nearest_neighbor (testbed_nerf.cu:671-690)
//   k_ema_grid       : ema_grid_samples_nerf (testbed_nerf.cu:710-740)
//   k_grid_mean_*    : deterministic two-stage mean (testbed_nerf.cu:3384-3389)
//   k_bitfield       : grid_to_bitfield + bitfield_max_pool (testbed_nerf.cu:748-795)
#include "kernels.h"
#include "occ_common.h"
#include <algorithm>

namespace neus {

// adam.h:137's bias correction of step k: sqrtf(1 - beta2^k) and 1 - beta1^k (the table and the fallback share it)
__device__ __forceinline__ void adam_bias_terms(float beta1, float beta2, uint32_t k, float& s2, float& d1) {
	s2 = sqrtf(1 - powf(beta2, (float)k));
	d1 = 1 - powf(beta1, (float)k);
}
__global__ void k_adam_bias_table(float beta1, float beta2, float* __restrict__ tab) {
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= ADAM_BIAS_TAB) return;
	float s2, d1;
	adam_bias_terms(beta1, beta2, k, s2, d1);
	tab[k] = s2;
	tab[ADAM_BIAS_TAB + k] = d1;
}
void launch_adam_bias_table(hipStream_t s, float beta1, float beta2, float* tab) {
	k_adam_bias_table<<<ADAM_BIAS_TAB / 256, 256, 0, s>>>(beta1, beta2, tab);
}

// One parameter's Adam step (adam.h:86-159) on registers: false when it is skipped (a zero gradient of a non-matrix
// parameter, or a disabled parameter class), leaving w / m1 / m2 / step unchanged.
__device__ __forceinline__ bool adam_param(const AdamParams& p, uint32_t i, float graw, float& w, float& m1v, float& m2v, uint32_t& st) {
	float gradient = p.pow2_scale ? graw * p.inv_loss_scale : graw / p.loss_scale;
	const bool is_matrix = i < p.n_matrix;
	const bool skip = is_matrix ? !p.optimize_matrix : (!p.optimize_non_matrix || gradient == 0.f);
	if (skip) return false;
	if (is_matrix) gradient += p.l2_reg * w;
	const float g2 = gradient * gradient;
	m1v = p.beta1 * m1v + (1 - p.beta1) * gradient;
	m2v = p.beta2 * m2v + (1 - p.beta2) * g2;
	const uint32_t cs = ++st;
	float lr;
	if (p.bias_tab && cs < ADAM_BIAS_TAB) lr = p.lr * p.bias_tab[cs] / p.bias_tab[ADAM_BIAS_TAB + cs];
	else if (p.bias_tab && p.bias_converged) lr = p.lr;  // (lr * 1.0f) / 1.0f
	else { float s2, d1; adam_bias_terms(p.beta1, p.beta2, cs, s2, d1); lr = p.lr * s2 / d1; }
	const float elr = fminf(fmaxf(lr / (sqrtf(m2v) + p.eps), 0.0f), 3.402823466e+38f);
	w = w - elr * m1v;
	return true;
}
// The per-parameter step count (adam.h:106, uint32 in the reference) is stored in 16 bits, saturating at 65535, when the
// bias table is converged: the count only enters the bias correction, which is exactly 1.0f from step ADAM_BIAS_TAB on
// (beta^k below 2^-30 there), so every later count gives the same update. Otherwise (betas whose correction has not
// converged by ADAM_BIAS_TAB) the counts are kept in 32 bits and never saturate (AdamSteps<uint32_t>).
template <class ST> struct AdamSteps;
template <> struct AdamSteps<uint16_t> {
	static __device__ __forceinline__ uint32_t sat(uint32_t st) { return st < 0xffffu ? st : 0xffffu; }
	static __device__ __forceinline__ void load4(const uint16_t* p, uint32_t g, uint32_t st[4]) {
		const uint2 S = ((const uint2*)p)[g];
		st[0] = S.x & 0xffffu; st[1] = S.x >> 16; st[2] = S.y & 0xffffu; st[3] = S.y >> 16;
	}
	static __device__ __forceinline__ void store4(uint16_t* p, uint32_t g, const uint32_t st[4]) {
		((uint2*)p)[g] = make_uint2(sat(st[0]) | (sat(st[1]) << 16), sat(st[2]) | (sat(st[3]) << 16));
	}
};
template <> struct AdamSteps<uint32_t> {
	static __device__ __forceinline__ uint32_t sat(uint32_t st) { return st; }
	static __device__ __forceinline__ void load4(const uint32_t* p, uint32_t g, uint32_t st[4]) {
		const uint4 S = ((const uint4*)p)[g];
		st[0] = S.x; st[1] = S.y; st[2] = S.z; st[3] = S.w;
	}
	static __device__ __forceinline__ void store4(uint32_t* p, uint32_t g, const uint32_t st[4]) { ((uint4*)p)[g] = make_uint4(st[0], st[1], st[2], st[3]); }
};
// Ema(ExponentialDecay) of the fp16 weight (ema.h:45-110): the running fp32 EMA, debiased
__device__ __forceinline__ float ema_param(const AdamParams& p, float ema, float wh) {
	return (ema * p.ema_decay * p.ema_debias_old + wh * (1 - p.ema_decay)) * p.ema_debias_new;
}
// the MLP's transposed / permuted fp16 copies of matrix weight i (prepare_weights)
__device__ __forceinline__ void adam_transpose_param(const AdamTranspose& tr, uint32_t i, half_t hv) {
	for (uint32_t j = 0; j < tr.n; ++j) {
		const uint32_t e = i - tr.off[j];
		if (i < tr.off[j] || e >= tr.rows[j] * tr.cols[j]) continue;
		const uint32_t r = e / tr.cols[j], c = e % tr.cols[j];
		tr.dst[j][(size_t)c * tr.rows[j] + r] = hv;
		if (j == 0 && tr.d0p) {
			const int32_t q = c < 48 ? tr.inv[c] : -1;
			if (q >= 0) { tr.d0p[(size_t)r * tr.din + q] = hv; tr.d0Tp[(size_t)q * tr.W + r] = hv; }
		}
	}
}

// grads fp32 (the reference keeps fp16 gradients); weights_fp fp32 master; weights_h fp16 copy used by every kernel;
// ema_tmp fp32 running EMA; ema_h fp16 inference weights. Four consecutive parameters per thread with 16-B (8-B for
// fp16) accesses; the optimizer state of a group is read and written only when one of its four parameters steps (a
// skipped parameter's values are written back unchanged); the n % 4 tail by block 0.
template <class ST>
__global__ void __launch_bounds__(256) k_adam_ema(AdamParams p, float* __restrict__ weights_fp, half_t* __restrict__ weights_h,
                                                  const float* __restrict__ grads, float* __restrict__ m1, float* __restrict__ m2,
                                                  ST* __restrict__ steps, float* __restrict__ ema_tmp, half_t* __restrict__ ema_h,
                                                  StepCounterArgs sc, AdamTranspose tr) {
	if (p.abort && *p.abort) return;  // (the step is re-run: nothing of it is applied)
	if (sc.st && blockIdx.x == 0 && threadIdx.x == 0) step_counters_update(sc.st, sc.target_batch, sc.max_samples, sc.world, sc.fixed_rays, sc.eval_cnt, sc.n_eval);
	const uint32_t ng = p.n / 4;
	for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += gridDim.x * blockDim.x) {
		const uint32_t i0 = 4 * g;
		const float4 G = ((const float4*)grads)[g];
		float4 E = ((const float4*)ema_tmp)[g];
		float gr[4] = {G.x, G.y, G.z, G.w}, e[4] = {E.x, E.y, E.z, E.w};
		half_t wh[4];
		// any parameter of the group steps? (the same skip test as adam_param)
		bool any = false;
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const float gk = p.pow2_scale ? gr[k] * p.inv_loss_scale : gr[k] / p.loss_scale;
			any |= (i0 + k < p.n_matrix) ? p.optimize_matrix != 0u : (p.optimize_non_matrix != 0u && gk != 0.f);
		}
		if (any) {  // (a skipped group reads neither its optimizer state nor its fp32 master weights: the EMA reads the fp16 copy)
			const float4 W = ((const float4*)weights_fp)[g];
			float w[4] = {W.x, W.y, W.z, W.w};
			float4 M1 = ((const float4*)m1)[g], M2 = ((const float4*)m2)[g];
			float a[4] = {M1.x, M1.y, M1.z, M1.w}, b[4] = {M2.x, M2.y, M2.z, M2.w};
			uint32_t st[4];
			AdamSteps<ST>::load4(steps, g, st);
			// the fp16 copy of every parameter of the group is the cast of its fp32 master (weights_h == half(weights_fp)
			// wherever either is written), so a stepping group needs no read of the fp16 copy: 2 B per parameter less
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				adam_param(p, i0 + k, gr[k], w[k], a[k], b[k], st[k]);
				wh[k] = (half_t)w[k];
			}
			((float4*)m1)[g] = make_float4(a[0], a[1], a[2], a[3]);
			((float4*)m2)[g] = make_float4(b[0], b[1], b[2], b[3]);
			AdamSteps<ST>::store4(steps, g, st);
			((float4*)weights_fp)[g] = make_float4(w[0], w[1], w[2], w[3]);
			((uint2*)weights_h)[g] = *(const uint2*)wh;
		} else {
			*(uint2*)wh = ((const uint2*)weights_h)[g];  // (the EMA of a skipped group reads the fp16 copy)
		}
		half_t eh[4];
#pragma unroll
		for (int k = 0; k < 4; ++k) { e[k] = ema_param(p, e[k], (float)wh[k]); eh[k] = (half_t)e[k]; }
		((float4*)ema_tmp)[g] = make_float4(e[0], e[1], e[2], e[3]);
		if (!p.skip_ema_h) ((uint2*)ema_h)[g] = *(const uint2*)eh;
		if (tr.n && i0 < p.n_matrix) {
#pragma unroll
			for (int k = 0; k < 4; ++k)
				if (i0 + k < p.n_matrix) adam_transpose_param(tr, i0 + k, wh[k]);
		}
	}
	// the tail
	if (blockIdx.x == 0 && threadIdx.x < p.n - 4 * ng) {
		const uint32_t i = 4 * ng + threadIdx.x;
		float w = weights_fp[i], a = m1[i], b = m2[i];
		uint32_t st = steps[i];
		if (adam_param(p, i, grads[i], w, a, b, st)) {
			m1[i] = a; m2[i] = b; steps[i] = (ST)AdamSteps<ST>::sat(st); weights_fp[i] = w; weights_h[i] = (half_t)w;
		}
		const float wh = (float)weights_h[i];
		const float f = ema_param(p, ema_tmp[i], wh);
		ema_tmp[i] = f;
		if (!p.skip_ema_h) ema_h[i] = (half_t)f;
		if (tr.n && i < p.n_matrix) adam_transpose_param(tr, i, (half_t)wh);
	}
}

// EGradientMode::Accumulate of the operator modules: dst += src
__global__ void k_add_f32(uint32_t n, const float* __restrict__ src, float* __restrict__ dst) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] += src[i];
}

__global__ void k_cast_half(uint32_t n, const float* __restrict__ in, half_t* __restrict__ out) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = (half_t)in[i];
}

// Fused-kernel copies of the first density layer: W0 columns / W0^T rows in the physical din order
// of the fused encode (mlp.hip din_logical); -1 entries are zero pads.
__global__ void k_permute_din(const half_t* __restrict__ d0, half_t* __restrict__ d0p, half_t* __restrict__ d0Tp, DinPerm perm) {
	const uint32_t n = perm.W * perm.din;
	for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) {
		const uint32_t row = e / perm.din, p = e % perm.din;
		const int32_t k = perm.p[p];
		const half_t v = k >= 0 ? d0[(size_t)row * perm.din + k] : (half_t)0.f;
		d0p[(size_t)row * perm.din + p] = v;
		d0Tp[(size_t)p * perm.W + row] = v;
	}
}

// dst[c][r] = src[r][c]  (all matrices are <= 64x64); with a DinPerm, the block after the last job does
// k_permute_din's work (one launch for both)
__global__ void k_transpose_w(TransposeJobs jobs, const half_t* __restrict__ d0, half_t* __restrict__ d0p, half_t* __restrict__ d0Tp,
                              DinPerm perm) {
	if (blockIdx.x == jobs.n) {
		const uint32_t n = perm.W * perm.din;
		for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) {
			const uint32_t row = e / perm.din, p = e % perm.din;
			const int32_t k = perm.p[p];
			const half_t v = k >= 0 ? d0[(size_t)row * perm.din + k] : (half_t)0.f;
			d0p[(size_t)row * perm.din + p] = v;
			d0Tp[(size_t)p * perm.W + row] = v;
		}
		return;
	}
	const TransposeJob J = jobs.j[blockIdx.x];
	for (uint32_t e = threadIdx.x; e < J.rows * J.cols; e += blockDim.x) {
		const uint32_t r = e / J.cols, c = e % J.cols;
		J.dst[(size_t)c * J.rows + r] = J.src[e];
	}
}

// positions: 3 floats (warped) per sample; indices: density grid cell.
// Samples i_begin .. i_end - 1 of the n_elements of one generate call (a data-parallel rank evaluates its shard
// of the global sample range), written from out_base on.
__global__ void k_grid_samples(uint32_t n_elements, uint32_t i_begin, uint32_t i_end, uint32_t out_base, uint64_t rng_state, uint64_t rng_inc,
                               uint32_t step, float aabb_min_x, float aabb_min_y, float aabb_min_z, float diag_x, float diag_y, float diag_z,
                               const float* __restrict__ grid_in, float* __restrict__ pos, uint32_t* __restrict__ indices,
                               uint32_t n_cascades, float thresh, PcgJumpTable jt) {
	const float amin[3] = {aabb_min_x, aabb_min_y, aabb_min_z}, diag[3] = {diag_x, diag_y, diag_z};
	for (uint32_t i = i_begin + blockIdx.x * blockDim.x + threadIdx.x; i < i_end; i += gridDim.x * blockDim.x) {
		float p[3];
		uint32_t idx;
		grid_sample(n_elements, i, rng_state, rng_inc, step, amin, diag, grid_in, n_cascades, thresh, p, idx, jt);
		const uint32_t o = out_base + (i - i_begin);
		pos[3 * (size_t)o + 0] = p[0];
		pos[3 * (size_t)o + 1] = p[1];
		pos[3 * (size_t)o + 2] = p[2];
		indices[o] = idx;
	}
}

__global__ void k_splat_max(uint32_t n, const uint32_t* __restrict__ indices, const float* __restrict__ density, float* __restrict__ grid_tmp) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
		atomicMax((uint32_t*)&grid_tmp[indices[i]], __float_as_uint(density[i]));
}

__global__ void k_ema_grid(uint32_t n, float decay, float* __restrict__ grid, const float* __restrict__ tmp) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const float prev = grid[i];
		grid[i] = (prev < 0.f) ? prev : fmaxf(prev * decay, tmp[i]);
	}
}

// Deterministic mean of max(grid,0)/G3: fixed-shape two-stage tree (fp32 partials of 1024 each).
__global__ void __launch_bounds__(256) k_grid_mean_partial(const float* __restrict__ grid, float* __restrict__ partial) {
	__shared__ float s[256];
	const uint32_t b = blockIdx.x;  // GRID3 / 1024 blocks
	float acc = 0.f;
	for (int k = 0; k < 4; ++k) acc += fmaxf(grid[b * 1024 + k * 256 + threadIdx.x], 0.f) / (float)GRID3;
	s[threadIdx.x] = acc;
	__syncthreads();
	for (int off = 128; off > 0; off >>= 1) { if (threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off]; __syncthreads(); }
	if (threadIdx.x == 0) partial[b] = s[0];
}
__global__ void __launch_bounds__(256) k_grid_mean_final(const float* __restrict__ partial, uint32_t n_partial, float* __restrict__ mean) {
	__shared__ float s[256];
	float acc = 0.f;
	for (uint32_t k = threadIdx.x; k < n_partial; k += 256) acc += partial[k];
	s[threadIdx.x] = acc;
	__syncthreads();
	for (int off = 128; off > 0; off >>= 1) { if (threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off]; __syncthreads(); }
	if (threadIdx.x == 0) *mean = s[0];
}

// The EMA of the grid (k_ema_grid) with the mean partials of cascade 0 computed by the same blocks over the same
// elements in the same order (k_grid_mean_partial's bits); k_grid_mean_final follows. (A last-block-done final sum
// needs agent-scope fences, which write back the XCD L2s: 50 us here.)
__global__ void __launch_bounds__(256) k_ema_mean(uint32_t n, float decay, float* __restrict__ grid, const float* __restrict__ tmp,
                                                 float* __restrict__ partial) {
	__shared__ float s[256];
	const uint32_t b = blockIdx.x;  // n / 1024 blocks of 1024 cells
	float acc = 0.f;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const uint32_t i = b * 1024 + k * 256 + threadIdx.x;
		const float prev = grid[i];
		const float v = (prev < 0.f) ? prev : fmaxf(prev * decay, tmp[i]);
		grid[i] = v;
		acc += fmaxf(v, 0.f) / (float)GRID3;
	}
	if (b >= GRID3 / 1024) return;  // the mean covers cascade 0 only
	s[threadIdx.x] = acc;
	__syncthreads();
	for (int off = 128; off > 0; off >>= 1) { if (threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off]; __syncthreads(); }
	if (threadIdx.x == 0) partial[b] = s[0];
}

__global__ void k_grid_to_bitfield(uint32_t n_bytes_total, uint32_t n_nonzero, const float* __restrict__ grid, uint8_t* __restrict__ bf,
                                   const float* __restrict__ mean) {
	const float thresh = fminf(NERF_MIN_OPTICAL_THICKNESS, *mean);
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_bytes_total; i += gridDim.x * blockDim.x) {
		if (i >= n_nonzero) { bf[i] = 0; continue; }
		uint8_t bits = 0;
#pragma unroll
		for (uint8_t j = 0; j < 8; ++j) bits |= grid[i * 8 + j] > thresh ? ((uint8_t)1 << j) : 0;
		bf[i] = bits;
	}
}

// All mip levels' max pools in one launch (the reference runs bitfield_max_pool once per level, each reading the
// previous level's final bytes; testbed_nerf.cu:3384-3392). A level-(m+1) bit in the inner region is set iff the
// corresponding level-m byte is nonzero, so the fixpoint is an OR over the level tree. A wave takes 64 consecutive
// bytes of a level (a 4x4x4-byte Morton block): the ballot of "byte nonzero" is exactly the 8 consecutive parent
// bytes (one 64-bit atomic OR); the parent bytes this OR turned nonzero then set their own parent bit, and so on up
// while a byte turns nonzero. Every byte that becomes nonzero is propagated by exactly the wave that made it so (or
// by its own wave when its grid bits were set); OR is order-independent, so the bits are the level-by-level pool's.
// The same launch converts mip 0 (which the pools only read) to the march's linear words (k_bitfield_linear) in
// its last GRID3 / 32 / 64 waves.
__global__ void k_bitfield_pool_all(uint32_t nbytes, uint8_t* __restrict__ bf, uint32_t* __restrict__ lin) {
	const uint32_t lane = threadIdx.x & 63, waves_per_level = nbytes / 64;
	const uint32_t n_waves = waves_per_level * (NERF_CASCADES - 1), n_lin_waves = lin ? GRID3 / 32 / 64 : 0u;
	for (uint32_t wg = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; wg < n_waves + n_lin_waves; wg += (gridDim.x * blockDim.x) >> 6) {
		if (wg >= n_waves) {
			const uint32_t w = (wg - n_waves) * 64 + lane;
			const uint32_t ix = w >> 9, iy = (w >> 2) & 127, iz0 = (w & 3) * 32;
			uint32_t word = 0;
			for (uint32_t b = 0; b < 32; ++b) {
				const uint32_t idx = morton3D(ix, iy, iz0 + b);
				word |= (uint32_t)((bf[idx / 8] >> (idx % 8)) & 1) << b;
			}
			lin[w] = word;
			continue;
		}
		const uint32_t level0 = wg / waves_per_level, w = wg % waves_per_level;
		const uint64_t M = __ballot(bf[(size_t)level0 * nbytes + 64 * w + lane] != 0);
		if (M == 0 || lane != 0) continue;
		// the 8 parent bytes: 8 morton(invert(w) + 8) .. + 7 at level0 + 1
		uint32_t q0 = 8u * morton3D(morton3D_invert(w >> 0) + NERF_GRIDSIZE / 16, morton3D_invert(w >> 1) + NERF_GRIDSIZE / 16,
		                             morton3D_invert(w >> 2) + NERF_GRIDSIZE / 16);
		const uint64_t old = atomicOr((unsigned long long*)(bf + (size_t)(level0 + 1) * nbytes + q0), (unsigned long long)M);
		uint32_t N = 0;  // parent bytes that turned nonzero
#pragma unroll
		for (int k = 0; k < 8; ++k) N |= (((old >> (8 * k)) & 0xffu) == 0 && ((M >> (8 * k)) & 0xffu) != 0) ? (1u << k) : 0u;
		uint32_t level = level0 + 1, p = q0;  // bytes p .. p + 7 of `level`, N: which turned nonzero
		while (N != 0 && level + 1 < NERF_CASCADES) {
			const uint32_t i = p >> 3;
			const uint32_t q = morton3D(morton3D_invert(i >> 0) + NERF_GRIDSIZE / 8, morton3D_invert(i >> 1) + NERF_GRIDSIZE / 8,
			                            morton3D_invert(i >> 2) + NERF_GRIDSIZE / 8);
			const size_t byte = (size_t)(level + 1) * nbytes + q;
			const uint32_t sh = 8u * (uint32_t)(byte & 3);
			const uint32_t o = atomicOr((uint32_t*)(bf + (byte & ~(size_t)3)), N << sh);
			if (((o >> sh) & 0xffu) != 0) break;  // the parent byte was already nonzero: its propagation is someone else's
			N = 1u << (q & 7); p = q & ~7u; ++level;
		}
	}
}

// World-space bounding box of every occupied cell of every mip (the union of the boxes the march's occupancy lookups can
// land in: cell c of mip m covers 0.5 + (c / 128 - 0.5) 2^m .. 0.5 + ((c + 1) / 128 - 0.5) 2^m per axis), padded by
// 1e-4 2^m for the float rounding of the lookup's index. A training ray that misses it cannot produce a sample
// (k_ray_gen culls it: the march of such a ray returns zero samples anyway). Two stages: per-block min / max, then one
// block; empty grid -> an empty box (+inf .. -inf).
constexpr uint32_t OCC_BBOX_BLOCKS = 256;
__global__ void __launch_bounds__(256) k_occ_bbox_partial(const uint8_t* __restrict__ bf, float* __restrict__ partial) {
	float lo[3] = {3.402823466e+38f, 3.402823466e+38f, 3.402823466e+38f}, hi[3] = {-3.402823466e+38f, -3.402823466e+38f, -3.402823466e+38f};
	const uint32_t nbytes = GRID3 / 8 * NERF_CASCADES;
	for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nbytes; b += gridDim.x * blockDim.x) {
		uint32_t bits = bf[b];
		if (!bits) continue;
		const uint32_t mip = b / (GRID3 / 8);
		const float sc = (float)(1u << mip), pad = 1e-4f * sc;
		while (bits) {
			const uint32_t k = (uint32_t)__builtin_ctz(bits);
			bits &= bits - 1;
			const uint32_t idx = (b % (GRID3 / 8)) * 8 + k;
			const uint32_t c[3] = {morton3D_invert(idx >> 0), morton3D_invert(idx >> 1), morton3D_invert(idx >> 2)};
#pragma unroll
			for (int d = 0; d < 3; ++d) {
				lo[d] = fminf(lo[d], 0.5f + ((float)c[d] / NERF_GRIDSIZE - 0.5f) * sc - pad);
				hi[d] = fmaxf(hi[d], 0.5f + ((float)(c[d] + 1) / NERF_GRIDSIZE - 0.5f) * sc + pad);
			}
		}
	}
	__shared__ float s[6][4];
#pragma unroll
	for (int off = 32; off > 0; off >>= 1)
#pragma unroll
		for (int d = 0; d < 3; ++d) { lo[d] = fminf(lo[d], __shfl_xor(lo[d], off)); hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], off)); }
	const uint32_t wv = threadIdx.x >> 6;
	if ((threadIdx.x & 63) == 0)
		for (int d = 0; d < 3; ++d) { s[d][wv] = lo[d]; s[3 + d][wv] = hi[d]; }
	__syncthreads();
	if (threadIdx.x < 6) {
		float v = s[threadIdx.x][0];
		for (int w = 1; w < 4; ++w) v = threadIdx.x < 3 ? fminf(v, s[threadIdx.x][w]) : fmaxf(v, s[threadIdx.x][w]);
		partial[blockIdx.x * 6 + threadIdx.x] = v;
	}
}
__global__ void __launch_bounds__(256) k_occ_bbox_final(const float* __restrict__ partial, uint32_t n, float* __restrict__ bbox) {
	float lo[3] = {3.402823466e+38f, 3.402823466e+38f, 3.402823466e+38f}, hi[3] = {-3.402823466e+38f, -3.402823466e+38f, -3.402823466e+38f};
	for (uint32_t b = threadIdx.x; b < n; b += blockDim.x)
#pragma unroll
		for (int d = 0; d < 3; ++d) { lo[d] = fminf(lo[d], partial[b * 6 + d]); hi[d] = fmaxf(hi[d], partial[b * 6 + 3 + d]); }
	__shared__ float s[6][4];
#pragma unroll
	for (int off = 32; off > 0; off >>= 1)
#pragma unroll
		for (int d = 0; d < 3; ++d) { lo[d] = fminf(lo[d], __shfl_xor(lo[d], off)); hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], off)); }
	const uint32_t wv = threadIdx.x >> 6;
	if ((threadIdx.x & 63) == 0)
		for (int d = 0; d < 3; ++d) { s[d][wv] = lo[d]; s[3 + d][wv] = hi[d]; }
	__syncthreads();
	if (threadIdx.x < 6) {
		float v = s[threadIdx.x][0];
		for (int w = 1; w < 4; ++w) v = threadIdx.x < 3 ? fminf(v, s[threadIdx.x][w]) : fmaxf(v, s[threadIdx.x][w]);
		bbox[threadIdx.x] = v;
	}
}

// ---------------------------------------------------------------- host launchers
static inline uint32_t nblk(uint64_t n, uint32_t cap = 4096) { return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, cap)); }
void launch_adam_ema(hipStream_t s, const AdamParams& p, float* weights_fp, half_t* weights_h, const float* grads, float* m1, float* m2,
                     void* steps, bool steps32, float* ema_tmp, half_t* ema_h, const StepCounterArgs* counters, const AdamTranspose* tr) {
	const StepCounterArgs sc = counters ? *counters : StepCounterArgs{nullptr, 0u, 0u, 1u, 0u, nullptr, 0u};
	AdamTranspose t{};
	if (tr) t = *tr;
	dbg_lds_gate(s);
	const uint32_t nb = nblk(std::max<uint64_t>(1, p.n / 4), 16384);
	if (steps32) k_adam_ema<uint32_t><<<nb, 256, 0, s>>>(p, weights_fp, weights_h, grads, m1, m2, (uint32_t*)steps, ema_tmp, ema_h, sc, t);
	else k_adam_ema<uint16_t><<<nb, 256, 0, s>>>(p, weights_fp, weights_h, grads, m1, m2, (uint16_t*)steps, ema_tmp, ema_h, sc, t);
}
void launch_adam_ema_range(hipStream_t s, AdamParams p, uint32_t lo, uint32_t hi, float* weights_fp, half_t* weights_h, const float* grads,
                           float* m1, float* m2, void* steps, bool steps32, float* ema_tmp, half_t* ema_h, const AdamTranspose* tr) {
	// parameters [lo, hi): 16-B group accesses need lo % 4 == 0; the transposed MLP copies index parameters from 0
	if (lo % 4 || hi < lo || hi > p.n) throw std::runtime_error("launch_adam_ema_range: lo must be a multiple of 4 and lo <= hi <= n");
	if (tr && tr->n && lo != 0) throw std::runtime_error("launch_adam_ema_range: the transposed copies need the range to start at 0");
	if (hi == lo) return;
	p.n_matrix = p.n_matrix > lo ? std::min(p.n_matrix - lo, hi - lo) : 0u;
	p.n = hi - lo;
	void* st = (uint8_t*)steps + (size_t)lo * (steps32 ? 4 : 2);
	launch_adam_ema(s, p, weights_fp + lo, weights_h + lo, grads + lo, m1 + lo, m2 + lo, st, steps32, ema_tmp + lo, ema_h + lo, nullptr, tr);
}
void launch_add_f32(hipStream_t s, uint32_t n, const float* src, float* dst) {
	if (n) k_add_f32<<<std::min<uint32_t>((n + 255) / 256, 8192), 256, 0, s>>>(n, src, dst);
}
void launch_cast_half(hipStream_t s, uint32_t n, const float* in, half_t* out) { k_cast_half<<<nblk(n), 256, 0, s>>>(n, in, out); }
void launch_transpose_w(hipStream_t s, const TransposeJobs& jobs) { if (jobs.n) k_transpose_w<<<jobs.n, 256, 0, s>>>(jobs, nullptr, nullptr, nullptr, DinPerm{}); }
void launch_transpose_permute(hipStream_t s, const TransposeJobs& jobs, const half_t* d0, half_t* d0p, half_t* d0Tp, const DinPerm& perm) {
	k_transpose_w<<<jobs.n + 1, 256, 0, s>>>(jobs, d0, d0p, d0Tp, perm);
}
void launch_permute_din(hipStream_t s, const half_t* d0, half_t* d0p, half_t* d0Tp, const DinPerm& perm) {
	k_permute_din<<<1, 256, 0, s>>>(d0, d0p, d0Tp, perm);
}
void launch_grid_samples(hipStream_t s, uint32_t n, uint32_t i_begin, uint32_t i_end, uint32_t out_base, uint64_t rng_state, uint64_t rng_inc,
                         uint32_t step, const float* aabb_min, const float* aabb_max, const float* grid_in, float* pos, uint32_t* indices,
                         uint32_t n_cascades, float thresh, const PcgJumpTable& jt) {
	if (i_end <= i_begin) return;
	k_grid_samples<<<nblk(i_end - i_begin), 256, 0, s>>>(n, i_begin, i_end, out_base, rng_state, rng_inc, step, aabb_min[0], aabb_min[1], aabb_min[2],
	                                        aabb_max[0] - aabb_min[0], aabb_max[1] - aabb_min[1], aabb_max[2] - aabb_min[2],
	                                        grid_in, pos, indices, n_cascades, thresh, jt);
}
void launch_splat_max(hipStream_t s, uint32_t n, const uint32_t* indices, const float* density, float* grid_tmp) {
	if (n) k_splat_max<<<nblk(n), 256, 0, s>>>(n, indices, density, grid_tmp);
}
void launch_ema_grid(hipStream_t s, uint32_t n, float decay, float* grid, const float* tmp) { dbg_lds_gate(s); k_ema_grid<<<nblk(n), 256, 0, s>>>(n, decay, grid, tmp); }
void launch_grid_mean(hipStream_t s, const float* grid, float* partial, float* mean) {
	dbg_lds_gate(s);
	k_grid_mean_partial<<<GRID3 / 1024, 256, 0, s>>>(grid, partial);
	dbg_lds_gate(s);
	k_grid_mean_final<<<1, 256, 0, s>>>(partial, GRID3 / 1024, mean);
}
void launch_bitfield(hipStream_t s, const float* grid, uint8_t* bitfield, const float* mean, uint32_t n_cascades, uint32_t* lin) {
	const uint32_t nbytes = GRID3 / 8;
	dbg_lds_gate(s);
	k_grid_to_bitfield<<<nblk(nbytes * NERF_CASCADES), 256, 0, s>>>(nbytes * NERF_CASCADES, nbytes * n_cascades, grid, bitfield, mean);
	dbg_lds_gate(s);
	k_bitfield_pool_all<<<nblk((uint64_t)nbytes * (NERF_CASCADES - 1), 2048), 256, 0, s>>>(nbytes, bitfield, lin);
}
size_t occ_bbox_scratch_floats() { return 6 + 6 * (size_t)OCC_BBOX_BLOCKS; }
void launch_occ_bbox(hipStream_t s, const uint8_t* bitfield, float* scratch) {
	dbg_lds_gate(s);
	k_occ_bbox_partial<<<OCC_BBOX_BLOCKS, 256, 0, s>>>(bitfield, scratch + 6);
	dbg_lds_gate(s);
	k_occ_bbox_final<<<1, 256, 0, s>>>(scratch + 6, OCC_BBOX_BLOCKS, scratch);
}
void launch_ema_mean(hipStream_t s, uint32_t n, float decay, float* grid, const float* tmp, float* partial, float* mean) {
	dbg_lds_gate(s);
	k_ema_mean<<<n / 1024, 256, 0, s>>>(n, decay, grid, tmp, partial);
	dbg_lds_gate(s);
	k_grid_mean_final<<<1, 256, 0, s>>>(partial, GRID3 / 1024, mean);
}

} // namespace neus
