// tcnn's FullyFusedMLP (my_tcnn src/fully_fused_mlp.cu) behind its Identity encoding: the network of tcnn::cpp::
// create_network(n_input_dims, n_output_dims, network) (my_tcnn src/cpp_api.cu:170-172), on v_mfma_f32_32x32x16_f16.
//
// Layout: activations sample-major [n][features] fp16 (the column-major matrices cpp::Module hands its caller), so a
// B fragment (k = feature, column = sample) is one 16-byte load per lane; weights row-major [out][in] fp16 staged in LDS
// per block (transposed when a backward pass multiplies by W^T). One wave computes 32 samples x every output row.
//
// The layer kernel covers every product of the network: the forward (activation applied to the fp16-rounded sum, as
// warp_activation on the half accumulator), the backward deltas and the backward-backward "front"/"back" chains (the
// activation derivative from the stored forward values, warp_activation_backward, common_device.h:174-225), the output
// layer and dL/dinput. Weight gradients dW = D^T X sum over samples with the sample on the MFMA k axis: both operands are
// staged transposed through LDS, per-block fp32 partial rows, summed in a fixed block order by k_mlp_grad_reduce
// (deterministic, where tcnn's split-K fp16 GEMM is not).
#include "kernels.h"
#include <algorithm>
#include <stdexcept>

namespace neus {

namespace {
__device__ __forceinline__ f16v ff_mfma(h8 a, h8 b, f16v c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }
// accumulator register i of lane half h holds row (i & 3) + 8 (i >> 2) + 4 h of the 32-row tile (natural k order)
__device__ __forceinline__ constexpr int ff_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
constexpr float FF_K_ACT = 10.0f;  // common_device.h:66

// warp_activation (common_device.h:68-113) on an fp16 value
__device__ __forceinline__ float ff_act(uint32_t act, float x) {
	switch (act) {
	case FF_RELU: return x > 0.f ? x : 0.f;
	case FF_EXP: return expf(x);
	case FF_SIGMOID: return 1.0f / (1.0f + expf(-x));
	case FF_SQUAREPLUS: { const float y = x * FF_K_ACT; return 0.5f * (y + sqrtf(y * y + 4)) / FF_K_ACT; }
	case FF_SOFTPLUS: return logf(expf(x * FF_K_ACT) + 1.0f) / FF_K_ACT;
	default: return x;
	}
}
// warp_activation_backward (common_device.h:174-225): the derivative factor from the forward's post-activation value y
__device__ __forceinline__ float ff_dact(uint32_t act, float y) {
	switch (act) {
	case FF_RELU: return y > 0.f ? 1.f : 0.f;
	case FF_EXP: return y;
	case FF_SIGMOID: return (float)(half_t)(y * (float)(half_t)(1.0f - y));  // (T)(y * ((T)1 - y)) in half
	case FF_SQUAREPLUS: { const float t = y * FF_K_ACT; return t * t / (t * t + 1); }
	case FF_SOFTPLUS: return 1.0f - expf(-y * FF_K_ACT);
	default: return 1.f;
	}
}
}  // namespace

// Out[s][o] = f(sum_k A[o][k] In[s][k]), o < O, k < K (multiple of 16), A = W [O][K] or (trans) W^T with W [K][O].
//   mode FF_MODE_ACT : f = act on the fp16-rounded sum, fp16 out
//   mode FF_MODE_DACT: f = (fp16 sum) * dact(aux[s][o]) rounded to fp16, fp16 out
//   mode FF_MODE_F32 : float out = (float)(fp16 sum), written for o < o_lim only
__global__ void __launch_bounds__(256) k_ff_layer(FfLayer L) {
	extern __shared__ half_t s_w[];
	const uint32_t Op = (L.O + 31) / 32 * 32, lda = L.K + 8;
	// stage A [Op][K] (+ 8 halves of row padding); rows >= O are zero
	for (uint32_t e = threadIdx.x; e < Op * L.K; e += blockDim.x) {
		const uint32_t o = e / L.K, k = e % L.K;
		half_t v = (half_t)0.f;
		if (o < L.O) v = L.trans ? L.W[(size_t)k * L.O + o] : L.W[(size_t)o * L.K + k];
		s_w[o * lda + k] = v;
	}
	__syncthreads();
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
	const uint32_t MT = Op / 32, KS = L.K / 16;
	for (uint32_t s0 = wave * 32; s0 < L.n; s0 += n_waves * 32) {
		const uint32_t s = s0 + r;
		const bool valid = s < L.n;
		f16v acc[4];
#pragma unroll
		for (int mt = 0; mt < 4; ++mt)
#pragma unroll
			for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;
		for (uint32_t ks = 0; ks < KS; ++ks) {
			h8 b = (h8){0, 0, 0, 0, 0, 0, 0, 0};
			if (valid) b = *(const h8*)(L.in + (size_t)s * L.ldi + 16 * ks + 8 * h);
#pragma unroll
			for (int mt = 0; mt < 4; ++mt) {
				if ((uint32_t)mt >= MT) break;
				const h8 a = *(const h8*)(s_w + (32 * mt + r) * lda + 16 * ks + 8 * h);
				acc[mt] = ff_mfma(a, b, acc[mt]);
			}
		}
		if (!valid) continue;
#pragma unroll
		for (int mt = 0; mt < 4; ++mt) {
			if ((uint32_t)mt >= MT) break;
#pragma unroll
			for (int i = 0; i < 16; ++i) {
				const uint32_t o = 32 * mt + ff_row(i, h);
				if (o >= L.O) continue;
				const float x = (float)(half_t)acc[mt][i];
				if (L.mode == FF_MODE_F32) {
					if (o < L.o_lim) L.out_f[(size_t)s * L.ldo + o] = x * L.out_scale;
				} else if (L.mode == FF_MODE_DACT) {
					const float d = (float)(half_t)ff_dact(L.act, (float)L.aux[(size_t)s * L.ldx + o]);
					L.out[(size_t)s * L.ldo + o] = (half_t)(x * d);
				} else {
					L.out[(size_t)s * L.ldo + o] = (half_t)ff_act(L.act, x);
				}
			}
		}
	}
}

// dW[o][i] (partial over this block's samples) = sum_s D[s][o] X[s][i] -> prow[block][off + o I + i] (fp32)
__global__ void __launch_bounds__(256) k_ff_wgrad(FfWgrad G) {
	extern __shared__ half_t s_t[];
	const uint32_t Op = (G.O + 31) / 32 * 32, Ip = (G.I + 31) / 32 * 32;
	half_t* Dt = s_t;                 // [Op][40]: the chunk's deltas, sample on the row
	half_t* Xt = s_t + Op * 40;       // [Ip][40]
	const uint32_t per = (G.n + gridDim.x - 1) / gridDim.x;
	const uint32_t b0 = blockIdx.x * per, b1 = min(G.n, b0 + per);
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wv = threadIdx.x >> 6;
	const uint32_t TO = Op / 32, TI = Ip / 32, NT = TO * TI;
	f16v acc[4];
#pragma unroll
	for (int t = 0; t < 4; ++t)
#pragma unroll
		for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
	for (uint32_t c0 = b0; c0 < b1; c0 += 32) {
		__syncthreads();
		for (uint32_t e = threadIdx.x; e < 32 * Op; e += blockDim.x) {
			const uint32_t k = e / Op, o = e % Op, s = c0 + k;
			Dt[o * 40 + k] = (s < b1 && o < G.O) ? G.D[(size_t)s * G.ldd + o] : (half_t)0.f;
		}
		for (uint32_t e = threadIdx.x; e < 32 * Ip; e += blockDim.x) {
			const uint32_t k = e / Ip, i = e % Ip, s = c0 + k;
			Xt[i * 40 + k] = (s < b1 && i < G.I) ? G.X[(size_t)s * G.ldx + i] : (half_t)0.f;
		}
		__syncthreads();
#pragma unroll
		for (int t = 0; t < 4; ++t) {
			const uint32_t tile = (uint32_t)wv + 4 * (uint32_t)t;
			if (tile >= NT) break;
			const uint32_t to = tile / TI, ti = tile % TI;
#pragma unroll
			for (int ks = 0; ks < 2; ++ks) {
				const h8 a = *(const h8*)(Dt + (32 * to + r) * 40 + 16 * ks + 8 * h);
				const h8 b = *(const h8*)(Xt + (32 * ti + r) * 40 + 16 * ks + 8 * h);
				acc[t] = ff_mfma(a, b, acc[t]);
			}
		}
	}
	float* prow = G.partial + (size_t)blockIdx.x * G.ld_partial + G.off;
#pragma unroll
	for (int t = 0; t < 4; ++t) {
		const uint32_t tile = (uint32_t)wv + 4 * (uint32_t)t;
		if (tile >= NT) break;
		const uint32_t to = tile / TI, ti = tile % TI;
#pragma unroll
		for (int i = 0; i < 16; ++i) {
			const uint32_t o = 32 * to + ff_row(i, h), c = 32 * ti + r;
			if (o < G.O && c < G.I) prow[(size_t)o * G.I + c] = acc[t][i];
		}
	}
}

// Identity encoding (identity.h:44-70): X0[s][k] = (half)(in[s][k] scale + offset) for k < n_in, 1 for the padding
// k < ld (the bias input of tcnn's padded encodings); mode 1: the backward-backward front, dL_ddLdinput scaled, padding 0
__global__ void k_ff_input(uint32_t n, uint32_t n_in, uint32_t ld, const float* __restrict__ in, float scale, float offset, half_t* __restrict__ x,
                           uint32_t grad) {
	for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < (uint64_t)n * ld; e += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t s = e / ld;
		const uint32_t k = (uint32_t)(e % ld);
		float v = grad ? 0.f : 1.f;
		if (k < n_in) v = grad ? in[s * n_in + k] * scale : in[s * n_in + k] * scale + offset;
		x[e] = (half_t)v;
	}
}
// the output activation's backward on dL/doutput (fully_fused_mlp.cu:985-1000): D[s][o] = dL[s][o] dact(out[s][o])
__global__ void k_ff_out_delta(uint32_t n, uint32_t ld, uint32_t act, const half_t* __restrict__ dL, const half_t* __restrict__ out, half_t* __restrict__ d) {
	for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < (uint64_t)n * ld; e += (uint64_t)gridDim.x * blockDim.x) {
		const float g = (float)dL[e];
		d[e] = act == FF_NONE ? dL[e] : (half_t)(g * (float)(half_t)ff_dact(act, (float)out[e]));
	}
}

static uint32_t ff_blocks(uint64_t n, uint32_t per, uint32_t cap) { return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + per - 1) / per, cap)); }

void launch_ff_layer(hipStream_t s, const FfLayer& L) {
	if (L.K % 16 || L.K == 0 || L.O == 0 || L.O > 128) throw std::runtime_error("ff layer: K must be a multiple of 16, 1 <= O <= 128");
	const size_t smem = (size_t)((L.O + 31) / 32 * 32) * (L.K + 8) * sizeof(half_t);
	k_ff_layer<<<ff_blocks(L.n, 128, 1024), 256, smem, s>>>(L);
}
uint32_t ff_wgrad_blocks(uint32_t n) { return ff_blocks(n, 1024, 512); }
void launch_ff_wgrad(hipStream_t s, const FfWgrad& G) {
	if (G.O == 0 || G.I == 0 || G.O > 128 || G.I > 128) throw std::runtime_error("ff wgrad: 1..128 rows and columns");
	const size_t smem = (size_t)((G.O + 31) / 32 * 32 + (G.I + 31) / 32 * 32) * 40 * sizeof(half_t);
	k_ff_wgrad<<<ff_wgrad_blocks(G.n), 256, smem, s>>>(G);
}
void launch_ff_input(hipStream_t s, uint32_t n, uint32_t n_in, uint32_t ld, const float* in, float scale, float offset, half_t* x, bool grad) {
	k_ff_input<<<ff_blocks((uint64_t)n * ld, 256, 4096), 256, 0, s>>>(n, n_in, ld, in, scale, offset, x, grad ? 1u : 0u);
}
void launch_ff_out_delta(hipStream_t s, uint32_t n, uint32_t ld, uint32_t act, const half_t* dL, const half_t* out, half_t* d) {
	k_ff_out_delta<<<ff_blocks((uint64_t)n * ld, 256, 4096), 256, 0, s>>>(n, ld, act, dL, out, d);
}

}  // namespace neus
