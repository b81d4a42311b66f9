// NeuS2 SDF + colour MLPs on gfx950 MFMA (v_mfma_f32_32x32x16_f16, fp16 in / fp32 accumulate).
//
// Formulation: every layer is computed TRANSPOSED, Y[neuron][sample] = W[neuron][k] X[k][sample],
// with 32 samples on the MFMA column (lane & 31) and the neurons in the accumulator registers.
// A 32x32 accumulator tile is then directly the B operand of the next layer (the contraction
// runs over its rows), so activations never leave registers between layers. The k order of a
// fragment built from an accumulator is permuted:   element j of lane half h <-> row pi(j,h),
//      pi(j,h) = 8*(j>>2) + 4*h + (j&3)      (16-row k-step)
// and every A (weight) fragment is loaded with the same permutation (loadA), as is every B
// fragment built from memory, so all products are consistent.
//
// Weights are staged once per block into LDS (row stride padded by 8 halves against bank
// conflicts) and every A fragment is read from there: the register file holds activations only,
// which keeps several waves per SIMD resident to hide the gather / HBM latency.
//
// Reference semantics (per sample):
//   density MLP  fully_fused_mlp.cu:678-812 (1 hidden ReLU layer, linear 16-wide output)
//   grad SDF     nerf_network.h:228-253 + kernel_grid_backward_input (grid.h:803-830)
//   SH deg 4     spherical_harmonics.h:47-100
//   rgb MLP      fully_fused_mlp.cu (2 hidden ReLU layers) ; output packing nerf_network.h:287-324
//   backward     nerf_network.h:330-601, FullyFusedMLP::backward_backward_input (:1088-1198)
// Storage rounding points (fp16) follow the reference: hidden activations, deltas, the
// density output, dSDF/d(input), the network output and dL/doutput.
#include <hip/hip_ext.h>
#include "kernels.h"
#include "scan_lookback.h"
#include "grid_common.h"
#include "occ_common.h"
// the loss's alpha terms (fused inference epilogue) keep the march / loss files' arithmetic: no FMA contraction, so they
// are bitwise k_loss_alpha's (march.hip) and the oracle's
#pragma clang fp contract(off)
#include "march_common.h"
#pragma clang fp contract(fast)
#include <algorithm>

namespace neus {

__device__ __forceinline__ f16v mfma(h8 a, h8 b, f16v c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ constexpr int pi_row(int j, int h) { return 8 * (j >> 2) + 4 * h + (j & 3); }
// accumulator register i of lane half h holds row acc_row(i,h) of the 32-row tile
__device__ __forceinline__ constexpr int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// A weight matrix [rows][ld] (fp16, row-major) in LDS or global memory.
struct MatRef { const half_t* p; uint32_t ld; };

__device__ __forceinline__ h8 loadA(MatRef W, uint32_t M, uint32_t row, uint32_t kbase, uint32_t h) {
	h8 a;
	if (row < M) {
		const half_t* p = W.p + (size_t)row * W.ld + kbase + 4 * h;
		const h4 lo = *(const h4*)p;
		const h4 hi = *(const h4*)(p + 8);
		a = (h8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
	} else {
		a = (h8){0, 0, 0, 0, 0, 0, 0, 0};
	}
	return a;
}
// B fragment (k-step s of an accumulator tile)
__device__ __forceinline__ h8 accB(const f16v& acc, int s) {
	h8 b;
#pragma unroll
	for (int j = 0; j < 8; ++j) b[j] = (half_t)acc[8 * s + j];
	return b;
}
__device__ __forceinline__ h8 shfl_xor_h8(h8 v, int m) {
	union { h8 h; int i[4]; } u;
	u.h = v;
#pragma unroll
	for (int k = 0; k < 4; ++k) u.i[k] = __shfl_xor(u.i[k], m);
	return u.h;
}
__device__ __forceinline__ f16v zero16() { f16v z; for (int i = 0; i < 16; ++i) z[i] = 0.f; return z; }
__device__ __forceinline__ f16v relu16(f16v a) { for (int i = 0; i < 16; ++i) a[i] = a[i] > 0.f ? a[i] : 0.f; return a; }
// round an accumulator tile to fp16 storage precision
__device__ __forceinline__ f16v rh16(f16v a) { for (int i = 0; i < 16; ++i) a[i] = rh(a[i]); return a; }

template <int L> struct Dims {
	static constexpr int DIN = ((3 + 2 * L) + 15) / 16 * 16;
	static constexpr int DKS = DIN / 16;           // density-input k-steps
	static constexpr int DMT = (DIN + 31) / 32;    // M tiles of a DIN-row result
	static constexpr int NF = 2 * L;               // encoding features
};

// ---------------------------------------------------------------- LDS weight staging
// copy a [rows][cols] fp16 matrix (cols % 8 == 0) into LDS with row stride cols + 8
__device__ __forceinline__ void stage_mat(half_t* dst, const half_t* __restrict__ src, uint32_t rows, uint32_t cols) {
	const uint32_t cv = cols / 8, n = rows * cv;
	for (uint32_t e = threadIdx.x; e < n; e += blockDim.x) {
		const uint32_t r = e / cv, c = (e % cv) * 8;
		*(h8*)(dst + (size_t)r * (cols + 8) + c) = *(const h8*)(src + (size_t)r * cols + c);
	}
}

// Re-derives a weight view from an offset the compiler cannot see through, once per loop
// iteration: without it the LDS fragment loads are loop-invariant and get hoisted into (and
// exhaust) the register file.
__device__ __forceinline__ MatRef rebase(MatRef m, uint32_t z) { return {m.p + z, m.ld}; }
__device__ __forceinline__ uint32_t opaque_zero() { uint32_t z = 0; asm volatile("" : "+v"(z)); return z; }

// Weight set of the forward pass. For the fused kernels d0 / d0T are the din-PERMUTED copies
// (MlpPtrs::d0p / d0Tp, see din_logical), for the training kernel the logical ones.
struct FwdW {
	MatRef d0, d1, d0T, r0, r1, r2;
	__device__ __forceinline__ FwdW at(uint32_t z) const { return {rebase(d0, z), rebase(d1, z), rebase(d0T, z), rebase(r0, z), rebase(r1, z), rebase(r2, z)}; }
};
template <int L, int W> struct FwdSmem {
	static constexpr int DIN = Dims<L>::DIN;
	static constexpr int D0 = 0, D1 = D0 + W * (DIN + 8), D0T = D1 + 16 * (W + 8), R0 = D0T + DIN * (W + 8);
	static constexpr int R1 = R0 + W * (48 + 8), R2 = R1 + W * (W + 8), END = R2 + 16 * (W + 8);
};
template <int L, int W>
__device__ __forceinline__ FwdW stage_fwd(half_t* sm, const half_t* d0, const half_t* d0T, const MlpPtrs& w) {
	using S = FwdSmem<L, W>;
	constexpr int DIN = Dims<L>::DIN;
	stage_mat(sm + S::D0, d0, W, DIN);
	stage_mat(sm + S::D1, w.d1, 16, W);
	stage_mat(sm + S::D0T, d0T, DIN, W);
	stage_mat(sm + S::R0, w.r0, W, 48);
	stage_mat(sm + S::R1, w.r1, W, W);
	stage_mat(sm + S::R2, w.r2, 16, W);
	FwdW f;
	f.d0 = {sm + S::D0, DIN + 8}; f.d1 = {sm + S::D1, W + 8}; f.d0T = {sm + S::D0T, W + 8};
	f.r0 = {sm + S::R0, 48 + 8}; f.r1 = {sm + S::R1, W + 8}; f.r2 = {sm + S::R2, W + 8};
	return f;
}

// ---------------------------------------------------------------- fused encode: din slot layout
// In the fused kernels each sample is held by two lanes (r, h = 0/1). Lane half h evaluates the
// hash-grid levels l = 2m + h (m = 0..M0-1) so both halves run the same instruction stream, and
// owns the density-input slots q = 0..DIN/2-1 of its fragments (physical row 16(q>>3)+pi(q&7,h)):
//   h = 0 : q 0..2 = x - 0.5, then features of levels 0, 2, 4, ...
//   h = 1 : features of levels 1, 3, 5, ...
// If h = 0 has one feature too many (L = 14: 3 + 14 > 16), its last feature moves to h = 1's
// next free slot through one cross-half shuffle. The first layer's weight columns (and W0^T's
// rows) are permuted on the host to this physical order (din_logical), so the product is the
// reference's W0 . din.
// Per-half select of two register values. Written on the bits: `h ? a[i] : a[j]` over a register
// array is otherwise turned into a dynamically indexed array (a 16-way compare/select chain).
__device__ __forceinline__ float hsel(int h, float v1, float v0) {
	const uint32_t m = 0u - (uint32_t)h;
	return __uint_as_float((__float_as_uint(v1) & m) | (__float_as_uint(v0) & ~m));
}

// Symmetric slot layout: slots 3.. hold the lane's own level features in the same order on both
// halves (feature k of the lane's level list: level 2(k/2)+h, feature k%2), so all but the first three
// slots need no per-half select. Slots 0..2 are xyz on h = 0; on h = 1 they take the features that do
// not fit (the lane's own first, then h = 0's, moved over by one cross-half shuffle), then zeros.
NEUS_HD int din_logical(int L, int h, int q) {
	const int DIN = ((3 + 2 * L) + 15) / 16 * 16, HALF = DIN / 2, FS = HALF - 3;
	const int M0 = (L + 1) / 2, M1 = L / 2;
	const int OV0 = 2 * M0 > FS ? 2 * M0 - FS : 0, OV1 = 2 * M1 > FS ? 2 * M1 - FS : 0;
	if (q >= HALF) return -1;
	if (q >= 3) {
		const int k = q - 3, M = h ? M1 : M0;
		if (k >= 2 * M || k >= FS) return -1;
		return 3 + 2 * (2 * (k / 2) + h) + (k % 2);
	}
	if (h == 0) return q;
	if (q < OV1) { const int k = FS + q; return 3 + 2 * (2 * (k / 2) + 1) + (k % 2); }
	if (q < OV1 + OV0) { const int k = FS + q - OV1; return 3 + 2 * (2 * (k / 2)) + (k % 2); }
	return -1;
}
NEUS_HD int din_physical_row(int h, int q) { return 16 * (q >> 3) + 8 * ((q & 7) >> 2) + 4 * h + (q & 3); }

template <int L> struct Fused {
	static constexpr int DIN = Dims<L>::DIN, HALF = DIN / 2, FS = HALF - 3;
	static constexpr int M0 = (L + 1) / 2, M1 = L / 2;
	static constexpr int OV0 = 2 * M0 > FS ? 2 * M0 - FS : 0, OV1 = 2 * M1 > FS ? 2 * M1 - FS : 0;
	static_assert(OV0 + OV1 <= 3, "din slot layout");
};

// Evaluates this lane's levels for position x: features ev[m] (level 2m+h) and, if DYDX, dy/dx.
// Same arithmetic as grid_common.h (bit-identical features / dy/dx), restructured for issue count and
// latency:
//  * level parameters are selected per lane half without branches; inactive levels (beyond
//    valid_level, or the missing odd level) are computed on valid addresses and zeroed by select;
//  * corner indices share their per-axis terms (dense: x + y res + z res^2, wrapped as the reference's
//    `% hashmap_size`; hashed: the xor hash masked by the power-of-two table size) and are formed as
//    32-bit entry offsets from the uniform table base (scalar-base loads, no 64-bit address math);
//  * software-pipelined: level m+1's 8 gathers are in flight while level m is interpolated;
//  * both features go through packed fp32 (v_pk_mul/v_pk_fma) and packed fp16 adds; the fp16 feature
//    accumulation result[f] += (half)(w * v) and the fmaf dy/dx terms are unchanged.
typedef float f2v __attribute__((ext_vector_type(2)));
struct LevelAddr { uint32_t e[8]; float f[3]; float sc; bool act; };
// Per-level constants {scale bits, res, table offset, table size}, staged in LDS once per block and
// read per lane by level index (a per-lane select between two levels' kernel-argument values would
// need every constant materialised in VGPRs for the whole kernel).
struct LevelSmem { uint4 p[16]; };
__device__ __forceinline__ void stage_levels(LevelSmem& sl, const GridLevels& gl, uint32_t L) {
	for (uint32_t t = threadIdx.x; t < L; t += blockDim.x)
		sl.p[t] = make_uint4(__float_as_uint(gl.scale[t]), gl.res[t], gl.offset[t], gl.offset[t + 1] - gl.offset[t]);
}
template <int L>
__device__ __forceinline__ void level_addr(const LevelSmem& sl, uint32_t dense_bits, uint32_t valid_level, const float x[3], int h, int m, LevelAddr& A) {
	const int l0 = 2 * m, l1 = 2 * m + 1 < L ? 2 * m + 1 : 2 * m;
	// opaque lane half: keeps the level-constant reads inside the loop body
	h = h | (int)opaque_zero();
	const uint32_t l = h ? (uint32_t)l1 : (uint32_t)l0;
	A.act = (h ? (2 * m + 1 < L) : true) && l <= valid_level;
	const uint4 P = sl.p[l];
	A.sc = __uint_as_float(P.x);
	const uint32_t res = P.y, o0 = P.z, hs = P.w;
	const bool dense = (dense_bits >> l) & 1u;
	uint32_t gp[3];
#pragma unroll
	for (int d = 0; d < 3; ++d) {
		// pos_fract (common_device.h:404-434): one FFMA as nvcc emits `input * scale + 0.5f`
		const float p = __builtin_fmaf(x[d], A.sc, 0.5f);
		const float fl = floorf(p);
		gp[d] = (uint32_t)(int)fl;
		A.f[d] = p - fl;
	}
	// The pair's two levels are both dense or both hashed for most pairs (dense_bits is a prefix): a wave-uniform
	// branch then computes only that index form; a mixed pair computes both, merged by mask (a per-lane select
	// here is turned into divergent branches).
	const uint32_t pair_dense = (dense_bits >> l0) & 1u, pair_dense1 = (dense_bits >> l1) & 1u;
	uint32_t yz[4];
	if (pair_dense & pair_dense1) {
#pragma unroll
		for (int k = 0; k < 4; ++k) yz[k] = (gp[1] + (k & 1)) * res + (gp[2] + (k >> 1)) * (res * res);
	} else if (!(pair_dense | pair_dense1)) {
#pragma unroll
		for (int k = 0; k < 4; ++k) yz[k] = ((gp[1] + (k & 1)) * 2654435761u) ^ ((gp[2] + (k >> 1)) * 805459861u);
#pragma unroll
		for (int c = 0; c < 8; ++c) A.e[c] = o0 + (((gp[0] + (c & 1)) ^ yz[c >> 1]) & (hs - 1u));
		return;
	} else {
		const uint32_t dm = 0u - (uint32_t)dense;
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint32_t yy = gp[1] + (k & 1), zz = gp[2] + (k >> 1);
			yz[k] = ((yy * res + zz * (res * res)) & dm) | (((yy * 2654435761u) ^ (zz * 805459861u)) & ~dm);
		}
	}
	const uint32_t dm = 0u - (uint32_t)dense;
	// A position inside the unit cube has every cell coordinate <= res - 1, so a dense corner index is below
	// 2 hs and one conditional subtract is the reference's `% hashmap_size`. Positions outside it (a sample moved
	// by the DeltaNetwork, a grid point beyond the aabb; negative cells wrap to huge unsigned values) take the
	// true modulo, on the rare lanes that need it.
	const bool outside = dense && (gp[0] >= res || gp[1] >= res || gp[2] >= res);
	if (__builtin_expect(outside, 0)) {
#pragma unroll
		for (int c = 0; c < 8; ++c) A.e[c] = o0 + (gp[0] + (c & 1) + yz[c >> 1]) % hs;
	} else {
#pragma unroll
		for (int c = 0; c < 8; ++c) {
			const uint32_t xx = gp[0] + (c & 1), k = c >> 1;
			const uint32_t ed = xx + yz[k];
			const uint32_t ew = min(ed, ed - hs);  // ed < 2 hs: the reference's % hashmap_size
			A.e[c] = o0 + ((ew & dm) | ((xx ^ yz[k]) & (hs - 1u) & ~dm));
		}
	}
}
#ifndef NEUS_GATHER
#define NEUS_GATHER 0
#endif
__device__ __forceinline__ void level_gather(const half_t* __restrict__ grid, const LevelAddr& A, uint32_t v[8]) {
	const char* base = (const char*)grid;
#if NEUS_GATHER == 0
#pragma unroll
	for (int c = 0; c < 8; ++c) v[c] = *(const uint32_t*)(base + (A.e[c] << 2));
#elif NEUS_GATHER == 1
	// x-neighbour corners (c, c+1) share an aligned 8-B entry pair when e1 == e0 ^ 1 (a hashed level with even x, a
	// dense level with even e0): one load for both; the other lanes load e1 by itself.
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const uint32_t e0 = A.e[2 * k], e1 = A.e[2 * k + 1];
		const uint2 w = *(const uint2*)(base + ((e0 & ~1u) << 2));
		const bool odd = e0 & 1u;
		v[2 * k] = odd ? w.y : w.x;
		uint32_t o = odd ? w.x : w.y;
		if ((e0 ^ e1) != 1u) o = *(const uint32_t*)(base + (e1 << 2));
		v[2 * k + 1] = o;
	}
#else
	// aligned 16-B entry quad holding e0; e1 from the same quad when it is there
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const uint32_t e0 = A.e[2 * k], e1 = A.e[2 * k + 1];
		const uint4 w = *(const uint4*)(base + ((e0 & ~3u) << 2));
		const uint32_t s0 = e0 & 3u, s1 = e1 & 3u;
		v[2 * k] = s0 & 2u ? (s0 & 1u ? w.w : w.z) : (s0 & 1u ? w.y : w.x);
		uint32_t o = s1 & 2u ? (s1 & 1u ? w.w : w.z) : (s1 & 1u ? w.y : w.x);
		if ((e0 ^ e1) > 3u) o = *(const uint32_t*)(base + (e1 << 2));
		v[2 * k + 1] = o;
	}
#endif
}
__device__ __forceinline__ f2v h2f(uint32_t u) {
	h2 hv = __builtin_bit_cast(h2, u);
	return (f2v){(float)hv[0], (float)hv[1]};
}
template <bool DYDX>
__device__ __forceinline__ void level_interp(const LevelAddr& A, const uint32_t v[8], h2& ev, float dy[2][3]) {
	const float wx[2] = {1.f - A.f[0], A.f[0]}, wy[2] = {1.f - A.f[1], A.f[1]}, wz[2] = {1.f - A.f[2], A.f[2]};
	f2v vf[8];
#pragma unroll
	for (int c = 0; c < 8; ++c) vf[c] = h2f(v[c]);
	// weights ((1 * wx) * wy) * wz, as the reference's loop
	h2 r = (h2){(half_t)0.f, (half_t)0.f};
#pragma unroll
	for (int c = 0; c < 8; ++c) {
		const float w = (wx[c & 1] * wy[(c >> 1) & 1]) * wz[c >> 2];
		const f2v t = (f2v){w, w} * vf[c];
		r = r + (h2){(half_t)t[0], (half_t)t[1]};
	}
	ev = A.act ? r : (h2){(half_t)0.f, (half_t)0.f};
	if (DYDX) {
		// weight = (scale * w_a) * w_b over the two non-gradient dims in increasing order
		const float sx[2] = {A.sc * wx[0], A.sc * wx[1]}, sy[2] = {A.sc * wy[0], A.sc * wy[1]};
		f2v g[3] = {(f2v){0.f, 0.f}, (f2v){0.f, 0.f}, (f2v){0.f, 0.f}};
#pragma unroll
		for (int gd = 0; gd < 3; ++gd)
#pragma unroll
			for (int idx = 0; idx < 4; ++idx) {
				const int b0 = idx & 1, b1 = (idx >> 1) & 1;
				float w;
				uint32_t cl;
				if (gd == 0) { w = sy[b0] * wz[b1]; cl = (b0 << 1) | (b1 << 2); }
				else if (gd == 1) { w = sx[b0] * wz[b1]; cl = b0 | (b1 << 2); }
				else { w = sx[b0] * wy[b1]; cl = b0 | (b1 << 1); }
				const uint32_t cr = cl | (1u << gd);
				g[gd] = __builtin_elementwise_fma((f2v){w, w}, vf[cr] - vf[cl], g[gd]);
			}
#pragma unroll
		for (int q = 0; q < 2; ++q)
#pragma unroll
			for (int d = 0; d < 3; ++d) {
				dy[q][d] = A.act ? g[d][q] : 0.f;
				// materialise here: sunk to its use in the MLP, the dy/dx arithmetic would keep all
				// levels' corner values live instead of 6 floats per level
				asm volatile("" : "+v"(dy[q][d]));
			}
	}
}
template <int L, bool DYDX, bool ALL = false>
__device__ __forceinline__ void fused_levels(const LevelSmem& sl, uint32_t dense_bits, uint32_t valid_level, const half_t* __restrict__ grid,
                                             const float x[3], int h, h2 ev[], float dy[][2][3]) {
	constexpr int M0 = Fused<L>::M0;
	LevelAddr A[2];
	uint32_t v[2][8];
	// Level pair m (levels 2m, 2m+1) is skipped when both are beyond valid_level (kernel-uniform branch):
	// the reference outputs zeros there without a lookup (grid.h:198-215), so no gather is issued.
	// ALL (every level active, the caller checked): no per-level branch, and a scheduling barrier between level
	// m+1's gathers and level m's interpolation. The branches split the unrolled loop into blocks, and the gathers were
	// then sunk to their use after the previous level's interpolation: one exposed memory round trip per level.
	level_addr<L>(sl, dense_bits, valid_level, x, h, 0, A[0]);
	level_gather(grid, A[0], v[0]);
#pragma unroll
	for (int m = 0; m < M0; ++m) {
		const int cur = m & 1, nxt = cur ^ 1;
		if (m + 1 < M0 && (ALL || (uint32_t)(2 * (m + 1)) <= valid_level)) {
			level_addr<L>(sl, dense_bits, valid_level, x, h, m + 1, A[nxt]);
			level_gather(grid, A[nxt], v[nxt]);
		}
		if (ALL) __builtin_amdgcn_sched_barrier(0);
		if (!ALL && m > 0 && (uint32_t)(2 * m) > valid_level) {
			ev[m] = (h2){(half_t)0.f, (half_t)0.f};
			if (DYDX)
#pragma unroll
				for (int q = 0; q < 2; ++q)
#pragma unroll
					for (int d = 0; d < 3; ++d) dy[m][q][d] = 0.f;
			continue;
		}
		float dtmp[2][3];
		level_interp<DYDX>(A[cur], v[cur], ev[m], DYDX ? dy[m] : dtmp);
	}
}

// Overflow features (see din_logical): ov[j] on h = 1 is slot j (< 3): its own features k >= FS
// first, then those of h = 0 (received by a cross-half shuffle).
template <int L>
__device__ __forceinline__ void overflow_values(int h, const h2 ev[], float ov[3]) {
	using F = Fused<L>;
#pragma unroll
	for (int j = 0; j < 3; ++j) ov[j] = 0.f;
#pragma unroll
	for (int j = 0; j < F::OV1; ++j) { const int k = F::FS + j; ov[j] = (float)ev[k / 2][k % 2]; }
#pragma unroll
	for (int j = 0; j < F::OV0; ++j) {
		const int k = F::FS + j;
		ov[F::OV1 + j] = __shfl_xor((float)ev[k / 2][k % 2], 32);
	}
}
template <int L>
__device__ __forceinline__ void overflow_dydx(const float dy[][2][3], float ovd[3][3]) {
	using F = Fused<L>;
#pragma unroll
	for (int j = 0; j < 3; ++j)
#pragma unroll
		for (int d = 0; d < 3; ++d) ovd[j][d] = 0.f;
#pragma unroll
	for (int j = 0; j < F::OV1; ++j) { const int k = F::FS + j;
#pragma unroll
		for (int d = 0; d < 3; ++d) ovd[j][d] = dy[k / 2][k % 2][d]; }
#pragma unroll
	for (int j = 0; j < F::OV0; ++j) { const int k = F::FS + j;
#pragma unroll
		for (int d = 0; d < 3; ++d) ovd[F::OV1 + j][d] = __shfl_xor(dy[k / 2][k % 2][d], 32); }
}
// Value of slot q on this lane (indices compile-time; a per-half select only where the halves differ)
template <int L>
__device__ __forceinline__ float slot_value(int q, int h, const float xm[3], const h2 ev[], const float ov[3]) {
	using F = Fused<L>;
	if (q < 3) return h ? ov[q] : xm[q];
	const int k = q - 3;
	if (k >= F::FS) return 0.f;
	const bool in0 = k < 2 * F::M0, in1 = k < 2 * F::M1;
	const float v = in0 ? (float)ev[k / 2][k % 2] : 0.f;
	if (in0 == in1) return v;
	return h ? 0.f : v;
}
// d(slot q)/dx_d on this lane (0 for pads; the xyz slots are the identity, handled by the caller)
template <int L>
__device__ __forceinline__ float slot_dydx(int q, int h, int d, const float dy[][2][3], const float ovd[3][3]) {
	using F = Fused<L>;
	if (q < 3) return h ? ovd[q][d] : 0.f;
	const int k = q - 3;
	if (k >= F::FS) return 0.f;
	const bool in0 = k < 2 * F::M0, in1 = k < 2 * F::M1;
	const float v = in0 ? dy[k / 2][k % 2][d] : 0.f;
	if (in0 == in1) return v;
	return h ? 0.f : v;
}

// fp16 B fragment (k-step s) of an accumulator tile, optionally through ReLU: (half)max(acc, 0) is the
// reference's fp16 storage of the post-activation value. The ReLU runs after the packed conversion as a packed
// fp16 max with 0 (rounding is monotone, so the values are those of rounding max(acc, 0)): one op per 2 values
// instead of an fp32 max per value plus the IEEE-mode quieting max the compiler puts before it (MFMA results are
// not known canonical; conversion results are). Non-finite inputs differ from the reference: its ReLU is x * (x > 0)
// (my_tcnn common_device.h:74, warp_activation), NaN for NaN and -inf, while the max gives 0 for both; a diverged
// run is still caught by the non-finite loss check, which sees the other non-finite outputs.
typedef _Float16 hh2v __attribute__((ext_vector_type(2)));
template <bool RELU>
__device__ __forceinline__ h8 frag(const f16v& acc, int s) {
	h8 b;
#pragma unroll
	for (int j = 0; j < 8; j += 2) {
		hh2v p = __builtin_convertvector((f2v){acc[8 * s + j], acc[8 * s + j + 1]}, hh2v);
		if (RELU) p = __builtin_elementwise_max(p, (hh2v)0);
		b[j] = p[0]; b[j + 1] = p[1];
	}
	return b;
}

__device__ __forceinline__ void sh16(const float wd[3], float out[16]) {
	const float x = wd[0] * 2.f - 1.f, y = wd[1] * 2.f - 1.f, z = wd[2] * 2.f - 1.f;
	const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
	out[0] = 0.28209479177387814f;
	out[1] = -0.48860251190291987f * y;
	out[2] = 0.48860251190291987f * z;
	out[3] = -0.48860251190291987f * x;
	out[4] = 1.0925484305920792f * xy;
	out[5] = -1.0925484305920792f * yz;
	out[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
	out[7] = -1.0925484305920792f * xz;
	out[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
	out[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
	out[10] = 2.8906114426405538f * xy * z;
	out[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
	out[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
	out[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
	out[14] = 1.4453057213202769f * z * (x2 - y2);
	out[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
}

// rgb MLP input fragments (ks0 = density output, ks1 = SH, ks2 = [xyz, grad sdf, 0...]) and the
// three rgb layers; returns the fp16-rounded output tile.
template <int W>
__device__ __forceinline__ f16v rgb_forward(const FwdW& w, const f16v& D1, const float x[3], const float wd[3], const float grad[3],
                                            int r, int h, h8 rinB[3], f16v* H1, f16v* H2) {
	constexpr int MT = (W + 31) / 32, HKS = W / 16;
	rinB[0] = accB(D1, 0);
	{
		float sh[16]; sh16(wd, sh);
#pragma unroll
		for (int j = 0; j < 8; ++j) rinB[1][j] = (half_t)hsel(h, sh[pi_row(j, 1)], sh[pi_row(j, 0)]);
		float r32[16];
#pragma unroll
		for (int k = 0; k < 16; ++k) r32[k] = 0.f;
		r32[0] = x[0]; r32[1] = x[1]; r32[2] = x[2];
		r32[3] = grad[0]; r32[4] = grad[1]; r32[5] = grad[2];
#pragma unroll
		for (int j = 0; j < 8; ++j) rinB[2][j] = (half_t)hsel(h, r32[pi_row(j, 1)], r32[pi_row(j, 0)]);
	}
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < 3; ++ks) acc = mfma(loadA(w.r0, W, 32 * mt + r, 16 * ks, h), rinB[ks], acc);
		H1[mt] = rh16(relu16(acc));
	}
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.r1, W, 32 * mt + r, 16 * ks, h), accB(H1[ks >> 1], ks & 1), acc);
		H2[mt] = rh16(relu16(acc));
	}
	f16v acc = zero16();
#pragma unroll
	for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.r2, 16, r, 16 * ks, h), accB(H2[ks >> 1], ks & 1), acc);
	return rh16(acc);
}

// rgb input fragments and the two hidden layers only (training: the output layer is not needed)
template <int W>
__device__ __forceinline__ void rgb_hidden(const FwdW& w, const f16v& D1, const float x[3], const float wd[3], const float grad[3],
                                           int r, int h, h8 rinB[3], f16v* H1, f16v* H2) {
	constexpr int MT = (W + 31) / 32, HKS = W / 16;
	rinB[0] = accB(D1, 0);
	{
		float sh[16]; sh16(wd, sh);
#pragma unroll
		for (int j = 0; j < 8; ++j) rinB[1][j] = (half_t)hsel(h, sh[pi_row(j, 1)], sh[pi_row(j, 0)]);
		float r32[16];
#pragma unroll
		for (int k = 0; k < 16; ++k) r32[k] = 0.f;
		r32[0] = x[0]; r32[1] = x[1]; r32[2] = x[2];
		r32[3] = grad[0]; r32[4] = grad[1]; r32[5] = grad[2];
#pragma unroll
		for (int j = 0; j < 8; ++j) rinB[2][j] = (half_t)hsel(h, r32[pi_row(j, 1)], r32[pi_row(j, 0)]);
	}
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < 3; ++ks) acc = mfma(loadA(w.r0, W, 32 * mt + r, 16 * ks, h), rinB[ks], acc);
		H1[mt] = rh16(relu16(acc));
	}
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.r1, W, 32 * mt + r, 16 * ks, h), accB(H1[ks >> 1], ks & 1), acc);
		H2[mt] = rh16(relu16(acc));
	}
}

// density layer 0 (+ReLU), layer 1 (16 outputs), G_h = relu'(H0) . W1d[0], G_in = W0d^T G_h
template <int L, int W>
__device__ __forceinline__ void density_forward(const FwdW& w, const h8* dinB, int r, int h, f16v* H0, f16v& D1, h8* GhB, f16v* Gi) {
	constexpr int DIN = Dims<L>::DIN, DKS = Dims<L>::DKS, DMT = Dims<L>::DMT, MT = (W + 31) / 32, HKS = W / 16;
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < DKS; ++ks) acc = mfma(loadA(w.d0, W, 32 * mt + r, 16 * ks, h), dinB[ks], acc);
		H0[mt] = rh16(relu16(acc));
	}
	{
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.d1, 16, r, 16 * ks, h), accB(H0[ks >> 1], ks & 1), acc);
		D1 = rh16(acc);
	}
	// row 0 of W1d loaded in the same (pi) order as the H0 fragments
#pragma unroll
	for (int ks = 0; ks < HKS; ++ks) {
		const h8 w1row = loadA(w.d1, 16, 0, 16 * ks, h);
		const f16v& hh = H0[ks >> 1];
		h8 g;
#pragma unroll
		for (int j = 0; j < 8; ++j) g[j] = hh[8 * (ks & 1) + j] > 0.f ? w1row[j] : (half_t)0.f;
		GhB[ks] = g;
	}
#pragma unroll
	for (int mt = 0; mt < DMT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.d0T, DIN, 32 * mt + r, 16 * ks, h), GhB[ks], acc);
		Gi[mt] = rh16(acc);
	}
}

// The same two forwards with the fp16-stored activations held as B fragments (half the registers of fp32
// tiles; the training kernels run at one wave per SIMD, so registers set their latency hiding). Fragment k of
// tile mt holds the tile's registers 8k .. 8k+7, i.e. rows 16 (2 mt + k) + pi_row(j, h): exactly the k-step
// 2 mt + k operand of the next layer and the rows store_frag writes. Values are bit-identical to rounding the
// fp32 tiles (frag: (half)relu(acc) == (half)rh(relu(acc))).
template <int L, int W>
__device__ __forceinline__ void density_forward_frag(const FwdW& w, const h8* dinB, int r, int h, h8* H0B, h8& D1B, h8* GhB, f16v* Gi) {
	constexpr int DIN = Dims<L>::DIN, DKS = Dims<L>::DKS, DMT = Dims<L>::DMT, MT = (W + 31) / 32, HKS = W / 16;
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < DKS; ++ks) acc = mfma(loadA(w.d0, W, 32 * mt + r, 16 * ks, h), dinB[ks], acc);
		H0B[2 * mt] = frag<true>(acc, 0);
		if (2 * mt + 1 < HKS) H0B[2 * mt + 1] = frag<true>(acc, 1);  // W = 16: one 16-row half
	}
	{
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.d1, 16, r, 16 * ks, h), H0B[ks], acc);
		D1B = frag<false>(acc, 0);
	}
#pragma unroll
	for (int ks = 0; ks < HKS; ++ks) {
		const h8 w1row = loadA(w.d1, 16, 0, 16 * ks, h);
#pragma unroll
		for (int j = 0; j < 8; ++j) GhB[ks][j] = H0B[ks][j] > (half_t)0.f ? w1row[j] : (half_t)0.f;
	}
#pragma unroll
	for (int mt = 0; mt < DMT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.d0T, DIN, 32 * mt + r, 16 * ks, h), GhB[ks], acc);
		Gi[mt] = rh16(acc);
	}
}
template <int W>
__device__ __forceinline__ void rgb_hidden_frag(const FwdW& w, const h8& D1B, const float x[3], const float wd[3], const float grad[3],
                                                int r, int h, h8 rinB[3], h8* H1B, h8* H2B) {
	constexpr int MT = (W + 31) / 32, HKS = W / 16;
	rinB[0] = D1B;
	{
		float sh[16]; sh16(wd, sh);
#pragma unroll
		for (int j = 0; j < 8; ++j) rinB[1][j] = (half_t)hsel(h, sh[pi_row(j, 1)], sh[pi_row(j, 0)]);
		float r32[16];
#pragma unroll
		for (int k = 0; k < 16; ++k) r32[k] = 0.f;
		r32[0] = x[0]; r32[1] = x[1]; r32[2] = x[2];
		r32[3] = grad[0]; r32[4] = grad[1]; r32[5] = grad[2];
#pragma unroll
		for (int j = 0; j < 8; ++j) rinB[2][j] = (half_t)hsel(h, r32[pi_row(j, 1)], r32[pi_row(j, 0)]);
	}
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < 3; ++ks) acc = mfma(loadA(w.r0, W, 32 * mt + r, 16 * ks, h), rinB[ks], acc);
		H1B[2 * mt] = frag<true>(acc, 0);
		if (2 * mt + 1 < HKS) H1B[2 * mt + 1] = frag<true>(acc, 1);
	}
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.r1, W, 32 * mt + r, 16 * ks, h), H1B[ks], acc);
		H2B[2 * mt] = frag<true>(acc, 0);
		if (2 * mt + 1 < HKS) H2B[2 * mt + 1] = frag<true>(acc, 1);
	}
}
// relu'(Y) . acc as a fragment: (half)acc where the stored activation fragment m is > 0, else 0
__device__ __forceinline__ h8 mask_frag(const f16v& acc, int k, const h8& m) {
	h8 b;
#pragma unroll
	for (int j = 0; j < 8; ++j) b[j] = m[j] > (half_t)0.f ? (half_t)acc[8 * k + j] : (half_t)0.f;
	return b;
}

// ------------------------------------------------------------------------------------------
// Fused pre-compaction forward (hash-grid encode + NerfNetwork::forward, nerf_network.h:145-328):
// coords AoS7 -> out AoS16 fp16. The encodings and dy/dx never leave the registers; only the 28 B
// coordinate and the 32 B output per sample touch HBM. Activations are kept as fp16 B fragments
// (their storage precision), not fp32 tiles. n from device memory; 32 samples per wave-iteration,
// grid-strided.
// ------------------------------------------------------------------------------------------
#ifndef NEUS_INFER_ALL_WPE
#define NEUS_INFER_ALL_WPE 2
#endif
// ALL: every level active (the launch checks valid_level): the gathers of level pair m+1 are pinned in flight during
// level pair m's interpolation (fused_levels ALL); that needs more registers than 3 waves per SIMD allow without spills
template <int L, int W, bool IDX, bool ALL = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ALL ? NEUS_INFER_ALL_WPE : 3, ALL ? NEUS_INFER_ALL_WPE : 3))) k_nerf_infer(const uint32_t* __restrict__ n_ptr, uint32_t n_fixed, const float* __restrict__ coords,
                                                    const GridLevels gl, uint32_t valid_level, const half_t* __restrict__ grid,
                                                    MlpPtrs wp, half_t* __restrict__ out, const uint32_t* __restrict__ idx, InferAlpha ia) {
	constexpr int DKS = Dims<L>::DKS, DMT = Dims<L>::DMT, HALF = Fused<L>::HALF, M0 = Fused<L>::M0;
	constexpr int MT = (W + 31) / 32, HKS = W / 16;
	__shared__ half_t sm[FwdSmem<L, W>::END];
	__shared__ LevelSmem s_lvl;
	const FwdW w0 = stage_fwd<L, W>(sm, wp.d0p, wp.d0Tp, wp);
	stage_levels(s_lvl, gl, L);
	__syncthreads();
	const uint32_t n = n_ptr ? *n_ptr : n_fixed;
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
	uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
	uint32_t lo = 0, hi = n;
	if (ia.xcd_parts == 8u) {  // (grid a multiple of 8: the launch rounds it)
		const uint32_t x = blockIdx.x & 7u, wpb = blockDim.x >> 6;
		lo = (uint32_t)((uint64_t)n * x / 8u); hi = (uint32_t)((uint64_t)n * (x + 1u) / 8u);
		wave = (blockIdx.x >> 3) * wpb + (threadIdx.x >> 6); n_waves = (gridDim.x >> 3) * wpb;
	}
	const half_t var_h = wp.var[0];
	const half_t bias_h = (half_t)wp.sdf_bias;
	if (ia.n_long && blockIdx.x == 0 && threadIdx.x == 0) *ia.n_long = 0u;  // the transmittance scan's long-ray list
	for (uint32_t base = lo + wave * 32; base < hi; base += n_waves * 32) {
		const FwdW w = w0.at(opaque_zero());
		const uint32_t j = base + r;
		const bool valid = j < hi;
		const uint32_t i = valid ? (IDX ? idx[j] : j) : 0;
		const float* c = coords + (size_t)i * COORD_W;
		const float x[3] = {c[0], c[1], c[2]}, wd[3] = {c[4], c[5], c[6]};
		// ---- encode this lane's levels
		h2 ev[M0];
		float dy[M0][2][3];
		fused_levels<L, true, ALL>(s_lvl, gl.dense_bits, valid_level, grid, x, h, ev, dy);
		__builtin_amdgcn_sched_barrier(0);  // keep the MLP's LDS weight reads out of the encode region
		float ov[3], ovd[3][3];
		overflow_values<L>(h, ev, ov);
		overflow_dydx<L>(dy, ovd);
		const float xm[3] = {rh(rh(x[0]) - 0.5f), rh(rh(x[1]) - 0.5f), rh(rh(x[2]) - 0.5f)};
		h8 dinB[DKS];
#pragma unroll
		for (int ks = 0; ks < DKS; ++ks)
#pragma unroll
			for (int j = 0; j < 8; ++j) dinB[ks][j] = (half_t)slot_value<L>(8 * ks + j, h, xm, ev, ov);
		// ---- density MLP (fragments of the fp16-stored activations)
		h8 H0B[HKS];
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < DKS; ++ks) acc = mfma(loadA(w.d0, W, 32 * mt + r, 16 * ks, h), dinB[ks], acc);
			H0B[2 * mt] = frag<true>(acc, 0);
			if (2 * mt + 1 < HKS) H0B[2 * mt + 1] = frag<true>(acc, 1);  // W = 16: one 16-row half
		}
		h8 D1B;
		{
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.d1, 16, r, 16 * ks, h), H0B[ks], acc);
			D1B = frag<false>(acc, 0);
		}
		// G_h = relu'(H0) . W1d[0]; G_in = W0d^T G_h (fp16-stored)
		h8 GhB[HKS];
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) {
			const h8 w1row = loadA(w.d1, 16, 0, 16 * ks, h);
#pragma unroll
			for (int j = 0; j < 8; ++j) GhB[ks][j] = H0B[ks][j] > (half_t)0.f ? w1row[j] : (half_t)0.f;
		}
		// dSDF/dx = sum_q G_in[q] dy/dx[q] (+ identity for the xyz slots of h = 0), halves summed
		float part[3] = {0.f, 0.f, 0.f};
#pragma unroll
		for (int mt = 0; mt < DMT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.d0T, Dims<L>::DIN, 32 * mt + r, 16 * ks, h), GhB[ks], acc);
#pragma unroll
			for (int reg = 0; reg < 16; ++reg) {
				const int q = 16 * mt + reg;
				if (q >= HALF) continue;
				const float gv = rh(acc[reg]);
#pragma unroll
				for (int d = 0; d < 3; ++d) {
					const float id = (q == d) ? (h ? 0.f : 1.f) : 0.f;
					part[d] += gv * (slot_dydx<L>(q, h, d, dy, ovd) + id);
				}
			}
		}
		float grad[3];
#pragma unroll
		for (int d = 0; d < 3; ++d) grad[d] = part[d] + __shfl_xor(part[d], 32);
		// ---- colour MLP: input [density out (16), SH4 (16), xyz, grad sdf, 0...]
		h8 rinB[3];
		rinB[0] = D1B;
		{
			float sh[16]; sh16(wd, sh);
#pragma unroll
			for (int j = 0; j < 8; ++j) rinB[1][j] = (half_t)hsel(h, sh[pi_row(j, 1)], sh[pi_row(j, 0)]);
			float r32[16];
#pragma unroll
			for (int k = 0; k < 16; ++k) r32[k] = 0.f;
			r32[0] = x[0]; r32[1] = x[1]; r32[2] = x[2];
			r32[3] = grad[0]; r32[4] = grad[1]; r32[5] = grad[2];
#pragma unroll
			for (int j = 0; j < 8; ++j) rinB[2][j] = (half_t)hsel(h, r32[pi_row(j, 1)], r32[pi_row(j, 0)]);
		}
		h8 H1B[HKS], H2B[HKS];
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < 3; ++ks) acc = mfma(loadA(w.r0, W, 32 * mt + r, 16 * ks, h), rinB[ks], acc);
			H1B[2 * mt] = frag<true>(acc, 0);
			if (2 * mt + 1 < HKS) H1B[2 * mt + 1] = frag<true>(acc, 1);  // W = 16: one 16-row half
		}
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.r1, W, 32 * mt + r, 16 * ks, h), H1B[ks], acc);
			H2B[2 * mt] = frag<true>(acc, 0);
			if (2 * mt + 1 < HKS) H2B[2 * mt + 1] = frag<true>(acc, 1);  // W = 16: one 16-row half
		}
		f16v O = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) O = mfma(loadA(w.r2, 16, r, 16 * ks, h), H2B[ks], O);
		const half_t row11 = (half_t)__shfl_xor(O[7], 32);  // lane h=0 holds row 11 in reg 7
		h8 o;
		if (h == 0) {
			o[0] = (half_t)O[0]; o[1] = (half_t)O[1]; o[2] = (half_t)O[2];
			o[3] = D1B[0] + bias_h;                              // half add (common_operation.cuh:964)
			o[4] = (half_t)grad[0]; o[5] = (half_t)grad[1]; o[6] = (half_t)grad[2];
			o[7] = var_h;
		} else {
			o[0] = (half_t)wd[0]; o[1] = (half_t)wd[1]; o[2] = (half_t)wd[2];
			o[3] = row11;
			o[4] = (half_t)O[4]; o[5] = (half_t)O[5]; o[6] = (half_t)O[6]; o[7] = (half_t)O[7];
		}
		if (valid) *(h8*)(out + (size_t)i * OUT_W + 8 * h) = o;
		if (ia.sa) {
			// the loss's alpha terms of this sample from its 16 outputs (the h = 1 half arrives by shuffle)
			half_t lo[16];
#pragma unroll
			for (int q = 0; q < 4; ++q) {
				const uint32_t mine = __builtin_bit_cast(uint32_t, (h2){o[2 * q], o[2 * q + 1]});
				const h2 other = __builtin_bit_cast(h2, (uint32_t)__shfl_xor((int)mine, 32));
				lo[2 * q] = o[2 * q]; lo[2 * q + 1] = o[2 * q + 1];
				lo[8 + 2 * q] = other[0]; lo[8 + 2 * q + 1] = other[1];
			}
			if (valid && h == 0) {
				const float dt = ia.dt_const ? unwarp_dt(warp_dt(MIN_CONE_STEPSIZE)) : unwarp_dt(c[3]);
				loss_alpha_sample(lo, dt, ia.cos_anneal, ia.sa, ia.ekt, i);
			}
		}
	}
}

// Density-only inference for the occupancy grid (NerfNetwork::density, nerf_network.h:656-739;
// sdf_to_density_variance_buffer, common_operation.cuh:306-324 in fp16 arithmetic), with the
// hash-grid encode fused in (no dy/dx needed).
// MODE 0: occupancy density of the positions in `pos` (AoS 3 f32).
// MODE 1: raw SDF (NerfNetwork::sdf, nerf_network.h:656-722 -> grid_samples_half_to_float, testbed_nerf.cu:692-708)
//         at the points of a uniform grid generated in-kernel (generate_grid_samples_nerf_uniform,
//         testbed_nerf.cu:596-609: p = x * (1/res) * (aabb.max - aabb.min) + aabb.min, nvcc-contracted to an
//         FMA, then warp_position into the training aabb); density[i] = float(sdf + bias) for grid point
//         offset + i. No 12-B position buffer: 1024^3 points read nothing but the grid table.
// MODE 2: the occupancy-grid update fused: sample g = os.lo + i of the update's global sample range is generated
//         in-kernel (grid_sample: the uniform call for g < n_u, the occupancy-biased call after it), its density
//         splatted into os.grid_tmp with the reference's atomicMax on the float bits (splat_grid_samples_nerf_max_
//         nearest_neighbor) - no position, cell index or density buffer.
//         With ug.delta (m_use_delta after prepare_for_test, nerf_network.h:664-676) the point goes through the
//         DeltaNetwork first: x' = R (x + t), as k_delta_apply.
struct UniformGrid { uint32_t res[3]; float inv_res[3], rmin[3], rdiag[3], tmin[3], tdiag[3]; uint64_t offset; const DeltaState* delta; };

template <int L, int W, int MODE>
__global__ void __launch_bounds__(256) k_nerf_density(uint32_t n, const float* __restrict__ pos, const UniformGrid ug, const OccSampling os,
                                                      const GridLevels gl, uint32_t valid_level, const half_t* __restrict__ grid, MlpPtrs wp,
                                                      float* __restrict__ density) {
	constexpr int DKS = Dims<L>::DKS, M0 = Fused<L>::M0, MT = (W + 31) / 32, HKS = W / 16;
	__shared__ half_t sm[FwdSmem<L, W>::END];
	__shared__ LevelSmem s_lvl;
	const FwdW w0 = stage_fwd<L, W>(sm, wp.d0p, wp.d0Tp, wp);
	stage_levels(s_lvl, gl, L);
	__syncthreads();
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
	const half_t var_h = wp.var[0];
	const half_t bias_h = (half_t)wp.sdf_bias;
	for (uint32_t base = wave * 32; base < n; base += n_waves * 32) {
		const FwdW w = w0.at(opaque_zero());
		const uint32_t i = base + r;
		const bool valid = i < n;
		const uint32_t ic = valid ? i : 0;
		float x[3];
		uint32_t cell = 0;
		if (MODE == 0) {
			x[0] = pos[3 * (size_t)ic]; x[1] = pos[3 * (size_t)ic + 1]; x[2] = pos[3 * (size_t)ic + 2];
		} else if (MODE == 2 && os.exclusive) {
			cell = os.lo + ic;
			grid_sample_cell(cell, os.rng_u_state, os.rng_u_inc, os.amin, os.diag, x, os.jt);
		} else if (MODE == 2) {
			// cell-ordered uniform samples first (coherent gathers), then the nonuniform ones of the rank's range
			const uint32_t kk = ic - os.n_ulist;
			const uint32_t g = os.ulist ? (ic < os.n_ulist ? os.ulist[ic] : max(os.lo, os.n_u) + (os.nulist ? os.nulist[kk] : kk)) : os.lo + ic;
			const bool uni = g < os.n_u;
			grid_sample(uni ? os.n_u : os.n_nu, uni ? g : g - os.n_u, uni ? os.rng_u_state : os.rng_nu_state, uni ? os.rng_u_inc : os.rng_nu_inc,
			            os.step, os.amin, os.diag, os.grid_in, os.n_cascades, uni ? -0.01f : os.thresh_nu, x, cell, os.jt);
		} else {
			const uint64_t g = ug.offset + ic;
			const uint64_t rxy = (uint64_t)ug.res[0] * ug.res[1];
			const uint32_t gz = (uint32_t)(g / rxy), gy = (uint32_t)((g - gz * rxy) / ug.res[0]);
			const uint32_t gx = (uint32_t)(g - gz * rxy - (uint64_t)gy * ug.res[0]);
			const uint32_t gi[3] = {gx, gy, gz};
#pragma unroll
			for (int k = 0; k < 3; ++k) {
				const float pk = __builtin_fmaf(__fmul_rn((float)gi[k], ug.inv_res[k]), ug.rdiag[k], ug.rmin[k]);
				x[k] = __fdiv_rn(__fsub_rn(pk, ug.tmin[k]), ug.tdiag[k]);
			}
			if (ug.delta) {
				const float* R = ug.delta->R;
				const float p[3] = {__fadd_rn(x[0], ug.delta->t[0]), __fadd_rn(x[1], ug.delta->t[1]), __fadd_rn(x[2], ug.delta->t[2])};
#pragma unroll
				for (int k = 0; k < 3; ++k)
					x[k] = __fadd_rn(__fadd_rn(__fmul_rn(R[3 * k], p[0]), __fmul_rn(R[3 * k + 1], p[1])), __fmul_rn(R[3 * k + 2], p[2]));
			}
		}
		h2 ev[M0];
		float dy[1][2][3];
		fused_levels<L, false>(s_lvl, gl.dense_bits, valid_level, grid, x, h, ev, dy);
		float ov[3];
		overflow_values<L>(h, ev, ov);
		const float xm[3] = {rh(rh(x[0]) - 0.5f), rh(rh(x[1]) - 0.5f), rh(rh(x[2]) - 0.5f)};
		h8 dinB[DKS];
#pragma unroll
		for (int ks = 0; ks < DKS; ++ks)
#pragma unroll
			for (int j = 0; j < 8; ++j) dinB[ks][j] = (half_t)slot_value<L>(8 * ks + j, h, xm, ev, ov);
		h8 H0B[HKS];
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < DKS; ++ks) acc = mfma(loadA(w.d0, W, 32 * mt + r, 16 * ks, h), dinB[ks], acc);
			H0B[2 * mt] = frag<true>(acc, 0);
			if (2 * mt + 1 < HKS) H0B[2 * mt + 1] = frag<true>(acc, 1);  // W = 16: one 16-row half
		}
		f16v acc = zero16();
#pragma unroll
		for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w.d1, 16, r, 16 * ks, h), H0B[ks], acc);
		if (MODE == 1) {
			if (valid && h == 0) density[i] = (float)((half_t)acc[0] + bias_h);
		} else if (valid && h == 0) {
			const half_t sdf = (half_t)acc[0] + bias_h;
			const half_t s = (half_t)__expf((float)(var_h * (half_t)10.0f));
			const half_t sig = (half_t)(1.0f / (1.0f + __expf(-(float)(sdf * s))));
			const half_t dens = (s * sig) * ((half_t)1.0f - sig);
			if (MODE == 2) {
				// an all-cells uniform pass over one cascade hits every cell exactly once (odd multiplier mod 2^21):
				// the splat's max is then the sample itself - a plain store
				if (os.exclusive) os.grid_tmp[cell] = (float)dens;
				else atomicMax((uint32_t*)&os.grid_tmp[cell], __float_as_uint((float)dens));
			}
			else density[i] = (float)dens;
		}
	}
}

// ------------------------------------------------------------------------------------------
// Training path: encodings and dy/dx come from k_grid_encode (logical din order).
// ------------------------------------------------------------------------------------------
// Reads this lane's encoding features and builds the density-input B fragments (logical order).
template <int L>
__device__ __forceinline__ void load_enc(uint32_t ev[L], const half_t* __restrict__ enc_h /*[L][ld] half2*/, uint32_t ld, uint32_t i) {
#pragma unroll
	for (int l = 0; l < L; ++l) ev[l] = ((const uint32_t*)enc_h)[(size_t)l * ld + i];
}
// (split from the loads, so a kernel can issue its other loads of the chunk in between)
template <int L>
__device__ __forceinline__ void build_din(h8* dinB, const float x[3], const uint32_t ev[L], int h) {
	constexpr int DIN = Dims<L>::DIN;
	float dv[DIN];
#pragma unroll
	for (int k = 0; k < DIN; ++k) {
		if (k < 3) dv[k] = rh(rh(x[k]) - 0.5f);
		else if (k < 3 + 2 * L) dv[k] = (float)__builtin_bit_cast(h2, ev[(k - 3) >> 1])[(k - 3) & 1];
		else dv[k] = 0.f;
	}
#pragma unroll
	for (int ks = 0; ks < Dims<L>::DKS; ++ks)
#pragma unroll
		for (int j = 0; j < 8; ++j) dinB[ks][j] = (half_t)hsel(h, dv[16 * ks + pi_row(j, 1)], dv[16 * ks + pi_row(j, 0)]);
}

// dy/dx of density-input slot k (k = 3 + 2 l + f: feature f of level l) for sample i, [6L][ld] f32 rows 3 (k - 3) + d.
// Slots outside the features read a clamped row; the caller masks them. The loads are unconditional on purpose: the
// slot depends on the lane half, and a lane-dependent branch around each load group made the compiler wait for
// every group before issuing the next (14 serial memory round trips per 32-sample chunk in the colour kernel).
template <int L>
__device__ __forceinline__ void load_dydx(const float* __restrict__ dydx, uint32_t ld, uint32_t i, int k, float dy[3]) {
	const int q = min(max(k - 3, 0), 2 * L - 1);
	const float* dp = dydx + (size_t)(3 * q) * ld + i;
	dy[0] = dp[0]; dy[1] = dp[ld]; dy[2] = dp[2 * (size_t)ld];
}

// backward weight set: transposed copies, staged after the forward set
struct BwdW { MatRef r2T, r1T, r0T, d1T; };
template <int L, int W> struct TrainSmem {
	static constexpr int R2T = FwdSmem<L, W>::END, R1T = R2T + W * (16 + 8), R0T = R1T + W * (W + 8), D1T = R0T + 48 * (W + 8);
	static constexpr int END = D1T + W * (16 + 8);
};

// ------------------------------------------------------------------------------------------
// Training forward-recompute + first- and second-order backward for 32 compacted samples per wave, with the
// weight-gradient GEMMs fused in: dW = sum over samples of D X^T (fully_fused_mlp.cu:967-1085, the split-K
// fc_multiply_split_k of :1007 / :1020, and the second-order terms of :1088-1198) accumulated in registers across
// the persistent loop, one partial row per block at the end. The operands (activations and deltas, held as B
// fragments with the sample on the MFMA column) are turned into "sample on the k dimension" fragments by an MFMA
// with a 0/1 selection matrix (exact: one nonzero product per output), so the per-sample operands never leave the
// registers (the split-K GEMM used to write ~340 MB of fp16 operands per step and read them back).
// ------------------------------------------------------------------------------------------
// The selection operand of transpose32: column 16 q + c (c < 16) picks k index kinv(c) = 8 ((c >> 2) & 1) + 4 (c >> 3)
// + (c & 3), the slot of fragment row c (pi_row(j, h) = c); columns of the other half are zero.
__device__ __forceinline__ h8 transpose_sel(int q) {
	const int lane = threadIdx.x & 63, col = lane & 31, h = lane >> 5, c = col & 15;
	const bool on = (col >> 4) == q && ((c >> 2) & 1) == h;
	const int j = 4 * (c >> 3) + (c & 3);
	h8 b;
#pragma unroll
	for (int k = 0; k < 8; ++k) b[k] = (on && k == j) ? (half_t)1.0f : (half_t)0.0f;
	return b;
}
// 32 rows of B fragments (f0: rows 32t + [0, 16), f1: rows 32t + [16, 32) if has1) -> the two k-step fragments of
// samples for the row on this lane's column: T[q][j] = row 32t + (lane & 31), sample acc_row(8q + j, lane >> 5).
__device__ __forceinline__ void transpose32(const h8& f0, const h8& f1, bool has1, const h8& s0, const h8& s1, h8 T[2]) {
	f16v acc = mfma(f0, s0, zero16());
	if (has1) acc = mfma(f1, s1, acc);
	T[0] = frag<false>(acc, 0);
	T[1] = frag<false>(acc, 1);
}
// LDS of a kernel whose weight staging is reused by flush_tile at the end (4 waves x 1024 floats)
constexpr int smem_halves(int staged) { return staged > 8192 ? staged : 8192; }
// dW tile (rows of D's tile, columns of X's tile) += TD . TX^T over the 32 samples
__device__ __forceinline__ f16v wg_acc(const h8 TD[2], const h8 TX[2], f16v a) { return mfma(TD[1], TX[1], mfma(TD[0], TX[0], a)); }
// The block's dW tiles summed over its four waves in a fixed order into its partial row (`red`: 4 KB per wave of LDS)
__device__ __forceinline__ void flush_tile(float* red, float* prow, const f16v& a, uint32_t off, int M, int K, int mt, int kt) {
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wv = threadIdx.x >> 6;
#pragma unroll
	for (int reg = 0; reg < 16; ++reg) red[wv * 1024 + acc_row(reg, h) * 32 + r] = a[reg];
	__syncthreads();
	for (uint32_t e = threadIdx.x; e < 1024; e += blockDim.x) {
		const int m = 32 * mt + (int)(e / 32), k = 32 * kt + (int)(e % 32);
		if (m < M && k < K) prow[off + (uint32_t)(m * K + k)] = (red[e] + red[1024 + e]) + (red[2048 + e] + red[3072 + e]);
	}
	__syncthreads();
}
// store an accumulator tile (rows 32*mt + acc_row) into SoA [rows][ldc] at column col, rows < R
__device__ __forceinline__ void store_acc(half_t* buf, size_t ldc, uint32_t col, const f16v& a, int mt, int R, int h) {
#pragma unroll
	for (int reg = 0; reg < 16; ++reg) {
		const int row = 32 * mt + acc_row(reg, h);
		if (row < R) buf[(size_t)row * ldc + col] = (half_t)a[reg];
	}
}

// Training is split in two kernels so that neither holds the whole forward + backward state:
//   k_mlp_train_rgb     : forward recompute (density + grad SDF + colour hidden layers), colour backward,
//                         dL/d(density output) and v = dL/d(grad SDF); dW of the three colour layers
//   k_mlp_train_density : density forward recompute, density backward (first order) and the second-order
//                         front pass h1' = relu'(H0) . (W0 u); dW of the two density layers, first + second order
// They communicate through d1_delta and v.
template <int L, int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_mlp_train_rgb(const uint32_t* __restrict__ n_valid_ptr, uint32_t n, uint32_t ld,
                                                       const float* __restrict__ coords, const half_t* __restrict__ enc_h,
                                                       const float* __restrict__ dydx, const half_t* __restrict__ dL_dout,
                                                       MlpPtrs w, TrainBufs tb) {
	constexpr int DKS = Dims<L>::DKS, DMT = Dims<L>::DMT;
	constexpr int MT = (W + 31) / 32, HKS = W / 16;
	if (n_valid_ptr && *n_valid_ptr == 0) return;
	__shared__ half_t sm[smem_halves(TrainSmem<L, W>::END)];  // (the end-of-kernel dW reduction reuses 16 KB of it)
	using TS = TrainSmem<L, W>;
	const FwdW fw0 = stage_fwd<L, W>(sm, w.d0, w.d0T, w);
	stage_mat(sm + TS::R2T, w.r2T, W, 16);
	stage_mat(sm + TS::R1T, w.r1T, W, W);
	stage_mat(sm + TS::R0T, w.r0T, 48, W);
	const BwdW bw0{{sm + TS::R2T, 16 + 8}, {sm + TS::R1T, W + 8}, {sm + TS::R0T, W + 8}, {sm + TS::D1T, 16 + 8}};
	__syncthreads();
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
	const h8 sel0 = transpose_sel(0), sel1 = transpose_sel(1);
	const h8 z8 = (h8){0, 0, 0, 0, 0, 0, 0, 0};
	// dW accumulators: r0 [W][48] (K tiles: rin rows 0..31, 32..47), r1 [W][W], r2 [16][W]
	f16v aR0[MT][2], aR1[MT][MT], aR2[MT];
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		aR0[mt][0] = zero16(); aR0[mt][1] = zero16(); aR2[mt] = zero16();
#pragma unroll
		for (int kt = 0; kt < MT; ++kt) aR1[mt][kt] = zero16();
	}
	float var_part = 0.f;
	for (uint32_t base = wave * 32; base < n; base += n_waves * 32) {
		const uint32_t z = opaque_zero();
		const FwdW fw = fw0.at(z);
		const BwdW bw{rebase(bw0.r2T, z), rebase(bw0.r1T, z), rebase(bw0.r0T, z), rebase(bw0.d1T, z)};
		const uint32_t i = base + r;
		const bool valid = i < n;
		const uint32_t ic = valid ? i : 0;
		const float* c = coords + (size_t)ic * COORD_W;
		const float x[3] = {c[0], c[1], c[2]}, wd[3] = {c[4], c[5], c[6]};
		// ---- forward recompute up to the colour hidden layers
		uint32_t ev[L];
		load_enc<L>(ev, enc_h, ld, ic);
		// all of the chunk's dy/dx loads (and dL/dout) are issued right after the encoding's, before the density forward:
		// one memory round trip per chunk, the dy/dx part overlapped with the forward's MFMAs (loads complete in order,
		// so the forward waits for the encoding only; the sched_barrier keeps them up front)
		float dyv[DMT * 16][3];
#pragma unroll
		for (int mt = 0; mt < DMT; ++mt)
#pragma unroll
			for (int reg = 0; reg < 16; ++reg) load_dydx<L>(dydx, ld, ic, 32 * mt + acc_row(reg, h), dyv[16 * mt + reg]);
		const h8 dlo_ld = *(const h8*)(dL_dout + (size_t)ic * OUT_W + 8 * h);  // h=0: rows 0..7, h=1: rows 8..15
		__builtin_amdgcn_sched_barrier(0);
		h8 dinB[DKS];
		build_din<L>(dinB, x, ev, h);
		h8 H0B[HKS], D1B, GhB[HKS];
		f16v Gi[DMT];
		density_forward_frag<L, W>(fw, dinB, r, h, H0B, D1B, GhB, Gi);
		// (feature slots: part += G dy/dx as one fma each; xyz slots: the fma adds 0 * dy, then the identity term -
		// the values of the former branchy form, bit for bit)
		float part[3] = {0.f, 0.f, 0.f};
#pragma unroll
		for (int mt = 0; mt < DMT; ++mt)
#pragma unroll
			for (int reg = 0; reg < 16; ++reg) {
				const int k = 32 * mt + acc_row(reg, h);
				const float gv = Gi[mt][reg];
				const float gf = (k >= 3 && k < 3 + 2 * L) ? gv : 0.f;
#pragma unroll
				for (int d = 0; d < 3; ++d) part[d] = fmaf(gf, dyv[16 * mt + reg][d], part[d]) + ((k == d) ? gv : 0.f);
			}
		float grad[3];
#pragma unroll
		for (int d = 0; d < 3; ++d) grad[d] = part[d] + __shfl_xor(part[d], 32);
		h8 rinB[3];
		h8 H1B[HKS], H2B[HKS];
		rgb_hidden_frag<W>(fw, D1B, x, wd, grad, r, h, rinB, H1B, H2B);
		// ---- colour backward (a lane without a sample gets dL/dout = 0: every delta, hence its dW share, is 0)
		const h8 dlo = valid ? dlo_ld : z8;
		const h8 dlo_o = shfl_xor_h8(dlo, 32);
		const h8 dlo_lo = h ? dlo_o : dlo;   // rows 0..7 on every lane
		const h8 dlo_hi = h ? dlo : dlo_o;   // rows 8..15 on every lane
		if (valid && h == 0) var_part += (float)dlo_lo[7];
		// delta_o (rows 0..2 = dL/drgb): B fragment, pi order -> lane h=0 elements 0..2
		h8 dOB = z8;
		if (h == 0) { dOB[0] = dlo_lo[0]; dOB[1] = dlo_lo[1]; dOB[2] = dlo_lo[2]; }
		{  // dW_r2 += dO . H2^T
			h8 TD[2];
			transpose32(dOB, z8, false, sel0, sel1, TD);
#pragma unroll
			for (int kt = 0; kt < MT; ++kt) {
				h8 TX[2];
				transpose32(H2B[2 * kt], 2 * kt + 1 < HKS ? H2B[2 * kt + 1] : z8, 2 * kt + 1 < HKS, sel0, sel1, TX);
				aR2[kt] = wg_acc(TD, TX, aR2[kt]);
			}
		}
		h8 dH2B[HKS], dH1B[HKS];
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			const f16v acc = mfma(loadA(bw.r2T, W, 32 * mt + r, 0, h), dOB, zero16());
			dH2B[2 * mt] = mask_frag(acc, 0, H2B[2 * mt]);
			if (2 * mt + 1 < HKS) dH2B[2 * mt + 1] = mask_frag(acc, 1, H2B[2 * mt + 1]);
		}
		{  // dW_r1 += dH2 . H1^T
			h8 TD[MT][2];
#pragma unroll
			for (int mt = 0; mt < MT; ++mt) transpose32(dH2B[2 * mt], 2 * mt + 1 < HKS ? dH2B[2 * mt + 1] : z8, 2 * mt + 1 < HKS, sel0, sel1, TD[mt]);
#pragma unroll
			for (int kt = 0; kt < MT; ++kt) {
				h8 TX[2];
				transpose32(H1B[2 * kt], 2 * kt + 1 < HKS ? H1B[2 * kt + 1] : z8, 2 * kt + 1 < HKS, sel0, sel1, TX);
#pragma unroll
				for (int mt = 0; mt < MT; ++mt) aR1[mt][kt] = wg_acc(TD[mt], TX, aR1[mt][kt]);
			}
		}
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(bw.r1T, W, 32 * mt + r, 16 * ks, h), dH2B[ks], acc);
			dH1B[2 * mt] = mask_frag(acc, 0, H1B[2 * mt]);
			if (2 * mt + 1 < HKS) dH1B[2 * mt + 1] = mask_frag(acc, 1, H1B[2 * mt + 1]);
		}
		{  // dW_r0 += dH1 . rin^T
			h8 TD[MT][2];
#pragma unroll
			for (int mt = 0; mt < MT; ++mt) transpose32(dH1B[2 * mt], 2 * mt + 1 < HKS ? dH1B[2 * mt + 1] : z8, 2 * mt + 1 < HKS, sel0, sel1, TD[mt]);
#pragma unroll
			for (int kt = 0; kt < 2; ++kt) {
				h8 TX[2];
				transpose32(rinB[2 * kt], kt == 0 ? rinB[1] : z8, kt == 0, sel0, sel1, TX);
#pragma unroll
				for (int mt = 0; mt < MT; ++mt) aR0[mt][kt] = wg_acc(TD[mt], TX, aR0[mt][kt]);
			}
		}
		f16v dRin[2];
#pragma unroll
		for (int mt = 0; mt < 2; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(bw.r0T, 48, 32 * mt + r, 16 * ks, h), dH1B[ks], acc);
			dRin[mt] = rh16(acc);
		}
		// delta_D1 = dL/drgb_in[0:16], row 0 += dL_dout[3] (half add)
		f16v dD1 = dRin[0];
		if (h == 0) dD1[0] = (float)((half_t)dD1[0] + dlo_lo[3]);
		// v = dL/d(grad sdf) (nerf_network.h:478-504): rows 35..37 of dL/drgb_in live at
		// tile 1: row 3 on h=0 reg 3, rows 4,5 on h=1 regs 0,1
		const float o3 = __shfl_xor(dRin[1][3], 32), o0 = __shfl_xor(dRin[1][0], 32), o1 = __shfl_xor(dRin[1][1], 32);
		float v[3];
		v[0] = h ? o3 : dRin[1][3];
		v[1] = h ? dRin[1][0] : o0;
		v[2] = h ? dRin[1][1] : o1;
		v[0] += (float)dlo_lo[4] / tb.indeed_batch; v[1] += (float)dlo_lo[5] / tb.indeed_batch; v[2] += (float)dlo_lo[6] / tb.indeed_batch;
		v[0] += (float)dlo_hi[0]; v[1] += (float)dlo_hi[1]; v[2] += (float)dlo_hi[2];
		if (valid) {
			store_acc(tb.d1_delta, ld, i, dD1, 0, 16, h);
			if (h == 0) tb.v[i] = make_float4(v[0], v[1], v[2], 0.f);
			// dL/d(rgb input xyz rows 32..34) for the global-movement gradient (nerf_network.h:613-616)
			if (tb.dpos && h == 0) tb.dpos[i] = make_float4(dRin[1][0], dRin[1][1], dRin[1][2], 0.f);
		}
	}
	// variance gradient: batch sum of dL/dout[7] (nerf_network.h:461-474); per block here, the blocks in a fixed
	// order in k_mlp_grad_reduce
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) var_part += __shfl_xor(var_part, off);
	__shared__ float s_var[4];
	if (lane == 0) s_var[threadIdx.x >> 6] = var_part;
	__syncthreads();  // (also: every wave is done with the staged weights; their LDS holds the dW reduction now)
	if (threadIdx.x == 0) tb.var_partial[blockIdx.x] = (s_var[0] + s_var[1]) + (s_var[2] + s_var[3]);
	float* red = (float*)sm;
	float* prow = tb.wpartial + (size_t)blockIdx.x * tb.n_matrix;
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
		for (int kt = 0; kt < 2; ++kt) flush_tile(red, prow, aR0[mt][kt], tb.off_r0, W, 48, mt, kt);
#pragma unroll
		for (int kt = 0; kt < MT; ++kt) flush_tile(red, prow, aR1[mt][kt], tb.off_r1, W, W, mt, kt);
		flush_tile(red, prow, aR2[mt], tb.off_r2, 16, W, 0, mt);
	}
}

template <int L, int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_mlp_train_density(const uint32_t* __restrict__ n_valid_ptr, uint32_t n, uint32_t ld,
                                                           const float* __restrict__ coords, const half_t* __restrict__ enc_h,
                                                           const float* __restrict__ dydx, MlpPtrs w, TrainBufs tb) {
	constexpr int DIN = Dims<L>::DIN, DKS = Dims<L>::DKS, DMT = Dims<L>::DMT;
	constexpr int MT = (W + 31) / 32, HKS = W / 16;
	if (n_valid_ptr && *n_valid_ptr == 0) return;
	__shared__ half_t sm[smem_halves(TrainSmem<L, W>::END)];  // (the end-of-kernel dW reduction reuses 16 KB of it)
	using TS = TrainSmem<L, W>;
	const FwdW fw0 = stage_fwd<L, W>(sm, w.d0, w.d0T, w);
	stage_mat(sm + TS::D1T, w.d1T, W, 16);
	const MatRef d1T0{sm + TS::D1T, 16 + 8};
	__syncthreads();
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
	const h8 sel0 = transpose_sel(0), sel1 = transpose_sel(1);
	const h8 z8 = (h8){0, 0, 0, 0, 0, 0, 0, 0};
	// dW accumulators: d0 [W][DIN], d1 [16][W] (first + second order)
	f16v aD0[MT][DMT], aD1[MT];
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		aD1[mt] = zero16();
#pragma unroll
		for (int kt = 0; kt < DMT; ++kt) aD0[mt][kt] = zero16();
	}
	for (uint32_t base = wave * 32; base < n; base += n_waves * 32) {
		const uint32_t z = opaque_zero();
		const FwdW fw = fw0.at(z);
		const MatRef d1T = rebase(d1T0, z);
		const uint32_t i = base + r;
		const bool valid = i < n;
		const uint32_t ic = valid ? i : 0;
		const float* c = coords + (size_t)ic * COORD_W;
		const float x[3] = {c[0], c[1], c[2]};
		// the chunk's loads up front (as the colour kernel): encoding, then dy/dx of this lane's density-input slots (the
		// accumulator rows k = 32 mt + acc_row(reg, h); fragment j of k-step ks is register 8 (ks & 1) + j of tile ks >> 1),
		// delta_D1 and v
		uint32_t ev[L];
		load_enc<L>(ev, enc_h, ld, ic);
		__builtin_amdgcn_sched_barrier(0);  // (the encoding's loads first: in-order completion lets the forward wait for them alone)
		float dyv[DMT * 16][3];
#pragma unroll
		for (int mt = 0; mt < DMT; ++mt)
#pragma unroll
			for (int reg = 0; reg < 16; ++reg) load_dydx<L>(dydx, ld, ic, 32 * mt + acc_row(reg, h), dyv[16 * mt + reg]);
		half_t d1v[8];
#pragma unroll
		for (int j = 0; j < 8; ++j) d1v[j] = tb.d1_delta[(size_t)(h ? pi_row(j, 1) : pi_row(j, 0)) * ld + ic];
		const float4 v4 = tb.v[ic];
		__builtin_amdgcn_sched_barrier(0);
		h8 dinB[DKS];
		build_din<L>(dinB, x, ev, h);
		h8 H0B[HKS], D1B, GhB[HKS];
		f16v Gi[DMT];
		density_forward_frag<L, W>(fw, dinB, r, h, H0B, D1B, GhB, Gi);
		if (valid) {
#pragma unroll
			for (int mt = 0; mt < DMT; ++mt)
#pragma unroll
				for (int reg = 0; reg < 16; ++reg) {
					const int k = 32 * mt + acc_row(reg, h);
					if (k >= 3 && k < 3 + 2 * L) tb.genc[((size_t)((k - 3) >> 1) * ld + i) * 2 + ((k - 3) & 1)] = (half_t)Gi[mt][reg];  // [L][ld] half2
				}
		}
		// delta_D1 from the colour kernel (d1_delta column i), B fragment in pi order (0 without a sample)
		h8 dD1B;
#pragma unroll
		for (int j = 0; j < 8; ++j) dD1B[j] = valid ? d1v[j] : (half_t)0.f;
		{  // dW_d1 (first order) += dD1 . H0^T
			h8 TD[2];
			transpose32(dD1B, z8, false, sel0, sel1, TD);
#pragma unroll
			for (int kt = 0; kt < MT; ++kt) {
				h8 TX[2];
				transpose32(H0B[2 * kt], 2 * kt + 1 < HKS ? H0B[2 * kt + 1] : z8, 2 * kt + 1 < HKS, sel0, sel1, TX);
				aD1[kt] = wg_acc(TD, TX, aD1[kt]);
			}
		}
		h8 dH0B[HKS];
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			const f16v acc = mfma(loadA(d1T, W, 32 * mt + r, 0, h), dD1B, zero16());
			dH0B[2 * mt] = mask_frag(acc, 0, H0B[2 * mt]);
			if (2 * mt + 1 < HKS) dH0B[2 * mt + 1] = mask_frag(acc, 1, H0B[2 * mt + 1]);
		}
		{  // dW_d0 (first order) += dH0 . din^T
			h8 TD[MT][2];
#pragma unroll
			for (int mt = 0; mt < MT; ++mt) transpose32(dH0B[2 * mt], 2 * mt + 1 < HKS ? dH0B[2 * mt + 1] : z8, 2 * mt + 1 < HKS, sel0, sel1, TD[mt]);
#pragma unroll
			for (int kt = 0; kt < DMT; ++kt) {
				h8 TX[2];
				transpose32(dinB[2 * kt], 2 * kt + 1 < DKS ? dinB[2 * kt + 1] : z8, 2 * kt + 1 < DKS, sel0, sel1, TX);
#pragma unroll
				for (int mt = 0; mt < MT; ++mt) aD0[mt][kt] = wg_acc(TD[mt], TX, aD0[mt][kt]);
			}
		}
		f16v dDin[DMT];
#pragma unroll
		for (int mt = 0; mt < DMT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(fw.d0T, DIN, 32 * mt + r, 16 * ks, h), dH0B[ks], acc);
			dDin[mt] = rh16(acc);
		}
		// dL/d(position) for the global-movement gradient (nerf_network.h:602-631): the grid's input gradient
		// sum_k dL/denc_k dy_k/dx (kernel_grid_backward_input) plus the density input's xyz rows; the colour
		// kernel stored the rgb input's xyz rows. Both lane halves hold parts of the k sum.
		float pg[3] = {0.f, 0.f, 0.f}, pd[3] = {0.f, 0.f, 0.f};
		if (tb.dpos) {
#pragma unroll
			for (int mt = 0; mt < DMT; ++mt)
#pragma unroll
				for (int reg = 0; reg < 16; ++reg) {
					const int k = 32 * mt + acc_row(reg, h);
					const float gv = dDin[mt][reg];
					const float gf = (k >= 3 && k < 3 + 2 * L) ? gv : 0.f;
#pragma unroll
					for (int d = 0; d < 3; ++d) {
						pd[d] += (k == d) ? gv : 0.f;
						pg[d] = fmaf(gf, dyv[16 * mt + reg][d], pg[d]);
					}
				}
#pragma unroll
			for (int d = 0; d < 3; ++d) { pg[d] += __shfl_xor(pg[d], 32); pd[d] += __shfl_xor(pd[d], 32); }
		}
		const float v[3] = {v4.x, v4.y, v4.z};
		// u = [v, dy/dx . v, 0] (grid.h:1182-1207), B fragments in pi order
		h8 uB[DKS];
#pragma unroll
		for (int ks = 0; ks < DKS; ++ks)
#pragma unroll
			for (int j = 0; j < 8; ++j) {
				const int k = 16 * ks + (h ? pi_row(j, 1) : pi_row(j, 0));
				const float* dy = dyv[16 * (ks >> 1) + 8 * (ks & 1) + j];
				const float du = dy[0] * v[0] + dy[1] * v[1] + dy[2] * v[2];
				const float vk = k == 0 ? v[0] : (k == 1 ? v[1] : v[2]);
				uB[ks][j] = (half_t)(k < 3 ? vk : (k < 3 + 2 * L ? du : 0.f));
			}
		// h1' = relu'(H0) . (W0d u)
		h8 H1pB[HKS];
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < DKS; ++ks) acc = mfma(loadA(fw.d0, W, 32 * mt + r, 16 * ks, h), uB[ks], acc);
			H1pB[2 * mt] = mask_frag(acc, 0, H0B[2 * mt]);
			if (2 * mt + 1 < HKS) H1pB[2 * mt + 1] = mask_frag(acc, 1, H0B[2 * mt + 1]);
		}
		{  // second order (fully_fused_mlp.cu:1088-1198): dW_d0 += b2 . u^T with b2 = relu'(H0) . W1d^T e0 (= GhB)
			h8 TD[MT][2];
#pragma unroll
			for (int mt = 0; mt < MT; ++mt) {
				const h8 g0 = valid ? GhB[2 * mt] : z8;
				const h8 g1 = (2 * mt + 1 < HKS && valid) ? GhB[2 * mt + 1] : z8;
				transpose32(g0, g1, 2 * mt + 1 < HKS, sel0, sel1, TD[mt]);
			}
#pragma unroll
			for (int kt = 0; kt < DMT; ++kt) {
				h8 TX[2];
				transpose32(uB[2 * kt], 2 * kt + 1 < DKS ? uB[2 * kt + 1] : z8, 2 * kt + 1 < DKS, sel0, sel1, TX);
#pragma unroll
				for (int mt = 0; mt < MT; ++mt) aD0[mt][kt] = wg_acc(TD[mt], TX, aD0[mt][kt]);
			}
		}
		{  // and dW_d1 += e0 . h1'^T: row 0 (this lane's column 0) collects the samples' h1', one per valid sample
			h8 TD[2];
#pragma unroll
			for (int q = 0; q < 2; ++q)
#pragma unroll
				for (int j = 0; j < 8; ++j) TD[q][j] = (r == 0 && base + acc_row(8 * q + j, h) < n) ? (half_t)1.0f : (half_t)0.0f;
#pragma unroll
			for (int kt = 0; kt < MT; ++kt) {
				h8 TX[2];
				transpose32(H1pB[2 * kt], 2 * kt + 1 < HKS ? H1pB[2 * kt + 1] : z8, 2 * kt + 1 < HKS, sel0, sel1, TX);
				aD1[kt] = wg_acc(TD, TX, aD1[kt]);
			}
		}
		if (valid) {
			if (tb.dpos && h == 0) {
				const float4 rg = tb.dpos[i];
				tb.dpos[i] = make_float4((pg[0] + rg.x) + pd[0], (pg[1] + rg.y) + pd[1], (pg[2] + rg.z) + pd[2], 0.f);
			}
			// ---- grid-scatter operand dL/denc = dDin rows 3.. (g = G_in rows 3.. went out after the forward)
#pragma unroll
			for (int mt = 0; mt < DMT; ++mt)
#pragma unroll
				for (int reg = 0; reg < 16; ++reg) {
					const int k = 32 * mt + acc_row(reg, h);
					if (k >= 3 && k < 3 + 2 * L) tb.dLdenc[((size_t)((k - 3) >> 1) * ld + i) * 2 + ((k - 3) & 1)] = (half_t)dDin[mt][reg];
				}
		}
	}
	__syncthreads();  // every wave is done with the staged weights: their LDS holds the dW reduction
	float* red = (float*)sm;
	float* prow = tb.wpartial + (size_t)blockIdx.x * tb.n_matrix;
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
		for (int kt = 0; kt < DMT; ++kt) flush_tile(red, prow, aD0[mt][kt], 0u, W, DIN, mt, kt);
		flush_tile(red, prow, aD1[mt], tb.off_d1, 16, W, 0, mt);
	}
}

// dW = the blocks' partial rows summed in a fixed order: a workgroup owns 64 parameters, its four waves sum the rows
// b = g, g + 4, ... (g = wave) with four interleaved chains each (16 independent loads in flight per lane), and the four
// wave sums are added in wave order. The workgroup after the last one sums the colour kernel's per-block variance
// partials in block order.
__global__ void __launch_bounds__(256) k_mlp_grad_reduce(MlpGradReduce rd) {
	const bool none = rd.n_valid && *rd.n_valid == 0;  // no samples: the gradients are zero (the training kernels wrote nothing)
	const uint32_t nblk_p = (rd.n_matrix + 63) / 64;
	if (blockIdx.x == nblk_p) {
		// fixed-order tree: thread t sums the partials t, t + 256, ..., then a pairwise tree over the threads
		__shared__ float s_v[256];
		float v = 0.f;
		for (uint32_t k = threadIdx.x; k < rd.var_blocks && !none; k += 256) v += rd.var_partial[k];
		s_v[threadIdx.x] = v;
		__syncthreads();
		for (uint32_t off = 128; off > 0; off >>= 1) {
			if (threadIdx.x < off) s_v[threadIdx.x] += s_v[threadIdx.x + off];
			__syncthreads();
		}
		if (threadIdx.x == 0 && rd.var_grad) *rd.var_grad = s_v[0];
		return;
	}
	__shared__ float s_part[4][64];
	const uint32_t p = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
	float a[4] = {0.f, 0.f, 0.f, 0.f};
	if (!none && p < rd.n_matrix) {
		const float* src = rd.partial + p;
		const size_t stride = rd.n_matrix;
		uint32_t b = g;
		for (; b + 12 < rd.n_blocks; b += 16) {
#pragma unroll
			for (int q = 0; q < 4; ++q) a[q] += src[(size_t)(b + 4 * q) * stride];
		}
		for (int q = 0; b < rd.n_blocks; b += 4, q = (q + 1) & 3) a[q] += src[(size_t)b * stride];
	}
	s_part[g][threadIdx.x & 63] = (a[0] + a[1]) + (a[2] + a[3]);
	__syncthreads();
	if (g == 0 && p < rd.n_matrix) {
		const uint32_t l = threadIdx.x;
		rd.g[p] = (s_part[0][l] + s_part[1][l]) + (s_part[2][l] + s_part[3][l]);
	}
}

// ------------------------------------------------------------------------------------------
// tcnn NetworkWithInputEncoding(HashGrid -> FullyFusedMLP, 1 hidden ReLU layer, linear 16-wide output) for the
// operator module (network_with_input_encoding.h:84-250; fully_fused_mlp.cu:678-812 forward, :967-1085 backward,
// :1088-1198 backward_backward_input). The MLP input is the encoding alone, padded to DE = next multiple of 16 of 2L
// (NetworkWithInputEncoding::set_alignment): logical row k = feature k of the paired encoding [L][n] half2.
//   MODE 0 forward : out [n][16] fp16 (the cpp::Module column-major view)
//   MODE 1 backward: dH0 = relu'(H0) . W1^T dL; dL/denc = W0^T dH0 -> paired; dW1 += dL H0^T, dW0 += dH0 din^T
//   MODE 2 bwd-bwd : b2 = relu'(H0) . W1^T dL; h1' = relu'(H0) . W0 u (u = dy/dx . dL_ddLdinput, paired);
//                    dW0 += b2 u^T, dW1 += dL h1'^T; g = W0^T b2 -> paired (the encoding's second-order operand)
// Weight gradients as in the training kernels: in registers, one partial row per block (k_mlp_grad_reduce).
// ------------------------------------------------------------------------------------------
template <int L> struct DimsE {
	static constexpr int DE = (2 * L + 15) / 16 * 16, DKS = DE / 16, DMT = (DE + 31) / 32;
};
template <int L, int W> struct DNetSmem {
	static constexpr int DE = DimsE<L>::DE;
	static constexpr int W0 = 0, W0T = W0 + W * (DE + 8), W1 = W0T + DE * (W + 8), W1T = W1 + 16 * (W + 8), END = W1T + W * (16 + 8);
};
template <int L>
__device__ __forceinline__ void build_din_enc(h8* dinB, const uint32_t* __restrict__ enc, uint32_t ld, uint32_t i, int h) {
	constexpr int DKS = DimsE<L>::DKS;
#pragma unroll
	for (int ks = 0; ks < DKS; ++ks)
#pragma unroll
		for (int j = 0; j < 8; ++j) {
			const int k = 16 * ks + (h ? pi_row(j, 1) : pi_row(j, 0));
			half_t v = (half_t)0.f;
			if (k < 2 * L) { const uint32_t u = enc[(size_t)(k >> 1) * ld + i]; v = __builtin_bit_cast(h2, u)[k & 1]; }
			dinB[ks][j] = v;
		}
}
// a DE-row accumulator set (rows 32 mt + acc_row) -> paired [L][ld] half2, rows < 2L
template <int L>
__device__ __forceinline__ void store_paired(uint32_t* out, uint32_t ld, uint32_t i, const f16v* a, int h) {
	constexpr int DMT = DimsE<L>::DMT;
	half_t* o = (half_t*)out;
#pragma unroll
	for (int mt = 0; mt < DMT; ++mt)
#pragma unroll
		for (int reg = 0; reg < 16; ++reg) {
			const int k = 32 * mt + acc_row(reg, h);
			if (k < 2 * L) o[((size_t)(k >> 1) * ld + i) * 2 + (k & 1)] = (half_t)a[mt][reg];
		}
}
struct DNetArgs {
	const half_t* w0; const half_t* w1;     // [W][DE], [16][W] fp16 (the module's parameters)
	const uint32_t* enc;                    // paired [L][n]
	const half_t* dL;                       // [n][16] fp16 (modes 1, 2)
	const uint32_t* u;                      // paired [L][n] (mode 2)
	half_t* out;                            // [n][16] (mode 0)
	uint32_t* denc;                         // paired [L][n] (modes 1, 2)
	float* wpartial;                        // [blocks][W DE + 16 W] (modes 1, 2)
};
template <int L, int W, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) k_dnet(uint32_t n, DNetArgs a) {
	constexpr int DE = DimsE<L>::DE, DKS = DimsE<L>::DKS, DMT = DimsE<L>::DMT;
	constexpr int MT = (W + 31) / 32, HKS = W / 16;
	using S = DNetSmem<L, W>;
	__shared__ half_t sm[smem_halves(S::END)];
	stage_mat(sm + S::W0, a.w0, W, DE);
	stage_mat(sm + S::W1, a.w1, 16, W);
	for (uint32_t e = threadIdx.x; e < (uint32_t)(W * DE); e += blockDim.x) {  // transposed copies
		const uint32_t r = e / DE, c = e % DE;
		sm[S::W0T + c * (W + 8) + r] = a.w0[e];
	}
	for (uint32_t e = threadIdx.x; e < (uint32_t)(16 * W); e += blockDim.x) {
		const uint32_t r = e / W, c = e % W;
		sm[S::W1T + c * (16 + 8) + r] = a.w1[e];
	}
	__syncthreads();
	const MatRef W0r{sm + S::W0, DE + 8}, W0Tr{sm + S::W0T, W + 8}, W1r{sm + S::W1, W + 8}, W1Tr{sm + S::W1T, 16 + 8};
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
	const h8 sel0 = transpose_sel(0), sel1 = transpose_sel(1);
	const h8 z8 = (h8){0, 0, 0, 0, 0, 0, 0, 0};
	f16v aW0[MT][DMT], aW1[MT];
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		aW1[mt] = zero16();
#pragma unroll
		for (int kt = 0; kt < DMT; ++kt) aW0[mt][kt] = zero16();
	}
	for (uint32_t base = wave * 32; base < n; base += n_waves * 32) {
		const uint32_t z = opaque_zero();
		const MatRef w0 = rebase(W0r, z), w0T = rebase(W0Tr, z), w1 = rebase(W1r, z), w1T = rebase(W1Tr, z);
		const uint32_t i = base + r;
		const bool valid = i < n;
		const uint32_t ic = valid ? i : 0;
		h8 dinB[DKS];
		build_din_enc<L>(dinB, a.enc, n, ic, h);
		h8 H0B[HKS];
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < DKS; ++ks) acc = mfma(loadA(w0, W, 32 * mt + r, 16 * ks, h), dinB[ks], acc);
			H0B[2 * mt] = frag<true>(acc, 0);
			if (2 * mt + 1 < HKS) H0B[2 * mt + 1] = frag<true>(acc, 1);
		}
		if (MODE == 0) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w1, 16, r, 16 * ks, h), H0B[ks], acc);
			if (valid)
#pragma unroll
				for (int reg = 0; reg < 8; ++reg) a.out[(size_t)i * 16 + acc_row(reg, h)] = (half_t)acc[reg];
			continue;
		}
		// dL [n][16] as a B fragment (rows pi_row(j, h)); 0 without a sample
		h8 dLB;
#pragma unroll
		for (int j = 0; j < 8; ++j) dLB[j] = valid ? a.dL[(size_t)ic * 16 + (h ? pi_row(j, 1) : pi_row(j, 0))] : (half_t)0.f;
		h8 dHB[HKS];  // relu'(H0) . W1^T dL (MODE 1: dH0; MODE 2: b2)
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) {
			const f16v acc = mfma(loadA(w1T, W, 32 * mt + r, 0, h), dLB, zero16());
			dHB[2 * mt] = mask_frag(acc, 0, H0B[2 * mt]);
			if (2 * mt + 1 < HKS) dHB[2 * mt + 1] = mask_frag(acc, 1, H0B[2 * mt + 1]);
		}
		// W0^T dHB -> paired (MODE 1: dL/denc; MODE 2: the encoding's second-order g)
		f16v dDin[DMT];
#pragma unroll
		for (int mt = 0; mt < DMT; ++mt) {
			f16v acc = zero16();
#pragma unroll
			for (int ks = 0; ks < HKS; ++ks) acc = mfma(loadA(w0T, DE, 32 * mt + r, 16 * ks, h), dHB[ks], acc);
			dDin[mt] = acc;
		}
		if (valid) store_paired<L>(a.denc, n, i, dDin, h);
		h8 TDL[2];
		transpose32(dLB, z8, false, sel0, sel1, TDL);
		h8 TDH[MT][2];
#pragma unroll
		for (int mt = 0; mt < MT; ++mt) transpose32(dHB[2 * mt], 2 * mt + 1 < HKS ? dHB[2 * mt + 1] : z8, 2 * mt + 1 < HKS, sel0, sel1, TDH[mt]);
		if (MODE == 1) {
			// dW1 += dL H0^T, dW0 += dH0 din^T
#pragma unroll
			for (int kt = 0; kt < MT; ++kt) {
				h8 TX[2];
				transpose32(H0B[2 * kt], 2 * kt + 1 < HKS ? H0B[2 * kt + 1] : z8, 2 * kt + 1 < HKS, sel0, sel1, TX);
				aW1[kt] = wg_acc(TDL, TX, aW1[kt]);
			}
#pragma unroll
			for (int kt = 0; kt < DMT; ++kt) {
				h8 TX[2];
				transpose32(dinB[2 * kt], 2 * kt + 1 < DKS ? dinB[2 * kt + 1] : z8, 2 * kt + 1 < DKS, sel0, sel1, TX);
#pragma unroll
				for (int mt = 0; mt < MT; ++mt) aW0[mt][kt] = wg_acc(TDH[mt], TX, aW0[mt][kt]);
			}
		} else {
			h8 uB[DKS];
			build_din_enc<L>(uB, a.u, n, ic, h);
			h8 H1pB[HKS];
#pragma unroll
			for (int mt = 0; mt < MT; ++mt) {
				f16v acc = zero16();
#pragma unroll
				for (int ks = 0; ks < DKS; ++ks) acc = mfma(loadA(w0, W, 32 * mt + r, 16 * ks, h), uB[ks], acc);
				H1pB[2 * mt] = mask_frag(acc, 0, H0B[2 * mt]);
				if (2 * mt + 1 < HKS) H1pB[2 * mt + 1] = mask_frag(acc, 1, H0B[2 * mt + 1]);
			}
			// dW0 += b2 u^T, dW1 += dL h1'^T
#pragma unroll
			for (int kt = 0; kt < DMT; ++kt) {
				h8 TX[2];
				transpose32(uB[2 * kt], 2 * kt + 1 < DKS ? uB[2 * kt + 1] : z8, 2 * kt + 1 < DKS, sel0, sel1, TX);
#pragma unroll
				for (int mt = 0; mt < MT; ++mt) aW0[mt][kt] = wg_acc(TDH[mt], TX, aW0[mt][kt]);
			}
#pragma unroll
			for (int kt = 0; kt < MT; ++kt) {
				h8 TX[2];
				transpose32(H1pB[2 * kt], 2 * kt + 1 < HKS ? H1pB[2 * kt + 1] : z8, 2 * kt + 1 < HKS, sel0, sel1, TX);
				aW1[kt] = wg_acc(TDL, TX, aW1[kt]);
			}
		}
	}
	if (MODE == 0) return;
	__syncthreads();
	float* red = (float*)sm;
	float* prow = a.wpartial + (size_t)blockIdx.x * (W * DE + 16 * W);
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
		for (int kt = 0; kt < DMT; ++kt) flush_tile(red, prow, aW0[mt][kt], 0u, W, DE, mt, kt);
		flush_tile(red, prow, aW1[mt], (uint32_t)(W * DE), 16, W, 0, mt);
	}
}

// MFMA fragment-layout probe (exact-integer check from tests): C = A(32x16) * B(16x32) with
// A, B given row-major, loaded in NATURAL k order.
__global__ void k_mfma_probe(const half_t* A, const half_t* B, float* C) {
	const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
	h8 a, b;
#pragma unroll
	for (int j = 0; j < 8; ++j) { a[j] = A[r * 16 + 8 * h + j]; b[j] = B[(8 * h + j) * 32 + r]; }
	f16v c = mfma(a, b, zero16());
#pragma unroll
	for (int reg = 0; reg < 16; ++reg) C[acc_row(reg, h) * 32 + r] = c[reg];
}

// Explicit instantiations used by the host (L levels, W hidden width).
// ---------------------------------------------------------------- host launchers
// Supported (levels, width) instantiations; the host checks mlp_supported() at reload time.
#define NEUS_MLP_CONFIGS(X) X(1, 16) X(1, 64) X(2, 64) X(4, 64) X(8, 64) X(14, 64) X(16, 64)

void mlp_din_permutation(uint32_t L, int32_t* perm) {
	const int DIN = ((3 + 2 * (int)L) + 15) / 16 * 16;
	for (int p = 0; p < DIN; ++p) perm[p] = -1;
	for (int h = 0; h < 2; ++h)
		for (int q = 0; q < DIN / 2; ++q) perm[din_physical_row(h, q)] = din_logical((int)L, h, q);
}

// blocks of `threads` that fit on the device at once (occupancy x CUs)
static uint32_t resident_blocks(const void* kernel, int threads) {
	int dev = 0, cus = 0, per_cu = 0;
	if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1u << 30;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu <= 0) return 1u << 30;
	return (uint32_t)(per_cu * cus);
}

bool mlp_supported(uint32_t L, uint32_t W) {
#define X(l, w) if (L == l && W == w) return true;
	NEUS_MLP_CONFIGS(X)
#undef X
	return false;
}

void launch_nerf_infer(hipStream_t s, uint32_t L, uint32_t W, const uint32_t* n_ptr, uint32_t n_fixed, const float* coords, const GridLevels& gl,
                       uint32_t valid_level, const half_t* grid, const MlpPtrs& w, half_t* out, uint32_t blocks, const uint32_t* idx,
                       const InferAlpha* ia) {
	InferAlpha a = ia ? *ia : InferAlpha{nullptr, nullptr, 0.f, 0u, nullptr};
	static const bool xcd_parts = [] { const char* e = std::getenv("NEUS_INFER_XCD_PARTS"); return e && e[0] == '1'; }();
	if (xcd_parts) a.xcd_parts = 8u;
	// persistent grid: at most the resident capacity (weights are staged once per block; both variants run at the
	// same 3 waves per SIMD, amdgpu_waves_per_eu)
	static const bool pipe = [] { const char* e = std::getenv("NEUS_INFER_PIPE"); return !(e && e[0] == '0'); }();
	const bool all = pipe && valid_level + 1 >= L;
	static const uint32_t grid_cap = [] { const char* e = std::getenv("NEUS_INFER_GRID"); return e ? (uint32_t)std::atoi(e) : 0u; }();  // (development)
	auto xg = [&](uint32_t b) { if (grid_cap) b = std::min(b, grid_cap); return a.xcd_parts ? std::max(8u, b & ~7u) : b; };
	dbg_lds_gate(s);
	const hipEvent_t ev0 = g_infer_ev[0], ev1 = g_infer_ev[1];
	g_infer_ev[0] = g_infer_ev[1] = nullptr;
	// (with timing events: the same launch through hipExtLaunchKernelGGL, which records them at the kernel's start and end)
	auto go = [&](auto kern, uint32_t nb, const uint32_t* ix) {
		if (ev0) hipExtLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, s, ev0, ev1, 0, n_ptr, n_fixed, coords, gl, valid_level, grid, w, out, ix, a);
		else kern<<<nb, 256, 0, s>>>(n_ptr, n_fixed, coords, gl, valid_level, grid, w, out, ix, a);
	};
#define X(l, w_) if (L == l && W == w_) { \
		static const uint32_t cap = resident_blocks((const void*)k_nerf_infer<l, w_, false>, 256); \
		static const uint32_t cap_all = resident_blocks((const void*)k_nerf_infer<l, w_, false, true>, 256); \
		if (all) { \
			if (idx) go(k_nerf_infer<l, w_, true, true>, xg(std::min(blocks, cap_all)), idx); \
			else go(k_nerf_infer<l, w_, false, true>, xg(std::min(blocks, cap_all)), nullptr); \
			return; } \
		if (idx) go(k_nerf_infer<l, w_, true>, xg(std::min(blocks, cap)), idx); \
		else go(k_nerf_infer<l, w_, false>, xg(std::min(blocks, cap)), nullptr); \
		return; }
	NEUS_MLP_CONFIGS(X)
#undef X
}
thread_local hipEvent_t g_infer_ev[2] = {nullptr, nullptr};
void launch_nerf_density(hipStream_t s, uint32_t L, uint32_t W, uint32_t n, const float* pos, const GridLevels& gl, uint32_t valid_level,
                         const half_t* grid, const MlpPtrs& w, float* density) {
	const uint32_t blocks = std::min<uint32_t>((n + 127) / 128, 8192);
	if (n == 0) return;
#define X(l, w_) if (L == l && W == w_) { k_nerf_density<l, w_, 0><<<blocks, 256, 0, s>>>(n, pos, UniformGrid{}, OccSampling{}, gl, valid_level, grid, w, density); return; }
	NEUS_MLP_CONFIGS(X)
#undef X
}
// One look-back scan tile per 4096 consecutive cells (16 per thread): each thread inverts the uniform hash for its
// cells, the kept ones (sample in [lo, hi)) are counted, scanned across the grid and written in cell order (no
// contended counter: a single list counter took ~370 us in 32K serialised wave atomics)
__global__ void __launch_bounds__(SCAN_THREADS) k_occ_uniform_list(uint32_t n_u, uint32_t step, uint32_t lo, uint32_t hi, uint32_t* __restrict__ list,
                                                                   ScanState* __restrict__ st, uint32_t tag) {
	__shared__ uint32_t s_prefix, s_wsum[SCAN_THREADS / 64];
	const ScanTile tl = scan_tile(tag);
	const uint32_t c0 = tl.tile * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
	// sample of cell c: (i + step n_u) = (c - 96925573) 53369 mod 2^21 (53369 = 56924617^-1 mod 2^21)
	auto sample_of = [&](uint32_t c) { return (((c - 96925573u) * 53369u) - step * n_u) & (GRID3 - 1u); };
	uint32_t keep = 0, cnt = 0;
#pragma unroll
	for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
		const uint32_t i = sample_of(c0 + k);
		const uint32_t b = (i >= lo && i < hi) ? 1u : 0u;
		keep |= b << k;
		cnt += b;
	}
	uint32_t agg;
	const uint32_t texcl = scan_block(cnt, s_wsum, agg);
	if (threadIdx.x < 64) {
		const uint32_t pre = scan_lookback(st, 0, tl, agg);
		if (threadIdx.x == 0) s_prefix = pre;
	}
	__syncthreads();
	uint32_t p = s_prefix + texcl;
#pragma unroll
	for (uint32_t k = 0; k < SCAN_ITEMS; ++k)
		if ((keep >> k) & 1u) list[p++] = sample_of(c0 + k);
}
void launch_occ_uniform_list(hipStream_t s, uint32_t n_u, uint32_t step, uint32_t lo, uint32_t hi, uint32_t* list, void* scan_tmp) {
	if (n_u > GRID3) throw std::runtime_error("launch_occ_uniform_list: more uniform samples than mip-0 cells");
	static_assert(GRID3 % SCAN_TILE == 0 && GRID3 / SCAN_TILE <= SCAN_MAX_TILES, "uniform list tiles");
	dbg_lds_gate(s);
	k_occ_uniform_list<<<GRID3 / SCAN_TILE, SCAN_THREADS, 0, s>>>(n_u, step, lo, hi, list, (ScanState*)scan_tmp, scan_next_tag(scan_tmp));
}
__global__ void __launch_bounds__(256) k_occ_nu_keys(uint32_t n, uint32_t g0, const OccSampling os, uint32_t* __restrict__ key,
                                                     uint32_t* __restrict__ hist) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
		const uint32_t i = g0 + k;
		pcg32 rng(os.rng_nu_state, os.rng_nu_inc);
		pcg_advance(rng, (uint64_t)(uint32_t)(i * 4), os.jt);
		const uint32_t idx = grid_sample_pick(os.n_nu, i, rng, os.step, os.grid_in, os.n_cascades, os.thresh_nu);
		const uint32_t b = (idx / GRID3) * 4096u + ((idx % GRID3) >> 9);
		key[k] = b;
		atomicAdd(&hist[b], 1u);
	}
}
__global__ void __launch_bounds__(256) k_occ_nu_place(uint32_t n, const uint32_t* __restrict__ key, uint32_t* __restrict__ cursor,
                                                      uint32_t* __restrict__ list) {
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) list[atomicAdd(&cursor[key[k]], 1u)] = k;
}
void launch_occ_nu_list(hipStream_t s, uint32_t n, uint32_t g0, const OccSampling& os, uint32_t* key, uint32_t* bins, uint32_t* list, void* scan_tmp,
                        size_t scan_tmp_bytes) {
	if (n == 0) return;
	const uint32_t nb = os.n_cascades * 4096u;
	if (hipMemsetAsync(bins, 0, (size_t)nb * 4, s) != hipSuccess) throw std::runtime_error("launch_occ_nu_list: memset failed");
	const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 2048);
	dbg_lds_gate(s);
	k_occ_nu_keys<<<blocks, 256, 0, s>>>(n, g0, os, key, bins);
	launch_exclusive_scan(s, scan_tmp, scan_tmp_bytes, bins, bins + nb, nb);
	k_occ_nu_place<<<blocks, 256, 0, s>>>(n, key, bins + nb, list);
}
void launch_occ_density(hipStream_t s, uint32_t L, uint32_t W, uint32_t n, const OccSampling& os, const GridLevels& gl, uint32_t valid_level,
                        const half_t* grid, const MlpPtrs& w) {
	const uint32_t blocks = std::min<uint32_t>((n + 127) / 128, 8192);
	if (n == 0) return;
	dbg_lds_gate(s);
#define X(l, w_) if (L == l && W == w_) { k_nerf_density<l, w_, 2><<<blocks, 256, 0, s>>>(n, nullptr, UniformGrid{}, os, gl, valid_level, grid, w, nullptr); return; }
	NEUS_MLP_CONFIGS(X)
#undef X
}
void launch_sdf_grid(hipStream_t s, uint32_t L, uint32_t W, const uint32_t res[3], const float render_min[3], const float render_max[3],
                     const float train_min[3], const float train_max[3], uint64_t offset, uint32_t n, const GridLevels& gl, uint32_t valid_level,
                     const half_t* grid, const MlpPtrs& w, float* sdf, const DeltaState* delta) {
	if (n == 0) return;
	UniformGrid ug{};
	ug.delta = delta;
	for (int k = 0; k < 3; ++k) {
		ug.res[k] = res[k]; ug.inv_res[k] = 1.f / (float)res[k];
		ug.rmin[k] = render_min[k]; ug.rdiag[k] = render_max[k] - render_min[k];
		ug.tmin[k] = train_min[k]; ug.tdiag[k] = train_max[k] - train_min[k];
	}
	ug.offset = offset;
	const uint32_t blocks = std::min<uint32_t>((n + 127) / 128, 16384);
#define X(l, w_) if (L == l && W == w_) { k_nerf_density<l, w_, 1><<<blocks, 256, 0, s>>>(n, nullptr, ug, OccSampling{}, gl, valid_level, grid, w, sdf); return; }
	NEUS_MLP_CONFIGS(X)
#undef X
}
void launch_mlp_train(hipStream_t s, uint32_t L, uint32_t W, const uint32_t* n_valid_ptr, uint32_t n, uint32_t ld, const float* coords,
                      const half_t* enc, const float* dydx, const half_t* dL_dout, const MlpPtrs& w, const TrainBufs& tb, int part) {
	const uint32_t blocks = mlp_train_blocks(L, W, n);
	if (n == 0) return;
#define X(l, w_) if (L == l && W == w_) { \
		dbg_lds_gate(s); \
		if (part != 2) k_mlp_train_rgb<l, w_><<<blocks, 256, 0, s>>>(n_valid_ptr, n, ld, coords, enc, dydx, dL_dout, w, tb); \
		dbg_lds_gate(s); \
		if (part != 1) k_mlp_train_density<l, w_><<<blocks, 256, 0, s>>>(n_valid_ptr, n, ld, coords, enc, dydx, w, tb); return; }
	NEUS_MLP_CONFIGS(X)
#undef X
}
void launch_mlp_grad_reduce(hipStream_t s, const MlpGradReduce& r) {
	dbg_lds_gate(s);
	k_mlp_grad_reduce<<<(r.n_matrix + 63) / 64 + 1, 256, 0, s>>>(r);
}
// persistent grid: at most the resident capacity of the two training kernels, so the ~53 KB weight staging runs
// once per block (one wave per SIMD: a grid of n / 128 blocks re-staged the weights for every 128 samples)
uint32_t mlp_train_blocks(uint32_t L, uint32_t W, uint32_t n) {
	uint32_t cap = 2048;
#define X(l, w_) if (L == l && W == w_) { \
		static const uint32_t c = std::min(resident_blocks((const void*)k_mlp_train_rgb<l, w_>, 256), \
		                                   resident_blocks((const void*)k_mlp_train_density<l, w_>, 256)); \
		cap = std::min(cap, c); }
	NEUS_MLP_CONFIGS(X)
#undef X
	static const uint32_t pct = [] { const char* e = std::getenv("NEUS_MLP_BLOCKS_PCT"); return e ? (uint32_t)std::atoi(e) : 100u; }();
	if (pct > 0 && pct != 100) cap = std::max<uint32_t>(1, cap * pct / 100);  // development: a smaller (or over-decomposed) grid
	return std::max<uint32_t>(1, std::min<uint32_t>((n + 127) / 128, cap));
}
void launch_mfma_probe(hipStream_t s, const half_t* A, const half_t* B, float* C) { k_mfma_probe<<<1, 64, 0, s>>>(A, B, C); }

#define NEUS_DNET_CONFIGS(X) X(1, 16) X(1, 64) X(2, 64) X(4, 64) X(8, 64) X(14, 64) X(16, 64)
bool dnet_supported(uint32_t L, uint32_t W) {
#define X(l, w) if (L == l && W == w) return true;
	NEUS_DNET_CONFIGS(X)
#undef X
	return false;
}
uint32_t dnet_blocks(uint32_t n) { return std::max<uint32_t>(1, std::min<uint32_t>((n + 127) / 128, 512)); }
void launch_dnet(hipStream_t s, uint32_t L, uint32_t W, int mode, uint32_t n, const DNetLaunch& d) {
	if (n == 0) return;
	DNetArgs a{d.w0, d.w1, d.enc, d.dL, d.u, d.out, d.denc, d.wpartial};
	const uint32_t blocks = dnet_blocks(n);
#define X(l, w_) if (L == l && W == w_) { \
		if (mode == 0) k_dnet<l, w_, 0><<<blocks, 256, 0, s>>>(n, a); \
		else if (mode == 1) k_dnet<l, w_, 1><<<blocks, 256, 0, s>>>(n, a); \
		else k_dnet<l, w_, 2><<<blocks, 256, 0, s>>>(n, a); \
		return; }
	NEUS_DNET_CONFIGS(X)
#undef X
	throw std::runtime_error("density network module: unsupported (n_levels, n_neurons)");
}

} // namespace neus
