// Global movement of the dynamic-scene path on gfx950.
//
//   k_delta_prepare : DeltaNetwork params (transition[4] | rotation 6D[8], read as fp16 like the reference's
//                     TrainableBuffer<T = half>) -> rotation matrix, its inverse and the translation
//                     (rotation_6d_to_matrix, common_operation.cuh:37-60)
//   k_delta_apply   : add_global_movement_with_rotation_6d (common_operation.cuh:416-492) on NerfCoordinate
//                     records (pos' = R (pos + t), dir' = (R (2 dir - 1) + 1) / 2) or on NerfPosition records
//   k_delta_grad    : add_loss_to_rotation_6d_each (common_operation.cuh:788-845) per training sample, the
//                     per-sample values rounded to fp16 (the reference's T buffers), block partial sums
//   k_delta_step    : fixed-order final sum (the reduce_sum calls of transform_network.h:206-245) and the
//                     global-move trainer's ExponentialDecay(Adam) step on the delta parameters (adam.h:51-160)
//
// The delta parameters live on the device and are updated there: a dynamic training step has no host sync.
// The accumulated movement that moves the training rays (global_movement_with_rotation_6d,
// testbed_nerf.cu:193-213) changes only at a frame switch and travels by value in DevDataset::motion.
// Compiled with -ffp-contract=off: the oracle restates the same expressions.
#include "kernels.h"

#include <algorithm>
#include <cmath>

namespace neus {

// rotation_6d_to_matrix: b1 = a1/|a1|, b2 = (a2 - (b1.a2) b1)/|..|, b3 = b1 x b2; columns b1, b2, b3 (row-major out).
NEUS_HD void rot6d_to_matrix(const float r6[6], float R[9]) {
	const float a1[3] = {r6[0], r6[1], r6[2]}, a2[3] = {r6[3], r6[4], r6[5]};
	const float n1 = sqrtf((a1[0] * a1[0] + a1[1] * a1[1]) + a1[2] * a1[2]);
	const float b1[3] = {a1[0] / n1, a1[1] / n1, a1[2] / n1};
	const float d = (b1[0] * a2[0] + b1[1] * a2[1]) + b1[2] * a2[2];
	const float u[3] = {a2[0] - d * b1[0], a2[1] - d * b1[1], a2[2] - d * b1[2]};
	const float n2 = sqrtf((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
	const float b2[3] = {u[0] / n2, u[1] / n2, u[2] / n2};
	const float b3[3] = {b1[1] * b2[2] - b1[2] * b2[1], b1[2] * b2[0] - b1[0] * b2[2], b1[0] * b2[1] - b1[1] * b2[0]};
	for (int k = 0; k < 3; ++k) { R[3 * k + 0] = b1[k]; R[3 * k + 1] = b2[k]; R[3 * k + 2] = b3[k]; }
}

// 3x3 inverse by cofactors (Eigen's Matrix3f::inverse for the rotation's inverse)
NEUS_HD void inverse3(const float m[9], float o[9]) {
	const float c00 = m[4] * m[8] - m[5] * m[7], c01 = m[5] * m[6] - m[3] * m[8], c02 = m[3] * m[7] - m[4] * m[6];
	const float det = (m[0] * c00 + m[1] * c01) + m[2] * c02;
	const float id = 1.0f / det;
	o[0] = c00 * id; o[1] = (m[2] * m[7] - m[1] * m[8]) * id; o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
	o[3] = c01 * id; o[4] = (m[0] * m[8] - m[2] * m[6]) * id; o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
	o[6] = c02 * id; o[7] = (m[1] * m[6] - m[0] * m[7]) * id; o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

NEUS_HD void matvec3(const float R[9], const float v[3], float o[3]) {
	for (int k = 0; k < 3; ++k) o[k] = (R[3 * k] * v[0] + R[3 * k + 1] * v[1]) + R[3 * k + 2] * v[2];
}

__global__ void k_delta_prepare(DeltaState* ds) {
	if (threadIdx.x != 0 || blockIdx.x != 0) return;
	float r6[6];
	for (int k = 0; k < 6; ++k) r6[k] = (float)(half_t)ds->p[4 + k];
	rot6d_to_matrix(r6, ds->R);
	inverse3(ds->R, ds->Rinv);
	for (int k = 0; k < 3; ++k) ds->t[k] = (float)(half_t)ds->p[k];
}

// in == out is allowed (each record is read before it is written by the same thread)
template <int STRIDE>
__global__ void __launch_bounds__(256) k_delta_apply(const uint32_t* __restrict__ n_ptr, uint32_t n_cap, const float* in, float* out,
                                                     const DeltaState* __restrict__ dst) {
	const uint32_t n = n_ptr ? min(*n_ptr, n_cap) : n_cap;
	float R[9], t[3];
#pragma unroll
	for (int k = 0; k < 9; ++k) R[k] = dst->R[k];
#pragma unroll
	for (int k = 0; k < 3; ++k) t[k] = dst->t[k];
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const float* c = in + (size_t)i * STRIDE;
		float* o = out + (size_t)i * STRIDE;
		float v[STRIDE];
#pragma unroll
		for (int k = 0; k < STRIDE; ++k) v[k] = c[k];
		const float p[3] = {v[0] + t[0], v[1] + t[1], v[2] + t[2]};
		float q[3]; matvec3(R, p, q);
		o[0] = q[0]; o[1] = q[1]; o[2] = q[2];
		if (STRIDE == COORD_W) {
			o[3] = v[3];
			const float d[3] = {v[4] * 2.0f - 1.0f, v[5] * 2.0f - 1.0f, v[6] * 2.0f - 1.0f};
			float e[3]; matvec3(R, d, e);
			o[4] = (e[0] + 1.0f) * 0.5f; o[5] = (e[1] + 1.0f) * 0.5f; o[6] = (e[2] + 1.0f) * 0.5f;
		}
	}
}

// gradient_rotation_matrix_to_6d (common_operation.cuh:62-157): the d_b1 / d_b2 accumulators are T (fp16) in
// the reference, the Vector3f intermediates fp32. G is the row-major 3x3 gradient of the rotation matrix.
NEUS_HD void grad_rot6d(const float r6[6], const float G[9], float g6[6]) {
	const float a1[3] = {r6[0], r6[1], r6[2]}, a2[3] = {r6[3], r6[4], r6[5]};
	const float n1 = sqrtf((a1[0] * a1[0] + a1[1] * a1[1]) + a1[2] * a1[2]);
	const float b1[3] = {a1[0] / n1, a1[1] / n1, a1[2] / n1};
	const float dd = (b1[0] * a2[0] + b1[1] * a2[1]) + b1[2] * a2[2];
	const float u[3] = {a2[0] - dd * b1[0], a2[1] - dd * b1[1], a2[2] - dd * b1[2]};
	const float n2 = sqrtf((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
	const float b2[3] = {u[0] / n2, u[1] / n2, u[2] / n2};
	float db1[3], db2[3];
	db1[0] = rh(G[0]); db1[1] = rh(G[3]); db1[2] = rh(G[6]);
	db2[0] = rh(G[1]); db2[1] = rh(G[4]); db2[2] = rh(G[7]);
	db1[0] = rh(db1[0] + (b2[1] * G[8] - b2[2] * G[5]));
	db1[1] = rh(db1[1] + (b2[2] * G[2] - b2[0] * G[8]));
	db1[2] = rh(db1[2] + (b2[0] * G[5] - b2[1] * G[2]));
	db2[0] = rh(db2[0] + (b1[2] * G[5] - b1[1] * G[8]));
	db2[1] = rh(db2[1] + (b1[0] * G[8] - b1[2] * G[2]));
	db2[2] = rh(db2[2] + (b1[1] * G[2] - b1[0] * G[5]));
	// gradients_for_normalize(v, g) (:62-90): J(v) g, J = (|v|^2 I - v v^T) / |v|^3
	float r[3], da1[3];
	{
		const float* v = u; const float* g = db2;
		const float nn = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]), n3 = nn * nn * nn;
		r[0] = g[0] * ((v[1] * v[1] + v[2] * v[2]) / n3) + g[1] * (-v[0] * v[1] / n3) + g[2] * (-v[0] * v[2] / n3);
		r[1] = g[0] * (-v[0] * v[1] / n3) + g[1] * ((v[0] * v[0] + v[2] * v[2]) / n3) + g[2] * (-v[1] * v[2] / n3);
		r[2] = g[0] * (-v[0] * v[2] / n3) + g[1] * (-v[1] * v[2] / n3) + g[2] * ((v[0] * v[0] + v[1] * v[1]) / n3);
	}
	float da2[3] = {r[0], r[1], r[2]};
	da2[0] += -r[0] * b1[0] * b1[0] - r[1] * b1[0] * b1[1] - r[2] * b1[0] * b1[2];
	da2[1] += -r[0] * b1[0] * b1[1] - r[1] * b1[1] * b1[1] - r[2] * b1[2] * b1[1];
	da2[2] += -r[0] * b1[0] * b1[2] - r[1] * b1[1] * b1[2] - r[2] * b1[2] * b1[2];
	float d1[3] = {db1[0], db1[1], db1[2]};
	d1[0] += -r[0] * (2.0f * b1[0] * a2[0] + b1[1] * a2[1] + b1[2] * a2[2]) - r[1] * b1[1] * a2[0] - r[2] * b1[2] * a2[0];
	d1[1] += -r[1] * (2.0f * b1[1] * a2[1] + b1[0] * a2[0] + b1[2] * a2[2]) - r[0] * b1[0] * a2[1] - r[2] * b1[2] * a2[1];
	d1[2] += -r[2] * (2.0f * b1[2] * a2[2] + b1[0] * a2[0] + b1[1] * a2[1]) - r[0] * b1[0] * a2[2] - r[1] * b1[1] * a2[2];
	{
		const float* v = a1; const float* g = d1;
		const float nn = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]), n3 = nn * nn * nn;
		da1[0] = g[0] * ((v[1] * v[1] + v[2] * v[2]) / n3) + g[1] * (-v[0] * v[1] / n3) + g[2] * (-v[0] * v[2] / n3);
		da1[1] = g[0] * (-v[0] * v[1] / n3) + g[1] * ((v[0] * v[0] + v[2] * v[2]) / n3) + g[2] * (-v[1] * v[2] / n3);
		da1[2] = g[0] * (-v[0] * v[2] / n3) + g[1] * (-v[1] * v[2] / n3) + g[2] * ((v[0] * v[0] + v[1] * v[1]) / n3);
	}
	g6[0] = da1[0]; g6[1] = da1[1]; g6[2] = da1[2];
	g6[3] = da2[0]; g6[4] = da2[1]; g6[5] = da2[2];
}

// Per training sample i < n: g = dL/d(deformed position) (dpos, float4), x = the undeformed position (coords);
// transition gradient R^-1 g, rotation gradient d6D of G = g (x + t)^T, each rounded to fp16 per sample
// (dL_dtransition_each / dL_drotation_quat_each are T matrices); per-block sums in a fixed tree.
constexpr uint32_t DELTA_BLOCKS = 256;
__global__ void __launch_bounds__(256) k_delta_grad(const uint32_t* __restrict__ n_ptr, uint32_t n_cap, const float* __restrict__ coords,
                                                    uint32_t stride, const float4* __restrict__ dpos, const DeltaState* __restrict__ dst,
                                                    float* __restrict__ partial /* [DELTA_BLOCKS][9] */) {
	const uint32_t n = n_ptr ? min(*n_ptr, n_cap) : n_cap;
	__shared__ float red[9][256];
	float Ri[9], t[3], r6[6];
#pragma unroll
	for (int k = 0; k < 9; ++k) Ri[k] = dst->Rinv[k];
#pragma unroll
	for (int k = 0; k < 3; ++k) t[k] = dst->t[k];
#pragma unroll
	for (int k = 0; k < 6; ++k) r6[k] = (float)(half_t)dst->p[4 + k];
	float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const float4 g4 = dpos[i];
		const float g[3] = {g4.x, g4.y, g4.z};
		const float* c = coords + (size_t)i * stride;
		const float x[3] = {c[0] + t[0], c[1] + t[1], c[2] + t[2]};
		float gt[3]; matvec3(Ri, g, gt);
		float G[9];
#pragma unroll
		for (int a = 0; a < 3; ++a)
#pragma unroll
			for (int b = 0; b < 3; ++b) G[3 * a + b] = g[a] * x[b];
		float g6[6]; grad_rot6d(r6, G, g6);
#pragma unroll
		for (int k = 0; k < 3; ++k) acc[k] += rh(gt[k]);
#pragma unroll
		for (int k = 0; k < 6; ++k) acc[3 + k] += rh(g6[k]);
	}
#pragma unroll
	for (int k = 0; k < 9; ++k) red[k][threadIdx.x] = acc[k];
	__syncthreads();
	for (uint32_t off = 128; off > 0; off >>= 1) {
		if (threadIdx.x < off)
#pragma unroll
			for (int k = 0; k < 9; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + off];
		__syncthreads();
	}
	if (threadIdx.x < 9) partial[blockIdx.x * 9 + threadIdx.x] = red[threadIdx.x][0];
}

// Final sum in block order -> fp16 gradients in the parameter layout (transition 0..2, rotation 4..9), then
// (a.optimize) the global-move trainer step: gradient / loss_scale, non-matrix parameters (no L2, exactly-zero
// gradients skipped, adam.h:109-112), per-parameter bias correction, AdaBound clamp.
__global__ void __launch_bounds__(64) k_delta_step(const float* __restrict__ partial, uint32_t n_partial, DeltaState* ds, DeltaAdam a) {
	__shared__ float g[DELTA_PARAMS];
	if (threadIdx.x < DELTA_PARAMS) g[threadIdx.x] = 0.f;
	__syncthreads();
	if (threadIdx.x < 9) {
		float s = 0.f;
		for (uint32_t b = 0; b < n_partial; ++b) s += partial[b * 9 + threadIdx.x];
		const uint32_t slot = threadIdx.x < 3 ? threadIdx.x : 4 + (threadIdx.x - 3);
		g[slot] = rh(s);
	}
	__syncthreads();
	if (threadIdx.x < DELTA_PARAMS) {
		const uint32_t i = threadIdx.x;
		ds->grad[i] = g[i];
		const float gradient = g[i] / a.loss_scale;
		if (a.optimize && gradient != 0.f) {
			const float fm = a.beta1 * ds->m1[i] + (1 - a.beta1) * gradient;
			const float sm = a.beta2 * ds->m2[i] + (1 - a.beta2) * (gradient * gradient);
			ds->m1[i] = fm; ds->m2[i] = sm;
			const uint32_t cs = ds->steps[i] + 1;
			ds->steps[i] = cs;
			const float lr = a.lr * sqrtf(1 - powf(a.beta2, (float)cs)) / (1 - powf(a.beta1, (float)cs));
			const float elr = fminf(fmaxf(lr / (sqrtf(sm) + a.eps), 0.0f), 3.402823466e+38f);
			ds->p[i] = ds->p[i] - elr * fm;
		}
	}
}

// ---------------------------------------------------------------- host launchers
void launch_delta_prepare(hipStream_t s, DeltaState* ds) { k_delta_prepare<<<1, 64, 0, s>>>(ds); }
void launch_delta_apply(hipStream_t s, const uint32_t* n_ptr, uint32_t n_cap, uint32_t stride, const float* in, float* out, const DeltaState* ds) {
	if (n_cap == 0) return;
	const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((n_cap + 255) / 256, 4096));
	if (stride == COORD_W) k_delta_apply<COORD_W><<<blocks, 256, 0, s>>>(n_ptr, n_cap, in, out, ds);
	else k_delta_apply<3><<<blocks, 256, 0, s>>>(n_ptr, n_cap, in, out, ds);
}
void launch_delta_backward(hipStream_t s, const uint32_t* n_ptr, uint32_t n_cap, const float* coords, uint32_t stride, const float4* dpos,
                           DeltaState* ds, float* partial, const DeltaAdam& a) {
	k_delta_grad<<<DELTA_BLOCKS, 256, 0, s>>>(n_ptr, n_cap, coords, stride, dpos, ds, partial);
	k_delta_step<<<1, 64, 0, s>>>(partial, DELTA_BLOCKS, ds, a);
}
void launch_delta_grad(hipStream_t s, const uint32_t* n_ptr, uint32_t n_cap, const float* coords, uint32_t stride, const float4* dpos,
                       const DeltaState* ds, float* partial) {
	k_delta_grad<<<DELTA_BLOCKS, 256, 0, s>>>(n_ptr, n_cap, coords, stride, dpos, ds, partial);
}
void launch_delta_step(hipStream_t s, const float* partial, DeltaState* ds, const DeltaAdam& a) {
	k_delta_step<<<1, 64, 0, s>>>(partial, DELTA_BLOCKS, ds, a);
}
size_t delta_partial_floats() { return (size_t)DELTA_BLOCKS * 9; }

// accumulate_global_movement_rotation_6d_kernel (common_operation.cuh:551-585), run on the host at a frame
// switch: R_acc <- R_local R_acc, t_acc <- R_local (t_acc + t_local); stored fp16-rounded like the reference's
// accumulated TrainableBuffer<T = half>.
void host_accumulate_movement(const float delta_p[DELTA_PARAMS], float accR[9], float acct[3]) {
	float r6[6], R[9];
	for (int k = 0; k < 6; ++k) r6[k] = rh(delta_p[4 + k]);
	rot6d_to_matrix(r6, R);
	float nR[9], nt[3];
	for (int i = 0; i < 3; ++i)
		for (int j = 0; j < 3; ++j) nR[3 * i + j] = (R[3 * i] * accR[j] + R[3 * i + 1] * accR[3 + j]) + R[3 * i + 2] * accR[6 + j];
	const float v[3] = {acct[0] + rh(delta_p[0]), acct[1] + rh(delta_p[1]), acct[2] + rh(delta_p[2])};
	matvec3(R, v, nt);
	for (int k = 0; k < 9; ++k) accR[k] = rh(nR[k]);
	for (int k = 0; k < 3; ++k) acct[k] = rh(nt[k]);
}

} // namespace neus
