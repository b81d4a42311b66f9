// Device helpers shared by the training march/loss (march.hip) and the renderer (render.hip):
// the reference's march constants and voxel stepping (testbed_nerf.cu:149-164, 356-378, 494-530,
// 624-638), image access, AABB tests, one march step, the NeuS SDF-to-alpha and the network-output
// readers. Included only by files compiled with -ffp-contract=off (bit parity with the oracle).
#pragma once
#pragma clang fp contract(off)
#include "kernels.h"

namespace neus {

__device__ __forceinline__ float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ float calc_dt(float t, float cone) { return clampf(t * cone, MIN_CONE_STEPSIZE, MAX_CONE_STEPSIZE); }
__device__ __forceinline__ float warp_dt(float dt) {
	const float max_stepsize = MIN_CONE_STEPSIZE * (1 << (NERF_CASCADES - 1));
	return (dt - MIN_CONE_STEPSIZE) / (max_stepsize - MIN_CONE_STEPSIZE);
}
__device__ __forceinline__ float unwarp_dt(float dt) {
	const float max_stepsize = MIN_CONE_STEPSIZE * (1 << (NERF_CASCADES - 1));
	return dt * (max_stepsize - MIN_CONE_STEPSIZE) + MIN_CONE_STEPSIZE;
}
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ uint32_t cascaded_grid_idx_at(float px, float py, float pz, uint32_t mip) {
	const float s = scalbnf(1.0f, -(int)mip);
	px = ((px - 0.5f) * s) + 0.5f; py = ((py - 0.5f) * s) + 0.5f; pz = ((pz - 0.5f) * s) + 0.5f;
	const int ix = (int)(px * NERF_GRIDSIZE), iy = (int)(py * NERF_GRIDSIZE), iz = (int)(pz * NERF_GRIDSIZE);
	return morton3D(clampi(ix, 0, NERF_GRIDSIZE - 1), clampi(iy, 0, NERF_GRIDSIZE - 1), clampi(iz, 0, NERF_GRIDSIZE - 1));
}
__device__ __forceinline__ bool occupied(float px, float py, float pz, const uint8_t* bf, uint32_t mip) {
	const uint32_t idx = cascaded_grid_idx_at(px, py, pz, mip);
	return bf[idx / 8 + GRID3 * mip / 8] & (1 << (idx % 8));
}
__device__ __forceinline__ int mip_from_pos(float px, float py, float pz) {
	int e;
	const float m = fmaxf(fmaxf(fabsf(px - 0.5f), fabsf(py - 0.5f)), fabsf(pz - 0.5f));
	frexpf(m, &e);
	return min((int)NERF_CASCADES - 1, max(0, e + 1));
}
__device__ __forceinline__ int mip_from_dt(float dt, float px, float py, float pz) {
	const int mip = mip_from_pos(px, py, pz);
	dt *= 2 * NERF_GRIDSIZE;
	if (dt < 1.f) return mip;
	int e; frexpf(dt, &e);
	return min((int)NERF_CASCADES - 1, max(e, mip));
}
// Exactly `while (t < target && k < kmax) { t += dt; ++k; }` for a constant dt > 0 and a finite t >= 0, in a few
// iterations per binade instead of one per step. Inside a binade [2^e, 2^(e+1)) every float is a multiple of its ulp,
// so t + dt rounds to t plus a fixed number of ulps - once the parity of t's significand is settled: a tie
// (dt / ulp = n + 1/2) rounds to the even neighbour, after which the increment stays fixed. Two exact steps that add the
// same increment prove the stretch linear; it is then jumped in the integer domain (positive floats order as their
// bit patterns) up to the first step at or past target, the step cap or the binade's end, whichever comes first.
// Single exact steps cross binades and settle the parity.
// Precondition checked: with t negative or not finite the jumps' integer arithmetic is meaningless (and the plain loop
// could spin without end), so nothing is stepped and false is returned: the caller ends the ray, and the march's exit
// check (a non-finite / negative t at a segment's end) raises STEP_FAIL_MARCH_T. dt: the constant step (> 0).
__device__ __forceinline__ bool step_until(float& t, uint32_t& k, float target, uint32_t kmax, float dt) {
	if (!(t >= 0.0f) || !(t < __builtin_huge_valf())) return false;
	while (t < target && k < kmax) {
		const float t2 = t + dt;
		const uint32_t b = __float_as_uint(t), b2 = __float_as_uint(t2), ex = b & 0x7f800000u;
		if (!(t2 < target) || k + 1u >= kmax || ex == 0u || (b2 & 0x7f800000u) != ex) { t = t2; ++k; continue; }
		const float t3 = t2 + dt;
		const uint32_t b3 = __float_as_uint(t3), inc = b2 - b;
		if (b3 - b2 != inc || (b3 & 0x7f800000u) != ex) { t = t2; ++k; continue; }
		const uint32_t e_end = ex + 0x00800000u;  // the next binade's first bit pattern
		const uint32_t tb = __float_as_uint(target);
		// j = min(the first step at or past target, the last step inside the binade) (both >= 2: t2 < target, t3 is inside),
		// with one division when the first is inside the binade
		uint32_t j = tb < e_end ? (tb - b + inc - 1u) / inc : 0xffffffffu;
		if (j == 0xffffffffu || b + j * inc >= e_end) j = (e_end - 1u - b) / inc;
		j = min(j, kmax - k);
		t = __uint_as_float(b + j * inc);
		k += j;
	}
	return true;
}
__device__ __forceinline__ float signf(float x) { return copysignf(1.0f, x); }
__device__ __forceinline__ float advance_to_next_voxel(float t, float cone, const float pos[3], const float dir[3], const float idir[3], uint32_t res) {
	float p[3], tt[3];
#pragma unroll
	for (int d = 0; d < 3; ++d) { p[d] = res * pos[d]; tt[d] = (floorf(p[d] + 0.5f + 0.5f * signf(dir[d])) - p[d]) * idir[d]; }
	const float tn = fminf(fminf(tt[0], tt[1]), tt[2]);
	const float t_target = t + fmaxf(tn / res, 0.0f);
	do { t += calc_dt(t, cone); } while (t < t_target);
	return t;
}
__device__ __forceinline__ float srgb_to_linear(float s) { return s <= 0.04045f ? s / 12.92f : powf((s + 0.055f) / 1.055f, 2.4f); }
__device__ __forceinline__ float linear_to_srgb(float l) { return l < 0.0031308f ? 12.92f * l : 1.055f * powf(l, 0.41666f) - 0.055f; }

__device__ __forceinline__ uint32_t image_idx(uint32_t base_idx, uint32_t n_rays, uint32_t n_rays_total, uint32_t n_img) {
	return (((base_idx + n_rays_total) * n_img) / n_rays) % n_img;
}
__device__ __forceinline__ void random_image_pos(pcg32& rng, int rx, int ry, float& x, float& y) {
	x = rng.next_float(); y = rng.next_float();
	const int ix = min(max((int)(x * (float)rx), 0), rx - 1);
	const int iy = min(max((int)(y * (float)ry), 0), ry - 1);
	x = ((float)ix + 0.5f) / (float)rx; y = ((float)iy + 0.5f) / (float)ry;
}
// read_rgba (ngp common_device.cuh:635-667), Byte path: premultiplied linear rgb, alpha
__device__ __forceinline__ void read_rgba(const DevDataset& ds, uint32_t img, float x, float y, float o[4]) {
	const int rx = ds.res[2 * img], ry = ds.res[2 * img + 1];
	const int px = clampi((int)(x * (float)rx), 0, rx - 1), py = clampi((int)(y * (float)ry), 0, ry - 1);
	const uint32_t v = ds.pixels[ds.pix_off[img] + (uint64_t)px + (uint64_t)py * rx];
	if (v == 0x00FF00FFu) { o[0] = o[1] = o[2] = o[3] = -1.0f; return; }
	const float a = (float)((v >> 24) & 0xff) * (1.0f / 255.0f);
	// srgb_to_linear((float)byte * (1 / 255)) from the dataset's 256-entry table (the same expression, evaluated once
	// per value by k_srgb_lut: bit-identical, without a powf per channel)
	o[0] = ds.lin_lut[v & 0xff] * a;
	o[1] = ds.lin_lut[(v >> 8) & 0xff] * a;
	o[2] = ds.lin_lut[(v >> 16) & 0xff] * a;
	o[3] = a;
}
__device__ __forceinline__ bool aabb_contains(const DevDataset& ds, const float p[3]) {
	// bitwise: no short-circuit branches in the march loop (same predicate)
	return (p[0] >= ds.aabb_min[0]) & (p[0] <= ds.aabb_max[0]) & (p[1] >= ds.aabb_min[1]) & (p[1] <= ds.aabb_max[1]) &
	       (p[2] >= ds.aabb_min[2]) & (p[2] <= ds.aabb_max[2]);
}
__device__ __forceinline__ void ray_intersect(const DevDataset& ds, const float o[3], const float d[3], float& tmin_o) {
	float tmin = (ds.aabb_min[0] - o[0]) / d[0], tmax = (ds.aabb_max[0] - o[0]) / d[0];
	if (tmin > tmax) { float t = tmin; tmin = tmax; tmax = t; }
	float tymin = (ds.aabb_min[1] - o[1]) / d[1], tymax = (ds.aabb_max[1] - o[1]) / d[1];
	if (tymin > tymax) { float t = tymin; tymin = tymax; tymax = t; }
	const float FM = 3.402823466e+38f;
	if (tmin > tymax || tymin > tmax) { tmin_o = FM; return; }
	if (tymin > tmin) tmin = tymin;
	if (tymax < tmax) tmax = tymax;
	float tzmin = (ds.aabb_min[2] - o[2]) / d[2], tzmax = (ds.aabb_max[2] - o[2]) / d[2];
	if (tzmin > tzmax) { float t = tzmin; tzmin = tzmax; tzmax = t; }
	if (tmin > tzmax || tzmin > tmax) { tmin_o = FM; return; }
	if (tzmin > tmin) tmin = tzmin;
	tmin_o = tmin;
}

struct MarchRay { float o[3], dir[3], idir[3]; };

// One iteration of the reference's march loop body (testbed_nerf.cu:1376-1405) with the same float
// operation sequence: returns 0 once the ray has left the AABB, 1 at an occupied sample (pos and dt
// set; the caller steps t += dt), 2 after skipping an empty voxel (t advanced). The loops around it
// stay flat (one sample-or-skip per iteration) so lanes of a wave do not wait on each other's skips.
// FAST: cone_angle == 0 (aabb_scale 1): constant dt, mip 0 answered from the linear bitfield, mip > 0
// (only the exact box centre and faces) from the Morton one.
template <bool FAST>
__device__ __forceinline__ int march_step(const DevDataset& ds, const uint8_t* __restrict__ bf, const uint32_t* __restrict__ lin,
                                          const MarchRay& r, float& t, float& dt, float pos[3]) {
#pragma unroll
	for (int d = 0; d < 3; ++d) pos[d] = r.o[d] + t * r.dir[d];
	if (!aabb_contains(ds, pos)) return 0;
	uint32_t mip;
	bool occ;
	if (FAST) {
		dt = MIN_CONE_STEPSIZE;  // calc_dt(t, 0)
		// mip_from_pos (dt * 256 < 1) is 0 iff 0 < max|p - 0.5| < 0.5 (frexpf(0) has exponent 0 -> mip 1)
		const float m = fmaxf(fmaxf(fabsf(pos[0] - 0.5f), fabsf(pos[1] - 0.5f)), fabsf(pos[2] - 0.5f));
		if ((m > 0.0f) & (m < 0.5f)) {
			mip = 0;
			// cascaded_grid_idx_at with scale 1: ((p - 0.5) * 1) + 0.5
			const int ix = clampi((int)(((pos[0] - 0.5f) + 0.5f) * NERF_GRIDSIZE), 0, NERF_GRIDSIZE - 1);
			const int iy = clampi((int)(((pos[1] - 0.5f) + 0.5f) * NERF_GRIDSIZE), 0, NERF_GRIDSIZE - 1);
			const int iz = clampi((int)(((pos[2] - 0.5f) + 0.5f) * NERF_GRIDSIZE), 0, NERF_GRIDSIZE - 1);
			occ = (lin[((uint32_t)ix << 9) | ((uint32_t)iy << 2) | ((uint32_t)iz >> 5)] >> (iz & 31)) & 1;
		} else {
			mip = (uint32_t)mip_from_pos(pos[0], pos[1], pos[2]);
			occ = occupied(pos[0], pos[1], pos[2], bf, mip);
		}
	} else {
		dt = calc_dt(t, ds.cone_angle);
		mip = (uint32_t)mip_from_dt(dt, pos[0], pos[1], pos[2]);
		occ = occupied(pos[0], pos[1], pos[2], bf, mip);
	}
	if (occ) return 1;
	if (FAST) {
		// advance_to_next_voxel with a constant step; t / res is an exact power-of-two scaling
		const uint32_t res = NERF_GRIDSIZE >> mip;
		float tn = 3.402823466e+38f;
#pragma unroll
		for (int d = 0; d < 3; ++d) {
			const float p = res * pos[d];
			tn = fminf(tn, (floorf(p + 0.5f + 0.5f * signf(r.dir[d])) - p) * r.idir[d]);
		}
		const float t_target = t + fmaxf(ldexpf(tn, -(int)(7 - mip)), 0.0f);
		do { t += MIN_CONE_STEPSIZE; } while (t < t_target);
	} else {
		t = advance_to_next_voxel(t, ds.cone_angle, pos, r.dir, r.idir, NERF_GRIDSIZE >> mip);
	}
	return 2;
}

// ---------------------------------------------------------------- NeuS alpha (shared)
struct Alpha { float alpha, p_div_c, inv_s, true_cos, iter_cos, next_sdf, dt; };
__device__ __forceinline__ Alpha neus_alpha(const half_t* lo, const float dir[3], float dt, float cos_anneal) {
	Alpha a;
	a.dt = dt;
	a.inv_s = det_expf((float)((half_t)10.0f * lo[7]));
	const float sdf = (float)lo[3];
	const float pg[3] = {(float)lo[4], (float)lo[5], (float)lo[6]};
	a.true_cos = dir[0] * pg[0] + dir[1] * pg[1] + dir[2] * pg[2];
	float a1 = (float)(-a.true_cos * 0.5 + 0.5); a1 = a1 > 0.0f ? a1 : 0.0f;
	float a2 = -a.true_cos; a2 = a2 > 0.0f ? a2 : 0.0f;
	a.iter_cos = -(a1 * (1.0 - cos_anneal) + a2 * cos_anneal);
	a.next_sdf = sdf + a.iter_cos * dt * 0.5;
	const float prev_sdf = sdf - a.iter_cos * dt * 0.5;
	const float next_cdf = det_logistic(a.next_sdf * a.inv_s);
	const float prev_cdf = det_logistic(prev_sdf * a.inv_s);
	const float p = prev_cdf - next_cdf, c = prev_cdf;
	a.p_div_c = (p + 1e-5f) / (c + 1e-5f);
	a.alpha = clampf(a.p_div_c, 0.0f, 1.0f);
	return a;
}

// direction used by the NeuS cosine: the network's warped-dir output rows 8..10 (BENT_DIR,
// testbed_nerf.cu:1583-1588). Static scenes write the same warped dir for every sample of a ray,
// so each sample can read its own row.
__device__ __forceinline__ void bent_dir(const half_t* lo, float dir[3]) {
	float u[3] = {(float)lo[8] * 2.0f - 1.0f, (float)lo[9] * 2.0f - 1.0f, (float)lo[10] * 2.0f - 1.0f};
	const float n2 = sqrtf((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
#pragma unroll
	for (int k = 0; k < 3; ++k) dir[k] = n2 > 0 ? u[k] / n2 : u[k];
}
__device__ __forceinline__ float grad_norm(const half_t* lo) {
	const float pg[3] = {(float)lo[4], (float)lo[5], (float)lo[6]};
	return sqrt((double)(pg[0] * pg[0] + pg[1] * pg[1] + pg[2] * pg[2]) + 1e-6);
}
// k_loss_alpha's per-sample work (compute_loss_kernel_train_nerf's alpha / colour / eikonal terms): {alpha, sigmoid(rgb)}
// and (|grad sdf| - 1)^2 of sample s from its 16 network outputs; also the fused inference's epilogue
__device__ __forceinline__ void loss_alpha_sample(const half_t* lo, float dt, float cos_anneal, float4* __restrict__ sa, float* __restrict__ ekt,
                                                  uint32_t s) {
	float dir[3]; bent_dir(lo, dir);
	const Alpha a = neus_alpha(lo, dir, dt, cos_anneal);
	sa[s] = make_float4(a.alpha, det_logistic((float)lo[0]), det_logistic((float)lo[1]), det_logistic((float)lo[2]));
	const float gn = grad_norm(lo);
	ekt[s] = (gn - 1.0f) * (gn - 1.0f);
}
__device__ __forceinline__ void load_out(const half_t* net_out, uint32_t s, half_t lo[16]) {
	const h8* p = (const h8*)(net_out + (size_t)s * OUT_W);
	const h8 a = p[0], b = p[1];
#pragma unroll
	for (int k = 0; k < 8; ++k) { lo[k] = a[k]; lo[8 + k] = b[k]; }
}

} // namespace neus
