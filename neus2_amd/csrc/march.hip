// NeuS ray sampling, SDF-to-alpha compositing, loss and deterministic compaction on gfx950.
//
//   k_march_count / k_march_write : generate_training_samples_nerf_with_global_movement
//                                   (testbed_nerf.cu:1263-1456), static path
//   k_loss_count  / k_loss_write  : compute_loss_kernel_train_nerf_with_global_movement
//                                   (testbed_nerf.cu:1475-1997), static path
//   k_rollover                    : fill_rollover(_and_rescale) (my_tcnn common_device.h:515-535)
//   k_step_counters               : Counters::update_after_training (testbed_nerf.cu:3399-3438)
//
// The reference appends rays and compacted samples with global atomics (non-deterministic
// order). Here each pass is split into a count kernel, a device-wide exclusive scan over ray
// slots (rocPRIM via hipCUB) and a write kernel, which yields the canonical ray-ordered layout
// with exactly the reference's keep/drop rule (a ray is kept iff scan_base + n <= cap).
// This file is compiled with -ffp-contract=off: the march and the alpha/transmittance
// arithmetic are bit-identical to the CPU oracle (no FMA contraction, det_expf).
#pragma clang fp contract(off)
#include "kernels.h"
#include <algorithm>

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
	o[0] = srgb_to_linear((float)(v & 0xff) * (1.0f / 255.0f)) * a;
	o[1] = srgb_to_linear((float)((v >> 8) & 0xff) * (1.0f / 255.0f)) * a;
	o[2] = srgb_to_linear((float)((v >> 16) & 0xff) * (1.0f / 255.0f)) * a;
	o[3] = a;
}
__device__ __forceinline__ bool aabb_contains(const DevDataset& ds, const float p[3]) {
	return p[0] >= ds.aabb_min[0] && p[0] <= ds.aabb_max[0] && p[1] >= ds.aabb_min[1] && p[1] <= ds.aabb_max[1] &&
	       p[2] >= ds.aabb_min[2] && p[2] <= ds.aabb_max[2];
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

// ---------------------------------------------------------------- pass 1: per-ray count
// rays: 6 floats/ray (o, unnormalized d); startt: 1 float/ray; nreq: requested steps (0 = none)
__global__ void __launch_bounds__(256) k_march_count(uint32_t cap_rays, const StepState* __restrict__ st, DPInfo dp, DevDataset ds,
                                                     const uint8_t* __restrict__ bitfield, uint64_t rng_state, uint64_t rng_inc,
                                                     float* __restrict__ rays, float* __restrict__ startt_out, uint32_t* __restrict__ nreq) {
	const uint32_t R = st->rays_per_batch;
	const uint32_t n_rays_global = R * dp.world, n_rays_total = st->n_rays_total;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap_rays; i += gridDim.x * blockDim.x) {
		uint32_t n = 0;
		float o[3] = {0, 0, 0}, du[3] = {0, 0, 0}, startt = 0.f;
		if (i < R) {
			const uint32_t ig = dp.rank * R + i;
			pcg32 rng(rng_state, rng_inc);
			const uint32_t img = image_idx(ig, n_rays_global, n_rays_total, ds.n_images);
			const int rx = ds.res[2 * img], ry = ds.res[2 * img + 1];
			rng.advance((int64_t)(uint32_t)(ig * N_MAX_RANDOM_SAMPLES_PER_RAY));
			float xx, yy; random_image_pos(rng, rx, ry, xx, yy);
			float rgba[4]; read_rgba(ds, img, xx, yy, rgba);
			bool drop = false;
			if (rgba[0] <= 0.0f) drop = (double)rng.next_float() >= 0.9;
			if (!drop) {
				(void)rng.next_float();  // motionblur_time
				const float fx = ds.focal[2 * img], fy = ds.focal[2 * img + 1], ppx = ds.pp[2 * img], ppy = ds.pp[2 * img + 1];
				const float* M = ds.xform + 12 * img;
				const float dc[3] = {(xx - ppx) * (float)rx / fx, (yy - ppy) * (float)ry / fy, 1.0f};
#pragma unroll
				for (int r = 0; r < 3; ++r) { du[r] = (M[4 * r] * dc[0] + M[4 * r + 1] * dc[1]) + M[4 * r + 2] * dc[2]; o[r] = M[4 * r + 3]; }
				const float nrm = sqrtf((du[0] * du[0] + du[1] * du[1]) + du[2] * du[2]);
				float dir[3];
#pragma unroll
				for (int r = 0; r < 3; ++r) dir[r] = nrm > 0.f ? du[r] / nrm : du[r];
				float tmin; ray_intersect(ds, o, dir, tmin);
				tmin = fmaxf(tmin, 0.0f);
				startt = tmin;
				startt += calc_dt(startt, ds.cone_angle) * rng.next_float();
				const float idir[3] = {1.0f / dir[0], 1.0f / dir[1], 1.0f / dir[2]};
				float t = startt;
				while (true) {
					const float pos[3] = {o[0] + t * dir[0], o[1] + t * dir[1], o[2] + t * dir[2]};
					if (!(aabb_contains(ds, pos) && n < NERF_STEPS)) break;
					const float dt = calc_dt(t, ds.cone_angle);
					const uint32_t mip = (uint32_t)mip_from_dt(dt, pos[0], pos[1], pos[2]);
					if (occupied(pos[0], pos[1], pos[2], bitfield, mip)) { ++n; t += dt; }
					else t = advance_to_next_voxel(t, ds.cone_angle, pos, dir, idir, NERF_GRIDSIZE >> mip);
				}
			}
		}
		float* rr = rays + 6 * (size_t)i;
		rr[0] = o[0]; rr[1] = o[1]; rr[2] = o[2]; rr[3] = du[0]; rr[4] = du[1]; rr[5] = du[2];
		startt_out[i] = startt;
		nreq[i] = n;
	}
}

// ---------------------------------------------------------------- pass 2: write kept rays
__global__ void __launch_bounds__(256) k_march_write(uint32_t cap_rays, StepState* __restrict__ st, DevDataset ds,
                                                     const uint8_t* __restrict__ bitfield, const float* __restrict__ rays,
                                                     const float* __restrict__ startt_in, const uint32_t* __restrict__ nreq,
                                                     const uint32_t* __restrict__ base, uint32_t* __restrict__ numsteps,
                                                     float* __restrict__ coords) {
	const uint32_t max_samples = st->max_inference;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap_rays; i += gridDim.x * blockDim.x) {
		const uint32_t n = nreq[i], b = base[i];
		if (i == cap_rays - 1) st->numsteps_counter = b + n;
		const bool keep = n > 0 && b + n <= max_samples;
		numsteps[2 * i] = keep ? n : 0;
		numsteps[2 * i + 1] = b;
		if (!keep) continue;
		atomicMax(&st->n_kept, b + n);
		atomicAdd(&st->n_rays_with_samples, 1u);
		const float* rr = rays + 6 * (size_t)i;
		const float o[3] = {rr[0], rr[1], rr[2]};
		const float nrm = sqrtf((rr[3] * rr[3] + rr[4] * rr[4]) + rr[5] * rr[5]);
		float dir[3];
#pragma unroll
		for (int r = 0; r < 3; ++r) dir[r] = nrm > 0.f ? rr[3 + r] / nrm : rr[3 + r];
		const float idir[3] = {1.0f / dir[0], 1.0f / dir[1], 1.0f / dir[2]};
		const float wd[3] = {(dir[0] + 1.0f) * 0.5f, (dir[1] + 1.0f) * 0.5f, (dir[2] + 1.0f) * 0.5f};
		const float diag[3] = {ds.aabb_max[0] - ds.aabb_min[0], ds.aabb_max[1] - ds.aabb_min[1], ds.aabb_max[2] - ds.aabb_min[2]};
		float* out = coords + (size_t)b * COORD_W;
		uint32_t j = 0;
		float t = startt_in[i];
		while (true) {
			const float pos[3] = {o[0] + t * dir[0], o[1] + t * dir[1], o[2] + t * dir[2]};
			if (!(aabb_contains(ds, pos) && j < n)) break;
			const float dt = calc_dt(t, ds.cone_angle);
			const uint32_t mip = (uint32_t)mip_from_dt(dt, pos[0], pos[1], pos[2]);
			if (occupied(pos[0], pos[1], pos[2], bitfield, mip)) {
				float* cc = out + (size_t)j * COORD_W;
				cc[0] = (pos[0] - ds.aabb_min[0]) / diag[0]; cc[1] = (pos[1] - ds.aabb_min[1]) / diag[1]; cc[2] = (pos[2] - ds.aabb_min[2]) / diag[2];
				cc[3] = warp_dt(dt);
				cc[4] = wd[0]; cc[5] = wd[1]; cc[6] = wd[2];
				++j; t += dt;
			} else t = advance_to_next_voxel(t, ds.cone_angle, pos, dir, idir, NERF_GRIDSIZE >> mip);
		}
	}
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

// ---------------------------------------------------------------- loss pass 1: compacted count
__global__ void __launch_bounds__(256) k_loss_count(uint32_t cap_rays, const StepState* __restrict__ st, DevDataset ds,
                                                    const float* __restrict__ rays, const uint32_t* __restrict__ numsteps,
                                                    const float* __restrict__ coords, const half_t* __restrict__ net_out,
                                                    float cos_anneal, uint32_t* __restrict__ ccount) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap_rays; i += gridDim.x * blockDim.x) {
		const uint32_t ns = numsteps[2 * i], base = numsteps[2 * i + 1];
		uint32_t cn = 0;
		if (ns > 0) {
			const float* rr = rays + 6 * (size_t)i;
			const float nr = sqrtf((rr[3] * rr[3] + rr[4] * rr[4]) + rr[5] * rr[5]);
			float dir[3] = {nr > 0 ? rr[3] / nr : rr[3], nr > 0 ? rr[4] / nr : rr[4], nr > 0 ? rr[5] / nr : rr[5]};
			float T = 1.f;
			for (; cn < ns; ++cn) {
				if (T < 1e-4f) break;
				const half_t* lo = net_out + (size_t)(base + cn) * OUT_W;
				const float* ci = coords + (size_t)(base + cn) * COORD_W;
				if (cn == 0) {
					float u[3] = {(float)lo[8] * 2.0f - 1.0f, (float)lo[9] * 2.0f - 1.0f, (float)lo[10] * 2.0f - 1.0f};
					const float n2 = sqrtf((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
#pragma unroll
					for (int k = 0; k < 3; ++k) dir[k] = n2 > 0 ? u[k] / n2 : u[k];
				}
				const Alpha a = neus_alpha(lo, dir, unwarp_dt(ci[3]), cos_anneal);
				T *= (1.f - a.alpha);
			}
		}
		ccount[i] = cn;
	}
}

// ---------------------------------------------------------------- loss pass 2: composite, loss, dL/dout
__global__ void __launch_bounds__(256) k_loss_write(uint32_t cap_rays, StepState* __restrict__ st, DPInfo dp, DevDataset ds, LossParams lp,
                                                    const float* __restrict__ rays, uint32_t* __restrict__ numsteps,
                                                    const float* __restrict__ coords, const half_t* __restrict__ net_out,
                                                    const uint32_t* __restrict__ ccount, const uint32_t* __restrict__ cbase,
                                                    float* __restrict__ coords_out, half_t* __restrict__ dL_dout,
                                                    float* __restrict__ loss_out, float* __restrict__ ek_out, float* __restrict__ mask_out) {
	const uint32_t R = st->rays_per_batch;
	const uint32_t n_rays_global = R * dp.world, n_rays_total = st->n_rays_total;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap_rays; i += gridDim.x * blockDim.x) {
		const uint32_t ns = numsteps[2 * i], base = numsteps[2 * i + 1];
		const uint32_t cn = ccount[i], cb = cbase[i];
		if (i == cap_rays - 1) st->compacted_counter = cb + cn;
		loss_out[i] = 0.f; ek_out[i] = 0.f; mask_out[i] = 0.f;
		if (ns == 0) { numsteps[2 * i] = 0; numsteps[2 * i + 1] = cb; continue; }
		const float* rr = rays + 6 * (size_t)i;
		const float ro[3] = {rr[0], rr[1], rr[2]};
		const float nr = sqrtf((rr[3] * rr[3] + rr[4] * rr[4]) + rr[5] * rr[5]);
		float dir[3] = {nr > 0 ? rr[3] / nr : rr[3], nr > 0 ? rr[4] / nr : rr[4], nr > 0 ? rr[5] / nr : rr[5]};
		const float diag[3] = {ds.aabb_max[0] - ds.aabb_min[0], ds.aabb_max[1] - ds.aabb_min[1], ds.aabb_max[2] - ds.aabb_min[2]};
		// first pass: composite (rgb_ray, weight_sum) over the cn used samples
		float T = 1.f, rgb_ray[3] = {0, 0, 0}, weight_sum = 0.f;
		for (uint32_t j = 0; j < cn; ++j) {
			const half_t* lo = net_out + (size_t)(base + j) * OUT_W;
			const float* ci = coords + (size_t)(base + j) * COORD_W;
			if (j == 0) {
				float u[3] = {(float)lo[8] * 2.0f - 1.0f, (float)lo[9] * 2.0f - 1.0f, (float)lo[10] * 2.0f - 1.0f};
				const float n2 = sqrtf((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
#pragma unroll
				for (int k = 0; k < 3; ++k) dir[k] = n2 > 0 ? u[k] / n2 : u[k];
			}
			const Alpha a = neus_alpha(lo, dir, unwarp_dt(ci[3]), lp.cos_anneal);
			const float weight = a.alpha * T;
#pragma unroll
			for (int k = 0; k < 3; ++k) rgb_ray[k] += weight * det_logistic((float)lo[k]);
			weight_sum += weight;
			T *= (1.f - a.alpha);
		}
		// target pixel and background (same RNG stream as the sampler)
		const uint32_t ig = dp.rank * R + i;
		pcg32 rng(lp.rng_state, lp.rng_inc);
		rng.advance((int64_t)(uint32_t)(ig * N_MAX_RANDOM_SAMPLES_PER_RAY));
		const uint32_t img = image_idx(ig, n_rays_global, n_rays_total, ds.n_images);
		const int rx = ds.res[2 * img], ry = ds.res[2 * img + 1];
		float xx, yy; random_image_pos(rng, rx, ry, xx, yy);
		float bg[3];
		bg[0] = rng.next_float(); bg[1] = rng.next_float(); bg[2] = rng.next_float();
#pragma unroll
		for (int k = 0; k < 3; ++k) bg[k] = srgb_to_linear(bg[k]);
		float tex[4]; read_rgba(ds, img, xx, yy, tex);
		float target[3];
#pragma unroll
		for (int k = 0; k < 3; ++k) {
			target[k] = 1.0f * tex[k] + (1.0f - tex[3]) * bg[k];
			target[k] = linear_to_srgb(target[k]);
			bg[k] = linear_to_srgb(bg[k]);
		}
		if (cn == ns) {
#pragma unroll
			for (int k = 0; k < 3; ++k) rgb_ray[k] += T * bg[k];
		}
		const uint32_t comp = min(lp.max_compacted - min(lp.max_compacted, cb), cn);
		numsteps[2 * i] = comp; numsteps[2 * i + 1] = cb;
		if (comp == 0) continue;
		float lgrad[3], lloss[3];
#pragma unroll
		for (int k = 0; k < 3; ++k) {
			const float diff = rgb_ray[k] - target[k], ad = fabsf(diff), sq = 0.5f / 0.1f * diff * diff;
			lloss[k] = (ad > 0.1f ? (ad - 0.5f * 0.1f) : sq) / 5.0f;
			lgrad[k] = (ad > 0.1f ? (diff > 0 ? 1.0f : -1.0f) : (diff / 0.1f)) / 5.0f;
		}
		const float mask_gt = (float)(tex[3] > 0.9999f);
		float gws;
		if (weight_sum >= 1.0 - 1e-4) { weight_sum = 1.0 - 1e-4; gws = 0.0f; }
		else if (weight_sum <= 1e-4) { weight_sum = 1e-4; gws = 0.0f; }
		else { const float sws = 1.0f / (1.0f + exp(-(double)weight_sum)); gws = (mask_gt - sws) * weight_sum * lp.mask_w; }
		const float mean_loss = ((lloss[0] + lloss[1]) + lloss[2]) / 3.0f;
		loss_out[i] = mean_loss / (float)n_rays_global;
		mask_out[i] = -(mask_gt * logf(weight_sum) + (1 - mask_gt) * logf(1 - weight_sum));
		const float loss_scale = lp.loss_scale / n_rays_global;
		// gradient pass (testbed_nerf.cu:1775-1959)
		float rgb2[3] = {0, 0, 0};
		float ek_acc = 0.f;
		T = 1.f;
		for (uint32_t j = 0; j < comp; ++j) {
			const float* ci = coords + (size_t)(base + j) * COORD_W;
			float* co = coords_out + (size_t)(cb + j) * COORD_W;
#pragma unroll
			for (int k = 0; k < COORD_W; ++k) co[k] = ci[k];
			const half_t* lo = net_out + (size_t)(base + j) * OUT_W;
			const Alpha a = neus_alpha(lo, dir, unwarp_dt(ci[3]), lp.cos_anneal);
			float raw[3], rgb[3];
#pragma unroll
			for (int k = 0; k < 3; ++k) { raw[k] = (float)lo[k]; rgb[k] = det_logistic(raw[k]); }
			const float weight = a.alpha * T;
#pragma unroll
			for (int k = 0; k < 3; ++k) rgb2[k] += weight * rgb[k];
			T *= (1.f - a.alpha);
			float dl[16];
#pragma unroll
			for (int k = 0; k < 16; ++k) dl[k] = 0.0f;
#pragma unroll
			for (int k = 0; k < 3; ++k) {
				const float sig = det_logistic(raw[k]);
				dl[k] = loss_scale * ((weight * lgrad[k]) * (sig * (1 - sig)) + fmaxf(0.0f, 0.0f * raw[k]));
			}
			float tr[3];
#pragma unroll
			for (int k = 0; k < 3; ++k) tr[k] = T * rgb[k] - (rgb_ray[k] - rgb2[k]);
			const float dot = (lgrad[0] * tr[0] + lgrad[1] * tr[1]) + lgrad[2] * tr[2];
			const float dloss_dalpha = (dot + gws * (1 - weight_sum)) / (1.0f - a.alpha + 1e-5);
			float dadem = 0, dem_dsdf = 0, dem_dinvs = 0, dadpe = 0, dpe_dinvs = 0, dpe_dic = 0, dem_dic = 0;
			if (!(a.p_div_c <= 0.0f || a.p_div_c >= 1.0f)) {
				const float plus_x = a.inv_s * a.iter_cos * a.dt;
				const float plus_e = det_expf(plus_x);
				const float e_minus = det_expf(-a.next_sdf * a.inv_s);
				dem_dsdf = -a.inv_s * e_minus;
				dem_dinvs = -a.next_sdf * e_minus;
				const float aa = 1 + e_minus;
				const float bb = 1 + plus_e * e_minus;
				const float cc = 1e-5 + 1 / (1 + plus_e * e_minus);
				const float delta = aa * (bb * bb) * (cc * cc);
				dadem = -(plus_e / (delta) - 1 / (aa * aa * cc));
				dadpe = -e_minus / (delta);
				dpe_dinvs = plus_e * a.iter_cos * a.dt;
				dpe_dic = plus_e * a.inv_s * a.dt;
				dem_dic = -a.inv_s * e_minus * a.dt * 0.5;
			}
			const float dloss_dinvs = dloss_dalpha * (dadem * dem_dinvs + dadpe * dpe_dinvs);
			const float dloss_dvar = dloss_dinvs * a.inv_s * 10;
			const float d_ic_tc = a.true_cos >= 0 ? 0.0f : 1.0f;
			const float pg[3] = {(float)lo[4], (float)lo[5], (float)lo[6]};
			const float gn = sqrt((double)(pg[0] * pg[0] + pg[1] * pg[1] + pg[2] * pg[2]) + 1e-6);
			const float gn_inv = 1 - 1 / gn;
			const float dloss_dnn = dloss_dalpha * (dadem * dem_dic + dpe_dic * dadpe) * d_ic_tc;
			const float dloss_dsdf = dloss_dalpha * dadem * dem_dsdf;
			dl[3] = loss_scale * dloss_dsdf;
			ek_acc += (gn - 1.0f) * (gn - 1.0f);
#pragma unroll
			for (int k = 0; k < 3; ++k) dl[4 + k] = rh(lp.ek_w * 2 * lp.loss_scale * gn_inv * pg[k]);
			dl[7] = rh(loss_scale * dloss_dvar);
#pragma unroll
			for (int k = 0; k < 3; ++k) dl[8 + k] = rh(loss_scale * dloss_dnn * dir[k]);
			h8 o0, o1;
#pragma unroll
			for (int k = 0; k < 8; ++k) { o0[k] = (half_t)dl[k]; o1[k] = (half_t)dl[8 + k]; }
			half_t* dst = dL_dout + (size_t)(cb + j) * OUT_W;
			*(h8*)dst = o0; *(h8*)(dst + 8) = o1;
		}
		ek_out[i] = ek_acc / ((float)comp * (float)n_rays_global);
	}
}

// ---------------------------------------------------------------- rollover (n_in from device)
__global__ void k_rollover(uint32_t n_elements, const StepState* __restrict__ st, float* __restrict__ coords, half_t* __restrict__ dL_dout) {
	const uint32_t n_in = min(st->compacted_counter, n_elements);
	if (blockIdx.x == 0 && threadIdx.x == 0) ((StepState*)st)->n_train = n_in ? n_elements : 0u;
	if (n_in == 0) return;
	for (uint32_t i = n_in + blockIdx.x * blockDim.x + threadIdx.x; i < n_elements; i += gridDim.x * blockDim.x) {
		const uint32_t src = i % n_in;
#pragma unroll
		for (int k = 0; k < COORD_W; ++k) coords[(size_t)i * COORD_W + k] = coords[(size_t)src * COORD_W + k];
#pragma unroll
		for (int k = 0; k < OUT_W; ++k) {
			const float r = (float)dL_dout[(size_t)src * OUT_W + k];
			dL_dout[(size_t)i * OUT_W + k] = (half_t)(r * n_in / n_elements);
		}
	}
}

// ---------------------------------------------------------------- per-step counters (1 thread)
// Counters::update_after_training (testbed_nerf.cu:3399-3438) + the next step's max_inference
// (testbed_nerf.cu:3771-3776) + n_rays_total (testbed_nerf.cu:3784-3790). `world` divides the
// all-reduced counters so every rank adapts R identically.
__global__ void k_step_counters(StepState* st, uint32_t target_batch, uint32_t max_samples, uint32_t world, uint32_t fixed_rays) {
	if (threadIdx.x != 0 || blockIdx.x != 0) return;
	const uint32_t R = st->rays_per_batch;
	st->n_rays_total += R * world;  // n_rays_total
	const uint32_t before = st->numsteps_counter / world;
	const uint32_t measured = st->compacted_counter / world;
	st->measured_before = before;
	st->measured_batch_size = measured;
	if (before == 0 || measured == 0) { st->zero_records = 1; return; }
	st->zero_records = 0;
	uint32_t mi = min(before, max_samples);
	st->max_inference = (mi + 127u) / 128u * 128u;
	if (fixed_rays) { st->rays_per_batch = fixed_rays; return; }
	uint32_t r = (uint32_t)((float)R * (float)target_batch / (float)measured);
	r = (r + 127u) / 128u * 128u;
	st->rays_per_batch = min(r, 1u << 18);
}

// ---------------------------------------------------------------- host launchers
static inline uint32_t ray_blocks(uint32_t cap) { return std::max<uint32_t>(1, std::min<uint32_t>((cap + 255) / 256, 2048)); }
void launch_march_count(hipStream_t s, uint32_t cap, const StepState* st, DPInfo dp, const DevDataset& ds, const uint8_t* bitfield,
                        uint64_t rng_state, uint64_t rng_inc, float* rays, float* startt, uint32_t* nreq) {
	k_march_count<<<ray_blocks(cap), 256, 0, s>>>(cap, st, dp, ds, bitfield, rng_state, rng_inc, rays, startt, nreq);
}
void launch_march_write(hipStream_t s, uint32_t cap, StepState* st, const DevDataset& ds, const uint8_t* bitfield, const float* rays,
                        const float* startt, const uint32_t* nreq, const uint32_t* base, uint32_t* numsteps, float* coords) {
	k_march_write<<<ray_blocks(cap), 256, 0, s>>>(cap, st, ds, bitfield, rays, startt, nreq, base, numsteps, coords);
}
void launch_loss_count(hipStream_t s, uint32_t cap, const StepState* st, const DevDataset& ds, const float* rays, const uint32_t* numsteps,
                       const float* coords, const half_t* net_out, float cos_anneal, uint32_t* ccount) {
	k_loss_count<<<ray_blocks(cap), 256, 0, s>>>(cap, st, ds, rays, numsteps, coords, net_out, cos_anneal, ccount);
}
void launch_loss_write(hipStream_t s, uint32_t cap, StepState* st, DPInfo dp, const DevDataset& ds, const LossParams& lp, const float* rays,
                       uint32_t* numsteps, const float* coords, const half_t* net_out, const uint32_t* ccount, const uint32_t* cbase,
                       float* coords_out, half_t* dL_dout, float* loss, float* ek, float* mask) {
	k_loss_write<<<ray_blocks(cap), 256, 0, s>>>(cap, st, dp, ds, lp, rays, numsteps, coords, net_out, ccount, cbase, coords_out, dL_dout, loss, ek, mask);
}
void launch_rollover(hipStream_t s, uint32_t n_elements, const StepState* st, float* coords, half_t* dL_dout) {
	k_rollover<<<std::max<uint32_t>(1, std::min<uint32_t>((n_elements + 255) / 256, 2048)), 256, 0, s>>>(n_elements, st, coords, dL_dout);
}
void launch_step_counters(hipStream_t s, StepState* st, uint32_t target_batch, uint32_t max_samples, uint32_t world, uint32_t fixed_rays) {
	k_step_counters<<<1, 64, 0, s>>>(st, target_batch, max_samples, world, fixed_rays);
}

} // namespace neus
