// NeuS rendering of a camera view on gfx950 (evaluation path of the PSNR metric).
//
//   k_render_init      : init_rays_with_payload_kernel_nerf + advance_pos_nerf (testbed_nerf.cu:2208-2330, 797-846),
//                        pinhole camera, snap_to_pixel_centers, no distortion / envmap / global movement
//   k_render_flags +   : compact_kernel_nerf (testbed_nerf.cu:2183-2206); the atomic append is replaced by a
//   k_render_compact     flag -> exclusive scan -> scatter pass (deterministic order; per-ray results do not
//                        depend on the order, only the alive count does)
//   k_render_gen       : generate_next_nerf_network_inputs (testbed_nerf.cu:877-934)
//   k_render_composite : composite_kernel_nerf, Shade mode (testbed_nerf.cu:936-1106) fused with
//                        shade_kernel_nerf (:2148-2181): a ray that dies writes its pixel directly
//                        (pixels are owned by exactly one ray, so no hit list is needed)
//   k_render_accumulate: accumulate_kernel, linear colour space (render_buffer.cu:217-260)
// The network evaluation between gen and composite is the fused inference kernel (mlp.hip) on the
// EMA weights (the reference's inference params). Compiled with -ffp-contract=off: the march is the
// training march, bit-identical with the CPU oracle.
#pragma clang fp contract(off)
#include "march_common.h"

namespace neus {

// NerfPayload (testbed_nerf.h / nerf.h:50-60) + the per-ray rgba of RaysNerfSoa, one 64-B record
struct RenderRay {
	float o[3], d[3], t, max_weight;
	uint32_t idx, n_steps, alive, pad;
	float4 rgba;
};
static_assert(sizeof(RenderRay) == 64, "RenderRay is one 64-B record");

// ld_random_val (random_val.cuh:284-288) for dimension 0: the Sobol dimension-0 direction numbers are
// the bit reversal, so sobol(index, 0) == reverse_bits(index).
__device__ __forceinline__ uint32_t rev32(uint32_t x) { return __builtin_bitreverse32(x); }
__device__ __forceinline__ uint32_t lk_perm(uint32_t x, uint32_t seed) {
	x += seed; x ^= x * 0x6c50b47cu; x ^= x * 0xb82f1e52u; x ^= x * 0xc7afe638u; x ^= x * 0x8d22f6e6u; return x;
}
__device__ __forceinline__ uint32_t nus_base2(uint32_t x, uint32_t seed) { return rev32(lk_perm(rev32(x), seed)); }
__device__ __forceinline__ uint32_t hash_combine(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }
__device__ __forceinline__ float ld_random_val0(uint32_t index, uint32_t seed) {
	index = nus_base2(index, seed);
	return (float)nus_base2(rev32(index), hash_combine(seed, 0)) * float(1.0 / 4294967296.0);
}

__global__ void __launch_bounds__(256) k_render_init(RenderCamera cam, uint32_t sample_index, DevDataset ds, const uint8_t* __restrict__ bf,
                                                     const uint32_t* __restrict__ lin, RenderRay* __restrict__ rays, float4* __restrict__ frame) {
	const uint32_t n = cam.width * cam.height;
	const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
	if (idx >= n) return;
	const uint32_t x = idx % cam.width, y = idx / cam.width;
	frame[idx] = make_float4(0.f, 0.f, 0.f, 0.f);  // CudaRenderBuffer::clear_frame
	RenderRay r{};
	r.idx = idx;
	// pixel_to_ray (common_device.cuh:246-303): uv = (pixel + offset) / res, pinhole, rotation then origin
	const float u = ((float)x + cam.pixel_offset[0]) / (float)cam.width, v = ((float)y + cam.pixel_offset[1]) / (float)cam.height;
	const float dc[3] = {(u - cam.screen_center[0]) * (float)cam.width / cam.focal[0], (v - cam.screen_center[1]) * (float)cam.height / cam.focal[1], 1.0f};
	float du[3];
#pragma unroll
	for (int k = 0; k < 3; ++k) { du[k] = (cam.xform[4 * k] * dc[0] + cam.xform[4 * k + 1] * dc[1]) + cam.xform[4 * k + 2] * dc[2]; r.o[k] = cam.xform[4 * k + 3]; }
	const float nrm = sqrtf((du[0] * du[0] + du[1] * du[1]) + du[2] * du[2]);
#pragma unroll
	for (int k = 0; k < 3; ++k) r.d[k] = nrm > 0.f ? du[k] / nrm : du[k];
	if (ds.motion.on) {  // global_movement_with_rotation_6d on the camera ray (testbed_nerf.cu:2285-2294)
		const float* M = ds.motion.R;
		float mo[3], md[3];
#pragma unroll
		for (int k = 0; k < 3; ++k) {
			mo[k] = ((M[3 * k] * r.o[0] + M[3 * k + 1] * r.o[1]) + M[3 * k + 2] * r.o[2]) + ds.motion.t[k];
			md[k] = (M[3 * k] * r.d[0] + M[3 * k + 1] * r.d[1]) + M[3 * k + 2] * r.d[2];
		}
#pragma unroll
		for (int k = 0; k < 3; ++k) { r.o[k] = mo[k]; r.d[k] = md[k]; }
	}
	float tmin; ray_intersect(ds, r.o, r.d, tmin);
	float t = fmaxf(tmin, NERF_RENDERING_NEAR_DISTANCE) + 1e-6f;
	float p[3];
#pragma unroll
	for (int k = 0; k < 3; ++k) p[k] = r.o[k] + t * r.d[k];
	r.alive = aabb_contains(ds, p) ? 1u : 0u;
	if (r.alive) {
		// advance_pos_nerf: jitter by one step, then skip empty space up to the first occupied sample
		MarchRay mr;
#pragma unroll
		for (int k = 0; k < 3; ++k) { mr.o[k] = r.o[k]; mr.dir[k] = r.d[k]; mr.idir[k] = 1.0f / r.d[k]; }
		const float dt0 = calc_dt(t, ds.cone_angle);
		t += ld_random_val0(sample_index, idx * 786433u) * dt0;
		while (true) {
			float dt, pos[3];
			const int k = march_step<false>(ds, bf, lin, mr, t, dt, pos);
			if (k == 0) { r.alive = 0; break; }
			if (k == 1) break;
		}
	}
	r.t = t;
	r.rgba = make_float4(0.f, 0.f, 0.f, 0.f);
	rays[idx] = r;
}

__global__ void __launch_bounds__(256) k_render_flags(uint32_t n, const RenderRay* __restrict__ rays, uint32_t* __restrict__ flags) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) flags[i] = rays[i].alive;
}

__global__ void __launch_bounds__(256) k_render_compact(uint32_t n, const RenderRay* __restrict__ src, const uint32_t* __restrict__ flags,
                                                        const uint32_t* __restrict__ base, RenderRay* __restrict__ dst, uint32_t* __restrict__ n_alive) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	if (flags[i]) dst[base[i]] = src[i];
	if (i == n - 1) *n_alive = base[i] + flags[i];
}

// generate_next_nerf_network_inputs: up to n_steps occupied samples per alive ray, sample j of ray i at
// row i + j * n_alive (the reference's layout); rows past a ray's exit get a zero coordinate.
__global__ void __launch_bounds__(256) k_render_gen(uint32_t n_alive, uint32_t n_steps, DevDataset ds, const uint8_t* __restrict__ bf,
                                                    const uint32_t* __restrict__ lin, RenderRay* __restrict__ rays, float* __restrict__ coords) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_alive) return;
	RenderRay& r = rays[i];
	MarchRay mr;
#pragma unroll
	for (int k = 0; k < 3; ++k) { mr.o[k] = r.o[k]; mr.dir[k] = r.d[k]; mr.idir[k] = 1.0f / r.d[k]; }
	const float diag[3] = {ds.aabb_max[0] - ds.aabb_min[0], ds.aabb_max[1] - ds.aabb_min[1], ds.aabb_max[2] - ds.aabb_min[2]};
	const float wd[3] = {(r.d[0] + 1.0f) * 0.5f, (r.d[1] + 1.0f) * 0.5f, (r.d[2] + 1.0f) * 0.5f};
	float t = r.t;
	uint32_t j = 0;
	bool exited = false;
	while (j < n_steps) {
		float dt, pos[3];
		const int k = march_step<false>(ds, bf, lin, mr, t, dt, pos);
		if (k == 0) { exited = true; break; }
		if (k == 2) continue;
		float* c = coords + ((size_t)i + (size_t)j * n_alive) * COORD_W;
		c[0] = (pos[0] - ds.aabb_min[0]) / diag[0]; c[1] = (pos[1] - ds.aabb_min[1]) / diag[1]; c[2] = (pos[2] - ds.aabb_min[2]) / diag[2];
		c[3] = warp_dt(dt);
		c[4] = wd[0]; c[5] = wd[1]; c[6] = wd[2];
		t += dt;
		++j;
	}
	for (uint32_t q = j; q < n_steps; ++q) {
		float* c = coords + ((size_t)i + (size_t)q * n_alive) * COORD_W;
#pragma unroll
		for (int k = 0; k < COORD_W; ++k) c[k] = 0.f;
	}
	r.n_steps = j;
	if (!exited) r.t = t;
}

// composite_kernel_nerf (Shade mode, no glow, show_accel < 0) + shade_kernel_nerf for rays that die here
__global__ void __launch_bounds__(256) k_render_composite(uint32_t n_alive, uint32_t n_steps, const float* __restrict__ coords,
                                                          const half_t* __restrict__ net_out, float cos_anneal, float min_transmittance,
                                                          uint32_t linear_colors, RenderRay* __restrict__ rays, float4* __restrict__ frame) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_alive) return;
	RenderRay& r = rays[i];
	float4 c = r.rgba;
	const uint32_t actual = r.n_steps;
	uint32_t j = 0;
	for (; j < actual; ++j) {
		const size_t row = (size_t)i + (size_t)j * n_alive;
		half_t lo[16]; load_out(net_out, (uint32_t)row, lo);
		const float T = 1.f - c.w;
		const float dt = unwarp_dt(coords[row * COORD_W + 3]);
		float dir[3]; bent_dir(lo, dir);
		const Alpha a = neus_alpha(lo, dir, dt, cos_anneal);
		const float weight = a.alpha * T;
		c.x += det_logistic((float)lo[0]) * weight;
		c.y += det_logistic((float)lo[1]) * weight;
		c.z += det_logistic((float)lo[2]) * weight;
		c.w += weight;
		if (weight > r.max_weight) r.max_weight = weight;
		if (c.w > (1.0f - min_transmittance)) {
			const float w = c.w;
			c.x /= w; c.y /= w; c.z /= w; c.w /= w;
			break;
		}
	}
	r.rgba = c;
	if (j < n_steps) {
		r.alive = 0;
		// compact_kernel_nerf keeps dead rays with alpha > 0.001 for shading; the frame starts cleared,
		// so shade_kernel_nerf's `tmp + frame * (1 - tmp.w)` is tmp (sRGB network colour -> linear unless the
		// network was trained in linear colours)
		if (c.w > 0.001f)
			frame[r.idx] = linear_colors ? c : make_float4(srgb_to_linear(c.x), srgb_to_linear(c.y), srgb_to_linear(c.z), c.w);
	}
}

// accumulate_kernel, linear colour space: accum = (accum * spp + frame) / (spp + 1)
__global__ void __launch_bounds__(256) k_render_accumulate(uint32_t n, float spp, const float4* __restrict__ frame, float4* __restrict__ accum) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const float4 f = frame[i];
	float4 a = spp == 0.f ? make_float4(0.f, 0.f, 0.f, 0.f) : accum[i];
	a.x = (a.x * spp + f.x) / (spp + 1); a.y = (a.y * spp + f.y) / (spp + 1);
	a.z = (a.z * spp + f.z) / (spp + 1); a.w = (a.w * spp + f.w) / (spp + 1);
	accum[i] = a;
}

static inline uint32_t nb(uint32_t n) { return (n + 255) / 256; }

size_t render_ray_bytes() { return sizeof(RenderRay); }
void launch_render_init(hipStream_t s, const RenderCamera& cam, uint32_t sample_index, const DevDataset& ds, const uint8_t* bf, const uint32_t* lin,
                        void* rays, float4* frame) {
	const uint32_t n = cam.width * cam.height;
	if (n) k_render_init<<<nb(n), 256, 0, s>>>(cam, sample_index, ds, bf, lin, (RenderRay*)rays, frame);
}
void launch_render_compact(hipStream_t s, uint32_t n, const void* src, uint32_t* flags, uint32_t* base, void* dst, uint32_t* n_alive,
                           void* scan_tmp, size_t scan_tmp_bytes) {
	if (n == 0) { (void)hipMemsetAsync(n_alive, 0, 4, s); return; }
	k_render_flags<<<nb(n), 256, 0, s>>>(n, (const RenderRay*)src, flags);
	launch_exclusive_scan(s, scan_tmp, scan_tmp_bytes, flags, base, n);
	k_render_compact<<<nb(n), 256, 0, s>>>(n, (const RenderRay*)src, flags, base, (RenderRay*)dst, n_alive);
}
void launch_render_gen(hipStream_t s, uint32_t n_alive, uint32_t n_steps, const DevDataset& ds, const uint8_t* bf, const uint32_t* lin, void* rays,
                       float* coords) {
	if (n_alive) k_render_gen<<<nb(n_alive), 256, 0, s>>>(n_alive, n_steps, ds, bf, lin, (RenderRay*)rays, coords);
}
void launch_render_composite(hipStream_t s, uint32_t n_alive, uint32_t n_steps, const float* coords, const half_t* net_out, float cos_anneal,
                             float min_transmittance, bool linear_colors, void* rays, float4* frame) {
	if (n_alive)
		k_render_composite<<<nb(n_alive), 256, 0, s>>>(n_alive, n_steps, coords, net_out, cos_anneal, min_transmittance, linear_colors ? 1u : 0u,
		                                                 (RenderRay*)rays, frame);
}
void launch_render_accumulate(hipStream_t s, uint32_t n, uint32_t spp, const float4* frame, float4* accum) {
	if (n) k_render_accumulate<<<nb(n), 256, 0, s>>>(n, (float)spp, frame, accum);
}

} // namespace neus
