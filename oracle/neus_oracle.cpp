// =============================================================================
// neus_oracle.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A plain C++ CPU restatement of the reference NeuS2 training hot path
// (zbqq/neus2 @ /root/reference). Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library, and only as the checker /
// CPU baseline, never as the thing measured or shipped.
//
// Every function cites the reference file:line it restates. Storage rounding
// points of the reference (fp16 params, fp16 activations, fp16 network output,
// fp16 dL/doutput) are reproduced with explicit round-to-half; arithmetic is fp32
// (fp64 for gradient accumulation) where the reference accumulates in fp16.
//
// Pinning: the reference ships no golden vectors and cannot
// be compiled here. The RNG is pinned against the published PCG32 known-answer
// vectors; everything else is a line-by-line restatement cross-checked against
// torch float64 autograd (tests/torch_ref.py, used by tests/test_oracle.py and
// tests/test_gpu_module.py). See DESIGN.md §Oracle.
//
// Determinism notes shared with the HIP path (both sides do exactly this):
//  * no FMA contraction (-ffp-contract=off here and in the HIP march/loss files);
//  * the compaction-relevant exponentials use det_expf(), a fixed-operation-order
//    expf, so the T<1e-4 early exit is bit-identical on CPU and GPU.
// =============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#include <immintrin.h>
#endif

namespace {

// ---------------------------------------------------------------- half helpers
// F16C conversions (round to nearest even, subnormals kept): the same results as a bit-level IEEE restatement, and
// the oracle's hottest operation (every fp16 storage point of the reference is a round trip through them).
static inline uint16_t f2h(float f) { return (uint16_t)_cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT); }
static inline float h2f(uint16_t h) { return _cvtsh_ss(h); }
static inline float rh(float f) { return h2f(f2h(f)); }

// --------------------------------------------- pcg32 (my_tcnn pcg32.h:43-170)
struct pcg32 {
	uint64_t state, inc;
	pcg32() : state(0x853c49e6748fea9bULL), inc(0xda3e39cb94b95bdbULL) {}
	explicit pcg32(uint64_t initstate, uint64_t initseq = 1u) { seed(initstate, initseq); }
	void seed(uint64_t initstate, uint64_t initseq = 1) {
		state = 0U; inc = (initseq << 1u) | 1u; next_uint(); state += initstate; next_uint();
	}
	uint32_t next_uint() {
		uint64_t oldstate = state;
		state = oldstate * 0x5851f42d4c957f2dULL + inc;
		uint32_t xorshifted = (uint32_t)(((oldstate >> 18u) ^ oldstate) >> 27u);
		uint32_t rot = (uint32_t)(oldstate >> 59u);
		return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
	}
	float next_float() {
		uint32_t u = (next_uint() >> 9) | 0x3f800000u; float f; std::memcpy(&f, &u, 4); return f - 1.0f;
	}
	void advance(int64_t delta_ = (1ll << 32)) {
		uint64_t cur_mult = 0x5851f42d4c957f2dULL, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
		uint64_t delta = (uint64_t)delta_;
		while (delta > 0) {
			if (delta & 1) { acc_mult *= cur_mult; acc_plus = acc_plus * cur_mult + cur_plus; }
			cur_plus = (cur_mult + 1) * cur_plus; cur_mult *= cur_mult; delta /= 2;
		}
		state = acc_mult * state + acc_plus;
	}
};

// ------------------------------------------ fixed-order expf (shared w/ HIP)
static inline float det_expf(float x) {
	if (!(x < 88.5f)) return x != x ? x : std::numeric_limits<float>::infinity();
	if (x < -103.0f) return 0.0f;
	float kf = std::nearbyint(x * 1.44269504088896341f);
	float r = x - kf * 0.693145751953125f;
	r = r - kf * 1.42860676533018672e-06f;
	float p = 1.3888889225e-3f;
	p = p * r + 8.3333337680e-3f;
	p = p * r + 4.1666667908e-2f;
	p = p * r + 1.6666667163e-1f;
	p = p * r + 0.5f;
	p = p * r + 1.0f;
	p = p * r + 1.0f;
	return std::ldexp(p, (int)kf);
}
static inline float det_logistic(float x) { return 1.0f / (1.0f + det_expf(-x)); }

// ----------------------------------------------- testbed_nerf.cu:57-81 consts
constexpr uint32_t NERF_GRIDSIZE = 128;
constexpr uint32_t NERF_STEPS = 1024;
constexpr uint32_t NERF_CASCADES = 8;
constexpr float SQRT3 = 1.73205080757f;
constexpr float STEPSIZE = SQRT3 / NERF_STEPS;
constexpr float MIN_CONE_STEPSIZE = STEPSIZE;
constexpr float MAX_CONE_STEPSIZE = STEPSIZE * (1 << (NERF_CASCADES - 1)) * NERF_STEPS / NERF_GRIDSIZE;
constexpr uint32_t N_MAX_RANDOM_SAMPLES_PER_RAY = 8;
constexpr float NERF_MIN_OPTICAL_THICKNESS = 0.1f;

struct V3 { float x, y, z; };
static inline V3 v3(float a, float b, float c) { return {a, b, c}; }

static inline float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline float calc_dt(float t, float cone) { return clampf(t * cone, MIN_CONE_STEPSIZE, MAX_CONE_STEPSIZE); }
static inline float warp_dt(float dt) {  // testbed_nerf.cu:494-497
	float max_stepsize = MIN_CONE_STEPSIZE * (1 << (NERF_CASCADES - 1));
	return (dt - MIN_CONE_STEPSIZE) / (max_stepsize - MIN_CONE_STEPSIZE);
}
static inline float unwarp_dt(float dt) {  // testbed_nerf.cu:499-502
	float max_stepsize = MIN_CONE_STEPSIZE * (1 << (NERF_CASCADES - 1));
	return dt * (max_stepsize - MIN_CONE_STEPSIZE) + MIN_CONE_STEPSIZE;
}
// my_tcnn common_device.h:335-365
static inline uint32_t expand_bits(uint32_t v) {
	v = (v * 0x00010001u) & 0xFF0000FFu; v = (v * 0x00000101u) & 0x0F00F00Fu;
	v = (v * 0x00000011u) & 0xC30C30C3u; v = (v * 0x00000005u) & 0x49249249u; return v;
}
static inline uint32_t morton3D(uint32_t x, uint32_t y, uint32_t z) { return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2); }
static inline uint32_t morton3D_invert(uint32_t x) {
	x = x & 0x49249249; x = (x | (x >> 2)) & 0xc30c30c3; x = (x | (x >> 4)) & 0x0f00f00f;
	x = (x | (x >> 8)) & 0xff0000ff; x = (x | (x >> 16)) & 0x0000ffff; return x;
}
static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
// testbed_nerf.cu:504-527
static inline uint32_t cascaded_grid_idx_at(V3 pos, uint32_t mip) {
	float mip_scale = std::scalbn(1.0f, -(int)mip);
	pos.x -= 0.5f; pos.y -= 0.5f; pos.z -= 0.5f;
	pos.x *= mip_scale; pos.y *= mip_scale; pos.z *= mip_scale;
	pos.x += 0.5f; pos.y += 0.5f; pos.z += 0.5f;
	int ix = (int)(pos.x * NERF_GRIDSIZE), iy = (int)(pos.y * NERF_GRIDSIZE), iz = (int)(pos.z * NERF_GRIDSIZE);
	return morton3D(clampi(ix, 0, NERF_GRIDSIZE - 1), clampi(iy, 0, NERF_GRIDSIZE - 1), clampi(iz, 0, NERF_GRIDSIZE - 1));
}
static inline bool density_grid_occupied_at(V3 pos, const uint8_t* bf, uint32_t mip) {  // :529-533
	uint32_t idx = cascaded_grid_idx_at(pos, mip);
	return bf[idx / 8 + (NERF_GRIDSIZE * NERF_GRIDSIZE * NERF_GRIDSIZE) * mip / 8] & (1 << (idx % 8));
}
static inline int mip_from_pos(V3 pos, uint32_t max_cascade = NERF_CASCADES - 1) {  // :624-629
	int exponent;
	float maxval = std::max(std::max(std::fabs(pos.x - 0.5f), std::fabs(pos.y - 0.5f)), std::fabs(pos.z - 0.5f));
	std::frexp(maxval, &exponent);
	return std::min((int)max_cascade, std::max(0, exponent + 1));
}
static inline int mip_from_dt(float dt, V3 pos, uint32_t max_cascade = NERF_CASCADES - 1) {  // :631-638
	int mip = mip_from_pos(pos, max_cascade);
	dt *= 2 * NERF_GRIDSIZE;
	if (dt < 1.f) return mip;
	int exponent; std::frexp(dt, &exponent);
	return std::min((int)max_cascade, std::max(exponent, mip));
}
static inline float signf(float x) { return std::copysign(1.0f, x); }
// testbed_nerf.cu:356-378
static inline float distance_to_next_voxel(V3 pos, V3 dir, V3 idir, uint32_t res) {
	V3 p = {res * pos.x, res * pos.y, res * pos.z};
	float tx = (std::floor(p.x + 0.5f + 0.5f * signf(dir.x)) - p.x) * idir.x;
	float ty = (std::floor(p.y + 0.5f + 0.5f * signf(dir.y)) - p.y) * idir.y;
	float tz = (std::floor(p.z + 0.5f + 0.5f * signf(dir.z)) - p.z) * idir.z;
	float t = std::fmin(std::fmin(tx, ty), tz);  // CUDA min(float,float) == fminf
	return std::fmax(t / res, 0.0f);
}
static inline float advance_to_next_voxel(float t, float cone, V3 pos, V3 dir, V3 idir, uint32_t res) {
	float t_target = t + distance_to_next_voxel(pos, dir, idir, res);
	do { t += calc_dt(t, cone); } while (t < t_target);
	return t;
}
// common_device.cuh (ngp) :31-61
static inline float srgb_to_linear(float s) { return s <= 0.04045f ? s / 12.92f : std::pow((s + 0.055f) / 1.055f, 2.4f); }
static inline float linear_to_srgb(float l) { return l < 0.0031308f ? 12.92f * l : 1.055f * std::pow(l, 0.41666f) - 0.055f; }

struct AABB { V3 mn, mx; };
static inline bool aabb_contains(const AABB& b, V3 p) {
	return p.x >= b.mn.x && p.x <= b.mx.x && p.y >= b.mn.y && p.y <= b.mx.y && p.z >= b.mn.z && p.z <= b.mx.z;
}
// bounding_box.cuh:163-215
static inline void ray_intersect(const AABB& b, V3 pos, V3 dir, float& tmin_o, float& tmax_o) {
	float tmin = (b.mn.x - pos.x) / dir.x, tmax = (b.mx.x - pos.x) / dir.x;
	if (tmin > tmax) std::swap(tmin, tmax);
	float tymin = (b.mn.y - pos.y) / dir.y, tymax = (b.mx.y - pos.y) / dir.y;
	if (tymin > tymax) std::swap(tymin, tymax);
	const float FM = std::numeric_limits<float>::max();
	if (tmin > tymax || tymin > tmax) { tmin_o = FM; tmax_o = FM; return; }
	if (tymin > tmin) tmin = tymin;
	if (tymax < tmax) tmax = tymax;
	float tzmin = (b.mn.z - pos.z) / dir.z, tzmax = (b.mx.z - pos.z) / dir.z;
	if (tzmin > tzmax) std::swap(tzmin, tzmax);
	if (tmin > tzmax || tzmin > tmax) { tmin_o = FM; tmax_o = FM; return; }
	if (tzmin > tmin) tmin = tzmin;
	if (tzmax < tmax) tmax = tzmax;
	tmin_o = tmin; tmax_o = tmax;
}

} // namespace

// =============================================================================
// Public C ABI of the oracle (ctypes from tests/ and bench.py's cpu_baseline).
// =============================================================================
extern "C" {

struct OrNetCfg {
	uint32_t n_levels;          // grid levels L
	uint32_t log2_hashmap_size; // T = 2^log2
	uint32_t base_resolution;
	float per_level_scale;
	uint32_t width;             // MLP hidden width (64 for base.json)
	uint32_t n_density_hidden;  // density MLP hidden layers (1)
	uint32_t n_rgb_hidden;      // rgb MLP hidden layers (2)
	uint32_t density_in;        // next_multiple(3 + 2L, 16)
	uint32_t rgb_in;            // next_multiple(3+3+16+16, 16) = 48
	float sdf_bias;             // -0.1 (nerf_network.h:87)
};

struct OrDataset {
	uint32_t n_images;
	const uint32_t* pixels;     // RGBA8, all images concatenated
	const uint64_t* pixel_offsets;
	const int32_t* resolution;  // 2 per image
	const float* focal;         // 2 per image
	const float* principal;     // 2 per image
	const float* xform;         // 12 per image, row-major 3x4 (camera-to-world, ngp convention)
	float aabb_min[3];
	float aabb_max[3];
	float cone_angle;           // 0 for aabb_scale 1 (testbed_nerf.cu:3091)
	float motion_R[9];          // accumulated global movement, row-major (frames >= 1 of a dynamic scene)
	float motion_t[3];
	uint32_t motion_on;
	uint32_t fixed_bg;          // 0: random background per ray (nerf.training.random_bg_color, the default)
	float bg_color[3];          // sRGB background when fixed_bg
	uint32_t target_mode;       // 0 color_space Linear (sRGB targets), 1 color_space SRGB, 2 linear_colors
};

namespace {
// global_movement_with_rotation_6d (testbed_nerf.cu:193-213): o' = R o + t, d' = R d (d normalized)
inline void move_ray(const OrDataset* ds, float o[3], float d[3]) {
	if (!ds->motion_on) return;
	const float* R = ds->motion_R;
	float no[3], nd[3];
	for (int k = 0; k < 3; ++k) {
		no[k] = ((R[3 * k] * o[0] + R[3 * k + 1] * o[1]) + R[3 * k + 2] * o[2]) + ds->motion_t[k];
		nd[k] = (R[3 * k] * d[0] + R[3 * k + 1] * d[1]) + R[3 * k + 2] * d[2];
	}
	for (int k = 0; k < 3; ++k) { o[k] = no[k]; d[k] = nd[k]; }
}
} // namespace

// ---------------------------------------------------------------- grid tables
// grid.h:1441-1501
uint32_t or_grid_tables(const OrNetCfg* c, uint32_t* offsets, uint32_t* res, float* scale) {
	uint32_t offset = 0;
	for (uint32_t i = 0; i < c->n_levels; ++i) {
		const float s = exp2f(i * std::log2(c->per_level_scale)) * c->base_resolution - 1.0f;
		const uint32_t r = (uint32_t)(std::ceil(s)) + 1;
		uint32_t max_params = std::numeric_limits<uint32_t>::max() / 2;
		uint32_t params_in_level = std::pow((float)r, 3) > (float)max_params ? max_params : r * r * r;
		params_in_level = (params_in_level + 7u) / 8u * 8u;
		params_in_level = std::min(params_in_level, (1u << c->log2_hashmap_size));
		offsets[i] = offset; res[i] = r; scale[i] = (float)(r - 1);
		offset += params_in_level;
	}
	offsets[c->n_levels] = offset;
	return offset * 2;
}

} // extern "C"

namespace {

struct Net {
	OrNetCfg c;
	std::vector<uint32_t> off, res;
	std::vector<float> scale;
	uint32_t n_grid_params;
	// param layout (nerf_network.h:741-785): density | rgb | grid | dir(0) | variance(4)
	struct Layer { uint32_t out, in, offset; };
	std::vector<Layer> dl, rl;
	uint32_t n_density, n_rgb, grid_off, var_off, n_params, n_matrix;
	explicit Net(const OrNetCfg& cfg) : c(cfg) {
		off.resize(c.n_levels + 1); res.resize(c.n_levels); scale.resize(c.n_levels);
		n_grid_params = or_grid_tables(&c, off.data(), res.data(), scale.data());
		uint32_t o = 0;
		dl.push_back({c.width, c.density_in, o}); o += c.width * c.density_in;
		for (uint32_t i = 1; i < c.n_density_hidden; ++i) { dl.push_back({c.width, c.width, o}); o += c.width * c.width; }
		dl.push_back({16, c.width, o}); o += 16 * c.width;
		n_density = o;
		rl.push_back({c.width, c.rgb_in, o}); o += c.width * c.rgb_in;
		for (uint32_t i = 1; i < c.n_rgb_hidden; ++i) { rl.push_back({c.width, c.width, o}); o += c.width * c.width; }
		rl.push_back({16, c.width, o}); o += 16 * c.width;
		n_rgb = o - n_density;
		n_matrix = o;
		grid_off = o; o += n_grid_params;
		var_off = o; o += 4;
		n_params = o;
	}
};

// grid.h:118-153
static inline uint32_t grid_index(uint32_t hashmap_size, uint32_t resolution, const uint32_t pos_grid[3]) {
	uint32_t stride = 1, index = 0;
	for (uint32_t dim = 0; dim < 3 && stride <= hashmap_size; ++dim) { index += pos_grid[dim] * stride; stride *= resolution; }
	if (hashmap_size < stride) index = pos_grid[0] * 1u ^ pos_grid[1] * 2654435761u ^ pos_grid[2] * 805459861u;
	return (index % hashmap_size) * 2;
}

// Per-level trilinear setup: pos_fract (common_device.h:404-434), linear interpolation.
struct LevelPos { float pos[3]; uint32_t grid[3]; float scale; uint32_t hsize, res, off; };
static inline LevelPos level_pos(const Net& n, uint32_t l, const float x[3]) {
	LevelPos lp;
	lp.scale = n.scale[l]; lp.res = n.res[l]; lp.off = n.off[l]; lp.hsize = n.off[l + 1] - n.off[l];
	for (int d = 0; d < 3; ++d) {
		float p = std::fmaf(x[d], lp.scale, 0.5f);  // nvcc contracts `input * scale + 0.5f` to one FFMA
		int tmp = (int)std::floor(p);
		lp.grid[d] = (uint32_t)tmp;
		lp.pos[d] = p - (float)tmp;
	}
	return lp;
}

// kernel_grid (grid.h:174-369): enc (half-rounded storage) + dy/dx (fp32)
static void grid_forward_one(const Net& n, const float* gparams, const float x[3], uint32_t valid_level, float* enc, float* dydx) {
	const uint32_t L = n.c.n_levels;
	for (uint32_t l = 0; l < L; ++l) {
		if (l > valid_level) {
			enc[2 * l] = enc[2 * l + 1] = 0.0f;
			if (dydx) for (int k = 0; k < 6; ++k) dydx[6 * l + k] = 0.0f;
			continue;
		}
		LevelPos lp = level_pos(n, l, x);
		const float* g = gparams + (size_t)lp.off * 2;
		float r0 = 0, r1 = 0;
		for (uint32_t idx = 0; idx < 8; ++idx) {
			float w = 1; uint32_t pl[3];
			for (int d = 0; d < 3; ++d) {
				if ((idx & (1u << d)) == 0) { w *= 1 - lp.pos[d]; pl[d] = lp.grid[d]; }
				else { w *= lp.pos[d]; pl[d] = lp.grid[d] + 1; }
			}
			uint32_t i = grid_index(lp.hsize, lp.res, pl);
			// the reference accumulates in the grid's precision: result[f] += (T)(weight * data), T = __half
			r0 = rh(r0 + rh(w * g[i])); r1 = rh(r1 + rh(w * g[i + 1]));
		}
		enc[2 * l] = r0; enc[2 * l + 1] = r1;
		if (dydx) {
			float gr[2][3] = {{0, 0, 0}, {0, 0, 0}};
			for (int gd = 0; gd < 3; ++gd) {
				for (uint32_t idx = 0; idx < 4; ++idx) {
					float w = lp.scale; uint32_t pl[3];
					for (int ngd = 0; ngd < 2; ++ngd) {
						const int d = ngd >= gd ? ngd + 1 : ngd;
						if ((idx & (1u << ngd)) == 0) { w *= 1 - lp.pos[d]; pl[d] = lp.grid[d]; }
						else { w *= lp.pos[d]; pl[d] = lp.grid[d] + 1; }
					}
					pl[gd] = lp.grid[gd]; uint32_t il = grid_index(lp.hsize, lp.res, pl);
					pl[gd] = lp.grid[gd] + 1; uint32_t ir = grid_index(lp.hsize, lp.res, pl);
					// grads += weight * (right - left) * pos_derivative(=1): one FFMA under nvcc --fmad=true
					gr[0][gd] = std::fmaf(w, g[ir] - g[il], gr[0][gd]);
					gr[1][gd] = std::fmaf(w, g[ir + 1] - g[il + 1], gr[1][gd]);
				}
			}
			for (int f = 0; f < 2; ++f) for (int d = 0; d < 3; ++d) dydx[6 * l + 3 * f + d] = gr[f][d];
		}
	}
}

static inline void atomic_add_d(double* p, double v) {
#ifdef _OPENMP
#pragma omp atomic
#endif
	*p += v;
}

// Grid-gradient semantics (or_set_grid_grad_mode; test-only, used to bound the device's record rounding):
//  0 = exact (default): every corner contribution summed unrounded in double;
//  1 = the reference's atomic operand: each contribution rounded to fp16, `(__half)((float)grad[f] * weight)`
//      (grid.h:418-421 for the first order, the same lambda at grid.h:926-929 for the second order with weight = -/+w),
//      summed in double;
//  2 = operand and accumulator in fp16: grad_t = __half (grid.h:1433), atomicAdd(__half2) - the adds land in the
//      thread schedule's order, as the reference's atomics do, so this mode is not reproducible run to run.
static int g_grid_grad_mode = 0;
static uint16_t* g_grid_half = nullptr;  // mode 2: the fp16 grid gradient (the grid's parameter index space)
static inline void half_atomic_add(uint16_t* p, uint16_t op) {
	uint16_t old = __atomic_load_n(p, __ATOMIC_RELAXED);
	for (;;) {
		const uint16_t nv = f2h(h2f(old) + h2f(op));
		if (__atomic_compare_exchange_n(p, &old, nv, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return;
	}
}
// one contribution `op32` (the reference's float product) to entry i of the level at parameter offset `off`
static inline void grid_add(double* gg, size_t off, uint32_t i, double exact, float op32) {
	if (g_grid_grad_mode == 0) atomic_add_d(&gg[i], exact);
	else if (g_grid_grad_mode == 1) atomic_add_d(&gg[i], (double)rh(op32));
	else half_atomic_add(g_grid_half + off + i, f2h(op32));
}

// kernel_grid_backward (grid.h:371-500) + kernel_grid_backward_input_backward_grid (grid.h:880-1007):
// first-order dL/denc * w_corner, plus second-order g_f * (+/- scale * v_d * prod w_other).
static void grid_scatter_one(const Net& n, const float x[3], uint32_t valid_level, const float* dL_denc, const float* g, const float* v, double* grad) {
	for (uint32_t l = 0; l < n.c.n_levels && l <= valid_level; ++l) {
		LevelPos lp = level_pos(n, l, x);
		const size_t go = (size_t)lp.off * 2;
		double* gg = grad + go;
		if (dL_denc) {
			for (uint32_t idx = 0; idx < 8; ++idx) {
				float w = 1; uint32_t pl[3];
				for (int d = 0; d < 3; ++d) {
					if ((idx & (1u << d)) == 0) { w *= 1 - lp.pos[d]; pl[d] = lp.grid[d]; }
					else { w *= lp.pos[d]; pl[d] = lp.grid[d] + 1; }
				}
				uint32_t i = grid_index(lp.hsize, lp.res, pl);
				grid_add(gg, go, i, (double)dL_denc[2 * l] * w, dL_denc[2 * l] * w);
				grid_add(gg, go, i + 1, (double)dL_denc[2 * l + 1] * w, dL_denc[2 * l + 1] * w);
			}
		}
		if (g && v) {
			for (int gd = 0; gd < 3; ++gd) {
				float grad_in = lp.scale * v[gd] * 1.0f;  // pos_derivative = 1 (linear)
				for (uint32_t idx = 0; idx < 4; ++idx) {
					float w = grad_in; uint32_t pl[3];
					for (int ngd = 0; ngd < 2; ++ngd) {
						const int d = ngd >= gd ? ngd + 1 : ngd;
						if ((idx & (1u << ngd)) == 0) { w *= 1 - lp.pos[d]; pl[d] = lp.grid[d]; }
						else { w *= lp.pos[d]; pl[d] = lp.grid[d] + 1; }
					}
					pl[gd] = lp.grid[gd]; uint32_t il = grid_index(lp.hsize, lp.res, pl);
					grid_add(gg, go, il, -(double)g[2 * l] * w, g[2 * l] * -w);
					grid_add(gg, go, il + 1, -(double)g[2 * l + 1] * w, g[2 * l + 1] * -w);
					pl[gd] = lp.grid[gd] + 1; uint32_t ir = grid_index(lp.hsize, lp.res, pl);
					grid_add(gg, go, ir, (double)g[2 * l] * w, g[2 * l] * w);
					grid_add(gg, go, ir + 1, (double)g[2 * l + 1] * w, g[2 * l + 1] * w);
				}
			}
		}
	}
}

// Spherical harmonics degree 4 (spherical_harmonics.h:47-100), input warped dir in [0,1].
static void sh4(const float wd[3], float* out) {
	float x = wd[0] * 2.f - 1.f, y = wd[1] * 2.f - 1.f, z = wd[2] * 2.f - 1.f;
	float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
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

// Summation order of the layer products (or_set_sum_order). Test-only: 0 = index order (the oracle); 1 = reversed,
// 2 = pairwise (recursive halves), 3 = blocked (sequential blocks of 8, then the block sums in order). The alternative
// orders measure how far the fp32 accumulation order alone moves a training step (fp16 activations flipping at
// rounding boundaries): the noise floor against which the device's MFMA-ordered sums are compared.
static int g_sum_order = 0;
static float sum_pairwise(const float* p, uint32_t n) {
	if (n == 1) return p[0];
	if (n == 2) return p[0] + p[1];
	const uint32_t h = n / 2;
	return sum_pairwise(p, h) + sum_pairwise(p + h, n - h);
}
// sum of the products p[0..n) in the active alternative order (g_sum_order != 0)
static float sum_ordered(const float* p, uint32_t n) {
	if (n == 0) return 0.0f;
	float s = 0;
	switch (g_sum_order) {
	case 1: for (uint32_t i = n; i-- > 0;) s += p[i]; return s;
	case 2: return sum_pairwise(p, n);
	case 3: {
		for (uint32_t b0 = 0; b0 < n; b0 += 8) {
			float bs = 0;
			for (uint32_t i = b0; i < std::min(n, b0 + 8); ++i) bs += p[i];
			s += bs;
		}
		return s;
	}
	default: for (uint32_t i = 0; i < n; ++i) s += p[i]; return s;
	}
}
// y = W x with W RM [out][in] (fp16-rounded weights), fp32 accumulation.
static inline void matvec(const float* W, uint32_t out, uint32_t in, const float* x, float* y) {
	for (uint32_t o = 0; o < out; ++o) {
		const float* w = W + (size_t)o * in;
		if (g_sum_order) {
			float p[64];
			for (uint32_t i = 0; i < in; ++i) p[i] = w[i] * x[i];
			y[o] = sum_ordered(p, in);
			continue;
		}
		if (o + 8 <= out) {  // eight independent index-order chains (the same sums, not latency-bound)
			float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
			for (uint32_t i = 0; i < in; ++i)
				for (int j = 0; j < 8; ++j) s8[j] += w[(size_t)j * in + i] * x[i];
			for (int j = 0; j < 8; ++j) y[o + j] = s8[j];
			o += 7;
			continue;
		}
		float s = 0;
		for (uint32_t i = 0; i < in; ++i) s += w[i] * x[i];
		y[o] = s;
	}
}
// y = W^T d
static inline void matvec_t(const float* W, uint32_t out, uint32_t in, const float* d, float* y) {
	if (g_sum_order) {
		for (uint32_t i = 0; i < in; ++i) {
			float p[64];
			for (uint32_t o = 0; o < out; ++o) p[o] = W[(size_t)o * in + i] * d[o];
			y[i] = sum_ordered(p, out);
		}
		return;
	}
	for (uint32_t i = 0; i < in; ++i) y[i] = 0;
	for (uint32_t o = 0; o < out; ++o) { const float* w = W + (size_t)o * in; for (uint32_t i = 0; i < in; ++i) y[i] += w[i] * d[o]; }
}
// sum_k a[k] * b[stride * k] over n terms (the grid-input gradients' sums over the 2L features)
static inline float dot_strided(const float* a, const float* b, uint32_t stride, uint32_t n) {
	if (g_sum_order) {
		float p[64];
		for (uint32_t k = 0; k < n; ++k) p[k] = a[k] * b[stride * k];
		return sum_ordered(p, n);
	}
	float s = 0;
	for (uint32_t k = 0; k < n; ++k) s += a[k] * b[stride * k];
	return s;
}

// Per-sample forward context (NerfNetwork::ForwardContext, nerf_network.h:1297-1315).
struct Ctx {
	float din[64], enc[64], dydx[192];
	float dh[4][64];      // density hidden activations (post-ReLU, half-rounded)
	float dout[16];       // density output (half)
	float gin[64];        // dSDF/d(density_input) (half)
	float grad_sdf[3];    // dSDF/dx (fp32)
	float rin[64];        // rgb input (half)
	float rh_[4][64];     // rgb hidden activations (half)
	float rout[16];
};

// NerfNetwork::forward_impl (nerf_network.h:145-328) for one sample.
static void net_forward_one(const Net& n, const float* P, const float* coord, uint32_t valid_level, Ctx& cx, uint16_t* out16) {
	const OrNetCfg& c = n.c;
	const uint32_t L = c.n_levels, W = c.width;
	const float* x = coord;  // warped position
	grid_forward_one(n, P + n.grid_off, x, valid_level, cx.enc, cx.dydx);
	// density_input = [x - 0.5 (half arithmetic), enc, 0...] (common_operation.cuh:181-194, nerf_network.h:206-212)
	for (uint32_t k = 0; k < c.density_in; ++k) cx.din[k] = 0;
	for (int d = 0; d < 3; ++d) cx.din[d] = rh(rh(x[d]) - rh(0.5f));
	for (uint32_t k = 0; k < 2 * L; ++k) cx.din[3 + k] = cx.enc[k];
	// density MLP forward (fully_fused_mlp.cu:678-812), hidden ReLU, output linear
	const float* in = cx.din; uint32_t nin = c.density_in;
	float tmp[64];
	for (size_t li = 0; li + 1 < n.dl.size(); ++li) {
		matvec(P + n.dl[li].offset, W, nin, in, tmp);
		for (uint32_t o = 0; o < W; ++o) cx.dh[li][o] = rh(tmp[o] > 0 ? tmp[o] : 0.0f);
		in = cx.dh[li]; nin = W;
	}
	matvec(P + n.dl.back().offset, 16, W, in, tmp);
	for (int o = 0; o < 16; ++o) cx.dout[o] = rh(tmp[o]);
	// dSDF/d(density_input): backward with dL/dout = e0 (nerf_network.h:228-253)
	float dcur[64]; for (int o = 0; o < 16; ++o) dcur[o] = o == 0 ? 1.0f : 0.0f;
	uint32_t nout = 16;
	for (int li = (int)n.dl.size() - 1; li >= 1; --li) {
		float t[64]; matvec_t(P + n.dl[li].offset, nout, W, dcur, t);
		for (uint32_t i = 0; i < W; ++i) dcur[i] = rh(cx.dh[li - 1][i] > 0 ? t[i] : 0.0f);
		nout = W;
	}
	{ float t[64]; matvec_t(P + n.dl[0].offset, nout, c.density_in, dcur, t); for (uint32_t i = 0; i < c.density_in; ++i) cx.gin[i] = rh(t[i]); }
	// kernel_grid_backward_input (grid.h:803-830) then identity path add (nerf_network.h:249-251)
	for (int d = 0; d < 3; ++d) {
		const float s = dot_strided(cx.gin + 3, cx.dydx + d, 3, 2 * L);
		cx.grad_sdf[d] = s + cx.gin[d];
	}
	// rgb input: [density_out(16), SH(16), xyz(3), grad_sdf(3), 0...] (nerf_network.h:262-280)
	for (uint32_t k = 0; k < c.rgb_in; ++k) cx.rin[k] = 0;
	for (int k = 0; k < 16; ++k) cx.rin[k] = cx.dout[k];
	float sh[16]; sh4(coord + 4, sh);
	for (int k = 0; k < 16; ++k) cx.rin[16 + k] = rh(sh[k]);
	for (int d = 0; d < 3; ++d) { cx.rin[32 + d] = rh(x[d]); cx.rin[35 + d] = rh(cx.grad_sdf[d]); }
	in = cx.rin; nin = c.rgb_in;
	for (size_t li = 0; li + 1 < n.rl.size(); ++li) {
		matvec(P + n.rl[li].offset, W, nin, in, tmp);
		for (uint32_t o = 0; o < W; ++o) cx.rh_[li][o] = rh(tmp[o] > 0 ? tmp[o] : 0.0f);
		in = cx.rh_[li]; nin = W;
	}
	matvec(P + n.rl.back().offset, 16, W, in, tmp);
	for (int o = 0; o < 16; ++o) cx.rout[o] = rh(tmp[o]);
	if (out16) {
		// output packing (nerf_network.h:287-324; common_operation.cuh:944-965, 326-352)
		for (int o = 0; o < 16; ++o) out16[o] = f2h(cx.rout[o]);
		out16[3] = f2h(cx.dout[0] + rh(c.sdf_bias));
		for (int d = 0; d < 3; ++d) out16[4 + d] = f2h(cx.grad_sdf[d]);
		out16[7] = f2h(P[n.var_off]);
		for (int d = 0; d < 3; ++d) out16[8 + d] = f2h(coord[4 + d]);
	}
}

// Weight-gradient accumulation target: double per param.
// NerfNetwork::backward_impl (nerf_network.h:330-601) for one sample.
// G: the matrix-parameter gradients, private to the calling thread (plain adds); Ggrid: the shared grid gradient (atomic)
static void net_backward_one(const Net& n, const float* P, const float* coord, uint32_t valid_level, const Ctx& cx,
                             const uint16_t* dout16, float indeed_batch, double* G, double* Ggrid, double* var_grad_acc,
                             float* dpos_out = nullptr) {
	const OrNetCfg& c = n.c;
	const uint32_t W = c.width, L = c.n_levels;
	float dLo[16]; for (int k = 0; k < 16; ++k) dLo[k] = h2f(dout16[k]);
	// rgb MLP backward (Overwrite) with dL_drgb = rows 0..2 (common_operation.cuh:1010-1024)
	float dcur[64]; for (int k = 0; k < 16; ++k) dcur[k] = k < 3 ? dLo[k] : 0.0f;
	uint32_t nout = 16;
	for (int li = (int)n.rl.size() - 1; li >= 0; --li) {
		const auto& ly = n.rl[li];
		const float* act = li == 0 ? cx.rin : cx.rh_[li - 1];
		for (uint32_t o = 0; o < ly.out; ++o) {
			if (dcur[o] == 0.0f) continue;
			double* g = G + ly.offset + (size_t)o * ly.in;
			for (uint32_t i = 0; i < ly.in; ++i) g[i] += (double)dcur[o] * act[i];
		}
		float t[64]; matvec_t(P + ly.offset, nout, ly.in, dcur, t);
		if (li > 0) { for (uint32_t i = 0; i < W; ++i) dcur[i] = rh(cx.rh_[li - 1][i] > 0 ? t[i] : 0.0f); nout = W; }
		else { for (uint32_t i = 0; i < ly.in; ++i) dcur[i] = rh(t[i]); }
	}
	float dL_drin[64]; for (uint32_t i = 0; i < c.rgb_in; ++i) dL_drin[i] = dcur[i];
	// dL/d density_out = dL/d rgb_in[0:16]; row 0 += dL_dout[3] as a half add (common_operation.cuh:1026-1037)
	for (int k = 0; k < 16; ++k) dcur[k] = dL_drin[k];
	dcur[0] = rh(dcur[0] + dLo[3]);
	nout = 16;
	float dL_ddin[64];
	for (int li = (int)n.dl.size() - 1; li >= 0; --li) {
		const auto& ly = n.dl[li];
		const float* act = li == 0 ? cx.din : cx.dh[li - 1];
		for (uint32_t o = 0; o < ly.out; ++o) {
			if (dcur[o] == 0.0f) continue;
			double* g = G + ly.offset + (size_t)o * ly.in;
			for (uint32_t i = 0; i < ly.in; ++i) g[i] += (double)dcur[o] * act[i];
		}
		float t[64]; matvec_t(P + ly.offset, nout, ly.in, dcur, t);
		if (li > 0) { for (uint32_t i = 0; i < W; ++i) dcur[i] = rh(cx.dh[li - 1][i] > 0 ? t[i] : 0.0f); nout = W; }
		else { for (uint32_t i = 0; i < ly.in; ++i) dL_ddin[i] = rh(t[i]); }
	}
	// variance gradient = batch sum of dL_dout[7] (nerf_network.h:461-474)
	*var_grad_acc += (double)dLo[7];
	// dL/d(position) for the DeltaNetwork (nerf_network.h:602-631): grid input gradient (kernel_grid_backward_input
	// of dL/denc) + rgb input xyz rows + density input xyz rows
	if (dpos_out)
		for (int d = 0; d < 3; ++d) {
			const float s = dot_strided(dL_ddin + 3, cx.dydx + d, 3, 2 * L);
			dpos_out[d] = (s + dL_drin[32 + d]) + dL_ddin[d];
		}
	// v = dL/d(grad_sdf): rgb-input rows 35..37 + eikonal/indeed_batch + bent-dir rows 8..10 (nerf_network.h:478-504)
	float v[3];
	for (int d = 0; d < 3; ++d) {
		v[d] = dL_drin[35 + d];
		v[d] += dLo[4 + d] / indeed_batch;
		v[d] += dLo[8 + d];
	}
	// grid gradients: first order (dL/denc) + second order (g = dSDF/denc, v) (nerf_network.h:423-442, 547-557)
	grid_scatter_one(n, coord, valid_level, dL_ddin + 3, cx.gin + 3, v, Ggrid);
	// pos_encoding_dy = dy/dx . v (grid.h:1182-1207), stored half
	float u[64]; for (uint32_t k = 0; k < c.density_in; ++k) u[k] = 0;
	for (int d = 0; d < 3; ++d) u[d] = rh(v[d]);
	for (uint32_t k = 0; k < 2 * L; ++k) {
		float s = 0; for (int d = 0; d < 3; ++d) s += cx.dydx[3 * k + d] * v[d];
		u[3 + k] = rh(s);
	}
	// FullyFusedMLP::backward_backward_input (fully_fused_mlp.cu:1088-1198), 1 hidden layer form
	// front: hf_i = relu'(h_{i-1}) . (W_{i-1} hf_{i-1}), hf_0 = u ; back: b_i = relu'(h) . (W^T b_{i+1}), b_top = e0
	constexpr size_t MAXL = 8;  // density layers (n_density_hidden + 1)
	float front[MAXL][64], back[MAXL + 1][64];
	std::copy(u, u + c.density_in, front[0]);
	for (size_t li = 1; li < n.dl.size(); ++li) {
		const auto& ly = n.dl[li - 1];
		float t[64]; matvec(P + ly.offset, ly.out, ly.in, front[li - 1], t);
		for (uint32_t o = 0; o < ly.out; ++o) front[li][o] = rh(cx.dh[li - 1][o] > 0 ? t[o] : 0.0f);
	}
	std::fill(back[n.dl.size()], back[n.dl.size()] + 16, 0.0f); back[n.dl.size()][0] = 1.0f;
	for (int li = (int)n.dl.size() - 1; li >= 1; --li) {
		const auto& ly = n.dl[li];
		float t[64]; matvec_t(P + ly.offset, ly.out, ly.in, back[li + 1], t);
		for (uint32_t i = 0; i < ly.in; ++i) back[li][i] = rh(cx.dh[li - 1][i] > 0 ? t[i] : 0.0f);
	}
	for (size_t li = 0; li < n.dl.size(); ++li) {
		const auto& ly = n.dl[li];
		const float* bk = back[li + 1];
		const float* fr = front[li];
		for (uint32_t o = 0; o < ly.out; ++o) {
			if (bk[o] == 0.0f) continue;
			double* g = G + ly.offset + (size_t)o * ly.in;
			for (uint32_t i = 0; i < ly.in; ++i) g[i] += (double)bk[o] * fr[i];
		}
	}
}

struct SampleRay { float o[3], d[3]; };  // Ray (unnormalized direction)

} // namespace

extern "C" {

uint32_t or_net_n_params(const OrNetCfg* c) { Net n(*c); return n.n_params; }
void or_set_sum_order(int order) { g_sum_order = order; }
void or_set_grid_grad_mode(int mode) { g_grid_grad_mode = mode; }
void or_net_layout(const OrNetCfg* c, uint32_t* out) {
	Net n(*c);
	out[0] = n.n_density; out[1] = n.n_rgb; out[2] = n.grid_off; out[3] = n.n_grid_params; out[4] = n.var_off; out[5] = n.n_params; out[6] = n.n_matrix;
}

// Parameter initialisation (trainer.h:54-109, fully_fused_mlp.cu:1229-1249, gpu_matrix.h:292-306,
// grid.h:2375-2380, random.h:67-91, nerf_network.h:815-886). `geo_init` (n_density floats) replaces the
// density MLP (the reference loads utils/mlp_weights*.txt).
static void init_params_from(const OrNetCfg* c, pcg32 rnd, const float* geo_init, float* params);
// Trainer (trainer.h:54-109): std::seed_seq{seed}.generate(2 values) -> pcg32{seeds[0]} -> model->initialize_params
void or_init_params(const OrNetCfg* c, uint32_t seed, const float* geo_init, float* params) {
	std::seed_seq seq{seed};
	std::vector<uint32_t> seeds(2);
	seq.generate(seeds.begin(), seeds.end());
	init_params_from(c, pcg32(seeds.front()), geo_init, params);
}
// tcnn::cpp::Module::initialize_params (cpp_api.cu:162-165): pcg32{seed} -> model->initialize_params
void or_init_params_pcg(const OrNetCfg* c, uint64_t seed, const float* geo_init, float* params) {
	init_params_from(c, pcg32(seed), geo_init, params);
}
// GridEncoding::initialize_params alone (grid.h:2375-2380) from pcg32{seed}: generate_random_uniform(rnd, n, -1e-4,
// 1e-4) with random.h:67-91's thread mapping (thread i draws 4 values for i + n_threads_padded * j)
void or_grid_init_pcg(uint64_t n, uint64_t seed, float* out) {
	pcg32 rnd(seed);
	const size_t N_TO_GEN = 4, n_threads = (n + N_TO_GEN - 1) / N_TO_GEN, n_pad = (n_threads + 127) / 128 * 128;
	for (size_t i = 0; i < n_pad; ++i) {
		pcg32 r = rnd; r.advance((int64_t)(i * N_TO_GEN));
		for (size_t j = 0; j < N_TO_GEN; ++j) {
			const size_t idx = i + n_pad * j;
			if (idx >= n) break;
			out[idx] = r.next_float() * (1e-4f - -1e-4f) + -1e-4f;
		}
	}
}
static void init_params_from(const OrNetCfg* c, pcg32 rnd, const float* geo_init, float* params) {
	Net n(*c);
	std::fill(params, params + n.n_params, 0.0f);
	auto xavier = [&](uint32_t off, uint32_t out, uint32_t in) {
		float scale = std::sqrt(6.0f / (float)(in + out));
		for (uint32_t i = 0; i < out * in; ++i) params[off + i] = rnd.next_float() * 2.0f * scale - scale;
	};
	for (auto& l : n.dl) xavier(l.offset, l.out, l.in);
	if (geo_init) std::memcpy(params, geo_init, sizeof(float) * n.n_density);
	for (auto& l : n.rl) xavier(l.offset, l.out, l.in);
	// grid: generate_random_uniform(rnd, n, -1e-4, 1e-4): thread i draws 4 values for i + n_threads*j
	{
		const size_t N = n.n_grid_params, N_TO_GEN = 4;
		const size_t n_threads = (N + N_TO_GEN - 1) / N_TO_GEN;
		const size_t n_threads_padded = (n_threads + 127) / 128 * 128;  // n_blocks_linear * 128
		for (size_t i = 0; i < n_threads_padded; ++i) {
			pcg32 r = rnd; r.advance((int64_t)(i * N_TO_GEN));
			for (size_t j = 0; j < N_TO_GEN; ++j) {
				size_t idx = i + n_threads_padded * j;
				if (idx >= N) break;
				params[n.grid_off + idx] = r.next_float() * (1e-4f - -1e-4f) + -1e-4f;
			}
		}
		rnd.advance((int64_t)N);
	}
	for (int k = 0; k < 4; ++k) params[n.var_off + k] = 0.3f;  // nerf_network.h:881-882
}

// Geometric init of the SDF MLP (my_tcnn/scripts/geometry_init_save_weights.py:291-331):
// W0[:, :3] ~ N(0, sqrt(2)/sqrt(out)), W0[:, 3:] = 0; hidden W ~ N(0, sqrt(2)/sqrt(out));
// last layer ~ N(sqrt(pi)/sqrt(in), 1e-5). Deterministic Box-Muller over pcg32(seed).
void or_geometric_init(const OrNetCfg* c, uint64_t seed, float* out) {
	Net n(*c);
	pcg32 r(seed);
	auto gauss = [&]() {
		float u1 = r.next_float(), u2 = r.next_float();
		if (u1 < 1e-7f) u1 = 1e-7f;
		return std::sqrt(-2.0f * std::log(u1)) * std::cos(6.28318530717958647692f * u2);
	};
	for (size_t li = 0; li < n.dl.size(); ++li) {
		const auto& ly = n.dl[li];
		for (uint32_t o = 0; o < ly.out; ++o) for (uint32_t i = 0; i < ly.in; ++i) {
			float v;
			if (li + 1 == n.dl.size()) v = std::sqrt(3.14159265358979f) / std::sqrt((float)ly.in) + 1e-5f * gauss();
			else if (li == 0) v = i < 3 ? std::sqrt(2.0f) / std::sqrt((float)ly.out) * gauss() : 0.0f;
			else v = std::sqrt(2.0f) / std::sqrt((float)ly.out) * gauss();
			out[ly.offset + (size_t)o * ly.in + i] = v;
		}
	}
}

void or_pcg32(uint64_t seed, uint64_t seq, int64_t advance, uint32_t n, uint32_t* out) {
	pcg32 r(seed, seq); if (advance) r.advance(advance);
	for (uint32_t i = 0; i < n; ++i) out[i] = r.next_uint();
}
float or_det_expf(float x) { return det_expf(x); }
void or_f2h(const float* in, uint16_t* out, uint64_t n) { for (uint64_t i = 0; i < n; ++i) out[i] = f2h(in[i]); }

// Hash-grid forward on n positions (AoS 3 floats); params are the full fp32 parameter vector
// (half-rounded internally, as the reference's m_params are fp16).
void or_grid_forward(const OrNetCfg* c, const float* params, uint32_t n_el, const float* pos, uint32_t valid_level, float* enc, float* dydx) {
	Net n(*c);
	std::vector<float> gp(n.n_grid_params);
	for (uint32_t i = 0; i < n.n_grid_params; ++i) gp[i] = rh(params[n.grid_off + i]);
	const uint32_t L = n.c.n_levels;
#pragma omp parallel for schedule(static)
	for (int64_t i = 0; i < (int64_t)n_el; ++i) grid_forward_one(n, gp.data(), pos + 3 * i, valid_level, enc + 2 * L * i, dydx ? dydx + 6 * L * i : nullptr);
}

static std::vector<float> half_params(const Net& n, const float* params) {
	std::vector<float> P(n.n_params);
	for (uint32_t i = 0; i < n.n_params; ++i) P[i] = rh(params[i]);
	return P;
}

// NerfNetwork::forward on n coords (AoS 7 floats) -> out AoS 16 halves.
void or_network_forward(const OrNetCfg* c, const float* params, uint32_t n_el, const float* coords, uint32_t valid_level, uint16_t* out) {
	Net n(*c);
	std::vector<float> P = half_params(n, params);
#pragma omp parallel for schedule(dynamic, 256)
	for (int64_t i = 0; i < (int64_t)n_el; ++i) { Ctx cx; net_forward_one(n, P.data(), coords + 7 * i, valid_level, cx, out + 16 * i); }
}

// Debug variant exposing the density-MLP internals for the autograd cross-check.
void or_network_forward_debug(const OrNetCfg* c, const float* params, const float* coord, uint32_t valid_level, float* grad_sdf, float* dout16, float* rout16) {
	Net n(*c);
	std::vector<float> P = half_params(n, params);
	Ctx cx; uint16_t o[16];
	net_forward_one(n, P.data(), coord, valid_level, cx, o);
	for (int d = 0; d < 3; ++d) grad_sdf[d] = cx.grad_sdf[d];
	for (int k = 0; k < 16; ++k) { dout16[k] = cx.dout[k]; rout16[k] = cx.rout[k]; }
}

// The matrix gradients accumulate per thread in double (plain adds) and are summed in thread order; the grid gradient
// (10 M entries) is shared, with atomic double adds.
static void network_backward_impl(const OrNetCfg* c, const float* params, uint32_t n_el, const float* coords, uint32_t valid_level,
                                  const uint16_t* dL_dout, uint32_t indeed_batch_size, float* grads, float* dpos) {
	Net n(*c);
	std::vector<float> P = half_params(n, params);
	std::vector<double> G(n.n_params, 0.0);
	const int nt = omp_get_max_threads();
	std::vector<std::vector<double>> Gm(nt);
	std::vector<double> var_acc(nt, 0.0);
	std::vector<uint16_t> Ghalf(g_grid_grad_mode == 2 ? n.n_grid_params : 0, (uint16_t)0);
	g_grid_half = Ghalf.data();
#pragma omp parallel
	{
		const int tid = omp_get_thread_num();
		Gm[tid].assign(n.n_matrix, 0.0);
#pragma omp for schedule(dynamic, 64)
		for (int64_t i = 0; i < (int64_t)n_el; ++i) {
			Ctx cx; net_forward_one(n, P.data(), coords + 7 * i, valid_level, cx, nullptr);
			if (dpos) dpos[4 * i + 3] = 0.f;
			net_backward_one(n, P.data(), coords + 7 * i, valid_level, cx, dL_dout + 16 * i, (float)indeed_batch_size, Gm[tid].data(),
			                 G.data() + n.grid_off, &var_acc[tid], dpos ? dpos + 4 * i : nullptr);
		}
	}
	double var = 0.0;
	for (int t = 0; t < nt; ++t) {
		var += var_acc[t];
		if (Gm[t].empty()) continue;
		for (uint32_t i = 0; i < n.n_matrix; ++i) G[i] += Gm[t][i];
	}
	if (g_grid_grad_mode == 2)
		for (uint32_t i = 0; i < n.n_grid_params; ++i) G[n.grid_off + i] = h2f(Ghalf[i]);
	g_grid_half = nullptr;
	for (uint32_t i = 0; i < n.n_params; ++i) grads[i] = (float)G[i];
	grads[n.var_off] = rh((float)var);
	for (int k = 1; k < 4; ++k) grads[n.var_off + k] = 0.0f;
}

// NerfNetwork::forward + backward (Overwrite) on n compacted coords with dL/doutput (AoS 16 halves).
// grads (n_params floats) is overwritten; variance grad = half(sum dL_dout[7]) (nerf_network.h:461-474).
void or_network_backward(const OrNetCfg* c, const float* params, uint32_t n_el, const float* coords, uint32_t valid_level,
                         const uint16_t* dL_dout, uint32_t indeed_batch_size, float* grads) {
	network_backward_impl(c, params, n_el, coords, valid_level, dL_dout, indeed_batch_size, grads, nullptr);
}

// or_network_backward plus dL/d(position) per sample (dpos: 4 floats per sample, the 4th 0).
void or_network_backward_pos(const OrNetCfg* c, const float* params, uint32_t n_el, const float* coords, uint32_t valid_level,
                             const uint16_t* dL_dout, uint32_t indeed_batch_size, float* grads, float* dpos) {
	network_backward_impl(c, params, n_el, coords, valid_level, dL_dout, indeed_batch_size, grads, dpos);
}

// -------------------------------------------------------------------------------------------
// generate_training_samples_nerf_with_global_movement (testbed_nerf.cu:1263-1456), static path
// (identity global movement, zero distortion, no envmap, cone_angle from the dataset), with the
// atomic appends replaced by the canonical ray-ordered layout: ray slot = ray index; rays with
// no samples or dropped by the max_samples cap get numsteps 0. Returns the reference's
// numsteps_counter (sum of requested steps, including dropped rays).
// rng_state/rng_inc: the m_rng passed by value to the kernel.
// -------------------------------------------------------------------------------------------
static inline uint32_t image_idx(uint32_t base_idx, uint32_t n_rays, uint32_t n_rays_total, uint32_t n_img) {
	return (((base_idx + n_rays_total) * n_img) / n_rays) % n_img;  // testbed_nerf.cu:1241-1261 (uint32 wrap)
}
static inline float read_rgba_x_alpha(const OrDataset* ds, uint32_t img, float xy_x, float xy_y, float rgba[4]) {
	const int rx = ds->resolution[2 * img], ry = ds->resolution[2 * img + 1];
	int px = clampi((int)(xy_x * (float)rx), 0, rx - 1);
	int py = clampi((int)(xy_y * (float)ry), 0, ry - 1);
	uint32_t v = ds->pixels[ds->pixel_offsets[img] + (uint64_t)px + (uint64_t)py * rx];
	if (v == 0x00FF00FFu) { rgba[0] = rgba[1] = rgba[2] = rgba[3] = -1.0f; return -1.0f; }
	float a = (float)((v >> 24) & 0xff) * (1.0f / 255.0f);
	rgba[0] = srgb_to_linear((float)(v & 0xff) * (1.0f / 255.0f)) * a;
	rgba[1] = srgb_to_linear((float)((v >> 8) & 0xff) * (1.0f / 255.0f)) * a;
	rgba[2] = srgb_to_linear((float)((v >> 16) & 0xff) * (1.0f / 255.0f)) * a;
	rgba[3] = a;
	return rgba[0];
}
static inline void random_image_pos(pcg32& rng, int rx, int ry, float& x, float& y) {  // :1226-1239
	x = rng.next_float(); y = rng.next_float();
	int ix = std::min(std::max((int)(x * (float)rx), 0), rx - 1);
	int iy = std::min(std::max((int)(y * (float)ry), 0), ry - 1);
	x = ((float)ix + 0.5f) / (float)rx; y = ((float)iy + 0.5f) / (float)ry;
}

struct RayGen { uint32_t n; float o[3], du[3], dir[3], startt, cone; bool valid; };

static RayGen gen_ray(const OrDataset* ds, const uint8_t* bitfield, uint32_t i, uint32_t n_rays_global, uint32_t n_rays_total, pcg32 rng) {
	RayGen g; g.valid = false; g.n = 0; g.startt = 0.f; g.cone = ds->cone_angle;
	for (int k = 0; k < 3; ++k) { g.o[k] = 0.f; g.du[k] = 0.f; g.dir[k] = 0.f; }
	uint32_t img = image_idx(i, n_rays_global, n_rays_total, ds->n_images);
	const int rx = ds->resolution[2 * img], ry = ds->resolution[2 * img + 1];
	rng.advance((int64_t)(uint32_t)(i * N_MAX_RANDOM_SAMPLES_PER_RAY));
	float xy_x, xy_y; random_image_pos(rng, rx, ry, xy_x, xy_y);
	float rgba[4];
	if (read_rgba_x_alpha(ds, img, xy_x, xy_y, rgba) <= 0.0f && rng.next_float() >= 0.9) return g;  // float vs double 0.9 (:1310)
	(void)rng.next_float();  // motionblur_time
	const float fx = ds->focal[2 * img], fy = ds->focal[2 * img + 1];
	const float ppx = ds->principal[2 * img], ppy = ds->principal[2 * img + 1];
	const float* M = ds->xform + 12 * img;
	float dc[3] = {(xy_x - ppx) * (float)rx / fx, (xy_y - ppy) * (float)ry / fy, 1.0f};
	for (int r = 0; r < 3; ++r) g.du[r] = (M[4 * r + 0] * dc[0] + M[4 * r + 1] * dc[1]) + M[4 * r + 2] * dc[2];
	for (int r = 0; r < 3; ++r) g.o[r] = M[4 * r + 3];
	float nrm = std::sqrt((g.du[0] * g.du[0] + g.du[1] * g.du[1]) + g.du[2] * g.du[2]);
	if (nrm > 0) { for (int r = 0; r < 3; ++r) g.dir[r] = g.du[r] / nrm; } else { for (int r = 0; r < 3; ++r) g.dir[r] = g.du[r]; }
	if (ds->motion_on) {  // moved ray; the record then holds the moved unit direction (testbed_nerf.cu:1380-1387)
		move_ray(ds, g.o, g.dir);
		for (int r = 0; r < 3; ++r) g.du[r] = g.dir[r];
	}
	AABB bb{{ds->aabb_min[0], ds->aabb_min[1], ds->aabb_min[2]}, {ds->aabb_max[0], ds->aabb_max[1], ds->aabb_max[2]}};
	V3 o = {g.o[0], g.o[1], g.o[2]}, dir = {g.dir[0], g.dir[1], g.dir[2]};
	float tmin, tmax; ray_intersect(bb, o, dir, tmin, tmax);
	g.cone = ds->cone_angle;
	tmin = std::fmax(tmin, 0.0f);
	float startt = tmin;
	startt += calc_dt(startt, g.cone) * rng.next_float();
	g.startt = startt;
	V3 idir = {1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z};
	uint32_t j = 0; float t = startt; V3 pos;
	while (true) {
		pos = {o.x + t * dir.x, o.y + t * dir.y, o.z + t * dir.z};
		if (!(aabb_contains(bb, pos) && j < NERF_STEPS)) break;
		float dt = calc_dt(t, g.cone);
		uint32_t mip = (uint32_t)mip_from_dt(dt, pos);
		if (density_grid_occupied_at(pos, bitfield, mip)) { ++j; t += dt; }
		else { uint32_t res = NERF_GRIDSIZE >> mip; t = advance_to_next_voxel(t, g.cone, pos, dir, idir, res); }
	}
	g.n = j; g.valid = j > 0;
	return g;
}

static void write_ray_samples(const OrDataset* ds, const uint8_t* bitfield, const RayGen& g, float* coords_out) {
	AABB bb{{ds->aabb_min[0], ds->aabb_min[1], ds->aabb_min[2]}, {ds->aabb_max[0], ds->aabb_max[1], ds->aabb_max[2]}};
	V3 o = {g.o[0], g.o[1], g.o[2]}, dir = {g.dir[0], g.dir[1], g.dir[2]};
	V3 idir = {1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z};
	float wd[3] = {(dir.x + 1.0f) * 0.5f, (dir.y + 1.0f) * 0.5f, (dir.z + 1.0f) * 0.5f};
	float diag[3] = {bb.mx.x - bb.mn.x, bb.mx.y - bb.mn.y, bb.mx.z - bb.mn.z};
	uint32_t j = 0; float t = g.startt; V3 pos;
	while (true) {
		pos = {o.x + t * dir.x, o.y + t * dir.y, o.z + t * dir.z};
		if (!(aabb_contains(bb, pos) && j < g.n)) break;
		float dt = calc_dt(t, g.cone);
		uint32_t mip = (uint32_t)mip_from_dt(dt, pos);
		if (density_grid_occupied_at(pos, bitfield, mip)) {
			float* cc = coords_out + 7 * (size_t)j;
			cc[0] = (pos.x - bb.mn.x) / diag[0]; cc[1] = (pos.y - bb.mn.y) / diag[1]; cc[2] = (pos.z - bb.mn.z) / diag[2];
			cc[3] = warp_dt(dt);
			cc[4] = wd[0]; cc[5] = wd[1]; cc[6] = wd[2];
			++j; t += dt;
		} else { uint32_t res = NERF_GRIDSIZE >> mip; t = advance_to_next_voxel(t, g.cone, pos, dir, idir, res); }
	}
}

// rays_out: 6 floats per ray (o, unnormalized d); numsteps_out: 2 per ray (n, base).
uint32_t or_generate_samples(const OrDataset* ds, const uint8_t* bitfield, uint32_t n_rays, uint32_t ray_offset, uint32_t n_rays_global,
                             uint32_t n_rays_total, uint64_t rng_state, uint64_t rng_inc, uint32_t max_samples,
                             float* rays_out, uint32_t* numsteps_out, float* coords_out, uint32_t* n_rays_with_samples) {
	pcg32 rng; rng.state = rng_state; rng.inc = rng_inc;
	std::vector<RayGen> gens(n_rays);
#pragma omp parallel for schedule(dynamic, 64)
	for (int64_t i = 0; i < (int64_t)n_rays; ++i) gens[i] = gen_ray(ds, bitfield, (uint32_t)i + ray_offset, n_rays_global, n_rays_total, rng);
	// Canonical order of the reference's atomicAdd(numsteps_counter): the counter advances for
	// every ray with samples, and a ray is kept iff base + n <= max_samples (a prefix).
	uint32_t base = 0, nr = 0;
	std::vector<uint32_t> bases(n_rays);
	for (uint32_t i = 0; i < n_rays; ++i) {
		bases[i] = base;
		const uint32_t n = gens[i].n;
		if (n > 0 && base + n <= max_samples) ++nr;
		else gens[i].valid = false;
		base += n;
	}
#pragma omp parallel for schedule(dynamic, 64)
	for (int64_t i = 0; i < (int64_t)n_rays; ++i) {
		const RayGen& g = gens[i];
		for (int k = 0; k < 3; ++k) { rays_out[6 * i + k] = g.o[k]; rays_out[6 * i + 3 + k] = g.du[k]; }
		numsteps_out[2 * i + 0] = g.valid ? g.n : 0;
		numsteps_out[2 * i + 1] = bases[i];
		if (g.valid) write_ray_samples(ds, bitfield, g, coords_out + 7 * (size_t)bases[i]);
	}
	if (n_rays_with_samples) *n_rays_with_samples = nr;
	// numsteps_counter counts every ray with j > 0, dropped or not (testbed_nerf.cu:1427-1431)
	return base;
}

// -------------------------------------------------------------------------------------------
// compute_loss_kernel_train_nerf_with_global_movement (testbed_nerf.cu:1475-1997), static path:
// Huber(0.1)/5 loss, Logistic rgb activation, linear color space with sRGB targets
// (color_space Linear, linear_colors false: :1671-1676), random background, no envmap/exposure/
// depth, mask-loss weight given, cos_anneal_ratio given. Canonical compaction order = ray order.
// Inputs: numsteps (2/ray as produced above), network_output AoS16 halves. Outputs: compacted
// coords, dL/doutput AoS16 halves, per-ray loss/ek/mask, numsteps rewritten to (n_compacted, base).
// Returns the compacted-sample counter (sum of requested compacted steps, pre-cap).
// -------------------------------------------------------------------------------------------
struct LossRay { uint32_t ncomp; };

// Target pixel (sRGB) over a random background and the background itself (testbed_nerf.cu:1632-1660).
static void ray_target(const OrDataset* ds, uint32_t ray_idx_global, uint32_t n_rays_global, uint32_t n_rays_total, pcg32 rng,
                       float target[3], float bg[3], float tex[4]) {
	rng.advance((int64_t)(uint32_t)(ray_idx_global * N_MAX_RANDOM_SAMPLES_PER_RAY));
	uint32_t img = image_idx(ray_idx_global, n_rays_global, n_rays_total, ds->n_images);
	const int rx = ds->resolution[2 * img], ry = ds->resolution[2 * img + 1];
	float xy_x, xy_y; random_image_pos(rng, rx, ry, xy_x, xy_y);
	// train_with_random_bg_color, else the testbed background colour (:1642-1645)
	if (ds->fixed_bg) for (int k = 0; k < 3; ++k) bg[k] = ds->bg_color[k];
	else { bg[0] = rng.next_float(); bg[1] = rng.next_float(); bg[2] = rng.next_float(); }
	for (int k = 0; k < 3; ++k) bg[k] = srgb_to_linear(bg[k]);
	read_rgba_x_alpha(ds, img, xy_x, xy_y, tex);
	for (int k = 0; k < 3; ++k) {
		if (ds->target_mode == 1) {  // color_space SRGB (:1664-1670)
			bg[k] = linear_to_srgb(bg[k]);
			target[k] = tex[3] > 0.0f ? linear_to_srgb(1.0f * tex[k] / tex[3]) * tex[3] + (1.0f - tex[3]) * bg[k] : bg[k];
		} else {                     // color_space Linear; linear_colors (mode 2) keeps linear targets (:1658-1663)
			target[k] = 1.0f * tex[k] + (1.0f - tex[3]) * bg[k];
			if (ds->target_mode == 0) { target[k] = linear_to_srgb(target[k]); bg[k] = linear_to_srgb(bg[k]); }
		}
	}
}

static void loss_ray(const OrDataset* ds, uint32_t i, uint32_t ray_idx_global, uint32_t n_rays_global, uint32_t n_rays_total, pcg32 rng,
                     const float* ray, const uint32_t numsteps, const float* coords_in, const uint16_t* net_out,
                     uint32_t compacted_base, uint32_t compacted_numsteps_cap, bool write, float loss_scale_orig,
                     float mean_density, float ek_w, float mask_w, float cos_anneal,
                     uint32_t* ncomp_out, float* coords_out, uint16_t* dout, float* loss_out, float* ek_out, float* mask_out) {
	AABB bb{{ds->aabb_min[0], ds->aabb_min[1], ds->aabb_min[2]}, {ds->aabb_max[0], ds->aabb_max[1], ds->aabb_max[2]}};
	float diag[3] = {bb.mx.x - bb.mn.x, bb.mx.y - bb.mn.y, bb.mx.z - bb.mn.z};
	float T = 1.f; const float EPSILON = 1e-4f;
	float rgb_ray[3] = {0, 0, 0}, hit[3] = {0, 0, 0};
	float depth_ray = 0.f, weight_sum = 0.f;
	uint32_t cn = 0;
	float ro[3] = {ray[0], ray[1], ray[2]};
	float dir[3];
	{ float nr = std::sqrt((ray[3] * ray[3] + ray[4] * ray[4]) + ray[5] * ray[5]); for (int k = 0; k < 3; ++k) dir[k] = nr > 0 ? ray[3 + k] / nr : ray[3 + k]; }
	for (; cn < numsteps; ++cn) {
		if (T < EPSILON) break;
		const uint16_t* lo = net_out + 16 * (size_t)cn;
		const float* ci = coords_in + 7 * (size_t)cn;
		float rgb[3]; for (int k = 0; k < 3; ++k) rgb[k] = det_logistic(h2f(lo[k]));
		float pos[3]; for (int k = 0; k < 3; ++k) pos[k] = (&bb.mn.x)[k] + ci[k] * diag[k];
		float dt = unwarp_dt(ci[3]);
		float dd[3] = {pos[0] - ro[0], pos[1] - ro[1], pos[2] - ro[2]};
		float cur_depth = std::sqrt((dd[0] * dd[0] + dd[1] * dd[1]) + dd[2] * dd[2]);
		if (cn == 0) {  // BENT_DIR (testbed_nerf.cu:1583-1588)
			float u[3]; for (int k = 0; k < 3; ++k) u[k] = h2f(lo[8 + k]) * 2.0f - 1.0f;
			float nr = std::sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
			for (int k = 0; k < 3; ++k) dir[k] = nr > 0 ? u[k] / nr : u[k];
		}
		float inv_s = det_expf(rh(10.0f * h2f(lo[7])));
		float sdf = h2f(lo[3]);
		float pg[3] = {h2f(lo[4]), h2f(lo[5]), h2f(lo[6])};
		float true_cos = dir[0] * pg[0] + dir[1] * pg[1] + dir[2] * pg[2];
		float a1 = (float)(-true_cos * 0.5 + 0.5); a1 = a1 > 0.0f ? a1 : 0.0f;
		float a2 = -true_cos; a2 = a2 > 0.0f ? a2 : 0.0f;
		float iter_cos = -(a1 * (1.0 - cos_anneal) + a2 * cos_anneal);
		float next_sdf = sdf + iter_cos * dt * 0.5;
		float prev_sdf = sdf - iter_cos * dt * 0.5;
		float next_cdf = det_logistic(next_sdf * inv_s);
		float prev_cdf = det_logistic(prev_sdf * inv_s);
		float p = prev_cdf - next_cdf, c = prev_cdf;
		float p_div_c = (p + 1e-5f) / (c + 1e-5f);
		const float alpha = clampf(p_div_c, 0.0f, 1.0f);
		const float weight = alpha * T;
		for (int k = 0; k < 3; ++k) { rgb_ray[k] += weight * rgb[k]; hit[k] += weight * pos[k]; }
		depth_ray += weight * cur_depth; weight_sum += weight;
		T *= (1.f - alpha);
	}
	*ncomp_out = cn;
	if (!write) return;

	float target[3], bg[3], tex[4];
	ray_target(ds, ray_idx_global, n_rays_global, n_rays_total, rng, target, bg, tex);
	if (cn == numsteps) for (int k = 0; k < 3; ++k) rgb_ray[k] += T * bg[k];

	uint32_t comp = std::min(compacted_numsteps_cap - std::min(compacted_numsteps_cap, compacted_base), cn);
	*ncomp_out = comp;
	if (comp == 0) return;

	// Huber(alpha=0.1)/5 (testbed_nerf.cu:311-327, 1469)
	float lgrad[3], lloss[3];
	for (int k = 0; k < 3; ++k) {
		float diff = rgb_ray[k] - target[k], ad = std::fabs(diff), sq = 0.5f / 0.1f * diff * diff;
		lloss[k] = (ad > 0.1f ? (ad - 0.5f * 0.1f) : sq) / 5.0f;
		lgrad[k] = (ad > 0.1f ? (diff > 0 ? 1.0f : -1.0f) : (diff / 0.1f)) / 5.0f;
	}
	float mask_gt = (float)(tex[3] > 0.9999f);
	float gws;
	if (weight_sum >= 1.0 - 1e-4) { weight_sum = 1.0 - 1e-4; gws = 0.0f; }
	else if (weight_sum <= 1e-4) { weight_sum = 1e-4; gws = 0.0f; }
	else { float sws = 1.0f / (1.0f + std::exp(-weight_sum)); gws = (mask_gt - sws) * weight_sum * mask_w; }
	float mean_loss = ((lloss[0] + lloss[1]) + lloss[2]) / 3.0f;
	loss_out[0] = mean_loss / (float)n_rays_global;
	mask_out[0] = -(mask_gt * std::log(weight_sum) + (1 - mask_gt) * std::log(1 - weight_sum));
	ek_out[0] = 0.f;

	const float loss_scale = loss_scale_orig / n_rays_global;
	const float output_l2_reg = 0.0f;  // Logistic activation
	(void)mean_density;
	float rgb2[3] = {0, 0, 0}; float ws2 = 0.f, depth2 = 0.f;
	T = 1.f;
	for (uint32_t j = 0; j < comp; ++j) {
		const float* ci = coords_in + 7 * (size_t)j;
		std::memcpy(coords_out + 7 * (size_t)j, ci, 7 * sizeof(float));
		const uint16_t* lo = net_out + 16 * (size_t)j;
		float pos[3]; for (int k = 0; k < 3; ++k) pos[k] = (&bb.mn.x)[k] + ci[k] * diag[k];
		float dd[3] = {pos[0] - ro[0], pos[1] - ro[1], pos[2] - ro[2]};
		float depth = std::sqrt((dd[0] * dd[0] + dd[1] * dd[1]) + dd[2] * dd[2]);
		float dt = unwarp_dt(ci[3]);
		float raw[3], rgb[3]; for (int k = 0; k < 3; ++k) { raw[k] = h2f(lo[k]); rgb[k] = det_logistic(raw[k]); }
		float inv_s = det_expf(rh(10.0f * h2f(lo[7])));
		float sdf = h2f(lo[3]);
		float pg[3] = {h2f(lo[4]), h2f(lo[5]), h2f(lo[6])};
		float true_cos = dir[0] * pg[0] + dir[1] * pg[1] + dir[2] * pg[2];
		float a1 = (float)(-true_cos * 0.5 + 0.5); a1 = a1 > 0.0f ? a1 : 0.0f;
		float a2 = -true_cos; a2 = a2 > 0.0f ? a2 : 0.0f;
		float iter_cos = -(a1 * (1.0 - cos_anneal) + a2 * cos_anneal);
		float next_sdf = sdf + iter_cos * dt * 0.5;
		float prev_sdf = sdf - iter_cos * dt * 0.5;
		float next_cdf = det_logistic(next_sdf * inv_s);
		float prev_cdf = det_logistic(prev_sdf * inv_s);
		float p = prev_cdf - next_cdf, c = prev_cdf;
		float p_div_c = (p + 1e-5f) / (c + 1e-5f);
		const float alpha = clampf(p_div_c, 0.0f, 1.0f);
		const float weight = alpha * T;
		for (int k = 0; k < 3; ++k) rgb2[k] += weight * rgb[k];
		depth2 += weight * depth; ws2 += weight;
		T *= (1.f - alpha);
		float suffix[3]; for (int k = 0; k < 3; ++k) suffix[k] = rgb_ray[k] - rgb2[k];
		float dl[16]; for (int k = 0; k < 16; ++k) dl[k] = 0.0f;
		for (int k = 0; k < 3; ++k) {
			float sig = det_logistic(raw[k]);
			dl[k] = loss_scale * ((weight * lgrad[k]) * (sig * (1 - sig)) + std::fmax(0.0f, output_l2_reg * raw[k]));
		}
		float tr[3]; for (int k = 0; k < 3; ++k) tr[k] = T * rgb[k] - suffix[k];
		float dot = (lgrad[0] * tr[0] + lgrad[1] * tr[1]) + lgrad[2] * tr[2];
		float dloss_dalpha = (dot + gws * (1 - weight_sum)) / (1.0f - alpha + 1e-5);
		float dadem = 0, dem_dsdf = 0, dem_dinvs = 0, dadpe = 0, dpe_dinvs = 0, dpe_dic = 0, dem_dic = 0;
		if (!(p_div_c <= 0.0f || p_div_c >= 1.0f)) {
			float plus_x = inv_s * iter_cos * dt;
			float plus_e = det_expf(plus_x);
			float e_minus = det_expf(-next_sdf * inv_s);
			dem_dsdf = -inv_s * e_minus;
			dem_dinvs = -next_sdf * e_minus;
			float a = 1 + e_minus;
			float b = 1 + plus_e * e_minus;
			float cc = 1e-5 + 1 / (1 + plus_e * e_minus);
			float delta = a * (b * b) * (cc * cc);
			dadem = -(plus_e / (delta) - 1 / (a * a * cc));
			dadpe = -e_minus / (delta);
			dpe_dinvs = plus_e * iter_cos * dt;
			dpe_dic = plus_e * inv_s * dt;
			dem_dic = -inv_s * e_minus * dt * 0.5;
		}
		float dloss_dinvs = dloss_dalpha * (dadem * dem_dinvs + dadpe * dpe_dinvs);
		float dloss_dvar = dloss_dinvs * inv_s * 10;
		float d_ic_tc = true_cos >= 0 ? 0.0f : 1.0f;
		float gn = std::sqrt(pg[0] * pg[0] + pg[1] * pg[1] + pg[2] * pg[2] + 1e-6);
		float gn_inv = 1 - 1 / gn;
		float dloss_dnn = dloss_dalpha * (dadem * dem_dic + dpe_dic * dadpe) * d_ic_tc;
		float dloss_dsdf = dloss_dalpha * dadem * dem_dsdf;
		dl[3] = loss_scale * dloss_dsdf;
		ek_out[0] += (gn - 1.0f) * (gn - 1.0f);
		for (int k = 0; k < 3; ++k) dl[4 + k] = rh(ek_w * 2 * loss_scale_orig * gn_inv * pg[k]);
		dl[7] = rh(loss_scale * dloss_dvar);
		for (int k = 0; k < 3; ++k) dl[8 + k] = rh(loss_scale * dloss_dnn * dir[k]);
		for (int k = 0; k < 16; ++k) dout[16 * (size_t)j + k] = f2h(dl[k]);
	}
	ek_out[0] /= (float)comp * (float)n_rays_global;
}

void or_ray_target(const OrDataset* ds, uint32_t ray_idx_global, uint32_t n_rays_global, uint32_t n_rays_total, uint64_t rng_state,
                   uint64_t rng_inc, float* target_srgb, float* bg_srgb) {
	pcg32 rng; rng.state = rng_state; rng.inc = rng_inc;
	float tex[4];
	ray_target(ds, ray_idx_global, n_rays_global, n_rays_total, rng, target_srgb, bg_srgb, tex);
}

uint32_t or_compute_loss(const OrDataset* ds, uint32_t n_rays, uint32_t ray_offset, uint32_t n_rays_global, uint32_t n_rays_total,
                         uint64_t rng_state, uint64_t rng_inc, uint32_t max_samples_compacted,
                         const float* rays, uint32_t* numsteps, const float* coords_in, const uint16_t* net_out,
                         float loss_scale, float mean_density, float ek_w, float mask_w, float cos_anneal,
                         float* coords_out, uint16_t* dL_dout, float* loss_out, float* ek_out, float* mask_out) {
	pcg32 rng; rng.state = rng_state; rng.inc = rng_inc;
	std::vector<uint32_t> cn(n_rays, 0);
#pragma omp parallel for schedule(dynamic, 64)
	for (int64_t i = 0; i < (int64_t)n_rays; ++i) {
		loss_out[i] = 0; ek_out[i] = 0; mask_out[i] = 0;
		const uint32_t ns = numsteps[2 * i], base = numsteps[2 * i + 1];
		if (ns == 0) continue;
		loss_ray(ds, (uint32_t)i, (uint32_t)i + ray_offset, n_rays_global, n_rays_total, rng, rays + 6 * i, ns, coords_in + 7 * (size_t)base, net_out + 16 * (size_t)base,
		         0, 0, false, loss_scale, mean_density, ek_w, mask_w, cos_anneal, &cn[i], nullptr, nullptr, nullptr, nullptr, nullptr);
	}
	std::vector<uint32_t> cbase(n_rays);
	uint32_t counter = 0;
	for (uint32_t i = 0; i < n_rays; ++i) { cbase[i] = counter; counter += cn[i]; }
#pragma omp parallel for schedule(dynamic, 64)
	for (int64_t i = 0; i < (int64_t)n_rays; ++i) {
		const uint32_t ns = numsteps[2 * i], base = numsteps[2 * i + 1];
		if (ns == 0) { numsteps[2 * i] = 0; numsteps[2 * i + 1] = cbase[i]; continue; }
		uint32_t comp = 0;
		const uint32_t cb = cbase[i];
		const bool fits = cb < max_samples_compacted;
		loss_ray(ds, (uint32_t)i, (uint32_t)i + ray_offset, n_rays_global, n_rays_total, rng, rays + 6 * i, ns, coords_in + 7 * (size_t)base, net_out + 16 * (size_t)base,
		         cb, max_samples_compacted, true, loss_scale, mean_density, ek_w, mask_w, cos_anneal, &comp,
		         fits ? coords_out + 7 * (size_t)cb : nullptr, fits ? dL_dout + 16 * (size_t)cb : nullptr, loss_out + i, ek_out + i, mask_out + i);
		numsteps[2 * i] = comp; numsteps[2 * i + 1] = cb;
	}
	return counter;
}

// fill_rollover_and_rescale / fill_rollover (my_tcnn common_device.h:515-535)
void or_fill_rollover(uint32_t n_elements, uint32_t n_in, float* coords, uint16_t* dL_dout) {
	if (n_in == 0) return;
	for (uint64_t i = (uint64_t)n_in * 7; i < (uint64_t)n_elements * 7; ++i) coords[i] = coords[i % ((uint64_t)n_in * 7)];
	for (uint64_t i = (uint64_t)n_in * 16; i < (uint64_t)n_elements * 16; ++i) {
		float r = h2f(dL_dout[i % ((uint64_t)n_in * 16)]);
		dL_dout[i] = f2h(r * n_in / n_elements);
	}
}

// Ema(Adam) step (adam.h:51-160, 266-330; ema.h:45-110; exponential_decay.h:61-80).
// grads are the fp32 (reference: fp16) gradients; loss_scale 128. n_matrix params get L2 and are
// never skipped; non-matrix params skip on an exactly-zero gradient. steps is per-param.
void or_adam_ema_step(uint32_t n, uint32_t n_matrix, float loss_scale, float lr, float beta1, float beta2, float eps, float l2_reg,
                      uint32_t optimizer_step /*after increment*/, float ema_decay,
                      float* weights_fp, const float* grads, float* m1, float* m2, uint32_t* steps, float* ema_tmp, float* ema_out) {
	float ema_old = 1 - (float)std::pow(ema_decay, optimizer_step - 1);
	float ema_new = 1.0f / (1 - (float)std::pow(ema_decay, optimizer_step));
#pragma omp parallel for schedule(static)
	for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
		const uint32_t i = (uint32_t)ii;
		float gradient = grads[i] / loss_scale;
		const bool is_matrix = i < n_matrix;
		bool skip = !is_matrix && gradient == 0;
		if (!skip) {
			const float w = weights_fp[i];
			if (is_matrix) gradient += l2_reg * w;
			const float g2 = gradient * gradient;
			float fm = m1[i] = beta1 * m1[i] + (1 - beta1) * gradient;
			const float sm = m2[i] = beta2 * m2[i] + (1 - beta2) * g2;
			float lr_i = lr;
			const uint32_t cs = ++steps[i];
			lr_i *= std::sqrt(1 - std::pow(beta2, (float)cs)) / (1 - std::pow(beta1, (float)cs));
			const float elr = std::fmin(std::fmax(lr_i / (std::sqrt(sm) + eps), 0.0f), std::numeric_limits<float>::max());
			weights_fp[i] = w - elr * fm;
		}
		float wh = rh(weights_fp[i]);
		float f = (ema_tmp[i] * ema_decay * ema_old + wh * (1 - ema_decay)) * ema_new;
		ema_tmp[i] = f; ema_out[i] = rh(f);
	}
}

// -------------------------------------------------------------------------------------------
// Occupancy grid update (testbed_nerf.cu:3293-3397, 640-795; nerf_network.h:656-739;
// common_operation.cuh:306-324). max_cascade = 0 path. density_grid: 128^3 floats; bitfield:
// 128^3/8 * 8 mips bytes. rng: density_grid_rng by value; returns rng advanced twice.
// -------------------------------------------------------------------------------------------
void or_density_grid_update(const OrNetCfg* c, const float* params, uint32_t valid_level, const float* aabb_min, const float* aabb_max,
                            uint32_t n_uniform, uint32_t n_nonuniform, uint32_t ema_step, float decay,
                            uint64_t* rng_state, uint64_t rng_inc, float* density_grid, uint8_t* bitfield, float* mean_out) {
	Net n(*c);
	std::vector<float> P = half_params(n, params);
	const uint32_t G3 = NERF_GRIDSIZE * NERF_GRIDSIZE * NERF_GRIDSIZE;
	const uint32_t n_cascades = 1;
	const uint32_t N = n_uniform + n_nonuniform;
	std::vector<float> pos(3 * (size_t)N); std::vector<uint32_t> idxs(N);
	pcg32 rng; rng.state = *rng_state; rng.inc = rng_inc;
	float diag[3] = {aabb_max[0] - aabb_min[0], aabb_max[1] - aabb_min[1], aabb_max[2] - aabb_min[2]};
	auto gen = [&](uint32_t n_el, uint32_t out_off, float thresh, pcg32 r0) {
#pragma omp parallel for schedule(static)
		for (int64_t ii = 0; ii < (int64_t)n_el; ++ii) {
			const uint32_t i = (uint32_t)ii;
			pcg32 r = r0; r.advance((int64_t)(uint32_t)(i * 4));
			uint32_t level = (uint32_t)(r.next_float() * n_cascades) % n_cascades;
			uint32_t idx = 0;
			for (uint32_t j = 0; j < 10; ++j) {
				idx = ((i + ema_step * n_el) * 56924617u + j * 19349663u + 96925573u) % G3;
				idx += level * G3;
				if (density_grid[idx] > thresh) break;
			}
			uint32_t pi = idx % G3;
			uint32_t x = morton3D_invert(pi >> 0), y = morton3D_invert(pi >> 1), z = morton3D_invert(pi >> 2);
			float rx = r.next_float(), ry = r.next_float(), rz = r.next_float();
			float sc = std::scalbn(1.0f, (int)level);
			float p[3] = {(((float)x + rx) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f, (((float)y + ry) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f,
			              (((float)z + rz) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f};
			for (int k = 0; k < 3; ++k) pos[3 * (size_t)(out_off + i) + k] = (p[k] - aabb_min[k]) / diag[k];
			idxs[out_off + i] = idx;
		}
	};
	gen(n_uniform, 0, -0.01f, rng); rng.advance();
	gen(n_nonuniform, n_uniform, NERF_MIN_OPTICAL_THICKNESS, rng); rng.advance();
	*rng_state = rng.state;
	std::vector<float> tmp(G3 * n_cascades, 0.0f);
	std::vector<float> dens(N);
	const float var_h = P[n.var_off];
#pragma omp parallel for schedule(dynamic, 256)
	for (int64_t i = 0; i < (int64_t)N; ++i) {
		// NerfNetwork::density -> sdf (grid fwd + density MLP, + bias half add) -> sdf_to_density_variance_buffer
		Ctx cx; float enc[64];
		grid_forward_one(n, P.data() + n.grid_off, &pos[3 * i], valid_level, enc, nullptr);
		float din[64] = {0};
		for (int d = 0; d < 3; ++d) din[d] = rh(rh(pos[3 * i + d]) - rh(0.5f));
		for (uint32_t k = 0; k < 2 * c->n_levels; ++k) din[3 + k] = enc[k];
		const float* in = din; uint32_t nin = c->density_in; float t[64], hbuf[4][64];
		for (size_t li = 0; li + 1 < n.dl.size(); ++li) {
			matvec(P.data() + n.dl[li].offset, c->width, nin, in, t);
			for (uint32_t o = 0; o < c->width; ++o) hbuf[li][o] = rh(t[o] > 0 ? t[o] : 0.0f);
			in = hbuf[li]; nin = c->width;
		}
		matvec(P.data() + n.dl.back().offset, 16, c->width, in, t);
		float sdf = rh(rh(t[0]) + rh(c->sdf_bias));
		float s = rh(std::exp(rh(var_h * 10.0f)));
		float sig = rh(1.0f / (1.0f + std::exp(-rh(sdf * s))));
		float d = rh(rh(s * sig) * rh(1.0f - sig));
		dens[i] = d;
		(void)cx;
	}
	for (uint32_t i = 0; i < N; ++i) {  // splat_grid_samples_nerf_max_nearest_neighbor (atomicMax on uint bits)
		uint32_t a, b; std::memcpy(&a, &tmp[idxs[i]], 4); std::memcpy(&b, &dens[i], 4);
		if (b > a) tmp[idxs[i]] = dens[i];
	}
	for (uint32_t i = 0; i < G3 * n_cascades; ++i) {  // ema_grid_samples_nerf
		float prev = density_grid[i];
		density_grid[i] = (prev < 0.f) ? prev : std::fmax(prev * decay, tmp[i]);
	}
	// update_density_grid_mean_and_bitfield (testbed_nerf.cu:3371-3397)
	double sum = 0.0;
	for (uint32_t i = 0; i < G3; ++i) sum += (double)(std::fmax(density_grid[i], 0.f) / (float)G3);
	const float mean = (float)sum;
	*mean_out = mean;
	const uint32_t nbytes = G3 / 8;
	const float thresh = std::min(NERF_MIN_OPTICAL_THICKNESS, mean);
	for (uint32_t i = 0; i < nbytes * NERF_CASCADES; ++i) {
		if (i >= nbytes * n_cascades) { bitfield[i] = 0; continue; }
		uint8_t bits = 0;
		for (uint8_t j = 0; j < 8; ++j) bits |= density_grid[i * 8 + j] > thresh ? ((uint8_t)1 << j) : 0;
		bitfield[i] = bits;
	}
	for (uint32_t level = 1; level < NERF_CASCADES; ++level) {
		const uint8_t* prev = bitfield + nbytes * (level - 1);
		uint8_t* next = bitfield + nbytes * level;
		for (uint32_t i = 0; i < G3 / 64; ++i) {
			uint8_t bits = 0;
			for (uint8_t j = 0; j < 8; ++j) bits |= prev[i * 8 + j] > 0 ? ((uint8_t)1 << j) : 0;
			uint32_t x = morton3D_invert(i >> 0) + NERF_GRIDSIZE / 8, y = morton3D_invert(i >> 1) + NERF_GRIDSIZE / 8, z = morton3D_invert(i >> 2) + NERF_GRIDSIZE / 8;
			next[morton3D(x, y, z)] |= bits;
		}
	}
}

int or_num_threads() {
#ifdef _OPENMP
	return omp_get_max_threads();
#else
	return 1;
#endif
}


// -------------------------------------------------------------------------------------------
// Rendering of one camera (Testbed::render_to_cpu, python_api.cu:123-169, Shade mode): per spp
// init_rays_with_payload_kernel_nerf + advance_pos_nerf (testbed_nerf.cu:2208-2330, 797-846), then
// NerfTracer::trace (:2479-2600): compact alive rays, n_steps = clamp(n_init / n_alive, 1, 8),
// generate_next_nerf_network_inputs (:877-934), network inference, composite_kernel_nerf (:936-1106),
// shade_kernel_nerf (:2148-2181) for rays with alpha > 0.001; accumulate_kernel in linear colour
// (render_buffer.cu:217-260). Pixel offsets: ld_random_pixel_offset (random_val.cuh:254-322).
// -------------------------------------------------------------------------------------------
static inline uint32_t or_rev(uint32_t x) {
	x = ((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1); x = ((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2);
	x = ((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4); x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
	return (x >> 16) | (x << 16);
}
static inline uint32_t or_lk(uint32_t x, uint32_t seed) {  // laine_karras_permutation (random_val.cuh:236-243)
	x += seed; x ^= x * 0x6c50b47cu; x ^= x * 0xb82f1e52u; x ^= x * 0xc7afe638u; x ^= x * 0x8d22f6e6u; return x;
}
static inline uint32_t or_scr(uint32_t x, uint32_t seed) { return or_rev(or_lk(or_rev(x), seed)); }
static inline uint32_t or_hc(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }
static uint32_t or_sobol(uint32_t index, uint32_t dim) {  // random_val.cuh:159-252, dimensions 0 and 1
	static uint32_t D[2][32];
	static bool init = false;
	if (!init) {
		uint32_t d = 0x80000000u;
		for (int b = 0; b < 32; ++b) { D[0][b] = 0x80000000u >> b; D[1][b] = d; d ^= d >> 1; }
		init = true;
	}
	uint32_t X = 0;
	for (uint32_t bit = 0; bit < 32; ++bit) X ^= ((index >> bit) & 1) * D[dim][bit];
	return X;
}
static float or_ld_random_val(uint32_t index, uint32_t seed) {
	index = or_scr(index, seed);
	return (float)or_scr(or_sobol(index, 0), or_hc(seed, 0)) * float(1.0 / 4294967296.0);
}
static void or_ld_random_val_2d(uint32_t index, uint32_t seed, float o[2]) {
	index = or_scr(index, seed);
	for (uint32_t i = 0; i < 2; ++i) o[i] = (float)or_scr(or_sobol(index, i), or_hc(seed, i)) * float(1.0 / 4294967296.0);
}

struct OrRenderCamera { float xform[12]; float focal[2], screen_center[2]; uint32_t width, height; };
struct OrRay { V3 o, d; float t; bool alive; uint32_t idx, n_steps; float rgba[4]; };

float or_ld_random_val_export(uint32_t index, uint32_t seed) { return or_ld_random_val(index, seed); }
uint32_t or_sobol_export(uint32_t index, uint32_t dim) { return or_sobol(index, dim & 1); }
void or_ld_random_val_2d_export(uint32_t index, uint32_t seed, float* o) { or_ld_random_val_2d(index, seed, o); }

void or_render(const OrNetCfg* c, const float* params, uint32_t valid_level, const OrDataset* ds, const uint8_t* bitfield,
               const OrRenderCamera* cam, uint32_t spp, int snap, float min_transmittance, float cos_anneal, float* rgba_out,
               uint32_t* n_iterations) {
	Net net(*c);
	std::vector<float> P = half_params(net, params);
	AABB bb{{ds->aabb_min[0], ds->aabb_min[1], ds->aabb_min[2]}, {ds->aabb_max[0], ds->aabb_max[1], ds->aabb_max[2]}};
	const float diag[3] = {bb.mx.x - bb.mn.x, bb.mx.y - bb.mn.y, bb.mx.z - bb.mn.z};
	const uint32_t W = cam->width, H = cam->height, N = W * H;
	const float cone = ds->cone_angle;
	std::vector<float> frame(4 * (size_t)N), accum(4 * (size_t)N, 0.f);
	std::vector<OrRay> rays(N);
	for (uint32_t sp = 0; sp < std::max(1u, spp); ++sp) {
		float a0[2], a1[2], off[2];
		or_ld_random_val_2d(0, 0xdeadbeefu, a0);
		or_ld_random_val_2d(snap ? 0 : sp, 0xdeadbeefu, a1);
		for (int k = 0; k < 2; ++k) { const float v = (0.5f - a0[k]) + a1[k]; off[k] = v - std::floor(v); }
		std::fill(frame.begin(), frame.end(), 0.f);
#pragma omp parallel for schedule(dynamic, 256)
		for (int64_t ii = 0; ii < (int64_t)N; ++ii) {
			const uint32_t idx = (uint32_t)ii, x = idx % W, y = idx / W;
			OrRay& r = rays[idx];
			r.idx = idx; r.n_steps = 0; r.rgba[0] = r.rgba[1] = r.rgba[2] = r.rgba[3] = 0.f;
			const float u = ((float)x + off[0]) / (float)W, v = ((float)y + off[1]) / (float)H;
			const float dc[3] = {(u - cam->screen_center[0]) * (float)W / cam->focal[0], (v - cam->screen_center[1]) * (float)H / cam->focal[1], 1.0f};
			float du[3];
			for (int k = 0; k < 3; ++k) du[k] = (cam->xform[4 * k] * dc[0] + cam->xform[4 * k + 1] * dc[1]) + cam->xform[4 * k + 2] * dc[2];
			r.o = {cam->xform[3], cam->xform[7], cam->xform[11]};
			const float nrm = std::sqrt((du[0] * du[0] + du[1] * du[1]) + du[2] * du[2]);
			r.d = nrm > 0.f ? V3{du[0] / nrm, du[1] / nrm, du[2] / nrm} : V3{du[0], du[1], du[2]};
			if (ds->motion_on) {  // testbed_nerf.cu:2285-2294
				float o3[3] = {r.o.x, r.o.y, r.o.z}, d3[3] = {r.d.x, r.d.y, r.d.z};
				move_ray(ds, o3, d3);
				r.o = {o3[0], o3[1], o3[2]}; r.d = {d3[0], d3[1], d3[2]};
			}
			float tmin, tmax; ray_intersect(bb, r.o, r.d, tmin, tmax);
			float t = std::fmax(tmin, 0.2f) + 1e-6f;  // NERF_RENDERING_NEAR_DISTANCE
			r.alive = aabb_contains(bb, V3{r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z});
			if (r.alive) {  // advance_pos_nerf
				const V3 idir = {1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
				t += or_ld_random_val(sp, idx * 786433u) * calc_dt(t, cone);
				while (true) {
					const V3 pos = {r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z};
					if (!aabb_contains(bb, pos)) { r.alive = false; break; }
					const float dt = calc_dt(t, cone);
					const uint32_t mip = (uint32_t)mip_from_dt(dt, pos);
					if (density_grid_occupied_at(pos, bitfield, mip)) break;
					t = advance_to_next_voxel(t, cone, pos, r.d, idir, NERF_GRIDSIZE >> mip);
				}
			}
			r.t = t;
		}
		std::vector<uint32_t> alive;
		for (uint32_t i = 0; i < N; ++i) if (rays[i].alive) alive.push_back(i);
		uint32_t iters = 0;
		for (uint32_t it = 1; it < 10000;) {  // MARCH_ITER
			std::vector<uint32_t> next;
			for (uint32_t id : alive) if (rays[id].alive) next.push_back(id);
			alive.swap(next);
			const uint32_t n_alive = (uint32_t)alive.size();
			if (n_alive == 0) break;
			const uint32_t n_steps = std::min(8u, std::max(1u, N / n_alive));
#pragma omp parallel for schedule(dynamic, 64)
			for (int64_t q = 0; q < (int64_t)n_alive; ++q) {
				OrRay& r = rays[alive[q]];
				const V3 idir = {1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
				const float wd[3] = {(r.d.x + 1.0f) * 0.5f, (r.d.y + 1.0f) * 0.5f, (r.d.z + 1.0f) * 0.5f};
				// generate_next_nerf_network_inputs
				float coords[8][7];
				uint32_t j = 0;
				float t = r.t;
				bool exited = false;
				for (; j < n_steps; ++j) {
					V3 pos; float dt;
					while (true) {
						pos = {r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z};
						if (!aabb_contains(bb, pos)) { exited = true; break; }
						dt = calc_dt(t, cone);
						const uint32_t mip = (uint32_t)mip_from_dt(dt, pos);
						if (density_grid_occupied_at(pos, bitfield, mip)) break;
						t = advance_to_next_voxel(t, cone, pos, r.d, idir, NERF_GRIDSIZE >> mip);
					}
					if (exited) break;
					float* cc = coords[j];
					cc[0] = (pos.x - bb.mn.x) / diag[0]; cc[1] = (pos.y - bb.mn.y) / diag[1]; cc[2] = (pos.z - bb.mn.z) / diag[2];
					cc[3] = warp_dt(dt); cc[4] = wd[0]; cc[5] = wd[1]; cc[6] = wd[2];
					t += dt;
				}
				r.n_steps = j;
				if (!exited) r.t = t;
				// inference + composite_kernel_nerf
				uint32_t k = 0;
				for (; k < r.n_steps; ++k) {
					uint16_t lo[16]; Ctx cx;
					net_forward_one(net, P.data(), coords[k], valid_level, cx, lo);
					const float T = 1.f - r.rgba[3];
					const float dt = unwarp_dt(coords[k][3]);
					float u3[3]; for (int e = 0; e < 3; ++e) u3[e] = h2f(lo[8 + e]) * 2.0f - 1.0f;
					const float nr = std::sqrt((u3[0] * u3[0] + u3[1] * u3[1]) + u3[2] * u3[2]);
					float dir[3]; for (int e = 0; e < 3; ++e) dir[e] = nr > 0 ? u3[e] / nr : u3[e];
					const float inv_s = det_expf(rh(10.0f * h2f(lo[7])));
					const float sdf = h2f(lo[3]);
					const float pg[3] = {h2f(lo[4]), h2f(lo[5]), h2f(lo[6])};
					const float true_cos = dir[0] * pg[0] + dir[1] * pg[1] + dir[2] * pg[2];
					float b1 = (float)(-true_cos * 0.5 + 0.5); b1 = b1 > 0.0f ? b1 : 0.0f;
					float b2 = -true_cos; b2 = b2 > 0.0f ? b2 : 0.0f;
					const float iter_cos = -(b1 * (1.0 - cos_anneal) + b2 * cos_anneal);
					const float next_sdf = sdf + iter_cos * dt * 0.5;
					const float prev_sdf = sdf - iter_cos * dt * 0.5;
					const float next_cdf = det_logistic(next_sdf * inv_s), prev_cdf = det_logistic(prev_sdf * inv_s);
					const float p = prev_cdf - next_cdf, cc = prev_cdf;
					const float alpha = clampf((p + 1e-5f) / (cc + 1e-5f), 0.0f, 1.0f);
					const float weight = alpha * T;
					for (int e = 0; e < 3; ++e) r.rgba[e] += det_logistic(h2f(lo[e])) * weight;
					r.rgba[3] += weight;
					if (r.rgba[3] > (1.0f - min_transmittance)) {
						const float w = r.rgba[3];
						for (int e = 0; e < 4; ++e) r.rgba[e] /= w;
						break;
					}
				}
				if (k < n_steps) {
					r.alive = false;
					if (r.rgba[3] > 0.001f) {
						float* f = &frame[4 * (size_t)r.idx];
						for (int e = 0; e < 3; ++e) f[e] = srgb_to_linear(r.rgba[e]);
						f[3] = r.rgba[3];
					}
				}
			}
			it += n_steps;
			++iters;
		}
		if (n_iterations) *n_iterations = iters;
		const float s = (float)sp;
		for (size_t i = 0; i < 4 * (size_t)N; ++i) accum[i] = (accum[i] * s + frame[i]) / (s + 1);
	}
	std::memcpy(rgba_out, accum.data(), accum.size() * sizeof(float));
}

// -------------------------------------------------------------------------------------------
// Marching cubes (marching_cubes.cu:276-420, gen_vertices / gen_faces) in the canonical deterministic
// order: vertices by (grid point linear index, axis x < y < z), triangles by (cube linear index, table
// row order). Vertex = fma(float(x) + dt, scale, aabb.min) per component (Eigen cwiseProduct + offset
// under nvcc --fmad=true), dt = (thresh - f0) / (f1 - f0), scale = (max - min) / res. The case table is
// passed in (oracle/mc_table.py builds it independently of the product). Call with null outputs to
// count. Returns n_verts; *n_tris_out = triangles.
// -------------------------------------------------------------------------------------------
uint64_t or_marching_cubes(const float* d, uint32_t rx, uint32_t ry, uint32_t rz, float thresh, const float* amin, const float* amax,
                           const int8_t* table /* 256 x 19 */, float* V, uint32_t* F, uint64_t* n_tris_out) {
	const uint64_t r1 = rx, r2 = (uint64_t)rx * ry, n = r2 * rz;
	float scale[3] = {(amax[0] - amin[0]) / (float)rx, (amax[1] - amin[1]) / (float)ry, (amax[2] - amin[2]) / (float)rz};
	auto flags = [&](uint64_t p) {
		const uint32_t z = (uint32_t)(p / r2), y = (uint32_t)((p % r2) / r1), x = (uint32_t)(p % r1);
		const bool in0 = d[p] > thresh;
		uint32_t f = 0;
		if (x + 1 < rx && in0 != (d[p + 1] > thresh)) f |= 1;
		if (y + 1 < ry && in0 != (d[p + r1] > thresh)) f |= 2;
		if (z + 1 < rz && in0 != (d[p + r2] > thresh)) f |= 4;
		return f;
	};
	std::vector<uint32_t> vbase(n);
	uint64_t nv = 0;
	for (uint64_t p = 0; p < n; ++p) {
		vbase[p] = (uint32_t)nv;
		const uint32_t f = flags(p);
		if (!f) continue;
		const uint32_t z = (uint32_t)(p / r2), y = (uint32_t)((p % r2) / r1), x = (uint32_t)(p % r1);
		const uint64_t step[3] = {1, r1, r2};
		for (int a = 0; a < 3; ++a) {
			if (!((f >> a) & 1)) continue;
			if (V) {
				const float f0 = d[p], f1 = d[p + step[a]];
				const float dt = (thresh - f0) / (f1 - f0);
				float q[3] = {(float)x, (float)y, (float)z};
				q[a] = q[a] + dt;
				for (int k = 0; k < 3; ++k) V[3 * nv + k] = std::fma(q[k], scale[k], amin[k]);
			}
			++nv;
		}
	}
	const uint64_t eoff[12] = {0, 1, r1, 0, r2, 1 + r2, r1 + r2, r2, 0, 1, 1 + r1, r1};
	const int eax[12] = {0, 1, 0, 1, 0, 1, 0, 1, 2, 2, 2, 2};
	uint64_t nt = 0;
	for (uint64_t p = 0; p < n; ++p) {
		const uint32_t z = (uint32_t)(p / r2), y = (uint32_t)((p % r2) / r1), x = (uint32_t)(p % r1);
		if (x + 1 >= rx || y + 1 >= ry || z + 1 >= rz) continue;
		uint32_t m = 0;
		const uint64_t c[8] = {p, p + 1, p + 1 + r1, p + r1, p + r2, p + 1 + r2, p + 1 + r1 + r2, p + r1 + r2};
		for (int k = 0; k < 8; ++k) m |= (uint32_t)(d[c[k]] > thresh) << k;
		const int8_t* row = table + 19 * m;
		for (int q = 0; q < 18 && row[q] >= 0; q += 3) {
			if (F)
				for (int j = 0; j < 3; ++j) {
					const int e = row[q + j];
					const uint64_t o = p + eoff[e];
					F[3 * nt + j] = vbase[o] + (uint32_t)__builtin_popcount(flags(o) & ((1u << eax[e]) - 1));
				}
			++nt;
		}
	}
	if (n_tris_out) *n_tris_out = nt;
	return nv;
}

// ---------------------------------------------------------------- training-image preparation (ngp::load_nerf)
// nerf_loader.cu:550-569 (alpha image: red channel through srgb_to_linear, common_device.cuh:31-37, truncated to
// uint8), :571-590 (dynamic mask: mask red != 0 -> 0x00FF00FF), then convert_rgba32 (:59-81) as set_training_image
// applies it: white / black rgb -> alpha 0, the mask colour re-keyed to hot pink.
static float or_srgb_to_linear(float srgb) { return srgb <= 0.04045f ? srgb / 12.92f : std::pow((srgb + 0.055f) / 1.055f, 2.4f); }
uint32_t or_prepare_image_rgba8(uint8_t* img, uint32_t w, uint32_t h, const uint8_t* alpha_img, const uint8_t* mask_img, int white_transparent,
                                int black_transparent) {
	const uint64_t n = (uint64_t)w * h;
	if (alpha_img)
		for (uint64_t i = 0; i < n; ++i) img[i * 4 + 3] = uint8_t(255.0f * or_srgb_to_linear(alpha_img[i * 4] * (1.f / 255.f)));
	uint32_t mask_color = 0;
	if (mask_img) {
		mask_color = 0x00FF00FF;
		for (uint64_t i = 0; i < n; ++i)
			if (mask_img[i * 4] != 0) std::memcpy(img + i * 4, &mask_color, 4);
	}
	for (uint64_t i = 0; i < n; ++i) {
		uint8_t rgba[4];
		std::memcpy(rgba, img + i * 4, 4);
		if (white_transparent && rgba[0] == 255 && rgba[1] == 255 && rgba[2] == 255) rgba[3] = 0;
		if (black_transparent && rgba[0] == 0 && rgba[1] == 0 && rgba[2] == 0) rgba[3] = 0;
		uint32_t v;
		std::memcpy(&v, rgba, 4);
		if (mask_color != 0 && mask_color == v) { rgba[0] = 0xFF; rgba[1] = 0x00; rgba[2] = 0xFF; rgba[3] = 0x00; }
		std::memcpy(img + i * 4, rgba, 4);
	}
	return mask_color;
}
} // extern "C"
