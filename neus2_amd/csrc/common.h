// Shared device/host helpers for the gfx950 NeuS2 hot path.
// Reference semantics cited per function; layouts documented in DESIGN.md §Data layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#define NEUS_HD __host__ __device__ __forceinline__

typedef _Float16 half_t;
typedef half_t h8 __attribute__((ext_vector_type(8)));
typedef half_t h4 __attribute__((ext_vector_type(4)));
typedef half_t h2 __attribute__((ext_vector_type(2)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));
// 4 B-aligned float vectors for the 28 B NerfCoordinate records (the hardware runs unaligned mode)
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));

namespace neus {

// ----------------------------------------------------------- constants (testbed_nerf.cu:57-81)
constexpr uint32_t NERF_GRIDSIZE = 128;
constexpr uint32_t NERF_STEPS = 1024;
constexpr uint32_t NERF_CASCADES = 8;
constexpr float SQRT3 = 1.73205080757f;
constexpr float STEPSIZE = SQRT3 / NERF_STEPS;
constexpr float MIN_CONE_STEPSIZE = STEPSIZE;
constexpr float MAX_CONE_STEPSIZE = STEPSIZE * (1 << (NERF_CASCADES - 1)) * NERF_STEPS / NERF_GRIDSIZE;
constexpr uint32_t N_MAX_RANDOM_SAMPLES_PER_RAY = 8;
constexpr float NERF_MIN_OPTICAL_THICKNESS = 0.1f;
constexpr uint32_t GRID3 = NERF_GRIDSIZE * NERF_GRIDSIZE * NERF_GRIDSIZE;
// Linear mip-0 occupancy for the constant-step march: GRID3 / 32 words in (x, y, z/32) order.
constexpr uint32_t LIN_WORDS = GRID3 / 32;
constexpr uint32_t MAX_LEVELS = 16;
constexpr uint32_t OUT_W = 16;      // padded network output width (nerf_network.h:935)
constexpr uint32_t COORD_W = 7;     // NerfCoordinate floats (nerf.h:76-102)

// ----------------------------------------------------------- pcg32 (my_tcnn pcg32.h:43-170)
struct pcg32 {
	uint64_t state, inc;
	NEUS_HD pcg32() : state(0x853c49e6748fea9bULL), inc(0xda3e39cb94b95bdbULL) {}
	NEUS_HD pcg32(uint64_t s, uint64_t i) : state(s), inc(i) {}
	NEUS_HD uint32_t next_uint() {
		uint64_t oldstate = state;
		state = oldstate * 0x5851f42d4c957f2dULL + inc;
		uint32_t xorshifted = (uint32_t)(((oldstate >> 18u) ^ oldstate) >> 27u);
		uint32_t rot = (uint32_t)(oldstate >> 59u);
		return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
	}
	NEUS_HD float next_float() {
		union { uint32_t u; float f; } x;
		x.u = (next_uint() >> 9) | 0x3f800000u;
		return x.f - 1.0f;
	}
	NEUS_HD void advance(int64_t delta_ = (1ll << 32)) {
		uint64_t cur_mult = 0x5851f42d4c957f2dULL, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
		uint64_t delta = (uint64_t)delta_;
		while (delta > 0) {
			if (delta & 1) { acc_mult *= cur_mult; acc_plus = acc_plus * cur_mult + cur_plus; }
			cur_plus = (cur_mult + 1) * cur_plus; cur_mult *= cur_mult; delta /= 2;
		}
		state = acc_mult * state + acc_plus;
	}
};
// Jump-ahead table of one pcg32 stream (increment `inc`): t[j][k] = the affine map of advance(k << 12 j), j < 3,
// k < 4096. advance(d) for d < 2^36 is then three table lookups and three 64-bit multiply-adds instead of
// ~log2(d) squaring steps (the LCG's jumps compose exactly, so the state is bit-identical).
struct PcgJump { unsigned long long mult, plus; };
struct PcgJumpTable { const PcgJump* t; uint64_t inc; };  // t: 3 x 4096 entries
constexpr uint32_t PCG_JUMP_BITS = 12, PCG_JUMP_N = 1u << PCG_JUMP_BITS, PCG_JUMP_LEVELS = 3;
NEUS_HD PcgJump pcg_jump(uint64_t inc, uint64_t delta) {
	uint64_t cur_mult = 0x5851f42d4c957f2dULL, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
	while (delta > 0) {
		if (delta & 1) { acc_mult *= cur_mult; acc_plus = acc_plus * cur_mult + cur_plus; }
		cur_plus = (cur_mult + 1) * cur_plus; cur_mult *= cur_mult; delta /= 2;
	}
	return PcgJump{acc_mult, acc_plus};
}
NEUS_HD void pcg_advance(pcg32& r, uint64_t delta, const PcgJumpTable& jt) {
	if (jt.t && r.inc == jt.inc && delta < (1ull << (PCG_JUMP_LEVELS * PCG_JUMP_BITS))) {
#pragma unroll
		for (uint32_t j = 0; j < PCG_JUMP_LEVELS; ++j) {
			const PcgJump a = jt.t[j * PCG_JUMP_N + ((delta >> (j * PCG_JUMP_BITS)) & (PCG_JUMP_N - 1))];
			r.state = a.mult * r.state + a.plus;
		}
	} else {
		r.advance((int64_t)delta);
	}
}

inline pcg32 make_pcg32(uint64_t initstate, uint64_t initseq = 1u) {
	pcg32 r; r.state = 0U; r.inc = (initseq << 1u) | 1u; r.next_uint(); r.state += initstate; r.next_uint(); return r;
}

// ----------------------------------------------------------- half helpers
NEUS_HD float rh(float f) { return (float)(half_t)f; }

// fixed-operation-order expf, identical on CPU oracle and GPU (no contraction in callers)
NEUS_HD float det_expf(float x) {
#pragma clang fp contract(off)  // the same bits in every translation unit, whatever its contraction flags
	if (!(x < 88.5f)) return x != x ? x : __builtin_huge_valf();
	if (x < -103.0f) return 0.0f;
	float kf = rintf(x * 1.44269504088896341f);
	float r = x - kf * 0.693145751953125f;
	r = r - kf * 1.42860676533018672e-06f;
	float p = 1.3888889225e-3f;
	p = p * r + 8.3333337680e-3f;
	p = p * r + 4.1666667908e-2f;
	p = p * r + 1.6666667163e-1f;
	p = p * r + 0.5f;
	p = p * r + 1.0f;
	p = p * r + 1.0f;
	return ldexpf(p, (int)kf);
}
NEUS_HD float det_logistic(float x) {
#pragma clang fp contract(off)
	return 1.0f / (1.0f + det_expf(-x));
}

// ----------------------------------------------------------- morton (my_tcnn common_device.h:335-365)
NEUS_HD uint32_t expand_bits(uint32_t v) {
	v = (v * 0x00010001u) & 0xFF0000FFu; v = (v * 0x00000101u) & 0x0F00F00Fu;
	v = (v * 0x00000011u) & 0xC30C30C3u; v = (v * 0x00000005u) & 0x49249249u; return v;
}
NEUS_HD uint32_t morton3D(uint32_t x, uint32_t y, uint32_t z) { return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2); }
NEUS_HD uint32_t morton3D_invert(uint32_t x) {
	x = x & 0x49249249; x = (x | (x >> 2)) & 0xc30c30c3; x = (x | (x >> 4)) & 0x0f00f00f;
	x = (x | (x >> 8)) & 0xff0000ff; x = (x | (x >> 16)) & 0x0000ffff; return x;
}

// ----------------------------------------------------------- hash grid addressing (grid.h:118-153)
struct GridLevels {
	uint32_t n_levels;
	uint32_t offset[MAX_LEVELS + 1];   // in entries (x2 features)
	uint32_t res[MAX_LEVELS];
	float scale[MAX_LEVELS];
	uint32_t dense_bits;               // bit l: level l is dense (res^3 <= entries), else hashed with 2^k entries
};
NEUS_HD uint32_t grid_index(uint32_t hashmap_size, uint32_t resolution, uint32_t x, uint32_t y, uint32_t z) {
	uint32_t stride = 1, index = 0;
	index += x * stride; stride *= resolution;
	if (stride <= hashmap_size) { index += y * stride; stride *= resolution; }
	if (stride <= hashmap_size) { index += z * stride; stride *= resolution; }
	if (hashmap_size < stride) index = x ^ (y * 2654435761u) ^ (z * 805459861u);
	return index % hashmap_size;
}

// Device-resident per-step counters: the host never syncs inside a training step.
struct StepState {
	uint32_t rays_per_batch;          // R (adapted on device, testbed_nerf.cu:3399-3438)
	uint32_t max_inference;           // next_multiple(min(Npre_prev, max_samples), 128)
	uint32_t measured_before;         // Npre requested counter of the last step (per rank)
	uint32_t numsteps_counter;        // this step: requested samples (all rays)
	uint32_t n_kept;                  // this step: samples actually written
	uint32_t compacted_counter;       // this step: requested compacted samples
	uint32_t measured_batch_size;     // compacted counter of the last step (per rank)
	uint32_t n_rays_with_samples;
	uint32_t zero_records;
	uint32_t n_rays_total;            // rays drawn since training step 0 (all ranks)
	uint32_t n_train;                 // compacted training batch (target) or 0 when no samples
	uint32_t march_est;               // ray slots the first march pass covers (0 = all); from the last step's kept extent
	unsigned long long trained_total; // real (non-rollover) training samples since step 0, this rank: sum of min(Nc measured, batch)
	uint32_t march_total;             // samples requested by the first march pass's rays
	uint32_t kept_extent;             // this step: 1 + the last kept ray slot (0 if none)
	// work counters since step 0 (this rank), for the whole-step roofline (bench.py roofline_step)
	unsigned long long pre_total;     // pre-compaction samples evaluated: sum of n_kept
	unsigned long long rays_total;    // rays marched: sum of rays_per_batch
	unsigned long long eval_total;    // samples the pre-compaction network pass evaluated (progressive rounds: their lists)
	uint32_t fail_flags;              // device health: STEP_FAIL_* bits (sticky; the host raises on the next readback)
	uint32_t eval_last;               // samples evaluated by the last step's pre-compaction pass
	unsigned long long prog_steps;    // steps that ran progressive (multi-round) inference
	// the step's compacted count and rays with samples summed over the ranks (k_loss_ray writes this rank's; the data-
	// parallel exchange all-reduces the pair right after the loss, so compacted_counter stays this rank's training batch
	// for the backward while the counters update and the next step's sampling can start before the backward ends)
	uint32_t compacted_global;
	uint32_t rays_ws_global;
	// the march cut (testbed.cpp march_cut_for): cut_abort - this step's training is not provably the full
	// march's (k_loss_grad copies it from the loss's abort word; all-reduced with the two counters above, so every rank
	// sees the same); while set, the optimizer and the step counters leave every state untouched and the host re-runs the
	// step with the full march. march_cut - this step's march covered only the slots below the cut estimate. mi_lb - a lower
	// bound of the reference's cap on this step's pre-compaction samples, max_inference = next_multiple(min(the last step's
	// requested count, max_samples)), when the last step's march was cut (its requested count is then known only for the
	// marched slots; max_inference is max_samples then, an upper bound); 0 when max_inference is exact.
	uint32_t cut_abort;
	uint32_t march_cut;
	uint32_t mi_lb;
	uint32_t pad32_;
};
static_assert(sizeof(StepState) == 128, "StepState is one 128-B record");
// fail_flags bits: a march step saw a non-finite or negative t (step_until's precondition; the ray is ended there);
// a look-back scan gave up waiting (set by the host from the scan state's counter)
constexpr uint32_t STEP_FAIL_MARCH_T = 1u, STEP_FAIL_SCAN = 2u;

// Counters::update_after_training (testbed_nerf.cu:3399-3438) at the end of a step: one thread (k_step_counters, or
// the Adam launch's block 0). eval_cnt: the progressive rounds' list lengths (n_eval of them; null: one pass over the
// kept samples)
__device__ __forceinline__ void step_counters_update(StepState* st, uint32_t target_batch, uint32_t max_samples, uint32_t world, uint32_t fixed_rays,
                                                     const uint32_t* eval_cnt = nullptr, uint32_t n_eval = 0) {
	if (st->cut_abort) return;  // the step is re-run with the full march (the march cut): no counter moves
	const uint32_t R = st->rays_per_batch;
	const bool mc = st->march_cut != 0;
	st->n_rays_total += R * world;  // n_rays_total
	st->pre_total += st->n_kept;
	st->rays_total += R;
	uint32_t ev = st->n_kept;
	if (eval_cnt) {
		ev = 0;
		for (uint32_t k = 0; k < n_eval; ++k) ev += eval_cnt[k];
		++st->prog_steps;
	}
	st->eval_last = ev;
	st->eval_total += ev;
	// next step's first march pass: the slots up to this step's kept extent plus a margin (all slots when every
	// ray with samples fitted under this step's cap)
	// (a cut march's kept extent is that of its marched slots: the estimate stays the last full march's)
	const bool fit = st->numsteps_counter <= st->max_inference;
	const uint32_t ext = st->kept_extent + st->kept_extent / 4 + 1024;
	if (!mc) st->march_est = fit ? 0u : (ext + 63u) / 64u * 64u;
	// per rank: the cap on the next step's pre-compaction samples follows this rank's own request count
	const uint32_t before = st->numsteps_counter;
	const uint32_t measured = st->compacted_global / world;
	st->measured_before = before;
	st->measured_batch_size = measured;
	st->trained_total += min(measured, target_batch);  // real training samples (the rest of the batch is rollover)
	if (before == 0 || measured == 0) { st->zero_records = 1; st->mi_lb = 0; return; }
	st->zero_records = 0;
	uint32_t mi = min(before, max_samples);
	st->max_inference = (mi + 127u) / 128u * 128u;
	// a cut march requested past max_samples (its drop marker), so max_inference is max_samples; the reference's is at
	// least the marched slots' count, rounded the same way
	st->mi_lb = mc ? max((min(st->march_total, max_samples) + 127u) / 128u * 128u, 1u) : 0u;
	if (fixed_rays) { st->rays_per_batch = fixed_rays; return; }
	uint32_t r = (uint32_t)((float)R * (float)target_batch / (float)measured);
	r = (r + 127u) / 128u * 128u;
	st->rays_per_batch = min(r, 1u << 18);
}

// ---------------------------------------------------------------- wave64 cross-lane steps on DPP (gfx9 family)
// Lane moves through the VALU's data-parallel-primitive operand modifier instead of ds_bpermute (an LDS-pipe op
// with LDS latency per step of a scan chain). wave_shr:1 / wave_shl:1 shift across the whole wave; row_shr:n
// within rows of 16 lanes; row_bcast:15 / :31 hand a row's last lane to the next row / to rows 2 and 3 (the wave64
// scan pattern). A lane whose source is out of range, or whose row is masked off, keeps `old`. Every lane of the
// wave must be active.
constexpr int DPP_ROW_SHR = 0x110, DPP_WAVE_SHL1 = 0x130, DPP_WAVE_SHR1 = 0x138, DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143;
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t x) {
	return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f32(float old, float x) {
	return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, x), CTRL, ROW_MASK, 0xf, false));
}
// inclusive prefix sum over the wave's 64 lanes (u32, exact)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
	x += dpp_u32<DPP_ROW_SHR + 1>(0u, x);
	x += dpp_u32<DPP_ROW_SHR + 2>(0u, x);
	x += dpp_u32<DPP_ROW_SHR + 4>(0u, x);
	x += dpp_u32<DPP_ROW_SHR + 8>(0u, x);
	x += dpp_u32<DPP_BCAST15, 0xa>(0u, x);
	x += dpp_u32<DPP_BCAST31, 0xc>(0u, x);
	return x;
}
__device__ __forceinline__ uint32_t wave_lane_value(uint32_t x, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)x, lane); }
// wave-wide sum / max (u32), the same value on every lane
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) { return wave_lane_value(wave_incl_sum(x), 63); }
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
	x = max(x, dpp_u32<DPP_ROW_SHR + 1>(0u, x));
	x = max(x, dpp_u32<DPP_ROW_SHR + 2>(0u, x));
	x = max(x, dpp_u32<DPP_ROW_SHR + 4>(0u, x));
	x = max(x, dpp_u32<DPP_ROW_SHR + 8>(0u, x));
	x = max(x, dpp_u32<DPP_BCAST15, 0xa>(0u, x));
	x = max(x, dpp_u32<DPP_BCAST31, 0xc>(0u, x));
	return wave_lane_value(x, 63);
}

} // namespace neus
