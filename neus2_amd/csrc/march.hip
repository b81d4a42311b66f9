// NeuS ray sampling, SDF-to-alpha compositing, loss and deterministic compaction on gfx950.
//
//   k_ray_gen / k_march / k_march_write : generate_training_samples_nerf_with_global_movement
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
#include "march_common.h"
#include "scan_lookback.h"
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace neus {



// ---------------------------------------------------------------- the occupancy march
// Mip-0 occupancy as 32-bit words in (x, y, z/32) order: one address computation and one word load per
// step instead of the Morton interleave of the reference's bitfield (built from it, same bits).
__global__ void k_bitfield_linear(const uint8_t* __restrict__ bf, uint32_t* __restrict__ lin) {
	const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
	if (w >= GRID3 / 32) return;
	const uint32_t ix = w >> 9, iy = (w >> 2) & 127, iz0 = (w & 3) * 32;
	uint32_t word = 0;
	for (uint32_t b = 0; b < 32; ++b) {
		const uint32_t idx = morton3D(ix, iy, iz0 + b);
		word |= (uint32_t)((bf[idx / 8] >> (idx % 8)) & 1) << b;
	}
	lin[w] = word;
}
// Conservative slab test of the ray o + t d, t >= 0, against the box bb = {min xyz, max xyz} (touching counts as a hit).
__device__ __forceinline__ bool ray_hits_box(const float o[3], const float d[3], const float bb[6]) {
	float tn = 0.0f, tf = 3.402823466e+38f;
#pragma unroll
	for (int k = 0; k < 3; ++k) {
		if (fabsf(d[k]) < 1e-20f) {
			if (o[k] < bb[k] || o[k] > bb[3 + k]) return false;
			continue;
		}
		const float inv = 1.0f / d[k];
		float a = (bb[k] - o[k]) * inv, b = (bb[3 + k] - o[k]) * inv;
		if (a > b) { const float t = a; a = b; b = t; }
		tn = fmaxf(tn, a); tf = fminf(tf, b);
	}
	return tn <= tf;
}
// ---------------------------------------------------------------- pass 0: ray generation
// Thread per ray slot: pixel/image pick from the ray's pcg32 stream, pinhole ray, AABB entry and
// jittered start (testbed_nerf.cu:1263-1375). rays: 6 floats (o, unnormalised d); tstart: the jittered
// start t, or -1 for a dropped ray and for slots >= R (nothing to march).
__global__ void __launch_bounds__(256) k_ray_gen(uint32_t cap_rays, const StepState* __restrict__ st_r, DPInfo dp, DevDataset ds,
                                                 uint64_t rng_state, uint64_t rng_inc, float* __restrict__ rays, float* __restrict__ tstart,
                                                 uint32_t* __restrict__ march_queue, StepState* __restrict__ st_w, PcgJumpTable jt,
                                                 uint32_t* __restrict__ zero_counters, uint32_t n_zero, const float* __restrict__ occ_bbox,
                                                 const uint32_t* __restrict__ est_cut, uint32_t est_div, uint32_t* __restrict__ nreq,
                                                 uint32_t* __restrict__ nrec, uint32_t max_samples) {
	if (blockIdx.x == 0 && threadIdx.x < n_zero) zero_counters[threadIdx.x] = 0u;  // the progressive rounds' list lengths
	// the march cut (MarchWork::est_cut): the same test as k_march_bal's; the slots past the estimate are not marched, so
	// they get no ray
	const uint32_t est0 = st_r->march_est ? min(st_r->march_est, cap_rays) : cap_rays;
	const uint32_t ec = est_cut ? *est_cut / est_div : 0u;
	const bool mcut = est_cut && ec < est0;
	const uint32_t lim = mcut ? ec : cap_rays;
	float bb[6] = {-3.402823466e+38f, -3.402823466e+38f, -3.402823466e+38f, 3.402823466e+38f, 3.402823466e+38f, 3.402823466e+38f};
	if (occ_bbox)
#pragma unroll
		for (int k = 0; k < 6; ++k) bb[k] = occ_bbox[k];
	if (blockIdx.x == 0 && threadIdx.x == 0) {  // the march passes' ray queues and counters (next kernels on the stream)
		march_queue[0] = 0; march_queue[1] = 0;
		st_w->march_total = 0; st_w->kept_extent = 0;
		st_w->n_kept = 0; st_w->n_rays_with_samples = 0;  // this step's march maxima / counts (k_march, k_march_write)
		st_w->march_cut = mcut ? 1u : 0u;
	}
	const uint32_t R = st_r->rays_per_batch;
	const uint32_t n_rays_global = R * dp.world, n_rays_total = st_r->n_rays_total;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap_rays; i += gridDim.x * blockDim.x) {
		if (i >= lim) {
			// a cut march's dropped slots (k_march_bal's pass 1 leaves them): the first requests past the cap, the rest
			// nothing; no ray
			nreq[i] = i == lim ? max_samples + 1u : 0u;
			nrec[i] = 0u;
			continue;
		}
		float o[3] = {0, 0, 0}, du[3] = {0, 0, 0}, startt = -1.0f;
		if (i < R) {
			const uint32_t ig = dp.rank * R + i;
			pcg32 rng(rng_state, rng_inc);
			const uint32_t img = image_idx(ig, n_rays_global, n_rays_total, ds.n_images);
			const int rx = ds.res[2 * img], ry = ds.res[2 * img + 1];
			pcg_advance(rng, (uint64_t)(uint32_t)(ig * N_MAX_RANDOM_SAMPLES_PER_RAY), jt);
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
				if (ds.motion.on) {
					// global_movement_with_rotation_6d (testbed_nerf.cu:1380-1387): o' = R o + t, d' = R d; the
					// record then holds the moved unit direction (load_march_ray does not renormalise it)
					const float* M = ds.motion.R;
					float mo[3], md[3];
#pragma unroll
					for (int r = 0; r < 3; ++r) {
						mo[r] = ((M[3 * r] * o[0] + M[3 * r + 1] * o[1]) + M[3 * r + 2] * o[2]) + ds.motion.t[r];
						md[r] = (M[3 * r] * dir[0] + M[3 * r + 1] * dir[1]) + M[3 * r + 2] * dir[2];
					}
#pragma unroll
					for (int r = 0; r < 3; ++r) { o[r] = mo[r]; dir[r] = md[r]; du[r] = md[r]; }
				}
				float tmin; ray_intersect(ds, o, dir, tmin);
				tmin = fmaxf(tmin, 0.0f);
				startt = tmin;
				startt += calc_dt(startt, ds.cone_angle) * rng.next_float();
				// a ray (t >= 0) that misses the occupied cells' padded box samples nothing: not marched
				if (occ_bbox && !ray_hits_box(o, dir, bb)) startt = -1.0f;
			}
		}
		float* rr = rays + 6 * (size_t)i;
		rr[0] = o[0]; rr[1] = o[1]; rr[2] = o[2]; rr[3] = du[0]; rr[4] = du[1]; rr[5] = du[2];
		tstart[i] = startt;
	}
}

// unit: the record holds a unit direction already (moved rays of a dynamic scene)
__device__ __forceinline__ void load_march_ray(const float* __restrict__ rays, uint32_t i, MarchRay& mr, bool unit) {
	const float* rr = rays + 6 * (size_t)i;
	const float du[3] = {rr[3], rr[4], rr[5]};
	const float nrm = sqrtf((du[0] * du[0] + du[1] * du[1]) + du[2] * du[2]);
#pragma unroll
	for (int d = 0; d < 3; ++d) {
		mr.o[d] = rr[d];
		mr.dir[d] = unit ? du[d] : (nrm > 0.f ? du[d] / nrm : du[d]);
		mr.idir[d] = 1.0f / mr.dir[d];
	}
}

// ---------------------------------------------------------------- pass 1: the march (count + sample runs)
// The reference marches every ray twice inside one thread (count, then write after an atomicAdd). Here the march
// runs once and records, per ray, runs of consecutive samples {t of the first sample, count} (MarchWork); the
// write pass rebuilds each sample's t by replaying the run's t += dt, the same float additions.
// Work distribution: a ray's step sequence is split over several lanes (8 per ray, or k_march_bal's 1-16 by length),
// which join in segment order (below), so a wave does not wait on one lane walking its longest ray alone.
// FAST (cone_angle 0, constant dt): inside an occupied interior cell every further step is a sample for as long
// as the cell index stays the same (same occupancy bit, inside the AABB, mip 0), so the run continues on the
// position and cell index alone (no bitfield read, no store per sample). Cells with an index 0 / 127 (a position
// on an AABB face takes mip 1) and the centre cell (max|p - 0.5| = 0 takes mip 1) go through march_step.
// One march event of a lane's ray segment: a sample run within a cell (FAST) or one march_step. k is the index of
// t in the ray's step sequence (t0 and its successive t += dt); the event stops at the segment end k_end (the first
// step at or past it is the next segment's). Returns false once the ray is finished (left the AABB).
// Sample runs go to `rec` as {t of the first sample, k_first << 8 | length} (segment-local records).
struct SegAcc { float t0; uint32_t k0, len, nrec, n; };
// dbg: MarchWork::dbg (development timing experiments; 0 in production)
__device__ __forceinline__ void seg_flush(uint2* __restrict__ rec, SegAcc& a, uint32_t dbg = 0) {
	if (a.len) {
		if (!(dbg & 1u)) rec[a.nrec] = make_uint2(__float_as_uint(a.t0), (a.k0 << 8) | a.len);
		++a.nrec; a.len = 0;
	}
}
__device__ __forceinline__ void seg_add(uint2* __restrict__ rec, SegAcc& a, float t, uint32_t k, uint32_t dbg = 0) {
	if (a.len == MARCH_RUN_MAX) seg_flush(rec, a, dbg);
	if (a.len == 0) { a.t0 = t; a.k0 = k; }
	++a.len; ++a.n;
}
__device__ __forceinline__ void mip0_cell(const float pos[3], int c[3]) {  // cascaded_grid_idx_at, mip 0 (march_step)
#pragma unroll
	for (int d = 0; d < 3; ++d) c[d] = clampi((int)(((pos[d] - 0.5f) + 0.5f) * NERF_GRIDSIZE), 0, NERF_GRIDSIZE - 1);
}
// the visited steps k0 .. k0 + 63 of a segment as bits (where the true trajectory may join it; a join further on
// is not seen and re-marches, which costs time, never a result). One event marks [kb, ke): a few instructions on
// both paths of the event where the first-events list it replaces took ~40 (a select chain under a branch).
struct Visits { unsigned long long m; uint32_t k0; };
__device__ __forceinline__ void visit(Visits& v, uint32_t kb, uint32_t ke) {
	const uint32_t a = kb - v.k0, n = ke - kb;   // kb >= k0, n >= 1
	const unsigned long long run = n >= 64u ? ~0ull : (1ull << n) - 1ull;
	v.m |= a < 64u ? run << a : 0ull;
}
__device__ __forceinline__ bool visited(const Visits& v, uint32_t k) {
	const uint32_t a = k - v.k0;
	return a < 64u && ((v.m >> a) & 1ull);
}

template <bool FAST>
__device__ __forceinline__ bool march_event(const DevDataset& ds, const uint8_t* __restrict__ bf, const uint32_t* __restrict__ lin,
                                            const MarchRay& mr, float& t, uint32_t& k, uint32_t k_end, SegAcc& acc, Visits& vis,
                                            uint2* __restrict__ rec, uint32_t dbg = 0) {
	const uint32_t kb = k;
	if (FAST) {
		float pos[3];
#pragma unroll
		for (int d = 0; d < 3; ++d) pos[d] = mr.o[d] + t * mr.dir[d];
		if (!aabb_contains(ds, pos)) return false;
		const float m = fmaxf(fmaxf(fabsf(pos[0] - 0.5f), fabsf(pos[1] - 0.5f)), fabsf(pos[2] - 0.5f));
		int c[3] = {-1, -1, -1};
		uint32_t mip = 0;
		bool occ, interior = false;
		if ((m > 0.0f) & (m < 0.5f)) {
			mip0_cell(pos, c);
			const uint32_t wi = ((uint32_t)c[0] << 9) | ((uint32_t)c[1] << 2) | ((uint32_t)c[2] >> 5);
			occ = ((dbg & 2u) ? (wi * 2654435761u) : lin[wi]) >> (c[2] & 31) & 1;
			interior = (c[0] >= 1) & (c[0] <= NERF_GRIDSIZE - 2) & (c[1] >= 1) & (c[1] <= NERF_GRIDSIZE - 2) & (c[2] >= 1) &
			           (c[2] <= NERF_GRIDSIZE - 2) & !((c[0] == NERF_GRIDSIZE / 2) & (c[1] == NERF_GRIDSIZE / 2) & (c[2] == NERF_GRIDSIZE / 2));
		} else {
			mip = (uint32_t)mip_from_pos(pos[0], pos[1], pos[2]);
			occ = occupied(pos[0], pos[1], pos[2], bf, mip);
		}
		if (occ) {
			seg_add(rec, acc, t, k, dbg); t += MIN_CONE_STEPSIZE; ++k;
			if (interior) {
				while (k < k_end) {
					float p2[3];
#pragma unroll
					for (int d = 0; d < 3; ++d) p2[d] = mr.o[d] + t * mr.dir[d];
					int c2[3]; mip0_cell(p2, c2);
					if ((c2[0] != c[0]) | (c2[1] != c[1]) | (c2[2] != c[2])) break;
					seg_add(rec, acc, t, k, dbg); t += MIN_CONE_STEPSIZE; ++k;
				}
			}
			visit(vis, kb, k);
			return true;
		}
		seg_flush(rec, acc, dbg);
		visit(vis, kb, kb + 1);
		// advance_to_next_voxel with a constant step (march_step)
		const uint32_t res = NERF_GRIDSIZE >> mip;
		float tn = 3.402823466e+38f;
#pragma unroll
		for (int d = 0; d < 3; ++d) {
			const float p = res * pos[d];
			tn = fminf(tn, (floorf(p + 0.5f + 0.5f * signf(mr.dir[d])) - p) * mr.idir[d]);
		}
		const float t_target = t + fmaxf(ldexpf(tn, -(int)(7 - mip)), 0.0f);
		t += MIN_CONE_STEPSIZE; ++k;
		// do { t += dt; ++k; } while (t < t_target); bounded: at cone angle 0 the box diagonal is NERF_STEPS steps, so
		// no skip spans 4 NERF_STEPS and the bound only ends a corrupted t (the ray is ended, the step reports it).
		// A mip-0 skip (to the next cell boundary, <= sqrt(3) / 128 away) spans at most 8 steps: plain steps first (the
		// loop itself), the exact integer-domain jump (two divisions) only for what remains (mip >= 1 skips)
#pragma unroll
		for (int s = 0; s < 8; ++s)
			if (t < t_target) { t += MIN_CONE_STEPSIZE; ++k; }
		if (t < t_target && !step_until(t, k, t_target, k + 4 * NERF_STEPS, MIN_CONE_STEPSIZE)) return false;
		return true;
	} else {
		float dt, pos[3];
		// march_step without its skip loop (the steps of the skip are counted here)
#pragma unroll
		for (int d = 0; d < 3; ++d) pos[d] = mr.o[d] + t * mr.dir[d];
		if (!aabb_contains(ds, pos)) return false;
		dt = calc_dt(t, ds.cone_angle);
		const uint32_t mip = (uint32_t)mip_from_dt(dt, pos[0], pos[1], pos[2]);
		if (occupied(pos[0], pos[1], pos[2], bf, mip)) {
			seg_add(rec, acc, t, k); t += dt; ++k;
			visit(vis, kb, k);
			return true;
		}
		seg_flush(rec, acc);
		visit(vis, kb, kb + 1);
		// advance_to_next_voxel (march_common.h) with the step count
		const uint32_t res = NERF_GRIDSIZE >> mip;
		float p[3], tt[3];
#pragma unroll
		for (int d = 0; d < 3; ++d) { p[d] = res * pos[d]; tt[d] = (floorf(p[d] + 0.5f + 0.5f * signf(mr.dir[d])) - p[d]) * mr.idir[d]; }
		const float tn = fminf(fminf(tt[0], tt[1]), tt[2]);
		const float t_target = t + fmaxf(tn / res, 0.0f);
		do { t += calc_dt(t, ds.cone_angle); ++k; } while (t < t_target);
		return true;
	}
}

// Marches one segment [k, k_end) of a ray from the visited step (k, t); returns its exit: the first visited step at or
// past k_end (k_end itself inside a sample run) as (k, t), or k = FINISHED when the ray left the AABB first.
constexpr uint32_t FINISHED = 0xffffffffu;
template <bool FAST>
__device__ __forceinline__ void march_segment(const DevDataset& ds, const uint8_t* __restrict__ bf, const uint32_t* __restrict__ lin,
                                              const MarchRay& mr, float& t, uint32_t& k, uint32_t k_end, SegAcc& acc, Visits& vis,
                                              uint2* __restrict__ rec, uint32_t rec_cap, uint32_t* n_ev = nullptr, uint32_t dbg = 0) {
	while (k < k_end) {
		if (n_ev) ++*n_ev;
		if (acc.nrec + 1 >= rec_cap || !march_event<FAST>(ds, bf, lin, mr, t, k, k_end, acc, vis, rec, dbg)) { k = FINISHED; break; }
	}
	seg_flush(rec, acc, dbg);
}

// Two passes over the ray slots. Only a prefix of the slots can be kept: slot i is kept iff n_i > 0 and
// sum_{j<i} n_j + n_i <= max_inference (<= max_samples), so once the rays before slot `est` request max_samples
// samples, every later ray is dropped whatever it would count. Pass 0 marches [0, est) (est from the previous
// step's kept extent) and sums its counts; pass 1 marches [est, R) only when that sum is below max_samples, and
// otherwise marks those slots dropped (nreq = 1: past the cap in the scan, nothing recorded). The kept rays, their
// samples and every training result are those of marching all slots; the requested-sample counter then reads a
// value at or above max_samples, which is all the reference ever uses of it (min(counter, max_samples),
// testbed_nerf.cu:3036-3039; the rest is the GUI's text).
//
// Each ray is marched by MG lanes at once (8 by default). The march's t values are the sequence t0, t0 + dt, ... (every update of
// the reference's loop is one t += dt, the skip included), so lane g starts at the first step k_g of the g-th slice
// of [t0, t_exit) by stepping there, and marches its segment [k_g, k_{g+1}) as if k_g were visited. The true march
// enters segment g at v_g, the exit of segment g - 1; the march is a deterministic function of its visited step, so
// when lane g's trajectory visits v_g the two coincide from there and lane g keeps its samples at k >= v_g; when it
// does not (a skip of the previous segment landed on a step lane g jumped over), lane g re-marches from v_g. The
// checks run in segment order. Samples past NERF_STEPS are cut (the reference's loop stops there). The result is the
// single-lane march's, sample for sample (tests/test_gpu_parity.py::test_sample_rays_bit_exact).
template <bool FAST, int MG>
#ifndef NEUS_MARCH_WPE
#define NEUS_MARCH_WPE 0
#endif
#if NEUS_MARCH_WPE
#define MARCH_OCC __attribute__((amdgpu_waves_per_eu(NEUS_MARCH_WPE, NEUS_MARCH_WPE)))
#else
#define MARCH_OCC
#endif
__global__ void __launch_bounds__(256) MARCH_OCC k_march(uint32_t cap_rays, uint32_t pass, uint32_t max_samples, StepState* __restrict__ st, DevDataset ds,
                                               const uint8_t* __restrict__ bitfield, const uint32_t* __restrict__ lin, const float* __restrict__ rays,
                                               const float* __restrict__ tstart, uint32_t* __restrict__ nreq, MarchWork mw) {
	const uint32_t est = st->march_est ? min(st->march_est, cap_rays) : cap_rays;
	const uint32_t lo = pass == 0 ? 0u : est, hi = pass == 0 ? est : cap_rays;
	if (lo >= hi) return;
	if (pass == 1 && st->march_total >= max_samples) {
		for (uint32_t k = lo + blockIdx.x * blockDim.x + threadIdx.x; k < hi; k += gridDim.x * blockDim.x) { nreq[k] = 1; mw.nrec[k] = 0; }
		return;
	}
	constexpr uint32_t SEG_CAP = MARCH_SEG_RECS / MG;  // segment-local records per lane
	const uint32_t lane = threadIdx.x & 63, g = lane % MG;
	const uint32_t groups = (gridDim.x * blockDim.x) / MG;
	uint32_t total = 0;
	// development timing (MarchWork::prof): wall clock (100 MHz) at the phases of the wave's first ray group
	unsigned long long* pw = mw.prof ? mw.prof + (size_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 8 : nullptr;
	bool first = true;
	uint32_t n_redo = 0;
	auto stamp = [&](int ph) { if (pw && first && lane == 0) pw[ph] = wall_clock64(); };
	stamp(0);
	for (uint32_t i = lo + (blockIdx.x * blockDim.x + threadIdx.x) / MG; i - lo < ((hi - lo + groups - 1) / groups) * groups; i += groups) {
		const bool have = i < hi;
		const float t0 = have ? tstart[i] : -1.f;
		MarchRay mr;
		float t_exit = t0;
		if (t0 >= 0.f) {
			load_march_ray(rays, i, mr, ds.motion.on != 0);
			float tx[3];
#pragma unroll
			for (int d = 0; d < 3; ++d) {
				const float a = (ds.aabb_min[d] - mr.o[d]) * mr.idir[d], b = (ds.aabb_max[d] - mr.o[d]) * mr.idir[d];
				tx[d] = fmaxf(a, b);
			}
			t_exit = fminf(fminf(tx[0], tx[1]), tx[2]);
		}
		const float span = t_exit - t0;
		const bool split = t0 >= 0.f && span > 0.f && span < 1e4f;
		// lane g's first step: step from t0 to the start of its slice (lane 0: t0 itself)
		float t = t0;
		uint32_t k = 0;
		const bool active = t0 >= 0.f && (g == 0 || split);
		if (active && g > 0) {
			const float t_g = t0 + span * ((float)g / (float)MG);
			if (FAST) step_until(t, k, t_g, 4 * NERF_STEPS, MIN_CONE_STEPSIZE);  // (a bad t ends the ray at its first event)
			else while (t < t_g && k < 4 * NERF_STEPS) { t += calc_dt(t, ds.cone_angle); ++k; }
		}
		stamp(1);
		uint32_t k_end = (uint32_t)__shfl((int)k, (int)((lane + 1) % 64));  // the next lane's start
		if (g == MG - 1 || !split) k_end = FINISHED;
		uint2* rec = mw.seg + ((size_t)i * MG + g) * SEG_CAP;
		SegAcc acc{0.f, 0u, 0u, 0u, 0u};
		Visits vis{0ull, k};
		float et = t;
		uint32_t ek = active ? k : FINISHED;
		uint32_t n_ev = 0;
		if (active) { march_segment<FAST>(ds, bitfield, lin, mr, et, ek, k_end, acc, vis, rec, SEG_CAP, &n_ev, mw.dbg); }
		// health: an active lane whose walk ends on a negative or non-finite t was handed a corrupted state
		if (__builtin_expect(__ballot(active && !((et >= 0.f) & (et < __builtin_huge_valf()))) != 0ull, 0) && lane == 0)
			atomicOr(&st->fail_flags, STEP_FAIL_MARCH_T);
		stamp(2);
		// segment order: lane g joins the exit of lane g - 1
		uint32_t vk = k;   // first valid step of this segment
		for (int q = 1; q < MG; ++q) {
			const uint32_t pk = (uint32_t)__shfl((int)ek, (int)(lane - 1) & 63);
			const float pt = __shfl(et, (int)(lane - 1) & 63);
			bool redo = false;
			if (g == (uint32_t)q && active) {
				if (pk == FINISHED || pk >= k_end) {  // the ray ended (or jumped past this segment) before it
					acc.n = 0; acc.nrec = 0; vk = pk; ek = pk; et = pt;
				} else {
					if (visited(vis, pk)) vk = pk;
					else redo = true;
				}
			}
			if (__ballot(redo)) {
				++n_redo;
				if (redo) {
					acc = SegAcc{0.f, 0u, 0u, 0u, 0u}; vis = Visits{0ull, pk};
					et = pt; ek = pk; vk = pk;
					march_segment<FAST>(ds, bitfield, lin, mr, et, ek, k_end, acc, vis, rec, SEG_CAP);
				}
			}
		}
		stamp(3);
		// samples of this segment at k >= vk (the first run may start before vk and is cut there)
		uint32_t n_g = 0, r_first = 0;
		float t_first = 0.f;
		uint32_t cut = 0;  // samples dropped from the first kept run
		if (active && vk != FINISHED) {
			for (uint32_t r = 0; r < acc.nrec; ++r) {
				const uint2 R = rec[r];
				const uint32_t k0 = R.y >> 8, len = R.y & 0xff;
				if (k0 + len <= vk) { r_first = r + 1; continue; }
				if (r == r_first && k0 < vk) { cut = vk - k0; }
				n_g += len - (r == r_first ? cut : 0u);
			}
		}
		if (!active || vk == FINISHED) { n_g = 0; r_first = acc.nrec; }
		// prefix over the ray's lanes (in segment order) of the samples, NERF_STEPS cap
		uint32_t before = 0;
		for (int q = 0; q < MG - 1; ++q) {
			const uint32_t pn = (uint32_t)__shfl((int)n_g, (int)(lane - g + q));
			if ((uint32_t)q < g) before += pn;
		}
		const uint32_t keep = before >= NERF_STEPS ? 0u : min(n_g, NERF_STEPS - before);
		// records this lane emits for its `keep` samples, and their prefix over the lanes
		uint32_t w_g = 0;
		{
			uint32_t got = 0;
			for (uint32_t r = r_first; r < acc.nrec && got < keep; ++r) {
				const uint32_t len = (rec[r].y & 0xff) - (r == r_first ? cut : 0u);
				got += len; ++w_g;
			}
		}
		uint32_t rbefore = 0, r_tot = 0;
		for (int q = 0; q < MG; ++q) {
			const uint32_t pw = (uint32_t)__shfl((int)w_g, (int)(lane - g + q));
			if ((uint32_t)q < g) rbefore += pw;
			r_tot += pw;
		}
		stamp(4);
		// final records: {t of the first sample, (samples of the ray before the run) << 16 | length}
		uint2* out = mw.rec + (size_t)i * NERF_STEPS;
		uint32_t written = 0, nr = rbefore;
		for (uint32_t r = r_first; r < acc.nrec && written < keep; ++r) {
			const uint2 R = rec[r];
			uint32_t len = R.y & 0xff;
			float tr = __uint_as_float(R.x);
			if (r == r_first && cut) {
				for (uint32_t c = 0; c < cut; ++c) tr += FAST ? MIN_CONE_STEPSIZE : calc_dt(tr, ds.cone_angle);
				len -= cut;
			}
			len = min(len, keep - written);
			out[nr++] = make_uint2(__float_as_uint(tr), ((before + written) << 16) | len);
			written += len;
		}
		// the ray's sample total from its last lane
		const uint32_t n_tot = (uint32_t)__shfl((int)(before + keep), (int)(lane - g + MG - 1));
		if (have && g == 0) {
			nreq[i] = t0 >= 0.f ? n_tot : 0u;
			mw.nrec[i] = t0 >= 0.f ? r_tot : 0u;
			total += t0 >= 0.f ? n_tot : 0u;
		}
		if (pw && first) {
			stamp(5);
			uint32_t ws = g == 0 && have && t0 >= 0.f ? n_tot : 0u;
#pragma unroll
			for (int off = 32; off > 0; off >>= 1) ws += (uint32_t)__shfl_xor((int)ws, off);
			uint32_t emax = n_ev, esum = n_ev;
#pragma unroll
			for (int off = 32; off > 0; off >>= 1) { emax = max(emax, (uint32_t)__shfl_xor((int)emax, off)); esum += (uint32_t)__shfl_xor((int)esum, off); }
			if (lane == 0) { pw[6] = ws; pw[7] = ((unsigned long long)emax << 32) | ((unsigned long long)esum << 8) | n_redo; }
		}
		first = false;
	}
	if (pass == 0) {  // the pass's requested samples (one atomic per wave)
		total = wave_sum(total);
		if (lane == 0 && total) atomicAdd(&st->march_total, total);
	}
}

constexpr uint32_t MARCH_BAL_MAX = 16;  // lanes of one ray at most (k_march_bal)
// Balanced lanes (MarchWork::balanced, constant-step march): a wave takes 8 consecutive ray slots and shares its 64
// lanes among them in proportion to the mip-0 cells each crosses inside the AABB (span x (|dx| + |dy| + |dz|): one march
// event per cell crossed), every active ray at least one lane and a ray's lanes contiguous. With 8 lanes per ray a wave
// lasted as long as its longest ray's slices while the lanes of short, dropped and culled rays idled (lane event mean
// 20.5 vs max 28.9 at the step-1600 state). The slices, joins and outputs are k_march's with a per-ray lane count m:
// where a lane starts never changes a result (the join keeps only samples of the true trajectory), so the output is
// the single-lane march's, bit for bit.
__global__ void __launch_bounds__(256) MARCH_OCC k_march_bal(uint32_t cap_rays, uint32_t pass, uint32_t max_samples, StepState* __restrict__ st,
                                                   DevDataset ds, const uint8_t* __restrict__ bitfield, const uint32_t* __restrict__ lin,
                                                   const float* __restrict__ rays, const float* __restrict__ tstart, uint32_t* __restrict__ nreq,
                                                   MarchWork mw) {
	constexpr bool FAST = true;
	uint32_t est = st->march_est ? min(st->march_est, cap_rays) : cap_rays;
	bool mcut = false;  // the march cut: pass 0 marches the slots below the estimate; pass 1 drops the rest behind one marker
	if (mw.est_cut && *mw.est_cut / mw.est_div < est) { est = *mw.est_cut / mw.est_div; mcut = true; }
	const uint32_t lo = pass == 0 ? 0u : est, hi = pass == 0 ? est : cap_rays;
	if (lo >= hi) return;
	// (a cut march: k_ray_gen marked the dropped slots - the first requests past the cap, so nothing after it is kept and
	// the requested count reads above max_samples, the next step's max_inference then max_samples; the rest nothing)
	if (pass == 1 && mcut) return;
	if (pass == 1 && st->march_total >= max_samples) {
		for (uint32_t k = lo + blockIdx.x * blockDim.x + threadIdx.x; k < hi; k += gridDim.x * blockDim.x) { nreq[k] = 1; mw.nrec[k] = 0; }
		return;
	}
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
	uint32_t total = 0;
	unsigned long long* pw = mw.prof ? mw.prof + (size_t)wave * 8 : nullptr;
	bool first = true;
	uint32_t n_redo = 0;
	auto stamp = [&](int ph) { if (pw && first && lane == 0) pw[ph] = wall_clock64(); };
	stamp(0);
	for (uint32_t b = lo + 8 * wave; b < hi; b += 8 * n_waves) {
		// ---- the group's rays on lanes 0..7: start, exit, weight
		float t0r = -1.f, wr = 0.f;
		if (lane < 8 && b + lane < hi) {
			t0r = tstart[b + lane];
			if (t0r >= 0.f) {
				MarchRay m;
				load_march_ray(rays, b + lane, m, ds.motion.on != 0);
				float te = 3.402823466e+38f;
#pragma unroll
				for (int d = 0; d < 3; ++d) te = fminf(te, fmaxf((ds.aabb_min[d] - m.o[d]) * m.idir[d], (ds.aabb_max[d] - m.o[d]) * m.idir[d]));
				const float span = te - t0r;
				if (span > 0.f && span < 1e4f) wr = span * (fabsf(m.dir[0]) + fabsf(m.dir[1]) + fabsf(m.dir[2]));
			}
		}
		// ---- lanes per ray (wave-uniform): 1 per active ray, the rest by weight, the remainder to the heaviest ray; at
		// most 16 per ray (the segment scratch of a ray, MARCH_SEG_RECS runs, is split over its lanes: at 16 a lane holds
		// 68 runs for its at most 1024 / 16 + 2 steps), lanes beyond that idle
		uint32_t mr[8], Lr[8];
		float W = 0.f, wmax = -1.f;
		uint32_t n_act = 0, heavy = 0;
		float wv[8];
#pragma unroll
		for (int r = 0; r < 8; ++r) {
			wv[r] = __shfl(wr, r);
			const bool act = __shfl(t0r, r) >= 0.f;
			mr[r] = act ? 1u : 0u;
			n_act += act ? 1u : 0u;
			W += wv[r];
			if (act && wv[r] > wmax) { wmax = wv[r]; heavy = (uint32_t)r; }
		}
		uint32_t used = n_act;
		if (W > 0.f) {
			const float extra = (float)(64u - n_act);
#pragma unroll
			for (int r = 0; r < 8; ++r) {
				const uint32_t add = mr[r] ? min((uint32_t)(extra * (wv[r] / W)), MARCH_BAL_MAX - 1u) : 0u;
				mr[r] += add;
				used += add;
			}
			if (used < 64u && wv[heavy] > 0.f) { const uint32_t add = min(64u - used, MARCH_BAL_MAX - mr[heavy]); mr[heavy] += add; used += add; }
		}
		uint32_t acc_l = 0, maxm = 1;
#pragma unroll
		for (int r = 0; r < 8; ++r) { Lr[r] = acc_l; acc_l += mr[r]; maxm = max(maxm, mr[r]); }
		// this lane's ray and segment
		int rr = -1;
#pragma unroll
		for (int r = 0; r < 8; ++r) if (mr[r] && lane >= Lr[r] && lane < Lr[r] + mr[r]) rr = r;
		const bool have = rr >= 0;
		const uint32_t MG = have ? mr[rr] : 1u, g = have ? lane - Lr[rr] : 0u;
		const uint32_t i = have ? b + (uint32_t)rr : b;
		const float t0 = __shfl(t0r, have ? rr : 0);
		MarchRay mr_{};
		float t_exit = t0;
		if (have && t0 >= 0.f) {
			load_march_ray(rays, i, mr_, ds.motion.on != 0);
			float tx[3];
#pragma unroll
			for (int d = 0; d < 3; ++d) {
				const float a = (ds.aabb_min[d] - mr_.o[d]) * mr_.idir[d], c = (ds.aabb_max[d] - mr_.o[d]) * mr_.idir[d];
				tx[d] = fmaxf(a, c);
			}
			t_exit = fminf(fminf(tx[0], tx[1]), tx[2]);
		}
		const float span = t_exit - t0;
		const bool split = have && t0 >= 0.f && span > 0.f && span < 1e4f;
		float t = t0;
		uint32_t k = 0;
		const bool active = have && t0 >= 0.f && (g == 0 || split);
		if (active && g > 0) step_until(t, k, t0 + span * ((float)g / (float)MG), 4 * NERF_STEPS, MIN_CONE_STEPSIZE);
		stamp(1);
		uint32_t k_end = (uint32_t)__shfl((int)k, (int)((lane + 1) & 63));  // the next lane's start
		if (g + 1 == MG || !split) k_end = FINISHED;
		const uint32_t seg_cap = MARCH_SEG_RECS / MG;
		uint2* rec = mw.seg + (size_t)i * MARCH_SEG_RECS + (size_t)g * seg_cap;
		SegAcc acc{0.f, 0u, 0u, 0u, 0u};
		Visits vis{0ull, k};
		float et = t;
		uint32_t ek = active ? k : FINISHED;
		uint32_t n_ev = 0;
		if (active) march_segment<FAST>(ds, bitfield, lin, mr_, et, ek, k_end, acc, vis, rec, seg_cap, &n_ev, mw.dbg);
		if (__builtin_expect(__ballot(active && !((et >= 0.f) & (et < __builtin_huge_valf()))) != 0ull, 0) && lane == 0)
			atomicOr(&st->fail_flags, STEP_FAIL_MARCH_T);
		stamp(2);
		// segment order: lane g joins the exit of lane g - 1 (the lanes of a ray are contiguous)
		uint32_t vk = k;
		for (uint32_t q = 1; q < maxm; ++q) {
			const uint32_t pk = (uint32_t)__shfl((int)ek, (int)((lane - 1) & 63));
			const float pt = __shfl(et, (int)((lane - 1) & 63));
			bool redo = false;
			if (g == q && active) {
				if (pk == FINISHED || pk >= k_end) {
					acc.n = 0; acc.nrec = 0; vk = pk; ek = pk; et = pt;
				} else {
					if (visited(vis, pk)) vk = pk;
					else redo = true;
				}
			}
			if (__ballot(redo)) {
				++n_redo;
				if (redo) {
					acc = SegAcc{0.f, 0u, 0u, 0u, 0u}; vis = Visits{0ull, pk};
					et = pt; ek = pk; vk = pk;
					march_segment<FAST>(ds, bitfield, lin, mr_, et, ek, k_end, acc, vis, rec, seg_cap);
				}
			}
		}
		stamp(3);
		uint32_t n_g = 0, r_first = 0, cut = 0;
		if (active && vk != FINISHED) {
			for (uint32_t r = 0; r < acc.nrec; ++r) {
				const uint2 R = rec[r];
				const uint32_t k0 = R.y >> 8, len = R.y & 0xff;
				if (k0 + len <= vk) { r_first = r + 1; continue; }
				if (r == r_first && k0 < vk) { cut = vk - k0; }
				n_g += len - (r == r_first ? cut : 0u);
			}
		}
		if (!active || vk == FINISHED) { n_g = 0; r_first = acc.nrec; }
		// prefix over the ray's lanes (in segment order) of the samples, NERF_STEPS cap
		const uint32_t L0 = lane - g;
		uint32_t before = 0;
		for (uint32_t q = 0; q + 1 < maxm; ++q) {
			const uint32_t pn = (uint32_t)__shfl((int)n_g, (int)((L0 + q) & 63));
			if (q < g) before += pn;
		}
		const uint32_t keep = before >= NERF_STEPS ? 0u : min(n_g, NERF_STEPS - before);
		uint32_t w_g = 0;
		{
			uint32_t got = 0;
			for (uint32_t r = r_first; r < acc.nrec && got < keep; ++r) {
				const uint32_t len = (rec[r].y & 0xff) - (r == r_first ? cut : 0u);
				got += len; ++w_g;
			}
		}
		uint32_t rbefore = 0, r_tot = 0;
		for (uint32_t q = 0; q < maxm; ++q) {
			const uint32_t pwg = (uint32_t)__shfl((int)w_g, (int)((L0 + q) & 63));
			if (q < g) rbefore += pwg;
			if (q < MG) r_tot += pwg;
		}
		stamp(4);
		uint2* out = mw.rec + (size_t)i * NERF_STEPS;
		uint32_t written = 0, nr = rbefore;
		for (uint32_t r = r_first; r < acc.nrec && written < keep; ++r) {
			const uint2 R = rec[r];
			uint32_t len = R.y & 0xff;
			float tr = __uint_as_float(R.x);
			if (r == r_first && cut) {
				for (uint32_t c = 0; c < cut; ++c) tr += MIN_CONE_STEPSIZE;
				len -= cut;
			}
			len = min(len, keep - written);
			out[nr++] = make_uint2(__float_as_uint(tr), ((before + written) << 16) | len);
			written += len;
		}
		const uint32_t n_tot = (uint32_t)__shfl((int)(before + keep), (int)((L0 + MG - 1) & 63));
		if (have && g == 0) {
			nreq[i] = t0 >= 0.f ? n_tot : 0u;
			mw.nrec[i] = t0 >= 0.f ? r_tot : 0u;
			total += t0 >= 0.f ? n_tot : 0u;
		}
		// slots of the group without a lane (b + r < hi, no samples: t0 < 0) report 0 from lanes 0..7
		if (lane < 8 && b + lane < hi && !(t0r >= 0.f)) { nreq[b + lane] = 0u; mw.nrec[b + lane] = 0u; }
		if (pw && first) {
			stamp(5);
			uint32_t ws = g == 0 && have && t0 >= 0.f ? n_tot : 0u;
#pragma unroll
			for (int off = 32; off > 0; off >>= 1) ws += (uint32_t)__shfl_xor((int)ws, off);
			uint32_t emax = n_ev, esum = n_ev;
#pragma unroll
			for (int off = 32; off > 0; off >>= 1) { emax = max(emax, (uint32_t)__shfl_xor((int)emax, off)); esum += (uint32_t)__shfl_xor((int)esum, off); }
			if (lane == 0) { pw[6] = ws; pw[7] = ((unsigned long long)emax << 32) | ((unsigned long long)esum << 8) | n_redo; }
		}
		first = false;
	}
	if (pass == 0) {
		total = wave_sum(total);
		if (lane == 0 && total) atomicAdd(&st->march_total, total);
	}
}

// t of local sample j of ray slot i from its runs: the run holding j, then the run's t += dt replayed
template <bool FAST>
__device__ __forceinline__ float run_sample_t(const MarchWork& mw, uint32_t i, uint32_t j, float cone) {
	const uint2* __restrict__ rr = mw.rec + (size_t)i * NERF_STEPS;
	uint32_t lo = 0, hi = mw.nrec[i];
	while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if ((rr[mid].y >> 16) <= j) lo = mid; else hi = mid; }
	const uint2 r = rr[lo];
	float t = __uint_as_float(r.x);
	for (uint32_t k = r.y >> 16; k < j; ++k) t += FAST ? MIN_CONE_STEPSIZE : calc_dt(t, cone);
	return t;
}

// ---------------------------------------------------------------- pass 2: write kept rays
// (a) k_march_scan, one launch (scan_lookback.h): the exclusive scan of the requested counts (base), and per ray slot
//     numsteps (n or 0, base), the requested total, the kept-sample extent / kept-ray count (one atomic triple per
//     4096-slot tile); with a round-0 list (progressive inference) also the exclusive scan of min(n, e1) (the slot of
//     each kept ray's first chunk in the list: the rays before a kept ray with samples are all kept, so the dropped
//     rays' terms never reach a kept ray's prefix) and the list's length (an atomic max per tile).
__global__ void __launch_bounds__(SCAN_THREADS) k_march_scan(uint32_t cap_rays, StepState* __restrict__ st, const uint32_t* __restrict__ nreq,
                                                             uint32_t* __restrict__ base, uint32_t* __restrict__ numsteps, ScanState* __restrict__ ss,
                                                             uint32_t tag, Round0List r0) {
	__shared__ uint32_t s_pre[2], s_wsum[2][SCAN_THREADS / 64], s_red[4][SCAN_THREADS / 64];
	const ScanTile tl = scan_tile(tag);
	const uint32_t max_samples = st->max_inference;
	const uint32_t i0 = tl.tile * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
	uint32_t v[SCAN_ITEMS];
	scan_load16(nreq, i0, cap_rays, true, v);
	uint32_t tsum = 0, tsum2 = 0;
#pragma unroll
	for (int k = 0; k < (int)SCAN_ITEMS; ++k) { tsum += v[k]; tsum2 += min(v[k], r0.e1); }
	uint32_t agg, agg2 = 0;
	const uint32_t tex = scan_block(tsum, s_wsum[0], agg);
	const uint32_t tex2 = r0.list ? scan_block(tsum2, s_wsum[1], agg2) : 0u;
	if (threadIdx.x < 64) {
		const uint32_t p = scan_lookback(ss, 0, tl, agg);
		const uint32_t p2 = r0.list ? scan_lookback(ss, 1, tl, agg2) : 0u;
		if (threadIdx.x == 0) { s_pre[0] = p; s_pre[1] = p2; }
	}
	__syncthreads();
	uint32_t b = s_pre[0] + tex, c = s_pre[1] + tex2;
	uint32_t bo[SCAN_ITEMS], ns[2 * SCAN_ITEMS], co[SCAN_ITEMS];
	uint32_t kmax = 0, kcnt = 0, kext = 0, cmax = 0;
#pragma unroll
	for (int k = 0; k < (int)SCAN_ITEMS; ++k) {
		const uint32_t n = v[k], i = i0 + k;
		const bool keep = n > 0 && b + n <= max_samples && i < cap_rays;
		if (i == cap_rays - 1) st->numsteps_counter = b + n;
		bo[k] = b; ns[2 * k] = keep ? n : 0u; ns[2 * k + 1] = b; co[k] = c;
		if (keep) { kmax = max(kmax, b + n); ++kcnt; kext = i + 1; cmax = max(cmax, c + min(n, r0.e1)); }
		b += n; c += min(n, r0.e1);
	}
	scan_store16(base, i0, cap_rays, true, bo);
	if (i0 + SCAN_ITEMS <= cap_rays) {
		uint4* p = (uint4*)(numsteps + 2 * (size_t)i0);
#pragma unroll
		for (int q = 0; q < (int)SCAN_ITEMS / 2; ++q) p[q] = make_uint4(ns[4 * q], ns[4 * q + 1], ns[4 * q + 2], ns[4 * q + 3]);
	} else {
#pragma unroll
		for (int k = 0; k < (int)SCAN_ITEMS; ++k) if (i0 + k < cap_rays) { numsteps[2 * (i0 + k)] = ns[2 * k]; numsteps[2 * (i0 + k) + 1] = ns[2 * k + 1]; }
	}
	if (r0.list) scan_store16(r0.c0, i0, cap_rays, true, co);
	// the tile's kept maxima / count: one atomic each
	kmax = wave_max(kmax); kcnt = wave_sum(kcnt); kext = wave_max(kext); cmax = wave_max(cmax);
	const uint32_t wv = threadIdx.x >> 6;
	if ((threadIdx.x & 63) == 0) { s_red[0][wv] = kmax; s_red[1][wv] = kcnt; s_red[2][wv] = kext; s_red[3][wv] = cmax; }
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int w = 1; w < (int)(SCAN_THREADS / 64); ++w) {
			kmax = max(kmax, s_red[0][w]); kcnt += s_red[1][w]; kext = max(kext, s_red[2][w]); cmax = max(cmax, s_red[3][w]);
		}
		if (kcnt) { atomicMax(&st->n_kept, kmax); atomicAdd(&st->n_rays_with_samples, kcnt); atomicMax(&st->kept_extent, kext); }
		if (r0.list && cmax) atomicMax(&r0.counters[0], cmax);  // the round-0 list's length (counters zeroed by k_ray_gen)
	}
}

// (b) block per WRITE_CHUNK consecutive output samples (balanced whatever the spread of samples over
//     rays; kept rays form a prefix of the slot order since base is monotone). The block finds the
//     ray slots overlapping its chunk by binary search over base, stages up to 256 of them (base, n,
//     o, d, record offsets) in LDS, maps each chunk sample to its run (one thread per run), then walks the
//     chunk with consecutive threads on consecutive samples: t replayed from the run's first sample exactly
//     as the march stepped it, NerfCoordinate with pos = o + t d, warped dt, warped dir.
constexpr uint32_t WRITE_CHUNK = 4096;
__device__ __forceinline__ uint32_t last_le(const uint32_t* __restrict__ a, uint32_t n, uint32_t q) {  // last k < n with a[k] <= q (a[0] <= q)
	uint32_t lo = 0, hi = n;
	while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (a[mid] <= q) lo = mid; else hi = mid; }
	return lo;
}
__global__ void __launch_bounds__(256) k_march_write(uint32_t cap_rays, StepState* __restrict__ st, DevDataset ds,
                                                     const float* __restrict__ rays, const MarchWork mw,
                                                     const uint32_t* __restrict__ nreq, const uint32_t* __restrict__ base,
                                                     float* __restrict__ coords, uint32_t* __restrict__ sample_ray, Round0List r0) {
	__shared__ float s_ray[6][256];
	__shared__ uint32_t s_b[256], s_n[256], s_roff[256], s_c0[256];
	__shared__ uint32_t s_range[3];
	__shared__ uint32_t s_t0[WRITE_CHUNK];  // per chunk sample: t of its run's first sample (bits)
	__shared__ uint16_t s_r[WRITE_CHUNK];   // its ray within the staged batch
	__shared__ uint8_t s_u[WRITE_CHUNK];    // its step within the run
	const uint32_t max_samples = st->max_inference, n_kept = st->n_kept;
	const uint32_t tid = threadIdx.x;
	const uint32_t q0 = blockIdx.x * WRITE_CHUNK;
	if (q0 >= max_samples) return;
	const uint32_t q1 = min(q0 + WRITE_CHUNK, max_samples);
	if (tid == 0) {
		s_range[0] = last_le(base, cap_rays, q0);
		s_range[1] = last_le(base, cap_rays, q1 - 1);
	}
	__syncthreads();
	const uint32_t r_lo = s_range[0], r_hi = s_range[1];
	const float diag[3] = {ds.aabb_max[0] - ds.aabb_min[0], ds.aabb_max[1] - ds.aabb_min[1], ds.aabb_max[2] - ds.aabb_min[2]};
	for (uint32_t rb = r_lo; rb <= r_hi; rb += 256) {
		const uint32_t nr = min(256u, r_hi + 1 - rb);
		if (tid < nr) {
			const uint32_t i = rb + tid;
			const uint32_t n = nreq[i], b = base[i];
			const bool keep = n > 0 && b + n <= max_samples;
			s_b[tid] = b; s_n[tid] = keep ? n : 0u;
			if (r0.list) s_c0[tid] = r0.c0[i];
			if (keep) {
				MarchRay mr;
				load_march_ray(rays, i, mr, ds.motion.on != 0);
#pragma unroll
				for (int d = 0; d < 3; ++d) { s_ray[d][tid] = mr.o[d]; s_ray[3 + d][tid] = mr.dir[d]; }
			}
		}
		// (1) one thread per sample RUN (record) of the batch's rays: for each of the run's samples in this chunk,
		//     the run's first t, the sample's step within the run and its ray go to LDS maps (a binary search over
		//     the ray's records per sample was a chain of dependent loads: waves waited ~75 % of the time)
		s_roff[tid] = tid < nr ? (s_n[tid] ? mw.nrec[rb + tid] : 0u) : 0u;
		__syncthreads();
		if (tid < 64) {  // exclusive scan of the 256 record counts (one wave, 4 per lane)
			uint32_t v[4], sum = 0;
#pragma unroll
			for (int k = 0; k < 4; ++k) { v[k] = s_roff[4 * tid + k]; sum += v[k]; }
			const uint32_t inc = wave_incl_sum(sum);
			uint32_t ex = inc - sum;
#pragma unroll
			for (int k = 0; k < 4; ++k) { s_roff[4 * tid + k] = ex; ex += v[k]; }
			if (tid == 63) s_range[2] = inc;  // records of the batch
		}
		__syncthreads();
		const uint32_t n_rec = s_range[2];
		for (uint32_t g = tid; g < n_rec; g += 256) {
			const uint32_t r = last_le(s_roff, nr, g);
			const uint32_t i = rb + r, k = g - s_roff[r];
			const uint2 R = mw.rec[(size_t)i * NERF_STEPS + k];
			const uint32_t qs = s_b[r] + (R.y >> 16), len = R.y & 0xffffu;
			for (uint32_t u = 0; u < len; ++u) {
				const uint32_t q = qs + u;
				if (q >= q0 && q < q1) { s_t0[q - q0] = R.x; s_u[q - q0] = (uint8_t)u; s_r[q - q0] = (uint16_t)r; }
			}
		}
		__syncthreads();
		// (2) consecutive threads on the batch's consecutive samples: t replayed from the run's first sample
		// (<= MARCH_RUN_MAX - 1 steps, exactly as the march stepped it; 41 -> 39 us with the constant step's jumps),
		// coalesced NerfCoordinate stores
		// slots at or past n_kept belong to no kept ray (the first ray over the cap and every later one): none of its
		// runs mapped them in (1), so their LDS map entries are stale and they are skipped
		const uint32_t qa = max(q0, s_b[0]);
		const uint32_t qb = min(rb + nr > r_hi ? q1 : min(q1, base[rb + nr]), n_kept);
		for (uint32_t q = qa + tid; q < qb; q += 256) {
			const uint32_t r = s_r[q - q0];
			const uint32_t j = q - s_b[r];
			if (j >= s_n[r]) continue;  // not a kept sample (no run wrote this slot)
			const uint32_t i = rb + r;
			float t = __uint_as_float(s_t0[q - q0]);
			if (ds.cone_angle == 0.0f) {  // the run's u constant steps in a few integer-domain jumps (exact, step_until)
				uint32_t kk = 0;
				if (!step_until(t, kk, __int_as_float(0x7f800000), s_u[q - q0], MIN_CONE_STEPSIZE)) atomicOr(&st->fail_flags, STEP_FAIL_MARCH_T);
			} else
			for (uint32_t u = s_u[q - q0]; u > 0; --u) t += ds.cone_angle == 0.0f ? MIN_CONE_STEPSIZE : calc_dt(t, ds.cone_angle);
			const float o[3] = {s_ray[0][r], s_ray[1][r], s_ray[2][r]}, dir[3] = {s_ray[3][r], s_ray[4][r], s_ray[5][r]};
			float pos[3];
#pragma unroll
			for (int d = 0; d < 3; ++d) pos[d] = o[d] + t * dir[d];
			const float dt = ds.cone_angle == 0.0f ? MIN_CONE_STEPSIZE : calc_dt(t, ds.cone_angle);
			// NerfCoordinate (28 B): one 16 B + one 12 B store (4 B-aligned vector stores)
			float* cc = coords + (size_t)q * COORD_W;
			const f4u p4 = {(pos[0] - ds.aabb_min[0]) / diag[0], (pos[1] - ds.aabb_min[1]) / diag[1], (pos[2] - ds.aabb_min[2]) / diag[2], warp_dt(dt)};
			*(f4u*)cc = p4;
			*(f3u*)(cc + 4) = (f3u){(dir[0] + 1.0f) * 0.5f, (dir[1] + 1.0f) * 0.5f, (dir[2] + 1.0f) * 0.5f};
			if (sample_ray) sample_ray[q] = i;  // (operator path only: the training step maps compacted samples by cmap)
			if (r0.list && j < r0.e1) r0.list[s_c0[r] + j] = q;  // the first chunk of the ray: progressive round 0
		}
		__syncthreads();
	}
}

// ---------------------------------------------------------------- spatial ray order (progressive rounds)
// k_nerf_infer's hash-grid gathers miss an XCD's 4 MB L2 on a list in ray-slot order (random pixels of random views:
// every wave touches the whole surface). With round 0's list in Morton order of 8^3 cells of each ray's first kept
// sample, and the rays in that order through k_loss_scan_chunk (so later rounds' lists follow it), the inference takes
// the list as 8 contiguous eighths, eighth x on XCD x (InferAlpha::xcd_parts): each XCD gathers from one eighth of the
// surface. A counting sort over the ray slots in RS_RPB-slot blocks: per-block LDS histograms into a [2][bin][block]
// matrix, one device-wide exclusive scan of it (scan.hip), placement with LDS cursors (global per-ray atomics on the
// ~300 rays of an occupied cell serialised at the memory side: ~50 us). Order within a cell is immaterial (every work
// item writes its own sample's slots, every ray's recurrence is its own), so results are unchanged.
constexpr uint32_t RS_RPB = 1024, RS_NB = RS_BINS + 1, RS_NB2 = 2 * RS_BINS + 1;
__device__ __forceinline__ uint32_t spread4(uint32_t v) {
	v &= 15u;
	v = (v | (v << 4)) & 0x0C3u;
	return (v | (v << 2)) & 0x249u;
}
__device__ __forceinline__ uint32_t ray_cell_key(const float* __restrict__ c) {  // Morton index of the 8^3 cell
	uint32_t k = 0;
#pragma unroll
	for (int d = 0; d < 3; ++d) k |= spread4((uint32_t)clampi((int)(c[d] * 8.0f), 0, 7)) << d;
	return k;
}
// block b, slots [b RS_RPB, (b + 1) RS_RPB), one per thread: per slot with kept samples its cell (first kept sample);
// the block's ray count and round-0 chunk samples per cell (bin RS_BINS: slots without samples) -> hist [2][RS_NB][nblk]
// Split (RaySplit, sp.est != null): bin = cell + RS_BINS for the slots at or past *est (pass B), the no-sample bin is 2 RS_BINS.
__global__ void __launch_bounds__(RS_RPB) k_ray_hist(uint32_t cap, const uint32_t* __restrict__ numsteps, const float* __restrict__ coords,
                                                     uint32_t e1, RaySort rs, RaySplit sp) {
	__shared__ uint32_t h[2][RS_NB2];
	const uint32_t nblk = gridDim.x, blk = blockIdx.x, t = threadIdx.x;
	const uint32_t nbins = sp.est ? 2 * RS_BINS : RS_BINS, NB = nbins + 1;
	const uint32_t est = sp.est ? min(*sp.est, cap) : cap;
	for (uint32_t b = t; b < 2 * RS_NB2; b += RS_RPB) (&h[0][0])[b] = 0u;
	__syncthreads();
	const uint32_t i = blk * RS_RPB + t;
	const bool in = i < cap;
	const uint32_t ns = in ? numsteps[2 * i] : 0u;
	if (ns) {
		const uint32_t key = ray_cell_key(coords + (size_t)numsteps[2 * i + 1] * COORD_W) + (i >= est ? RS_BINS : 0u);
		rs.key[i] = (uint16_t)key;
		atomicAdd(&h[0][key], 1u);
		atomicAdd(&h[1][key], min(ns, e1));
	}
	if (sp.est && in && (!ns || i >= est)) sp.ccount[i] = 0u;  // (pass A's cut: the slots it does not scan count 0)
	const unsigned long long m = __ballot(in && !ns);
	if ((t & 63) == 0 && m) atomicAdd(&h[0][nbins], (uint32_t)__popcll(m));
	__syncthreads();
	for (uint32_t b = t; b < NB; b += RS_RPB) {
		rs.hist[(size_t)b * nblk + blk] = h[0][b];
		rs.hist[((size_t)NB + b) * nblk + blk] = h[1][b];
	}
}
// each slot to its place in the order (LDS cursors from the scanned matrix); a ray with samples also writes its round-0
// chunk [0, min(n, e1)) into its cell's part of the list, each wave's chunks written lane-contiguously. Block 0 writes
// the ordered slot count and the round-0 list length.
// Split: pass A's rays and chunks at perm [0, nA) / list [0, lenA), pass B's at perm [perm_b, +nB) / list [list_b, +lenB);
// the rays without samples are placed nowhere (neither pass scans them; k_ray_hist zeroed their ccount).
__global__ void __launch_bounds__(RS_RPB) k_ray_sort_place(uint32_t cap, const uint32_t* __restrict__ numsteps, uint32_t e1, RaySort rs,
                                                           uint32_t* __restrict__ list, uint32_t* __restrict__ list_len, RaySplit sp) {
	__shared__ uint32_t cur[2][RS_NB2];
	const uint32_t nblk = gridDim.x, blk = blockIdx.x, t = threadIdx.x, lane = t & 63;
	const uint32_t nbins = sp.est ? 2 * RS_BINS : RS_BINS, NB = nbins + 1;
	const size_t n = 2 * (size_t)NB * nblk, h1 = (size_t)NB * nblk;
	const uint32_t h0_total = rs.off[h1];  // every slot (h0 counts them all)
	for (uint32_t b = t; b < NB; b += RS_RPB) {
		cur[0][b] = rs.off[(size_t)b * nblk + blk];
		cur[1][b] = rs.off[h1 + (size_t)b * nblk + blk] - h0_total;
	}
	// split: the start of the B bins (rays, round-0 samples) and of the no-sample bin
	const uint32_t nA = sp.est ? rs.off[(size_t)RS_BINS * nblk] : 0u, nAB = sp.est ? rs.off[(size_t)2 * RS_BINS * nblk] : 0u;
	const uint32_t lenA = sp.est ? rs.off[h1 + (size_t)RS_BINS * nblk] - h0_total : 0u;
	const uint32_t len = (uint32_t)(rs.off[n - 1] + rs.hist[n - 1] - h0_total);
	if (blk == 0 && t == 0) {
		if (sp.est) {
			*rs.n_perm = nA; *list_len = lenA;
			sp.cutw[CW_NB] = nAB - nA; sp.cutw[CW_LENB] = len - lenA;
		} else {
			*rs.n_perm = h0_total; *list_len = len;
		}
	}
	__syncthreads();
	const uint32_t i = blk * RS_RPB + t;
	const bool in = i < cap;
	const uint32_t ns = in ? numsteps[2 * i] : 0u, base = in ? numsteps[2 * i + 1] : 0u;
	uint32_t w = 0, dst = 0;
	if (ns) {
		const uint32_t key = rs.key[i];
		const uint32_t p = atomicAdd(&cur[0][key], 1u);
		const bool b = sp.est && key >= RS_BINS;
		rs.perm[b ? sp.perm_b + (p - nA) : p] = i;
		w = min(ns, e1);
		dst = atomicAdd(&cur[1][key], w);
		if (b) dst = sp.list_b + (dst - lenA);
	}
	const unsigned long long m = __ballot(in && !ns);
	if (m && !sp.est) {
		uint32_t p0 = 0;
		if (lane == 0) p0 = atomicAdd(&cur[0][nbins], (uint32_t)__popcll(m));
		p0 = wave_lane_value(p0, 0);
		if (in && !ns) rs.perm[p0 + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
	}
	// each ray's chunk written by the whole wave, one ray at a time (consecutive lanes, consecutive slots)
	unsigned long long todo = __ballot(w > 0);
	while (todo) {
		const int o = __ffsll(todo) - 1;
		todo &= todo - 1ull;
		const uint32_t w_o = wave_lane_value(w, o), d_o = wave_lane_value(dst, o), s_o = wave_lane_value(base, o);
		for (uint32_t j = lane; j < w_o; j += 64) list[d_o + j] = s_o + j;
	}
}
uint32_t ray_sort_blocks(uint32_t cap) { return std::max<uint32_t>(1, (cap + RS_RPB - 1) / RS_RPB); }
void launch_ray_sort(hipStream_t s, uint32_t cap, const uint32_t* numsteps, const float* coords, uint32_t e1, const RaySort& rs, uint32_t* list,
                     uint32_t* list_len, void* scan_temp, size_t scan_temp_bytes, const RaySplit* split) {
	const uint32_t nblk = ray_sort_blocks(cap);
	const RaySplit sp = split ? *split : RaySplit{nullptr, nullptr, nullptr, 0u, 0u};
	if (sp.est && (!sp.ccount || !sp.cutw)) throw std::runtime_error("launch_ray_sort: the split needs ccount and the cut words");
	dbg_lds_gate(s);
	k_ray_hist<<<nblk, RS_RPB, 0, s>>>(cap, numsteps, coords, e1, rs, sp);
	launch_exclusive_scan(s, scan_temp, scan_temp_bytes, rs.hist, rs.off, 2 * (sp.est ? RS_NB2 : RS_NB) * nblk);
	dbg_lds_gate(s);
	k_ray_sort_place<<<nblk, RS_RPB, 0, s>>>(cap, numsteps, e1, rs, list, list_len, sp);
}

// Development statistic: per ray, march_step calls and skip-loop additions of the march
// (SIMT-efficiency analysis; neus_debug_march_stats).
__global__ void k_march_stats(uint32_t n_rays, const float* __restrict__ rays, const float* __restrict__ tstart, const uint32_t* __restrict__ lin,
                              DevDataset ds, const uint8_t* __restrict__ bf, uint32_t* __restrict__ out) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_rays) return;
	uint32_t outer = 0, inner = 0, n = 0;
	float t = tstart[i];
	if (t >= 0.f) {
		MarchRay mr;
		load_march_ray(rays, i, mr, ds.motion.on != 0);
		while (n < NERF_STEPS) {
			float dt, pos[3];
			const float t0 = t;
			const int k = march_step<true>(ds, bf, lin, mr, t, dt, pos);
			++outer;
			if (k == 0) break;
			if (k == 1) { ++n; t += dt; }
			else inner += (uint32_t)((t - t0) / MIN_CONE_STEPSIZE + 0.5f);
		}
	}
	out[3 * i] = outer; out[3 * i + 1] = inner; out[3 * i + 2] = n;
}


// ---------------------------------------------------------------- loss, restructured for gfx950
// The reference walks each ray's samples serially in one thread, twice (composite, then gradient).
// Here only the transmittance recurrence stays serial, over 20 B per sample; everything pointwise
// runs one thread per sample with coalesced loads/stores:
//   A  k_loss_alpha     (per pre-compaction sample): alpha, sigmoid(rgb), eikonal term
//   B  k_loss_scan_ray  (per ray, serial): T, cn (T < 1e-4 cut), rgb_ray, weight_sum; per-sample
//                       prefix {T_before, rgb prefix incl. the sample}, eikonal prefix
//      exclusive scan of cn -> compacted base
//   C  k_loss_ray       (per ray): target pixel + background (same pcg32 stream as the sampler),
//                       Huber loss, mask term, comp = min(cap - base, cn), numsteps := (comp, base)
//   D  k_loss_grad      (per pre-compaction sample): dL/doutput of the compacted samples
// The float operation sequence of every quantity is the reference's (and the oracle's), so the
// compaction and the gradients stay bit-identical to the serial formulation.


// n = min(*n_ptr, cap) samples; with idx, work item j is sample idx[j] (a progressive-inference round)
__global__ void __launch_bounds__(256) k_loss_alpha(uint32_t cap, const uint32_t* __restrict__ n_ptr, const uint32_t* __restrict__ idx,
                                                    const float* __restrict__ coords, const half_t* __restrict__ net_out, float cos_anneal,
                                                    float4* __restrict__ sa, float* __restrict__ ekt, uint32_t* __restrict__ n_long,
                                                    bool dt_const) {
	if (n_long && blockIdx.x == 0 && threadIdx.x == 0) *n_long = 0u;  // the transmittance scan's long-ray list (next kernel)
	const uint32_t n = min(*n_ptr, cap);
	// cone angle 0: k_march_write stored warp_dt(MIN_CONE_STEPSIZE) in every record; the same round trip here
	// (bit-identical) saves touching the 28-B records' lines for one float each
	const float dt0 = unwarp_dt(warp_dt(MIN_CONE_STEPSIZE));
	for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
		const uint32_t s = idx ? idx[j] : j;
		half_t lo[16]; load_out(net_out, s, lo);
		loss_alpha_sample(lo, dt_const ? dt0 : unwarp_dt(coords[(size_t)s * COORD_W + 3]), cos_anneal, sa, ekt, s);
	}
}

// Transmittance recurrence state of a ray (reference order: w = a T; rgb += w c; ws += w; ek += e; T *= 1 - a).
struct RecState { float T, r0, r1, r2, ek; };
constexpr uint32_t SCAN_CK = 8;  // checkpoint stride of the stored scan state (in global sample index)
constexpr uint32_t LONG_RAY = 32; // rays with more samples go to k_loss_scan_list

// Replays the recurrence from the last stored checkpoint at or before sample s (or the ray start)
// through sample s; returns T before s in T_before, and the state after s.
__device__ __forceinline__ RecState scan_replay(uint32_t base, uint32_t s, const float4* __restrict__ sa, const float* __restrict__ ekt,
                                                 const float4* __restrict__ ck4, const float* __restrict__ cke, float& T_before) {
	const uint32_t g = s & ~(SCAN_CK - 1);
	RecState st{1.f, 0.f, 0.f, 0.f, 0.f};
	uint32_t k = base;
	if (g > base) { const float4 c = ck4[g / SCAN_CK]; st = {c.x, c.y, c.z, c.w, cke[g / SCAN_CK]}; k = g; }
	for (; k <= s; ++k) {
		const float4 q = sa[k];
		const float w = q.x * st.T;
		st.r0 += w * q.y; st.r1 += w * q.z; st.r2 += w * q.w;
		st.ek += ekt[k];
		if (k == s) T_before = st.T;
		st.T *= (1.f - q.x);
	}
	return st;
}

// The recurrence state a ray carries between progressive-inference rounds (cn = samples composited so far).
struct RayScan { float T, r0, r1, r2, ws, ek; uint32_t cn; };

// One thread per ray over all its samples, software-pipelined: the next U samples' {alpha, rgb} and eikonal terms
// are in flight while the current U go through the serial recurrence. Loads use clamped indices so they issue
// unconditionally, ahead of the data-dependent exit. Consecutive rays go to consecutive BLOCKS: the rays that carry
// samples are a prefix of the ray range (few and long early in training), and this spreads them over all CUs. The
// state is stored only every SCAN_CK samples (scan_replay rebuilds the rest exactly), which keeps the scattered
// per-lane stores off the critical path. 16 samples per group: early in training a few hundred rays carry hundreds
// of samples each and the kernel time is their load-latency chain.
// Rays with more than LONG_RAY samples are deferred to the long list (when given) for k_loss_scan_list.
template <bool STORE = true>
__global__ void __launch_bounds__(256) k_loss_scan_ray(uint32_t cap_rays, const uint32_t* __restrict__ numsteps, const float4* __restrict__ sa,
                                                       const float* __restrict__ ekt, float4* __restrict__ ck4, float* __restrict__ cke,
                                                       uint32_t* __restrict__ ccount, float4* __restrict__ racc, float* __restrict__ rT,
                                                       uint32_t* __restrict__ long_rays, uint32_t* __restrict__ n_long) {
	const uint32_t stride = gridDim.x * blockDim.x;
	for (uint32_t k = threadIdx.x * gridDim.x + blockIdx.x; k < ((cap_rays + stride - 1) / stride) * stride; k += stride) {
		const uint32_t i = k;
		if (i >= cap_rays) continue;
		const uint32_t ns = numsteps[2 * i], base = numsteps[2 * i + 1];
		if (long_rays && ns > LONG_RAY) { long_rays[atomicAdd(n_long, 1u)] = i; continue; }
		uint32_t cn = 0;
		float T = 1.f, r0 = 0.f, r1 = 0.f, r2 = 0.f, ws = 0.f, ek = 0.f;
		if (ns > 0) {
			constexpr uint32_t U = 16;
			const uint32_t last = base + ns - 1;
			float4 qn[U]; float en[U];
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) { const uint32_t s = min(base + u, last); qn[u] = sa[s]; en[u] = ekt[s]; }
			bool done = false;
			for (uint32_t c = 0; c < ns && !done; c += U) {
				float4 q[U]; float e[U];
#pragma unroll
				for (uint32_t u = 0; u < U; ++u) { q[u] = qn[u]; e[u] = en[u]; }
				if (c + U < ns) {
#pragma unroll
					for (uint32_t u = 0; u < U; ++u) { const uint32_t s = min(base + c + U + u, last); qn[u] = sa[s]; en[u] = ekt[s]; }
				}
#pragma unroll
				for (uint32_t u = 0; u < U; ++u) {
					if (c + u >= ns || T < 1e-4f) { done = true; break; }
					const uint32_t s = base + c + u;
					if (STORE && (s & (SCAN_CK - 1)) == 0) { ck4[s / SCAN_CK] = make_float4(T, r0, r1, r2); cke[s / SCAN_CK] = ek; }
					const float w = q[u].x * T;
					r0 += w * q[u].y; r1 += w * q[u].z; r2 += w * q[u].w;
					ws += w;
					ek += e[u];
					T *= (1.f - q[u].x);
					++cn;
				}
			}
		}
		ccount[i] = cn;
		racc[i] = make_float4(r0, r1, r2, ws);
		rT[i] = T;
	}
}

// The long rays (early in training a few thousand rays carry hundreds of samples each), 64 to a wave, one lane per
// ray as k_loss_scan_ray but with the loads made coalesced: per 16-sample group, 16 lanes fetch one ray's 16
// samples (256 B contiguous), 4 rays per load instruction, staged through LDS (row stride 17 float4: conflict-free
// reads), the next groups' fetches in flight while the current one runs through the recurrence. One lane per ray
// loading its own samples put 64 different lines behind every load instruction. Same float operation sequence, so
// the results are k_loss_scan_ray's bits.
__global__ void __launch_bounds__(64) k_loss_scan_list(const uint32_t* __restrict__ numsteps, const float4* __restrict__ sa,
                                                       const float* __restrict__ ekt, float4* __restrict__ ck4, float* __restrict__ cke,
                                                       uint32_t* __restrict__ ccount, float4* __restrict__ racc, float* __restrict__ rT,
                                                       const uint32_t* __restrict__ long_rays, const uint32_t* __restrict__ n_long) {
	constexpr uint32_t U = 16, PAD = U + 1;  // two groups in flight (slots A and B)
	typedef float f4v __attribute__((ext_vector_type(4)));  // (HIP's float4 struct arrays are not kept in registers here)
	__shared__ f4v s_q[64 * PAD];
	__shared__ float s_e[64 * PAD];
	const uint32_t lane = threadIdx.x, sub = lane >> 4, el = lane & 15;
	const uint32_t nl = *n_long;
	const char* sab = (const char*)sa;
	const char* ekb = (const char*)ekt;
	for (uint32_t w0 = blockIdx.x * 64; w0 < nl; w0 += gridDim.x * 64) {
		const uint32_t k = w0 + lane;
		const uint32_t i = k < nl ? long_rays[k] : 0u;
		const uint32_t ns = k < nl ? numsteps[2 * i] : 0u, base = k < nl ? numsteps[2 * i + 1] : 0u;
		// loader view: load instruction j fetches element el of ray 4 j + sub; past the ray's end it re-reads the ray's
		// last sample (unconditional loads, 32-bit offsets from the uniform base; the values are never used)
		uint32_t lb[U], ll[U];
#pragma unroll
		for (uint32_t j = 0; j < U; ++j) {
			lb[j] = __shfl(base, 4 * j + sub);
			const uint32_t n = __shfl(ns, 4 * j + sub);
			ll[j] = lb[j] + (n ? n - 1u : 0u);
		}
		auto fetch = [&](f4v (&q)[U], float (&e)[U], uint32_t c) {
#pragma unroll
			for (uint32_t j = 0; j < U; ++j) {
				const uint32_t g = min(lb[j] + c + el, ll[j]);
				q[j] = *(const f4v*)(sab + (g << 4));
				e[j] = *(const float*)(ekb + (g << 2));
			}
		};
		uint32_t cn = 0;
		float T = 1.f, r0 = 0.f, r1 = 0.f, r2 = 0.f, ws = 0.f, ek = 0.f;
		bool live = ns > 0;  // the recurrence still runs (the reference's loop: j < numsteps and T >= 1e-4)
		// one group: stage slot (q, e) = group c through LDS, refill the slot with group c + 2 U, run the recurrence
		auto group = [&](f4v (&qs)[U], float (&es)[U], uint32_t c) {
			__builtin_amdgcn_wave_barrier();
#pragma unroll
			for (uint32_t j = 0; j < U; ++j) { s_q[(4 * j + sub) * PAD + el] = qs[j]; s_e[(4 * j + sub) * PAD + el] = es[j]; }
			__builtin_amdgcn_wave_barrier();
			fetch(qs, es, c + 2 * U);
			f4v q[U]; float e[U];
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) { q[u] = s_q[lane * PAD + u]; e[u] = s_e[lane * PAD + u]; }
			// branch-free: the state advances only while live (same operations, in the same order, on those samples)
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) {
				live = live && (c + u < ns) && !(T < 1e-4f);
				const uint32_t s = base + c + u;
				if (live && (s & (SCAN_CK - 1)) == 0) { ck4[s / SCAN_CK] = make_float4(T, r0, r1, r2); cke[s / SCAN_CK] = ek; }
				const float w = q[u][0] * T;
				const float n0 = r0 + w * q[u][1], n1 = r1 + w * q[u][2], n2 = r2 + w * q[u][3];
				const float nws = ws + w, nek = ek + e[u], nT = T * (1.f - q[u][0]);
				r0 = live ? n0 : r0; r1 = live ? n1 : r1; r2 = live ? n2 : r2;
				ws = live ? nws : ws; ek = live ? nek : ek; T = live ? nT : T;
				cn += live ? 1u : 0u;
			}
			__builtin_amdgcn_wave_barrier();
		};
		f4v qa[U], qb[U]; float ea[U], eb[U];
		fetch(qa, ea, 0);
		fetch(qb, eb, U);
		for (uint32_t c = 0;; c += 2 * U) {
			if (__ballot(live && c < ns) == 0) break;
			group(qa, ea, c);
			if (__ballot(live && c + U < ns) == 0) break;
			group(qb, eb, c + U);
		}
		if (k < nl) {
			ccount[i] = cn;
			racc[i] = make_float4(r0, r1, r2, ws);
			rT[i] = T;
		}
	}
}

// ---------------------------------------------------------------- progressive (cut-off-aware) inference
// Late in training most of a long ray's samples lie behind the surface, past the T < 1e-4 cut, and the loss never
// reads their network outputs (23-45 % of the kept samples are composited at steps 800-2000). The
// step then evaluates the network in rounds of per-ray sample chunks [e_k, e_k+1): round k infers only the chunk of
// the rays whose recurrence is still open after round k-1. Every composited sample is evaluated exactly as in one
// pass and the recurrence runs over the same samples in the same order, so the results are bit-identical; only
// samples past the cut are never evaluated. The work lists hold sample indices; their order is immaterial (each
// work item writes its own sample's slots).

// Round k's recurrence over [e0, e1) of each ray still open (all rays with samples when e0 == 0), continuing from
// the stored state; rays that stay open append their next chunk [e1, min(ns, e2)) to the next round's list and
// themselves to the next round's ray list (rays_out), so a later round visits only the rays still open (rays_in,
// *n_rays_in of them) instead of sweeping every ray slot for its stored state.
// 64 rays to a one-wave block (consecutive slots in round 0, the open-ray list after it), one lane per ray, the loads
// made coalesced as in k_loss_scan_list: per
// 16-sample group 16 lanes fetch one ray's 16 samples (4 rays per load instruction), staged through LDS, the next
// group's fetches in flight while the current one runs through the recurrence (one lane loading its own ray's samples
// put 64 lines behind every load instruction). The appends are one atomic per wave and a cooperative write of the
// wave's concatenated chunks (consecutive lanes, consecutive list slots). Same float operation sequence per ray, so
// the state is bitwise the one-thread-per-ray loop's.
// groups in flight: 1 (130 VGPRs, 3 waves per SIMD) measured 2 us/step faster than 2 (170 VGPRs, 2 waves), 1 at 4 waves
// per SIMD (5 spilled dwords) slower (profiles/r05nb_scan_groups_ab.txt)
#ifndef NEUS_SCAN_NB
#define NEUS_SCAN_NB 1
#endif
#ifndef NEUS_SCAN_WPE
#define NEUS_SCAN_WPE 0
#endif
#if NEUS_SCAN_WPE
#define SCAN_OCC __attribute__((amdgpu_waves_per_eu(NEUS_SCAN_WPE, NEUS_SCAN_WPE)))
#else
#define SCAN_OCC
#endif
__global__ void __launch_bounds__(64) SCAN_OCC k_loss_scan_chunk(uint32_t cap_rays, const uint32_t* __restrict__ numsteps, const float4* __restrict__ sa,
                                                        const float* __restrict__ ekt, float4* __restrict__ ck4, float* __restrict__ cke,
                                                        uint32_t* __restrict__ ccount, float4* __restrict__ racc, float* __restrict__ rT,
                                                        float* __restrict__ rek, uint32_t e0, uint32_t e1, uint32_t e2,
                                                        uint32_t* __restrict__ list, uint32_t* __restrict__ next_counter,
                                                        const uint32_t* __restrict__ rays_in, const uint32_t* __restrict__ n_rays_in,
                                                        uint32_t* __restrict__ rays_out, uint32_t* __restrict__ n_rays_out) {
	// U samples per ray and group: U lanes load U consecutive samples of one ray (64 / U rays per load instruction),
	// transposed through LDS to one ray per lane. U = 8 (was 16): half the LDS and registers per wave, so twice the
	// waves per CU hide the per-ray state loads. NB groups are in flight, the next group's fetch issued before the
	// current one runs through the recurrence (a 4-deep fetch in the later rounds measured the same as 2:
	// profiles/r05q_scan_ab.txt; 1 is the default, above)
	constexpr uint32_t U = 8, PAD = U + 1, RPI = 64 / U, NB = NEUS_SCAN_NB;
	typedef float f4v __attribute__((ext_vector_type(4)));
	__shared__ f4v s_q[64 * PAD];
	__shared__ float s_e[64 * PAD];
	const uint32_t lane = threadIdx.x, sub = lane / U, el = lane % U;
	const char* sab = (const char*)sa;
	const char* ekb = (const char*)ekt;
	const uint32_t n_slots = rays_in ? min(*n_rays_in, cap_rays) : cap_rays;
	for (uint32_t w0 = blockIdx.x * 64; w0 < n_slots; w0 += gridDim.x * 64) {
		const bool inr = w0 + lane < n_slots;
		const uint32_t i = rays_in ? (inr ? rays_in[w0 + lane] : 0u) : w0 + lane;
		const uint32_t ns = inr ? numsteps[2 * i] : 0u, base = inr ? numsteps[2 * i + 1] : 0u;
		RayScan S{1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0u};
		bool open = inr && (e0 == 0 || ns > 0);  // this round runs (and stores) the ray's state
		if (e0 > 0 && inr) {
			// the stored state, loaded together with numsteps (one round trip; read for closed rays too)
			const uint32_t cn = ccount[i];
			const float T = rT[i];
			const float4 a = racc[i];
			const float ek = rek[i];
			S.cn = cn;
			if (!open || cn != e0 || e0 >= ns || T < 1e-4f) open = false;  // closed in an earlier round (or no samples)
			else { S.T = T; S.r0 = a.x; S.r1 = a.y; S.r2 = a.z; S.ws = a.w; S.ek = ek; }
		}
		const uint32_t to = min(ns, e1);
		bool live = open && to > e0;
		const uint32_t g0 = live ? base + e0 : 0u, gl = live ? base + to - 1u : 0u;  // the round's samples [g0, gl]
		uint32_t lb[U], ll[U];
#pragma unroll
		for (uint32_t j = 0; j < U; ++j) { lb[j] = __shfl(g0, RPI * j + sub); ll[j] = __shfl(gl, RPI * j + sub); }
		auto fetch = [&](f4v (&q)[U], float (&e)[U], uint32_t c) {
#pragma unroll
			for (uint32_t j = 0; j < U; ++j) {
				const uint32_t g = min(lb[j] + c + el, ll[j]);
				q[j] = *(const f4v*)(sab + ((size_t)g << 4));
				e[j] = *(const float*)(ekb + ((size_t)g << 2));
			}
		};
		auto group = [&](f4v (&qs)[U], float (&es)[U], uint32_t c) {
			__builtin_amdgcn_wave_barrier();
#pragma unroll
			for (uint32_t j = 0; j < U; ++j) { s_q[(RPI * j + sub) * PAD + el] = qs[j]; s_e[(RPI * j + sub) * PAD + el] = es[j]; }
			__builtin_amdgcn_wave_barrier();
			fetch(qs, es, c + NB * U);
			f4v q[U]; float e[U];
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) { q[u] = s_q[lane * PAD + u]; e[u] = s_e[lane * PAD + u]; }
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) {
				live = live && (e0 + c + u < to) && !(S.T < 1e-4f);
				const uint32_t s = base + e0 + c + u;
				if (live && (s & (SCAN_CK - 1)) == 0) { ck4[s / SCAN_CK] = make_float4(S.T, S.r0, S.r1, S.r2); cke[s / SCAN_CK] = S.ek; }
				const float w = q[u][0] * S.T;
				const float n0 = S.r0 + w * q[u][1], n1 = S.r1 + w * q[u][2], n2 = S.r2 + w * q[u][3];
				const float nws = S.ws + w, nek = S.ek + e[u], nT = S.T * (1.f - q[u][0]);
				S.r0 = live ? n0 : S.r0; S.r1 = live ? n1 : S.r1; S.r2 = live ? n2 : S.r2;
				S.ws = live ? nws : S.ws; S.ek = live ? nek : S.ek; S.T = live ? nT : S.T;
				S.cn += live ? 1u : 0u;
			}
			__builtin_amdgcn_wave_barrier();
		};
		if (__ballot(live)) {
			f4v qs[NB][U]; float es[NB][U];
#pragma unroll
			for (uint32_t bf = 0; bf < NB; ++bf) fetch(qs[bf], es[bf], bf * U);
			for (uint32_t c = 0;; c += NB * U) {
				bool more = true;
#pragma unroll
				for (uint32_t bf = 0; bf < NB; ++bf) {
					if (more && __ballot(live && e0 + c + bf * U < to) == 0) more = false;
					if (more) group(qs[bf], es[bf], c + bf * U);
				}
				if (!more) break;
			}
		}
		if (open) {
			ccount[i] = S.cn;
			racc[i] = make_float4(S.r0, S.r1, S.r2, S.ws);
			rT[i] = S.T;
			rek[i] = S.ek;
		}
		if (list || rays_out) {
			// the next round's chunk of every ray still open: one reservation per wave, written lane-contiguously (no list:
			// the open rays only - k_prog_next builds the next list from them, past the compaction cut)
			const uint32_t m = (open && S.cn == e1 && e1 < ns && S.T >= 1e-4f) ? min(ns, e2) - e1 : 0u;
			const uint32_t incl = wave_incl_sum(m);
			const uint32_t total = wave_lane_value(incl, 63);
			if (total) {
				if (list) {
					uint32_t p0 = 0;
					if (lane == 0) p0 = atomicAdd(next_counter, total);
					p0 = wave_lane_value(p0, 0);
					// each open ray's next chunk written by the whole wave, one ray at a time (consecutive lanes, consecutive
					// slots: the same list as each lane writing its own, in the same positions)
					const uint32_t pre = incl - m, src = base + e1;
					unsigned long long todo = __ballot(m > 0);
					while (todo) {
						const int o = __ffsll(todo) - 1;
						todo &= todo - 1ull;
						const uint32_t m_o = wave_lane_value(m, o), p_o = p0 + wave_lane_value(pre, o), s_o = wave_lane_value(src, o);
						for (uint32_t j = lane; j < m_o; j += 64) list[p_o + j] = s_o + j;
					}
				}
				if (rays_out) {  // the open rays, one reservation per wave
					const unsigned long long mk = __ballot(m > 0);
					uint32_t q0 = 0;
					if (lane == 0) q0 = atomicAdd(n_rays_out, (uint32_t)__popcll(mk));
					q0 = wave_lane_value(q0, 0);
					if (m > 0) rays_out[q0 + (uint32_t)__popcll(mk & ((1ull << lane) - 1ull))] = i;
				}
			}
		}
	}
}

// ---- the compaction cut of the progressive rounds (fixed rays per batch; NeusTestbed::prog_cut)
// The loss compacts the composited samples in ray-slot order and keeps the first `batch` (compute_loss_kernel_train_nerf,
// testbed_nerf.cu:1682-1688: a ray whose compacted base is past the batch contributes nothing). After a round, ccount[i] is
// the ray's composited count so far - exact if it is closed, a lower bound if it is open - and counts only grow in later
// rounds. So once the inclusive prefix of ccount over the slots reaches the batch at slot c, every slot after c has a
// compaction base of at least the batch whatever its remaining samples hold: the later rounds skip those rays. `excl` is
// the exclusive scan of ccount; exactly one thread writes the cut (the crossing slot, or cap_rays when the prefix never
// reaches the batch).
// mode 0 (after pass A of a split round 0, the slots it did not scan counting 0): when the prefix reaches the batch in pass
// A's slots, pass B has nothing to do (its counts 0), else pass B runs on everything the sort gave it. mode 1 (the cut the
// later rounds use): also the next step's split estimate (the cut + 1/4 + 1024, whole waves) and pass B's samples added to
// the round-0 evaluated count.
__global__ void __launch_bounds__(256) k_prog_cut(uint32_t cap_rays, const uint32_t* __restrict__ ccount, const uint32_t* __restrict__ excl,
                                                  uint32_t batch, uint32_t* __restrict__ cutw, int mode, uint32_t* __restrict__ eval0,
                                                  uint32_t* __restrict__ abort_if_none) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= cap_rays) return;
	const uint32_t e = excl[i], incl = e + ccount[i];
	const bool cross = e < batch && incl >= batch, none = i == cap_rays - 1 && incl < batch;
	if (!cross && !none) return;
	const uint32_t c = cross ? i : cap_rays;
	if (mode == 0) {
		cutw[CW_CUT_A] = c;
		cutw[CW_LENB_EFF] = cross ? 0u : cutw[CW_LENB];
		cutw[CW_NB_EFF] = cross ? 0u : cutw[CW_NB];
	} else {
		cutw[CW_CUT] = c;
		cutw[CW_EST] = min(cap_rays, (c + c / 4u + 1024u + 63u) & ~63u);
		if (eval0) *eval0 += cutw[CW_LENB_EFF];
		// (a split round 0 whose pass B was not run - a cut march's step: pass A's slots must reach the batch, or the step
		// is re-run; the march cut's witness word)
		if (abort_if_none && !cross) *abort_if_none = 1u;
	}
}
// The exclusive scan of ccount (k_scan_lookback's single pass) with k_prog_cut fused into its epilogue: the thread holding
// the crossing slot (or the last slot, when the prefix never reaches the batch) writes the cut words. One launch instead
// of two on the step's critical path; the scan and the words are those of the pair.
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_prog_cut(const uint32_t* __restrict__ ccount, uint32_t* __restrict__ excl, uint32_t n,
                                                                ScanState* __restrict__ ss, uint32_t tag, uint32_t batch, uint32_t* __restrict__ cutw,
                                                                int mode, uint32_t* __restrict__ eval0, uint32_t* __restrict__ abort_if_none) {
	__shared__ uint32_t s_prefix, s_wsum[SCAN_THREADS / 64];
	const ScanTile tl = scan_tile(tag);
	const size_t b0 = (size_t)tl.tile * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
	uint32_t v[SCAN_ITEMS];
	scan_load16(ccount, b0, n, true, v);
	uint32_t tsum = 0;
#pragma unroll
	for (int k = 0; k < (int)SCAN_ITEMS; ++k) tsum += v[k];
	uint32_t agg;
	const uint32_t texcl = scan_block(tsum, s_wsum, agg);
	if (threadIdx.x < 64) {
		const uint32_t pre = scan_lookback(ss, 0, tl, agg);
		if (threadIdx.x == 0) s_prefix = pre;
	}
	__syncthreads();
	uint32_t run = s_prefix + texcl;
#pragma unroll
	for (int k = 0; k < (int)SCAN_ITEMS; ++k) {
		const uint32_t x = v[k], i = (uint32_t)b0 + (uint32_t)k;
		v[k] = run;
		const bool cross = run < batch && run + x >= batch, none = i == n - 1 && run + x < batch;
		run += x;
		if ((cross || none) && i < n) {
			const uint32_t c = cross ? i : n;
			if (mode == 0) {
				cutw[CW_CUT_A] = c;
				cutw[CW_LENB_EFF] = cross ? 0u : cutw[CW_LENB];
				cutw[CW_NB_EFF] = cross ? 0u : cutw[CW_NB];
			} else {
				cutw[CW_CUT] = c;
				cutw[CW_EST] = min(n, (c + c / 4u + 1024u + 63u) & ~63u);
				if (eval0) *eval0 += cutw[CW_LENB_EFF];
				if (abort_if_none && !cross) *abort_if_none = 1u;
			}
		}
	}
	scan_store16(excl, b0, n, true, v);
}
void launch_scan_prog_cut(hipStream_t s, void* scan_temp, const uint32_t* ccount, uint32_t* excl, uint32_t n, uint32_t batch, uint32_t* cutw, int mode,
                          uint32_t* eval0, uint32_t* abort_if_none) {
	const uint32_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
	if (n == 0 || tiles > SCAN_MAX_TILES || (((uintptr_t)ccount | (uintptr_t)excl) & 15u))
		throw std::runtime_error("launch_scan_prog_cut: 1 .. SCAN_MAX_TILES tiles of 16-B aligned counts");
	dbg_lds_gate(s);
	k_scan_prog_cut<<<tiles, SCAN_THREADS, 0, s>>>(ccount, excl, n, (ScanState*)scan_temp, scan_next_tag(scan_temp), batch, cutw, mode, eval0,
	                                               abort_if_none);
}

// The next round's work from the rays still open (rays_in: the scan's rays_out), the rays at or before the cut only: the
// ray to rays_out and its next chunk [e1, min(ns, e2)) to the sample list; one reservation per wave for each (the list
// order differs from the scan's own append, which changes no result: every sample and every ray is independent).
__global__ void __launch_bounds__(256) k_prog_next(const uint32_t* __restrict__ rays_in, const uint32_t* __restrict__ n_in,
                                                   const uint32_t* __restrict__ numsteps, const uint32_t* __restrict__ cut, uint32_t e1, uint32_t e2,
                                                   uint32_t* __restrict__ list, uint32_t* __restrict__ list_counter,
                                                   uint32_t* __restrict__ rays_out, uint32_t* __restrict__ n_out) {
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t n = *n_in, c = *cut, n64 = (n + 63u) & ~63u;
	for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n64; k += gridDim.x * blockDim.x) {
		const uint32_t i = k < n ? rays_in[k] : 0u;
		const uint32_t ns = k < n ? numsteps[2 * i] : 0u, base = k < n ? numsteps[2 * i + 1] : 0u;
		const uint32_t m = (k < n && i <= c && ns > e1) ? min(ns, e2) - e1 : 0u;
		const uint32_t incl = wave_incl_sum(m);
		const uint32_t total = wave_lane_value(incl, 63);
		if (!total) continue;
		uint32_t p0 = 0;
		if (lane == 0) p0 = atomicAdd(list_counter, total);
		p0 = wave_lane_value(p0, 0);
		const uint32_t pre = incl - m, src = base + e1;
		unsigned long long todo = __ballot(m > 0);
		while (todo) {
			const int o = __ffsll(todo) - 1;
			todo &= todo - 1ull;
			const uint32_t m_o = wave_lane_value(m, o), p_o = p0 + wave_lane_value(pre, o), s_o = wave_lane_value(src, o);
			for (uint32_t j = lane; j < m_o; j += 64) list[p_o + j] = s_o + j;
		}
		const unsigned long long mk = __ballot(m > 0);
		uint32_t q0 = 0;
		if (lane == 0) q0 = atomicAdd(n_out, (uint32_t)__popcll(mk));
		q0 = wave_lane_value(q0, 0);
		if (m > 0) rays_out[q0 + (uint32_t)__popcll(mk & ((1ull << lane) - 1ull))] = i;
	}
}

// One thread per ray. The grid-stride loop runs to cap_rays rounded up to 64, so a wave's lanes run it together and
// fill the sample -> ray map of their 64 consecutive rays cooperatively at the end of each iteration: each ray's range
// is written by consecutive lanes (coalesced stores) instead of every lane storing its own range one element per
// instruction (64 scattered lines per store). Lanes past cap_rays (any ray count: neus_loss_compact takes 1..2^18)
// take part in the fill with an empty range.
__global__ void __launch_bounds__(256) k_loss_ray(uint32_t cap_rays, StepState* __restrict__ st, DPInfo dp, DevDataset ds, LossParams lp,
                                                  uint32_t* __restrict__ numsteps, const uint32_t* __restrict__ ccount,
                                                  const uint32_t* __restrict__ cbase, const float4* __restrict__ sa, const float* __restrict__ ekt,
                                                  const float4* __restrict__ ck4, const float* __restrict__ cke,
                                                  float4* __restrict__ racc, const float* __restrict__ rT, float4* __restrict__ rgr,
                                                  float* __restrict__ loss_out, float* __restrict__ ek_out, float* __restrict__ mask_out,
                                                  uint32_t* __restrict__ cmap) {
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t R = st->rays_per_batch;
	const uint32_t n_rays_global = R * dp.world, n_rays_total = st->n_rays_total;
	const uint32_t cap64 = (cap_rays + 63u) & ~63u;
	// the march cut's witness: the next step's abort word cleared; this step's set when (a) the march was cut
	// and its slots do not fill the batch (the full march's later rays would have), or (b) a contributing ray ends past
	// mi_lb (the last step's march was cut, so the reference's cap on this step's samples is known only to be at least
	// mi_lb: a contributing ray past it might not have been kept there)
	const uint32_t mi_lb = st->mi_lb;
	if (lp.abort_w && blockIdx.x == 0 && threadIdx.x == 0) lp.abort_w[lp.abort_slot ^ 1u] = 0u;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap64; i += gridDim.x * blockDim.x) {
		uint32_t comp = 0, cb = 0;
		if (i < cap_rays) {
			const uint32_t ns = numsteps[2 * i], base = numsteps[2 * i + 1];
			const uint32_t cn = ccount[i];
			cb = cbase[i];
			if (i == cap_rays - 1) {
				if (lp.abort_w && st->march_cut && cb + cn < lp.max_compacted) lp.abort_w[lp.abort_slot] = 1u;
				st->compacted_counter = cb + cn;
				st->compacted_global = cb + cn;                     // (all-reduced by the data-parallel exchange)
				st->rays_ws_global = st->n_rays_with_samples;
				st->n_train = min(cb + cn, lp.max_compacted) ? lp.max_compacted : 0u;  // the training batch (k_rollover sets it too)
			}
			loss_out[i] = 0.f; ek_out[i] = 0.f; mask_out[i] = 0.f;
			if (ns == 0) {
				numsteps[2 * i] = 0; numsteps[2 * i + 1] = cb;
			} else {
				const float4 acc = racc[i];
				float rgb_ray[3] = {acc.x, acc.y, acc.z}, weight_sum = acc.w;
				const float T = rT[i];
				// target pixel and background (same RNG stream as the sampler; testbed_nerf.cu:1632-1660)
				const uint32_t ig = dp.rank * R + i;
				pcg32 rng(lp.rng_state, lp.rng_inc);
				pcg_advance(rng, (uint64_t)(uint32_t)(ig * N_MAX_RANDOM_SAMPLES_PER_RAY), lp.jt);
				const uint32_t img = image_idx(ig, n_rays_global, n_rays_total, ds.n_images);
				const int rx = ds.res[2 * img], ry = ds.res[2 * img + 1];
				float xx, yy; random_image_pos(rng, rx, ry, xx, yy);
				float bg[3];
				if (ds.target.fixed_bg) { bg[0] = ds.target.bg[0]; bg[1] = ds.target.bg[1]; bg[2] = ds.target.bg[2]; }
				else { bg[0] = rng.next_float(); bg[1] = rng.next_float(); bg[2] = rng.next_float(); }
	#pragma unroll
				for (int k = 0; k < 3; ++k) bg[k] = srgb_to_linear(bg[k]);
				float tex[4]; read_rgba(ds, img, xx, yy, tex);
				float target[3];
				const uint32_t tmode = ds.target.mode;
	#pragma unroll
				for (int k = 0; k < 3; ++k) {
					if (tmode != 1) {  // Linear colour space (sRGB targets unless linear_colors) (:1658-1663)
						target[k] = 1.0f * tex[k] + (1.0f - tex[3]) * bg[k];
						if (tmode == 0) { target[k] = linear_to_srgb(target[k]); bg[k] = linear_to_srgb(bg[k]); }
					} else {           // SRGB colour space (:1664-1670)
						bg[k] = linear_to_srgb(bg[k]);
						target[k] = tex[3] > 0.0f ? linear_to_srgb(1.0f * tex[k] / tex[3]) * tex[3] + (1.0f - tex[3]) * bg[k] : bg[k];
					}
				}
				if (cn == ns) {
	#pragma unroll
					for (int k = 0; k < 3; ++k) rgb_ray[k] += T * bg[k];
				}
				comp = min(lp.max_compacted - min(lp.max_compacted, cb), cn);
				if (lp.abort_w && mi_lb && comp > 0 && base + ns > mi_lb) lp.abort_w[lp.abort_slot] = 1u;
				numsteps[2 * i] = comp; numsteps[2 * i + 1] = cb;
				if (comp > 0) {
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
					float Tb;
					const RecState sc = scan_replay(base, base + comp - 1, sa, ekt, ck4, cke, Tb);
					ek_out[i] = sc.ek / ((float)comp * (float)n_rays_global);
					rgr[i] = make_float4(lgrad[0], lgrad[1], lgrad[2], gws * (1 - weight_sum));
					racc[i] = make_float4(rgb_ray[0], rgb_ray[1], rgb_ray[2], 0.f);
				}
			}
		}
		// cmap[cb + j] = i for j < comp, by the whole wave: one lane's range at a time (wave-uniform loop over the lanes
		// that have one), written by consecutive lanes to consecutive slots
		unsigned long long todo = __ballot(comp > 0);
		const uint32_t i0 = i - lane;
		while (todo) {
			const int o = __ffsll(todo) - 1;
			todo &= todo - 1ull;
			const uint32_t c_o = wave_lane_value(comp, o), d_o = wave_lane_value(cb, o);
			for (uint32_t j = lane; j < c_o; j += 64) cmap[d_o + j] = i0 + (uint32_t)o;
		}
	}
}

// gradient of one compacted sample (testbed_nerf.cu:1775-1959): one thread per compacted sample cs (its ray from the
// map k_loss_ray wrote; the pre-compaction samples past each ray's composited prefix are never visited)
__global__ void __launch_bounds__(256) k_loss_grad(StepState* __restrict__ st, DPInfo dp, LossParams lp,
                                                   const float* __restrict__ coords, const half_t* __restrict__ net_out,
                                                   const uint32_t* __restrict__ numsteps, const uint32_t* __restrict__ cmap,
                                                   const uint32_t* __restrict__ rbase, const float4* __restrict__ sa, const float* __restrict__ ekt,
                                                   const float4* __restrict__ ck4, const float* __restrict__ cke, const float4* __restrict__ racc,
                                                   const float4* __restrict__ rgr, float* __restrict__ coords_out, half_t* __restrict__ dL_dout) {
	if (lp.dbg_fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
	if (lp.abort_w && blockIdx.x == 0 && threadIdx.x == 0) {  // (k_loss_ray's witness)
		const uint32_t a = lp.abort_w[lp.abort_slot];
		st->cut_abort = a;
		if (lp.abort_host) __hip_atomic_store(lp.abort_host, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	}
	const uint32_t n = min(st->compacted_counter, lp.max_compacted);
	const uint32_t n_rays_global = st->rays_per_batch * dp.world;
	const float loss_scale = lp.loss_scale / n_rays_global;
	for (uint32_t cs = blockIdx.x * blockDim.x + threadIdx.x; cs < n; cs += gridDim.x * blockDim.x) {
		const uint32_t r = cmap[cs];
		const uint32_t rb = rbase[r];
		const uint32_t cb = numsteps[2 * r + 1];
		const uint32_t j = cs - cb;
		const uint32_t s = rb + j;
		const float* ci = coords + (size_t)s * COORD_W;
		float* co = coords_out + (size_t)(cb + j) * COORD_W;
#pragma unroll
		for (int k = 0; k < COORD_W; ++k) co[k] = ci[k];
		half_t lo[16]; load_out(net_out, s, lo);
		float dir[3]; bent_dir(lo, dir);
		const Alpha a = neus_alpha(lo, dir, unwarp_dt(ci[3]), lp.cos_anneal);
		float Tb;
		const RecState P = scan_replay(rb, s, sa, ekt, ck4, cke, Tb);
		const float4 G = rgr[r], A = racc[r];
		const float lgrad[3] = {G.x, G.y, G.z}, rgb_ray[3] = {A.x, A.y, A.z}, rgb2[3] = {P.r0, P.r1, P.r2};
		const float4 q = sa[s];
		const float rgb[3] = {q.y, q.z, q.w};
		float raw[3];
#pragma unroll
		for (int k = 0; k < 3; ++k) raw[k] = (float)lo[k];
		const float weight = a.alpha * Tb;
		const float T = Tb * (1.f - a.alpha);
		float dl[16];
#pragma unroll
		for (int k = 0; k < 16; ++k) dl[k] = 0.0f;
#pragma unroll
		for (int k = 0; k < 3; ++k) {
			const float sig = rgb[k];
			dl[k] = loss_scale * ((weight * lgrad[k]) * (sig * (1 - sig)) + fmaxf(0.0f, 0.0f * raw[k]));
		}
		float tr[3];
#pragma unroll
		for (int k = 0; k < 3; ++k) tr[k] = T * rgb[k] - (rgb_ray[k] - rgb2[k]);
		const float dot = (lgrad[0] * tr[0] + lgrad[1] * tr[1]) + lgrad[2] * tr[2];
		const float dloss_dalpha = (dot + G.w) / (1.0f - a.alpha + 1e-5);
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
		const float gn = grad_norm(lo);
		const float gn_inv = 1 - 1 / gn;
		const float dloss_dnn = dloss_dalpha * (dadem * dem_dic + dpe_dic * dadpe) * d_ic_tc;
		const float dloss_dsdf = dloss_dalpha * dadem * dem_dsdf;
		dl[3] = loss_scale * dloss_dsdf;
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
}

// sample -> ray map and per-ray base for callers that bring their own numsteps (operator path);
// the training step gets both from k_march_write / the march scan.
__global__ void __launch_bounds__(256) k_ray_index(uint32_t cap_rays, const uint32_t* __restrict__ numsteps, StepState* __restrict__ st,
                                                   uint32_t* __restrict__ sample_ray, uint32_t* __restrict__ rbase) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap_rays; i += gridDim.x * blockDim.x) {
		const uint32_t ns = numsteps[2 * i], base = numsteps[2 * i + 1];
		rbase[i] = base;
		if (ns == 0) continue;
		for (uint32_t j = 0; j < ns; ++j) sample_ray[base + j] = i;
		atomicMax(&st->n_kept, base + ns);
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
__global__ void k_step_counters(StepState* st, uint32_t target_batch, uint32_t max_samples, uint32_t world, uint32_t fixed_rays,
                                const uint32_t* eval_cnt, uint32_t n_eval, uint32_t* abort_host) {
	if (threadIdx.x != 0 || blockIdx.x != 0) return;
	// (the march cut's all-reduced witness word to the host, system scope: the host polls it before its next step)
	if (abort_host) __hip_atomic_store(abort_host, st->cut_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	step_counters_update(st, target_batch, max_samples, world, fixed_rays, eval_cnt, n_eval);
}

// ---------------------------------------------------------------- host launchers
static inline uint32_t ray_blocks(uint32_t cap) { return std::max<uint32_t>(1, std::min<uint32_t>((cap + 255) / 256, 2048)); }
void launch_bitfield_linear(hipStream_t s, const uint8_t* bitfield, uint32_t* lin) {
	k_bitfield_linear<<<GRID3 / 32 / 256, 256, 0, s>>>(bitfield, lin);
}
void launch_march_count(hipStream_t s, uint32_t cap, uint32_t max_samples, StepState* st, DPInfo dp, const DevDataset& ds, const uint8_t* bitfield,
                        const uint32_t* lin, uint64_t rng_state, uint64_t rng_inc, float* rays, float* tstart, uint32_t* nreq, const MarchWork& mw,
                        uint32_t* zero_counters, uint32_t n_zero, const float* occ_bbox) {
	if (n_zero > 256) throw std::runtime_error("launch_march_count: at most 256 counters to zero");
	dbg_lds_gate(s);
	if (mw.est_cut && !(ds.cone_angle == 0.0f && mw.lanes_per_ray == 8 && mw.balanced))
		throw std::runtime_error("launch_march_count: the march cut needs the balanced constant-step march");
	k_ray_gen<<<ray_blocks(cap), 256, 0, s>>>(cap, st, dp, ds, rng_state, rng_inc, rays, tstart, mw.counter, st, mw.jt, zero_counters,
	                                          zero_counters ? n_zero : 0u, occ_bbox, mw.est_cut, std::max(1u, mw.est_div), nreq, mw.nrec, max_samples);
	const uint32_t waves = mw.waves ? std::min(mw.waves, (cap + 63) / 64) : (cap + 63) / 64;
	const uint32_t blocks = std::max<uint32_t>(1, (waves + 3) / 4);
	for (uint32_t pass = 0; pass < 2; ++pass) {
		dbg_lds_gate(s);
		if (ds.cone_angle == 0.0f) {
			if (mw.lanes_per_ray == 1) k_march<true, 1><<<blocks, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, lin, rays, tstart, nreq, mw);
			else if (mw.lanes_per_ray == 8 && mw.balanced) k_march_bal<<<blocks * 8, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, lin, rays, tstart, nreq, mw);
			else if (mw.lanes_per_ray == 8) k_march<true, 8><<<blocks * 8, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, lin, rays, tstart, nreq, mw);
			else if (mw.lanes_per_ray == 16) k_march<true, 16><<<blocks * 16, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, lin, rays, tstart, nreq, mw);
			else k_march<true, 4><<<blocks * 4, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, lin, rays, tstart, nreq, mw);
		} else {
			if (mw.lanes_per_ray == 1) k_march<false, 1><<<blocks, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, nullptr, rays, tstart, nreq, mw);
			else if (mw.lanes_per_ray == 8) k_march<false, 8><<<blocks * 8, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, nullptr, rays, tstart, nreq, mw);
			else if (mw.lanes_per_ray == 16) k_march<false, 16><<<blocks * 16, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, nullptr, rays, tstart, nreq, mw);
			else k_march<false, 4><<<blocks * 4, 256, 0, s>>>(cap, pass, max_samples, st, ds, bitfield, nullptr, rays, tstart, nreq, mw);
		}
	}
}
// Test hook: every CU's LDS filled with `pattern` by resident workgroups (volatile stores: kept), so that a kernel that
// reads LDS it never wrote sees garbage, not the zeros of a fresh device
__global__ void __launch_bounds__(256) k_fill_lds(uint32_t pattern) {
	extern __shared__ uint32_t s_fill[];
	volatile uint32_t* v = s_fill;
	for (uint32_t i = threadIdx.x; i < FILL_LDS_BYTES / 4; i += 256) v[i] = pattern;
}
thread_local uint32_t g_dbg_lds_fill = 0;
thread_local uint32_t g_dbg_xcd_shift = 0;
__global__ void k_xcd_shift() {}
void launch_xcd_shift(hipStream_t s, uint32_t n_blocks) { k_xcd_shift<<<n_blocks, 64, 0, s>>>(); }
void launch_fill_lds(hipStream_t s, uint32_t pattern) {
	// 40 KB per workgroup, 4 resident per CU: the whole 160 KB of every CU (256 CUs), twice over
	k_fill_lds<<<2048, 256, FILL_LDS_BYTES, s>>>(pattern);
}

// Diagnostic (scripts/diag_denorm.py): fp32 denormal arithmetic per lane — det_expf into the denormal range, a product
// of denormal results, ldexpf below FLT_MIN, a product that passes through a denormal and is scaled back — plus the
// wave's MODE register (denormal / rounding controls, s_getreg: a register read). The host compares every launch's bits
// with the same expressions evaluated on the CPU (denormals kept, as the kernels' code objects request).
NEUS_HD void denorm_probe_values(uint32_t i, float v[4]) {
	v[0] = det_expf(-87.0f - (float)(i & 1023u) * 0.015f);
	v[1] = v[0] * 3.7f;
	v[2] = ldexpf(1.5f, -127 - (int)(i % 20u));
	const float a = 1e-20f * (float)(1u + (i & 7u));
	const float b = a * 1e-19f;
	v[3] = b * 1e20f;
}
__global__ void __launch_bounds__(256) k_denorm_probe(uint32_t n, uint32_t* __restrict__ out) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	float v[4];
	denorm_probe_values(i, v);
	uint32_t* o = out + (size_t)i * 5;
#pragma unroll
	for (int k = 0; k < 4; ++k) o[k] = __float_as_uint(v[k]);
	o[4] = (uint32_t)__builtin_amdgcn_s_getreg(1 | (31 << 11));  // HW_REG_MODE, bits 0..31
}
// stats: [0] launches, [1] mismatching values, [2..5] mismatches by 16-lane row of the wave, [6] values flushed to 0,
// [7] distinct MODE values seen, [8] first MODE, [9] a MODE differing from the first (0 if none)
void debug_denorm_probe(hipStream_t s, uint32_t n, uint32_t launches, uint64_t* stats) {
	uint32_t* d = nullptr;
	if (hipMalloc((void**)&d, (size_t)n * 5 * 4) != hipSuccess) throw std::runtime_error("denorm probe: hipMalloc");
	std::vector<uint32_t> h((size_t)n * 5), want((size_t)n * 4);
	for (uint32_t i = 0; i < n; ++i) {
		float v[4];
		denorm_probe_values(i, v);
		for (int k = 0; k < 4; ++k) std::memcpy(&want[(size_t)i * 4 + k], &v[k], 4);
	}
	for (int k = 0; k < 10; ++k) stats[k] = 0;
	uint32_t mode0 = 0;
	bool have_mode = false;
	for (uint32_t l = 0; l < launches; ++l) {
		k_denorm_probe<<<(n + 255) / 256, 256, 0, s>>>(n, d);
		if (hipMemcpyAsync(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
			(void)hipFree(d);
			throw std::runtime_error("denorm probe: copy");
		}
		++stats[0];
		for (uint32_t i = 0; i < n; ++i) {
			for (int k = 0; k < 4; ++k) {
				const uint32_t g = h[(size_t)i * 5 + k], w = want[(size_t)i * 4 + k];
				if (g != w) {
					++stats[1];
					++stats[2 + ((i & 63u) >> 4)];
					if ((g & 0x7fffffffu) == 0) ++stats[6];
				}
			}
			const uint32_t m = h[(size_t)i * 5 + 4];
			if (!have_mode) { mode0 = m; have_mode = true; stats[7] = 1; stats[8] = m; }
			else if (m != mode0 && stats[9] == 0) { stats[9] = m; stats[7] = 2; }
		}
	}
	(void)hipFree(d);
}

void launch_march_write(hipStream_t s, uint32_t cap, StepState* st, const DevDataset& ds, const float* rays, const MarchWork& mw, const uint32_t* nreq,
                        uint32_t* base, uint32_t* numsteps, float* coords, uint32_t* sample_ray, uint32_t sample_cap, void* scan_temp,
                        const Round0List* round0, uint32_t lds_fill) {
	const Round0List r0 = round0 ? *round0 : Round0List{0u, nullptr, nullptr, nullptr, 0u};
	if (cap % 4 || ((uintptr_t)nreq | (uintptr_t)base | (uintptr_t)numsteps | (uintptr_t)r0.c0) & 15)
		throw std::runtime_error("launch_march_write: ray buffers must be 16-B aligned, cap a multiple of 4");
	const uint32_t tiles = (cap + SCAN_TILE - 1) / SCAN_TILE;
	if (tiles > SCAN_MAX_TILES) throw std::runtime_error("launch_march_write: too many ray slots");
	dbg_lds_gate(s);
	k_march_scan<<<tiles, SCAN_THREADS, 0, s>>>(cap, st, nreq, base, numsteps, (ScanState*)scan_temp, scan_next_tag(scan_temp), r0);
	if (lds_fill) launch_fill_lds(s, lds_fill);  // tests: the write kernel finds garbage in every CU's LDS
	else dbg_lds_gate(s);
	// one block per WRITE_CHUNK samples of the largest possible kept extent (max_inference <= sample_cap)
	k_march_write<<<std::max<uint32_t>(1, (sample_cap + WRITE_CHUNK - 1) / WRITE_CHUNK), 256, 0, s>>>(cap, st, ds, rays, mw, nreq, base, coords, sample_ray,
	                                                                                                      r0);
}
void debug_launch_march_stats(hipStream_t s, uint32_t n_rays, const float* rays, const float* tstart, const uint32_t* lin, const DevDataset& ds,
                              const uint8_t* bf, uint32_t* out) {
	k_march_stats<<<(n_rays + 255) / 256, 256, 0, s>>>(n_rays, rays, tstart, lin, ds, bf, out);
}
static inline uint32_t sample_blocks(uint32_t cap) { return std::max<uint32_t>(1, std::min<uint32_t>((cap + 255) / 256, 16384)); }
void launch_loss_alpha(hipStream_t s, uint32_t cap_samples, const StepState* st, const float* coords, const half_t* net_out, float cos_anneal,
                       const LossWork& w, bool dt_const) {
	dbg_lds_gate(s);
	k_loss_alpha<<<sample_blocks(cap_samples), 256, 0, s>>>(cap_samples, &st->n_kept, nullptr, coords, net_out, cos_anneal, w.sa, w.ekt, w.n_long,
	                                                        dt_const);
}
void launch_loss_alpha_list(hipStream_t s, uint32_t cap_samples, const uint32_t* n_ptr, const uint32_t* idx, const float* coords,
                            const half_t* net_out, float cos_anneal, const LossWork& w, bool dt_const) {
	dbg_lds_gate(s);
	k_loss_alpha<<<sample_blocks(cap_samples), 256, 0, s>>>(cap_samples, n_ptr, idx, coords, net_out, cos_anneal, w.sa, w.ekt, nullptr, dt_const);
}
void launch_loss_scan_chunk(hipStream_t s, uint32_t cap_rays, const uint32_t* numsteps, const LossWork& w, uint32_t* ccount, uint32_t e0,
                            uint32_t e1, uint32_t e2, uint32_t* list, uint32_t* next_counter, const uint32_t* rays_in, const uint32_t* n_rays_in,
                            uint32_t* rays_out, uint32_t* n_rays_out) {
	dbg_lds_gate(s);
	k_loss_scan_chunk<<<std::max<uint32_t>(1, std::min<uint32_t>((cap_rays + 63) / 64, 8192)), 64, 0, s>>>(
		cap_rays, numsteps, w.sa, w.ekt, w.ck4, w.cke, ccount, w.racc, w.rT, w.rek, e0, e1, e2, list, next_counter, rays_in, n_rays_in,
		rays_out, n_rays_out);
}
void launch_prog_cut(hipStream_t s, uint32_t cap_rays, const uint32_t* ccount, const uint32_t* excl, uint32_t batch, uint32_t* cutw, int mode,
                     uint32_t* eval0, uint32_t* abort_if_none) {
	k_prog_cut<<<(cap_rays + 255) / 256, 256, 0, s>>>(cap_rays, ccount, excl, batch, cutw, mode, eval0, abort_if_none);
}
void launch_prog_next(hipStream_t s, uint32_t cap_rays, const uint32_t* rays_in, const uint32_t* n_in, const uint32_t* numsteps, const uint32_t* cut,
                      uint32_t e1, uint32_t e2, uint32_t* list, uint32_t* list_counter, uint32_t* rays_out, uint32_t* n_out) {
	k_prog_next<<<std::max<uint32_t>(1, std::min<uint32_t>((cap_rays + 255) / 256, 1024)), 256, 0, s>>>(rays_in, n_in, numsteps, cut, e1, e2, list,
	                                                                                                   list_counter, rays_out, n_out);
}
// w.n_long is zeroed by the k_loss_alpha launch before it
void launch_loss_scan_ray(hipStream_t s, uint32_t cap_rays, const uint32_t* numsteps, const LossWork& w, uint32_t* ccount) {
	const uint32_t blocks = ray_blocks(cap_rays);
	dbg_lds_gate(s);
	k_loss_scan_ray<true><<<blocks, 256, 0, s>>>(cap_rays, numsteps, w.sa, w.ekt, w.ck4, w.cke, ccount, w.racc, w.rT, w.long_rays, w.n_long);
	// the long rays, 64 to a one-wave block
	if (w.long_rays) dbg_lds_gate(s);
	if (w.long_rays) k_loss_scan_list<<<std::max<uint32_t>(1, std::min<uint32_t>((cap_rays + 63) / 64, 4096)), 64, 0, s>>>(
		numsteps, w.sa, w.ekt, w.ck4, w.cke, ccount, w.racc, w.rT, w.long_rays, w.n_long);
}
// timing experiments (neus_debug_time_kernel): variant 1 = the recurrence without its per-sample stores, one
// thread per ray for every ray
void debug_launch_loss_scan(hipStream_t s, int variant, uint32_t cap_rays, const uint32_t* numsteps, const LossWork& w, uint32_t* ccount) {
	if (variant == 1) k_loss_scan_ray<false><<<ray_blocks(cap_rays), 256, 0, s>>>(cap_rays, numsteps, w.sa, w.ekt, w.ck4, w.cke, ccount, w.racc, w.rT,
	                                                                           nullptr, nullptr);
	else {
		if (w.n_long) (void)hipMemsetAsync(w.n_long, 0, 4, s);
		launch_loss_scan_ray(s, cap_rays, numsteps, w, ccount);
	}
}
__global__ void k_srgb_lut(float* __restrict__ lut) {
	const uint32_t b = threadIdx.x;
	lut[b] = srgb_to_linear((float)b * (1.0f / 255.0f));
}
void launch_srgb_lut(hipStream_t s, float* lut) { k_srgb_lut<<<1, 256, 0, s>>>(lut); }
void launch_loss_ray(hipStream_t s, uint32_t cap_rays, StepState* st, DPInfo dp, const DevDataset& ds, const LossParams& lp, uint32_t* numsteps,
                     const uint32_t* ccount, const uint32_t* cbase, const LossWork& w, float* loss, float* ek, float* mask) {
	if (!w.cmap) throw std::runtime_error("launch_loss_ray: LossWork::cmap (max_compacted entries) is required");
	dbg_lds_gate(s);
	k_loss_ray<<<ray_blocks(cap_rays), 256, 0, s>>>(cap_rays, st, dp, ds, lp, numsteps, ccount, cbase, w.sa, w.ekt, w.ck4, w.cke, w.racc, w.rT,
	                                                  w.rgr, loss, ek, mask, w.cmap);
}
void launch_loss_grad(hipStream_t s, uint32_t cap_samples, StepState* st, DPInfo dp, const LossParams& lp, const float* coords,
                      const half_t* net_out, const uint32_t* numsteps, const LossWork& w, float* coords_out, half_t* dL_dout) {
	(void)cap_samples;  // (the compacted samples: at most lp.max_compacted)
	dbg_lds_gate(s);
	k_loss_grad<<<sample_blocks(lp.max_compacted), 256, 0, s>>>(st, dp, lp, coords, net_out, numsteps, w.cmap, w.rbase, w.sa,
	                                                         w.ekt, w.ck4, w.cke, w.racc, w.rgr, coords_out, dL_dout);
}
void launch_ray_index(hipStream_t s, uint32_t cap_rays, const uint32_t* numsteps, StepState* st, uint32_t* sample_ray, uint32_t* rbase) {
	k_ray_index<<<ray_blocks(cap_rays), 256, 0, s>>>(cap_rays, numsteps, st, sample_ray, rbase);
}
void launch_rollover(hipStream_t s, uint32_t n_elements, const StepState* st, float* coords, half_t* dL_dout) {
	k_rollover<<<std::max<uint32_t>(1, std::min<uint32_t>((n_elements + 255) / 256, 2048)), 256, 0, s>>>(n_elements, st, coords, dL_dout);
}
void launch_step_counters(hipStream_t s, StepState* st, uint32_t target_batch, uint32_t max_samples, uint32_t world, uint32_t fixed_rays,
                          const uint32_t* eval_cnt, uint32_t n_eval, uint32_t* abort_host) {
	dbg_lds_gate(s);
	k_step_counters<<<1, 64, 0, s>>>(st, target_batch, max_samples, world, fixed_rays, eval_cnt, n_eval, abort_host);
}

} // namespace neus
