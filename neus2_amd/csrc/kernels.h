// Host-callable launchers of the gfx950 kernels (defined in the .hip files) and the structs
// shared between the host orchestration (testbed.cpp) and the kernels.
#pragma once
#include <functional>
#include <vector>
#include "common.h"

namespace neus {

struct MlpPtrs {
	const half_t* d0;  const half_t* d1;                     // density W0 [W][DIN], W1 [16][W]
	const half_t* r0;  const half_t* r1;  const half_t* r2;  // rgb W0 [W][48], W1 [W][W], W2 [16][W]
	const half_t* d0T; const half_t* d1T;                    // transposed copies [DIN][W], [W][16]
	const half_t* r0T; const half_t* r1T; const half_t* r2T; // [48][W], [W][W], [W][16]
	const half_t* d0p; const half_t* d0Tp;                   // W0 with din-permuted columns / W0^T permuted rows (fused kernels)
	const half_t* var;                                       // variance param (fp16)
	float sdf_bias;                                          // -0.1
};

struct TrainBufs {
	half_t* d1_delta;                 // [16][ld] dL/d(density output) (colour kernel -> density kernel)
	half_t* dLdenc; half_t* genc;     // [L][ld] half2 (features 2l, 2l+1): the grid scatter's operands
	float4* v;                        // [ld]
	float* var_grad;                  // variance gradient (written by the gradient reduction)
	float* var_partial;               // [blocks of the colour kernel] per-block sums of dL/dout[7]
	float indeed_batch;
	float4* dpos;                     // [ld] dL/d(network input position), first order (null: not needed)
	// MLP weight gradients, accumulated in registers by the training kernels: one row of n_matrix floats per block
	// (the density kernel fills [0, n_density), the colour kernel [n_density, n_matrix)), summed over the blocks in
	// a fixed order by k_mlp_grad_reduce
	float* wpartial;
	uint32_t n_matrix, off_d1, off_r0, off_r1, off_r2;
};
struct MlpGradReduce {
	const float* partial; uint32_t n_blocks, n_matrix; float* g; const uint32_t* n_valid;
	const float* var_partial; uint32_t var_blocks; float* var_grad;
};

// Dynamic scenes. DeltaNetwork parameters in the reference's order: transition[4] |
// rotation 6D[8] (transform_network.h:313-333); only slots 0..2 and 4..9 carry values.
constexpr uint32_t DELTA_PARAMS = 12;
struct DeltaState {
	float p[DELTA_PARAMS];                      // fp32 master (the forward reads them fp16-rounded)
	float m1[DELTA_PARAMS], m2[DELTA_PARAMS];   // Adam moments
	uint32_t steps[DELTA_PARAMS];               // per-parameter Adam steps
	float grad[DELTA_PARAMS];                   // last gradient (fp16 values, loss-scaled)
	float R[9], Rinv[9], t[3];                  // k_delta_prepare: rotation (row-major), inverse, translation
};
struct DeltaAdam { float lr, beta1, beta2, eps, loss_scale; uint32_t optimize; };
// Accumulated global movement applied to every ray (global_movement_with_rotation_6d, testbed_nerf.cu:193-213).
struct RayMotion { float R[9]; float t[3]; uint32_t on; };
// Loss-target options; all-zero = the reference drivers' defaults (random background, colour space Linear,
// linear_colors off: sRGB targets). mode: 0 Linear colour space, 1 SRGB colour space, 2 train in linear colours.
struct TrainTarget { uint32_t fixed_bg; float bg[3]; uint32_t mode; };

struct DevDataset {
	const uint32_t* pixels;
	const uint64_t* pix_off;
	const int32_t* res;       // 2 per image
	const float* focal;       // 2 per image
	const float* pp;          // 2 per image
	const float* xform;       // 12 per image (row-major 3x4)
	uint32_t n_images;
	float aabb_min[3], aabb_max[3];
	float cone_angle;
	RayMotion motion;         // frames >= 1 of a dynamic scene: o' = R o + t, d' = R d (normalized d)
	TrainTarget target;       // background / colour space of the loss targets (testbed_nerf.cu:1642-1671)
	const float* lin_lut;     // 256 entries: srgb_to_linear(b / 255) as the device computes it (read_rgba's byte path)
};

struct DPInfo { uint32_t rank, world; };

// Render camera (Testbed::set_camera_to_training_view, testbed.cu:264-270; render_nerf, testbed_nerf.cu:2670-2760):
// camera-to-world 3x4 row-major, focal length in pixels, screen centre (= the view's principal point), and the
// sub-pixel offset of pixel_to_ray (ld_random_pixel_offset, computed on the host).
struct RenderCamera {
	float xform[12];
	float focal[2], screen_center[2], pixel_offset[2];
	uint32_t width, height;
};
constexpr float NERF_RENDERING_NEAR_DISTANCE = 0.2f;  // testbed_nerf.cu:57
constexpr uint32_t MARCH_ITER = 10000;                  // testbed_nerf.cu:78
constexpr uint32_t MAX_STEPS_INBETWEEN_COMPACTION = 8;  // testbed_nerf.cu:81

struct LossParams {
	float loss_scale;      // LOSS_SCALE = 128 (testbed.h:246)
	float ek_w, mask_w, cos_anneal;
	uint32_t max_compacted; // target batch size
	uint64_t rng_state, rng_inc;
	PcgJumpTable jt;
	uint32_t dbg_fence = 0;  // development (NEUS_DBG_LOSS_FENCE=1): an agent-scope acquire fence at the loss-gradient kernel's start
	// the march cut's witness (k_loss_ray): abort_w[abort_slot] set when this step's training is not provably the full
	// march's, abort_w[abort_slot ^ 1] cleared for the next step; k_loss_grad copies the word to StepState::cut_abort.
	// Null: no witness (cut_abort stays 0)
	uint32_t* abort_w = nullptr;
	uint32_t abort_slot = 0;
	uint32_t* abort_host = nullptr;  // (one rank) host-coherent pinned word the copy is also stored to, system scope
};

// binned hash-grid gradient scatter (grid.hip)
// bucket = 2048 grid entries: 32 KB of int64 pairs in LDS, four accumulation workgroups per CU (4096-entry buckets, two
// per CU: 158 -> 148 us per step of scatter at the bench state; 1024 entries: 166 us, the region tables' reads grow)
#ifndef NEUS_SB_SHIFT
#define NEUS_SB_SHIFT 11
#endif
constexpr uint32_t SB_SHIFT = NEUS_SB_SHIFT, SB_SIZE = 1u << SB_SHIFT;
constexpr uint32_t SB_MAX_BUCKETS = (1u << 24) / SB_SIZE;      // 16 levels x 2^19 entries / SB_SIZE (+ level boundaries: 4096 at 4096-entry buckets)
constexpr uint32_t SB_LEVEL_BUCKETS = (1u << 19) / SB_SIZE + 2; // buckets one level can touch (2^19-entry tables)
struct ScatterWork {
	uint32_t* counts;   // [n_buckets * n_blocks + 1] contributions per (bucket, block), bucket-major
	uint32_t* offs;     // exclusive scan of counts
	h2* rec_g;          // [capacity] contribution (feature 0, feature 1), fp16 as the reference's per-corner half2 atomic operand
	uint16_t* rec_i;    // [capacity] entry within the bucket
	uint32_t n_buckets, n_blocks;
	// accumulation workgroups (scatter_accum_jobs): {bucket, part, parts, split slot}; the buckets of the small dense
	// levels collect most records, so they are split over `parts` workgroups whose int64 sums meet in `split`
	const uint4* jobs;
	unsigned long long* split;  // [n_split][2 * SB_SIZE] int64 partial sums (zero between uses)
	uint32_t* split_done;       // [n_split] parts finished (reset by the last part)
	uint32_t n_jobs;
	uint32_t n_active;          // buckets counted / scanned (those below it hold every record of the step)
	uint32_t n_chunks, chunk;   // workgroups of the wide-block / region binning (modes 0, 2) and their samples (512 or 1024)
	uint32_t mode;              // 2 per-block record regions (default), 0 wide-block binning, 1 the 256-sample hist / scan / bin path
	// mode 2: bucket starts of every [level][block] region (u16, SB_LEVEL_BUCKETS + 1 per region) and the accumulation
	// jobs over level-local buckets {level, bucket, part | parts << 16, split slot}, level-major
	uint16_t* rtab;
	const uint4* jobs2;
	uint32_t n_jobs2;
	uint32_t xcd_group = 1;     // the region accumulation's jobs per XCD group (k_scatter_accum_r; 1 = list order)
	uint32_t jobs2_before[17];  // jobs of the levels below l (l <= 16): the launch takes those up to the valid level
	uint32_t level_groups;      // mode 2: workgroups per sample chunk, each binning levels y, y + groups, ... (0: one per level)
};

// accumulation workgroups of the scatter (flattened uint4 {bucket, part, parts, split slot}); n_split = split buckets
std::vector<uint32_t> scatter_accum_jobs(const GridLevels& gl, uint32_t n_buckets, uint32_t& n_split);
// mode-2 jobs (flattened uint4) and the jobs of the levels below l (jobs_before_level[l], L + 1 entries)
std::vector<uint32_t> scatter_region_jobs(const GridLevels& gl, uint32_t& n_split, std::vector<uint32_t>& jobs_before_level);

// per-sample / per-ray scratch of the restructured loss (march.hip)
struct LossWork {
	float4* sa;             // [samples] alpha, sigmoid(rgb)
	float4* ck4;            // [samples / 8 + 1] state {T, rgb prefix} before each sample s with s % 8 == 0
	float* cke;             // [samples / 8 + 1] eikonal-term prefix before the same samples
	float* ekt;             // [samples] eikonal term
	uint32_t* sample_ray;   // [samples] owning ray
	const uint32_t* rbase;  // [rays] first sample of the ray (pre-compaction)
	float4* racc;           // [rays] rgb_ray, weight_sum
	float* rT;              // [rays] final transmittance
	float* rek;             // [rays] eikonal-term sum (progressive inference: the state between rounds)
	uint32_t* long_rays;    // [rays] rays the transmittance scan runs one wave per ray (nullable: one thread per ray)
	uint32_t* n_long;       // their count (zeroed by k_loss_alpha)
	float4* rgr;            // [rays] dL/drgb_ray (Huber'), gws * (1 - weight_sum)
	uint32_t* cmap;         // [max_compacted] owning ray of each compacted sample (k_loss_ray; k_loss_grad's work items)
};

// Adam's bias-correction factors by per-parameter step: tab[k] = sqrtf(1 - powf(beta2, k)) and
// tab[ADAM_BIAS_TAB + k] = 1 - powf(beta1, k) for k < ADAM_BIAS_TAB, evaluated once by k_adam_bias_table with the
// expressions of adam.h:137 (the two powf per parameter were ~3/4 of the Adam pass's VALU work); past the table both
// are exactly 1.0f when `bias_converged` (beta^k below 2^-30 there), so lr = (lr * 1) / 1 = lr.
constexpr uint32_t ADAM_BIAS_TAB = 4096;
struct AdamParams {
	uint32_t n, n_matrix;
	float loss_scale, lr, beta1, beta2, eps, l2_reg;
	float ema_decay, ema_debias_old, ema_debias_new;
	uint32_t optimize_matrix, optimize_non_matrix;
	const float* bias_tab;    // [2 * ADAM_BIAS_TAB] or null (powf per parameter)
	uint32_t bias_converged;
	float inv_loss_scale;     // 1 / loss_scale when that is a power of two (the product is then the exact quotient)
	uint32_t pow2_scale;
	uint32_t skip_ema_h;      // leave the fp16 EMA copy to a later cast of the fp32 EMA (NeusTestbed::sync_ema_h)
	const uint32_t* abort;    // StepState::cut_abort, or null: while set the launch changes nothing (the step is re-run)
};
void launch_adam_bias_table(hipStream_t s, float beta1, float beta2, float* tab);

// The Adam launch's two riders (each optional): the step-end counters (k_step_counters' work, done by thread 0 of block
// 0) and the transposed / permuted fp16 copies of the MLP matrices (prepare_weights), written by the threads that
// update the matrix parameters (the launch after it no longer has to re-transpose)
struct StepCounterArgs { StepState* st; uint32_t target_batch, max_samples, world, fixed_rays; const uint32_t* eval_cnt; uint32_t n_eval; };
struct AdamTranspose {
	uint32_t n;                                    // matrices (0: none)
	uint32_t off[5], rows[5], cols[5];             // parameter offset and shape of matrix j
	half_t* dst[5];                                // its transposed copy [cols][rows]
	int32_t inv[48];                               // matrix 0 (the density input layer): logical column -> physical, -1 none
	half_t* d0p; half_t* d0Tp; uint32_t din, W;    // its permuted copy [W][din] and transposed permuted copy [din][W]
};
struct TransposeJob { const half_t* src; half_t* dst; uint32_t rows, cols; };
struct TransposeJobs { TransposeJob j[8]; uint32_t n; };

// grid.hip
// the training batch's rollover done by the encode (k_grid_encode): n_in = *n_in_ptr (compacted count) records are real,
// the rest of the n_elements batch copies record i % n_in (coordinates in place through `coords`, the writable view of
// the encode's coordinate input; dL_dout rescaled)
struct EncodeRollover { const uint32_t* n_in_ptr; uint32_t n_elements; half_t* dL_dout; float* coords; };
void launch_grid_encode(hipStream_t s, const uint32_t* n_ptr, uint32_t n_fixed, uint32_t ld, const float* coords, uint32_t coord_stride,
                        const GridLevels& gl, uint32_t valid_level, const half_t* grid, uint32_t* enc, float* dydx, uint32_t grid_x, const EncodeRollover* ro = nullptr);
size_t scatter_records_capacity(uint32_t n_cap, uint32_t n_levels);
uint32_t scatter_n_buckets(const GridLevels& gl);
// Level groups of the accumulation (region mode): the accumulation runs group by group, level-major, and after the
// launch of the levels [lo, hi) `done(lo, hi)` is called (their gradient range is final once that launch completes on
// the stream): the data-parallel step all-reduces it beside the accumulation of the next group
struct ScatterSplit { uint32_t n_groups; uint32_t level_end[8]; std::function<void(uint32_t, uint32_t)> done; };
void launch_grid_scatter(hipStream_t s, const uint32_t* n_ptr, uint32_t n_cap, uint32_t ld, const float* coords, uint32_t coord_stride,
                         const GridLevels& gl, uint32_t valid_level, const half_t* dLdenc, const half_t* g, const float4* v, float* grads,
                         const ScatterWork& w, void* scan_tmp, size_t scan_tmp_bytes, const ScatterSplit* split = nullptr);
// mlp.hip
bool mlp_supported(uint32_t n_levels, uint32_t width);
void mlp_din_permutation(uint32_t L, int32_t* perm /* DIN entries: physical row -> logical din index or -1 */);
// the loss's alpha pass fused into the inference epilogue (k_loss_alpha's per-sample terms of every evaluated sample):
// sa / ekt of LossWork, the cosine anneal, dt_const (cone angle 0: every record's dt is the constant step) and the
// long-ray counter to zero (nullable)
struct InferAlpha {
	float4* sa; float* ekt; float cos_anneal; uint32_t dt_const; uint32_t* n_long;
	uint32_t xcd_parts = 0;  // 8: the work items cut into 8 contiguous parts, part x run by the blocks of XCD x (blockIdx mod 8)
};
void launch_nerf_infer(hipStream_t s, uint32_t L, uint32_t W, const uint32_t* n_ptr, uint32_t n_fixed, const float* coords, const GridLevels& gl,
                       uint32_t valid_level, const half_t* grid, const MlpPtrs& w, half_t* out, uint32_t blocks,
                       const uint32_t* idx = nullptr /* work item j -> sample idx[j] (progressive-inference rounds) */, const InferAlpha* ia = nullptr);
void launch_nerf_density(hipStream_t s, uint32_t L, uint32_t W, uint32_t n, const float* pos, const GridLevels& gl, uint32_t valid_level,
                         const half_t* grid, const MlpPtrs& w, float* density);
// Occupancy-grid update, fused (MODE 2 of k_nerf_density): density-grid samples [lo, lo + n) of the update's
// uniform (n_u) + occupancy-biased (n_nu) samples generated in-kernel, density splatted (atomicMax) into grid_tmp.
struct OccSampling {
	uint32_t n_u, n_nu, lo;
	uint64_t rng_u_state, rng_u_inc, rng_nu_state, rng_nu_inc;
	uint32_t step, n_cascades;
	float thresh_nu;
	float amin[3], diag[3];
	const float* grid_in;
	float* grid_tmp;
	PcgJumpTable jt;
	uint32_t exclusive;   // the all-cells uniform pass over one cascade: index = cell (occ_common.h grid_sample_cell), plain stores
	// the uniform samples of this rank in the order of their mip-0 cells (k_occ_uniform_list; nullable): work item k < n_ulist
	// is uniform sample ulist[k], the rest are the nonuniform samples in index order
	const uint32_t* ulist;
	uint32_t n_ulist;
	// (with ulist) the rank's occupancy-biased samples in the order of their coarse cells (launch_occ_nu_list; nullable):
	// work item n_ulist + k is occupancy-biased sample nulist[k] of the rank
	const uint32_t* nulist = nullptr;
};
// The occupancy-biased samples [0, n) of a rank (global index g0 + k) binned by their coarse cell (cascade, 8^3-cell
// Morton block: n_cascades x 4096 bins) into `list` - the order the density pass evaluates them in, for coherent
// gathers; each sample's value and the max splat do not depend on it. key [n], bins [2 * n_cascades * 4096] scratch.
void launch_occ_nu_list(hipStream_t s, uint32_t n, uint32_t g0, const OccSampling& os, uint32_t* key, uint32_t* bins, uint32_t* list, void* scan_tmp,
                        size_t scan_tmp_bytes);
// Cell-ordered list of the uniform samples [lo, hi) (n_u <= 128^3): the uniform hash (the first try always taken) maps
// sample i to cell ((i + step n_u) 56924617 + 96925573) mod 2^21 bijectively, so walking the cells in (Morton) order and
// inverting gives the samples in spatially coherent order; one look-back-scan pass (scan_tmp: a scan_temp_bytes state),
// list[] gets hi - lo entries
void launch_occ_uniform_list(hipStream_t s, uint32_t n_u, uint32_t step, uint32_t lo, uint32_t hi, uint32_t* list, void* scan_tmp);
void launch_occ_density(hipStream_t s, uint32_t L, uint32_t W, uint32_t n, const OccSampling& os, const GridLevels& gl, uint32_t valid_level,
                        const half_t* grid, const MlpPtrs& w);
// raw SDF on a uniform grid (marching cubes input), grid points offset .. offset + n - 1 (x fastest)
void launch_sdf_grid(hipStream_t s, uint32_t L, uint32_t W, const uint32_t res[3], const float render_min[3], const float render_max[3],
                     const float train_min[3], const float train_max[3], uint64_t offset, uint32_t n, const GridLevels& gl, uint32_t valid_level,
                     const half_t* grid, const MlpPtrs& w, float* sdf, const DeltaState* delta = nullptr);
void launch_mlp_train(hipStream_t s, uint32_t L, uint32_t W, const uint32_t* n_valid_ptr, uint32_t n, uint32_t ld, const float* coords,
                      const half_t* enc, const float* dydx, const half_t* dL_dout, const MlpPtrs& w, const TrainBufs& tb, int part = 0 /* 0 both, 1 colour, 2 density */);
void launch_mlp_grad_reduce(hipStream_t s, const MlpGradReduce& r);  // MLP weight + variance gradients (fixed order)
uint32_t mlp_train_blocks(uint32_t L, uint32_t W, uint32_t n);  // grid of the training MLP kernels (= the variance partial count)
void launch_mfma_probe(hipStream_t s, const half_t* A, const half_t* B, float* C);
// operator module: tcnn NetworkWithInputEncoding(HashGrid -> FullyFusedMLP 1 hidden ReLU layer -> 16 linear), mlp.hip k_dnet
struct DNetLaunch {
	const half_t* w0; const half_t* w1; const uint32_t* enc; const half_t* dL; const uint32_t* u; half_t* out; uint32_t* denc; float* wpartial;
};
bool dnet_supported(uint32_t L, uint32_t W);
uint32_t dnet_blocks(uint32_t n);  // the grid of launch_dnet (= the partial rows of modes 1 and 2)
void launch_dnet(hipStream_t s, uint32_t L, uint32_t W, int mode /* 0 fwd, 1 bwd, 2 bwd-bwd */, uint32_t n, const DNetLaunch& d);
// ffmlp.hip: tcnn FullyFusedMLP behind the Identity encoding (cpp_api.cu:170-172, the network of create_network)
enum : uint32_t { FF_NONE = 0, FF_RELU = 1, FF_EXP = 2, FF_SIGMOID = 3, FF_SQUAREPLUS = 4, FF_SOFTPLUS = 5 };
enum : uint32_t { FF_MODE_ACT = 0, FF_MODE_DACT = 1, FF_MODE_F32 = 2 };
struct FfLayer {
	const half_t* W; uint32_t O, K; uint32_t trans;  // A = W [O][K] or (trans) W^T of W [K][O]
	const half_t* in; uint32_t ldi;                    // [n][ldi] fp16
	half_t* out; float* out_f; uint32_t ldo, o_lim;    // [n][ldo] fp16 (modes ACT, DACT) or f32 (mode F32, o < o_lim)
	float out_scale = 1.f;                             // mode F32: the fp16-rounded sum times this (an Identity encoding's scale)
	const half_t* aux; uint32_t ldx;                   // mode DACT: forward post-activation values [n][ldx]
	uint32_t mode, act, n;
};
struct FfWgrad {
	const half_t* D; uint32_t ldd, O;                  // [n][ldd] deltas
	const half_t* X; uint32_t ldx, I;                  // [n][ldx] layer inputs
	float* partial; uint32_t ld_partial, off;          // partial rows [blocks][ld_partial], this matrix at off (O x I)
	uint32_t n;
};
void launch_ff_layer(hipStream_t s, const FfLayer& L);
uint32_t ff_wgrad_blocks(uint32_t n);  // blocks (= partial rows) of launch_ff_wgrad for n samples
void launch_ff_wgrad(hipStream_t s, const FfWgrad& G);
void launch_ff_input(hipStream_t s, uint32_t n, uint32_t n_in, uint32_t ld, const float* in, float scale, float offset, half_t* x, bool grad);
void launch_ff_out_delta(hipStream_t s, uint32_t n, uint32_t ld, uint32_t act, const half_t* dL, const half_t* out, half_t* d);
// march.hip
void launch_bitfield_linear(hipStream_t s, const uint8_t* bitfield, uint32_t* lin /* LIN_WORDS */);
// world-space box of every occupied cell of every mip -> scratch[0..6) = {min xyz, max xyz} (optim.hip); the ray
// generation culls rays that miss it. scratch: occ_bbox_scratch_floats() floats.
size_t occ_bbox_scratch_floats();
void launch_occ_bbox(hipStream_t s, const uint8_t* bitfield, float* scratch);
// Sample runs of the march (march.hip): per ray slot up to NERF_STEPS records {t of the run's first sample,
// (samples of the ray before the run) << 16 | run length}; a run's samples are t, t + dt(t), ... (the reference's
// t += dt), at most MARCH_RUN_MAX of them. nrec: records per slot; counter: the persistent march's ray queue.
// seg: per ray slot MARCH_SEG_RECS segment-local run records (the multi-lane march's scratch, split evenly over the
// lanes of a ray; a segment never holds more runs than its ~NERF_STEPS / lanes steps).
constexpr uint32_t MARCH_RUN_MAX = 16;
constexpr uint32_t MARCH_SEG_RECS = NERF_STEPS + 64;
struct MarchWork {
	uint2* rec; uint32_t* nrec; uint32_t* counter /* 2: the two passes' ray queues */; uint32_t waves; /* 0 = one lane per ray */
	uint2* seg; uint32_t lanes_per_ray;  /* 1, 4, 8 or 16 */
	PcgJumpTable jt;                      /* jump-ahead of the ray generator's per-ray rng offsets */
	unsigned long long* prof = nullptr;   /* development: per-wave phase timestamps of the march (8 per wave), or null */
	uint32_t dbg = 0;                     /* development timing experiments (wrong results): 1 no record stores, 2 no occupancy loads */
	uint32_t balanced = 0;                /* 8 lanes per ray on average, shared by the 8 rays of a wave by length (k_march_bal, constant-step
	                                         march only) */
	const uint32_t* est_cut = nullptr;    /* the march cut (k_ray_gen, k_march_bal): when this device word (the compaction cut's split
	                                         estimate, cutw[CW_EST]) is below the first pass's slots, only the slots below it are generated
	                                         and marched, the rest dropped behind one marker over the cap (StepState::march_cut) */
	uint32_t est_div = 1;                 /* test hook (NEUS_DBG_MARCH_CUT_DIV): the march cut's estimate divided by this, so that its
	                                         witness fails and the host's re-run path runs */
};
// Ray generation + the occupancy march: rays (6 f32 per slot), tstart (1 per slot), nreq (requested
// samples per slot) and the sample runs (MarchWork).
void launch_march_count(hipStream_t s, uint32_t cap, uint32_t max_samples /* global cap: 16 x batch */, StepState* st, DPInfo dp, const DevDataset& ds, const uint8_t* bitfield,
                        const uint32_t* lin, uint64_t rng_state, uint64_t rng_inc, float* rays, float* tstart, uint32_t* nreq, const MarchWork& mw,
                        uint32_t* zero_counters = nullptr, uint32_t n_zero = 0,
                        const float* occ_bbox = nullptr /* launch_occ_bbox; null: no culling */);
// Progressive round 0's work list, written by the march (the first min(n, e1) samples of every kept ray at the
// exclusive scan c0 of those counts); counters[0] = its length, counters[1 .. n_counters) zeroed for the later rounds.
struct Round0List { uint32_t e1; uint32_t* c0; uint32_t* list; uint32_t* counters; uint32_t n_counters; };
// Spatial ray order of the progressive rounds (march.hip k_ray_hist, a scan, k_ray_sort_place): hist and off are
// [2][RS_BINS + 1][ray_sort_blocks(cap)] (per block of slots: ray count and round-0 chunk samples per 8^3 Morton cell;
// bin RS_BINS = slots without kept samples) and its exclusive scan; key [cap] per ray slot; perm [cap] the slots in
// order, *n_perm of them
constexpr uint32_t RS_BINS = 512;
struct RaySort { uint32_t* hist; uint32_t* off; uint16_t* key; uint32_t* perm; uint32_t* n_perm; };
// The split of round 0 for the compaction cut (est != null; NeusTestbed::prog_cut): the rays of the slots below *est first
// (pass A: perm [0, n_perm), list [0, list_len)), the rest apart (pass B: perm from perm_b, list from list_b, their counts in
// cutw[CW_NB] / cutw[CW_LENB]); ccount zeroed for the slots without samples or past *est (pass A's cut reads it); rays
// without samples are left out of both passes. hist / off then hold [2][2 RS_BINS + 1][blocks].
struct RaySplit { const uint32_t* est; uint32_t* ccount; uint32_t* cutw; uint32_t perm_b, list_b; };
// cutw words (march.hip k_prog_cut)
constexpr uint32_t CW_CUT = 0, CW_LENB_EFF = 1, CW_NB_EFF = 2, CW_CUT_A = 3, CW_LENB = 4, CW_NB = 5, CW_EST = 6, CW_ABORT = 8 /* 2 words */,
                   CW_WORDS = 16;
uint32_t ray_sort_blocks(uint32_t cap);
void launch_ray_sort(hipStream_t s, uint32_t cap, const uint32_t* numsteps, const float* coords, uint32_t e1, const RaySort& rs, uint32_t* list,
                     uint32_t* list_len, void* scan_temp, size_t scan_temp_bytes, const RaySplit* split = nullptr);
// k_march_scan (the scan of the requested counts fused with numsteps, scan_temp = a scan_temp_bytes buffer) and
// k_march_write; round0 nullable
void launch_march_write(hipStream_t s, uint32_t cap, StepState* st, const DevDataset& ds, const float* rays, const MarchWork& mw, const uint32_t* nreq,
                        uint32_t* base, uint32_t* numsteps, float* coords, uint32_t* sample_ray, uint32_t sample_cap, void* scan_temp,
                        const Round0List* round0 = nullptr, uint32_t lds_fill = 0 /* tests: garbage-fill LDS before the write kernel */);
constexpr uint32_t FILL_LDS_BYTES = 40 * 1024;
void launch_fill_lds(hipStream_t s, uint32_t pattern);
// Determinism test hook (neus_debug_set_lds_fill_all): while the calling host thread runs a training step with it set,
// every CU's LDS is filled with this pattern before each kernel of the step (the launchers call dbg_lds_gate before their
// launches), so a kernel that read LDS it had not written in this launch would read garbage and change the step's
// results. 0 (always, outside the tests): no fill.
extern thread_local uint32_t g_dbg_lds_fill;
// Placement test hook (neus_debug_set_xcd_shift): a one-wave kernel of this many workgroups before each kernel of the
// step shifts the round-robin workgroup -> XCD placement of the next launch (results must not depend on it)
extern thread_local uint32_t g_dbg_xcd_shift;
// inference timing (testbed.cpp it_arm): when set, the next launch_nerf_infer launch records these two events at its
// kernel's start and end (hipExtLaunchKernelGGL), then clears them
extern thread_local hipEvent_t g_infer_ev[2];
void debug_denorm_probe(hipStream_t s, uint32_t n, uint32_t launches, uint64_t* stats);
void launch_xcd_shift(hipStream_t s, uint32_t n_blocks);
inline void dbg_lds_gate(hipStream_t s) {
	if (g_dbg_lds_fill) launch_fill_lds(s, g_dbg_lds_fill);
	if (g_dbg_xcd_shift) launch_xcd_shift(s, g_dbg_xcd_shift);
}
void debug_launch_march_stats(hipStream_t s, uint32_t n_rays, const float* rays, const float* tstart, const uint32_t* lin, const DevDataset& ds,
                              const uint8_t* bf, uint32_t* out);
// dt_const: every sample's dt is MIN_CONE_STEPSIZE (cone angle 0, coordinates from k_march_write): the kernel
// evaluates the same warp / unwarp instead of reading the coordinate record
void launch_loss_alpha(hipStream_t s, uint32_t cap_samples, const StepState* st, const float* coords, const half_t* net_out, float cos_anneal,
                       const LossWork& w, bool dt_const = false);
void launch_loss_scan_ray(hipStream_t s, uint32_t cap_rays, const uint32_t* numsteps, const LossWork& w, uint32_t* ccount);
// progressive (cut-off-aware) inference rounds (march.hip)
void launch_loss_alpha_list(hipStream_t s, uint32_t cap_samples, const uint32_t* n_ptr, const uint32_t* idx, const float* coords,
                            const half_t* net_out, float cos_anneal, const LossWork& w, bool dt_const = false);
// rays_in / *n_rays_in: the rays still open (rounds after the first; nullptr: every ray slot); rays_out / n_rays_out: the
// rays that stay open, for the next round (nullptr in the last round, with list)
// the compaction cut of the progressive rounds (march.hip k_prog_cut / k_prog_next)
// mode 0: after round 0's pass A (split sort): cutw[CW_CUT_A], and pass B's counts cutw[CW_LENB_EFF] / [CW_NB_EFF] (0 when the
// cut lies in pass A's slots); mode 1: the final cut cutw[CW_CUT], the next step's split estimate cutw[CW_EST], and pass B's
// evaluated samples added to *eval0 (null: none)
void launch_prog_cut(hipStream_t s, uint32_t cap_rays, const uint32_t* ccount, const uint32_t* excl, uint32_t batch, uint32_t* cutw, int mode,
                     uint32_t* eval0, uint32_t* abort_if_none = nullptr);
// launch_exclusive_scan(ccount -> excl) and launch_prog_cut in one launch (the look-back scan's state in scan_temp)
void launch_scan_prog_cut(hipStream_t s, void* scan_temp, const uint32_t* ccount, uint32_t* excl, uint32_t n, uint32_t batch, uint32_t* cutw, int mode,
                          uint32_t* eval0, uint32_t* abort_if_none = nullptr);
void launch_prog_next(hipStream_t s, uint32_t cap_rays, const uint32_t* rays_in, const uint32_t* n_in, const uint32_t* numsteps, const uint32_t* cut,
                      uint32_t e1, uint32_t e2, uint32_t* list, uint32_t* list_counter, uint32_t* rays_out, uint32_t* n_out);
void launch_loss_scan_chunk(hipStream_t s, uint32_t cap_rays, const uint32_t* numsteps, const LossWork& w, uint32_t* ccount, uint32_t e0,
                            uint32_t e1, uint32_t e2, uint32_t* list /* nullptr in the last round */, uint32_t* next_counter,
                            const uint32_t* rays_in = nullptr, const uint32_t* n_rays_in = nullptr, uint32_t* rays_out = nullptr,
                            uint32_t* n_rays_out = nullptr);
void launch_srgb_lut(hipStream_t s, float* lut);
void launch_loss_ray(hipStream_t s, uint32_t cap_rays, StepState* st, DPInfo dp, const DevDataset& ds, const LossParams& lp, uint32_t* numsteps,
                     const uint32_t* ccount, const uint32_t* cbase, const LossWork& w, float* loss, float* ek, float* mask);
void launch_loss_grad(hipStream_t s, uint32_t cap_samples, StepState* st, DPInfo dp, const LossParams& lp, const float* coords,
                      const half_t* net_out, const uint32_t* numsteps, const LossWork& w, float* coords_out, half_t* dL_dout);
void debug_launch_loss_scan(hipStream_t s, int variant, uint32_t cap_rays, const uint32_t* numsteps, const LossWork& w, uint32_t* ccount);
void launch_ray_index(hipStream_t s, uint32_t cap_rays, const uint32_t* numsteps, StepState* st, uint32_t* sample_ray, uint32_t* rbase);
void launch_rollover(hipStream_t s, uint32_t n_elements, const StepState* st, float* coords, half_t* dL_dout);
void launch_step_counters(hipStream_t s, StepState* st, uint32_t target_batch, uint32_t max_samples, uint32_t world, uint32_t fixed_rays,
                          const uint32_t* eval_cnt = nullptr, uint32_t n_eval = 0, uint32_t* abort_host = nullptr);
// render.hip (rays: RenderRay records, render_ray_bytes() each)
size_t render_ray_bytes();
void launch_render_init(hipStream_t s, const RenderCamera& cam, uint32_t sample_index, const DevDataset& ds, const uint8_t* bf, const uint32_t* lin,
                        void* rays, float4* frame);
void launch_render_compact(hipStream_t s, uint32_t n, const void* src, uint32_t* flags, uint32_t* base, void* dst, uint32_t* n_alive,
                           void* scan_tmp, size_t scan_tmp_bytes);
void launch_render_gen(hipStream_t s, uint32_t n_alive, uint32_t n_steps, const DevDataset& ds, const uint8_t* bf, const uint32_t* lin, void* rays,
                       float* coords);
void launch_render_composite(hipStream_t s, uint32_t n_alive, uint32_t n_steps, const float* coords, const half_t* net_out, float cos_anneal,
                             float min_transmittance, bool linear_colors, void* rays, float4* frame);
void launch_render_accumulate(hipStream_t s, uint32_t n, uint32_t spp, const float4* frame, float4* accum);
// mc.hip (marching cubes over a density grid; chunked, deterministic)
uint32_t mc_n_chunks(const uint32_t res[3]);
void mc_table_host(int8_t* out /* 256 x 19 */);
void launch_mc_count(hipStream_t s, const uint32_t res[3], const float amin[3], const float amax[3], float thresh, const float* density,
                     uint32_t* cnt_v, uint32_t* cnt_t);
void launch_mc_emit(hipStream_t s, const uint32_t res[3], const float amin[3], const float amax[3], float thresh, const float* density,
                    const uint32_t* off_v, const uint32_t* off_t, float* verts, uint32_t* vidx, uint32_t* tris);
void launch_mesh_coords(hipStream_t s, uint32_t n, const float* verts, const DevDataset& ds, float* coords);
// transform_mesh_with_6d (testbed_nerf.cu:109-138): v' = R^-1 (v - t) with the accumulated movement
void launch_mesh_unmove(hipStream_t s, uint32_t n, const RayMotion& m, float* verts);
// motion.hip (dynamic scenes)
void launch_delta_prepare(hipStream_t s, DeltaState* ds);
void launch_delta_apply(hipStream_t s, const uint32_t* n_ptr, uint32_t n_cap, uint32_t stride, const float* in, float* out, const DeltaState* ds);
void launch_delta_backward(hipStream_t s, const uint32_t* n_ptr, uint32_t n_cap, const float* coords, uint32_t stride, const float4* dpos,
                           DeltaState* ds, float* partial, const DeltaAdam& a);
// the two halves of launch_delta_backward (a data-parallel step all-reduces the partial sums in between)
void launch_delta_grad(hipStream_t s, const uint32_t* n_ptr, uint32_t n_cap, const float* coords, uint32_t stride, const float4* dpos,
                       const DeltaState* ds, float* partial);
void launch_delta_step(hipStream_t s, const float* partial, DeltaState* ds, const DeltaAdam& a);
size_t delta_partial_floats();
void host_accumulate_movement(const float delta_p[DELTA_PARAMS], float accR[9], float acct[3]);
// scan.hip
size_t scan_temp_bytes(uint32_t n);
// zero the look-back state at the start of a scan temp buffer once after allocating it; scan_failures reads its
// bounded-wait failure count (0 unless the state was corrupted)
void scan_temp_reset(hipStream_t s, void* temp);
// the look-back tag of the next scan launch on this temp buffer (scan.hip; used by the fused scans of march.hip)
uint32_t scan_next_tag(void* temp);
uint32_t scan_failures(void* temp);
void scan_temp_release(void* temp);  // forget the buffer's tag counter (it is being freed)
// tests: the scan with its first tile never published, so every later tile's look-back gives up (a failure count)
void debug_scan_skip_first_tile(hipStream_t s, void* temp, const uint32_t* in, uint32_t* out, uint32_t n);
void launch_exclusive_scan(hipStream_t s, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n);
void launch_sum_f32(hipStream_t s, void* temp, size_t temp_bytes, const float* in, float* out, uint32_t n);
// optim.hip
void launch_adam_ema(hipStream_t s, const AdamParams& p, float* weights_fp, half_t* weights_h, const float* grads, float* m1, float* m2,
                     void* steps, bool steps32, float* ema_tmp, half_t* ema_h,
                     const StepCounterArgs* counters = nullptr, const AdamTranspose* tr = nullptr);
// Ema(Adam) over the parameters [lo, hi) of a p.n-parameter vector (lo % 4 == 0): the optimizer step in pieces, each as
// soon as its gradient range is final (NeusTestbed::adam_overlap); no step counters on these launches
void launch_adam_ema_range(hipStream_t s, AdamParams p, uint32_t lo, uint32_t hi, float* weights_fp, half_t* weights_h, const float* grads,
                           float* m1, float* m2, void* steps, bool steps32, float* ema_tmp, half_t* ema_h, const AdamTranspose* tr);
void launch_cast_half(hipStream_t s, uint32_t n, const float* in, half_t* out);
void launch_add_f32(hipStream_t s, uint32_t n, const float* src, float* dst);
// operator-module encoding helpers (grid.hip)
void launch_enc_input_grad(hipStream_t s, uint32_t n, uint32_t ld, uint32_t L, const half_t* dLdy, const float* dydx, float* dLdx, uint32_t stride);
void launch_enc_ddLdoutput(hipStream_t s, uint32_t n, uint32_t ld, uint32_t L, const float* ddx, const float* dydx, half_t* out, float4* v4);
// encoding output layouts of the operator module: paired [L][n] half2 <-> AoS [n][2L] / SoA [2L][n] fp16
enum : uint32_t { ENC_LAYOUT_AOS = 0, ENC_LAYOUT_SOA = 1, ENC_LAYOUT_PAIRED = 2 };
void launch_enc_to_layout(hipStream_t s, uint32_t n, uint32_t L, const uint32_t* paired, half_t* dst, uint32_t layout);
void launch_enc_from_layout(hipStream_t s, uint32_t n, uint32_t L, const half_t* src, uint32_t layout, uint32_t* paired);
// fp32 HashGrid (grid_f32.hip): create_encoding with requested_precision = fp32 (cpp_api.cu:174-180)
void launch_grid_f32_forward(hipStream_t s, uint32_t n, const GridLevels& gl, uint32_t valid_level, const float* coords, const float* table,
                             float* out, uint32_t layout, float* dydx);
void launch_grid_f32_backward(hipStream_t s, uint32_t n, const GridLevels& gl, uint32_t valid_level, const float* coords, const float* dLdy,
                              uint32_t layout, float* grads, const float* dydx, float* dLdx);
void launch_grid_f32_bbi(hipStream_t s, uint32_t n, const GridLevels& gl, uint32_t valid_level, const float* coords, const float* ddx,
                         const float* dLdy, uint32_t layout, float* grads, const float* dydx, float* ddLdy);
// paired [L][n] <-> sample rows [n][ld] (features in columns [0, 2L), zero padding up to ld): a FullyFusedMLP's input
void launch_enc_to_rows(hipStream_t s, uint32_t n, uint32_t L, const uint32_t* paired, half_t* rows, uint32_t ld);
void launch_enc_from_rows(hipStream_t s, uint32_t n, uint32_t L, const half_t* rows, uint32_t ld, uint32_t* paired);
void launch_grad_to_half(hipStream_t s, uint32_t n, const float* g, half_t* out, bool accumulate);
void launch_transpose_w(hipStream_t s, const TransposeJobs& jobs);
struct DinPerm { int32_t p[48]; uint32_t din, W; };
void launch_permute_din(hipStream_t s, const half_t* d0, half_t* d0p, half_t* d0Tp, const DinPerm& perm);
void launch_transpose_permute(hipStream_t s, const TransposeJobs& jobs, const half_t* d0, half_t* d0p, half_t* d0Tp, const DinPerm& perm);
// samples [i_begin, i_end) of an n-sample generate_grid_samples_nerf_nonuniform call, written from out_base
void launch_grid_samples(hipStream_t s, uint32_t n, uint32_t i_begin, uint32_t i_end, uint32_t out_base, uint64_t rng_state, uint64_t rng_inc,
                         uint32_t step, const float* aabb_min, const float* aabb_max, const float* grid_in, float* pos, uint32_t* indices,
                         uint32_t n_cascades, float thresh, const PcgJumpTable& jt);
void launch_splat_max(hipStream_t s, uint32_t n, const uint32_t* indices, const float* density, float* grid_tmp);
void launch_ema_grid(hipStream_t s, uint32_t n, float decay, float* grid, const float* tmp);
void launch_grid_mean(hipStream_t s, const float* grid, float* partial, float* mean);
void launch_bitfield(hipStream_t s, const float* grid, uint8_t* bitfield, const float* mean, uint32_t n_cascades,
                     uint32_t* lin = nullptr /* also the march's linear mip-0 words */);
// EMA of the grid + its cascade-0 mean (n multiple of 1024)
void launch_ema_mean(hipStream_t s, uint32_t n, float decay, float* grid, const float* tmp, float* partial, float* mean);

} // namespace neus
