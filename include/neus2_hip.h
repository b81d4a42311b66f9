/*
 * neus2_hip.h — C-ABI drop-in boundary of the MI355X (gfx950) NeuS2 training hot path.
 *
 * Plain pointers and sizes only (no torch / STL types). Every entry point returns an int
 * status (0 = ok, nonzero = error; neus_last_error() gives the message), mirroring the
 * reference's C++ exceptions that pybind11 turns into Python RuntimeError.
 *
 * Each entry point replaces one interface of the reference (zbqq/neus2 @ /root/reference):
 *
 *   Testbed surface (include/neural-graphics-primitives/testbed.h:63-940, src/python_api.cu:216-600)
 *     neus_testbed_create              Testbed::Testbed                       src/testbed.cu:2583-2632
 *     neus_testbed_set_dataset         Testbed::load_training_data -> load_nerf src/testbed_nerf.cu:2964-3095
 *                                      (images/cameras decoded by the host mirror, nerf_loader.cu:197-751)
 *     neus_testbed_reload_network      Testbed::reload_network_from_json -> reset_network src/testbed.cu:2084-2349
 *     neus_testbed_train               Testbed::train(batch) x n_steps        src/testbed.cu:2640-2736
 *     neus_testbed_get_stats           Testbed::m_training_step / m_loss_scalar / counters (python_api.cu:447-449)
 *     neus_testbed_{get,set}_params    Trainer params / serialize             trainer.h:72-109, 281-300
 *     neus_testbed_{get,set}_density_grid  Nerf::density_grid(_bitfield)      testbed.h:688-694
 *     neus_testbed_restore_state       Testbed::load_snapshot (counters, step, loss, grid bitfield)  testbed.cu:3197-3254
 *     neus_testbed_render              Testbed::render_to_cpu -> render_nerf / NerfTracer::trace  python_api.cu:123-169, testbed_nerf.cu:2397-2760
 *     neus_testbed_sdf_on_grid         Testbed::get_density_on_grid          testbed_nerf.cu:4096-4139
 *     neus_testbed_marching_cubes      Testbed::marching_cubes / marching_cubes_gpu  testbed_nerf.cu:4175-4226, marching_cubes.cu:794-822
 *     neus_testbed_get_mesh            Testbed::compute_marching_cubes_mesh (V, F)   python_api.cu:99-121
 *     neus_testbed_init_data_parallel  (new) RCCL data parallelism over ray batches
 *
 *   Operator surface (my_tcnn DifferentiableObject / cpp_api.h:66-106 for the NerfNetwork, plus
 *   the NeuS step kernels of src/testbed_nerf.cu), on caller-owned device buffers:
 *     neus_net_forward                 NerfNetwork::forward_impl               nerf_network.h:145-328
 *     neus_net_backward                NerfNetwork::backward_impl (Overwrite)  nerf_network.h:330-654
 *     neus_grid_encode                 GridEncoding forward (kernel_grid)      grid.h:174-369
 *     neus_sample_rays                 generate_training_samples_nerf_with_global_movement  testbed_nerf.cu:1263-1456
 *     neus_loss_compact                compute_loss_kernel_train_nerf_with_global_movement  testbed_nerf.cu:1475-1997
 *     neus_optimizer_step              Trainer::optimizer_step (Ema/ExpDecay/Adam)          trainer.h:170-172
 *     neus_occ_update                  Testbed::update_density_grid_nerf                    testbed_nerf.cu:3293-3397
 *
 * Layouts (DESIGN.md §Data layout): coords AoS 7 x f32 (pos[3], dt, dir[3]) per sample;
 * network output / dL/doutput AoS 16 x fp16 per sample; params fp32 [P] in the reference's
 * set_params order [density MLP | rgb MLP | grid | variance(4)].
 */
#ifndef NEUS2_HIP_H
#define NEUS2_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct NeusTestbed NeusTestbed;

/* configs/nerf/base.json surface, parsed by the host mirror (neus2_amd/pyngp.py). */
typedef struct NeusNetworkConfig {
	/* encoding (grid.h GridEncodingTemplated; testbed.cu:2151-2197) */
	uint32_t n_levels;
	uint32_t n_features_per_level;   /* must be 2 */
	uint32_t log2_hashmap_size;
	uint32_t base_resolution;
	float per_level_scale;           /* derived as testbed.cu:2185 when <= 0 */
	float top_resolution;
	float valid_level_scale;         /* progressive levels, grid.h:2427-2440 */
	float base_valid_level_scale;
	uint32_t base_training_step;
	/* networks (nerf_network.h:53-96): FullyFusedMLP, ReLU, no output activation */
	uint32_t n_neurons;              /* 16, 32 or 64 */
	uint32_t n_density_hidden;       /* must be 1 on the GPU path */
	uint32_t n_rgb_hidden;           /* must be 2 on the GPU path */
	/* optimizer: Ema(decay) -> ExponentialDecay -> Adam */
	float learning_rate, beta1, beta2, epsilon, l2_reg;
	float ema_decay;
	uint32_t decay_start, decay_interval;
	float decay_base;
	/* hyperparams (testbed.cu:2115-2137) */
	float ek_loss_weight, mask_loss_weight;
	uint32_t anneal_end;
	uint32_t batch_size;             /* target compacted samples per step (2^18) */
	float sdf_bias;                  /* -0.1 (nerf_network.h:87) */
	float density_grid_decay;        /* 0.95 (testbed.h:659) */
	uint32_t seed;                   /* 1337 (testbed.h:524) */
	uint32_t fixed_rays_per_batch;   /* 0 = adaptive R (reference); >0 freezes R (benchmarks) */
	/* dynamic scenes (testbed.cu:2115-2133, base.json "hyperparams" / "globalmove") */
	uint32_t predict_global_movement;          /* hyperparams.predict_global_movement */
	uint32_t global_movement_steps;            /* predict_global_movement_training_step (50) */
	uint32_t finetune_global_movement;         /* keep training the movement with the canonical network */
	uint32_t reset_density_grid_after_global_movement;
	float after_learning_rate;                 /* Adam learning rate for frames >= 1 */
	float gm_learning_rate, gm_beta1, gm_beta2, gm_epsilon;   /* globalmove optimizer: ExponentialDecay(Adam) */
	uint32_t gm_decay_start, gm_decay_interval;
	float gm_decay_base;
} NeusNetworkConfig;

typedef struct NeusImage {
	int32_t width, height;
	const uint32_t* rgba8;           /* host pointer, width*height packed RGBA8 (R in the low byte) */
	float focal[2];                  /* pixels */
	float principal[2];              /* normalized [0,1] */
	float xform[12];                 /* camera-to-world 3x4 row-major, ngp convention (nerf_loader.h:112-134) */
} NeusImage;

typedef struct NeusTrainStats {
	uint32_t training_step;
	uint32_t rays_per_batch;
	uint32_t measured_batch_size;            /* compacted samples of the last step (Nc, per rank) */
	uint32_t measured_batch_size_before_compaction; /* Npre requested, per rank */
	uint32_t n_rays_total;
	uint32_t valid_level;
	uint32_t zero_records;
	float loss;                               /* m_loss_scalar (EMA as the reference) */
	float ek_loss;
	float mask_loss;
	float last_loss;                          /* last raw loss scalar */
	float density_grid_mean;
	float ray_loss;                           /* mean Huber loss over the rays that had samples (last logged step) */
	uint32_t n_rays_with_samples;             /* rays kept by the sampler in the last logged step */
	uint64_t trained_samples_total;           /* compacted (non-rollover) training samples since step 0, per rank */
	uint32_t march_first_pass_rays;           /* ray slots the next step's first march pass covers (0 = all) */
	uint32_t kept_ray_extent;                 /* 1 + the last ray slot kept by the last step's sampler */
	uint32_t nonfinite_loss;                  /* a logged loss sum was NaN / Inf (all-reduced, so every rank sees it) */
	uint32_t training_aborted;                /* zero compacted samples (testbed_nerf.cu:3542-3548) or a non-finite loss */
	/* work since the network was (re)loaded, this rank (the whole-step roofline of bench.py counts bytes from them) */
	uint64_t pre_samples_total;               /* pre-compaction samples evaluated (sum of the kept samples per step) */
	uint64_t rays_total;                      /* rays marched (sum of rays_per_batch) */
	uint64_t occ_samples_total;               /* occupancy-grid samples evaluated by this rank (its shard of each update) */
	uint32_t occ_updates;                     /* occupancy-grid updates (update_density_grid_nerf calls) */
	uint32_t health_flags;                    /* device health bits (sticky): 1 the occupancy march met a non-finite / negative t,
	                                           * 2 a look-back scan gave up waiting; either makes neus_testbed_train fail */
	uint64_t evaluated_samples_total;         /* samples the pre-compaction network pass evaluated (progressive inference: the
	                                           * rounds' work lists, a subset of the kept samples) */
	uint64_t progressive_steps;               /* steps that ran progressive (multi-round) inference */
	uint32_t evaluated_samples_last;          /* samples the last step's pre-compaction pass evaluated */
	uint32_t progressive_chunk_end;           /* end of the progressive inference's first chunk (the rounds are [0, e), [e, 2e), ...
	                                           * by default; neus_testbed_set_progressive_inference) */
	uint64_t lookahead_steps;                 /* (ABI 5) steps whose ray sampling was issued beside the step before them */
	uint64_t adam_split_steps;                /* (ABI 5) steps whose optimizer ran in pieces beside the scatter (adam_overlap) */
	uint64_t cut_steps;                       /* (ABI 5) steps whose later progressive rounds skipped the rays past the
	                                           * compaction cut (fixed rays per batch; never a step the host reads back) */
	uint64_t march_cut_steps;                 /* (ABI 6) steps whose ray sampling marched only the slots below the compaction cut's
	                                           * estimate (NEUS_MARCH_CUT) */
	uint64_t march_cut_reruns;                /* (ABI 6) steps run again with the full march because the witness of a cut march failed
	                                           * (nothing of the first run was applied) */
} NeusTrainStats;

/* Testbed::render_to_cpu (python_api.cu:123-169) after set_camera_to_training_view (testbed.cu:264-270). */
typedef struct NeusRenderRequest {
	int32_t width, height;
	uint32_t spp;                    /* samples per pixel, accumulated in linear colour (render_buffer.cu:217-260) */
	int32_t training_view;           /* >= 0: the camera of this training image; < 0: xform/focal/screen_center below */
	float xform[12];                 /* camera-to-world 3x4 row-major (ngp convention) */
	float focal[2];                  /* pixels at width x height */
	float screen_center[2];          /* normalized principal point */
	int32_t snap_to_pixel_centers;   /* render_utils.py:272 sets it for evaluation */
	float min_transmittance;         /* nerf.rendering_min_transmittance (render_utils.py:275: 1e-4) */
	int32_t use_ema;                 /* 1: inference params = EMA weights (the reference); 0: training weights */
} NeusRenderRequest;

typedef struct NeusNetLayout {
	uint64_t n_params, n_density, n_rgb, grid_offset, n_grid_params, variance_offset, n_matrix;
	uint32_t density_input_width, rgb_input_width;
	float per_level_scale;           /* derived per_level_scale actually used (testbed.cu:2185) */
	uint32_t n_levels;
} NeusNetLayout;

/* ABI version of this header (bumped on any incompatible signature or struct change; version 2: neus_module_create_network
 * became tcnn's create_network(n_input_dims, n_output_dims, network), the NerfNetwork factory neus_module_create_nerf_network;
 * version 3: NeusDataParallelInfo gained host_group; version 4: neus_module_create_encoding gained requested_precision;
 * version 5: neus_testbed_{set_,}exchange_timing, neus_host_group_create gained job_token; version 6: NeusTrainStats gained
 * march_cut_steps and march_cut_reruns).
 * Bindings compare it on load so that a stale library or binding fails loudly instead of misreading arguments. */
#define NEUS_ABI_VERSION 6u
int neus_abi_version(uint32_t* out);
const char* neus_last_error(void);
int neus_device_count(int* count);
int neus_device_synchronize(void);

/* ------------------------------------------------------------------ Testbed */
int neus_testbed_create(int device, NeusTestbed** out);
int neus_testbed_destroy(NeusTestbed* tb);
int neus_testbed_set_dataset(NeusTestbed* tb, uint32_t n_images, const NeusImage* images, float aabb_scale);
int neus_testbed_reload_network(NeusTestbed* tb, const NeusNetworkConfig* cfg, const float* geometric_init /* nullable: n_density floats */);
int neus_testbed_layout(NeusTestbed* tb, NeusNetLayout* out);
int neus_testbed_train(NeusTestbed* tb, uint32_t n_steps);
int neus_testbed_get_stats(NeusTestbed* tb, NeusTrainStats* out);
int neus_testbed_get_params(NeusTestbed* tb, float* host_out, uint64_t n);
int neus_testbed_set_params(NeusTestbed* tb, const float* host_in, uint64_t n);
int neus_testbed_get_gradients(NeusTestbed* tb, float* host_out, uint64_t n);
int neus_testbed_get_ema_params(NeusTestbed* tb, float* host_out, uint64_t n);
/* The fp16 parameter copies the kernels read (network_precision_t params, trainer.h:72-109): which = 0 training
 * weights, 1 inference (EMA) weights (Ema::custom_weights, ema.h:45-110). host_out: n fp16 bit patterns. */
int neus_testbed_get_half_params(NeusTestbed* tb, int which, uint16_t* host_out, uint64_t n);
int neus_testbed_get_density_grid(NeusTestbed* tb, float* grid_out /*128^3*/, uint8_t* bitfield_out /*128^3/8*8*/);
int neus_testbed_set_density_grid(NeusTestbed* tb, const float* grid /*nullable*/, const uint8_t* bitfield /*nullable*/);
/* Testbed::load_snapshot's non-parameter state (testbed.cu:3210-3248), applied after reload_network + set_params +
 * set_density_grid: training step, loss scalar, counters_rgb; the inference (EMA) weights := the loaded weights
 * (Trainer::set_params, trainer.h:72-109); rebuild_bitfield != 0 recomputes the grid mean and occupancy bitfield
 * from the density grid (update_density_grid_mean_and_bitfield). */
typedef struct NeusRestoreState {
	uint32_t training_step;
	uint32_t rays_per_batch;                  /* multiple of 128, <= 2^18 */
	uint32_t measured_batch_size;
	uint32_t measured_batch_size_before_compaction;
	float loss;
	int32_t rebuild_bitfield;
} NeusRestoreState;
int neus_testbed_restore_state(NeusTestbed* tb, const NeusRestoreState* state);
/* rgba_out: height*width*4 floats, linear colour, premultiplied alpha (the reference's render(..., linear=True)).
 * n_iterations (nullable): march/composite iterations of the last spp. */
int neus_testbed_render(NeusTestbed* tb, const NeusRenderRequest* req, float* rgba_out, uint32_t* n_iterations);
/* get_density_on_grid (testbed_nerf.cu:4096-4139): raw SDF (inference/EMA weights) at the res[0]*res[1]*res[2]
 * points x/res * (aabb_max - aabb_min) + aabb_min, x fastest; host_out gets the floats. */
int neus_testbed_sdf_on_grid(NeusTestbed* tb, const int32_t res[3], const float aabb_min[3], const float aabb_max[3], float* host_out);
/* Testbed::marching_cubes (testbed_nerf.cu:4175-4226): res rounded up to multiples of 16, SDF grid, mesh at
 * `thresh` (0 for NeuS). With density_dev (device pointer, res^3 floats, x fastest) the grid is taken as
 * given and res is used unrounded. Deterministic vertex / triangle order. */
int neus_testbed_marching_cubes(NeusTestbed* tb, const int32_t res[3], const float aabb_min[3], const float aabb_max[3], float thresh,
                                const float* density_dev, uint32_t* n_verts, uint32_t* n_tris);
/* Grid points [offset, offset + count) (linear index, x fastest) of the SDF grid the last network marching_cubes
 * computed (get_density_on_grid), to host floats: sub-block checks of large (1024^3) grids. */
int neus_testbed_mc_density(NeusTestbed* tb, uint64_t offset, uint64_t count, float* host_out);
/* The last mesh: verts n_verts x 3 f32, tris n_tris x 3 u32 (host buffers, nullable). */
int neus_testbed_get_mesh(NeusTestbed* tb, float* verts, uint32_t* tris);
/* compute_mesh_vertex_colors (testbed_nerf.cu:4071-4094): n_verts x 3 f32 sRGB colours of the last mesh. */
int neus_testbed_mesh_vertex_colors(NeusTestbed* tb, float* rgb);
/* The marching-cubes case table the kernels use: 256 rows x 19 int8 (edge triples, -1 terminated). */
int neus_mc_table(int8_t* out);
/* Training-image preparation of ngp::load_nerf (host side, in the reference's order), in place on w x h RGBA8:
 *   alpha_rgba (nullable, w x h RGBA8: the frame's `<file_path>.alpha.<ext>` image): alpha := uint8(255 *
 *     srgb_to_linear(red / 255)) (nerf_loader.cu:550-569);
 *   mask_rgba (nullable, w x h RGBA8: the frame's `dynamic_mask_<basename>.png`): pixels whose mask red is nonzero
 *     become the hot-pink key 0x00FF00FF, which read_rgba turns into a masked-away (negative) target
 *     (nerf_loader.cu:571-590, common_device.cuh:635-667);
 *   flags NEUS_IMAGE_WHITE_TRANSPARENT / NEUS_IMAGE_BLACK_TRANSPARENT (transforms.json `white_transparent` /
 *     `black_transparent`): alpha := 0 on pure white / pure black rgb, then the mask key is re-applied
 *     (convert_rgba32, nerf_loader.cu:59-81, applied by NerfDataset::set_training_image).
 * Returns in *mask_color the key the image carries (0x00FF00FF with a mask, else 0). */
#define NEUS_IMAGE_WHITE_TRANSPARENT 1u
#define NEUS_IMAGE_BLACK_TRANSPARENT 2u
int neus_prepare_image_rgba8(uint8_t* rgba, uint32_t width, uint32_t height, const uint8_t* alpha_rgba, const uint8_t* mask_rgba,
                             uint32_t flags, uint32_t* mask_color);
int neus_testbed_get_rng(NeusTestbed* tb, uint64_t* state_inc /*4: rng, density_grid_rng*/);
/* Dynamic scenes. Testbed::training_network_next_frame (testbed.cu:2001-2082) with load_nerf(frame)
 * (testbed_nerf.cu:3096-3113): the next frame's images/cameras (same aabb), the frame's local movement folded
 * into the accumulated ray transform (accumulate_global_movement, nerf_network.h:1163-1177), training
 * weights := inference (EMA) weights (save/load_snapshot_incremental, testbed.cu:3180-3266), fresh optimizer and
 * global-move trainer state, m_rng reset, training step 0, canonical training off for global_movement_steps. */
int neus_testbed_next_frame(NeusTestbed* tb, uint32_t n_images, const NeusImage* images);
/* Movement state. global12: accumulated rotation (3x3 row-major) + translation (testbed_nerf.cu:193-213);
 * local12: DeltaNetwork params, transition[4] | rotation 6D[8] (transform_network.h:313-333). Each nullable. */
int neus_testbed_get_movement(NeusTestbed* tb, float* global12, float* local12);
int neus_testbed_set_movement(NeusTestbed* tb, const float* global12, const float* local12);
/* frame_state (4 u32): current frame, canonical training step, train_canonical, train_delta. */
int neus_testbed_frame_state(NeusTestbed* tb, uint32_t* out4);
/* Testbed::change_to_frame (testbed.cu:1939-1985; python_api.cu:437): frame index := frame, that frame's images and
 * cameras (load_nerf(frame)), training step 0 and a fresh optimizer (Adam moments / steps / EMA state); the
 * parameters, the accumulated movement and the phase flags stay (run_dynamic.py then calls load_snapshot). */
int neus_testbed_change_frame(NeusTestbed* tb, uint32_t frame, uint32_t n_images, const NeusImage* images);
/* Testbed::prepare_for_test (testbed.cu:1987-1999; python_api.cu:438): render, SDF grid and mesh colours go through
 * the DeltaNetwork (m_use_delta) iff current frame != 0 and train_delta. Each training step sets the same flag
 * (testbed.cu:2704-2710). out_use_delta (nullable) receives it. */
int neus_testbed_prepare_for_test(NeusTestbed* tb, int* out_use_delta);
/* Testbed::save_transform's values (testbed.cu:3118-3141, save_global_movement_rotation_6d_kernel,
 * common_operation.cuh:588-623): the current frame's DeltaNetwork movement composed with the accumulated one,
 * R = R_local R_acc (row-major 9) and t = R_local (t_acc + t_local) (3), rounded to fp16 (precision_t). */
int neus_testbed_saved_transform(NeusTestbed* tb, float* out12);

/* Loss-target and sampling options (testbed.h Nerf::Training; python_api.cu:530-560):
 *   random_bg_color      nerf.training.random_bg_color (1, the default: a random background per ray)
 *   background_color     testbed.background_color rgb (sRGB) - the fixed training background otherwise
 *   color_space          testbed.color_space: 0 Linear (default), 1 SRGB (testbed_nerf.cu:1657-1671)
 *   linear_colors        nerf.training.linear_colors: targets and rendering stay linear
 *   cone_angle_constant  nerf.cone_angle_constant (load_nerf sets 0 for aabb_scale 1, else 1/256)
 *   near_distance        nerf.training.near_distance (stored; the NeuS sampler does not read it)
 *   depth_supervision_lambda  nerf.training.depth_supervision_lambda (python_api.cu:555; stored: the reference computes
 *                        the depth term, testbed_nerf.cu:1697-1698 / 1836, and adds it to no gradient or loss) */
typedef struct NeusTrainingOptions {
	int32_t random_bg_color;
	float background_color[3];
	int32_t color_space;
	int32_t linear_colors;
	float cone_angle_constant;
	float near_distance;
	float depth_supervision_lambda;
} NeusTrainingOptions;
int neus_testbed_get_training_options(NeusTestbed* tb, NeusTrainingOptions* out);
/* Trainer::serialize(include_optimizer_state) / deserialize (trainer.h:281-305): the Ema(ExponentialDecay(Adam))
 * state - Adam current_step, first / second moments, per-parameter steps (adam.h:424-445), the decay's learning
 * rate and factor (exponential_decay.h:128-140), the fp16 EMA weights (ema.h:182-194; the fp32 accumulator is
 * rebuilt from them on set). Arrays are n_params long, host memory, nullable on get; steps nullable on set.
 * Per-parameter steps (uint32 in the reference): when the betas' bias correction has converged to 1.0f by step 4096
 * (beta^4095 < 2^-30: the default betas 0.9 / 0.99), the device keeps them in 16 bits and they saturate at 65535 - every
 * count past 4095 gives the same update, so training is unchanged, but a count above 65535 reads back as 65535. With
 * betas whose correction has not converged there, they are kept in 32 bits and round-trip exactly. */
typedef struct NeusOptimizerState {
	uint32_t n_params;
	uint32_t current_step;
	float learning_rate;
	float learning_rate_factor;
} NeusOptimizerState;
int neus_testbed_get_optimizer_state(NeusTestbed* tb, NeusOptimizerState* st, float* m1, float* m2, uint32_t* steps, uint16_t* ema_half);
int neus_testbed_set_optimizer_state(NeusTestbed* tb, const NeusOptimizerState* st, const float* m1, const float* m2, const uint32_t* steps,
                                     const uint16_t* ema_half);
int neus_testbed_set_training_options(NeusTestbed* tb, const NeusTrainingOptions* opts);
/* Progressive (cut-off-aware) inference of the training step: the network runs in rounds over per-ray sample chunks
 * [0, e_0), [e_0, e_1), ..., [e_last, end) and a ray's next chunk only while its transmittance is >= 1e-4, so samples
 * past the cut-off (never read by the loss) are not evaluated; bit-identical to one pass. mode 0 off, 1 auto (on when
 * under 70 % of the kept samples were composited at the last loss readback; the default), 2 always. chunk_ends
 * (strictly increasing, at most 14; nullable to keep the current ones): given, they are fixed from then on; by default
 * they follow the training state (three rounds {e, 2e, rest}, e from the mean composited samples per ray at each loss
 * readback). A performance option of this implementation (no reference counterpart:
 * testbed_nerf.cu:3802-3811 infers every kept sample). */
int neus_testbed_set_progressive_inference(NeusTestbed* tb, int mode, const uint32_t* chunk_ends, uint32_t n_ends);
/* Per-ray counters of the last step (first n rays, host buffers, each nullable): samples requested by
 * the march, samples composited before transmittance < 1e-4, and numsteps = (compacted count, base). */
int neus_testbed_ray_counts(NeusTestbed* tb, uint32_t n, uint32_t* nreq, uint32_t* ccount, uint32_t* numsteps /* 2n */);
/* Development timing hook: regenerates the last step's samples and times `iters` launches of one
 * kernel (the ids of neus_testbed_time_kernel; 11 the level-major encode alone over the pre-compaction samples,
 * variant = workgroups per level; 12 the Adam / EMA pass, which advances the optimizer) in implementation
 * `variant` (0 = production; 99 = no re-preparation); median ms per launch. */
int neus_debug_time_kernel(NeusTestbed* tb, int kernel, int variant, int iters, float* ms_out);
/* Median launch duration (hipEvents on the testbed stream between `iters` back-to-back launches) of one hot-path
 * kernel replayed on the current training state, and the work units of one launch.
 * kernel: 0 ray generation + march (units: ray slots), 1 coordinate write, 2 loss transmittance scan,
 * 3 fused inference, 4 loss alpha (units: pre-compaction samples), 5 training MLP, 6 weight gradients,
 * 7 grid-gradient scatter, 8 training-batch grid encode, 9 / 10 the colour / density training-MLP kernel alone
 * (units: compacted samples), 12 the Adam / EMA pass (units: parameters; the replays advance the optimizer), 13 ray
 * generation + march of a cut step (the march cut: only the slots below the compaction cut's estimate; units: those
 * slots; it leaves the state of a cut march behind, so it goes after the other replays). */
int neus_testbed_time_kernel(NeusTestbed* tb, int kernel, int iters, float* ms_out, uint32_t* units_out);
// Development statistic of the last step's march: per ray {march_step calls, skip-loop additions,
// samples} (3 x u32 per ray, n rays; cone_angle 0 only).
int neus_debug_march_stats(NeusTestbed* tb, uint32_t n, uint32_t* out);
/* Development timing of the occupancy march (ray generation + both passes on the current state): per wave of the
 * first pass, 8 u64 = wall-clock stamps (100 MHz) at start, slice start reached, segment marched, segments joined,
 * samples counted, records written, then the wave's samples and its re-march rounds; pass 1 overwrites its waves'
 * stamps only where it marches. */
int neus_debug_march_profile(NeusTestbed* tb, unsigned long long* out, uint32_t max_waves, uint32_t* n_waves);
/* Development statistic of the last grid-gradient scatter (region mode): records written per level (out[L], after the
 * wave run merge) and the largest per-(level, block) region. */
int neus_debug_scatter_stats(NeusTestbed* tb, uint64_t* records_per_level, uint32_t* max_region);
/* The region scatter's job plan: per level, the workgroups one level-local bucket is split over (1: not split; the heavy
 * buckets of the small dense levels meet through 64-bit integer atomics). */
int neus_debug_scatter_parts(NeusTestbed* tb, uint32_t* parts_per_level /* n_levels */);
/* Development check of the single-pass exclusive scan the step's compactions use (scan.hip): device buffers in / out
 * of n u32 on `hip_stream`, `reps` launches on one fresh state (the epoch re-arm), synchronous; failures = bounded-wait
 * give-ups (0 expected). */
int neus_debug_exclusive_scan(void* hip_stream, const uint32_t* in, uint32_t* out, uint32_t n, int reps, uint32_t* failures);
/* Test hook of the scan's bounded wait: the same scan with its first tile never run, so every later tile gives up
 * waiting (n > 4096 elements); failures = the give-ups counted (nonzero expected). */
int neus_debug_scan_giveup(void* hip_stream, const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* failures);
/* Test hook of the training step's health check: raises device health bits (1 march t, 2 scan give-up) in the
 * testbed's step state / scan state, as the kernels would; the next loss readback makes neus_testbed_train fail. */
int neus_debug_inject_health(NeusTestbed* tb, uint32_t flags);
/* Test hook: every training step fills every CU's LDS with `pattern` (0: off) before its march write kernel. */
int neus_debug_set_lds_fill(NeusTestbed* tb, uint32_t pattern);
/* Test hook: every training step fills every CU's LDS with `pattern` (its complement on odd steps; 0: off) before each of
 * the step's kernels, so a kernel that read LDS it had not written in its own launch would change the results (the
 * determinism test of the whole step: tests/test_gpu_determinism.py). */
int neus_debug_set_lds_fill_all(NeusTestbed* tb, uint32_t pattern);
/* Test hook: every training step launches a no-op kernel of n_blocks workgroups before each of its kernels, shifting the
 * round-robin workgroup -> XCD placement (0: off); the step's results must not depend on the placement. */
int neus_debug_set_xcd_shift(NeusTestbed* tb, uint32_t n_blocks);
/* Development: the last step's compacted training batch (coords batch x 7 f32, dL/doutput batch x 16 fp16 bits) and
 * per-ray losses (2^18 f32); host buffers, each nullable. */
int neus_debug_get_batch(NeusTestbed* tb, float* coords_out, uint16_t* dl_dout_out, float* loss_out);
/* Diagnostic: `launches` launches of an fp32-denormal arithmetic probe (march.hip k_denorm_probe) over n threads on a
 * stream of its own, every value compared with the CPU's bits. stats[10]: launches, mismatches, mismatches by 16-lane row
 * of the wave (4), values flushed to zero, distinct MODE register values (1 or 2), the first MODE, a differing MODE. */
int neus_debug_denorm_probe(int device, uint32_t n, uint32_t launches, uint64_t* stats);
/* Development: nbytes at offset of one step-workspace buffer (ids in testbed.cpp neus_debug_get_buffer). */
int neus_debug_get_buffer(NeusTestbed* tb, int id, uint64_t offset, uint64_t nbytes, void* host);
/* Development: the loss-gradient kernel replayed on the last step's state into a separate buffer (batch x 16 fp16). */
int neus_debug_replay_loss_grad(NeusTestbed* tb, uint16_t* dl_dout_out);
/* neus_sample_rays (rank 0 of 1) plus the progressive round-0 work list the training step's march writes (the first
 * min(n, chunk_end) samples of every kept ray, in ray order; list: device, max_samples u32, list_len: host u32), with
 * lds_fill != 0 every CU's LDS filled with that pattern between the scan and the write kernel (stale-LDS test). */
int neus_debug_sample_rays_round0(NeusTestbed* tb, void* stream, uint32_t n_rays, uint32_t n_rays_total, uint64_t rng_state, uint64_t rng_inc,
                                  uint32_t max_samples, const uint8_t* bitfield, float* rays, uint32_t* numsteps, float* coords,
                                  uint32_t* counters_out, uint32_t chunk_end, uint32_t* list, uint32_t* list_len, uint32_t lds_fill);
int neus_testbed_stream(NeusTestbed* tb, void** hip_stream);
int neus_testbed_synchronize(NeusTestbed* tb);
/* Per-phase step timing with hipEvents recorded on the testbed stream (profiling on), mean ms per step:
 * ms_out[0] occupancy update, [1] ray sampling (march count/scan/write), [2] fused hash-grid encode +
 * network forward on the pre-compaction samples, [3] loss + compaction + rollover, [4] training
 * hash-grid encode, [5] fused MLP fwd/bwd/2nd-order, [6] weight-gradient GEMMs, [7] hash-grid gradient
 * scatter, [8] all-reduce + counters, [9] Ema(Adam); ms_out[NEUS_N_PHASES] = number of profiled steps,
 * [+1] mean pre-compaction samples per step (the inference kernel's n), [+2] mean compacted training
 * samples per step. Phases 2 and 4-7 are single kernels. */
#define NEUS_N_PHASES 10
int neus_testbed_set_profiling(NeusTestbed* tb, int on);
int neus_testbed_kernel_times(NeusTestbed* tb, float* ms_out /* NEUS_N_PHASES + 3 entries */);
/* Inference timing of the training step as it runs: with it on, every pre-compaction network launch of a step (the
 * one pass, or each progressive round's k_nerf_infer) is bracketed by hipEvents on the testbed stream and the host
 * waits for them after the step (a measurement pass, not for timed runs). Totals since it was turned on: summed launch
 * ms, launches, steps; the samples those launches evaluated are NeusTrainStats::evaluated_samples_total's growth. */
int neus_testbed_set_infer_timing(NeusTestbed* tb, int on);
int neus_testbed_infer_timing(NeusTestbed* tb, double* ms_total, uint64_t* launches, uint64_t* steps);
/* Exchange timing of the data-parallel step (ABI 5; no effect without collectives): per step, hipEvents where the
 * backward is done on the step's stream and where the last collective ends on the exchange stream. Totals since it was
 * turned on: exposed_ms = sum of max(0, exchange end - backward end), the time the join before the optimizer waits;
 * span_ms = sum of (exchange end - loss end), the exchange's whole window (the counters' all-reduce starts after the
 * loss); steps. Collected without a per-step host wait, so it may run inside a timed region. */
int neus_testbed_set_exchange_timing(NeusTestbed* tb, int on);
int neus_testbed_exchange_timing(NeusTestbed* tb, double* exposed_ms_total, double* span_ms_total, uint64_t* steps);

/* ------------------------------------------------------------------ data parallel (RCCL over xGMI) */
int neus_nccl_unique_id(uint8_t* out /* 128 bytes */);
int neus_testbed_init_data_parallel(NeusTestbed* tb, int rank, int world, const uint8_t* unique_id /* 128 bytes */);
/* As neus_testbed_init_data_parallel; flags bit 0 (NEUS_DP_FORCE_COLLECTIVES): create the RCCL communicator and issue
 * every collective of the step even at world 1 (a one-rank all-reduce is the identity: tests run the RCCL path with it). */
#define NEUS_DP_FORCE_COLLECTIVES 1
int neus_testbed_init_data_parallel_ex(NeusTestbed* tb, int rank, int world, const uint8_t* unique_id, uint32_t flags);
typedef struct NeusDataParallelInfo {
	uint32_t rank, world;
	uint32_t has_communicator;       /* an RCCL communicator exists (world > 1, or forced) */
	uint32_t local_group;            /* in-process group (host-staged collectives) */
	uint64_t collective_calls;       /* all-reduce calls issued since init */
	uint64_t allreduce_bytes;        /* bytes all-reduced since init (per rank, payload) */
	uint64_t last_step_allreduce_bytes;
	uint32_t host_group;             /* cross-process host-staged group (neus_host_group_create) */
} NeusDataParallelInfo;
int neus_testbed_data_parallel_info(NeusTestbed* tb, NeusDataParallelInfo* out);
/* Overlapped gradient exchange (default on): the MLP blocks are all-reduced after the weight-gradient reduction and the
 * hash-grid levels in three groups as the scatter finishes them, on a communication stream beside the rest of the
 * backward; off: one grouped exchange after the backward (the same elementwise sums). */
int neus_testbed_set_exchange_overlap(NeusTestbed* tb, int on);
/* In-process ranks: `world` testbeds driven from `world` host threads exchange through host staging buffers
 * (same step and collectives as the RCCL path: sharded occupancy update + max all-reduce, gradient / counter /
 * loss / DeltaNetwork sum all-reduces). For several ranks on one device (tests); collectives block until every
 * rank has arrived (120 s timeout -> error). The group must outlive its testbeds' training calls. */
typedef struct NeusLocalGroup NeusLocalGroup;
int neus_local_group_create(int world, NeusLocalGroup** out);
int neus_local_group_destroy(NeusLocalGroup* group);
int neus_testbed_init_local_group(NeusTestbed* tb, NeusLocalGroup* group, int rank);
/* Cross-process host-staged collectives (hostgroup.h): ranks in separate processes (e.g. several on one GPU, which RCCL
 * refuses) exchange over TCP, rank 0 at host:port (IPv4) reducing in rank order (bitwise the in-process group's sums).
 * Each collective is staged on the testbed's communication stream (device -> pinned host, a host function for the
 * exchange, host -> device), gated by the same events as the RCCL collectives, so the overlapped exchange runs beside the
 * backward. Every rank creates its group (rank 0 listens, the others connect; 120 s timeouts) and attaches its testbed;
 * the ranks must issue the same collectives (a mismatch fails loudly). The group must outlive its testbed's training.
 * job_token (ABI 5): a per-job value every rank passes alike (e.g. random, broadcast by the launcher with the port); rank 0
 * drops connections whose hello carries another token or an already-joined rank and keeps waiting. It keeps stray and
 * foreign processes out, it does not authenticate: keep host at 127.0.0.1 unless the port's network is trusted. */
typedef struct NeusHostGroup NeusHostGroup;
int neus_host_group_create(int rank, int world, const char* host, int port, uint64_t job_token, NeusHostGroup** out);
int neus_host_group_destroy(NeusHostGroup* group);
int neus_testbed_init_host_group(NeusTestbed* tb, NeusHostGroup* group);
/* Test hook (no GPU): one collective of the group's protocol on a host buffer of n 4-byte elements, type 0 f32 / 1 u32,
 * op 0 sum / 1 max; a failed exchange poisons the group and returns its error. */
int neus_debug_host_group_allreduce(NeusHostGroup* group, void* host, uint64_t n, int type, int op);

/* ------------------------------------------------------------------ tcnn-shaped operator modules
 * tcnn::cpp::Module (dependencies/my_tcnn/include/tiny-cuda-nn/cpp_api.h:66-110) over the gfx950 kernels, with
 * explicit parameter pointers, a forward context and EGradientMode (object.h:90-94). Device buffers throughout;
 * `stream` is the hipStream_t the call runs on (NULL: the null stream). Factories, named as tcnn's (cpp_api.h:108-110):
 *   neus_module_create_network   create_network(n_input_dims, n_output_dims, network) (cpp_api.cu:170-172): an Identity
 *                                encoding (inputs padded to 16 with ones) in front of a FullyFusedMLP (n_neurons 16 / 32 /
 *                                64 / 128, n_hidden_layers >= 1, activation / output_activation None, ReLU, Exponential,
 *                                Sigmoid, Squareplus, Softplus); input [n][n_input_dims] f32, output [n][padded out] fp16,
 *                                params [W x in_pad | (N - 1) x W x W | out_pad x W] fp16 (fully_fused_mlp.cu:816-879);
 *                                n must be a multiple of 128 (fully_fused_mlp.cu:779-781).
 *   neus_module_create_encoding  create_encoding (HashGrid, grid.h): input [n][3] f32; output layout from the config's
 *                                "output_layout": "AoS" [n][2L] fp16 (default: the column-major matrix cpp::Module wraps,
 *                                cpp_api.cu:58-70), "SoA" [2L][n] (GridEncoding::preferred_output_layout, grid.h:2357-2359) or
 *                                "paired" [L][n] half2 (this build's kernels); params [n_grid] fp16. requested_precision
 *                                (cpp_api.h:110, cpp_api.cu:174-180): NEUS_PRECISION_FP16 = GridEncoding<__half> (the
 *                                kernels of the training step), NEUS_PRECISION_FP32 = GridEncoding<float>: params, output,
 *                                dL_doutput, dL_ddLdoutput and dL_dparams f32 (AoS / SoA layouts).
 *   neus_module_create_network_with_input_encoding  {HashGrid, Identity} -> FullyFusedMLP of any depth (below).
 *   neus_module_create_nerf_network  the NeuS NerfNetwork (nerf_network.h; the full config object with "encoding",
 *                                "network", "rgb_network"): input NerfCoordinate [n][7] f32 (pos, dt, dir), output
 *                                [n][16] fp16; params [n_params] fp16 in the layout of neus_testbed_layout. Its backward
 *                                needs n % 128 == 0 and includes the eikonal second order (as nerf_network.h:330-601); its
 *                                dL_dinput ([n][7] f32) carries the position columns (dt / direction columns written 0).
 * Parameter gradients dL_dparams are param precision (fp16, tcnn's trainer.h:72-109) unless the config sets
 * "gradient_precision": "fp32". backward_backward_input is the encoding's (grid.h:1697-1800, without the dL_dinput term),
 * the network-with-input-encoding's and create_network's (fully_fused_mlp.cu:1088-1198: parameter gradients only).
 * Progressive levels follow set_training_step (grid.h:2427-2437; 0 = all levels). */
typedef struct NeusModule NeusModule;
typedef struct NeusContext NeusContext;
enum { NEUS_GRADIENT_IGNORE = 0, NEUS_GRADIENT_OVERWRITE = 1, NEUS_GRADIENT_ACCUMULATE = 2 };
enum { NEUS_PRECISION_FP32 = 0, NEUS_PRECISION_FP16 = 1 };
typedef struct NeusModuleInfo {
	uint64_t n_params;
	uint32_t n_input_dims, n_output_dims;
	int32_t param_precision, output_precision, gradient_precision;
	uint32_t batch_capacity;
	uint32_t n_levels;
	uint64_t grid_offset;   /* first hash-grid parameter (network modules) */
	float per_level_scale;
} NeusModuleInfo;
int neus_module_create_network(uint32_t n_input_dims, uint32_t n_output_dims, const char* network_json, uint32_t batch_capacity, NeusModule** out);
int neus_module_create_nerf_network(const char* config_json, uint32_t batch_capacity, NeusModule** out);
int neus_module_create_encoding(uint32_t n_input_dims, const char* encoding_json, int requested_precision, uint32_t batch_capacity,
                                NeusModule** out);
/* create_network_with_input_encoding (cpp_api.h:108; network_with_input_encoding.h): `encoding` HashGrid (input [n][3] f32) or
 * Identity ({"scale", "offset"}, identity.h; input [n][n_input_dims] f32) in front of a FullyFusedMLP as create_network's.
 * Output [n][padded n_output_dims] fp16 (column-major, as cpp_api.cu:58-70); params [network matrices in order | grid] fp16
 * (NetworkWithInputEncoding: network first, network_with_input_encoding.h:262-270), the MLP's input width DE = 2 n_levels
 * padded to 16 with zeros (grid.h:1540-1550). HashGrid -> 1 hidden ReLU layer of 16 / 64 neurons -> linear output of <= 16
 * dims runs as one fused kernel; other shapes as the grid kernels feeding the FullyFusedMLP layers. backward_backward_input
 * follows network_with_input_encoding.h:159-250 / fully_fused_mlp.cu:1088-1198 (parameter gradients only; dL_ddLdoutput and
 * dL_dinput are not written, as in the reference). */
int neus_module_create_network_with_input_encoding(uint32_t n_input_dims, uint32_t n_output_dims, const char* encoding_json,
                                                   const char* network_json, uint32_t batch_capacity, NeusModule** out);
int neus_module_destroy(NeusModule* m);
int neus_context_destroy(NeusContext* ctx);
int neus_module_info(const NeusModule* m, NeusModuleInfo* out);
/* Module::hyperparams as JSON text (len = its length; buf gets a NUL-terminated prefix of up to cap - 1 bytes). */
int neus_module_hyperparams(const NeusModule* m, char* buf, uint64_t cap, uint64_t* len);
int neus_module_set_training_step(NeusModule* m, int training_step);
/* NeuS backward: the eikonal entries of dL_doutput are divided by this batch size (0 = each call's n). */
int neus_module_set_indeed_batch_size(NeusModule* m, uint32_t indeed_batch_size);
/* Module::initialize_params: fp32 initial parameters (trainer.h:54-109 seed_seq{seed} -> pcg32) into a device buffer. */
int neus_module_initialize_params(NeusModule* m, uint64_t seed, float* params_full_precision);
int neus_module_inference(NeusModule* m, void* stream, uint32_t n_elements, const float* input, void* output, const void* params);
int neus_module_forward(NeusModule* m, void* stream, uint32_t n_elements, const float* input, void* output, const void* params,
                        int prepare_input_gradients, NeusContext** ctx);
int neus_module_backward(NeusModule* m, void* stream, const NeusContext* ctx, uint32_t n_elements, float* dL_dinput, const void* dL_doutput,
                         void* dL_dparams, const float* input, const void* output, const void* params, int gradient_mode);
int neus_module_backward_backward_input(NeusModule* m, void* stream, const NeusContext* ctx, uint32_t n_elements, const float* dL_ddLdinput,
                                        const float* input, const void* dL_doutput, void* dL_dparams, void* dL_ddLdoutput,
                                        float* dL_dinput, const void* params, int gradient_mode);

/* ------------------------------------------------------------------ operator surface (device buffers) */
/* Hash-grid forward on n positions (AoS, `coord_stride` floats per sample, xyz first).
 * enc: [2L][ld] fp16, dydx: [6L][ld] f32 (nullable). */
int neus_grid_encode(NeusTestbed* tb, void* stream, uint32_t n, uint32_t ld, const float* coords, uint32_t coord_stride,
                     uint32_t valid_level, uint16_t* enc, float* dydx);
/* NerfNetwork forward: coords AoS7 f32 -> out AoS16 fp16 (training weights). */
int neus_net_forward(NeusTestbed* tb, void* stream, uint32_t n, const float* coords, uint32_t valid_level, uint16_t* out);
/* NerfNetwork forward+backward (first- and second-order), gradient Overwrite into grads_out
 * (fp32 [P], device). n must be a multiple of 128. */
int neus_net_backward(NeusTestbed* tb, void* stream, uint32_t n, const float* coords, uint32_t valid_level, const uint16_t* dL_dout,
                      uint32_t indeed_batch_size, float* grads_out);
/* neus_net_backward plus dL/d(input position) per sample (dpos: [n][4] f32, device; the first-order gradient
 * the global-movement backward consumes, nerf_network.h:602-631). */
int neus_net_backward_pos(NeusTestbed* tb, void* stream, uint32_t n, const float* coords, uint32_t valid_level, const uint16_t* dL_dout,
                          uint32_t indeed_batch_size, float* grads_out, float* dpos);
/* DeltaNetwork forward with the testbed's local movement (add_global_movement_with_rotation_6d,
 * common_operation.cuh:416-492): stride 7 (NerfCoordinate: position and direction) or 3 (position only). */
int neus_delta_apply(NeusTestbed* tb, void* stream, uint32_t n, uint32_t stride, const float* in, float* out);
/* DeltaNetwork backward (add_loss_to_rotation_6d_each + reduce_sum, common_operation.cuh:788-845,
 * transform_network.h:206-245): coords = undeformed inputs, dpos = dL/d(deformed position) [n][4];
 * grads12_host gets the fp16-valued, loss-scaled parameter gradients (no optimizer step). */
int neus_delta_backward(NeusTestbed* tb, void* stream, uint32_t n, uint32_t stride, const float* coords, const float* dpos, float* grads12_host);
/* Training-sample generation with the testbed's dataset on the given bitfield. Outputs are
 * per ray slot (canonical ray order): rays 6 f32, numsteps 2 u32 (n, base), coords AoS7.
 * counters_out (host, 3 u32): numsteps_counter, n_kept, n_rays_with_samples. */
int neus_sample_rays(NeusTestbed* tb, void* stream, uint32_t n_rays, uint32_t rank, uint32_t world, uint32_t n_rays_total,
                     uint64_t rng_state, uint64_t rng_inc, uint32_t max_samples, const uint8_t* bitfield,
                     float* rays, uint32_t* numsteps, float* coords, uint32_t* counters_out);
/* NeuS composite + loss + compaction given network outputs. numsteps is rewritten to
 * (n_compacted, compacted_base). counters_out (host): compacted_counter. */
int neus_loss_compact(NeusTestbed* tb, void* stream, uint32_t n_rays, uint32_t rank, uint32_t world, uint32_t n_rays_total,
                      uint64_t rng_state, uint64_t rng_inc, uint32_t max_compacted, const float* rays, uint32_t* numsteps,
                      const float* coords, const uint16_t* net_out, float* coords_out, uint16_t* dL_dout,
                      float* loss, float* ek_loss, float* mask_loss, uint32_t* counters_out);
/* One Ema(Adam) step on the testbed's parameters with the given fp32 gradients (device). */
int neus_optimizer_step(NeusTestbed* tb, void* stream, const float* grads);
/* fill_rollover_and_rescale (my_tcnn common_device.h:515-535; testbed_nerf.cu:3922-3930): rows [n_in, n_elements)
 * of coords (AoS7 f32) and dL_dout (AoS16 fp16) become copies of row i % n_in, dL_dout scaled by n_in / n_elements.
 * n_in is clamped to n_elements; n_in = 0 leaves both untouched. Device buffers. */
int neus_fill_rollover(NeusTestbed* tb, void* stream, uint32_t n_elements, uint32_t n_in, float* coords, uint16_t* dL_dout);
/* One occupancy-grid update (density_grid + bitfield) of the testbed's state. */
int neus_occ_update(NeusTestbed* tb, void* stream, uint32_t n_uniform, uint32_t n_nonuniform);
/* MFMA fragment-layout probe: C[32x32] = A[32x16] * B[16x32], fp16 row-major in, f32 out. */
int neus_mfma_probe(const uint16_t* A, const uint16_t* B, float* C);

#ifdef __cplusplus
}
#endif

#endif /* NEUS2_HIP_H */
