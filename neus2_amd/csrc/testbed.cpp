// Host orchestration of the NeuS2 training hot path on gfx950 and its C-ABI (include/neus2_hip.h).
//
// NeusTestbed restates the training-relevant part of the reference Testbed
// (include/neural-graphics-primitives/testbed.h:63-940; src/testbed.cu:2084-2349, 2640-2736;
// src/testbed_nerf.cu:3293-3548, 3723-4016) MI355X-first:
//   * one HIP stream per testbed, every counter device-resident (no host sync inside a step);
//   * deterministic count -> scan -> write compaction instead of atomic appends;
//   * fp32 gradients and master weights, fp16 weights for the kernels (the reference keeps fp16
//     gradients), RCCL all-reduce of the gradient buffer for data parallelism over ray batches.
#include <rocprofiler-sdk-roctx/roctx.h>
#include "kernels.h"
#include "scan_lookback.h"
#include "json_lite.h"
#include "hostgroup.h"
#include "../../include/neus2_hip.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <functional>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

using namespace neus;

namespace {

thread_local std::string g_err;

#define HIP_CHECK(x)                                                                                   \
	do {                                                                                               \
		hipError_t e_ = (x);                                                                           \
		if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + " failed: " + hipGetErrorString(e_)); \
	} while (0)
#define NCCL_CHECK(x)                                                                                  \
	do {                                                                                               \
		ncclResult_t r_ = (x);                                                                         \
		if (r_ != ncclSuccess) throw std::runtime_error(std::string(#x) + " failed: " + ncclGetErrorString(r_)); \
	} while (0)

// Debug: NEUS_DBG_POISON="byte[:lo:hi]" fills the fresh device allocations number lo .. hi-1 (counted from the last
// testbed creation) with `byte`; NEUS_DBG_ALLOC_LOG=1 lists them (number, bytes) on stderr. A result that changes with
// the fill reads memory no kernel wrote (i.e. depends on what a recycled allocation held). Off: one getenv per alloc.
std::atomic<uint64_t> g_alloc_seq{0}, g_alloc_base{0};
void dbg_poison(void* p, size_t bytes) {
	const uint64_t k = g_alloc_seq++ - g_alloc_base.load();
	if (std::getenv("NEUS_DBG_ALLOC_LOG")) std::fprintf(stderr, "neus alloc %llu %zu\n", (unsigned long long)k, bytes);
	const char* e = std::getenv("NEUS_DBG_POISON");
	if (!e) return;
	unsigned v = 0;
	unsigned long long lo = 0, hi = ~0ull;
	if (std::sscanf(e, "%u:%llu:%llu", &v, &lo, &hi) < 1) return;
	if (k >= lo && k < hi) HIP_CHECK(hipMemset(p, (int)v, bytes));
}

template <class T> struct Dev {
	T* p = nullptr;
	size_t n = 0;
	void alloc(size_t k) {
		if (k <= n && p) return;
		release();
		if (k == 0) return;
		HIP_CHECK(hipMalloc((void**)&p, k * sizeof(T)));
		dbg_poison(p, k * sizeof(T));
		n = k;
	}
	void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
	~Dev() { release(); }
};
// A scan temp buffer (scan_temp_bytes: look-back state + hipCUB scratch): its host-side launch tag (scan.hip) is dropped
// with the buffer
struct ScanTemp : Dev<uint8_t> {
	void alloc(size_t k) { if (k <= n && p) return; release(); Dev<uint8_t>::alloc(k); }
	void release() { if (p) scan_temp_release(p); Dev<uint8_t>::release(); }
	~ScanTemp() { release(); }
};

constexpr uint32_t MAX_RAYS = 1u << 18;  // testbed_nerf.cu:3435 cap on rays_per_batch
constexpr float LOSS_SCALE = 128.f;      // testbed.h:246

uint32_t next_multiple(uint32_t v, uint32_t m) { return (v + m - 1) / m * m; }

// ld_random_pixel_offset (random_val.cuh:254-288, 317-322): scrambled Sobol 2-D value of the spp index,
// offset = fract(0.5 - v(0) + v(spp)). Sobol dimension 0 is the bit reversal; dimension 1 has direction
// numbers d[0] = 2^31, d[b] = d[b-1] ^ (d[b-1] >> 1).
uint32_t rev_bits(uint32_t x) {
	x = ((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1); x = ((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2);
	x = ((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4); x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
	return (x >> 16) | (x << 16);
}
uint32_t nus_scramble(uint32_t x, uint32_t seed) {
	x = rev_bits(x);
	x += seed; x ^= x * 0x6c50b47cu; x ^= x * 0xb82f1e52u; x ^= x * 0xc7afe638u; x ^= x * 0x8d22f6e6u;
	return rev_bits(x);
}
uint32_t sobol_dim(uint32_t index, uint32_t dim) {
	uint32_t X = 0, d = 0x80000000u;
	for (uint32_t bit = 0; bit < 32; ++bit) {
		const uint32_t dir = dim == 0 ? (0x80000000u >> bit) : d;
		if ((index >> bit) & 1) X ^= dir;
		d ^= d >> 1;
	}
	return X;
}
void ld_random_val_2d(uint32_t index, uint32_t seed, float out[2]) {
	const float S = float(1.0 / 4294967296.0);
	index = nus_scramble(index, seed);
	for (uint32_t i = 0; i < 2; ++i) out[i] = (float)nus_scramble(sobol_dim(index, i), seed ^ (i + (seed << 6) + (seed >> 2))) * S;
}
void ld_pixel_offset(uint32_t spp, float out[2]) {
	float a[2], b[2];
	ld_random_val_2d(0, 0xdeadbeefu, a);
	ld_random_val_2d(spp, 0xdeadbeefu, b);
	for (int k = 0; k < 2; ++k) { const float v = (0.5f - a[k]) + b[k]; out[k] = v - std::floor(v); }
}

struct Layout {
	uint32_t din, W, L;
	uint32_t off_d0, off_d1, off_r0, off_r1, off_r2, n_density, n_rgb, n_matrix, grid_off, n_grid, var_off, P;
};

} // namespace

// In-process data-parallel group: `world` testbeds driven from `world` host threads exchange through host staging
// buffers (sum in rank order, max), with the same call sequence as the RCCL path. It lets the data-parallel step
// (sharded occupancy update, gradient / counter / loss / DeltaNetwork all-reduces) run with several ranks on one
// device, e.g. in tests; production ranks use RCCL (neus_testbed_init_data_parallel).
struct NeusLocalGroup {
	enum Op { SUM, MAX };
	uint32_t world;
	std::mutex mu;
	std::condition_variable cv;
	uint32_t arrived = 0, generation = 0;
	bool failed = false;  // a rank timed out: every later collective fails fast instead of pairing the wrong ranks
	std::vector<std::vector<uint8_t>> stage;
	explicit NeusLocalGroup(uint32_t w) : world(w), stage(w) {}
	void barrier() {
		std::unique_lock<std::mutex> lk(mu);
		if (failed) throw std::runtime_error("local group: a previous collective failed (the group is poisoned)");
		const uint32_t gen = generation;
		if (++arrived == world) { arrived = 0; ++generation; cv.notify_all(); return; }
		if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen || failed; }) || failed) {
			if (generation == gen) --arrived;  // this rank's arrival is withdrawn
			failed = true;
			cv.notify_all();
			throw std::runtime_error("local group: barrier timeout (a rank did not reach the collective)");
		}
	}
	// in-place all-reduce of n elements of T on the device, on `s` (host-synchronous)
	template <class T> void allreduce(uint32_t rank, T* dev, size_t n, Op op, hipStream_t s) {
		std::vector<uint8_t>& mine = stage[rank];
		mine.resize(n * sizeof(T));
		HIP_CHECK(hipMemcpyAsync(mine.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		barrier();
		std::vector<T> out(n);
		for (uint32_t r = 0; r < world; ++r) {
			const T* v = (const T*)stage[r].data();
			for (size_t k = 0; k < n; ++k) out[k] = r == 0 ? v[k] : (op == SUM ? (T)(out[k] + v[k]) : std::max(out[k], v[k]));
		}
		barrier();  // every rank has read every stage before the next collective overwrites one
		HIP_CHECK(hipMemcpyAsync(dev, out.data(), n * sizeof(T), hipMemcpyHostToDevice, s));
		HIP_CHECK(hipStreamSynchronize(s));
	}
};

struct NeusTestbed {
	int device = 0;
	hipStream_t stream = nullptr;
	// side stream of the backward: the weight-gradient GEMM runs there beside the grid scatter (disjoint inputs and
	// outputs; both deterministic), forked from and joined back into the step's stream by events
	hipStream_t aux_stream = nullptr;
	hipEvent_t ev_fork = nullptr, ev_join = nullptr;
	// Lookahead (NEUS_LOOKAHEAD): the next step's ray sampling (ray generation, march, march write, ray sort) issued on
	// la_stream right after this step's loss, beside its backward and optimizer, which read none of its outputs. Only
	// between steps of one neus_testbed_train call (nothing pending between calls), at one rank, on static scenes, and
	// not before a step that starts with an occupancy update or a loss readback (train_step: la_go).
	bool la_on = [] { const char* e = std::getenv("NEUS_LOOKAHEAD"); return !(e && e[0] == '0'); }();
	// adam_overlap: the step's Adam parameters; next: the first parameter not issued; on: the exchange stream the pieces
	// follow their ranges' all-reduces on (data parallel), or null (one rank: ad_stream, behind the step's stream)
	struct AdamSplit { AdamParams p; uint32_t next; hipStream_t on; };
	bool la_pending = false, la_next_in_call = false;
	uint64_t la_steps = 0, adam_split_steps = 0;  // (stats: lookahead_steps, adam_split_steps)
	const bool la_stat = [] { const char* e = std::getenv("NEUS_LA_STAT"); return e && e[0] == '1'; }();
	// Where in the backward the lookahead is issued (one rank; with a group it goes out with the counters' exchange):
	// 0 right after the loss, 1 after the training encode, 2 after the training MLP kernels, 3 after the weight-gradient
	// reduction, 4 after the scatter. A cut march's sampling is small and goes after the encode (it then no longer shares
	// the gather-bound encode: 0.770 -> 0.759 ms/step at step 800, 0.876 -> 0.854 at step 1600,
	// profiles/r06la_issue_point_ab.txt); a full march needs the whole backward to hide in and goes right after the loss
	// (round 5: 1 as 0, 2 and 3 slower, r05la_issue_point_ab.txt). NEUS_LA_AT / NEUS_LA_AT_FULL override the two.
	const int la_at_cut = [] { const char* e = std::getenv("NEUS_LA_AT"); return e ? std::atoi(e) : 1; }();
	const int la_at_full = [] { const char* e = std::getenv("NEUS_LA_AT_FULL"); return e ? std::atoi(e) : 0; }();
	int la_at = 0;  // the pending lookahead's issue point
	std::function<void()> la_deferred;
	void la_fire(int at) {
		if (la_deferred && at >= la_at) { auto f = std::move(la_deferred); la_deferred = nullptr; f(); }
	}
	int main_prio = 0;  // the step's streams' priority (0: created without one; the communication stream follows it)
	hipStream_t la_stream = nullptr;
	hipEvent_t ev_la_start = nullptr, ev_la_done = nullptr;
	// development (NEUS_LA_STAT=1): per lookahead, timing events around its sampling (la stream) and around the next
	// step's wait for it (main stream); summed and printed at the end of each neus_testbed_train call
	std::vector<hipEvent_t> la_stat_ev;
	size_t la_stat_used = 0;
	hipEvent_t la_stat_next() {
		if (la_stat_used == la_stat_ev.size()) {
			hipEvent_t e;
			HIP_CHECK(hipEventCreate(&e));
			la_stat_ev.push_back(e);
		}
		return la_stat_ev[la_stat_used++];
	}
	void la_stat_report() {
		if (la_stat_used < 4) { la_stat_used = 0; return; }
		HIP_CHECK(hipDeviceSynchronize());
		// groups of 4: la begin, la end (previous step), wait begin, wait end (this step)
		double wait = 0, dur = 0, slack = 0;
		size_t n = 0;
		for (size_t k = 0; k + 4 <= la_stat_used; k += 4, ++n) {
			float a = 0, b = 0, c = 0;
			HIP_CHECK(hipEventElapsedTime(&a, la_stat_ev[k + 2], la_stat_ev[k + 3]));
			HIP_CHECK(hipEventElapsedTime(&b, la_stat_ev[k], la_stat_ev[k + 1]));
			HIP_CHECK(hipEventElapsedTime(&c, la_stat_ev[k + 1], la_stat_ev[k + 2]));
			wait += a; dur += b; slack += c;
		}
		std::fprintf(stderr, "la_stat n=%zu wait_us=%.1f sampling_us=%.1f slack_us=%.1f\n", n, 1e3 * wait / n, 1e3 * dur / n, 1e3 * slack / n);
		la_stat_used = 0;
	}
	NeusNetworkConfig cfg{};
	bool have_net = false, have_data = false;
	Layout lay{};
	GridLevels gl{};
	// dataset
	Dev<uint32_t> pixels; Dev<uint64_t> pix_off; Dev<int32_t> res; Dev<float> focal, pp, xform;
	DevDataset ds{};
	Dev<float> srgb_lut;  // read_rgba's byte -> linear table
	std::vector<float> host_focal, host_pp, host_xform;
	std::vector<int32_t> host_res;
	uint32_t max_cascade = 0;
	float aabb_scale = 1.f;
	// parameters
	Dev<float> params_fp, grads, m1, m2, ema_tmp;
	// per-parameter Adam steps: u16 [P] saturating at 65535 while the bias table is converged (optim.hip AdamSteps), else
	// u32 [P] (steps32); P x 4 B either way
	Dev<uint32_t> adam_steps;
	bool steps32 = false;
	Dev<half_t> params_h, ema_h, wT;
	MlpPtrs mlp{};
	DinPerm din_perm{};
	// inference params (EMA weights, the reference's Ema::custom_weights) for rendering
	Dev<half_t> wT_ema;
	// The fp16 EMA (inference) weights are only read outside the training step (render, SDF grid, mesh colours, snapshots,
	// the frame restart), so the step updates the fp32 EMA alone and the fp16 copy is cast from it when first read: the
	// same bits the Adam kernel would have written (ema_h = half(ema_tmp) after every step), 2 B per parameter less per step
	bool ema_h_stale = false;
	void sync_ema_h() {
		if (!ema_h_stale) return;
		launch_cast_half(stream, lay.P, ema_tmp.p, ema_h.p);
		HIP_CHECK(hipGetLastError());
		HIP_CHECK(hipStreamSynchronize(stream));  // (readers may use another stream or the host)
		ema_h_stale = false;
	}
	MlpPtrs mlp_ema{};
	// renderer workspace (NerfTracer, testbed_nerf.cu:2397-2630)
	Dev<uint8_t> r_rays[2];
	ScanTemp r_scan_tmp;
	Dev<uint32_t> r_flags, r_base, r_alive;
	Dev<float> r_coords, r_coords_def;
	Dev<half_t> r_out;
	Dev<float4> r_frame, r_accum;
	size_t r_scan_bytes = 0;
	// marching cubes workspace and the last mesh (Testbed::m_mesh, testbed.h:596-610)
	Dev<float> mc_density, mesh_v;
	Dev<uint32_t> mc_vidx, mc_cnt, mesh_f;
	ScanTemp mc_scan_tmp;
	size_t mc_scan_bytes = 0;
	uint32_t mesh_nv = 0, mesh_nt = 0;
	// dynamic scenes (testbed.h:455-477, 889-890): frame, phase flags, the DeltaNetwork state on the device,
	// deformed copies of the sample coordinates, dL/d(position) of the training batch
	uint32_t cur_frame = 0, canonical_step = 0, delta_step = 0;
	bool train_canonical = true, train_delta = false;
	bool nonfinite = false, aborted = false;  // training health (consume_loss); cleared by reset_network
	bool render_delta = false;     // prepare_for_test (testbed.cu:1987-1999): render / mesh through the DeltaNetwork
	float near_distance = 0.f;     // nerf.training.near_distance: stored; the NeuS sampler does not read it (testbed_nerf.cu:1525)
	// nerf.training.depth_supervision_lambda (testbed.h:649): stored. The reference's loss kernel computes the depth term
	// (testbed_nerf.cu:1697-1698, 1836) but adds it to no gradient and no loss output, so it never changes training; the
	// step here keeps that (no depth term; tests/test_gpu_depth.py checks a lambda > 0 run against lambda = 0 bitwise)
	float depth_lambda = 0.f;
	int32_t color_space_when_linear = 0;  // color_space as set while linear_colors overrides it
	float delta_lr_factor = 1.f;
	Dev<DeltaState> delta;
	Dev<float> delta_partial, coords_def, coords_cdef;
	Dev<float4> dpos;
	// occupancy grid
	Dev<float> density_grid, density_tmp, grid_mean, grid_partial, occ_pos, occ_density;
	Dev<uint32_t> occ_idx;
	Dev<uint32_t> occ_ulist;  // the cell-ordered uniform samples, OccSampling::ulist
	bool occ_sort = true;     // NEUS_OCC_SORT=0: uniform samples in index order (A/B reference)
	Dev<uint8_t> bitfield;
	Dev<uint32_t> bf_lin;   // mip-0 occupancy in (x, y, z/32) word order for the constant-step march
	Dev<float> occ_bbox;    // world box of the occupied cells of every mip (+ stage-1 scratch): the ray generation's cull
	Dev<float> adam_bias;   // Adam bias-correction table (AdamParams::bias_tab) for betas bias_b1 / bias_b2
	float bias_b1 = -1.f, bias_b2 = -1.f;
	bool bias_conv = false;
	Dev<uint32_t> dbg_enc;  // debug timing only (neus_debug_time_kernel 11): [L][16 Nc] encodings of the inference samples
	bool ray_cull = true;   // NEUS_RAY_CULL=0: march every ray (A/B reference)
	uint32_t dbg_lds_fill = 0;  // tests (neus_debug_set_lds_fill): garbage-fill every CU's LDS before the step's march write
	bool dbg_loss_replay = [] { const char* e = std::getenv("NEUS_DBG_LOSS_REPLAY"); return e && e[0] == '1'; }();
	Dev<float> dbg_co; Dev<half_t> dbg_dl;
	static constexpr int DBG_SNAP_N = 15;
	Dev<uint8_t> dbg_snap[DBG_SNAP_N];  // the loss-gradient inputs right after its launch (ids 0..14 of neus_debug_get_buffer)
	uint32_t dbg_lds_fill_all = 0;
	uint32_t dbg_xcd_shift = 0;  // tests (neus_debug_set_xcd_shift): workgroups of a no-op kernel before every kernel of the step  // tests (neus_debug_set_lds_fill_all): ... before every kernel of the step (g_dbg_lds_fill)
	Dev<PcgJump> pcg_tab;   // pcg32 jump-ahead table (common.h PcgJumpTable)
	uint32_t density_grid_ema_step = 0;
	uint64_t occ_samples = 0;  // occupancy-grid samples this rank evaluated since the network was loaded
	uint32_t occ_updates = 0;
	// step workspace
	uint32_t batch = 0, max_samples = 0;
	Dev<float> rays, startt, coords, coords_c, loss, ek, mask, loss_sum;
	Dev<uint32_t> health_buf;  // [0] march fail flags, [1] scan give-ups (all-reduced at every loss readback); [2..3] setting checks
	Dev<uint32_t> nreq, base, numsteps, ccount, cbase, enc, march_nrec, march_queue;
	Dev<uint2> march_rec, march_seg;
	MarchWork mwork{};
	Dev<float> dydx;
	Dev<half_t> net_out, dL_dout, trainbuf;
	Dev<float4> vbuf;
	Dev<float> wgrad_partial, var_partial;  // per-block MLP weight-gradient rows, per-block variance sums
	uint32_t mlp_blocks = 0;                // grid of the training MLP kernels at the batch capacity
	ScanTemp scan_tmp, scan_tmp_la;  // (scan_tmp_la: the lookahead's march scans, on la_stream)
	size_t scan_tmp_bytes = 0;
	Dev<StepState> st;
	ScatterWork swork{};
	Dev<uint32_t> sc_counts, sc_offs, sc_jobs, sc_split_done;
	Dev<unsigned long long> sc_split;
	std::vector<uint32_t> sc_jobs_before;  // [n_buckets + 1] accumulation jobs of the buckets below b
	uint32_t sc_zero_from = 0;             // the grads' grid part is known zero from this bucket on
	Dev<uint32_t> sc_jobs2;
	Dev<uint16_t> sc_rtab;
	std::vector<uint32_t> sc_jobs2_before;  // [L + 1] region-scatter jobs of the levels below l
	uint32_t sc_zero_from_e = 0;            // region scatter: grid entries from here on hold zero gradients
	bool scatter_noskip = false;            // NEUS_SCATTER_NOSKIP=1: zero the grid gradient every step (A/B reference)
	Dev<h2> sc_rec_g;
	Dev<uint16_t> sc_rec_i;
	// restructured loss scratch (kernels.h LossWork)
	Dev<float4> l_sa, l_ck4, l_racc, l_rgr;
	Dev<float> l_ekt, l_cke, l_rT, l_rek;
	Dev<uint32_t> sample_ray;
	Dev<uint32_t> cmap;  // compacted sample -> ray (LossWork::cmap)
	// progressive (cut-off-aware) inference: 0 off, 1 auto (when under PROGRESSIVE_RATIO of the kept samples were
	// composited at the last loss readback), 2 always; chunk ends of the rounds before the last (march.hip)
	int progressive_mode = 1;
	std::vector<uint32_t> chunk_ends{32, 64, 96};  // NEUS_CHUNK_ENDS="e0,e1,..." at creation overrides (A/B of schedules)
	std::vector<uint32_t> chunk_ends_cut;          // the chunk ends of a cut step (chosen with chunk_ends; empty: chunk_ends)
	const std::vector<uint32_t>& ends_for(bool cut) const { return cut && !chunk_ends_cut.empty() ? chunk_ends_cut : chunk_ends; }
	// Chunk ends chosen from the training state (chunk_auto: no explicit ends given): at each loss readback the mean
	// composited samples per ray with samples, mc (all-reduced counters: the same on every rank), sets three rounds
	// {e, 2e, rest} with e = 0.5 mc + 12 rounded to 8 in [24, 128]. Measured at the bench workload (Config S, R = Nc =
	// 2^18, profiles/r04fg_chunk_ends_sweep.txt, r04hi_*): step 800 (mc ~117) best at e = 64 (1.237 ms vs 1.283 for
	// {32, 64, 96}), step 1600 (mc ~39) best at e = 32 (1.203 ms vs 1.308 for e = 64). The rounds only change which
	// samples are evaluated, never a result (bit-identical to the one pass).
	bool chunk_auto = true;
	void choose_chunk_ends(uint32_t composited, uint32_t rays_with_samples) {
		if (!chunk_auto || rays_with_samples == 0) return;
		const float mc = (float)composited / (float)rays_with_samples;
		const uint32_t e = std::min(128u, std::max(24u, 8u * (uint32_t)std::lround((0.5f * mc + 12.f) / 8.f)));
		chunk_ends.assign({e, 2 * e});
		// With the compaction cut (and the march cut) the later rounds see only the rays before the cut (a few thousand at
		// the bench's shape), so their fixed cost - launches, scans, the cut - outweighs the samples a third round saves:
		// two rounds, the first twice as long (steps 800 / 1600: 0.815 / 0.895 -> 0.773 / 0.878 ms/step,
		// profiles/r06y_chunk_ends_cut_sweep.txt). NEUS_CHUNK_SCALE / NEUS_CHUNK_ROUNDS (2 or 3) override, for sweeps.
		static const float scale = [] { const char* v = std::getenv("NEUS_CHUNK_SCALE"); return v ? (float)std::atof(v) : 2.f; }();
		static const int rounds = [] { const char* v = std::getenv("NEUS_CHUNK_ROUNDS"); return v ? std::atoi(v) : 2; }();
		const uint32_t ec = std::min(256u, std::max(24u, 8u * (uint32_t)std::lround(scale * (0.5f * mc + 12.f) / 8.f)));
		if (rounds == 2) chunk_ends_cut.assign({ec});
		else chunk_ends_cut.assign({ec, 2 * ec});
	}
	float last_keep_ratio = 1.f;
	static constexpr float PROGRESSIVE_RATIO = 0.7f;
	Dev<uint32_t> chunk_list, chunk_cnt;  // chunk_cnt: [k] round k's sample list length, [16] the long-ray list's, [32 + k] open rays
	Dev<uint32_t> open_rays[2];          // the rays still open after a round (ping-pong: round k reads [(k - 1) & 1])
	// spatial ray order of the progressive rounds (RaySort; NEUS_RAY_SORT=0: slot order, one-XCD-agnostic lists)
	Dev<uint32_t> rs_hist, rs_off, rs_perm;
	Dev<uint16_t> rs_key;
	bool ray_sort = [] { const char* e = std::getenv("NEUS_RAY_SORT"); return !(e && e[0] == '0'); }();
	static constexpr uint32_t OPEN_CNT = 32;
	static constexpr uint32_t RS_N_PERM = 48;  // chunk_cnt slot: the ray order's length (k_ray_sort_scan)
	static constexpr uint32_t RAW_CNT = 49;    // chunk_cnt [49 + k]: rays open after round k, before the compaction cut (k = 0)
	// The compaction cut (march.hip k_prog_cut): with fixed rays per batch the later progressive rounds skip the rays whose
	// compaction base is already past the batch after a round. Training is bitwise the same; what changes is the summed
	// composited count of such a step (a lower bound, still >= the batch), which with fixed rays feeds no result - only the
	// logged loss scale, the chunk-end rule and the stats. So a step that the host reads back (a loss readback step, the last
	// step of a train call) never cuts, and every value the host sees is the uncut one. NEUS_PROG_CUT=0 turns it off.
	bool prog_cut = [] { const char* e = std::getenv("NEUS_PROG_CUT"); return !(e && e[0] == '0'); }();
	// With the spatial ray order, round 0 itself is split too: the sort puts the rays of the slots below the previous step's
	// cut (+ 1/4, + 1024: cutw[CW_EST]) first (pass A); once pass A is scanned the cut is known whenever the prefix reaches
	// the batch in those slots, and pass B (the rest of round 0) then has nothing to do.
	Dev<uint32_t> open_raw, cutw;  // the rays open after round 0, before the cut; the cut words (kernels.h CW_*)
	uint64_t cut_steps = 0;
	uint32_t call_left = 0;        // steps of the current train call after the current one
	bool la_cut = false;           // the pending lookahead's step cuts (its sort was split)
	bool la_mcut = false;          // the pending lookahead's march was cut (march_cut_for)
	bool cut_for(uint32_t step, bool progressive, bool last_in_call, bool dyn) const {
		const uint32_t nch = (uint32_t)chunk_ends.size() + 1;
		return prog_cut && progressive && cfg.fixed_rays_per_batch && !dyn && step % 16 != 0 && !last_in_call && nch >= 2 && nch <= 15;
	}
	// The march cut: on a cut step the compaction cut lies, nearly always, well inside the slots below the
	// split estimate (cutw[CW_EST]: at the bench's step 800, 5.6 K of the 41 K kept slots), and no ray past it contributes a
	// training sample. So such a step generates and marches only those slots (MarchWork::est_cut). Two things make that
	// step's training differ from the full march's, and k_loss_ray checks both (the witness): the marched slots may not
	// fill the batch, and - on the step after - the reference's cap on the pre-compaction samples (max_inference, from the
	// cut step's requested count) is then known only to be at least the marched slots' count, so a contributing ray past
	// that bound might have been dropped there. Either sets StepState::cut_abort (all-reduced with the step's counters):
	// the optimizer and the step counters of that step then change nothing, the host sees the word before it queues the
	// next step, restores its own state to the step's start and runs the step again with the full march (after recounting
	// the step before it in full when that one was cut, which makes its cap exact). The trained parameters are those of
	// the full march in every case. A step the host reads back, one with (or before) an occupancy update, and the last two
	// steps of a train call never cut the march, so the loss readback and the end of a call need no extra wait.
	// NEUS_MARCH_CUT=0 turns it off.
	bool march_cut_on = [] { const char* e = std::getenv("NEUS_MARCH_CUT"); return !(e && e[0] == '0'); }();
	bool force_full = false;      // the step being re-run marches every slot
	// the occupancy-biased samples binned by their coarse cell before the density pass (NEUS_OCC_NU_SORT=1): bitwise the
	// same grid, but 0.756-0.764 -> 0.765-0.771 ms/step at step 800 (profiles/r06occ_nu_sort_ab.txt: the binning's
	// atomics on the few occupied bins cost more than the pass saves); off
	bool occ_nu_sort = [] { const char* e = std::getenv("NEUS_OCC_NU_SORT"); return e && e[0] == '1'; }();
	Dev<uint32_t> occ_nu_key, occ_nu_list, occ_nu_bins;
	bool abort_direct = false;            // the last risky step's word comes through abort_word (one rank)
	volatile uint32_t* abort_word = nullptr;  // host-coherent pinned word k_loss_grad stores the witness to (one rank)
	uint32_t mcut_div = [] { const char* e = std::getenv("NEUS_DBG_MARCH_CUT_DIV"); return e ? (uint32_t)std::max(1, std::atoi(e)) : 1u; }();  // test hook
	bool mc_hist[2] = {false, false};  // the march of the last issued step / of the one before it was cut
	struct StepSnap {
		uint32_t training_step = 0, canonical_step = 0, adam_step = 0, call_left = 0;
		int enc_step = 0;
		float lr_factor = 1.f;
		pcg32 rng{};
		uint64_t la_steps = 0, cut_steps = 0, adam_split_steps = 0, mcut_steps = 0;
	};
	StepSnap snap[2];             // the host's step state at the start of the last issued step / of the one before it
	bool abort_pending = false;   // the last issued step's abort word is on its way to pinned[100] (ev_abort)
	hipEvent_t ev_abort = nullptr, ev_abort_src = nullptr;
	uint64_t mcut_steps = 0, mcut_reruns = 0;
	Dev<StepState> st_recount;
	static bool occ_at(uint32_t cs) { const uint32_t n_prep = std::min(16u, std::max(1u, cs / 16u)); return cs % n_prep == 0; }
	bool march_cut_for(uint32_t step, bool cut, uint32_t left_at_step) const {
		if (!march_cut_on || force_full || !cut || profiling || !mwork.balanced || mwork.lanes_per_ray != 8 || ds.cone_angle != 0.0f) return false;
		return (step + 1) % 16 != 0 && left_at_step >= 2 && !occ_at(step) && !occ_at(step + 1);
	}
	Dev<uint32_t> long_rays;  // the loss scan's wave-per-ray list (+ its counter in chunk_cnt[16])
	TrainBufs tbuf{};
	// RNG + counters (testbed.cu:2087-2101)
	pcg32 rng, density_grid_rng;
	uint32_t training_step = 0;
	uint32_t adam_step = 0;
	float lr_factor = 1.f;
	// the grid encoding's training step (GridEncoding::set_training_step, testbed.cu:2651-2657): set by every train
	// step (minus the global-movement steps on frames >= 1), 0 for a fresh network; render / SDF grid / mesh colours
	// use its progressive level, as the reference's inference does
	int enc_step = 0;
	// stats
	float loss_scalar_ema = 0.f, last_loss = 0.f, ek_loss = 0.f, mask_loss = 0.f, ray_loss = 0.f;
	uint32_t last_rays_with_samples = 0;
	bool loss_ema_init = false;
	float* pinned = nullptr;  // [0..3]: loss sum, ek sum, mask sum, grid mean; [32..47] render / mesh counts; [48]: the step scans'
	                          // give-up count; [64..]: StepState copy
	bool loss_pending = false;
	hipEvent_t ev_loss = nullptr;  // after the logged step's readback copies (consume_loss waits on it, not on the stream)
	// data parallel: RCCL communicator (production) or an in-process group
	ncclComm_t comm = nullptr;
	NeusLocalGroup* group = nullptr;
	// cross-process host-staged group (hostgroup.h): every collective staged on comm_stream through a pinned buffer
	NeusHostGroup* hgroup = nullptr;
	uint8_t* hg_stage = nullptr;
	size_t hg_stage_bytes = 0;
	uint32_t rank = 0, world = 1;
	// the exchange setting must be the same on every rank (the overlapped and grouped exchanges issue different
	// collective sequences): checked by an all-reduce at the first step after init or a change
	bool overlap_verified = false;
	bool force_coll = false;  // issue the collectives at world 1 too (a forced one-rank communicator, tests)
	// Overlapped gradient exchange: each finished gradient range is all-reduced as soon as its producer
	// finishes - the MLP blocks after the weight-gradient reduction, the grid levels group by group beside the scatter's
	// accumulation of the later groups - on comm_stream (RCCL; one stream keeps every rank's collectives in one order),
	// which the step's stream joins before the optimizer. Off (NEUS_EXCHANGE_OVERLAP=0, neus_testbed_set_exchange_overlap):
	// one grouped exchange after the backward. Elementwise sums are the same either way (bitwise with two ranks).
	bool exchange_overlap = true;
	hipStream_t comm_stream = nullptr;
	hipEvent_t ev_x[16] = {};
	uint32_t ev_x_n = 0;
	hipEvent_t ev_xdone = nullptr;
	bool x_pending = false;
	static constexpr uint32_t X_GROUPS = 3;   // grid level groups of the overlapped exchange (~equal bytes at L=14)
	// on comm_stream after the work queued so far on the step's stream (RCCL); the in-process group stages on the host
	hipStream_t x_stream() {
		if (!comm && !hgroup) return stream;
		if (!comm_stream) {
			if (main_prio) HIP_CHECK(hipStreamCreateWithPriority(&comm_stream, hipStreamNonBlocking, main_prio));
			else HIP_CHECK(hipStreamCreateWithFlags(&comm_stream, hipStreamNonBlocking));
			HIP_CHECK(hipEventCreateWithFlags(&ev_xdone, hipEventDisableTiming));
		}
		hipEvent_t& e = ev_x[ev_x_n++ % 16];
		if (!e) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
		HIP_CHECK(hipEventRecord(e, stream));
		HIP_CHECK(hipStreamWaitEvent(comm_stream, e, 0));
		x_pending = true;
		return comm_stream;
	}
	void x_join() {  // the step's stream waits for every exchange issued on comm_stream
		if (!x_pending) return;
		HIP_CHECK(hipEventRecord(ev_xdone, comm_stream));
		HIP_CHECK(hipStreamWaitEvent(stream, ev_xdone, 0));
		x_pending = false;
	}
	// level groups of the overlapped exchange: the active levels cut where the cumulative parameter count passes 1/3, 2/3
	ScatterSplit x_split(uint32_t valid, float* grid_grads) {
		ScatterSplit sp{};
		const uint32_t n_act = std::min(valid + 1, gl.n_levels);
		sp.n_groups = X_GROUPS;
		const uint64_t tot = gl.offset[n_act];
		uint32_t gi = 0;
		for (uint32_t l = 1; l < n_act && gi + 1 < X_GROUPS; ++l)
			if ((uint64_t)gl.offset[l] * X_GROUPS >= tot * (gi + 1)) sp.level_end[gi++] = l;
		for (; gi + 1 < X_GROUPS; ++gi) sp.level_end[gi] = n_act;
		sp.level_end[X_GROUPS - 1] = n_act;
		sp.done = [this, grid_grads](uint32_t lo, uint32_t hi) {
			hipStream_t xs = x_stream();
			allreduce_f32(grid_grads + 2 * (size_t)gl.offset[lo], 2 * (size_t)(gl.offset[hi] - gl.offset[lo]), false, xs);
		};
		return sp;
	}
	uint64_t coll_calls = 0, coll_bytes = 0, coll_bytes_step = 0;
	bool coll_on() const { return world > 1 || force_coll; }
	// profiling
	bool profiling = false;
	static constexpr int N_PHASES = NEUS_N_PHASES;
	// Two sets of phase events (steps alternate), so reading one step's timings never idles the GPU:
	// the step after it is already queued. The phase marks skip the system-scope release fence (it
	// writes back and invalidates the caches, which would slow the kernel after every mark).
	hipEvent_t ev[2][N_PHASES + 1] = {};
	hipEvent_t ev_done[2] = {};
	StepState* prof_st = nullptr;  // pinned, one StepState copy per event set
	bool prof_pending[2] = {false, false};
	int prof_par = 0;
	double phase_ms[N_PHASES] = {};
	double phase_npre = 0, phase_ntrain = 0;
	uint32_t phase_steps = 0;

	NeusTestbed(int dev) : device(dev) {
		HIP_CHECK(hipSetDevice(device));
		{
			// The step's streams at the highest priority, the lookahead's at the lowest (train_step). With the step's
			// streams at the default priority, a testbed created after another one was destroyed ran the 16-level bench leg
			// at 1.91 ms/step instead of 1.27 with the lookahead at the lowest priority (profiles/r05l16_priorities_ab.txt),
			// presumably from how the runtime maps the streams onto its few hardware queues; explicit priorities on every
			// stream keep it at 1.24. NEUS_MAIN_PRIO=0: the default priority.
			const char* e = std::getenv("NEUS_MAIN_PRIO");
			int lo = 0, hi = 0;
			HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
			main_prio = hi;
			if (!(e && e[0] == '0')) {
				HIP_CHECK(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, hi));
				HIP_CHECK(hipStreamCreateWithPriority(&aux_stream, hipStreamNonBlocking, hi));
			} else {
				main_prio = 0;
				HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
				HIP_CHECK(hipStreamCreateWithFlags(&aux_stream, hipStreamNonBlocking));
			}
		}
		HIP_CHECK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
		HIP_CHECK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
		HIP_CHECK(hipEventCreateWithFlags(&ev_loss, hipEventDisableTiming));
		HIP_CHECK(hipHostMalloc((void**)&pinned, 128 * sizeof(float)));
		for (auto& set : ev)
			for (auto& e : set) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
		for (auto& e : ev_done) HIP_CHECK(hipEventCreate(&e));
		HIP_CHECK(hipHostMalloc((void**)&prof_st, 2 * sizeof(StepState)));
		st.alloc(1);
		HIP_CHECK(hipMemset(st.p, 0, sizeof(StepState)));
		// pcg32 jump-ahead table of the streams this Testbed draws from (pcg32{seed} / pcg32{next_uint()}: increment 3)
		std::vector<PcgJump> jt(PCG_JUMP_LEVELS * PCG_JUMP_N);
		for (uint32_t j = 0; j < PCG_JUMP_LEVELS; ++j)
			for (uint32_t k = 0; k < PCG_JUMP_N; ++k) jt[j * PCG_JUMP_N + k] = pcg_jump(PCG_INC, (uint64_t)k << (j * PCG_JUMP_BITS));
		pcg_tab.alloc(jt.size());
		HIP_CHECK(hipMemcpy(pcg_tab.p, jt.data(), jt.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
	}
	static constexpr uint64_t PCG_INC = 3u;  // make_pcg32(s) = pcg32 stream 1: inc = (1 << 1) | 1
	PcgJumpTable jump_table() const { return PcgJumpTable{pcg_tab.p, PCG_INC}; }
	~NeusTestbed() {
		if (stream) (void)hipStreamSynchronize(stream);
		if (comm) ncclCommDestroy(comm);
		for (auto& set : ev)
			for (auto& e : set) if (e) (void)hipEventDestroy(e);
		for (auto& e : ev_done) if (e) (void)hipEventDestroy(e);
		if (prof_st) (void)hipHostFree(prof_st);
		if (pinned) (void)hipHostFree(pinned);
		if (abort_word) (void)hipHostFree((void*)abort_word);
		if (aux_stream) { (void)hipStreamSynchronize(aux_stream); (void)hipStreamDestroy(aux_stream); }
		if (la_stream) { (void)hipStreamSynchronize(la_stream); (void)hipStreamDestroy(la_stream); }
		if (ev_la_start) (void)hipEventDestroy(ev_la_start);
		if (ev_la_done) (void)hipEventDestroy(ev_la_done);
		for (auto& e : ad_ev) if (e) (void)hipEventDestroy(e);
		if (ad_done) (void)hipEventDestroy(ad_done);
		for (auto& e : xt_ev) for (auto& x : e) if (x) (void)hipEventDestroy(x);
		for (hipEvent_t e : la_stat_ev) (void)hipEventDestroy(e);
		if (ev_fork) (void)hipEventDestroy(ev_fork);
		if (ev_join) (void)hipEventDestroy(ev_join);
		if (ev_loss) (void)hipEventDestroy(ev_loss);
		if (comm_stream) { (void)hipStreamSynchronize(comm_stream); (void)hipStreamDestroy(comm_stream); }
		if (hg_stage) (void)hipHostFree(hg_stage);
		for (auto& e : ev_x) if (e) (void)hipEventDestroy(e);
		if (ev_xdone) (void)hipEventDestroy(ev_xdone);
		for (auto& e : it_ev) if (e) (void)hipEventDestroy(e);
		if (stream) (void)hipStreamDestroy(stream);
	}

	// ------------------------------------------------------------ dataset (load_nerf, testbed_nerf.cu:2964-3095)
	void set_dataset(uint32_t n_images, const NeusImage* imgs, float aabb_scale_) {
		if (n_images == 0) throw std::runtime_error("set_dataset: no images");
		aabb_scale = aabb_scale_;
		const int s = (int)aabb_scale;
		if (s < 1 || (s & (s - 1)) != 0) throw std::runtime_error("NeRF dataset's `aabb_scale` must be a power of two");
		if (s > (1 << (NERF_CASCADES - 1))) throw std::runtime_error("NeRF dataset must have aabb_scale <= 128");
		std::vector<uint64_t> offs(n_images);
		std::vector<int32_t> r(2 * n_images);
		std::vector<float> f(2 * n_images), p(2 * n_images), x(12 * n_images);
		uint64_t total = 0;
		for (uint32_t i = 0; i < n_images; ++i) {
			offs[i] = total;
			total += (uint64_t)imgs[i].width * imgs[i].height;
			r[2 * i] = imgs[i].width; r[2 * i + 1] = imgs[i].height;
			f[2 * i] = imgs[i].focal[0]; f[2 * i + 1] = imgs[i].focal[1];
			p[2 * i] = imgs[i].principal[0]; p[2 * i + 1] = imgs[i].principal[1];
			std::memcpy(&x[12 * i], imgs[i].xform, 12 * sizeof(float));
		}
		pixels.alloc(total); pix_off.alloc(n_images); res.alloc(2 * n_images); focal.alloc(2 * n_images); pp.alloc(2 * n_images); xform.alloc(12 * n_images);
		for (uint32_t i = 0; i < n_images; ++i)
			HIP_CHECK(hipMemcpy(pixels.p + offs[i], imgs[i].rgba8, (size_t)imgs[i].width * imgs[i].height * 4, hipMemcpyHostToDevice));
		HIP_CHECK(hipMemcpy(pix_off.p, offs.data(), n_images * 8, hipMemcpyHostToDevice));
		HIP_CHECK(hipMemcpy(res.p, r.data(), r.size() * 4, hipMemcpyHostToDevice));
		HIP_CHECK(hipMemcpy(focal.p, f.data(), f.size() * 4, hipMemcpyHostToDevice));
		HIP_CHECK(hipMemcpy(pp.p, p.data(), p.size() * 4, hipMemcpyHostToDevice));
		HIP_CHECK(hipMemcpy(xform.p, x.data(), x.size() * 4, hipMemcpyHostToDevice));
		ds.pixels = pixels.p; ds.pix_off = pix_off.p; ds.res = res.p; ds.focal = focal.p; ds.pp = pp.p; ds.xform = xform.p;
		srgb_lut.alloc(256);
		launch_srgb_lut(stream, srgb_lut.p);
		HIP_CHECK(hipStreamSynchronize(stream));
		ds.lin_lut = srgb_lut.p;
		ds.n_images = n_images;
		host_focal = f; host_pp = p; host_xform = x; host_res = r;
		const float infl = 0.5f * (float)std::min(1 << (NERF_CASCADES - 1), s);
		for (int d = 0; d < 3; ++d) { ds.aabb_min[d] = 0.5f - infl; ds.aabb_max[d] = 0.5f + infl; }
		max_cascade = 0;
		while ((1 << max_cascade) < s) ++max_cascade;
		ds.cone_angle = s <= 1 ? 0.0f : (1.0f / 256.0f);
		have_data = true;
		const uint32_t n_cells = GRID3 * (max_cascade + 1);
		density_grid.alloc(n_cells); density_tmp.alloc(n_cells);
		HIP_CHECK(hipMemset(density_grid.p, 0, n_cells * 4));
		bitfield.alloc(GRID3 / 8 * NERF_CASCADES);
		HIP_CHECK(hipMemset(bitfield.p, 0xff, GRID3 / 8 * NERF_CASCADES));
		bf_lin.alloc(LIN_WORDS);
		launch_bitfield_linear(stream, bitfield.p, bf_lin.p);
		occ_bbox.alloc(occ_bbox_scratch_floats());
		launch_occ_bbox(stream, bitfield.p, occ_bbox.p);
		{ const char* e = std::getenv("NEUS_RAY_CULL"); ray_cull = !(e && e[0] == '0'); }
		{ const char* e = std::getenv("NEUS_EXCHANGE_OVERLAP"); exchange_overlap = !(e && e[0] == '0'); }
		{ const char* e = std::getenv("NEUS_OCC_SORT"); occ_sort = !(e && e[0] == '0'); }
		if (const char* e = std::getenv("NEUS_CHUNK_ENDS")) {
			std::vector<uint32_t> v;
			for (const char* p = e; *p;) { char* q = nullptr; const unsigned long x = std::strtoul(p, &q, 10); if (q == p) break; v.push_back((uint32_t)x); p = *q ? q + 1 : q; }
			bool ok = !v.empty() && v.size() <= 14 && v[0] > 0;
			for (size_t k = 1; k < v.size(); ++k) ok = ok && v[k] > v[k - 1];
			if (ok) { chunk_ends = v; chunk_auto = false; chunk_ends_cut.clear(); }
		}
		{ const char* e = std::getenv("NEUS_SCATTER_NOSKIP"); scatter_noskip = e && e[0] == '1'; }
		grid_mean.alloc(4); grid_partial.alloc(GRID3 / 1024);
		HIP_CHECK(hipMemset(grid_mean.p, 0, 16));
	}

	// ------------------------------------------------------------ network (reset_network, testbed.cu:2084-2349)
	void reset_network(const NeusNetworkConfig& c, const float* geo) {
		if (!have_data) throw std::runtime_error("reload_network: load training data first");
		setup_network(c, geo);
		alloc_step_workspace();
	}

	// initial parameters (trainer.h:54-109): seed_seq{seed} -> pcg32; xavier MLPs (the density MLP replaced by
	// `geo` when given), hash grid U(-1e-4, 1e-4), variance 0.3
	std::vector<float> initial_params(uint32_t seed, const float* geo) const {
		std::seed_seq seq{seed};
		std::vector<uint32_t> seeds(2);
		seq.generate(seeds.begin(), seeds.end());
		return initial_params_rng(make_pcg32(seeds.front()), geo);
	}
	// NerfNetwork::initialize_params (nerf_network.h:741-886) drawing from `rnd`
	std::vector<float> initial_params_rng(pcg32 rnd, const float* geo) const {
		const Layout& l = lay;
		const uint32_t P = l.P;
		std::vector<float> h(P, 0.f);
		{
			auto xavier = [&](uint32_t off, uint32_t out, uint32_t in) {
				const float scale = std::sqrt(6.0f / (float)(in + out));
				for (uint32_t i = 0; i < out * in; ++i) h[off + i] = rnd.next_float() * 2.0f * scale - scale;
			};
			xavier(l.off_d0, l.W, l.din); xavier(l.off_d1, 16, l.W);
			if (geo) std::memcpy(h.data(), geo, sizeof(float) * l.n_density);
			xavier(l.off_r0, l.W, 48); xavier(l.off_r1, l.W, l.W); xavier(l.off_r2, 16, l.W);
			// grid: generate_random_uniform(rnd, n, -1e-4, 1e-4) (random.h:67-91; 128-thread blocks)
			const size_t N = l.n_grid, per = 4, n_threads = (N + per - 1) / per, n_pad = (n_threads + 127) / 128 * 128;
			for (size_t i = 0; i < n_pad; ++i) {
				pcg32 r = rnd; r.advance((int64_t)(i * per));
				for (size_t j = 0; j < per; ++j) {
					const size_t idx = i + n_pad * j;
					if (idx >= N) break;
					h[l.grid_off + idx] = r.next_float() * (1e-4f - -1e-4f) + -1e-4f;
				}
			}
			rnd.advance((int64_t)N);
			for (int k = 0; k < 4; ++k) h[l.var_off + k] = 0.3f;  // nerf_network.h:881-882
		}
		return h;
	}

	// The network half of reset_network: config checks, grid tables, parameter layout and initial parameters, the
	// fp16 / transposed weight copies and the workspace of one forward + backward over `batch` samples (encode,
	// training MLP, weight gradients, grid scatter). The tcnn-shaped operator modules (neus_module_*) use only this.
	void setup_network(const NeusNetworkConfig& c, const float* geo, bool with_mlp = true) {
		if (c.n_features_per_level != 2) throw std::runtime_error("GridEncoding: only n_features_per_level = 2 is supported");
		if (c.n_levels == 0 || c.n_levels > MAX_LEVELS) throw std::runtime_error("GridEncoding: 1..16 levels supported");
		if (with_mlp && (c.n_density_hidden != 1 || c.n_rgb_hidden != 2)) throw std::runtime_error("NerfNetwork: density 1 hidden layer, rgb 2 hidden layers required on gfx950");
		if (with_mlp && !mlp_supported(c.n_levels, c.n_neurons)) throw std::runtime_error("NerfNetwork: unsupported (n_levels, n_neurons) combination for the gfx950 MLP kernels");
		if (c.batch_size == 0 || c.batch_size % 128 != 0) throw std::runtime_error("batch_size must be a positive multiple of 128");
		cfg = c;
		// per_level_scale (testbed.cu:2184-2187), grid tables (grid.h:1466-1501)
		float pls = c.per_level_scale;
		if (pls <= 0.f) pls = c.n_levels > 1 ? std::exp(std::log(c.top_resolution * aabb_scale / (float)c.base_resolution) / (c.n_levels - 1)) : 2.0f;
		cfg.per_level_scale = pls;
		gl = GridLevels{};
		gl.n_levels = c.n_levels;
		uint32_t offset = 0;
		for (uint32_t i = 0; i < c.n_levels; ++i) {
			const float scale = exp2f(i * std::log2(pls)) * c.base_resolution - 1.0f;
			const uint32_t resolution = (uint32_t)(std::ceil(scale)) + 1;
			const uint32_t max_params = 0xffffffffu / 2;
			uint32_t pil = std::pow((float)resolution, 3) > (float)max_params ? max_params : resolution * resolution * resolution;
			pil = next_multiple(pil, 8u);
			pil = std::min(pil, 1u << c.log2_hashmap_size);
			gl.offset[i] = offset; gl.res[i] = resolution; gl.scale[i] = (float)(resolution - 1);
			offset += pil;
		}
		gl.offset[c.n_levels] = offset;
		gl.dense_bits = 0;
		for (uint32_t i = 0; i < c.n_levels; ++i) {
			const uint64_t r = gl.res[i], hs = gl.offset[i + 1] - gl.offset[i];
			if (r * r * r <= hs) gl.dense_bits |= 1u << i;
			else if ((hs & (hs - 1)) != 0) throw std::runtime_error("hashed grid level with a non-power-of-two table");
		}
		// parameter layout (nerf_network.h:741-785)
		Layout& l = lay;
		l.L = c.n_levels; l.W = c.n_neurons; l.din = next_multiple(3 + 2 * c.n_levels, 16);
		l.off_d0 = 0; l.off_d1 = l.W * l.din; l.n_density = l.off_d1 + 16 * l.W;
		l.off_r0 = l.n_density; l.off_r1 = l.off_r0 + l.W * 48; l.off_r2 = l.off_r1 + l.W * l.W;
		l.n_rgb = l.off_r2 + 16 * l.W - l.n_density;
		l.n_matrix = l.n_density + l.n_rgb;
		l.grid_off = l.n_matrix; l.n_grid = offset * 2;
		l.var_off = l.grid_off + l.n_grid; l.P = l.var_off + 4;
		const uint32_t P = l.P;
		params_fp.alloc(P); grads.alloc(P); m1.alloc(P); m2.alloc(P); ema_tmp.alloc(P); adam_steps.alloc(P);
		params_h.alloc(P); ema_h.alloc(P);
		wT.alloc(l.din * l.W + l.W * 16 + 48 * l.W + l.W * l.W + l.W * 16 + 2 * l.din * l.W + 64);
		wT_ema.alloc(wT.n);
		const std::vector<float> h = initial_params(c.seed, geo);
		HIP_CHECK(hipMemcpy(params_fp.p, h.data(), (size_t)P * 4, hipMemcpyHostToDevice));
		HIP_CHECK(hipMemset(m1.p, 0, (size_t)P * 4)); HIP_CHECK(hipMemset(m2.p, 0, (size_t)P * 4));
		HIP_CHECK(hipMemset(ema_tmp.p, 0, (size_t)P * 4)); HIP_CHECK(hipMemset(adam_steps.p, 0, (size_t)P * 4));
		HIP_CHECK(hipMemset(ema_h.p, 0, (size_t)P * 2)); HIP_CHECK(hipMemset(grads.p, 0, (size_t)P * 4));
		ema_h_stale = false;
		launch_cast_half(stream, P, params_fp.p, params_h.p);
		setup_mlp_ptrs();
		prepare_weights();
		// RNG state (testbed.cu:2087-2101)
		rng = make_pcg32(c.seed);
		density_grid_rng = make_pcg32(rng.next_uint());
		(void)rng.next_uint();  // tv_loss_rng
		training_step = 0; adam_step = 0; lr_factor = 1.f; density_grid_ema_step = 0; enc_step = 0;
		occ_samples = 0; occ_updates = 0;
		loss_ema_init = false; loss_scalar_ema = last_loss = ek_loss = mask_loss = 0.f; loss_pending = false;
		nonfinite = aborted = false;
		// forward + backward workspace of one training batch
		batch = c.batch_size;
		max_samples = batch * 16;  // testbed_nerf.cu:3725
		enc.alloc((size_t)l.L * batch); dydx.alloc((size_t)6 * l.L * batch);  // training batch only: inference fuses the encode
		const size_t ld = batch;
		trainbuf.alloc(16 * ld + 2 * (2 * (size_t)l.L * ld) + 64);
		vbuf.alloc(batch);
		half_t* q = trainbuf.p;
		auto take = [&](size_t k) { half_t* r = q; q += (k + 7) / 8 * 8; return r; };
		tbuf = TrainBufs{};
		tbuf.d1_delta = take(16 * ld);
		tbuf.dLdenc = take(2 * (size_t)l.L * ld); tbuf.genc = take(2 * (size_t)l.L * ld);
		tbuf.v = vbuf.p;
		tbuf.var_grad = grads.p + l.var_off;
		mlp_blocks = mlp_train_blocks(l.L, l.W, batch);
		var_partial.alloc(mlp_blocks);
		tbuf.var_partial = var_partial.p;
		// one row of MLP weight-gradient partials per training-kernel block
		wgrad_partial.alloc((size_t)mlp_blocks * l.n_matrix);
		tbuf.wpartial = wgrad_partial.p;
		tbuf.n_matrix = l.n_matrix; tbuf.off_d1 = l.off_d1; tbuf.off_r0 = l.off_r0; tbuf.off_r1 = l.off_r1; tbuf.off_r2 = l.off_r2;
		tbuf.indeed_batch = (float)batch * (float)world;
		// binned grid-gradient scatter workspace (grid.hip)
		swork = ScatterWork{};
		swork.n_blocks = (batch + 255) / 256;
		// wide-block binning: 512-sample workgroups (NEUS_SCATTER_CHUNK=1024: 1024-sample ones)
		{
			const char* e = std::getenv("NEUS_SCATTER_CHUNK");
			swork.chunk = (e && std::string(e) == "1024") ? 1024u : (e && std::string(e) == "256") ? 256u : 512u;
		}
		swork.n_chunks = (batch + swork.chunk - 1) / swork.chunk;
		// per-block record regions (mode 2); NEUS_SCATTER=wide / binned select the wide-block (0) or the 256-sample (1)
		// histogram / scan / bin paths (bitwise A/B references)
		{
			const char* e = std::getenv("NEUS_SCATTER");
			swork.mode = !e ? 2u : std::string(e) == "binned" ? 1u : std::string(e) == "wide" ? 0u : 2u;
			if (swork.mode != 2 && swork.chunk == 256) { swork.chunk = 512; swork.n_chunks = (batch + 511) / 512; }  // wide binning: 512 / 1024
			// NEUS_SCATTER_LG=k: k workgroups per chunk each binning every k-th level (default: one per level)
			const char* lg = std::getenv("NEUS_SCATTER_LG");
			swork.level_groups = lg ? (uint32_t)std::max(0, std::atoi(lg)) : 0u;
		}
		swork.n_buckets = scatter_n_buckets(gl);
		if (swork.n_buckets > SB_MAX_BUCKETS) throw std::runtime_error("hash grid too large for the scatter buckets");
		const size_t n_bins = (size_t)swork.n_buckets * swork.n_blocks + 1;
		sc_counts.alloc(n_bins); sc_offs.alloc(n_bins);
		const size_t n_rec = std::max(scatter_records_capacity(swork.n_blocks * 256, l.L), (size_t)l.L * swork.n_chunks * swork.chunk * 8);
		sc_rec_g.alloc(n_rec); sc_rec_i.alloc(n_rec);
		swork.counts = sc_counts.p; swork.offs = sc_offs.p; swork.rec_g = sc_rec_g.p; swork.rec_i = sc_rec_i.p;
		{
			uint32_t n_split = 0;
			const std::vector<uint32_t> jobs = scatter_accum_jobs(gl, swork.n_buckets, n_split);
			sc_jobs.alloc(jobs.size());
			HIP_CHECK(hipMemcpy(sc_jobs.p, jobs.data(), jobs.size() * 4, hipMemcpyHostToDevice));
			uint32_t n_split2 = 0;
			const std::vector<uint32_t> jobs2 = scatter_region_jobs(gl, n_split2, sc_jobs2_before);
			sc_jobs2.alloc(jobs2.size());
			HIP_CHECK(hipMemcpy(sc_jobs2.p, jobs2.data(), jobs2.size() * 4, hipMemcpyHostToDevice));
			swork.jobs2 = (const uint4*)sc_jobs2.p; swork.n_jobs2 = (uint32_t)(jobs2.size() / 4);
			swork.xcd_group = 4;
			if (const char* e = std::getenv("NEUS_SC_XCD_GROUP")) swork.xcd_group = std::max(1u, (uint32_t)std::strtoul(e, nullptr, 10));
			if (sc_jobs2_before.size() > 17) throw std::runtime_error("region scatter: at most 16 levels");
			for (size_t k = 0; k < sc_jobs2_before.size(); ++k) swork.jobs2_before[k] = sc_jobs2_before[k];
			sc_rtab.alloc((size_t)l.L * swork.n_chunks * (SB_LEVEL_BUCKETS + 1));
			swork.rtab = sc_rtab.p;
			n_split = std::max(n_split, n_split2);
			sc_split.alloc(std::max<size_t>(1, (size_t)n_split * 2 * SB_SIZE)); sc_split_done.alloc(std::max(1u, n_split));
			HIP_CHECK(hipMemset(sc_split.p, 0, sc_split.n * sizeof(unsigned long long)));
			HIP_CHECK(hipMemset(sc_split_done.p, 0, sc_split_done.n * 4));
			swork.jobs = (const uint4*)sc_jobs.p; swork.split = sc_split.p; swork.split_done = sc_split_done.p;
			swork.n_jobs = (uint32_t)(jobs.size() / 4);
			swork.n_active = swork.n_buckets;
			sc_jobs_before.assign(swork.n_buckets + 1, 0u);
			for (size_t j = 0; j < jobs.size() / 4; ++j) sc_jobs_before[jobs[4 * j] + 1] = (uint32_t)j + 1;
			for (uint32_t b = 1; b <= swork.n_buckets; ++b) sc_jobs_before[b] = std::max(sc_jobs_before[b], sc_jobs_before[b - 1]);
			sc_zero_from = swork.n_buckets;  // nothing assumed
			sc_zero_from_e = gl.offset[gl.n_levels];
		}
		scan_tmp_bytes = std::max({scan_temp_bytes(MAX_RAYS), scan_temp_bytes((uint32_t)n_bins),
		                           scan_temp_bytes(2 * (2 * RS_BINS + 1) * ray_sort_blocks(MAX_RAYS))});
		scan_tmp.alloc(scan_tmp_bytes + 256);
		scan_temp_reset(stream, scan_tmp.p);
		HIP_CHECK(hipStreamSynchronize(stream));
	}

	// The training-step half of reset_network: ray / march / loss / compaction buffers (per-step state sized for
	// MAX_RAYS rays and 16 x batch samples), occupancy-update scratch, device counters, dynamic-scene state.
	void alloc_step_workspace() {
		rays.alloc(6 * (size_t)MAX_RAYS); startt.alloc((size_t)MAX_RAYS);
		march_rec.alloc((size_t)MAX_RAYS * NERF_STEPS); march_nrec.alloc(MAX_RAYS); march_queue.alloc(2);
		march_seg.alloc((size_t)MAX_RAYS * MARCH_SEG_RECS);
		mwork = MarchWork{march_rec.p, march_nrec.p, march_queue.p, march_waves(), march_seg.p, march_lanes(), jump_table()};
		{ const char* e = std::getenv("NEUS_MARCH_BALANCE"); mwork.balanced = !(e && e[0] == '0') ? 1u : 0u; }
		nreq.alloc(MAX_RAYS); base.alloc(MAX_RAYS);
		numsteps.alloc(2 * (size_t)MAX_RAYS); ccount.alloc(MAX_RAYS); cbase.alloc(MAX_RAYS);
		l_sa.alloc(max_samples); l_ekt.alloc(max_samples); sample_ray.alloc(max_samples); cmap.alloc(batch);
		l_ck4.alloc(max_samples / 8 + 1); l_cke.alloc(max_samples / 8 + 1);
		l_racc.alloc(MAX_RAYS); l_rgr.alloc(MAX_RAYS); l_rT.alloc(MAX_RAYS); l_rek.alloc(MAX_RAYS);
		// (the split round 0 of the compaction cut: pass B's list from max_samples, its rays from MAX_RAYS)
		chunk_list.alloc(2 * (size_t)max_samples); chunk_cnt.alloc(64); long_rays.alloc(MAX_RAYS);
		open_rays[0].alloc(MAX_RAYS); open_rays[1].alloc(MAX_RAYS); open_raw.alloc(MAX_RAYS); cutw.alloc(CW_WORDS);
		{ uint32_t w[CW_WORDS] = {}; w[CW_EST] = MAX_RAYS; HIP_CHECK(hipMemcpy(cutw.p, w, sizeof(w), hipMemcpyHostToDevice)); }
		rs_hist.alloc(2 * (size_t)(2 * RS_BINS + 1) * ray_sort_blocks(MAX_RAYS)); rs_off.alloc(rs_hist.n);
		rs_perm.alloc(2 * (size_t)MAX_RAYS); rs_key.alloc(MAX_RAYS);
		loss.alloc(MAX_RAYS); ek.alloc(MAX_RAYS); mask.alloc(MAX_RAYS); loss_sum.alloc(4); health_buf.alloc(4);
		coords.alloc((size_t)max_samples * COORD_W); net_out.alloc((size_t)max_samples * OUT_W);
		coords_c.alloc((size_t)batch * COORD_W); dL_dout.alloc((size_t)batch * OUT_W);
		const NeusNetworkConfig& c = cfg;
		const uint32_t n_occ = GRID3 * (max_cascade + 1) * 2;
		occ_pos.alloc(3 * (size_t)n_occ); occ_idx.alloc(n_occ); occ_density.alloc(n_occ);
		// device step state (Counters, testbed.h:596-616)
		StepState s{};
		s.rays_per_batch = c.fixed_rays_per_batch ? c.fixed_rays_per_batch : (1u << 12);
		s.max_inference = max_samples;
		HIP_CHECK(hipMemcpy(st.p, &s, sizeof(s), hipMemcpyHostToDevice));
		HIP_CHECK(hipMemset(density_grid.p, 0, density_grid.n * 4));
		// dynamic scenes: identity accumulated movement, identity local movement (DeltaNetwork::initialize_params,
		// transform_network.h:335-383; NerfNetwork::init_accumulation_movement, nerf_network.h:1042-1105)
		coords_def.alloc((size_t)max_samples * COORD_W); coords_cdef.alloc((size_t)batch * COORD_W); dpos.alloc(batch);
		delta.alloc(1); delta_partial.alloc(delta_partial_floats());
		reset_delta();
		ds.motion = RayMotion{};
		ds.motion.R[0] = ds.motion.R[4] = ds.motion.R[8] = 1.f;
		// the frame index and the phase flags belong to the Testbed, not the network: reset_network keeps them
		// (testbed.cu:2084-2349; load_snapshot on frame k of run_dynamic.py's test pass relies on it)
		canonical_step = 0;
		HIP_CHECK(hipStreamSynchronize(stream));
		have_net = true;
	}

	// a fresh global-move trainer: identity local movement, zero Adam state (testbed.cu:2569-2578)
	void reset_delta() {
		DeltaState h{};
		h.p[4] = 1.f; h.p[8] = 1.f;  // rotation 6D (1, 0, 0, 0, 1, 0)
		HIP_CHECK(hipMemcpyAsync(delta.p, &h, sizeof(h), hipMemcpyHostToDevice, stream));
		launch_delta_prepare(stream, delta.p);
		delta_step = 0; delta_lr_factor = 1.f;
	}

	// ------------------------------------------------------------ dynamic scenes: next frame (testbed.cu:2001-2082)
	void next_frame(uint32_t n_images, const NeusImage* imgs) {
		if (!have_net) throw std::runtime_error("next_frame: no network");
		HIP_CHECK(hipStreamSynchronize(stream));
		consume_loss();
		// accumulate_global_movement: fold this frame's local movement into the ray transform
		DeltaState h{};
		HIP_CHECK(hipMemcpy(&h, delta.p, sizeof(h), hipMemcpyDeviceToHost));
		RayMotion m = ds.motion;
		host_accumulate_movement(h.p, m.R, m.t);
		m.on = 1;
		// load_nerf(frame): the next frame's images and cameras (same aabb_scale)
		set_dataset(n_images, imgs, aabb_scale);
		ds.motion = m;
		++cur_frame;
		training_step = 0; canonical_step = 0;
		// save/load_snapshot_incremental: the new trainer starts from the serialized inference (EMA) weights,
		// fp16, with fresh optimizer state (Adam moments, per-parameter steps, EMA)
		const uint32_t P = lay.P;
		{
			std::vector<half_t> eh(P);
			sync_ema_h();
			HIP_CHECK(hipMemcpy(eh.data(), ema_h.p, (size_t)P * 2, hipMemcpyDeviceToHost));
			std::vector<float> ef(P);
			for (uint32_t i = 0; i < P; ++i) ef[i] = (float)eh[i];
			HIP_CHECK(hipMemcpy(params_fp.p, ef.data(), (size_t)P * 4, hipMemcpyHostToDevice));
			HIP_CHECK(hipMemcpy(params_h.p, eh.data(), (size_t)P * 2, hipMemcpyHostToDevice));
		}
		HIP_CHECK(hipMemset(m1.p, 0, (size_t)P * 4)); HIP_CHECK(hipMemset(m2.p, 0, (size_t)P * 4));
		HIP_CHECK(hipMemset(adam_steps.p, 0, (size_t)P * 4));
		// the fp32 EMA starts at the loaded weights: the first EMA step weighs it by 1 - decay^0 = 0, and until the
		// canonical optimizer steps (after the global-movement phase) it is what get_ema_params reports
		HIP_CHECK(hipMemcpy(ema_tmp.p, params_fp.p, (size_t)P * 4, hipMemcpyDeviceToDevice));
		adam_step = 0; lr_factor = 1.f;
		prepare_weights();
		// reset_network_incremental (testbed.cu:2351-2370): m_rng = seed, rays_per_batch = 4096, counters
		rng = make_pcg32(cfg.seed);
		StepState s{};
		s.rays_per_batch = cfg.fixed_rays_per_batch ? cfg.fixed_rays_per_batch : (1u << 12);
		s.max_inference = max_samples;
		HIP_CHECK(hipMemcpy(st.p, &s, sizeof(s), hipMemcpyHostToDevice));
		reset_delta();
		train_canonical = false;
		train_delta = cfg.predict_global_movement != 0;
		HIP_CHECK(hipStreamSynchronize(stream));
	}
	// Testbed::change_to_frame (testbed.cu:1939-1985): load frame `k`'s images and restart the step count with a
	// fresh optimizer (Adam moments, steps, EMA state); parameters, density grid state of the network, the ray
	// movement and the training phase flags stay (run_dynamic.py follows it with load_snapshot).
	void change_frame(uint32_t k, uint32_t n_images, const NeusImage* imgs) {
		if (!have_net) throw std::runtime_error("change_to_frame: no network");
		HIP_CHECK(hipStreamSynchronize(stream));
		consume_loss();
		const RayMotion m = ds.motion;
		set_dataset(n_images, imgs, aabb_scale);
		ds.motion = m;
		cur_frame = k;
		training_step = 0; canonical_step = 0;
		const uint32_t P = lay.P;
		HIP_CHECK(hipMemset(m1.p, 0, (size_t)P * 4)); HIP_CHECK(hipMemset(m2.p, 0, (size_t)P * 4));
		HIP_CHECK(hipMemset(adam_steps.p, 0, (size_t)P * 4));
		{  // the fp32 EMA restarts from the inference weights (weighted by 0 at the next EMA step)
			std::vector<half_t> eh(P);
			sync_ema_h();
			HIP_CHECK(hipMemcpy(eh.data(), ema_h.p, (size_t)P * 2, hipMemcpyDeviceToHost));
			std::vector<float> ef(P);
			for (uint32_t i = 0; i < P; ++i) ef[i] = (float)eh[i];
			HIP_CHECK(hipMemcpy(ema_tmp.p, ef.data(), (size_t)P * 4, hipMemcpyHostToDevice));
		}
		adam_step = 0; lr_factor = 1.f;
		HIP_CHECK(hipStreamSynchronize(stream));
	}
	// march waves launched (NEUS_MARCH_WAVES overrides). Default 0 = one lane per ray slot: the march is
	// latency-bound (occupancy lookups), and measured on MI355X every wave fewer than the slots was slower
	// (R = 2^18: 4096 waves 0.58 ms, 2048 0.75 ms, 1024 1.28 ms); the queue then only re-fills dropped slots.
	uint32_t march_waves() const {
		if (const char* e = std::getenv("NEUS_MARCH_WAVES")) return (uint32_t)std::strtoul(e, nullptr, 10);
		return 0;
	}
	// lanes marching one ray (segments of its step sequence, see march.hip): 8 (NEUS_MARCH_LANES = 1 / 4 / 8).
	// Measured on MI355X (Config S, R = 2^18, step 5): sampling 0.52 ms with 1 lane, 0.24 with 4, 0.21 with 8.
	uint32_t march_lanes() const {
		if (const char* e = std::getenv("NEUS_MARCH_LANES")) { const uint32_t v = (uint32_t)std::strtoul(e, nullptr, 10); return v == 1 || v == 4 || v == 16 ? v : 8u; }
		return 8;
	}
	uint32_t gm_steps() const { return cfg.predict_global_movement ? cfg.global_movement_steps : 0u; }

	void setup_mlp_ptrs() {
		setup_mlp_ptrs_for(params_h.p, wT.p, mlp);
		setup_mlp_ptrs_for(ema_h.p, wT_ema.p, mlp_ema);
		din_perm = DinPerm{};
		mlp_din_permutation(lay.L, din_perm.p);
		din_perm.din = lay.din; din_perm.W = lay.W;
	}
	void setup_mlp_ptrs_for(const half_t* base, half_t* t, MlpPtrs& mlp) {
		const Layout& l = lay;
		mlp.d0 = base + l.off_d0; mlp.d1 = base + l.off_d1;
		mlp.r0 = base + l.off_r0; mlp.r1 = base + l.off_r1; mlp.r2 = base + l.off_r2;
		auto take = [&](size_t k) { half_t* r = t; t += (k + 7) / 8 * 8; return r; };
		mlp.d0T = take(l.din * l.W); mlp.d1T = take(l.W * 16); mlp.r0T = take(48 * l.W); mlp.r1T = take(l.W * l.W); mlp.r2T = take(l.W * 16);
		mlp.d0p = take(l.din * l.W); mlp.d0Tp = take(l.din * l.W);
		mlp.var = base + l.var_off;
		mlp.sdf_bias = cfg.sdf_bias;
	}
	void prepare_weights() { prepare_weights_for(mlp); }
	void prepare_weights_for(const MlpPtrs& mlp) {
		const Layout& l = lay;
		TransposeJobs tj{};
		tj.j[0] = {mlp.d0, (half_t*)mlp.d0T, l.W, l.din};
		tj.j[1] = {mlp.d1, (half_t*)mlp.d1T, 16, l.W};
		tj.j[2] = {mlp.r0, (half_t*)mlp.r0T, l.W, 48};
		tj.j[3] = {mlp.r1, (half_t*)mlp.r1T, l.W, l.W};
		tj.j[4] = {mlp.r2, (half_t*)mlp.r2T, 16, l.W};
		tj.n = 5;
		launch_transpose_permute(stream, tj, mlp.d0, (half_t*)mlp.d0p, (half_t*)mlp.d0Tp, din_perm);
	}

	// progressive levels (grid.h:2427-2440)
	uint32_t valid_level_at(int step) const {
		if (step <= 0) return cfg.n_levels;
		const float v = std::ceil(cfg.base_valid_level_scale * cfg.n_levels + cfg.valid_level_scale * std::max(0, (int)(step - (int)cfg.base_training_step)));
		return std::min(cfg.n_levels, (uint32_t)v);
	}
	float cos_anneal() const { return cfg.anneal_end == 0 ? 1.0f : std::min(1.0f, (float)training_step / cfg.anneal_end); }

	// ------------------------------------------------------------ network stages
	void encode(const uint32_t* n_ptr, uint32_t n_fixed, uint32_t n_cap, uint32_t ld, const float* c, uint32_t stride, uint32_t valid, bool want_dydx, hipStream_t s,
	            const EncodeRollover* ro = nullptr) {
		const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>((n_cap + 255) / 256, 2048));
		launch_grid_encode(s, n_ptr, n_fixed, ld, c, stride, gl, valid, params_h.p + lay.grid_off, enc.p, want_dydx ? dydx.p : nullptr, gx, ro);
	}
	void net_forward(const uint32_t* n_ptr, uint32_t n_fixed, uint32_t n_cap, const float* c, uint32_t valid, half_t* out, hipStream_t s) {
		const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((n_cap + 127) / 128, 8192));
		launch_nerf_infer(s, lay.L, lay.W, n_ptr, n_fixed, c, gl, valid, params_h.p + lay.grid_off, mlp, out, blocks);
	}
	// the reduction of the training kernels' per-block weight-gradient rows (and variance partials) into g
	MlpGradReduce grad_reduce(uint32_t n, float* g, const uint32_t* n_valid) const {
		MlpGradReduce r{};
		r.partial = wgrad_partial.p; r.n_blocks = mlp_train_blocks(lay.L, lay.W, n); r.n_matrix = lay.n_matrix; r.g = g;
		r.n_valid = n_valid; r.var_partial = var_partial.p; r.var_blocks = r.n_blocks; r.var_grad = g + lay.var_off;
		return r;
	}
	// The grid-gradient buckets past the progressive valid level get no records: their gradient is zero. For the
	// testbed's own gradient buffer the scatter skips them once they hold zeros (early in training ~2,500 of ~2,600
	// buckets, each a 64 KB-LDS workgroup), zeroing first the range a lower valid level than the previous step's
	// leaves stale (a reloaded network, a frame switch).
	ScatterWork scatter_work_for(float* g_grid, uint32_t valid, hipStream_t s) {
		if (g_grid != grads.p + lay.grid_off || sc_jobs_before.empty()) return swork;
		const uint32_t L = gl.n_levels, n_entries = gl.offset[L];
		if (scatter_noskip) {  // A/B reference: the whole grid gradient zeroed before every scatter
			HIP_CHECK(hipMemsetAsync(g_grid, 0, (size_t)n_entries * 2 * sizeof(float), s));
			sc_zero_from = swork.n_buckets; sc_zero_from_e = n_entries;
			return swork;
		}
		if (swork.mode == 2) {
			// the accumulation writes exactly the entries of the levels up to the valid one
			const uint32_t lv = std::min(valid + 1, L), e_end = gl.offset[lv];
			if (sc_zero_from_e > e_end) HIP_CHECK(hipMemsetAsync(g_grid + 2 * (size_t)e_end, 0, (size_t)(sc_zero_from_e - e_end) * 2 * sizeof(float), s));
			sc_zero_from_e = e_end;
			ScatterWork w = swork;
			w.n_jobs2 = sc_jobs2_before[lv];
			return w;
		}
		const uint32_t sb = valid + 1 >= L ? swork.n_buckets : std::min(swork.n_buckets, (gl.offset[valid + 1] + SB_SIZE - 1) / SB_SIZE);
		if (sc_zero_from > sb) {
			const size_t e_lo = (size_t)sb * SB_SIZE, e_hi = std::min<size_t>((size_t)sc_zero_from * SB_SIZE, n_entries);
			if (e_hi > e_lo) HIP_CHECK(hipMemsetAsync(g_grid + 2 * e_lo, 0, (e_hi - e_lo) * 2 * sizeof(float), s));
		}
		sc_zero_from = sb;
		ScatterWork w = swork;
		w.n_jobs = sc_jobs_before[sb];
		w.n_active = sb;  // histogram and scan only the buckets that can receive records
		return w;
	}
	// forward recompute + backward into g (fp32 [P], zeroed by the caller)
	void net_backward(const uint32_t* n_valid_ptr, const uint32_t* n_train_ptr, uint32_t n, const float* c, uint32_t valid,
	                  const half_t* dlo, float* g, hipStream_t s, bool marks = false, bool canonical = true, const EncodeRollover* ro = nullptr,
	                  bool exchange = false, AdamSplit* as = nullptr) {
		const uint32_t ld = n;
		encode(n_train_ptr, n, n, ld, c, COORD_W, valid, true, s, ro);
		la_fire(1);
		if (marks) mark(5);
		TrainBufs t = tbuf;
		t.var_grad = g + lay.var_off;
		launch_mlp_train(s, lay.L, lay.W, n_valid_ptr, n, ld, c, (const half_t*)enc.p, dydx.p, dlo, mlp, t);
		la_fire(2);
		if (marks) mark(6);
		if (!canonical) { if (marks) mark(7); return; }  // global-movement phase: canonical gradients unused
		// the MLP weight gradients were accumulated inside the training kernels: one small fixed-order reduction
		launch_mlp_grad_reduce(s, grad_reduce(n, g, n_train_ptr));
		la_fire(3);
		if (exchange) {  // the MLP blocks and the variance are final: their exchange runs beside the grid scatter
			hipStream_t xs = x_stream();
			allreduce_f32(g, lay.grid_off, false, xs);
			allreduce_f32(g + lay.var_off, lay.P - lay.var_off, false, xs);
			if (as) as->on = xs;  // (the optimizer's pieces follow their ranges' all-reduces on the exchange stream)
		}
		if (as) adam_issue(*as, lay.grid_off, g, true);  // the MLP blocks (and their transposed copies) beside the scatter
		if (marks) mark(7);
		const ScatterWork sw = scatter_work_for(g + lay.grid_off, valid, s);
		ScatterSplit sp = exchange && sw.mode == 2 ? x_split(valid, g + lay.grid_off) : ScatterSplit{};
		const bool a_split = as && sw.mode == 2;
		if (a_split) {  // the level groups of the overlapped exchange; each group's Adam once its accumulation (and exchange) is queued
			if (!exchange) sp = x_split(valid, g + lay.grid_off);
			auto xdone = exchange ? sp.done : std::function<void(uint32_t, uint32_t)>();
			sp.done = [this, as, g, xdone](uint32_t lo, uint32_t hi) {
				if (xdone) xdone(lo, hi);
				adam_issue(*as, lay.grid_off + 2 * gl.offset[hi], g, false);
			};
		}
		launch_grid_scatter(s, n_train_ptr, n, ld, c, COORD_W, gl, valid, tbuf.dLdenc, tbuf.genc, tbuf.v, g + lay.grid_off, sw, scan_tmp.p,
		                    scan_tmp_bytes, (exchange || a_split) && sw.mode == 2 ? &sp : nullptr);
		if (exchange && sw.mode != 2) {  // other scatter modes: the grid exchange after the whole scatter
			const size_t grid_act = 2 * (size_t)gl.offset[std::min(valid + 1, gl.n_levels)];
			allreduce_f32(g + lay.grid_off, grid_act, false, x_stream());
		}
	}

	// ------------------------------------------------------------ collectives
	void coll_begin() { if (comm) NCCL_CHECK(ncclGroupStart()); }
	void coll_end() { if (comm) NCCL_CHECK(ncclGroupEnd()); }
	void allreduce_f32(float* p, size_t n, bool max_op = false, hipStream_t on = nullptr) {
		if (!coll_on() || n == 0) return;
		++coll_calls; coll_bytes += n * 4; coll_bytes_step += n * 4;
		if (comm) NCCL_CHECK(ncclAllReduce(p, p, n, ncclFloat32, max_op ? ncclMax : ncclSum, comm, on ? on : stream));
		else if (hgroup) hg_allreduce(p, n * 4, NeusHostGroup::F32, max_op ? NeusHostGroup::MAX : NeusHostGroup::SUM, on);
		else if (group) group->allreduce<float>(rank, p, n, max_op ? NeusLocalGroup::MAX : NeusLocalGroup::SUM, stream);
		else throw std::runtime_error("data parallel: no communicator");
	}
	void allreduce_u32(uint32_t* p, size_t n, hipStream_t on = nullptr) {
		if (!coll_on() || n == 0) return;
		++coll_calls; coll_bytes += n * 4; coll_bytes_step += n * 4;
		if (comm) NCCL_CHECK(ncclAllReduce(p, p, n, ncclUint32, ncclSum, comm, on ? on : stream));
		else if (hgroup) hg_allreduce(p, n * 4, NeusHostGroup::U32, NeusHostGroup::SUM, on);
		else if (group) group->allreduce<uint32_t>(rank, p, n, NeusLocalGroup::SUM, stream);
		else throw std::runtime_error("data parallel: no communicator");
	}
	// A host-group collective on comm_stream: device -> pinned stage, the socket exchange in a host function, stage ->
	// device. Issued from the step's stream (on == nullptr / stream), it is gated after the work queued there and the step's
	// stream waits for it; issued on comm_stream (the overlapped exchange), the stream order is the gate.
	void hg_allreduce(void* dev, size_t bytes, uint32_t type, uint32_t op, hipStream_t on) {
		const bool own = !(on && on == comm_stream);
		hipStream_t cs = own ? x_stream() : on;
		if (bytes > hg_stage_bytes) {  // grow: the queued collectives still read the old stage
			if (comm_stream) HIP_CHECK(hipStreamSynchronize(comm_stream));
			if (hg_stage) HIP_CHECK(hipHostFree(hg_stage));
			hg_stage_bytes = std::max(bytes, (size_t)1 << 20);
			HIP_CHECK(hipHostMalloc((void**)&hg_stage, hg_stage_bytes));
		}
		HIP_CHECK(hipMemcpyAsync(hg_stage, dev, bytes, hipMemcpyDeviceToHost, cs));
		HostCollCall* c = new HostCollCall{hgroup, hg_stage, bytes, type, op};
		HIP_CHECK(hipLaunchHostFunc(cs, [](void* a) {
			HostCollCall* c = (HostCollCall*)a;
			c->g->allreduce_host(c->host, c->bytes, c->type, c->op);
			delete c;
		}, c));
		HIP_CHECK(hipMemcpyAsync(dev, hg_stage, bytes, hipMemcpyHostToDevice, cs));
		if (own) x_join();
	}
	// every rank must run the same exchange (overlapped or grouped): sum of the setting over the ranks is 0 or world
	void verify_uniform_exchange() {
		if (overlap_verified || !coll_on()) return;
		health_buf.alloc(4);
		const uint32_t v[2] = {exchange_overlap ? 1u : 0u, 1u};
		HIP_CHECK(hipMemcpyAsync(health_buf.p + 2, v, 8, hipMemcpyHostToDevice, stream));
		allreduce_u32(health_buf.p + 2, 2);
		uint32_t h[2] = {0, 0};
		HIP_CHECK(hipMemcpyAsync(h, health_buf.p + 2, 8, hipMemcpyDeviceToHost, stream));
		HIP_CHECK(hipStreamSynchronize(stream));
		if (hgroup) hgroup->check();
		if (h[1] != world) throw std::runtime_error("data parallel: the exchange-setting check saw " + std::to_string(h[1]) + " of " + std::to_string(world) + " ranks");
		if (h[0] != 0 && h[0] != world)
			throw std::runtime_error("data parallel: the exchange overlap is on for " + std::to_string(h[0]) + " of " + std::to_string(world) +
			                         " ranks (neus_testbed_set_exchange_overlap / NEUS_EXCHANGE_OVERLAP must be the same on every rank)");
		overlap_verified = true;
	}

	// ------------------------------------------------------------ occupancy grid (testbed_nerf.cu:3293-3397, 4003-4016)
	void occ_update(uint32_t n_uniform, uint32_t n_nonuniform, uint32_t valid, bool use_delta = false) {
		hipStream_t s = stream;
		const uint32_t n_cells = GRID3 * (max_cascade + 1);
		if (training_step == 0) { HIP_CHECK(hipMemsetAsync(density_grid.p, 0, n_cells * 4, s)); density_grid_ema_step = 0; }
		// the first 256 steps' all-cells uniform pass writes every cell exactly once (fused path, one cascade): on a
		// single GPU no clearing is needed; with shards each rank writes only its cells, the rest must read 0
		const bool exclusive = !use_delta && n_nonuniform == 0 && n_uniform == GRID3 && max_cascade == 0;
		if (!exclusive || world > 1) HIP_CHECK(hipMemsetAsync(density_tmp.p, 0, n_cells * 4, s));
		// data parallel: rank r evaluates the global samples [lo, hi) (same density_grid_rng on every rank; in the
		// exclusive pass the cells [lo, hi), i.e. the samples that land there); the max-splatted grids are then
		// max-all-reduced, which equals the single-GPU splat (max is exact)
		const uint32_t NT = n_uniform + n_nonuniform;
		const uint32_t lo = (uint32_t)((uint64_t)NT * rank / world), hi = (uint32_t)((uint64_t)NT * (rank + 1) / world);
		const uint32_t N = hi - lo;
		occ_samples += N; ++occ_updates;
		const pcg32 rng_u = density_grid_rng;
		density_grid_rng.advance();
		const pcg32 rng_nu = density_grid_rng;
		density_grid_rng.advance();
		if (!use_delta) {
			// sample generation + NerfNetwork::density + splat in one kernel
			OccSampling os{};
			os.n_u = n_uniform; os.n_nu = n_nonuniform; os.lo = lo;
			os.rng_u_state = rng_u.state; os.rng_u_inc = rng_u.inc; os.rng_nu_state = rng_nu.state; os.rng_nu_inc = rng_nu.inc;
			os.step = density_grid_ema_step; os.n_cascades = max_cascade + 1; os.thresh_nu = NERF_MIN_OPTICAL_THICKNESS;
			for (int d = 0; d < 3; ++d) { os.amin[d] = ds.aabb_min[d]; os.diag[d] = ds.aabb_max[d] - ds.aabb_min[d]; }
			os.grid_in = density_grid.p; os.grid_tmp = density_tmp.p;
			os.jt = jump_table();
			os.exclusive = exclusive ? 1u : 0u;
			// the uniform part in cell order (spatially coherent gathers; the max splat is order-independent): one cascade
			// of cells or fewer uniform samples, so the uniform hash is a bijection onto the cells
			const uint32_t u_lo = std::min(lo, n_uniform), u_hi = std::min(hi, n_uniform);
			if (!exclusive && occ_sort && u_hi > u_lo && n_uniform <= GRID3) {
				if (!occ_ulist.p) occ_ulist.alloc(GRID3);
				launch_occ_uniform_list(s, n_uniform, density_grid_ema_step, u_lo, u_hi, occ_ulist.p, scan_tmp.p);
				os.ulist = occ_ulist.p; os.n_ulist = u_hi - u_lo;
				// (occ_nu_sort: the occupancy-biased samples binned by their coarse cell as well; in index order the biased half
				// takes 294 of the pass's 479 us, the cell-ordered uniform half 187 - profiles/r06occ_split.txt)
				const uint32_t nu_lo = std::max(lo, n_uniform), n_nu_rank = hi > nu_lo ? hi - nu_lo : 0u;
				if (occ_nu_sort && n_nu_rank) {
					if (occ_nu_key.n < n_nu_rank) { occ_nu_key.alloc(n_nu_rank); occ_nu_list.alloc(n_nu_rank); }
					occ_nu_bins.alloc(2 * 4096 * (size_t)(max_cascade + 1));
					launch_occ_nu_list(s, n_nu_rank, nu_lo - n_uniform, os, occ_nu_key.p, occ_nu_bins.p, occ_nu_list.p, scan_tmp.p, scan_tmp_bytes);
					os.nulist = occ_nu_list.p;
				}
			}
			launch_occ_density(s, lay.L, lay.W, N, os, gl, valid, params_h.p + lay.grid_off, mlp);
		} else {
			launch_grid_samples(s, n_uniform, std::min(lo, n_uniform), std::min(hi, n_uniform), 0, rng_u.state, rng_u.inc, density_grid_ema_step,
			                    ds.aabb_min, ds.aabb_max, density_grid.p, occ_pos.p, occ_idx.p, max_cascade + 1, -0.01f, jump_table());
			launch_grid_samples(s, n_nonuniform, std::max(lo, n_uniform) - n_uniform, std::max(hi, n_uniform) - n_uniform,
			                    std::max(lo, n_uniform) - lo, rng_nu.state, rng_nu.inc, density_grid_ema_step, ds.aabb_min, ds.aabb_max,
			                    density_grid.p, occ_pos.p, occ_idx.p, max_cascade + 1, NERF_MIN_OPTICAL_THICKNESS, jump_table());
			// NerfNetwork::density on the moved positions (the DeltaNetwork is active, nerf_network.h:664-675)
			launch_delta_apply(s, nullptr, N, 3, occ_pos.p, occ_pos.p, delta.p);
			launch_nerf_density(s, lay.L, lay.W, N, occ_pos.p, gl, valid, params_h.p + lay.grid_off, mlp, occ_density.p);
			launch_splat_max(s, N, occ_idx.p, occ_density.p, density_tmp.p);
		}
		allreduce_f32(density_tmp.p, n_cells, true);
		// EMA + mean partials (one launch), final mean, bitfield, mip pools + the march's linear words (one launch)
		launch_ema_mean(s, n_cells, cfg.density_grid_decay, density_grid.p, density_tmp.p, grid_partial.p, grid_mean.p);
		++density_grid_ema_step;
		launch_bitfield(s, density_grid.p, bitfield.p, grid_mean.p, max_cascade + 1, bf_lin.p);
		launch_occ_bbox(s, bitfield.p, occ_bbox.p);
	}

	// ------------------------------------------------------------ optimizer (trainer.h:170-172)
	void optimizer_step(const float* g, const StepCounterArgs* counters = nullptr) {
		const AdamParams p = adam_params();
		const AdamTranspose tr = adam_transpose();  // the transposed / permuted MLP copies are written by the Adam launch itself
		launch_adam_ema(stream, p, params_fp.p, params_h.p, g, m1.p, m2.p, adam_steps.p, steps32, ema_tmp.p, ema_h.p, counters, &tr);
		if (p.skip_ema_h) ema_h_stale = true;
	}
	// The host side of one optimizer step (advances the step count and the learning-rate decay): call once per step
	AdamParams adam_params() {
		// ExponentialDecay (exponential_decay.h:61-80): evaluated with the nested step count before the Adam step
		const uint32_t sb = adam_step;
		if (sb == 0) lr_factor = 1.0f;
		if (sb >= cfg.decay_start && (sb - cfg.decay_start) % cfg.decay_interval == 0 && sb <= 10000000u) lr_factor *= cfg.decay_base;
		++adam_step;
		AdamParams p{};
		p.n = lay.P; p.n_matrix = lay.n_matrix; p.loss_scale = LOSS_SCALE;
		p.lr = (cur_frame ? cfg.after_learning_rate : cfg.learning_rate) * lr_factor;  // testbed.cu:2695-2702
		p.beta1 = cfg.beta1; p.beta2 = cfg.beta2; p.eps = cfg.epsilon; p.l2_reg = cfg.l2_reg;
		p.ema_decay = cfg.ema_decay;
		p.ema_debias_old = 1 - (float)std::pow(cfg.ema_decay, adam_step - 1);
		p.ema_debias_new = 1.0f / (1 - (float)std::pow(cfg.ema_decay, adam_step));
		p.optimize_matrix = 1; p.optimize_non_matrix = 1;
		int e2 = 0;
		p.pow2_scale = std::frexp(p.loss_scale, &e2) == 0.5f ? 1u : 0u;
		p.inv_loss_scale = 1.0f / p.loss_scale;
		ensure_bias_table();
		p.bias_tab = adam_bias.p; p.bias_converged = bias_conv ? 1u : 0u;
		{ static const bool eager = [] { const char* e = std::getenv("NEUS_EAGER_EMA_H"); return e && e[0] == '1'; }(); p.skip_ema_h = eager ? 0u : 1u; }
		p.abort = &st.p->cut_abort;  // (the march cut's witness: a step that is re-run applies nothing)
		return p;
	}
	// Adam in pieces beside the backward (adam_overlap; one rank, static scenes): the MLP blocks once the weight-gradient
	// reduction is done (beside the grid scatter), each grid level group once its accumulation launch is done (beside the
	// next group's), on ad_stream; the step's stream joins it where the one Adam launch used to be. Elementwise, so the
	// parameters are bitwise those of the one launch. Cut points are rounded down to 4 parameters (the kernel's 16-B
	// groups): a range may start with the last few parameters of the level before it, whose gradient is final already.
	bool adam_overlap = [] { const char* e = std::getenv("NEUS_ADAM_OVERLAP"); return e && e[0] == '1'; }();
	// ad_stream is the step's side stream (aux_stream, created with the step's stream at its priority): a stream of its own
	// would be a fifth HIP stream of the process over GPU_MAX_HW_QUEUES = 4 hardware queues and share one - measured
	// 1.12 -> 1.99 ms/step when it landed behind the lookahead's low-priority march (profiles/r06b_adam_overlap_ab.txt)
	hipStream_t ad_stream = nullptr;
	hipEvent_t ad_ev[8] = {}, ad_done = nullptr;
	int ad_n = 0;
	void adam_issue(AdamSplit& a, uint32_t hi, const float* g, bool with_tr) {
		if (!ad_stream) {
			ad_stream = aux_stream;
			for (auto& e : ad_ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
			HIP_CHECK(hipEventCreateWithFlags(&ad_done, hipEventDisableTiming));
		}
		hi = hi >= lay.P ? lay.P : hi / 4 * 4;
		if (hi <= a.next) return;
		hipStream_t on = a.on;
		if (!on) {
			hipEvent_t e = ad_ev[ad_n++ % 8];
			HIP_CHECK(hipEventRecord(e, stream));
			HIP_CHECK(hipStreamWaitEvent(ad_stream, e, 0));
			on = ad_stream;
		}
		const AdamTranspose tr = with_tr ? adam_transpose() : AdamTranspose{};
		launch_adam_ema_range(on, a.p, a.next, hi, params_fp.p, params_h.p, g, m1.p, m2.p, adam_steps.p, steps32, ema_tmp.p, ema_h.p,
		                      with_tr ? &tr : nullptr);
		a.next = hi;
	}
	void adam_join(AdamSplit& a, const float* g) {
		adam_issue(a, lay.P, g, false);  // (whatever is left: the levels past the valid one, the variance)
		if (!a.on) {  // (on the exchange stream the step's x_join has waited for every piece already)
			HIP_CHECK(hipEventRecord(ad_done, ad_stream));
			HIP_CHECK(hipStreamWaitEvent(stream, ad_done, 0));
		}
		if (a.p.skip_ema_h) ema_h_stale = true;
	}
	// bias-correction table for the config's betas (rebuilt only when they change), and the step counts' width for it:
	// u16 while the table is converged, u32 otherwise (moved through the host when the betas change)
	void ensure_bias_table() {
		const float b1 = cfg.beta1, b2 = cfg.beta2;
		if (b1 == bias_b1 && b2 == bias_b2) return;
		adam_bias.alloc(2 * ADAM_BIAS_TAB);
		launch_adam_bias_table(stream, b1, b2, adam_bias.p);
		float last[2];
		HIP_CHECK(hipStreamSynchronize(stream));
		HIP_CHECK(hipMemcpy(&last[0], adam_bias.p + ADAM_BIAS_TAB - 1, 4, hipMemcpyDeviceToHost));
		HIP_CHECK(hipMemcpy(&last[1], adam_bias.p + 2 * ADAM_BIAS_TAB - 1, 4, hipMemcpyDeviceToHost));
		const double k = ADAM_BIAS_TAB - 1;
		bias_conv = last[0] == 1.0f && last[1] == 1.0f && std::pow((double)b1, k) < 0x1p-30 && std::pow((double)b2, k) < 0x1p-30;
		bias_b1 = b1; bias_b2 = b2;
		if (steps32 == bias_conv) {
			std::vector<uint32_t> h(lay.P);
			get_steps(h.data());
			steps32 = !bias_conv;
			put_steps(h.data());
		}
	}
	void get_steps(uint32_t* out) {
		if (steps32) { HIP_CHECK(hipMemcpy(out, adam_steps.p, lay.P * 4, hipMemcpyDeviceToHost)); return; }
		std::vector<uint16_t> h(lay.P);
		HIP_CHECK(hipMemcpy(h.data(), adam_steps.p, lay.P * 2, hipMemcpyDeviceToHost));
		for (size_t i = 0; i < lay.P; ++i) out[i] = h[i];
	}
	void put_steps(const uint32_t* in) {  // in = nullptr: zeros
		if (!in) { HIP_CHECK(hipMemset(adam_steps.p, 0, lay.P * 4)); return; }
		if (steps32) { HIP_CHECK(hipMemcpy(adam_steps.p, in, lay.P * 4, hipMemcpyHostToDevice)); return; }
		std::vector<uint16_t> h(lay.P);
		for (size_t i = 0; i < lay.P; ++i) h[i] = (uint16_t)std::min<uint32_t>(in[i], 0xffffu);
		HIP_CHECK(hipMemcpy(adam_steps.p, h.data(), lay.P * 2, hipMemcpyHostToDevice));
	}
	AdamTranspose adam_transpose() const {
		const Layout& l = lay;
		AdamTranspose t{};
		t.n = 5;
		const uint32_t off[5] = {l.off_d0, l.off_d1, l.off_r0, l.off_r1, l.off_r2}, rows[5] = {l.W, 16, l.W, l.W, 16}, cols[5] = {l.din, l.W, 48, l.W, l.W};
		half_t* dst[5] = {(half_t*)mlp.d0T, (half_t*)mlp.d1T, (half_t*)mlp.r0T, (half_t*)mlp.r1T, (half_t*)mlp.r2T};
		for (int j = 0; j < 5; ++j) { t.off[j] = off[j]; t.rows[j] = rows[j]; t.cols[j] = cols[j]; t.dst[j] = dst[j]; }
		for (int k = 0; k < 48; ++k) t.inv[k] = -1;
		for (uint32_t q = 0; q < din_perm.din && q < 48; ++q) if (din_perm.p[q] >= 0 && din_perm.p[q] < 48) t.inv[din_perm.p[q]] = (int32_t)q;
		t.d0p = (half_t*)mlp.d0p; t.d0Tp = (half_t*)mlp.d0Tp; t.din = din_perm.din; t.W = din_perm.W;
		return t;
	}

	// each phase mark also closes the previous roctx range and opens the phase's (host enqueue spans of the step's kernel
	// groups in `rocprofv3 --marker-trace`; the calls are no-ops without a tool attached)
	int rx_open = -1;
	void mark(int i) {
		static const char* const names[N_PHASES] = {"neus:occupancy", "neus:march", "neus:inference", "neus:loss", "neus:encode",
		                                            "neus:mlp", "neus:wgrad", "neus:scatter", "neus:exchange", "neus:optimizer"};
		if (profiling) HIP_CHECK(hipEventRecord(ev[prof_par][i], stream));
		if (rx_open >= 0) roctxRangePop();
		rx_open = i < N_PHASES ? i : -1;
		if (rx_open >= 0) roctxRangePushA(names[i]);
	}
	// Inference timing (neus_testbed_set_infer_timing): every pre-compaction network launch of the step (the one pass, or
	// each progressive round's k_nerf_infer) records a pair of hipEvents at its kernel's start and end (launched through
	// hipExtLaunchKernelGGL: events recorded between launches also counted the dispatch gap and overlapped the previous
	// kernel's tail, 182 against the kernel trace's 146 us per launch), summed per step after the step (host waits: timing
	// passes only, never the bench's timed region)
	bool infer_timing = false;
	static constexpr int IT_MAX = 16;
	hipEvent_t it_ev[2 * IT_MAX] = {};
	int it_n = 0;
	double it_ms = 0.0;
	uint64_t it_launches = 0, it_steps = 0;
	void it_arm() {
		if (!infer_timing || it_n + 2 > 2 * IT_MAX) return;
		for (int k = 0; k < 2; ++k)
			if (!it_ev[it_n + k]) HIP_CHECK(hipEventCreate(&it_ev[it_n + k]));
		g_infer_ev[0] = it_ev[it_n];
		g_infer_ev[1] = it_ev[it_n + 1];
		it_n += 2;
	}
	void it_collect() {
		if (!infer_timing || it_n < 2) { it_n = 0; return; }
		HIP_CHECK(hipEventSynchronize(it_ev[it_n - 1]));
		for (int i = 0; i + 1 < it_n; i += 2) {
			float ms = 0.f;
			HIP_CHECK(hipEventElapsedTime(&ms, it_ev[i], it_ev[i + 1]));
			it_ms += ms;
			++it_launches;
		}
		++it_steps;
		it_n = 0;
	}

	// Exchange timing (neus_testbed_set_exchange_timing, data parallel): per step, an event on the step's stream where the
	// backward is done (the gradients' last use before the join) and one on the exchange's stream after its last
	// collective. exposed = max(0, done - backward done): what the join before Adam waits for; span = done - the loss's end
	// (the counters' exchange starts there). A ring of event sets collected lazily (the oldest has long completed when the
	// ring wraps, the host running at most 16 steps ahead), so timing runs inside timed regions without a per-step sync.
	bool xt_on = false;
	static constexpr int XT_RING = 64;
	hipEvent_t xt_ev[XT_RING][3] = {};  // [loss end (step stream), backward done (step stream), exchange done (exchange stream)]
	int xt_head = 0, xt_n = 0;
	double xt_exposed_ms = 0.0, xt_span_ms = 0.0;
	uint64_t xt_steps = 0;
	hipEvent_t* xt_slot() {
		if (xt_n == XT_RING) xt_collect_one();
		hipEvent_t* e = xt_ev[(xt_head + xt_n) % XT_RING];
		for (int k = 0; k < 3; ++k)
			if (!e[k]) HIP_CHECK(hipEventCreate(&e[k]));
		++xt_n;
		return e;
	}
	void xt_collect_one() {
		hipEvent_t* e = xt_ev[xt_head];
		HIP_CHECK(hipEventSynchronize(e[2]));
		HIP_CHECK(hipEventSynchronize(e[1]));
		float exposed = 0.f, span = 0.f;
		HIP_CHECK(hipEventElapsedTime(&exposed, e[1], e[2]));
		HIP_CHECK(hipEventElapsedTime(&span, e[0], e[2]));
		xt_exposed_ms += std::max(0.f, exposed);
		xt_span_ms += span;
		++xt_steps;
		xt_head = (xt_head + 1) % XT_RING;
		--xt_n;
	}
	void xt_collect_all() { while (xt_n) xt_collect_one(); }

	// ------------------------------------------------------------ rendering (render_to_cpu, python_api.cu:123-169)
	// NerfTracer::init_rays_from_camera + trace (testbed_nerf.cu:2397-2600) once per spp, accumulated in linear
	// colour. The alive count is read back every iteration (it sets the steps per iteration, as the reference).
	uint32_t render(const NeusRenderRequest& rq, float* host_rgba) {
		if (!have_net) throw std::runtime_error("render: no network (reload_network first)");
		if (rq.width <= 0 || rq.height <= 0) throw std::runtime_error("render: empty resolution");
		const uint64_t n64 = (uint64_t)rq.width * (uint64_t)rq.height;
		if (n64 > (1ull << 26)) throw std::runtime_error("render: at most 2^26 pixels per call");
		const uint32_t n = (uint32_t)n64;
		RenderCamera cam{};
		cam.width = (uint32_t)rq.width; cam.height = (uint32_t)rq.height;
		if (rq.training_view >= 0) {
			if ((uint32_t)rq.training_view >= ds.n_images) throw std::runtime_error("render: training_view out of range");
			const uint32_t v = (uint32_t)rq.training_view;
			std::memcpy(cam.xform, &host_xform[12 * v], 12 * sizeof(float));
			// set_camera_to_training_view: relative focal length = focal / res[fov_axis = 1], rescaled to the render height
			for (int k = 0; k < 2; ++k) {
				cam.focal[k] = host_focal[2 * v + k] / (float)host_res[2 * v + 1] * (float)rq.height;
				cam.screen_center[k] = host_pp[2 * v + k];
			}
		} else {
			std::memcpy(cam.xform, rq.xform, sizeof(cam.xform));
			cam.focal[0] = rq.focal[0]; cam.focal[1] = rq.focal[1];
			cam.screen_center[0] = rq.screen_center[0]; cam.screen_center[1] = rq.screen_center[1];
		}
		hipStream_t s = stream;
		const size_t rb = render_ray_bytes();
		r_rays[0].alloc(n * rb); r_rays[1].alloc(n * rb);
		r_flags.alloc(n); r_base.alloc(n); r_alive.alloc(1);
		r_coords.alloc((size_t)n * MAX_STEPS_INBETWEEN_COMPACTION * COORD_W);
		r_out.alloc((size_t)n * MAX_STEPS_INBETWEEN_COMPACTION * OUT_W);
		r_frame.alloc(n); r_accum.alloc(n);
		const size_t sb = scan_temp_bytes(n);
		if (sb > r_scan_bytes || !r_scan_tmp.p) { r_scan_tmp.alloc(sb + 256); r_scan_bytes = sb; scan_temp_reset(s, r_scan_tmp.p); }
		const MlpPtrs& w = rq.use_ema ? mlp_ema : mlp;
		const half_t* grid = (rq.use_ema ? ema_h.p : params_h.p) + lay.grid_off;
		if (rq.use_ema) { sync_ema_h(); prepare_weights_for(mlp_ema); }
		const uint32_t valid = valid_level_at(enc_step);
		const uint32_t spp = std::max(1u, rq.spp);
		// m_use_delta (prepare_for_test): the network sees the sample positions through the DeltaNetwork
		const bool use_delta = render_delta && cur_frame >= 1;
		if (use_delta) { r_coords_def.alloc((size_t)n * MAX_STEPS_INBETWEEN_COMPACTION * COORD_W); launch_delta_prepare(s, delta.p); }
		uint32_t iters = 0;
		for (uint32_t sp = 0; sp < spp; ++sp) {
			const uint32_t offs_index = rq.snap_to_pixel_centers ? 0 : sp;
			ld_pixel_offset(offs_index, cam.pixel_offset);
			launch_render_init(s, cam, sp, ds, bitfield.p, bf_lin.p, r_rays[0].p, r_frame.p);
			uint32_t n_alive = n, cur = 0;
			iters = 0;
			for (uint32_t i = 1; i < MARCH_ITER;) {
				launch_render_compact(s, n_alive, r_rays[cur].p, r_flags.p, r_base.p, r_rays[cur ^ 1].p, r_alive.p, r_scan_tmp.p, r_scan_bytes);
				cur ^= 1;
				HIP_CHECK(hipMemcpyAsync(pinned + 32, r_alive.p, 4, hipMemcpyDeviceToHost, s));
				HIP_CHECK(hipStreamSynchronize(s));
				std::memcpy(&n_alive, pinned + 32, 4);
				if (n_alive == 0) break;
				const uint32_t n_steps = std::min(MAX_STEPS_INBETWEEN_COMPACTION, std::max(1u, n / n_alive));
				launch_render_gen(s, n_alive, n_steps, ds, bitfield.p, bf_lin.p, r_rays[cur].p, r_coords.p);
				const uint32_t n_el = n_alive * n_steps;
				const float* c_in = r_coords.p;
				if (use_delta) { launch_delta_apply(s, nullptr, n_el, COORD_W, r_coords.p, r_coords_def.p, delta.p); c_in = r_coords_def.p; }
				launch_nerf_infer(s, lay.L, lay.W, nullptr, n_el, c_in, gl, valid, grid, w, r_out.p,
				                  std::max<uint32_t>(1, std::min<uint32_t>((n_el + 127) / 128, 8192)));
				launch_render_composite(s, n_alive, n_steps, r_coords.p, r_out.p, cos_anneal(), rq.min_transmittance, ds.target.mode == 2,
				                        r_rays[cur].p, r_frame.p);
				i += n_steps;
				++iters;
			}
			launch_render_accumulate(s, n, sp, r_frame.p, r_accum.p);
		}
		HIP_CHECK(hipMemcpyAsync(host_rgba, r_accum.p, (size_t)n * 16, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		return iters;
	}

	// ------------------------------------------------------------ marching cubes (testbed_nerf.cu:4096-4226)
	// get_density_on_grid: raw SDF of the inference (EMA) weights at every grid point, written to dst.
	void sdf_on_grid(const uint32_t res[3], const float amin[3], const float amax[3], float* dst) {
		if (!have_net) throw std::runtime_error("sdf_on_grid: no network");
		sync_ema_h(); prepare_weights_for(mlp_ema);
		const uint64_t n = (uint64_t)res[0] * res[1] * res[2];
		const uint32_t valid = valid_level_at(enc_step);
		const bool use_delta = render_delta && cur_frame >= 1;
		if (use_delta) launch_delta_prepare(stream, delta.p);
		for (uint64_t off = 0; off < n; off += (1ull << 30)) {
			const uint32_t cnt = (uint32_t)std::min<uint64_t>(n - off, 1ull << 30);
			launch_sdf_grid(stream, lay.L, lay.W, res, amin, amax, ds.aabb_min, ds.aabb_max, off, cnt, gl, valid, ema_h.p + lay.grid_off, mlp_ema,
			                dst + off, use_delta ? delta.p : nullptr);
		}
	}
	// Testbed::marching_cubes: SDF grid (unless a device density grid is given), then the deterministic
	// count / scan / emit passes of mc.hip. The mesh stays on the device until get_mesh.
	void marching_cubes(const int32_t res_in[3], const float amin[3], const float amax[3], float thresh, const float* density_dev) {
		uint32_t res[3];
		for (int k = 0; k < 3; ++k) {
			if (res_in[k] < 2) throw std::runtime_error("marching_cubes: resolution must be >= 2");
			res[k] = density_dev ? (uint32_t)res_in[k] : next_multiple((uint32_t)res_in[k], 16u);  // testbed_nerf.cu:4176-4178
		}
		const uint64_t n = (uint64_t)res[0] * res[1] * res[2];
		if (n >= (1ull << 36)) throw std::runtime_error("marching_cubes: grid too large");
		hipStream_t s = stream;
		const float* d = density_dev;
		if (!d) {
			mc_density.alloc(n);
			sdf_on_grid(res, amin, amax, mc_density.p);
			d = mc_density.p;
		}
		const uint32_t nc = mc_n_chunks(res);
		mc_cnt.alloc(4 * (size_t)nc + 4);
		uint32_t *cv = mc_cnt.p, *ct = cv + nc, *ov = ct + nc, *ot = ov + nc;
		launch_mc_count(s, res, amin, amax, thresh, d, cv, ct);
		const size_t sb = scan_temp_bytes(nc);
		if (sb > mc_scan_bytes || !mc_scan_tmp.p) { mc_scan_tmp.alloc(sb + 256); mc_scan_bytes = sb; scan_temp_reset(s, mc_scan_tmp.p); }
		launch_exclusive_scan(s, mc_scan_tmp.p, mc_scan_bytes, cv, ov, nc);
		launch_exclusive_scan(s, mc_scan_tmp.p, mc_scan_bytes, ct, ot, nc);
		uint32_t last[4];
		HIP_CHECK(hipMemcpyAsync(pinned + 40, cv + nc - 1, 4, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipMemcpyAsync(pinned + 41, ct + nc - 1, 4, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipMemcpyAsync(pinned + 42, ov + nc - 1, 4, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipMemcpyAsync(pinned + 43, ot + nc - 1, 4, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		std::memcpy(last, pinned + 40, 16);
		const uint64_t nv = (uint64_t)last[2] + last[0], nt = (uint64_t)last[3] + last[1];
		if (nv >= (1ull << 32) || 3 * nt >= (1ull << 32)) throw std::runtime_error("marching_cubes: mesh exceeds 32-bit indices");
		mesh_v.alloc(3 * std::max<uint64_t>(nv, 1));
		mc_vidx.alloc(n);
		mesh_f.alloc(3 * std::max<uint64_t>(nt, 1));
		launch_mc_emit(s, res, amin, amax, thresh, d, ov, ot, mesh_v.p, mc_vidx.p, mesh_f.p);
		if (!density_dev) launch_mesh_unmove(s, (uint32_t)nv, ds.motion, mesh_v.p);  // transform_mesh_with_6d
		HIP_CHECK(hipStreamSynchronize(s));
		mesh_nv = (uint32_t)nv; mesh_nt = (uint32_t)nt;
	}

	// compute_mesh_vertex_colors (testbed_nerf.cu:4071-4094): network colour (inference weights) at each vertex,
	// looking outward from the aabb centre; sRGB (the network is trained on sRGB targets).
	void mesh_colors(float* host_rgb) {
		if (!mesh_nv) return;
		sync_ema_h(); prepare_weights_for(mlp_ema);
		Dev<float> c; Dev<half_t> o;
		c.alloc((size_t)mesh_nv * COORD_W); o.alloc((size_t)mesh_nv * OUT_W);
		launch_mesh_coords(stream, mesh_nv, mesh_v.p, ds, c.p);
		if (render_delta && cur_frame >= 1) {  // m_use_delta: the vertices go through the DeltaNetwork too
			launch_delta_prepare(stream, delta.p);
			launch_delta_apply(stream, nullptr, mesh_nv, COORD_W, c.p, c.p, delta.p);
		}
		launch_nerf_infer(stream, lay.L, lay.W, nullptr, mesh_nv, c.p, gl, valid_level_at(enc_step), ema_h.p + lay.grid_off, mlp_ema, o.p,
		                  std::max<uint32_t>(1, std::min<uint32_t>((mesh_nv + 127) / 128, 8192)));
		std::vector<half_t> h((size_t)mesh_nv * OUT_W);
		HIP_CHECK(hipMemcpyAsync(h.data(), o.p, h.size() * sizeof(half_t), hipMemcpyDeviceToHost, stream));
		HIP_CHECK(hipStreamSynchronize(stream));
		for (size_t i = 0; i < mesh_nv; ++i)
			for (int k = 0; k < 3; ++k) host_rgb[3 * i + k] = 1.0f / (1.0f + std::exp(-(float)h[i * OUT_W + k]));
	}

	// ------------------------------------------------------------ one Testbed::train step (testbed.cu:2640-2736)
	void train_step() {
		if (abort_pending) check_abort();
		train_step_body();
	}
	// The last issued step's march-cut witness (march_cut_on): when it aborted, its state changes were withheld on the
	// device; the host state goes back to its start and the step runs again with the full march.
	void check_abort() {
		abort_pending = false;
		uint32_t a = 0;
		if (abort_direct) {
			// one rank: k_loss_grad stored the word to host-coherent memory (sentinel ~0 before the step): poll it, and
			// after a bounded spin wait for the step's stream (the kernel has then run)
			const volatile uint32_t* w = abort_word;
			for (uint32_t k = 0; k < (1u << 22) && *w == ~0u; ++k) __builtin_ia32_pause();
			if (*w == ~0u) HIP_CHECK(hipStreamSynchronize(stream));
			a = *w;
			if (a == ~0u) throw std::runtime_error("march cut: the witness word was not written");
		} else {
			HIP_CHECK(hipEventSynchronize(ev_abort));
			std::memcpy(&a, pinned + 100, 4);
		}
		if (!a) return;
		// this testbed's streams drained (not the device's: another rank of an in-process group may share it)
		for (hipStream_t q : {stream, aux_stream, la_stream, comm_stream})
			if (q) HIP_CHECK(hipStreamSynchronize(q));
		la_pending = false;
		la_deferred = nullptr;
		const uint32_t left = call_left;
		const StepSnap s0 = snap[0], s1 = snap[1];
		const bool prev_mc = mc_hist[1];
		training_step = s0.training_step; canonical_step = s0.canonical_step; adam_step = s0.adam_step; call_left = s0.call_left;
		enc_step = s0.enc_step; lr_factor = s0.lr_factor; rng = s0.rng;
		la_steps = s0.la_steps; cut_steps = s0.cut_steps; adam_split_steps = s0.adam_split_steps; mcut_steps = s0.mcut_steps;
		StepState h{};
		HIP_CHECK(hipMemcpy(&h, st.p, sizeof(h), hipMemcpyDeviceToHost));
		if (prev_mc) {
			// the step before was cut too: its requested count in full (its rays again, from its rng and its n_rays_total), so
			// that this step's cap is the reference's exactly (the bitfield is the one it marched: no occupancy update since)
			StepState t = h;
			t.n_rays_total = h.n_rays_total - h.rays_per_batch * world;
			st_recount.alloc(1);
			HIP_CHECK(hipMemcpy(st_recount.p, &t, sizeof(t), hipMemcpyHostToDevice));
			launch_march_count(stream, MAX_RAYS, max_samples, st_recount.p, DPInfo{rank, world}, ds, bitfield.p, bf_lin.p, s1.rng.state, s1.rng.inc,
			                   rays.p, startt.p, nreq.p, mwork, nullptr, 0, ray_cull ? occ_bbox.p : nullptr);
			launch_march_write(stream, MAX_RAYS, st_recount.p, ds, rays.p, mwork, nreq.p, base.p, numsteps.p, coords.p, nullptr, max_samples,
			                   scan_tmp.p, nullptr, 0);
			HIP_CHECK(hipStreamSynchronize(stream));
			HIP_CHECK(hipMemcpy(&t, st_recount.p, sizeof(t), hipMemcpyDeviceToHost));
			const uint32_t before = t.numsteps_counter;
			h.measured_before = before;
			h.max_inference = (std::min(before, max_samples) + 127u) / 128u * 128u;
		}
		h.mi_lb = 0;
		h.cut_abort = 0;
		HIP_CHECK(hipMemcpy(st.p, &h, sizeof(h), hipMemcpyHostToDevice));
		HIP_CHECK(hipMemset(cutw.p + CW_ABORT, 0, 2 * sizeof(uint32_t)));
		snap[0] = s1;
		mc_hist[0] = prev_mc;
		++mcut_reruns;
		force_full = true;
		try { train_step_body(); } catch (...) { force_full = false; throw; }
		force_full = false;
		call_left = left;
	}
	void train_step_body() {
		if (!have_net) throw std::runtime_error("train: no network (reload_network first)");
		hipStream_t s = stream;
		snap[1] = snap[0];
		snap[0] = StepSnap{training_step, canonical_step, adam_step, call_left, enc_step, lr_factor, rng, la_steps, cut_steps, adam_split_steps, mcut_steps};
		mc_hist[1] = mc_hist[0];
		mc_hist[0] = false;
		if (hgroup) hgroup->check();
		verify_uniform_exchange();
		// the readback of 16 steps back (long done on the device) is checked at this step boundary, before anything of
		// this step is queued: a health failure (all-reduced, so every rank sees it) stops every rank on the same step
		// with no collective half-issued and no step half-applied; the host stays at most 16 steps ahead of the device
		if (training_step % 16 == 0 && loss_pending) consume_loss();
		// dynamic scenes (testbed.cu:2651-2712): progressive levels count from the end of the global-movement
		// phase; at its end canonical training starts (and the movement keeps training when finetuned)
		const bool dyn = cur_frame >= 1;
		if (dyn && training_step == gm_steps()) {
			train_canonical = true;
			if (!cfg.finetune_global_movement) train_delta = false;
			if (cfg.reset_density_grid_after_global_movement) {
				HIP_CHECK(hipMemsetAsync(density_grid.p, 0, density_grid.n * 4, s));
				density_grid_ema_step = 0;
			}
		}
		const bool use_delta = dyn && train_delta;
		const bool la_have = la_pending;
		la_pending = false;
		render_delta = use_delta;  // m_nerf_network->m_use_delta follows the training step (testbed.cu:2704-2710)
		enc_step = dyn ? (int)training_step - (int)gm_steps() : (int)training_step;
		const uint32_t valid = valid_level_at(enc_step);
		if (use_delta) launch_delta_prepare(s, delta.p);
		const uint32_t n_prep = std::min(16u, std::max(1u, canonical_step / 16u));
		mark(0);
		if (canonical_step % n_prep == 0) {
			const uint32_t nc = GRID3 * (max_cascade + 1);
			if (training_step < 256) occ_update(nc, 0, valid, use_delta);
			else occ_update(nc / 4, nc / 4, valid, use_delta);
		}
		// ---- train_nerf_step (testbed_nerf.cu:3723-4001)
		if (training_step == 0 || canonical_step == 0) HIP_CHECK(hipMemsetAsync(&st.p->n_rays_total, 0, 4, s));
		const DPInfo dp{rank, world};  // (n_kept, n_rays_with_samples: zeroed by k_ray_gen)
		mark(1);
		// progressive (cut-off-aware) inference this step: its round-0 list is written by the march
		const bool progressive = progressive_mode == 2 || (progressive_mode == 1 && last_keep_ratio < PROGRESSIVE_RATIO);
		const bool sorted_rays = progressive && ray_sort;  // round 0's list by k_ray_sort_place instead of the march write
		const RaySort rsort{rs_hist.p, rs_off.p, rs_key.p, rs_perm.p, chunk_cnt.p + RS_N_PERM};
		if (la_have) {
			if (canonical_step % n_prep == 0) throw std::runtime_error("train: lookahead issued before an occupancy update");
			++la_steps;
			if (la_stat && la_stat_used % 4 == 2) HIP_CHECK(hipEventRecord(la_stat_next(), s));
			HIP_CHECK(hipStreamWaitEvent(s, ev_la_done, 0));  // this step's samples came from the previous step's lookahead
			if (la_stat && la_stat_used % 4 == 3) HIP_CHECK(hipEventRecord(la_stat_next(), s));
		}
		const bool cut = la_have ? la_cut : cut_for(training_step, progressive, call_left == 0, dyn);
		const std::vector<uint32_t>& ce = ends_for(cut);  // (a cut step's rounds: chunk_ends_cut)
		const uint32_t nch = (uint32_t)ce.size() + 1;
		const bool mcut = la_have ? la_mcut : march_cut_for(training_step, cut && sorted_rays, call_left);
		if (!la_have) issue_march(s, dp, rng, progressive, scan_tmp.p, cut, mcut);
		mc_hist[0] = mcut;
		// (this step's witness can fail: the host waits for its word; a re-run step is exact by construction - not cut, and
		// the step before it recounted when that one was cut)
		const bool risky = (mc_hist[0] || mc_hist[1]) && !force_full;
		const bool split = cut && sorted_rays;
		if (cut) ++cut_steps;
		if (mcut) ++mcut_steps;
		mark(2);
		// DeltaNetwork forward on the samples (nerf_network.h:162-182); the loss keeps the undeformed records
		const float* c_in = coords.p;
		if (use_delta) { launch_delta_apply(s, &st.p->n_kept, max_samples, COORD_W, coords.p, coords_def.p, delta.p); c_in = coords_def.p; }
		LossParams lp{};
		lp.loss_scale = LOSS_SCALE; lp.ek_w = cfg.ek_loss_weight; lp.mask_w = cfg.mask_loss_weight; lp.cos_anneal = cos_anneal();
		lp.max_compacted = batch; lp.rng_state = rng.state; lp.rng_inc = rng.inc; lp.jt = jump_table();
		lp.abort_w = cutw.p + CW_ABORT; lp.abort_slot = training_step & 1u;
		if (risky && !coll_on()) {
			// one rank: the word goes straight from k_loss_grad to host memory (no copy, no event on the step's streams)
			if (!abort_word) {
				void* p = nullptr;
				HIP_CHECK(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
				abort_word = (volatile uint32_t*)p;
			}
			*abort_word = ~0u;
			lp.abort_host = (uint32_t*)abort_word;
		}
		{ static const bool f = [] { const char* e = std::getenv("NEUS_DBG_LOSS_FENCE"); return e && e[0] == '1'; }(); lp.dbg_fence = f ? 1u : 0u; }
		const LossWork w = loss_work(base.p);
		if (progressive) {
			// rounds of per-ray chunks, each: network on the round's samples, alpha, the recurrence continued (march.hip);
			// the "infer" phase mark then covers the composite as well
			uint32_t e0 = 0;
			// the compaction cut (prog_cut, cut_for): fixed rays per batch, not a step the host reads back (the loss readback
			// steps, the last step of a train call), one rank's own batch
			for (uint32_t k = 0; k < nch; ++k) {
				const uint32_t e1 = k + 1 < nch ? ce[k] : 0xffffffffu;
				const uint32_t e2 = k + 2 < nch ? ce[k + 1] : 0xffffffffu;
				// the loss's alpha terms in the inference epilogue (k_loss_alpha's work on the round's samples)
				const InferAlpha ia{w.sa, w.ekt, lp.cos_anneal, ds.cone_angle == 0.0f ? 1u : 0u, nullptr, sorted_rays ? 8u : 0u};
				it_arm();
				launch_nerf_infer(s, lay.L, lay.W, chunk_cnt.p + k, 0, c_in, gl, valid, params_h.p + lay.grid_off, mlp, net_out.p, 8192, chunk_list.p,
				                  use_delta ? nullptr : &ia);
				if (use_delta) launch_loss_alpha_list(s, max_samples, chunk_cnt.p + k, chunk_list.p, coords.p, net_out.p, lp.cos_anneal, w, ds.cone_angle == 0.0f);
				const bool more = k + 1 < nch;
				// the cut after round 0 (the rays of the later rounds are then all at or before it: each round continues
				// only the rays of the round before it)
				const bool cut_k = cut && k == 0 && more;
				launch_loss_scan_chunk(s, MAX_RAYS, numsteps.p, w, ccount.p, e0, e1, e2, more && !cut_k ? chunk_list.p : nullptr, chunk_cnt.p + k + 1,
				                       k ? open_rays[(k - 1) & 1].p : (sorted_rays ? rs_perm.p : nullptr),
				                       k ? chunk_cnt.p + OPEN_CNT + k - 1 : (sorted_rays ? rsort.n_perm : nullptr),
				                       more ? (cut_k ? open_raw.p : open_rays[k & 1].p) : nullptr,
				                       more ? chunk_cnt.p + (cut_k ? RAW_CNT : OPEN_CNT) + k : nullptr);
				if (cut_k) {
					// the cut after this round (cbase as the scan's scratch: the compaction rewrites it after the rounds), then
					// the next round's rays and samples from the open rays at or before it
					// a cut march's step: pass B (the slots past the estimate) was not marched, so it is skipped; pass A's
					// slots must reach the batch, or the step is re-run (the witness word, set by the cut below)
					const bool split_b = split && !mcut;
					if (split_b) {
						// pass A was the rays below the estimate: its cut, then pass B (empty when the cut lies in pass A's slots)
						launch_scan_prog_cut(s, scan_tmp.p, ccount.p, cbase.p, MAX_RAYS, batch, cutw.p, 0, nullptr);
						const InferAlpha iab{w.sa, w.ekt, lp.cos_anneal, ds.cone_angle == 0.0f ? 1u : 0u, nullptr, 8u};
						it_arm();
						launch_nerf_infer(s, lay.L, lay.W, cutw.p + CW_LENB_EFF, 0, c_in, gl, valid, params_h.p + lay.grid_off, mlp, net_out.p, 8192,
						                  chunk_list.p + max_samples, &iab);
						launch_loss_scan_chunk(s, MAX_RAYS, numsteps.p, w, ccount.p, 0, e1, e2, nullptr, nullptr, rs_perm.p + MAX_RAYS,
						                       cutw.p + CW_NB_EFF, open_raw.p, chunk_cnt.p + RAW_CNT + k);
					}
					launch_scan_prog_cut(s, scan_tmp.p, ccount.p, cbase.p, MAX_RAYS, batch, cutw.p, 1, split_b ? chunk_cnt.p : nullptr,
					                     mcut ? cutw.p + CW_ABORT + (training_step & 1u) : nullptr);
					launch_prog_next(s, MAX_RAYS, open_raw.p, chunk_cnt.p + RAW_CNT + k, numsteps.p, cutw.p + CW_CUT, e1, e2, chunk_list.p,
					                 chunk_cnt.p + k + 1, open_rays[k & 1].p, chunk_cnt.p + OPEN_CNT + k);
				}
				e0 = e1;
			}
			mark(3);
		} else {
			const InferAlpha ia{w.sa, w.ekt, lp.cos_anneal, ds.cone_angle == 0.0f ? 1u : 0u, w.n_long};
			it_arm();
			launch_nerf_infer(s, lay.L, lay.W, &st.p->n_kept, 0, c_in, gl, valid, params_h.p + lay.grid_off, mlp, net_out.p, 8192, nullptr,
			                  use_delta ? nullptr : &ia);
			mark(3);
			if (use_delta) launch_loss_alpha(s, max_samples, st.p, coords.p, net_out.p, lp.cos_anneal, w, ds.cone_angle == 0.0f);
			launch_loss_scan_ray(s, MAX_RAYS, numsteps.p, w, ccount.p);
		}
		launch_exclusive_scan(s, scan_tmp.p, scan_tmp_bytes, ccount.p, cbase.p, MAX_RAYS);
		launch_loss_ray(s, MAX_RAYS, st.p, dp, ds, lp, numsteps.p, ccount.p, cbase.p, w, loss.p, ek.p, mask.p);
		launch_loss_grad(s, max_samples, st.p, dp, lp, coords.p, net_out.p, numsteps.p, w, coords_c.p, dL_dout.p);
		if (dbg_loss_replay) {  // development (NEUS_DBG_LOSS_REPLAY=1): the same launch again, into separate outputs, and
			                     // copies of the loss-gradient kernel's inputs as they were right after it
			dbg_co.alloc((size_t)batch * COORD_W); dbg_dl.alloc((size_t)batch * OUT_W);
			launch_loss_grad(s, max_samples, st.p, dp, lp, coords.p, net_out.p, numsteps.p, w, dbg_co.p, dbg_dl.p);
			const std::pair<const void*, size_t> src[DBG_SNAP_N] = {
				{l_sa.p, l_sa.n * 16}, {l_ekt.p, l_ekt.n * 4}, {l_ck4.p, l_ck4.n * 16}, {l_cke.p, l_cke.n * 4}, {l_racc.p, l_racc.n * 16},
				{l_rgr.p, l_rgr.n * 16}, {l_rT.p, l_rT.n * 4}, {l_rek.p, l_rek.n * 4}, {ccount.p, ccount.n * 4}, {net_out.p, net_out.n * 2},
				{coords.p, coords.n * 4}, {base.p, base.n * 4}, {numsteps.p, numsteps.n * 4}, {cmap.p, cmap.n * 4}, {nreq.p, nreq.n * 4}};
			for (int k = 0; k < DBG_SNAP_N; ++k) {
				dbg_snap[k].alloc(src[k].second);
				HIP_CHECK(hipMemcpyAsync(dbg_snap[k].p, src[k].first, src[k].second, hipMemcpyDeviceToDevice, s));
			}
		}
		// ---- the step's counters over the ranks (data parallel): the compacted count and the rays with samples, summed
		// right after the loss into StepState::compacted_global / rays_ws_global (compacted_counter stays this rank's
		// training batch for the backward). On the communication stream with the overlapped exchange, so the backward
		// does not wait for it; the gradients' collectives follow on the same stream, in the same order on every rank.
		const bool xo = coll_on() && exchange_overlap && (!dyn || train_canonical);
		coll_bytes_step = 0;
		hipStream_t cs = s;  // the stream the counters (and the lookahead's start) are ordered on
		hipEvent_t* xt = coll_on() && xt_on ? xt_slot() : nullptr;
		if (xt) HIP_CHECK(hipEventRecord(xt[0], s));
		if (coll_on()) {
			cs = xo ? x_stream() : stream;
			coll_begin();
			allreduce_u32(&st.p->compacted_global, 3, cs);  // (+ cut_abort: every rank re-runs the step, or none)
			coll_end();
		}
		if (risky) {
			abort_pending = true;
			abort_direct = !coll_on();
		}
		// ---- lookahead: the next step's ray sampling beside this step's backward (la_on; see the members)
		const bool get_loss = training_step % 16 == 0;
		const StepCounterArgs sca{st.p, batch, max_samples, world, cfg.fixed_rays_per_batch, progressive ? chunk_cnt.p : nullptr, nch};
		bool counters_done = false;
		const uint32_t cs1 = training_step + 1;  // the next step's canonical step (static scenes)
		const uint32_t n_prep1 = std::min(16u, std::max(1u, cs1 / 16u));
		const bool la_go = la_on && la_next_in_call && !dyn && !use_delta && !profiling && !dbg_loss_replay &&
		                   !dbg_lds_fill && g_dbg_lds_fill == 0 && g_dbg_xcd_shift == 0 && cs1 % 16 != 0 && cs1 % n_prep1 != 0 &&
		                   !(get_loss && loss_pending);
		// with a group, the all-reduced word goes to the host from the step counters' launch that the lookahead puts right
		// behind the exchange (a system-scope store, as k_loss_grad's at one rank); otherwise by a copy and an event
		uint32_t* abort_host_ctr = nullptr;
		if (risky && coll_on() && la_go) {
			if (!abort_word) {
				void* p = nullptr;
				HIP_CHECK(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
				abort_word = (volatile uint32_t*)p;
			}
			*abort_word = ~0u;
			abort_host_ctr = (uint32_t*)abort_word;
			abort_direct = true;
		}
		if (risky && !abort_direct) {
			// the all-reduced abort word to the host, off the step's stream (the backward starts at once)
			if (!ev_abort) {
				HIP_CHECK(hipEventCreateWithFlags(&ev_abort, hipEventDisableTiming));
				HIP_CHECK(hipEventCreateWithFlags(&ev_abort_src, hipEventDisableTiming));
			}
			HIP_CHECK(hipEventRecord(ev_abort_src, cs));
			HIP_CHECK(hipStreamWaitEvent(aux_stream, ev_abort_src, 0));
			*(volatile uint32_t*)(pinned + 100) = ~0u;
			HIP_CHECK(hipMemcpyAsync(pinned + 100, &st.p->cut_abort, 4, hipMemcpyDeviceToHost, aux_stream));
			HIP_CHECK(hipEventRecord(ev_abort, aux_stream));
			abort_pending = true;
		}
		{
			if (la_go) {
				// the host's StepState readback first (its place in the step without the lookahead: nothing it reads is
				// written between here and there - the ranks' counts are already summed), then the step counters the next
				// step's sampling reads; both behind the counters' exchange (cs)
				if (get_loss) HIP_CHECK(hipMemcpyAsync(pinned + 64, st.p, sizeof(StepState), hipMemcpyDeviceToHost, cs));
				launch_step_counters(cs, st.p, batch, max_samples, world, cfg.fixed_rays_per_batch, sca.eval_cnt, sca.n_eval, abort_host_ctr);
				counters_done = true;
				if (!la_stream) {
					// the lookahead stream at the lowest priority: the backward's workgroups are dispatched first and the march's
					// fill what they leave (1.154 -> 1.107 ms/step at the bench state; the default priority 1.139, the highest
					// 1.141: profiles/r05lap_lookahead_priority_ab.txt). NEUS_LA_PRIO: -1 lowest, 0 default, 1 highest.
					const char* e = std::getenv("NEUS_LA_PRIO");
					const int want = e ? std::atoi(e) : -1;
					int lo = 0, hi = 0;
					HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));  // (lo: least urgent, hi: most urgent; hi <= lo numerically)
					if (want == 0) HIP_CHECK(hipStreamCreateWithFlags(&la_stream, hipStreamNonBlocking));
					else HIP_CHECK(hipStreamCreateWithPriority(&la_stream, hipStreamNonBlocking, want > 0 ? hi : lo));
					// (device-side hand-offs between the step's and the lookahead's kernels: no system-scope fence - its
					// L2 write-back held the step's stream ~6 us at the record; NEUS_EV_SYSFENCE=1 keeps it, for A/B)
					const char* f = std::getenv("NEUS_EV_SYSFENCE");
					const unsigned fl = hipEventDisableTiming | (f && f[0] == '1' ? 0u : hipEventDisableSystemFence);
					HIP_CHECK(hipEventCreateWithFlags(&ev_la_start, fl));
					HIP_CHECK(hipEventCreateWithFlags(&ev_la_done, fl));
				}
				if (!scan_tmp_la.p || scan_tmp_la.n < scan_tmp_bytes + 256) {
					scan_tmp_la.alloc(scan_tmp_bytes + 256);
					scan_temp_reset(s, scan_tmp_la.p);
				}
				pcg32 r1 = rng;
				r1.advance();
				const bool prog1 = progressive_mode == 2 || (progressive_mode == 1 && last_keep_ratio < PROGRESSIVE_RATIO);
				la_cut = cut_for(training_step + 1, prog1, call_left <= 1, false);
				la_mcut = march_cut_for(training_step + 1, la_cut && ray_sort, call_left - 1);
				const bool cut1 = la_cut, mcut1 = la_mcut;
				la_at = mcut1 ? la_at_cut : la_at_full;
				la_deferred = [this, cs, dp, r1, prog1, cut1, mcut1] {
					HIP_CHECK(hipEventRecord(ev_la_start, cs));
					HIP_CHECK(hipStreamWaitEvent(la_stream, ev_la_start, 0));
					if (la_stat) { la_stat_used -= la_stat_used % 4; HIP_CHECK(hipEventRecord(la_stat_next(), la_stream)); }
					issue_march(la_stream, dp, r1, prog1, scan_tmp_la.p, cut1, mcut1);
					if (la_stat) HIP_CHECK(hipEventRecord(la_stat_next(), la_stream));
					HIP_CHECK(hipEventRecord(ev_la_done, la_stream));
				};
				if (cs != s) la_fire(0x7fffffff);  // (the communication stream: issued now, before the gradients' collectives queue there)
				la_fire(0);
				la_pending = true;
			}
		}
		// the rollover copies are made by the training encode (static scenes); the DeltaNetwork reads the whole batch first
		if (use_delta) launch_rollover(s, batch, st.p, coords_c.p, dL_dout.p);
		const EncodeRollover ro{&st.p->compacted_counter, batch, dL_dout.p, coords_c.p};
		// the canonical backward writes every gradient entry (weight tiles and variance by k_wgrad_reduce, every grid
		// entry by k_scatter_accum, zeros with no samples); the global-movement phase skips it: zero the buffer there
		if (!(!dyn || train_canonical)) HIP_CHECK(hipMemsetAsync(grads.p, 0, (size_t)lay.P * 4, s));
		mark(4);
		// the overlapped exchange (xo): the canonical backward all-reduces its gradient ranges as they finish; adam_overlap
		// (one rank, static scenes): the optimizer step in pieces beside the scatter
		AdamSplit asp{};
		const bool a_over = adam_overlap && !dyn && (!coll_on() || xo);
		if (a_over) asp.p = adam_params();
		if (use_delta) {
			// the training forward runs on the deformed batch; dL/d(position) feeds the DeltaNetwork backward
			launch_delta_apply(s, nullptr, batch, COORD_W, coords_c.p, coords_cdef.p, delta.p);
			tbuf.dpos = dpos.p;
			net_backward(&st.p->compacted_counter, &st.p->n_train, batch, coords_cdef.p, valid, dL_dout.p, grads.p, s, true, train_canonical, nullptr, xo);
			tbuf.dpos = nullptr;
		} else {
			net_backward(&st.p->compacted_counter, &st.p->n_train, batch, coords_c.p, valid, dL_dout.p, grads.p, s, true, train_canonical, &ro, xo,
			             a_over ? &asp : nullptr);
		}
		la_fire(99);  // (issued by now in any case)
		// DeltaNetwork gradient partial sums (the first half of its backward; the Adam step follows the exchange)
		if (use_delta) launch_delta_grad(s, &st.p->n_train, batch, coords_c.p, COORD_W, dpos.p, delta.p, delta_partial.p);
		mark(8);
		if (get_loss) {
			launch_sum_f32(s, scan_tmp.p, scan_tmp_bytes, loss.p, loss_sum.p + 0, MAX_RAYS);
			launch_sum_f32(s, scan_tmp.p, scan_tmp_bytes, ek.p, loss_sum.p + 1, MAX_RAYS);
			launch_sum_f32(s, scan_tmp.p, scan_tmp_bytes, mask.p, loss_sum.p + 2, MAX_RAYS);
			// this rank's health words, summed over the ranks with the loss sums (any rank's failure stops all of them)
			HIP_CHECK(hipMemcpyAsync(health_buf.p, &st.p->fail_flags, 4, hipMemcpyDeviceToDevice, s));
			HIP_CHECK(hipMemcpyAsync(health_buf.p + 1, scan_tmp.p + offsetof(ScanState, fail), 4, hipMemcpyDeviceToDevice, s));
		}
		if (coll_on()) {
			// collective 1 (gradients; DeltaNetwork partials) and 3 (counters, loss scalars) of SURVEY §8(e). The gradient
			// of the grid levels past the progressive valid level is zero on every rank: the scatter writes no records there
			// and keeps that range zeroed (scatter_work_for's sc_zero_from / sc_zero_from_e invariant: every grid entry from
			// gl.offset[valid + 1] on holds 0 after the backward, on every rank), so only the MLP blocks, the active levels'
			// tables and the variance move. Overlapped: the gradients went out during the backward (net_backward).
			const size_t grid_act = 2 * (size_t)gl.offset[std::min(valid + 1, gl.n_levels)];
			if (xt) HIP_CHECK(hipEventRecord(xt[1], s));  // the backward is done (and the loss sums, when logged)
			hipStream_t xs = xo ? x_stream() : stream;
			coll_begin();
			if (!xo) {
				allreduce_f32(grads.p, (size_t)lay.grid_off + grid_act);
				allreduce_f32(grads.p + lay.var_off, lay.P - lay.var_off);
			}
			if (use_delta) allreduce_f32(delta_partial.p, delta_partial_floats(), false, xs);
			if (get_loss) { allreduce_f32(loss_sum.p, 3, false, xs); allreduce_u32(health_buf.p, 2, xs); }
			coll_end();
			if (a_over) adam_issue(asp, lay.P, grads.p, false);  // the optimizer's last piece, behind the exchange
			if (xt) HIP_CHECK(hipEventRecord(xt[2], xs));
			x_join();
		}
		if (get_loss) {
			if (loss_pending) consume_loss();  // (consumed at this step's start already; a restored state may leave one)
			HIP_CHECK(hipMemcpyAsync(pinned, loss_sum.p, 3 * 4, hipMemcpyDeviceToHost, s));
			HIP_CHECK(hipMemcpyAsync(pinned + 52, health_buf.p, 8, hipMemcpyDeviceToHost, s));
			if (!counters_done) HIP_CHECK(hipMemcpyAsync(pinned + 64, st.p, sizeof(StepState), hipMemcpyDeviceToHost, s));
			HIP_CHECK(hipMemcpyAsync(pinned + 48, scan_tmp.p + offsetof(ScanState, fail), 4, hipMemcpyDeviceToHost, s));
			HIP_CHECK(hipEventRecord(ev_loss, s));
			loss_pending = true;
		}
		// the step-end counters ride on the Adam launch when the canonical optimizer steps (k_step_counters otherwise)
		// (progressive inference: the samples evaluated are the rounds' list lengths chunk_cnt[0, nch))
		const bool canon_opt = !dyn || train_canonical;
		if (!canon_opt && !counters_done) launch_step_counters(s, st.p, batch, max_samples, world, cfg.fixed_rays_per_batch, sca.eval_cnt, sca.n_eval);
		rng.advance();
		mark(9);
		// ---- optimizers (testbed_nerf.cu:3503-3508): the canonical trainer, the global-move trainer
		if (canon_opt && a_over) {
			++adam_split_steps;
			if (!counters_done) launch_step_counters(s, st.p, batch, max_samples, world, cfg.fixed_rays_per_batch, sca.eval_cnt, sca.n_eval);
			adam_join(asp, grads.p);
		} else if (canon_opt) {
			optimizer_step(grads.p, counters_done ? nullptr : &sca);
		}
		if (use_delta) {
			// ExponentialDecay of the globalmove optimizer (exponential_decay.h:61-80), its own step count
			if (delta_step == 0) delta_lr_factor = 1.f;
			if (delta_step >= cfg.gm_decay_start && (delta_step - cfg.gm_decay_start) % std::max(1u, cfg.gm_decay_interval) == 0)
				delta_lr_factor *= cfg.gm_decay_base;
			++delta_step;
			DeltaAdam a{cfg.gm_learning_rate * delta_lr_factor, cfg.gm_beta1, cfg.gm_beta2, cfg.gm_epsilon, LOSS_SCALE, 1u};
			launch_delta_step(s, delta_partial.p, delta.p, a);
		}
		mark(10);
		++training_step;
		// m_canonical_training_step (testbed_nerf.cu:3512-3527)
		if (!cfg.predict_global_movement || cur_frame == 0) canonical_step = training_step;
		else if (training_step >= gm_steps()) canonical_step = training_step - gm_steps();
		if (profiling) {
			HIP_CHECK(hipMemcpyAsync(&prof_st[prof_par], st.p, sizeof(StepState), hipMemcpyDeviceToHost, stream));
			HIP_CHECK(hipEventRecord(ev_done[prof_par], stream));
			prof_pending[prof_par] = true;
			prof_par ^= 1;
			if (prof_pending[prof_par]) accumulate_phases(prof_par);  // the previous step
		}
		it_collect();
	}

	// A step's ray sampling: ray generation + the march's two passes, the coordinate write (and round 0's list, unsorted
	// progressive), the spatial ray sort (sorted progressive); rng / progressive: the step's own (train_step, or the
	// lookahead for the next step), scan: the look-back state of the stream it runs on.
	void issue_march(hipStream_t s, const DPInfo& dp, const pcg32& r, bool progressive, uint8_t* scan, bool cut = false, bool mcut = false) {
		const std::vector<uint32_t>& ce = ends_for(cut);
		const uint32_t nch = (uint32_t)ce.size() + 1;
		const Round0List r0{ce[0], cbase.p, chunk_list.p, chunk_cnt.p, nch + 1};
		const bool sorted_rays = progressive && ray_sort;
		MarchWork mw = mwork;
		if (mcut) mw.est_cut = cutw.p + CW_EST;  // (the split sort's estimate: pass A's slots are the marched ones)
		mw.est_div = mcut_div;
		launch_march_count(s, MAX_RAYS, max_samples, st.p, dp, ds, bitfield.p, bf_lin.p, r.state, r.inc, rays.p, startt.p, nreq.p, mw,
		                   progressive ? chunk_cnt.p : nullptr, RAW_CNT + nch, ray_cull ? occ_bbox.p : nullptr);  // list lengths + open-ray counts
		launch_march_write(s, MAX_RAYS, st.p, ds, rays.p, mw, nreq.p, base.p, numsteps.p, coords.p, nullptr, max_samples, scan,
		                   progressive && !sorted_rays ? &r0 : nullptr, dbg_lds_fill);
		const RaySort rsort{rs_hist.p, rs_off.p, rs_key.p, rs_perm.p, chunk_cnt.p + RS_N_PERM};
		const RaySplit split{cutw.p + CW_EST, ccount.p, cutw.p, MAX_RAYS, max_samples};
		if (sorted_rays)
			launch_ray_sort(s, MAX_RAYS, numsteps.p, coords.p, ce[0], rsort, chunk_list.p, chunk_cnt.p, scan, scan_tmp_bytes, cut ? &split : nullptr);
	}

	LossWork loss_work(const uint32_t* rbase) {
		LossWork w{};
		w.sa = l_sa.p; w.ck4 = l_ck4.p; w.cke = l_cke.p; w.ekt = l_ekt.p; w.sample_ray = sample_ray.p; w.rbase = rbase; w.cmap = cmap.p;
		w.racc = l_racc.p; w.rT = l_rT.p; w.rgr = l_rgr.p; w.rek = l_rek.p;
		w.long_rays = long_rays.p; w.n_long = chunk_cnt.p + 16;
		return w;
	}

	void accumulate_phases(int par) {
		HIP_CHECK(hipEventSynchronize(ev_done[par]));
		for (int i = 0; i < N_PHASES; ++i) {
			float ms = 0.f;
			HIP_CHECK(hipEventElapsedTime(&ms, ev[par][i], ev[par][i + 1]));
			phase_ms[i] += ms;
		}
		const StepState& h = prof_st[par];
		phase_npre += h.n_kept;
		phase_ntrain += std::min(h.compacted_global / std::max(1u, world), batch);
		++phase_steps;
		prof_pending[par] = false;
	}
	void flush_phases() {
		// oldest first: the set about to be reused is the older one
		if (prof_pending[prof_par]) accumulate_phases(prof_par);
		if (prof_pending[prof_par ^ 1]) accumulate_phases(prof_par ^ 1);
	}

	// raise = false (stats): record the health bits and the abort without throwing
	void consume_loss(bool raise = true) {
		if (!loss_pending) return;
		HIP_CHECK(hipEventSynchronize(ev_loss));
		const StepState* sst = (const StepState*)(pinned + 64);
		const float measured = (float)sst->compacted_global / (float)world;
		const float scale = measured / (float)batch;
		last_loss = pinned[0] * scale;
		ek_loss = pinned[1] * scale;
		mask_loss = pinned[2] * scale;
		last_rays_with_samples = sst->rays_ws_global;
		last_keep_ratio = sst->n_kept ? measured / (float)sst->n_kept : 1.f;  // composited / kept (progressive inference)
		choose_chunk_ends(sst->compacted_global, sst->rays_ws_global);
		ray_loss = sst->rays_ws_global ? pinned[0] * (float)(sst->rays_per_batch * world) / (float)sst->rays_ws_global : 0.f;
		if (!loss_ema_init) { loss_scalar_ema = last_loss; loss_ema_init = true; }
		else loss_scalar_ema = 0.99f * loss_scalar_ema + 0.01f * last_loss;
		// health: a non-finite loss sum (a NaN / Inf flag on the loss; the sums are all-reduced, so every
		// rank raises it on the same step), and the zero-sample guard (testbed_nerf.cu:3542-3548: loss scalars 0,
		// training stops - the Python frame() loop reads training_aborted)
		if (!std::isfinite(pinned[0]) || !std::isfinite(pinned[1]) || !std::isfinite(pinned[2])) { nonfinite = true; aborted = true; }
		if (sst->compacted_global == 0) {
			loss_scalar_ema = last_loss = ek_loss = mask_loss = 0.f;
			aborted = true;
		}
		loss_pending = false;
		// device health (sticky): a march that met a non-finite / negative t, a look-back scan that gave up waiting. Either
		// means corrupted sampling or compaction bases: training stops with an error instead of continuing on bad data.
		uint32_t scan_fail = 0, all[2] = {0, 0};
		std::memcpy(&scan_fail, pinned + 48, 4);
		std::memcpy(all, pinned + 52, 8);  // the health words summed over the ranks (this rank's alone at world 1)
		const uint32_t local = sst->fail_flags | (scan_fail ? STEP_FAIL_SCAN : 0u);
		// the words are sums over the ranks, not bit sets: word 0 sums the ranks' fail_flags (the march sets only
		// STEP_FAIL_MARCH_T there), word 1 the scans' give-up counters; any nonzero sum names its cause
		const uint32_t global = (all[0] ? STEP_FAIL_MARCH_T : 0u) | (all[1] ? STEP_FAIL_SCAN : 0u);
		health_raise(local | (coll_on() ? global : 0u), local == 0 && coll_on() && global != 0, raise);
	}
	uint32_t fail_seen = 0;
	void health_raise(uint32_t flags, bool other_rank = false, bool raise = true) {
		if (!flags) return;
		fail_seen |= flags;
		aborted = true;
		if (!raise) return;
		std::string m = other_rank ? "training step: device health check failed on another rank:" : "training step: device health check failed:";
		if (flags & STEP_FAIL_MARCH_T) m += " the occupancy march met a non-finite or negative t (corrupted sampling state);";
		if (flags & STEP_FAIL_SCAN) m += " a look-back scan gave up waiting for a predecessor tile (compaction bases are wrong);";
		throw std::runtime_error(m);
	}
};

namespace {
template <class F> int guard(F&& f) {
	try { f(); return 0; }
	catch (const std::exception& e) { g_err = e.what(); return 1; }
	catch (...) { g_err = "unknown error"; return 1; }
}
hipStream_t as_stream(NeusTestbed* tb, void* s) { return s ? (hipStream_t)s : tb->stream; }
}

extern "C" {

const char* neus_last_error(void) { return g_err.c_str(); }
int neus_abi_version(uint32_t* out) {
	if (!out) return 1;
	*out = NEUS_ABI_VERSION;
	return 0;
}
int neus_device_count(int* count) { return guard([&] { HIP_CHECK(hipGetDeviceCount(count)); }); }
int neus_device_synchronize(void) { return guard([&] { HIP_CHECK(hipDeviceSynchronize()); }); }

int neus_testbed_create(int device, NeusTestbed** out) {
	return guard([&] {
		g_alloc_base = g_alloc_seq.load();
		*out = new NeusTestbed(device);
	});
}
int neus_testbed_destroy(NeusTestbed* tb) { return guard([&] { delete tb; }); }
int neus_testbed_set_dataset(NeusTestbed* tb, uint32_t n_images, const NeusImage* images, float aabb_scale) {
	return guard([&] { tb->set_dataset(n_images, images, aabb_scale); });
}
int neus_testbed_reload_network(NeusTestbed* tb, const NeusNetworkConfig* cfg, const float* geo) {
	return guard([&] { tb->reset_network(*cfg, geo); });
}
int neus_testbed_layout(NeusTestbed* tb, NeusNetLayout* o) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		const Layout& l = tb->lay;
		o->n_params = l.P; o->n_density = l.n_density; o->n_rgb = l.n_rgb; o->grid_offset = l.grid_off; o->n_grid_params = l.n_grid;
		o->variance_offset = l.var_off; o->n_matrix = l.n_matrix; o->density_input_width = l.din; o->rgb_input_width = 48;
		o->per_level_scale = tb->cfg.per_level_scale; o->n_levels = l.L;
	});
}
int neus_testbed_train(NeusTestbed* tb, uint32_t n_steps) {
	return guard([&] {
		HIP_CHECK(hipSetDevice(tb->device));
		// the LDS-garbage test hook is this thread's while its steps are queued (other testbeds / threads unaffected);
		// the pattern alternates with its complement from step to step
		struct FillScope { ~FillScope() { g_dbg_lds_fill = 0; g_dbg_xcd_shift = 0; } } fill_scope;
		// (a lookahead left pending by a step that threw is dropped: the next step marches again, the same samples)
		struct LaScope { NeusTestbed* t; ~LaScope() { if (t->la_pending) { (void)hipStreamSynchronize(t->la_stream); t->la_pending = false; } t->la_next_in_call = false; if (t->la_stat) t->la_stat_report(); } } la_scope{tb};
		for (uint32_t i = 0; i < n_steps; ++i) {
			g_dbg_lds_fill = tb->dbg_lds_fill_all ? ((tb->training_step & 1) ? ~tb->dbg_lds_fill_all : tb->dbg_lds_fill_all) : 0u;
			g_dbg_xcd_shift = tb->dbg_xcd_shift;
			tb->la_next_in_call = i + 1 < n_steps;
			tb->call_left = n_steps - i - 1;
			tb->train_step();
		}
	});
}
int neus_testbed_get_stats(NeusTestbed* tb, NeusTrainStats* o) {
	return guard([&] {
		tb->consume_loss(false);  // health bits and the abort are reported below, not raised
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		StepState s{};
		HIP_CHECK(hipMemcpy(&s, tb->st.p, sizeof(s), hipMemcpyDeviceToHost));
		float mean = 0.f;
		if (tb->grid_mean.p) HIP_CHECK(hipMemcpy(&mean, tb->grid_mean.p, 4, hipMemcpyDeviceToHost));
		o->training_step = tb->training_step; o->rays_per_batch = s.rays_per_batch; o->measured_batch_size = s.measured_batch_size;
		o->measured_batch_size_before_compaction = s.measured_before; o->n_rays_total = s.n_rays_total;
		o->valid_level = tb->valid_level_at(tb->enc_step); o->zero_records = s.zero_records;
		o->loss = tb->loss_scalar_ema; o->ek_loss = tb->ek_loss; o->mask_loss = tb->mask_loss; o->last_loss = tb->last_loss;
		o->density_grid_mean = mean;
		o->ray_loss = tb->ray_loss; o->n_rays_with_samples = tb->last_rays_with_samples;
		o->trained_samples_total = s.trained_total;
		o->march_first_pass_rays = s.march_est; o->kept_ray_extent = s.kept_extent;
		o->nonfinite_loss = tb->nonfinite ? 1u : 0u;
		o->training_aborted = (tb->aborted || (tb->training_step > 0 && s.zero_records)) ? 1u : 0u;
		o->pre_samples_total = s.pre_total; o->rays_total = s.rays_total;
		o->occ_samples_total = tb->occ_samples; o->occ_updates = tb->occ_updates;
		o->progressive_chunk_end = tb->chunk_ends.empty() ? 0u : tb->chunk_ends[0];
		o->lookahead_steps = tb->la_steps;
		o->cut_steps = tb->cut_steps;
		o->march_cut_steps = tb->mcut_steps;
		o->march_cut_reruns = tb->mcut_reruns;
		o->adam_split_steps = tb->adam_split_steps;
		o->health_flags = s.fail_flags | tb->fail_seen | (scan_failures(tb->scan_tmp.p) ? STEP_FAIL_SCAN : 0u);
		o->evaluated_samples_total = s.eval_total; o->progressive_steps = s.prog_steps; o->evaluated_samples_last = s.eval_last;
	});
}
static int copy_param_vec(NeusTestbed* tb, const float* dev, float* host, uint64_t n) {
	return guard([&] {
		if (!tb->have_net || n != tb->lay.P) throw std::runtime_error("parameter count mismatch");
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		HIP_CHECK(hipMemcpy(host, dev, n * 4, hipMemcpyDeviceToHost));
	});
}
int neus_testbed_get_params(NeusTestbed* tb, float* o, uint64_t n) { return copy_param_vec(tb, tb->params_fp.p, o, n); }
int neus_testbed_get_gradients(NeusTestbed* tb, float* o, uint64_t n) { return copy_param_vec(tb, tb->grads.p, o, n); }
int neus_testbed_get_ema_params(NeusTestbed* tb, float* o, uint64_t n) { return copy_param_vec(tb, tb->ema_tmp.p, o, n); }
int neus_testbed_get_half_params(NeusTestbed* tb, int which, uint16_t* o, uint64_t n) {
	return guard([&] {
		if (!tb->have_net || n != tb->lay.P) throw std::runtime_error("parameter count mismatch");
		if (which != 0 && which != 1) throw std::runtime_error("get_half_params: which must be 0 (training) or 1 (inference)");
		if (which) tb->sync_ema_h();
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		HIP_CHECK(hipMemcpy(o, which ? tb->ema_h.p : tb->params_h.p, n * 2, hipMemcpyDeviceToHost));
	});
}
int neus_testbed_set_params(NeusTestbed* tb, const float* in, uint64_t n) {
	return guard([&] {
		if (!tb->have_net || n != tb->lay.P) throw std::runtime_error("parameter count mismatch");
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		HIP_CHECK(hipMemcpy(tb->params_fp.p, in, n * 4, hipMemcpyHostToDevice));
		launch_cast_half(tb->stream, (uint32_t)n, tb->params_fp.p, tb->params_h.p);
		tb->prepare_weights();
		HIP_CHECK(hipStreamSynchronize(tb->stream));
	});
}
int neus_testbed_get_density_grid(NeusTestbed* tb, float* g, uint8_t* bf) {
	return guard([&] {
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		if (g) HIP_CHECK(hipMemcpy(g, tb->density_grid.p, (size_t)GRID3 * 4, hipMemcpyDeviceToHost));
		if (bf) HIP_CHECK(hipMemcpy(bf, tb->bitfield.p, GRID3 / 8 * NERF_CASCADES, hipMemcpyDeviceToHost));
	});
}
int neus_testbed_set_density_grid(NeusTestbed* tb, const float* g, const uint8_t* bf) {
	return guard([&] {
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		if (g) HIP_CHECK(hipMemcpy(tb->density_grid.p, g, (size_t)GRID3 * 4, hipMemcpyHostToDevice));
		if (bf) {
			HIP_CHECK(hipMemcpy(tb->bitfield.p, bf, GRID3 / 8 * NERF_CASCADES, hipMemcpyHostToDevice));
			launch_bitfield_linear(tb->stream, tb->bitfield.p, tb->bf_lin.p);
			launch_occ_bbox(tb->stream, tb->bitfield.p, tb->occ_bbox.p);
			HIP_CHECK(hipStreamSynchronize(tb->stream));
		}
	});
}
// Testbed::load_snapshot after reset_network + Trainer::deserialize (testbed.cu:3197-3254, trainer.h:295-304):
// training step, loss scalar, adaptive-batch counters; the inference (EMA) weights start as the loaded ones
// (Trainer::set_params writes m_params_inference too); density grid mean + bitfield rebuilt
// (update_density_grid_mean_and_bitfield, testbed.cu:3240).
int neus_testbed_restore_state(NeusTestbed* tb, const NeusRestoreState* in) {
	return guard([&] {
		if (!in) throw std::runtime_error("restore_state: null argument");
		if (!tb->have_net) throw std::runtime_error("restore_state: no network (reload_network first)");
		if (in->rays_per_batch == 0 || in->rays_per_batch > MAX_RAYS || in->rays_per_batch % 128 != 0)
			throw std::runtime_error("restore_state: rays_per_batch must be a positive multiple of 128 <= 2^18");
		HIP_CHECK(hipSetDevice(tb->device));
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		tb->consume_loss();
		StepState s{};
		HIP_CHECK(hipMemcpy(&s, tb->st.p, sizeof(s), hipMemcpyDeviceToHost));
		s.rays_per_batch = in->rays_per_batch;
		s.measured_batch_size = in->measured_batch_size;
		s.measured_before = in->measured_batch_size_before_compaction;
		HIP_CHECK(hipMemcpy(tb->st.p, &s, sizeof(s), hipMemcpyHostToDevice));
		tb->training_step = in->training_step;
		tb->loss_scalar_ema = tb->last_loss = in->loss;
		tb->loss_ema_init = true;
		HIP_CHECK(hipMemcpy(tb->ema_h.p, tb->params_h.p, (size_t)tb->lay.P * 2, hipMemcpyDeviceToDevice));
		tb->ema_h_stale = false;
		// the fp32 EMA follows the loaded inference weights (the first EMA step after a reload weighs it by 0)
		HIP_CHECK(hipMemcpy(tb->ema_tmp.p, tb->params_fp.p, (size_t)tb->lay.P * 4, hipMemcpyDeviceToDevice));
		if (in->rebuild_bitfield) {
			launch_grid_mean(tb->stream, tb->density_grid.p, tb->grid_partial.p, tb->grid_mean.p);
			launch_bitfield(tb->stream, tb->density_grid.p, tb->bitfield.p, tb->grid_mean.p, tb->max_cascade + 1);
			launch_bitfield_linear(tb->stream, tb->bitfield.p, tb->bf_lin.p);
			launch_occ_bbox(tb->stream, tb->bitfield.p, tb->occ_bbox.p);
		}
		HIP_CHECK(hipStreamSynchronize(tb->stream));
	});
}
int neus_testbed_get_optimizer_state(NeusTestbed* tb, NeusOptimizerState* st, float* m1, float* m2, uint32_t* steps, uint16_t* ema_half) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("optimizer state: no network");
		tb->sync_ema_h();
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		const size_t P = tb->lay.P;
		if (st) {
			st->n_params = (uint32_t)P;
			st->current_step = tb->adam_step;
			st->learning_rate = tb->cur_frame ? tb->cfg.after_learning_rate : tb->cfg.learning_rate;
			st->learning_rate_factor = tb->lr_factor;
		}
		if (m1) HIP_CHECK(hipMemcpy(m1, tb->m1.p, P * 4, hipMemcpyDeviceToHost));
		if (m2) HIP_CHECK(hipMemcpy(m2, tb->m2.p, P * 4, hipMemcpyDeviceToHost));
		if (steps) tb->get_steps(steps);  // (saturated at 65535 while the bias table is converged: optim.hip AdamSteps)
		if (ema_half) HIP_CHECK(hipMemcpy(ema_half, tb->ema_h.p, P * 2, hipMemcpyDeviceToHost));
	});
}
int neus_testbed_set_optimizer_state(NeusTestbed* tb, const NeusOptimizerState* st, const float* m1, const float* m2, const uint32_t* steps,
                                     const uint16_t* ema_half) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("optimizer state: no network");
		if (!st || !m1 || !m2 || !ema_half) throw std::runtime_error("set_optimizer_state: state, moments and EMA weights are required");
		const size_t P = tb->lay.P;
		if (st->n_params != P) throw std::runtime_error("set_optimizer_state: parameter count mismatch");
		HIP_CHECK(hipSetDevice(tb->device));
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		HIP_CHECK(hipMemcpy(tb->m1.p, m1, P * 4, hipMemcpyHostToDevice));
		HIP_CHECK(hipMemcpy(tb->m2.p, m2, P * 4, hipMemcpyHostToDevice));
		// Adam::deserialize: param_steps absent -> zeros (adam.h:437-442)
		tb->ensure_bias_table();  // (the counts' width follows the betas' bias table)
		tb->put_steps(steps);
		// Ema::deserialize (ema.h:189-194): the EMA weights, and the fp32 accumulator cast from them
		HIP_CHECK(hipMemcpy(tb->ema_h.p, ema_half, P * 2, hipMemcpyHostToDevice));
		tb->ema_h_stale = false;
		std::vector<float> f(P);
		for (size_t i = 0; i < P; ++i) { half_t h; std::memcpy(&h, &ema_half[i], 2); f[i] = (float)h; }
		HIP_CHECK(hipMemcpy(tb->ema_tmp.p, f.data(), P * 4, hipMemcpyHostToDevice));
		tb->adam_step = st->current_step;
		tb->lr_factor = st->learning_rate_factor;
		tb->sync_ema_h(); tb->prepare_weights_for(tb->mlp_ema);
		HIP_CHECK(hipStreamSynchronize(tb->stream));
	});
}
int neus_testbed_render(NeusTestbed* tb, const NeusRenderRequest* rq, float* rgba_out, uint32_t* n_iterations) {
	return guard([&] {
		if (!rq || !rgba_out) throw std::runtime_error("render: null argument");
		HIP_CHECK(hipSetDevice(tb->device));
		const uint32_t it = tb->render(*rq, rgba_out);
		if (n_iterations) *n_iterations = it;
	});
}
int neus_testbed_sdf_on_grid(NeusTestbed* tb, const int32_t res[3], const float aabb_min[3], const float aabb_max[3], float* host_out) {
	return guard([&] {
		HIP_CHECK(hipSetDevice(tb->device));
		uint32_t r[3];
		for (int k = 0; k < 3; ++k) { if (res[k] < 1) throw std::runtime_error("sdf_on_grid: empty resolution"); r[k] = (uint32_t)res[k]; }
		const uint64_t n = (uint64_t)r[0] * r[1] * r[2];
		tb->mc_density.alloc(n);
		tb->sdf_on_grid(r, aabb_min, aabb_max, tb->mc_density.p);
		HIP_CHECK(hipMemcpyAsync(host_out, tb->mc_density.p, n * 4, hipMemcpyDeviceToHost, tb->stream));
		HIP_CHECK(hipStreamSynchronize(tb->stream));
	});
}
int neus_testbed_marching_cubes(NeusTestbed* tb, const int32_t res[3], const float aabb_min[3], const float aabb_max[3], float thresh,
                                const float* density_dev, uint32_t* n_verts, uint32_t* n_tris) {
	return guard([&] {
		HIP_CHECK(hipSetDevice(tb->device));
		tb->marching_cubes(res, aabb_min, aabb_max, thresh, density_dev);
		if (n_verts) *n_verts = tb->mesh_nv;
		if (n_tris) *n_tris = tb->mesh_nt;
	});
}
int neus_testbed_mc_density(NeusTestbed* tb, uint64_t offset, uint64_t count, float* host_out) {
	return guard([&] {
		if (!host_out || offset + count > tb->mc_density.n) throw std::runtime_error("mc_density: range outside the last SDF grid");
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		HIP_CHECK(hipMemcpy(host_out, tb->mc_density.p + offset, count * 4, hipMemcpyDeviceToHost));
	});
}
int neus_testbed_get_mesh(NeusTestbed* tb, float* verts, uint32_t* tris) {
	return guard([&] {
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		if (verts && tb->mesh_nv) HIP_CHECK(hipMemcpy(verts, tb->mesh_v.p, (size_t)tb->mesh_nv * 12, hipMemcpyDeviceToHost));
		if (tris && tb->mesh_nt) HIP_CHECK(hipMemcpy(tris, tb->mesh_f.p, (size_t)tb->mesh_nt * 12, hipMemcpyDeviceToHost));
	});
}
int neus_testbed_mesh_vertex_colors(NeusTestbed* tb, float* rgb) {
	return guard([&] {
		if (!rgb) throw std::runtime_error("mesh_vertex_colors: null output");
		HIP_CHECK(hipSetDevice(tb->device));
		tb->mesh_colors(rgb);
	});
}
int neus_mc_table(int8_t* out) { return guard([&] { mc_table_host(out); }); }
int neus_prepare_image_rgba8(uint8_t* rgba, uint32_t w, uint32_t h, const uint8_t* alpha_rgba, const uint8_t* mask_rgba, uint32_t flags,
                             uint32_t* mask_color_out) {
	return guard([&] {
		if (!rgba) throw std::runtime_error("prepare_image: null image");
		const uint64_t n = (uint64_t)w * h;
		if (alpha_rgba) {
			// srgb_to_linear (common_device.cuh:31-37) of the alpha image's red channel, as a 256-entry table
			uint8_t lut[256];
			for (int v = 0; v < 256; ++v) {
				const float srgb = (float)v * (1.f / 255.f);
				const float lin = srgb <= 0.04045f ? srgb / 12.92f : std::pow((srgb + 0.055f) / 1.055f, 2.4f);
				lut[v] = (uint8_t)(255.0f * lin);
			}
			for (uint64_t i = 0; i < n; ++i) rgba[4 * i + 3] = lut[alpha_rgba[4 * i]];
		}
		const uint32_t key = mask_rgba ? 0x00FF00FFu : 0u;  // hot pink
		if (mask_rgba)
			for (uint64_t i = 0; i < n; ++i)
				if (mask_rgba[4 * i] != 0) std::memcpy(rgba + 4 * i, &key, 4);
		const bool wt = flags & NEUS_IMAGE_WHITE_TRANSPARENT, bt = flags & NEUS_IMAGE_BLACK_TRANSPARENT;
		if (wt || bt || key)
			for (uint64_t i = 0; i < n; ++i) {
				uint8_t* p = rgba + 4 * i;
				if (wt && p[0] == 255 && p[1] == 255 && p[2] == 255) p[3] = 0;
				if (bt && p[0] == 0 && p[1] == 0 && p[2] == 0) p[3] = 0;
				uint32_t v;
				std::memcpy(&v, p, 4);
				if (key != 0 && v == key) { p[0] = 0xFF; p[1] = 0x00; p[2] = 0xFF; p[3] = 0x00; }
			}
		if (mask_color_out) *mask_color_out = key;
	});
}
int neus_testbed_next_frame(NeusTestbed* tb, uint32_t n_images, const NeusImage* images) {
	return guard([&] {
		HIP_CHECK(hipSetDevice(tb->device));
		tb->next_frame(n_images, images);
	});
}
int neus_testbed_change_frame(NeusTestbed* tb, uint32_t frame, uint32_t n_images, const NeusImage* images) {
	return guard([&] {
		HIP_CHECK(hipSetDevice(tb->device));
		tb->change_frame(frame, n_images, images);
	});
}
int neus_testbed_prepare_for_test(NeusTestbed* tb, int* out_use_delta) {
	return guard([&] {
		tb->render_delta = tb->cur_frame != 0 && tb->train_delta;
		if (out_use_delta) *out_use_delta = tb->render_delta ? 1 : 0;
	});
}
int neus_testbed_saved_transform(NeusTestbed* tb, float* out12) {
	return guard([&] {
		if (!out12) throw std::runtime_error("saved_transform: null output");
		if (!tb->have_net) throw std::runtime_error("save_transform: no network");
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		DeltaState h{};
		HIP_CHECK(hipMemcpy(&h, tb->delta.p, sizeof(h), hipMemcpyDeviceToHost));
		float R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t[3] = {0, 0, 0};
		if (tb->ds.motion.on) { std::memcpy(R, tb->ds.motion.R, sizeof(R)); std::memcpy(t, tb->ds.motion.t, sizeof(t)); }
		host_accumulate_movement(h.p, R, t);
		std::memcpy(out12, R, sizeof(R)); std::memcpy(out12 + 9, t, sizeof(t));
	});
}
int neus_testbed_get_training_options(NeusTestbed* tb, NeusTrainingOptions* o) {
	return guard([&] {
		if (!o) throw std::runtime_error("get_training_options: null output");
		const TrainTarget& t = tb->ds.target;
		o->random_bg_color = t.fixed_bg ? 0 : 1;
		for (int k = 0; k < 3; ++k) o->background_color[k] = t.bg[k];
		o->color_space = t.mode == 1 ? 1 : 0;
		o->linear_colors = t.mode == 2 ? 1 : 0;
		if (t.mode == 2) o->color_space = tb->color_space_when_linear;
		o->cone_angle_constant = tb->ds.cone_angle;
		o->near_distance = tb->near_distance;
		o->depth_supervision_lambda = tb->depth_lambda;
	});
}
int neus_testbed_set_progressive_inference(NeusTestbed* tb, int mode, const uint32_t* chunk_ends, uint32_t n_ends) {
	return guard([&] {
		if (mode < 0 || mode > 2) throw std::runtime_error("progressive inference mode must be 0 (off), 1 (auto) or 2 (always)");
		if (chunk_ends && n_ends) {
			if (n_ends > 14) throw std::runtime_error("at most 14 chunk ends");
			for (uint32_t k = 0; k < n_ends; ++k)
				if (chunk_ends[k] == 0 || (k && chunk_ends[k] <= chunk_ends[k - 1])) throw std::runtime_error("chunk ends must increase from >= 1");
			tb->chunk_ends.assign(chunk_ends, chunk_ends + n_ends);
			tb->chunk_ends_cut.clear();
			tb->chunk_auto = false;
		}
		tb->progressive_mode = mode;
	});
}

int neus_testbed_set_training_options(NeusTestbed* tb, const NeusTrainingOptions* o) {
	return guard([&] {
		if (!o) throw std::runtime_error("set_training_options: null options");
		if (o->color_space != 0 && o->color_space != 1) throw std::runtime_error("color_space must be 0 (Linear) or 1 (SRGB)");
		if (!(o->cone_angle_constant >= 0.0f)) throw std::runtime_error("cone_angle_constant must be >= 0");
		HIP_CHECK(hipStreamSynchronize(tb->stream));  // kernels in flight read ds by value; later steps see the new targets
		TrainTarget t{};
		t.fixed_bg = o->random_bg_color ? 0u : 1u;
		for (int k = 0; k < 3; ++k) t.bg[k] = o->background_color[k];
		// train_in_linear_colors wins over the colour space (testbed_nerf.cu:1658)
		t.mode = o->linear_colors ? 2u : (o->color_space == 1 ? 1u : 0u);
		tb->color_space_when_linear = o->color_space;
		tb->ds.target = t;
		tb->ds.cone_angle = o->cone_angle_constant;
		tb->near_distance = o->near_distance;
		if (!(o->depth_supervision_lambda >= 0.f)) throw std::runtime_error("depth_supervision_lambda must be >= 0");
		tb->depth_lambda = o->depth_supervision_lambda;
	});
}
int neus_testbed_get_movement(NeusTestbed* tb, float* global12, float* local12) {
	return guard([&] {
		if (global12) { std::memcpy(global12, tb->ds.motion.R, 9 * 4); std::memcpy(global12 + 9, tb->ds.motion.t, 3 * 4); }
		if (local12) {
			if (!tb->have_net) throw std::runtime_error("get_movement: no network");
			DeltaState h{};
			HIP_CHECK(hipStreamSynchronize(tb->stream));
			HIP_CHECK(hipMemcpy(&h, tb->delta.p, sizeof(h), hipMemcpyDeviceToHost));
			std::memcpy(local12, h.p, DELTA_PARAMS * 4);
		}
	});
}
int neus_testbed_set_movement(NeusTestbed* tb, const float* global12, const float* local12) {
	return guard([&] {
		if (global12) {
			std::memcpy(tb->ds.motion.R, global12, 9 * 4); std::memcpy(tb->ds.motion.t, global12 + 9, 3 * 4);
			const float I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
			bool ident = global12[9] == 0.f && global12[10] == 0.f && global12[11] == 0.f;
			for (int k = 0; k < 9; ++k) ident = ident && global12[k] == I[k];
			tb->ds.motion.on = ident ? 0u : 1u;
		}
		if (local12) {
			if (!tb->have_net) throw std::runtime_error("set_movement: no network");
			DeltaState h{};
			HIP_CHECK(hipStreamSynchronize(tb->stream));
			HIP_CHECK(hipMemcpy(&h, tb->delta.p, sizeof(h), hipMemcpyDeviceToHost));
			std::memcpy(h.p, local12, DELTA_PARAMS * 4);
			HIP_CHECK(hipMemcpy(tb->delta.p, &h, sizeof(h), hipMemcpyHostToDevice));
			launch_delta_prepare(tb->stream, tb->delta.p);
			HIP_CHECK(hipStreamSynchronize(tb->stream));
		}
	});
}
int neus_testbed_frame_state(NeusTestbed* tb, uint32_t* o) {
	return guard([&] { o[0] = tb->cur_frame; o[1] = tb->canonical_step; o[2] = tb->train_canonical; o[3] = tb->train_delta; });
}
int neus_testbed_get_rng(NeusTestbed* tb, uint64_t* o) {
	return guard([&] { o[0] = tb->rng.state; o[1] = tb->rng.inc; o[2] = tb->density_grid_rng.state; o[3] = tb->density_grid_rng.inc; });
}
int neus_testbed_ray_counts(NeusTestbed* tb, uint32_t n, uint32_t* nreq, uint32_t* ccount, uint32_t* numsteps) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		n = std::min(n, MAX_RAYS);
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		if (nreq) HIP_CHECK(hipMemcpy(nreq, tb->nreq.p, (size_t)n * 4, hipMemcpyDeviceToHost));
		if (ccount) HIP_CHECK(hipMemcpy(ccount, tb->ccount.p, (size_t)n * 4, hipMemcpyDeviceToHost));
		if (numsteps) HIP_CHECK(hipMemcpy(numsteps, tb->numsteps.p, (size_t)n * 8, hipMemcpyDeviceToHost));
	});
}
static void time_kernel_impl(NeusTestbed* tb, int kernel, int variant, int iters, float* ms_out);
int neus_debug_time_kernel(NeusTestbed* tb, int kernel, int variant, int iters, float* ms_out) {
	return guard([&] { time_kernel_impl(tb, kernel, variant, iters, ms_out); });
}
int neus_testbed_time_kernel(NeusTestbed* tb, int kernel, int iters, float* ms_out, uint32_t* units_out) {
	return guard([&] {
		time_kernel_impl(tb, kernel, 0, iters, ms_out);
		StepState h{};
		HIP_CHECK(hipMemcpy(&h, tb->st.p, sizeof(StepState), hipMemcpyDeviceToHost));
		// work units of one launch: ray slots (march), pre-compaction samples (write, inference, loss),
		// compacted training samples (encode, MLP, weight gradients, grid scatter), parameters (Adam / EMA)
		*units_out = kernel == 0 ? MAX_RAYS : kernel <= 4 ? h.n_kept : kernel == 12 ? tb->lay.P : tb->batch;
		if (kernel == 13) {  // the slots a cut march generates and marches
			uint32_t est = MAX_RAYS;
			HIP_CHECK(hipMemcpy(&est, tb->cutw.p + CW_EST, 4, hipMemcpyDeviceToHost));
			const uint32_t e0 = h.march_est ? std::min(h.march_est, MAX_RAYS) : MAX_RAYS;
			*units_out = std::min(est, e0);
		}
	});
}
static void time_kernel_impl(NeusTestbed* tb, int kernel, int variant, int iters, float* ms_out) {
	{
		if (!tb->have_net) throw std::runtime_error("no network");
		NeusTestbed& t = *tb;
		hipStream_t s = t.stream;
		const DPInfo dp{t.rank, t.world};
		const uint32_t valid = t.valid_level_at((int)t.training_step);
		const uint32_t* lin = t.bf_lin.p;
		auto march = [&]() {
			launch_march_count(s, MAX_RAYS, t.max_samples, t.st.p, dp, t.ds, t.bitfield.p, lin, t.rng.state, t.rng.inc, t.rays.p, t.startt.p, t.nreq.p, t.mwork,
			                   nullptr, 0, t.ray_cull ? t.occ_bbox.p : nullptr);
			launch_march_write(s, MAX_RAYS, t.st.p, t.ds, t.rays.p, t.mwork, t.nreq.p, t.base.p, t.numsteps.p, t.coords.p,
			                   t.sample_ray.p, t.max_samples, t.scan_tmp.p);
		};
		const LossWork w = t.loss_work(t.base.p);
		if (variant != 99) {  // 99: no re-preparation (counter runs: only the timed kernel is launched)
			march();
			launch_nerf_infer(s, t.lay.L, t.lay.W, &t.st.p->n_kept, 0, t.coords.p, t.gl, valid, t.params_h.p + t.lay.grid_off, t.mlp, t.net_out.p, 8192);
			launch_loss_alpha(s, t.max_samples, t.st.p, t.coords.p, t.net_out.p, t.cos_anneal(), w);
		}
		// one event between consecutive launches (fence-free: timing only); the median launch is reported
		iters = std::max(1, iters);
		std::vector<hipEvent_t> evs((size_t)iters + 1);
		for (auto& e : evs) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
		for (int k = 0; k < iters; ++k) {
			// (variant 98: no event between the launches - back to back, for the queue gaps of a kernel trace)
			if (variant != 98 || k == 0) HIP_CHECK(hipEventRecord(evs[k], s));
			switch (kernel) {
			case 0: launch_march_count(s, MAX_RAYS, t.max_samples, t.st.p, dp, t.ds, t.bitfield.p, lin, t.rng.state, t.rng.inc, t.rays.p, t.startt.p, t.nreq.p, t.mwork,
			                   nullptr, 0, t.ray_cull ? t.occ_bbox.p : nullptr); break;
			case 1: launch_march_write(s, MAX_RAYS, t.st.p, t.ds, t.rays.p, t.mwork, t.nreq.p, t.base.p, t.numsteps.p,
			                           t.coords.p, t.sample_ray.p, t.max_samples, t.scan_tmp.p); break;
			case 2: debug_launch_loss_scan(s, variant, MAX_RAYS, t.numsteps.p, w, t.ccount.p); break;
			case 3: launch_nerf_infer(s, t.lay.L, t.lay.W, &t.st.p->n_kept, 0, t.coords.p, t.gl, valid, t.params_h.p + t.lay.grid_off, t.mlp,
			                          t.net_out.p, 8192); break;
			case 4: launch_loss_alpha(s, t.max_samples, t.st.p, t.coords.p, t.net_out.p, t.cos_anneal(), w); break;
			case 5: case 9: case 10: {  // the training-MLP kernels (5 both, 9 colour, 10 density) on the last compacted batch
				TrainBufs tbuf = t.tbuf;
				tbuf.var_grad = t.grads.p + t.lay.var_off;
				launch_mlp_train(s, t.lay.L, t.lay.W, nullptr, t.batch, t.batch, t.coords_c.p, (const half_t*)t.enc.p, t.dydx.p, t.dL_dout.p, t.mlp, tbuf,
				                 kernel == 5 ? 0 : kernel - 8);
				break;
			}
			case 6: launch_mlp_grad_reduce(s, t.grad_reduce(t.batch, t.grads.p, nullptr)); break;
			case 7:
				launch_grid_scatter(s, nullptr, t.batch, t.batch, t.coords_c.p, COORD_W, t.gl, valid, t.tbuf.dLdenc, t.tbuf.genc, t.tbuf.v,
				                    t.grads.p + t.lay.grid_off, t.swork, t.scan_tmp.p, t.scan_tmp_bytes);
				t.sc_zero_from = t.swork.n_buckets;  // the replay wrote every bucket: nothing is known zero for the next step
				t.sc_zero_from_e = t.gl.offset[t.gl.n_levels];
				break;
			case 8: t.encode(nullptr, t.batch, t.batch, t.batch, t.coords_c.p, COORD_W, valid, true, s); break;
			case 11: {
				// level-partitioned gather experiment: the level-major encode (enc only, no dy/dx) over the
				// inference's pre-compaction samples; variant = workgroups per level (0: 2048)
				if (!t.dbg_enc.p) t.dbg_enc.alloc((size_t)t.lay.L * t.max_samples);
				launch_grid_encode(s, &t.st.p->n_kept, 0, t.max_samples, t.coords.p, COORD_W, t.gl, valid, t.params_h.p + t.lay.grid_off,
				                   t.dbg_enc.p, nullptr, variant > 0 && variant != 99 ? (uint32_t)variant : 2048u, nullptr);
				break;
			}
			case 12: t.optimizer_step(t.grads.p); break;  // the Adam / EMA pass on the last gradient (advances the optimizer)
			case 14: {  // development: the occupancy update's density pass (k_nerf_density MODE 2 into the scratch grid) on the
				        // current state: variant 0 both halves (after step 256), 1 the uniform half, 2 the occupancy-biased half
				const uint32_t nc = GRID3 * (t.max_cascade + 1);
				const uint32_t n_u = variant == 2 ? 0u : nc / 4, n_nu = variant == 1 ? 0u : nc / 4;
				pcg32 r = t.density_grid_rng;
				const pcg32 rng_u = r;
				r.advance();
				const pcg32 rng_nu = r;
				OccSampling os{};
				os.n_u = n_u; os.n_nu = n_nu; os.lo = 0;
				os.rng_u_state = rng_u.state; os.rng_u_inc = rng_u.inc; os.rng_nu_state = rng_nu.state; os.rng_nu_inc = rng_nu.inc;
				os.step = t.density_grid_ema_step; os.n_cascades = t.max_cascade + 1; os.thresh_nu = NERF_MIN_OPTICAL_THICKNESS;
				for (int d = 0; d < 3; ++d) { os.amin[d] = t.ds.aabb_min[d]; os.diag[d] = t.ds.aabb_max[d] - t.ds.aabb_min[d]; }
				os.grid_in = t.density_grid.p; os.grid_tmp = t.density_tmp.p;
				os.jt = t.jump_table();
				if (n_u) {
					if (!t.occ_ulist.p) t.occ_ulist.alloc(GRID3);
					launch_occ_uniform_list(s, n_u, t.density_grid_ema_step, 0, n_u, t.occ_ulist.p, t.scan_tmp.p);
					os.ulist = t.occ_ulist.p; os.n_ulist = n_u;
				}
				launch_occ_density(s, t.lay.L, t.lay.W, n_u + n_nu, os, t.gl, valid, t.params_h.p + t.lay.grid_off, t.mlp);
				break;
			}
			case 13: {  // the march of a cut step: ray generation + the march over the slots below the cut's estimate
				MarchWork mw = t.mwork;
				mw.est_cut = t.cutw.p + CW_EST;
				launch_march_count(s, MAX_RAYS, t.max_samples, t.st.p, dp, t.ds, t.bitfield.p, lin, t.rng.state, t.rng.inc, t.rays.p, t.startt.p, t.nreq.p,
				                   mw, nullptr, 0, t.ray_cull ? t.occ_bbox.p : nullptr);
				break;
			}
			default: throw std::runtime_error("unknown kernel id");
			}
		}
		HIP_CHECK(hipEventRecord(evs[iters], s));
		HIP_CHECK(hipStreamSynchronize(s));
		std::vector<float> d((size_t)iters);
		if (variant == 98) {
			float all = 0.f;
			HIP_CHECK(hipEventElapsedTime(&all, evs[0], evs[iters]));
			for (auto& x : d) x = all / (float)iters;
		} else
			for (int k = 0; k < iters; ++k) HIP_CHECK(hipEventElapsedTime(&d[k], evs[k], evs[k + 1]));
		std::sort(d.begin(), d.end());
		*ms_out = d[(size_t)iters / 2];
		for (auto& e : evs) HIP_CHECK(hipEventDestroy(e));
	}
}
int neus_debug_march_stats(NeusTestbed* tb, uint32_t n, uint32_t* out) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		if (tb->ds.cone_angle != 0.0f) throw std::runtime_error("march stats: cone_angle 0 only");
		n = std::min(n, MAX_RAYS);
		Dev<uint32_t> o; o.alloc(3 * (size_t)n);
		debug_launch_march_stats(tb->stream, n, tb->rays.p, tb->startt.p, tb->bf_lin.p, tb->ds, tb->bitfield.p, o.p);
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		HIP_CHECK(hipMemcpy(out, o.p, 12 * (size_t)n, hipMemcpyDeviceToHost));
	});
}
int neus_debug_scatter_stats(NeusTestbed* tb, uint64_t* records_per_level, uint32_t* max_region) {
	return guard([&] {
		if (!tb->have_net || tb->swork.mode != 2) throw std::runtime_error("scatter stats: region mode only");
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		const uint32_t L = tb->lay.L, nb = tb->swork.n_chunks;
		std::vector<uint16_t> h((size_t)L * nb * (SB_LEVEL_BUCKETS + 1));
		HIP_CHECK(hipMemcpy(h.data(), tb->sc_rtab.p, h.size() * 2, hipMemcpyDeviceToHost));
		uint32_t mx = 0;
		for (uint32_t l = 0; l < L; ++l) {
			const uint32_t size = tb->gl.offset[l + 1] - tb->gl.offset[l], nlb = (size + SB_SIZE - 1) / SB_SIZE;
			uint64_t t = 0;
			for (uint32_t b = 0; b < nb; ++b) {
				const uint32_t r = h[((size_t)l * nb + b) * (SB_LEVEL_BUCKETS + 1) + nlb];
				t += r; mx = std::max(mx, r);
			}
			if (records_per_level) records_per_level[l] = t;
		}
		if (max_region) *max_region = mx;
	});
}
int neus_debug_scatter_parts(NeusTestbed* tb, uint32_t* parts_per_level) {
	return guard([&] {
		if (!tb->have_net || tb->swork.mode != 2) throw std::runtime_error("scatter parts: region mode only");
		std::vector<uint32_t> jobs(4 * (size_t)tb->swork.n_jobs2);
		HIP_CHECK(hipMemcpy(jobs.data(), tb->sc_jobs2.p, jobs.size() * 4, hipMemcpyDeviceToHost));
		for (uint32_t l = 0; l < tb->lay.L; ++l) parts_per_level[l] = 0;
		for (size_t j = 0; j < jobs.size() / 4; ++j) parts_per_level[jobs[4 * j]] = std::max(parts_per_level[jobs[4 * j]], jobs[4 * j + 2] >> 16);
	});
}
int neus_debug_march_profile(NeusTestbed* tb, unsigned long long* out, uint32_t max_waves, uint32_t* n_waves) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		NeusTestbed& t = *tb;
		hipStream_t s = t.stream;
		const uint32_t waves = MAX_RAYS * t.mwork.lanes_per_ray / 64;
		Dev<unsigned long long> buf; buf.alloc((size_t)waves * 8);
		HIP_CHECK(hipMemsetAsync(buf.p, 0, (size_t)waves * 64, s));
		MarchWork mw = t.mwork;
		mw.prof = buf.p;
		if (const char* e = std::getenv("NEUS_MARCH_DBG")) mw.dbg = (uint32_t)std::strtoul(e, nullptr, 10);
		launch_march_count(s, MAX_RAYS, t.max_samples, t.st.p, DPInfo{t.rank, t.world}, t.ds, t.bitfield.p, t.bf_lin.p, t.rng.state, t.rng.inc,
		                   t.rays.p, t.startt.p, t.nreq.p, mw, nullptr, 0, t.ray_cull ? t.occ_bbox.p : nullptr);
		HIP_CHECK(hipStreamSynchronize(s));
		const uint32_t n = std::min(waves, max_waves);
		HIP_CHECK(hipMemcpy(out, buf.p, (size_t)n * 64, hipMemcpyDeviceToHost));
		if (n_waves) *n_waves = n;
	});
}
int neus_debug_exclusive_scan(void* stream, const uint32_t* in, uint32_t* out, uint32_t n, int reps, uint32_t* failures) {
	return guard([&] {
		hipStream_t s = (hipStream_t)stream;
		const size_t tb_ = scan_temp_bytes(std::max(1u, n));
		ScanTemp tmp; tmp.alloc(tb_ + 256); scan_temp_reset(s, tmp.p);
		for (int r = 0; r < std::max(1, reps); ++r) launch_exclusive_scan(s, tmp.p, tb_, in, out, n);
		HIP_CHECK(hipStreamSynchronize(s));
		if (failures) *failures = scan_failures(tmp.p);
	});
}
int neus_testbed_stream(NeusTestbed* tb, void** s) { return guard([&] { *s = (void*)tb->stream; }); }
int neus_testbed_synchronize(NeusTestbed* tb) { return guard([&] { HIP_CHECK(hipStreamSynchronize(tb->stream)); }); }
int neus_testbed_set_profiling(NeusTestbed* tb, int on) {
	return guard([&] {
		tb->flush_phases();
		tb->profiling = on != 0;
		for (auto& m : tb->phase_ms) m = 0;
		tb->phase_steps = 0; tb->phase_npre = tb->phase_ntrain = 0;
	});
}
int neus_testbed_set_infer_timing(NeusTestbed* tb, int on) {
	return guard([&] {
		tb->infer_timing = on != 0;
		tb->it_n = 0; tb->it_ms = 0.0; tb->it_launches = 0; tb->it_steps = 0;
	});
}
int neus_testbed_infer_timing(NeusTestbed* tb, double* ms_total, uint64_t* launches, uint64_t* steps) {
	return guard([&] {
		if (ms_total) *ms_total = tb->it_ms;
		if (launches) *launches = tb->it_launches;
		if (steps) *steps = tb->it_steps;
	});
}
int neus_testbed_set_exchange_timing(NeusTestbed* tb, int on) {
	return guard([&] {
		tb->xt_collect_all();
		tb->xt_on = on != 0;
		tb->xt_exposed_ms = tb->xt_span_ms = 0.0; tb->xt_steps = 0;
	});
}
int neus_testbed_exchange_timing(NeusTestbed* tb, double* exposed_ms_total, double* span_ms_total, uint64_t* steps) {
	return guard([&] {
		HIP_CHECK(hipSetDevice(tb->device));
		tb->xt_collect_all();
		if (exposed_ms_total) *exposed_ms_total = tb->xt_exposed_ms;
		if (span_ms_total) *span_ms_total = tb->xt_span_ms;
		if (steps) *steps = tb->xt_steps;
	});
}
int neus_testbed_kernel_times(NeusTestbed* tb, float* ms) {
	return guard([&] {
		tb->flush_phases();
		for (int i = 0; i < NeusTestbed::N_PHASES; ++i) ms[i] = tb->phase_steps ? (float)(tb->phase_ms[i] / tb->phase_steps) : 0.f;
		ms[NeusTestbed::N_PHASES] = (float)tb->phase_steps;
		ms[NeusTestbed::N_PHASES + 1] = tb->phase_steps ? (float)(tb->phase_npre / tb->phase_steps) : 0.f;
		ms[NeusTestbed::N_PHASES + 2] = tb->phase_steps ? (float)(tb->phase_ntrain / tb->phase_steps) : 0.f;
	});
}

int neus_nccl_unique_id(uint8_t* out) {
	return guard([&] {
		ncclUniqueId id;
		NCCL_CHECK(ncclGetUniqueId(&id));
		static_assert(sizeof(id) == 128, "ncclUniqueId size");
		std::memcpy(out, &id, 128);
	});
}
int neus_testbed_init_data_parallel_ex(NeusTestbed* tb, int rank, int world, const uint8_t* uid, uint32_t flags) {
	return guard([&] {
		if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("invalid rank/world");
		if (tb->comm || tb->group || tb->hgroup) throw std::runtime_error("init_data_parallel: the testbed already has a communicator");
		HIP_CHECK(hipSetDevice(tb->device));
		tb->rank = (uint32_t)rank; tb->world = (uint32_t)world;
		tb->force_coll = (flags & NEUS_DP_FORCE_COLLECTIVES) != 0;
		tb->overlap_verified = false;
		tb->tbuf.indeed_batch = (float)tb->batch * (float)world;
		tb->coll_calls = tb->coll_bytes = tb->coll_bytes_step = 0;
		if (world > 1 || tb->force_coll) {
			if (!uid) throw std::runtime_error("init_data_parallel: no unique id");
			ncclUniqueId id;
			std::memcpy(&id, uid, 128);
			NCCL_CHECK(ncclCommInitRank(&tb->comm, world, id, rank));
		}
	});
}
int neus_testbed_set_exchange_overlap(NeusTestbed* tb, int on) {
	return guard([&] {
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		tb->exchange_overlap = on != 0;
		tb->overlap_verified = false;
	});
}
int neus_testbed_init_data_parallel(NeusTestbed* tb, int rank, int world, const uint8_t* uid) {
	return neus_testbed_init_data_parallel_ex(tb, rank, world, uid, 0u);
}
int neus_testbed_data_parallel_info(NeusTestbed* tb, NeusDataParallelInfo* o) {
	return guard([&] {
		o->rank = tb->rank; o->world = tb->world;
		o->has_communicator = tb->comm ? 1u : 0u; o->local_group = tb->group ? 1u : 0u; o->host_group = tb->hgroup ? 1u : 0u;
		o->collective_calls = tb->coll_calls; o->allreduce_bytes = tb->coll_bytes; o->last_step_allreduce_bytes = tb->coll_bytes_step;
	});
}

int neus_local_group_create(int world, NeusLocalGroup** out) {
	return guard([&] {
		if (world < 1 || world > 64) throw std::runtime_error("local group: world must be 1..64");
		*out = new NeusLocalGroup((uint32_t)world);
	});
}
int neus_local_group_destroy(NeusLocalGroup* g) { return guard([&] { delete g; }); }
int neus_testbed_init_local_group(NeusTestbed* tb, NeusLocalGroup* g, int rank) {
	return guard([&] {
		if (!g || rank < 0 || (uint32_t)rank >= g->world) throw std::runtime_error("invalid local group / rank");
		if (tb->comm) throw std::runtime_error("testbed already has an RCCL communicator");
		tb->group = g; tb->rank = (uint32_t)rank; tb->world = g->world;
		tb->tbuf.indeed_batch = (float)tb->batch * (float)tb->world;
		tb->overlap_verified = false;
	});
}

int neus_host_group_create(int rank, int world, const char* host, int port, uint64_t job_token, NeusHostGroup** out) {
	return guard([&] {
		if (world < 1 || world > 64 || rank < 0 || rank >= world) throw std::runtime_error("host group: world must be 1..64, 0 <= rank < world");
		if (port <= 0 || port > 65535) throw std::runtime_error("host group: invalid port");
		*out = new NeusHostGroup(rank, world, host ? host : "127.0.0.1", port, job_token);
	});
}
int neus_host_group_destroy(NeusHostGroup* g) { return guard([&] { delete g; }); }
int neus_debug_host_group_allreduce(NeusHostGroup* g, void* host, uint64_t n, int type, int op) {
	return guard([&] {
		if (!g) throw std::runtime_error("invalid host group");
		g->allreduce_host(host, (size_t)n * 4, type ? NeusHostGroup::U32 : NeusHostGroup::F32, op ? NeusHostGroup::MAX : NeusHostGroup::SUM);
		g->check();
	});
}
int neus_testbed_init_host_group(NeusTestbed* tb, NeusHostGroup* g) {
	return guard([&] {
		if (!g) throw std::runtime_error("invalid host group");
		if (tb->comm || tb->group || tb->hgroup) throw std::runtime_error("init_host_group: the testbed already has a communicator");
		HIP_CHECK(hipSetDevice(tb->device));
		tb->hgroup = g; tb->rank = (uint32_t)g->rank; tb->world = (uint32_t)g->world;
		tb->tbuf.indeed_batch = (float)tb->batch * (float)tb->world;
		tb->coll_calls = tb->coll_bytes = tb->coll_bytes_step = 0;
		tb->overlap_verified = false;
	});
}

// ------------------------------------------------------------ operator surface
int neus_grid_encode(NeusTestbed* tb, void* stream, uint32_t n, uint32_t ld, const float* coords, uint32_t stride, uint32_t valid,
                     uint16_t* enc, float* dydx) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, 4096));
		launch_grid_encode(as_stream(tb, stream), nullptr, n, ld, coords, stride, tb->gl, valid, tb->params_h.p + tb->lay.grid_off,
		                   (uint32_t*)enc, dydx, gx);
		HIP_CHECK(hipGetLastError());
	});
}
int neus_net_forward(NeusTestbed* tb, void* stream, uint32_t n, const float* coords, uint32_t valid, uint16_t* out) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		tb->net_forward(nullptr, n, n, coords, valid, (half_t*)out, as_stream(tb, stream));
		HIP_CHECK(hipGetLastError());
	});
}
int neus_net_backward(NeusTestbed* tb, void* stream, uint32_t n, const float* coords, uint32_t valid, const uint16_t* dlo,
                      uint32_t indeed, float* grads_out) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		if (n == 0 || n % 128 != 0) throw std::runtime_error("neus_net_backward: batch must be a positive multiple of 128 (fully_fused_mlp.cu:779-781)");
		if (n > tb->batch) throw std::runtime_error("neus_net_backward: n exceeds batch_size");
		hipStream_t s = as_stream(tb, stream);
		HIP_CHECK(hipMemsetAsync(grads_out, 0, (size_t)tb->lay.P * 4, s));
		const float saved = tb->tbuf.indeed_batch;
		tb->tbuf.indeed_batch = (float)indeed;
		tb->net_backward(nullptr, nullptr, n, coords, valid, (const half_t*)dlo, grads_out, s);
		tb->tbuf.indeed_batch = saved;
		HIP_CHECK(hipGetLastError());
	});
}
int neus_net_backward_pos(NeusTestbed* tb, void* stream, uint32_t n, const float* coords, uint32_t valid, const uint16_t* dlo,
                          uint32_t indeed, float* grads_out, float* dpos) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		if (n == 0 || n % 128 != 0) throw std::runtime_error("neus_net_backward_pos: batch must be a positive multiple of 128");
		if (n > tb->batch) throw std::runtime_error("neus_net_backward_pos: n exceeds batch_size");
		hipStream_t s = as_stream(tb, stream);
		HIP_CHECK(hipMemsetAsync(grads_out, 0, (size_t)tb->lay.P * 4, s));
		const float saved = tb->tbuf.indeed_batch;
		tb->tbuf.indeed_batch = (float)indeed;
		tb->tbuf.dpos = (float4*)dpos;
		tb->net_backward(nullptr, nullptr, n, coords, valid, (const half_t*)dlo, grads_out, s);
		tb->tbuf.dpos = nullptr;
		tb->tbuf.indeed_batch = saved;
		HIP_CHECK(hipGetLastError());
	});
}
int neus_delta_apply(NeusTestbed* tb, void* stream, uint32_t n, uint32_t stride, const float* in, float* out) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		if (stride != 3 && stride != COORD_W) throw std::runtime_error("neus_delta_apply: stride must be 3 or 7");
		hipStream_t s = as_stream(tb, stream);
		launch_delta_prepare(s, tb->delta.p);
		launch_delta_apply(s, nullptr, n, stride, in, out, tb->delta.p);
		HIP_CHECK(hipGetLastError());
	});
}
int neus_delta_backward(NeusTestbed* tb, void* stream, uint32_t n, uint32_t stride, const float* coords, const float* dpos, float* grads12) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		hipStream_t s = as_stream(tb, stream);
		launch_delta_prepare(s, tb->delta.p);
		DeltaAdam a{0.f, 0.f, 0.f, 0.f, LOSS_SCALE, 0u};
		launch_delta_backward(s, nullptr, n, coords, stride, (const float4*)dpos, tb->delta.p, tb->delta_partial.p, a);
		DeltaState h{};
		HIP_CHECK(hipMemcpyAsync(&h, tb->delta.p, sizeof(h), hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		std::memcpy(grads12, h.grad, DELTA_PARAMS * 4);
	});
}
static void sample_rays_impl(NeusTestbed* tb, void* stream, uint32_t n_rays, uint32_t rank, uint32_t world, uint32_t n_rays_total,
                             uint64_t rng_state, uint64_t rng_inc, uint32_t max_samples, const uint8_t* bitfield, float* rays, uint32_t* numsteps,
                             float* coords, uint32_t* counters_out, uint32_t e1, uint32_t* list, uint32_t* list_len, uint32_t lds_fill);
int neus_sample_rays(NeusTestbed* tb, void* stream, uint32_t n_rays, uint32_t rank, uint32_t world, uint32_t n_rays_total,
                     uint64_t rng_state, uint64_t rng_inc, uint32_t max_samples, const uint8_t* bitfield, float* rays, uint32_t* numsteps,
                     float* coords, uint32_t* counters_out) {
	return guard([&] {
		sample_rays_impl(tb, stream, n_rays, rank, world, n_rays_total, rng_state, rng_inc, max_samples, bitfield, rays, numsteps, coords, counters_out,
		                 0u, nullptr, nullptr, 0u);
	});
}
int neus_debug_sample_rays_round0(NeusTestbed* tb, void* stream, uint32_t n_rays, uint32_t n_rays_total, uint64_t rng_state, uint64_t rng_inc,
                                  uint32_t max_samples, const uint8_t* bitfield, float* rays, uint32_t* numsteps, float* coords, uint32_t* counters_out,
                                  uint32_t chunk_end, uint32_t* list, uint32_t* list_len, uint32_t lds_fill) {
	return guard([&] {
		if (chunk_end == 0 || !list || !list_len) throw std::runtime_error("sample_rays_round0: chunk_end > 0, list and list_len required");
		sample_rays_impl(tb, stream, n_rays, 0u, 1u, n_rays_total, rng_state, rng_inc, max_samples, bitfield, rays, numsteps, coords, counters_out,
		                 chunk_end, list, list_len, lds_fill);
	});
}
int neus_debug_scan_giveup(void* stream, const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* failures) {
	return guard([&] {
		hipStream_t s = (hipStream_t)stream;
		ScanTemp tmp; tmp.alloc(scan_temp_bytes(n) + 256); scan_temp_reset(s, tmp.p);
		debug_scan_skip_first_tile(s, tmp.p, in, out, n);
		HIP_CHECK(hipStreamSynchronize(s));
		*failures = scan_failures(tmp.p);
	});
}
int neus_debug_set_lds_fill(NeusTestbed* tb, uint32_t pattern) { return guard([&] { tb->dbg_lds_fill = pattern; }); }
int neus_debug_set_lds_fill_all(NeusTestbed* tb, uint32_t pattern) { return guard([&] { tb->dbg_lds_fill_all = pattern; }); }
int neus_debug_set_xcd_shift(NeusTestbed* tb, uint32_t n_blocks) { return guard([&] { tb->dbg_xcd_shift = n_blocks; }); }
// Diagnostic: `launches` launches of the fp32-denormal probe on a stream of its own (device `device`), each compared with
// the CPU's bits; stats as debug_denorm_probe (march.hip)
int neus_debug_denorm_probe(int device, uint32_t n, uint32_t launches, uint64_t* stats) {
	return guard([&] {
		if (!stats || n == 0) throw std::runtime_error("neus_debug_denorm_probe: bad argument");
		HIP_CHECK(hipSetDevice(device));
		hipStream_t s = nullptr;
		HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
		try { debug_denorm_probe(s, n, launches, stats); } catch (...) { (void)hipStreamDestroy(s); throw; }
		HIP_CHECK(hipStreamDestroy(s));
	});
}
// Development: raw bytes of one step-workspace buffer (ids: 0 sa, 1 ekt, 2 ck4, 3 cke, 4 racc, 5 rgr, 6 rT, 7 rek,
// 8 ccount, 9 net_out, 10 coords, 11 base, 12 numsteps, 13 cmap, 14 nreq)
int neus_debug_get_buffer(NeusTestbed* tb, int id, uint64_t offset, uint64_t nbytes, void* host) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		const void* p = nullptr;
		size_t cap = 0;
		auto pick = [&](const void* q, size_t bytes) { p = q; cap = bytes; };
		switch (id) {
		case 0: pick(tb->l_sa.p, tb->l_sa.n * 16); break;
		case 1: pick(tb->l_ekt.p, tb->l_ekt.n * 4); break;
		case 2: pick(tb->l_ck4.p, tb->l_ck4.n * 16); break;
		case 3: pick(tb->l_cke.p, tb->l_cke.n * 4); break;
		case 4: pick(tb->l_racc.p, tb->l_racc.n * 16); break;
		case 5: pick(tb->l_rgr.p, tb->l_rgr.n * 16); break;
		case 6: pick(tb->l_rT.p, tb->l_rT.n * 4); break;
		case 7: pick(tb->l_rek.p, tb->l_rek.n * 4); break;
		case 8: pick(tb->ccount.p, tb->ccount.n * 4); break;
		case 9: pick(tb->net_out.p, tb->net_out.n * 2); break;
		case 10: pick(tb->coords.p, tb->coords.n * 4); break;
		case 11: pick(tb->base.p, tb->base.n * 4); break;
		case 12: pick(tb->numsteps.p, tb->numsteps.n * 4); break;
		case 13: pick(tb->cmap.p, tb->cmap.n * 4); break;
		case 14: pick(tb->nreq.p, tb->nreq.n * 4); break;
		case 15: pick(tb->dbg_dl.p, tb->dbg_dl.n * 2); break;
		case 20: case 21: case 22: case 23: case 24: case 25: case 26: case 27: case 28: case 29: case 30: case 31: case 32: case 33: case 34:
			pick(tb->dbg_snap[id - 20].p, tb->dbg_snap[id - 20].n); break;
		default: throw std::runtime_error("debug_get_buffer: unknown id");
		}
		if (offset + nbytes > cap) throw std::runtime_error("debug_get_buffer: range past the buffer");
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		HIP_CHECK(hipMemcpy(host, (const char*)p + offset, nbytes, hipMemcpyDeviceToHost));
	});
}
// Development: k_loss_grad replayed on the last step's state (same inputs as the step's launch) into separate outputs;
// dl_dout_out: batch x 16 fp16 bits (host). Valid after a static-scene step at the default options.
int neus_debug_replay_loss_grad(NeusTestbed* tb, uint16_t* dl_dout_out) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		NeusTestbed& t = *tb;
		hipStream_t s = t.stream;
		LossParams lp{};
		lp.loss_scale = LOSS_SCALE; lp.ek_w = t.cfg.ek_loss_weight; lp.mask_w = t.cfg.mask_loss_weight;
		// the cos-anneal of the step that ran (training_step was incremented after it)
		const int ts = (int)t.training_step - 1;
		lp.cos_anneal = t.cfg.anneal_end == 0 ? 1.0f : std::min(1.0f, (float)std::max(ts, 0) / t.cfg.anneal_end);
		lp.max_compacted = t.batch;
		const LossWork w = t.loss_work(t.base.p);
		Dev<float> co; co.alloc((size_t)t.batch * COORD_W);
		Dev<half_t> dl; dl.alloc((size_t)t.batch * OUT_W);
		HIP_CHECK(hipMemsetAsync(dl.p, 0, dl.n * 2, s));
		launch_loss_grad(s, t.max_samples, t.st.p, DPInfo{t.rank, t.world}, lp, t.coords.p, t.net_out.p, t.numsteps.p, w, co.p, dl.p);
		HIP_CHECK(hipStreamSynchronize(s));
		HIP_CHECK(hipMemcpy(dl_dout_out, dl.p, dl.n * 2, hipMemcpyDeviceToHost));
	});
}
int neus_debug_get_batch(NeusTestbed* tb, float* coords_out, uint16_t* dl_dout_out, float* loss_out) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		if (coords_out) HIP_CHECK(hipMemcpy(coords_out, tb->coords_c.p, (size_t)tb->batch * COORD_W * 4, hipMemcpyDeviceToHost));
		if (dl_dout_out) HIP_CHECK(hipMemcpy(dl_dout_out, tb->dL_dout.p, (size_t)tb->batch * OUT_W * 2, hipMemcpyDeviceToHost));
		if (loss_out) HIP_CHECK(hipMemcpy(loss_out, tb->loss.p, (size_t)MAX_RAYS * 4, hipMemcpyDeviceToHost));
	});
}
int neus_debug_inject_health(NeusTestbed* tb, uint32_t flags) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		HIP_CHECK(hipStreamSynchronize(tb->stream));
		if (flags & STEP_FAIL_MARCH_T) {
			StepState h{};
			HIP_CHECK(hipMemcpy(&h, tb->st.p, sizeof(h), hipMemcpyDeviceToHost));
			h.fail_flags |= STEP_FAIL_MARCH_T;
			HIP_CHECK(hipMemcpy(tb->st.p, &h, sizeof(h), hipMemcpyHostToDevice));
		}
		if (flags & STEP_FAIL_SCAN) {
			const uint32_t one = 1;
			HIP_CHECK(hipMemcpy(tb->scan_tmp.p + offsetof(ScanState, fail), &one, 4, hipMemcpyHostToDevice));
		}
	});
}
static void sample_rays_impl(NeusTestbed* tb, void* stream, uint32_t n_rays, uint32_t rank, uint32_t world, uint32_t n_rays_total,
                             uint64_t rng_state, uint64_t rng_inc, uint32_t max_samples, const uint8_t* bitfield, float* rays, uint32_t* numsteps,
                             float* coords, uint32_t* counters_out, uint32_t e1, uint32_t* list, uint32_t* list_len, uint32_t lds_fill) {
	{
		if (!tb->have_data || !tb->have_net) throw std::runtime_error("no dataset/network");
		if (n_rays == 0 || n_rays > MAX_RAYS) throw std::runtime_error("n_rays out of range");
		hipStream_t s = as_stream(tb, stream);
		Dev<StepState> sst; sst.alloc(1);
		StepState h{}; h.rays_per_batch = n_rays; h.max_inference = max_samples; h.n_rays_total = n_rays_total;
		HIP_CHECK(hipMemcpyAsync(sst.p, &h, sizeof(h), hipMemcpyHostToDevice, s));
		Dev<float> st_t; st_t.alloc(n_rays); Dev<uint32_t> nr, bs, nrec, q; nr.alloc(n_rays); bs.alloc(n_rays); nrec.alloc(n_rays); q.alloc(2);
		Dev<uint2> rec; rec.alloc((size_t)n_rays * NERF_STEPS);
		Dev<uint2> seg; seg.alloc((size_t)n_rays * MARCH_SEG_RECS);
		MarchWork mw{rec.p, nrec.p, q.p, tb->mwork.waves, seg.p, tb->mwork.lanes_per_ray};
		mw.balanced = tb->mwork.balanced;
		ScanTemp tmp; const size_t tb_ = scan_temp_bytes(n_rays); tmp.alloc(tb_ + 256); scan_temp_reset(s, tmp.p);
		Dev<uint32_t> lin; lin.alloc(LIN_WORDS);
		launch_bitfield_linear(s, bitfield, lin.p);
		// the occupied-box cull of the training step, from this bitfield (exact: culled rays march to zero samples)
		Dev<float> bb; bb.alloc(occ_bbox_scratch_floats());
		launch_occ_bbox(s, bitfield, bb.p);
		// progressive round 0's list (the training step's, written by the march): its slots and counters
		Dev<uint32_t> c0, cnt;
		if (list) { c0.alloc(n_rays); cnt.alloc(2); }
		const Round0List r0{e1, c0.p, list, cnt.p, 2u};
		launch_march_count(s, n_rays, max_samples, sst.p, DPInfo{rank, world}, tb->ds, bitfield, lin.p, rng_state, rng_inc, rays, st_t.p, nr.p, mw,
		                   list ? cnt.p : nullptr, list ? 2u : 0u, tb->ray_cull ? bb.p : nullptr);
		Dev<uint32_t> sr; sr.alloc(std::max<uint32_t>(1, max_samples));
		launch_march_write(s, n_rays, sst.p, tb->ds, rays, mw, nr.p, bs.p, numsteps, coords, sr.p, max_samples, tmp.p, list ? &r0 : nullptr, lds_fill);
		HIP_CHECK(hipMemcpyAsync(&h, sst.p, sizeof(h), hipMemcpyDeviceToHost, s));
		if (list) HIP_CHECK(hipMemcpyAsync(list_len, cnt.p, 4, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		if (h.fail_flags) throw std::runtime_error("sample_rays: the march met a non-finite or negative t");
		if (scan_failures(tmp.p)) throw std::runtime_error("sample_rays: the look-back scan gave up");
		counters_out[0] = h.numsteps_counter; counters_out[1] = h.n_kept; counters_out[2] = h.n_rays_with_samples;
	}
}
int neus_loss_compact(NeusTestbed* tb, void* stream, uint32_t n_rays, uint32_t rank, uint32_t world, uint32_t n_rays_total,
                      uint64_t rng_state, uint64_t rng_inc, uint32_t max_compacted, const float* rays, uint32_t* numsteps,
                      const float* coords, const uint16_t* net_out, float* coords_out, uint16_t* dlo, float* loss, float* ek,
                      float* mask, uint32_t* counters_out) {
	return guard([&] {
		if (!tb->have_data || !tb->have_net) throw std::runtime_error("no dataset/network");
		if (n_rays == 0 || n_rays > MAX_RAYS) throw std::runtime_error("n_rays out of range");
		hipStream_t s = as_stream(tb, stream);
		// sample count of the caller's layout (operator path only; the training step keeps it on the device)
		std::vector<uint32_t> hn(2 * (size_t)n_rays);
		HIP_CHECK(hipMemcpyAsync(hn.data(), numsteps, hn.size() * 4, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		uint32_t n_samples = 1;
		for (uint32_t i = 0; i < n_rays; ++i) if (hn[2 * i]) n_samples = std::max(n_samples, hn[2 * i] + hn[2 * i + 1]);
		Dev<StepState> sst; sst.alloc(1);
		StepState h{}; h.rays_per_batch = n_rays; h.n_rays_total = n_rays_total;
		HIP_CHECK(hipMemcpyAsync(sst.p, &h, sizeof(h), hipMemcpyHostToDevice, s));
		Dev<uint32_t> cc, cb, rb, sr; cc.alloc(n_rays); cb.alloc(n_rays); rb.alloc(n_rays); sr.alloc(n_samples);
		Dev<float4> sa, ck4, racc, rgr; sa.alloc(n_samples); ck4.alloc(n_samples / 8 + 1); racc.alloc(n_rays); rgr.alloc(n_rays);
		Dev<float> ekt, cke, rT; ekt.alloc(n_samples); cke.alloc(n_samples / 8 + 1); rT.alloc(n_rays);
		ScanTemp tmp; const size_t tb_ = scan_temp_bytes(n_rays); tmp.alloc(tb_ + 256); scan_temp_reset(s, tmp.p);
		LossParams lp{};
		lp.loss_scale = LOSS_SCALE; lp.ek_w = tb->cfg.ek_loss_weight; lp.mask_w = tb->cfg.mask_loss_weight; lp.cos_anneal = tb->cos_anneal();
		lp.max_compacted = max_compacted; lp.rng_state = rng_state; lp.rng_inc = rng_inc;
		LossWork w{};
		w.sa = sa.p; w.ck4 = ck4.p; w.cke = cke.p; w.ekt = ekt.p; w.sample_ray = sr.p; w.rbase = rb.p; w.racc = racc.p; w.rT = rT.p; w.rgr = rgr.p;
		Dev<uint32_t> cm; cm.alloc(std::max(1u, max_compacted)); w.cmap = cm.p;
		Dev<uint32_t> lr, nl; lr.alloc(n_rays); nl.alloc(1);
		w.long_rays = lr.p; w.n_long = nl.p;
		const DPInfo dp{rank, world};
		launch_ray_index(s, n_rays, numsteps, sst.p, sr.p, rb.p);
		launch_loss_alpha(s, n_samples, sst.p, coords, (const half_t*)net_out, lp.cos_anneal, w);
		launch_loss_scan_ray(s, n_rays, numsteps, w, cc.p);
		launch_exclusive_scan(s, tmp.p, tb_, cc.p, cb.p, n_rays);
		launch_loss_ray(s, n_rays, sst.p, dp, tb->ds, lp, numsteps, cc.p, cb.p, w, loss, ek, mask);
		launch_loss_grad(s, n_samples, sst.p, dp, lp, coords, (const half_t*)net_out, numsteps, w, coords_out, (half_t*)dlo);
		HIP_CHECK(hipMemcpyAsync(&h, sst.p, sizeof(h), hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		counters_out[0] = h.compacted_counter;
	});
}
int neus_optimizer_step(NeusTestbed* tb, void* stream, const float* grads) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		if (stream && (hipStream_t)stream != tb->stream) HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
		tb->optimizer_step(grads);
		HIP_CHECK(hipStreamSynchronize(tb->stream));
	});
}
int neus_fill_rollover(NeusTestbed* tb, void* stream, uint32_t n_elements, uint32_t n_in, float* coords, uint16_t* dL_dout) {
	return guard([&] {
		if (!tb) throw std::runtime_error("fill_rollover: null testbed");
		hipStream_t s = as_stream(tb, stream);
		Dev<StepState> sst; sst.alloc(1);
		StepState h{}; h.compacted_counter = n_in;
		HIP_CHECK(hipMemcpyAsync(sst.p, &h, sizeof(h), hipMemcpyHostToDevice, s));
		launch_rollover(s, n_elements, sst.p, coords, (half_t*)dL_dout);
		HIP_CHECK(hipStreamSynchronize(s));
	});
}
int neus_occ_update(NeusTestbed* tb, void* stream, uint32_t n_uniform, uint32_t n_nonuniform) {
	return guard([&] {
		if (!tb->have_net) throw std::runtime_error("no network");
		(void)stream;
		tb->occ_update(n_uniform, n_nonuniform, tb->valid_level_at((int)tb->training_step));
		HIP_CHECK(hipStreamSynchronize(tb->stream));
	});
}
int neus_mfma_probe(const uint16_t* A, const uint16_t* B, float* C) {
	return guard([&] {
		launch_mfma_probe(nullptr, (const half_t*)A, (const half_t*)B, C);
		HIP_CHECK(hipDeviceSynchronize());
	});
}

} // extern "C"

// ============================================================ tcnn-shaped operator modules (cpp_api.h:66-110)
// A module owns a private NeusTestbed core holding only the network half (setup_network): grid tables, parameter
// layout, the fp16 / transposed weight copies the kernels read and one batch of forward / backward workspace. The
// parameters come in through the explicit `params` pointer of every call (copied into the core's fp16 buffer and
// re-prepared), as tcnn::cpp::Module does; gradients leave through dL_dparams with EGradientMode semantics
// (object.h:90-94). Kinds: the NeuS NerfNetwork (nerf_network.h: encoding + density MLP + rgb MLP + variance,
// input NerfCoordinate [n][7] f32, output [n][16] fp16) and the HashGrid encoding (grid.h, input [n][3] f32, output
// [L][n] half2 = features 2l, 2l+1 of level l adjacent).
namespace {

std::string fmt_float(float v) { char b[32]; std::snprintf(b, sizeof(b), "%.9g", (double)v); return b; }
// `standalone`: a HashGrid module (create_encoding): tcnn's defaults for the keys a config omits
// (create_grid_encoding_templated, grid.h:2499-2525); otherwise the NeuS Testbed's (testbed.cu:2175-2187, base.json)
NeusNetworkConfig module_config(const JsonValue& enc, const JsonValue& net, const JsonValue& rgb, uint32_t batch, bool standalone = false) {
	NeusNetworkConfig c{};
	const uint32_t nf = (uint32_t)enc.number("n_features_per_level", 2);
	c.n_levels = enc.number("n_features", 0) > 0 ? (uint32_t)enc.number("n_features", 0) / nf : (uint32_t)enc.number("n_levels", 16);
	c.n_features_per_level = nf;
	c.log2_hashmap_size = (uint32_t)enc.number("log2_hashmap_size", standalone ? 19 : 15);
	c.base_resolution = (uint32_t)enc.number("base_resolution", standalone ? 16 : 0);
	if (!c.base_resolution) c.base_resolution = 1u << (c.log2_hashmap_size / 3);
	c.per_level_scale = (float)enc.number("per_level_scale", standalone ? 2.0 : 0.0);
	c.top_resolution = (float)enc.number("top_resolution", 2048.0);
	c.valid_level_scale = (float)enc.number("valid_level_scale", standalone ? 0.01 : 0.02);
	c.base_valid_level_scale = (float)enc.number("base_valid_level_scale", standalone ? 0.5 : 0.2);
	c.base_training_step = (uint32_t)enc.number("base_training_step", standalone ? 200 : 100);
	c.n_neurons = (uint32_t)net.number("n_neurons", 64);
	if ((uint32_t)rgb.number("n_neurons", c.n_neurons) != c.n_neurons) throw std::runtime_error("density and rgb networks must share n_neurons");
	c.n_density_hidden = (uint32_t)net.number("n_hidden_layers", 1);
	c.n_rgb_hidden = (uint32_t)rgb.number("n_hidden_layers", 2);
	c.batch_size = batch;
	c.sdf_bias = -0.1f;
	c.seed = 1337;
	return c;
}

struct StreamSwap {  // run a call's launches on the caller's stream (NULL: the null stream, as tcnn's cudaStream_t 0)
	NeusTestbed& t; hipStream_t saved;
	StreamSwap(NeusTestbed& tb, void* s) : t(tb), saved(tb.stream) { t.stream = (hipStream_t)s; }
	~StreamSwap() { t.stream = saved; }
};

}  // namespace

struct NeusContext {
	uint32_t n = 0;
	Dev<float> dydx;     // encoding: dy/dx [6L][n] of the forward (prepare_input_gradients)
	Dev<uint32_t> enc;   // network with input encoding: the forward's paired encoding [L][n] (the MLP input)
	Dev<half_t> acts;    // FullyFusedMLP: the forward's input X0 [n][in_pad] and hidden outputs [N][n][W] (post-activation)
};

// tcnn FullyFusedMLP shape (fully_fused_mlp.cu:816-879): weight matrices [W][in_pad], (N - 1) x [W][W], [out_pad][W]
struct FfNet {
	uint32_t W = 0, N = 0, n_in = 0, in_pad = 0, n_out = 0, out_pad = 0, act = FF_RELU, out_act = FF_NONE;
	float in_scale = 1.f, in_offset = 0.f;  // the Identity encoding's scale / offset (identity.h:44-70)
	std::vector<uint32_t> off, rows, cols;
	uint32_t P = 0;
	void build() {
		off.clear(); rows.clear(); cols.clear(); P = 0;
		for (uint32_t l = 0; l <= N; ++l) {
			const uint32_t r = l == N ? out_pad : W, c = l == 0 ? in_pad : W;
			off.push_back(P); rows.push_back(r); cols.push_back(c); P += r * c;
		}
	}
	size_t acts_halves(uint32_t n) const { return (size_t)n * (in_pad + (size_t)N * W); }
	static uint32_t activation(const std::string& s) {
		if (s == "None") return FF_NONE;
		if (s == "ReLU") return FF_RELU;
		if (s == "Exponential") return FF_EXP;
		if (s == "Sigmoid") return FF_SIGMOID;
		if (s == "Squareplus") return FF_SQUAREPLUS;
		if (s == "Softplus") return FF_SOFTPLUS;
		throw std::runtime_error("FullyFusedMLP: activation '" + s + "' is not supported on gfx950 (None, ReLU, Exponential, Sigmoid, Squareplus, "
		                         "Softplus; Sine has no backward in tcnn's fully fused MLP)");
	}
};

struct NeusModule {
	// Network: the NeuS NerfNetwork; Encoding: a HashGrid; DensityNet: tcnn's NetworkWithInputEncoding(HashGrid ->
	// FullyFusedMLP with 1 hidden ReLU layer -> 16 linear outputs), the network whose backward_backward_input tcnn
	// implements (network_with_input_encoding.h:159-250, fully_fused_mlp.cu:1088-1198)
	// Mlp: tcnn::cpp::create_network = NetworkWithInputEncoding(Identity -> FullyFusedMLP) (cpp_api.cu:170-172), ffmlp.hip
	// GridMlp: NetworkWithInputEncoding(HashGrid -> any FullyFusedMLP), composed of the encoding kernels and ffmlp.hip's layers
	enum Kind { Network = 0, Encoding = 1, DensityNet = 2, Mlp = 3, GridMlp = 4 } kind;
	FfNet ff;
	Dev<half_t> ff_acts, ff_front, ff_d[2];  // Mlp: inference activations, backward-backward fronts, delta ping-pong
	Dev<float> ff_partial, ff_dummy;         // Mlp: per-block weight-gradient rows
	uint32_t n_mlp = 0, dn_width = 0, dn_de = 0;  // DensityNet: MLP parameters W DE + 16 W ahead of the grid, width, padded input
	Dev<uint32_t> u_tmp;                          // DensityNet: dy/dx . dL_ddLdinput, paired
	Dev<float> dn_partial, dn_dummy;              // DensityNet: per-block weight-gradient rows
	NeusTestbed core;
	uint32_t capacity = 0, n_in = 0, n_out = 0;
	int training_step = 0;              // GridEncoding::set_training_step (grid.h:2427-2437): 0 = every level
	uint32_t indeed_batch = 0;          // NeuS backward normalisation of the eikonal entries; 0 = the call's n
	std::string hyper;
	// encoding output layout (ENC_LAYOUT_*): AoS [n][2L] = the column-major matrix tcnn's cpp::Module wraps around the
	// caller's buffer (cpp_api.cu:58-70); SoA [2L][n] = GridEncoding::preferred_output_layout (grid.h:2357-2359);
	// paired [L][n] half2 = this build's kernels
	uint32_t layout = ENC_LAYOUT_AOS;
	bool grad_fp16 = true;              // dL_dparams in param precision (fp16, trainer.h:72-109) or fp32
	bool f32 = false;                   // Encoding created with requested_precision fp32: float params / output / gradients
	Dev<uint32_t> enc_tmp, denc_tmp;    // paired-layout staging of non-paired module I/O
	Dev<float> gtmp;                    // gradients of an Accumulate call (and of every fp16-gradient call)
	Dev<float4> dpos, v4;
	Dev<half_t> zero_h;
	Dev<float4> zero_v;
	explicit NeusModule(int device) : core(device) {}
	uint64_t n_params() const {
		if (kind == Mlp) return ff.P;
		if (kind == GridMlp) return ff.P + core.lay.n_grid;
		return kind == Network ? core.lay.P : (kind == DensityNet ? n_mlp + core.lay.n_grid : core.lay.n_grid);
	}
	uint32_t valid() const { return core.valid_level_at(training_step); }
	void load_params(const void* params, hipStream_t s) {
		if (!params) throw std::runtime_error("module: null params");
		if (kind == Network) {
			HIP_CHECK(hipMemcpyAsync(core.params_h.p, params, (size_t)core.lay.P * 2, hipMemcpyDeviceToDevice, s));
			core.prepare_weights();
		} else {
			HIP_CHECK(hipMemcpyAsync(core.params_h.p + core.lay.grid_off, params, (size_t)core.lay.n_grid * 2, hipMemcpyDeviceToDevice, s));
		}
	}
	void check_n(uint32_t n, bool backward) const {
		if (n > capacity) throw std::runtime_error("module: n_elements exceeds the module's batch capacity");
		if (backward && kind == Network && (n == 0 || n % 128 != 0))
			throw std::runtime_error("module backward: n_elements must be a positive multiple of 128 (fully_fused_mlp.cu:779-781)");
		if ((kind == Mlp || kind == GridMlp) && n % 128 != 0) throw std::runtime_error("FullyFusedMLP: batch size must be a multiple of 128 (fully_fused_mlp.cu:779-781)");
	}
	// the destination of this call's parameter gradients (Overwrite: dL_dparams itself; Accumulate: a scratch buffer)
	float* grad_target(void* dL_dparams, int mode) {
		if (mode == NEUS_GRADIENT_IGNORE) return nullptr;
		if (!dL_dparams) throw std::runtime_error("module: dL_dparams is null with a gradient mode other than Ignore");
		if (mode != NEUS_GRADIENT_OVERWRITE && mode != NEUS_GRADIENT_ACCUMULATE) throw std::runtime_error("module: unknown gradient mode");
		if (mode == NEUS_GRADIENT_OVERWRITE && !grad_fp16) return (float*)dL_dparams;
		return gtmp.p;
	}
	void finish_grad(void* dL_dparams, int mode, hipStream_t s) {
		if (grad_fp16) launch_grad_to_half(s, (uint32_t)n_params(), gtmp.p, (half_t*)dL_dparams, mode == NEUS_GRADIENT_ACCUMULATE);
		else if (mode == NEUS_GRADIENT_ACCUMULATE) launch_add_f32(s, (uint32_t)n_params(), gtmp.p, (float*)dL_dparams);
	}
	// a caller-layout encoding tensor (dL_doutput) as the kernels' paired layout
	const half_t* paired_in(const void* x, uint32_t n, hipStream_t s) {
		if (layout == ENC_LAYOUT_PAIRED) return (const half_t*)x;
		launch_enc_from_layout(s, n, core.lay.L, (const half_t*)x, layout, denc_tmp.p);
		return (const half_t*)denc_tmp.p;
	}
};

// module options (this build's keys, beside tcnn's): "gradient_precision": "fp16" (default, tcnn's param precision) |
// "fp32"; encoding "output_layout": "AoS" (default: cpp::Module's column-major view) | "SoA" | "paired"
static void module_options(NeusModule* m, const JsonValue& j) {
	const std::string gp = j.string("gradient_precision", "fp16");
	if (gp != "fp16" && gp != "fp32") throw std::runtime_error("module: gradient_precision must be fp16 or fp32");
	m->grad_fp16 = gp == "fp16";
	const std::string ol = j.string("output_layout", "AoS");
	if (ol == "AoS") m->layout = ENC_LAYOUT_AOS;
	else if (ol == "SoA") m->layout = ENC_LAYOUT_SOA;
	else if (ol == "paired") m->layout = ENC_LAYOUT_PAIRED;
	else throw std::runtime_error("encoding module: output_layout must be AoS, SoA or paired");
}
static void module_common_init(NeusModule* m, uint32_t capacity) {
	m->capacity = capacity;
	const size_t P = m->n_params();
	m->gtmp.alloc(P);
	m->dpos.alloc(capacity); m->v4.alloc(capacity);
	m->zero_h.alloc((size_t)2 * m->core.lay.L * capacity); m->zero_v.alloc(capacity);
	if ((m->kind == NeusModule::Encoding && m->layout != ENC_LAYOUT_PAIRED) || m->kind == NeusModule::DensityNet || m->kind == NeusModule::GridMlp) {
		m->enc_tmp.alloc((size_t)m->core.lay.L * capacity); m->denc_tmp.alloc((size_t)m->core.lay.L * capacity);
	}
	if (m->kind == NeusModule::GridMlp) {
		const FfNet& f = m->ff;
		m->u_tmp.alloc((size_t)m->core.lay.L * capacity);
		m->ff_acts.alloc(f.acts_halves(capacity));
		m->ff_front.alloc((size_t)capacity * (f.in_pad + (size_t)f.N * f.W));
		const uint32_t dmax = std::max(std::max(f.W, f.out_pad), f.in_pad);
		m->ff_d[0].alloc((size_t)capacity * dmax); m->ff_d[1].alloc((size_t)capacity * dmax);
		m->ff_partial.alloc((size_t)ff_wgrad_blocks(capacity) * f.P);
		m->ff_dummy.alloc(4);
	}
	if (m->kind == NeusModule::DensityNet) {
		m->u_tmp.alloc((size_t)m->core.lay.L * capacity);
		m->dn_partial.alloc((size_t)dnet_blocks(capacity) * m->n_mlp);
		m->dn_dummy.alloc(4);
	}
	HIP_CHECK(hipMemset(m->zero_h.p, 0, m->zero_h.n * sizeof(half_t)));
	HIP_CHECK(hipMemset(m->zero_v.p, 0, m->zero_v.n * sizeof(float4)));
	HIP_CHECK(hipStreamSynchronize(m->core.stream));
}

int neus_module_create_nerf_network(const char* config_json, uint32_t batch_capacity, NeusModule** out) {
	return guard([&] {
		if (!config_json || !out) throw std::runtime_error("neus_module_create_nerf_network: null argument");
		if (batch_capacity == 0 || batch_capacity % 128 != 0 || batch_capacity > (1u << 24))
			throw std::runtime_error("batch_capacity must be a positive multiple of 128 (<= 2^24)");
		const JsonValue j = parse_json(config_json);
		int dev = 0;
		HIP_CHECK(hipGetDevice(&dev));
		auto m = std::make_unique<NeusModule>(dev);
		m->kind = NeusModule::Network;
		module_options(m.get(), j);
		m->layout = ENC_LAYOUT_AOS;
		m->core.setup_network(module_config(j.object("encoding"), j.object("network"), j.object("rgb_network"), batch_capacity), nullptr);
		m->n_in = COORD_W; m->n_out = OUT_W;
		const NeusNetworkConfig& c = m->core.cfg;
		m->hyper = "{\"otype\": \"NerfNetwork\", \"n_levels\": " + std::to_string(c.n_levels) + ", \"n_neurons\": " + std::to_string(c.n_neurons) +
		           ", \"log2_hashmap_size\": " + std::to_string(c.log2_hashmap_size) + ", \"per_level_scale\": " + fmt_float(c.per_level_scale) +
		           ", \"gradient_precision\": \"" + (m->grad_fp16 ? "fp16" : "fp32") + "\"}";
		module_common_init(m.get(), batch_capacity);
		*out = m.release();
	});
}

int neus_module_create_encoding(uint32_t n_input_dims, const char* encoding_json, int requested_precision, uint32_t batch_capacity,
                                NeusModule** out) {
	return guard([&] {
		if (!encoding_json || !out) throw std::runtime_error("neus_module_create_encoding: null argument");
		if (n_input_dims != 3) throw std::runtime_error("HashGrid module: n_input_dims must be 3");
		if (batch_capacity == 0 || batch_capacity % 128 != 0 || batch_capacity > (1u << 24))
			throw std::runtime_error("batch_capacity must be a positive multiple of 128 (<= 2^24)");
		const JsonValue j = parse_json(encoding_json);
		const std::string ot = j.string("otype", "HashGrid");
		if (ot != "HashGrid" && ot != "Grid") throw std::runtime_error("encoding module: only HashGrid is implemented on gfx950");
		int dev = 0;
		HIP_CHECK(hipGetDevice(&dev));
		auto m = std::make_unique<NeusModule>(dev);
		m->kind = NeusModule::Encoding;
		module_options(m.get(), j);
		// cpp_api.cu:174-180: Fp32 -> GridEncoding<float> (float params, output and gradients), Fp16 -> GridEncoding<__half>
		if (requested_precision != NEUS_PRECISION_FP32 && requested_precision != NEUS_PRECISION_FP16)
			throw std::runtime_error("create_encoding: requested_precision must be NEUS_PRECISION_FP32 or NEUS_PRECISION_FP16");
		m->f32 = requested_precision == NEUS_PRECISION_FP32;
		if (m->f32) {
			if (m->layout == ENC_LAYOUT_PAIRED) throw std::runtime_error("fp32 HashGrid: output_layout AoS or SoA (paired is the fp16 kernels' layout)");
			m->grad_fp16 = false;
		}
		JsonValue none; none.kind = JsonValue::Object;
		m->core.setup_network(module_config(j, none, none, batch_capacity, true), nullptr, false);
		m->n_in = 3; m->n_out = 2 * m->core.lay.L;
		const NeusNetworkConfig& c = m->core.cfg;
		static const char* lay_names[3] = {"AoS", "SoA", "paired"};
		m->hyper = "{\"otype\": \"HashGrid\", \"n_levels\": " + std::to_string(c.n_levels) + ", \"n_features_per_level\": 2, \"log2_hashmap_size\": " +
		           std::to_string(c.log2_hashmap_size) + ", \"base_resolution\": " + std::to_string(c.base_resolution) + ", \"per_level_scale\": " +
		           fmt_float(c.per_level_scale) + ", \"valid_level_scale\": " + fmt_float(c.valid_level_scale) + ", \"base_valid_level_scale\": " +
		           fmt_float(c.base_valid_level_scale) + ", \"base_training_step\": " + std::to_string(c.base_training_step) +
		           ", \"output_layout\": \"" + lay_names[m->layout] + "\", \"gradient_precision\": \"" + (m->grad_fp16 ? "fp16" : "fp32") +
		           "\", \"precision\": \"" + (m->f32 ? "fp32" : "fp16") + "\"}";
		module_common_init(m.get(), batch_capacity);
		*out = m.release();
	});
}

static std::string grid_hyper(const NeusNetworkConfig& c) {
	return "{\"otype\": \"HashGrid\", \"n_levels\": " + std::to_string(c.n_levels) + ", \"n_features_per_level\": 2, \"log2_hashmap_size\": " +
	       std::to_string(c.log2_hashmap_size) + ", \"base_resolution\": " + std::to_string(c.base_resolution) + ", \"per_level_scale\": " +
	       fmt_float(c.per_level_scale) + "}";
}
static FfNet ff_from_json(const JsonValue& j, uint32_t n_input_dims, uint32_t n_output_dims);
static std::string ff_hyper(const FfNet& f);
static NeusModule* make_mlp_module(const FfNet& f, const JsonValue& j, uint32_t batch_capacity);
// create_network_with_input_encoding (cpp_api.h:108; network_with_input_encoding.h): an Identity encoding (any input
// width; scale / offset) or a HashGrid (3 inputs) in front of a FullyFusedMLP of any depth, width 16 / 32 / 64 / 128 and
// activations. The HashGrid -> one hidden ReLU layer -> linear network of width 16 / 64 runs on the fused k_dnet kernel;
// every other HashGrid network is the encoding's kernels composed with ffmlp.hip's layers (GridMlp).
int neus_module_create_network_with_input_encoding(uint32_t n_input_dims, uint32_t n_output_dims, const char* encoding_json,
                                                   const char* network_json, uint32_t batch_capacity, NeusModule** out) {
	return guard([&] {
		if (!encoding_json || !network_json || !out) throw std::runtime_error("neus_module_create_network_with_input_encoding: null argument");
		if (batch_capacity == 0 || batch_capacity % 128 != 0 || batch_capacity > (1u << 24))
			throw std::runtime_error("batch_capacity must be a positive multiple of 128 (<= 2^24)");
		const JsonValue je = parse_json(encoding_json), jn = parse_json(network_json);
		const std::string ot = je.string("otype", "HashGrid");
		if (ot == "Identity") {
			FfNet f = ff_from_json(jn, n_input_dims, n_output_dims);
			f.in_scale = (float)je.number("scale", 1.0);
			f.in_offset = (float)je.number("offset", 0.0);
			*out = make_mlp_module(f, jn, batch_capacity);
			return;
		}
		if (ot != "HashGrid" && ot != "Grid") throw std::runtime_error("network with input encoding: the encoding must be Identity or HashGrid on gfx950");
		if (n_input_dims != 3) throw std::runtime_error("network with input encoding: a HashGrid encodes 3 input dims");
		int dev = 0;
		HIP_CHECK(hipGetDevice(&dev));
		auto m = std::make_unique<NeusModule>(dev);
		module_options(m.get(), jn);
		m->layout = ENC_LAYOUT_AOS;
		JsonValue none; none.kind = JsonValue::Object;
		m->core.setup_network(module_config(je, none, none, batch_capacity, true), nullptr, false);
		const uint32_t L = m->core.lay.L;
		const FfNet f = ff_from_json(jn, 2 * L, n_output_dims);
		const bool fused = f.act == FF_RELU && f.out_act == FF_NONE && f.N == 1 && n_output_dims <= 16 && dnet_supported(L, f.W);
		m->n_in = 3;
		if (fused) {
			m->kind = NeusModule::DensityNet;
			m->dn_width = f.W;
			m->dn_de = (2 * L + 15) / 16 * 16;
			m->n_mlp = m->dn_width * m->dn_de + 16 * m->dn_width;
			m->n_out = 16;
		} else {
			m->kind = NeusModule::GridMlp;
			m->ff = f;
			m->n_out = f.out_pad;
		}
		m->hyper = "{\"otype\": \"NetworkWithInputEncoding\", \"encoding\": " + grid_hyper(m->core.cfg) + ", \"network\": " + ff_hyper(f) +
		           ", \"n_output_dims\": " + std::to_string(n_output_dims) + ", \"gradient_precision\": \"" + (m->grad_fp16 ? "fp16" : "fp32") + "\"}";
		module_common_init(m.get(), batch_capacity);
		*out = m.release();
	});
}

// A FullyFusedMLP from its config (fully_fused_mlp.cu:816-879): n_neurons 16 / 32 / 64 / 128, n_hidden_layers >= 1, input and
// output padded to multiples of 16
static FfNet ff_from_json(const JsonValue& j, uint32_t n_input_dims, uint32_t n_output_dims) {
	const std::string ot = j.string("otype", "FullyFusedMLP");
	if (ot != "FullyFusedMLP" && ot != "MegakernelMLP" && ot != "CutlassMLP")
		throw std::runtime_error("only FullyFusedMLP networks are implemented on gfx950");
	FfNet f;
	f.W = (uint32_t)j.number("n_neurons", 64);
	if (f.W != 16 && f.W != 32 && f.W != 64 && f.W != 128)
		throw std::runtime_error("FullyFusedMLP only supports 16, 32, 64, and 128 neurons, but got " + std::to_string(f.W));
	const double nh = j.number("n_hidden_layers", 1);
	if (nh < 1 || nh > 32) throw std::runtime_error("FullyFusedMLP requires at least 1 hidden layer (3 layers in total).");
	f.N = (uint32_t)nh;
	if (n_input_dims == 0 || n_input_dims > 128) throw std::runtime_error("FullyFusedMLP: 1..128 input dims on gfx950");
	if (n_output_dims == 0 || n_output_dims > 128) throw std::runtime_error("FullyFusedMLP: 1..128 output dims on gfx950");
	f.n_in = n_input_dims; f.in_pad = (n_input_dims + 15) / 16 * 16;
	f.n_out = n_output_dims; f.out_pad = (n_output_dims + 15) / 16 * 16;
	f.act = FfNet::activation(j.string("activation", "ReLU"));
	f.out_act = FfNet::activation(j.string("output_activation", "None"));
	f.build();
	return f;
}
static std::string ff_hyper(const FfNet& f) {
	static const char* an[6] = {"None", "ReLU", "Exponential", "Sigmoid", "Squareplus", "Softplus"};
	return "{\"otype\": \"FullyFusedMLP\", \"n_neurons\": " + std::to_string(f.W) + ", \"n_hidden_layers\": " + std::to_string(f.N) +
	       ", \"activation\": \"" + an[f.act] + "\", \"output_activation\": \"" + an[f.out_act] + "\"}";
}

// tcnn::cpp::create_network(n_input_dims, n_output_dims, network) (cpp_api.cu:170-172): NetworkWithInputEncoding with an
// Identity encoding (scale 1, offset 0; padded to 16 inputs with ones, identity.h:44-70) and a FullyFusedMLP
// (fully_fused_mlp.cu:816-879: n_neurons 16 / 32 / 64 / 128, n_hidden_layers >= 1, output padded to 16)
int neus_module_create_network(uint32_t n_input_dims, uint32_t n_output_dims, const char* network_json, uint32_t batch_capacity, NeusModule** out) {
	return guard([&] {
		if (!network_json || !out) throw std::runtime_error("neus_module_create_network: null argument");
		if (batch_capacity == 0 || batch_capacity % 128 != 0 || batch_capacity > (1u << 24))
			throw std::runtime_error("batch_capacity must be a positive multiple of 128 (<= 2^24)");
		const JsonValue j = parse_json(network_json);
		*out = make_mlp_module(ff_from_json(j, n_input_dims, n_output_dims), j, batch_capacity);
	});
}
// NetworkWithInputEncoding(Identity{scale, offset} -> FullyFusedMLP) as a module (create_network, and
// create_network_with_input_encoding with an Identity encoding)
static NeusModule* make_mlp_module(const FfNet& f, const JsonValue& j, uint32_t batch_capacity) {
	{
		int dev = 0;
		HIP_CHECK(hipGetDevice(&dev));
		auto m = std::make_unique<NeusModule>(dev);
		m->kind = NeusModule::Mlp;
		module_options(m.get(), j);
		m->ff = f;
		m->n_in = f.n_in; m->n_out = f.out_pad;  // cpp::Module::n_output_dims = the padded output width
		m->capacity = batch_capacity;
		m->gtmp.alloc(f.P);
		m->ff_acts.alloc(f.acts_halves(batch_capacity));
		m->ff_front.alloc((size_t)batch_capacity * (f.in_pad + (size_t)f.N * f.W));
		const uint32_t dmax = std::max(std::max(f.W, f.out_pad), f.in_pad);
		m->ff_d[0].alloc((size_t)batch_capacity * dmax); m->ff_d[1].alloc((size_t)batch_capacity * dmax);
		m->ff_partial.alloc((size_t)ff_wgrad_blocks(batch_capacity) * f.P);
		m->ff_dummy.alloc(4);
		m->hyper = "{\"otype\": \"NetworkWithInputEncoding\", \"encoding\": {\"otype\": \"Identity\", \"scale\": " + fmt_float(f.in_scale) +
		           ", \"offset\": " + fmt_float(f.in_offset) + "}, \"network\": " + ff_hyper(f) + ", \"n_input_dims\": " + std::to_string(f.n_in) +
		           ", \"n_output_dims\": " + std::to_string(f.n_out) + ", \"gradient_precision\": \"" + (m->grad_fp16 ? "fp16" : "fp32") + "\"}";
		HIP_CHECK(hipStreamSynchronize(m->core.stream));
		return m.release();
	}
}

namespace {
// FullyFusedMLP passes (ffmlp.hip). acts: X0 [n][in_pad] then hidden l at n (in_pad + l W), each [n][W].
const half_t* ff_mat(const FfNet& f, const void* params, uint32_t l) { return (const half_t*)params + f.off[l]; }
half_t* ff_hidden(const FfNet& f, half_t* acts, uint32_t n, uint32_t l) { return acts + (size_t)n * f.in_pad + (size_t)l * n * f.W; }
FfLayer ff_layer(const half_t* W, uint32_t O, uint32_t K, bool trans, const half_t* in, uint32_t ldi, uint32_t n) {
	FfLayer L{};
	L.W = W; L.O = O; L.K = K; L.trans = trans ? 1u : 0u; L.in = in; L.ldi = ldi; L.n = n;
	return L;
}
// forward (mlp_fused_forward, fully_fused_mlp.cu:678-812): hidden layers act(W x), output out_act(W_N h)
void ff_forward(const FfNet& f, hipStream_t s, uint32_t n, const float* input, const void* params, half_t* acts, half_t* output) {
	if (input) launch_ff_input(s, n, f.n_in, f.in_pad, input, f.in_scale, f.in_offset, acts, false);  // (null: X0 already in acts)
	const half_t* x = acts;
	uint32_t ldx = f.in_pad;
	for (uint32_t l = 0; l <= f.N; ++l) {
		FfLayer L = ff_layer(ff_mat(f, params, l), f.rows[l], f.cols[l], false, x, ldx, n);
		L.mode = FF_MODE_ACT;
		L.act = l == f.N ? f.out_act : f.act;
		L.out = l == f.N ? output : ff_hidden(f, acts, n, l);
		L.ldo = l == f.N ? f.out_pad : f.W;
		launch_ff_layer(s, L);
		x = L.out; ldx = f.W;
	}
}
// delta through layer l (l >= 1) to the input of layer l: act'(h_{l-1}) (W_l^T d)
void ff_back_through(const FfNet& f, hipStream_t s, uint32_t n, const void* params, uint32_t l, const half_t* d, uint32_t ldd, const half_t* acts_fwd,
                     half_t* out) {
	FfLayer L = ff_layer(ff_mat(f, params, l), f.cols[l], f.rows[l], true, d, ldd, n);
	L.mode = FF_MODE_DACT; L.act = f.act; L.out = out; L.ldo = f.W;
	L.aux = ff_hidden(f, const_cast<half_t*>(acts_fwd), n, l - 1); L.ldx = f.W;
	launch_ff_layer(s, L);
}
void ff_wgrad(const FfNet& f, hipStream_t s, uint32_t n, uint32_t l, const half_t* d, uint32_t ldd, const half_t* x, uint32_t ldx, float* partial) {
	FfWgrad G{};
	G.D = d; G.ldd = ldd; G.O = f.rows[l]; G.X = x; G.ldx = ldx; G.I = f.cols[l];
	G.partial = partial; G.ld_partial = f.P; G.off = f.off[l]; G.n = n;
	launch_ff_wgrad(s, G);
}
// FullyFusedMLP::backward_impl (fully_fused_mlp.cu:967-1085) of a module's network down to dL/d(its input) as fp16 rows
// [n][in_pad] (returned; the module's delta ping-pong buffer), with the weight-gradient partials when wgrad
const half_t* ff_backward_chain(NeusModule* m, hipStream_t s, uint32_t n, const void* params, const half_t* acts, const half_t* dL_doutput,
                                const half_t* output, bool wgrad) {
	const FfNet& f = m->ff;
	const half_t* d = dL_doutput;
	int pp = 0;
	if (f.out_act != FF_NONE) { launch_ff_out_delta(s, n, f.out_pad, f.out_act, d, output, m->ff_d[0].p); d = m->ff_d[0].p; pp = 1; }
	uint32_t ldd = f.out_pad;
	for (uint32_t l = f.N + 1; l-- > 0;) {
		const half_t* x = l == 0 ? acts : ff_hidden(f, const_cast<half_t*>(acts), n, l - 1);
		if (wgrad) ff_wgrad(f, s, n, l, d, ldd, x, l == 0 ? f.in_pad : f.W, m->ff_partial.p);
		if (l > 0) {
			ff_back_through(f, s, n, params, l, d, ldd, acts, m->ff_d[pp].p);
			d = m->ff_d[pp].p; pp ^= 1; ldd = f.W;
		} else {
			FfLayer L = ff_layer(ff_mat(f, params, 0), f.in_pad, f.W, true, d, ldd, n);
			L.mode = FF_MODE_ACT; L.act = FF_NONE; L.out = m->ff_d[pp].p; L.ldo = f.in_pad;
			launch_ff_layer(s, L);
			d = m->ff_d[pp].p;
		}
	}
	return d;
}
// FullyFusedMLP::backward_backward_input_impl (fully_fused_mlp.cu:1088-1198), parameter gradients only, with the front
// f_0 = the network's dL_ddLdinput already in m->ff_front as rows [n][in_pad]: fronts f_i = act'(h_{i-1}) (W_{i-1} f_{i-1});
// backs b_{N+2} = dL_doutput, b_i = act'(h_{i-2}) (W_{i-1}^T b_{i+1}); dW_{i-1} = b_{i+1} f_{i-1}^T into the partials
void ff_bbi_chain(NeusModule* m, hipStream_t s, uint32_t n, const void* params, const half_t* acts, const half_t* dL_doutput) {
	const FfNet& f = m->ff;
	half_t* fr = m->ff_front.p;
	auto front = [&](uint32_t i) { return i == 0 ? fr : fr + (size_t)n * f.in_pad + (size_t)(i - 1) * n * f.W; };
	for (uint32_t i = 1; i <= f.N; ++i) {
		FfLayer L = ff_layer(ff_mat(f, params, i - 1), f.rows[i - 1], f.cols[i - 1], false, front(i - 1), i == 1 ? f.in_pad : f.W, n);
		L.mode = FF_MODE_DACT; L.act = f.act; L.out = front(i); L.ldo = f.W;
		L.aux = ff_hidden(f, const_cast<half_t*>(acts), n, i - 1); L.ldx = f.W;
		launch_ff_layer(s, L);
	}
	const half_t* b = dL_doutput;
	uint32_t ldb = f.out_pad;
	int pp = 0;
	for (uint32_t l = f.N + 1; l-- > 0;) {
		ff_wgrad(f, s, n, l, b, ldb, front(l), l == 0 ? f.in_pad : f.W, m->ff_partial.p);
		if (l > 0) {
			ff_back_through(f, s, n, params, l, b, ldb, acts, m->ff_d[pp].p);
			b = m->ff_d[pp].p; pp ^= 1; ldb = f.W;
		}
	}
}
}  // namespace

int neus_module_destroy(NeusModule* m) { return guard([&] { delete m; }); }
int neus_context_destroy(NeusContext* c) { return guard([&] { delete c; }); }

int neus_module_info(const NeusModule* m, NeusModuleInfo* o) {
	return guard([&] {
		if (!m || !o) throw std::runtime_error("neus_module_info: null argument");
		o->n_params = m->n_params();
		o->n_input_dims = m->n_in;
		o->n_output_dims = m->n_out;
		o->param_precision = m->f32 ? NEUS_PRECISION_FP32 : NEUS_PRECISION_FP16;
		o->output_precision = m->f32 ? NEUS_PRECISION_FP32 : NEUS_PRECISION_FP16;
		o->gradient_precision = NEUS_PRECISION_FP32;
		o->batch_capacity = m->capacity;
		o->n_levels = m->core.lay.L;
		o->grid_offset = m->kind == NeusModule::Network ? m->core.lay.grid_off : (m->kind == NeusModule::DensityNet ? m->n_mlp : 0);
		if (m->kind == NeusModule::Mlp) { o->n_levels = 0; o->grid_offset = m->ff.P; }  // no encoding parameters
		if (m->kind == NeusModule::GridMlp) o->grid_offset = m->ff.P;
		o->per_level_scale = m->core.cfg.per_level_scale;
	});
}

int neus_module_hyperparams(const NeusModule* m, char* buf, uint64_t cap, uint64_t* len) {
	return guard([&] {
		if (!m) throw std::runtime_error("neus_module_hyperparams: null module");
		if (len) *len = m->hyper.size();
		if (buf && cap) { const size_t k = std::min<size_t>(cap - 1, m->hyper.size()); std::memcpy(buf, m->hyper.data(), k); buf[k] = 0; }
	});
}

int neus_module_set_training_step(NeusModule* m, int training_step) { return guard([&] { m->training_step = training_step; }); }
int neus_module_set_indeed_batch_size(NeusModule* m, uint32_t n) { return guard([&] { m->indeed_batch = n; }); }

int neus_module_initialize_params(NeusModule* m, uint64_t seed, float* params_full_precision) {
	return guard([&] {
		if (!m || !params_full_precision) throw std::runtime_error("neus_module_initialize_params: null argument");
		HIP_CHECK(hipSetDevice(m->core.device));
		std::vector<float> h;
		// cpp::Module::initialize_params draws from pcg32{seed} (cpp_api.cu:162-165; the Trainer's seed_seq is not involved)
		if (m->kind == NeusModule::Mlp) {
			// NetworkWithInputEncoding::initialize_params: Identity has none; FullyFusedMLP::initialize_params
			// (fully_fused_mlp.cu:1229-1256): every matrix xavier-uniform in order, U(+-sqrt(6 / (fan_in + fan_out)))
			// (gpu_matrix.h:292-306) from pcg32{seed} (cpp_api.cu:162-165)
			h.assign(m->ff.P, 0.f);
			pcg32 rnd = make_pcg32(seed);
			for (uint32_t l = 0; l <= m->ff.N; ++l) {
				const float scale = std::sqrt(6.0f / (float)(m->ff.rows[l] + m->ff.cols[l]));
				for (uint32_t i = 0; i < m->ff.rows[l] * m->ff.cols[l]; ++i) h[m->ff.off[l] + i] = rnd.next_float() * 2.0f * scale - scale;
			}
		} else if (m->kind == NeusModule::Network) {
			h = m->core.initial_params_rng(make_pcg32(seed), nullptr);
		} else {  // [FullyFusedMLP xavier matrices (fully_fused_mlp.cu:1229-1256)] then GridEncoding::initialize_params:
			      // generate_random_uniform(rnd, n_params, -1e-4, 1e-4) (grid.h:2375-2380)
			h.assign(m->n_params(), 0.f);
			pcg32 rnd = make_pcg32(seed);
			size_t off = 0;
			if (m->kind == NeusModule::GridMlp) {  // NetworkWithInputEncoding::initialize_params: the network, then the encoding
				for (uint32_t l = 0; l <= m->ff.N; ++l) {
					const float scale = std::sqrt(6.0f / (float)(m->ff.rows[l] + m->ff.cols[l]));
					for (uint32_t i = 0; i < m->ff.rows[l] * m->ff.cols[l]; ++i) h[off + i] = rnd.next_float() * 2.0f * scale - scale;
					off += (size_t)m->ff.rows[l] * m->ff.cols[l];
				}
			}
			if (m->kind == NeusModule::DensityNet) {
				auto xavier = [&](uint32_t out, uint32_t in) {
					const float scale = std::sqrt(6.0f / (float)(in + out));
					for (uint32_t i = 0; i < out * in; ++i) h[off + i] = rnd.next_float() * 2.0f * scale - scale;
					off += (size_t)out * in;
				};
				xavier(m->dn_width, m->dn_de);
				xavier(16, m->dn_width);
			}
			float* hg = h.data() + off;
			const size_t N = h.size() - off, per = 4, n_threads = (N + per - 1) / per, n_pad = (n_threads + 127) / 128 * 128;
			for (size_t i = 0; i < n_pad; ++i) {
				pcg32 r = rnd; r.advance((int64_t)(i * per));
				for (size_t k = 0; k < per; ++k) {
					const size_t idx = i + n_pad * k;
					if (idx >= N) break;
					hg[idx] = r.next_float() * (1e-4f - -1e-4f) + -1e-4f;
				}
			}
		}
		HIP_CHECK(hipMemcpy(params_full_precision, h.data(), h.size() * 4, hipMemcpyHostToDevice));
	});
}

static void module_forward(NeusModule* m, hipStream_t s, uint32_t n, const float* input, void* output, const void* params, NeusContext* ctx) {
	if (!input || !output) throw std::runtime_error("module forward: null input / output");
	m->check_n(n, false);
	NeusTestbed& t = m->core;
	if (m->kind == NeusModule::Mlp) {
		if (!params) throw std::runtime_error("module: null params");
		if (ctx) ctx->acts.alloc(std::max<size_t>(1, m->ff.acts_halves(n)));
		ff_forward(m->ff, s, n, input, params, ctx ? ctx->acts.p : m->ff_acts.p, (half_t*)output);
		HIP_CHECK(hipGetLastError());
		return;
	}
	if (m->kind == NeusModule::GridMlp) {
		// NetworkWithInputEncoding::forward (network_with_input_encoding.h:113-124): the HashGrid (zero-padded to the MLP's
		// input width, grid.h:1540-1550), then the FullyFusedMLP on it
		if (!params) throw std::runtime_error("module: null params");
		const FfNet& f = m->ff;
		uint32_t* enc = m->enc_tmp.p;
		float* dydx = nullptr;
		half_t* acts = m->ff_acts.p;
		if (ctx) {
			ctx->dydx.alloc((size_t)6 * t.lay.L * std::max(1u, n)); dydx = ctx->dydx.p;
			ctx->enc.alloc((size_t)t.lay.L * std::max(1u, n)); enc = ctx->enc.p;
			ctx->acts.alloc(std::max<size_t>(1, f.acts_halves(n))); acts = ctx->acts.p;
		}
		const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, 4096));
		launch_grid_encode(s, nullptr, n, n, input, 3, t.gl, m->valid(), (const half_t*)params + f.P, enc, dydx, gx);
		launch_enc_to_rows(s, n, t.lay.L, enc, acts, f.in_pad);
		ff_forward(f, s, n, nullptr, params, acts, (half_t*)output);
		HIP_CHECK(hipGetLastError());
		return;
	}
	if (m->kind == NeusModule::DensityNet) {
		// NetworkWithInputEncoding::forward (network_with_input_encoding.h:84-111): encoding, then the MLP on it
		if (!params) throw std::runtime_error("module: null params");
		const half_t* ph = (const half_t*)params;
		float* dydx = nullptr;
		uint32_t* enc = m->enc_tmp.p;
		if (ctx) {
			ctx->dydx.alloc((size_t)6 * t.lay.L * std::max(1u, n)); dydx = ctx->dydx.p;
			ctx->enc.alloc((size_t)t.lay.L * std::max(1u, n)); enc = ctx->enc.p;
		}
		const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, 4096));
		launch_grid_encode(s, nullptr, n, n, input, 3, t.gl, m->valid(), ph + m->n_mlp, enc, dydx, gx);
		DNetLaunch d{};
		d.w0 = ph; d.w1 = ph + (size_t)m->dn_width * m->dn_de; d.enc = enc; d.out = (half_t*)output;
		launch_dnet(s, t.lay.L, m->dn_width, 0, n, d);
		HIP_CHECK(hipGetLastError());
		return;
	}
	if (m->f32) {  // GridEncoding<float>::forward (kernel_grid with T = float)
		if (!params) throw std::runtime_error("module: null params");
		float* dydx = nullptr;
		if (ctx) { ctx->dydx.alloc((size_t)6 * t.lay.L * std::max(1u, n)); dydx = ctx->dydx.p; }
		launch_grid_f32_forward(s, n, t.gl, m->valid(), input, (const float*)params, (float*)output, m->layout, dydx);
		HIP_CHECK(hipGetLastError());
		return;
	}
	m->load_params(params, s);
	if (m->kind == NeusModule::Network) {
		t.net_forward(nullptr, n, n, input, m->valid(), (half_t*)output, s);
	} else {
		float* dydx = nullptr;
		if (ctx) { ctx->dydx.alloc((size_t)6 * t.lay.L * std::max(1u, n)); dydx = ctx->dydx.p; }
		const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, 4096));
		uint32_t* enc = m->layout == ENC_LAYOUT_PAIRED ? (uint32_t*)output : m->enc_tmp.p;
		launch_grid_encode(s, nullptr, n, n, input, 3, t.gl, m->valid(), t.params_h.p + t.lay.grid_off, enc, dydx, gx);
		if (m->layout != ENC_LAYOUT_PAIRED) launch_enc_to_layout(s, n, t.lay.L, enc, (half_t*)output, m->layout);
	}
	HIP_CHECK(hipGetLastError());
}

int neus_module_inference(NeusModule* m, void* stream, uint32_t n, const float* input, void* output, const void* params) {
	return guard([&] {
		HIP_CHECK(hipSetDevice(m->core.device));
		StreamSwap sw(m->core, stream);
		module_forward(m, m->core.stream, n, input, output, params, nullptr);
	});
}

int neus_module_forward(NeusModule* m, void* stream, uint32_t n, const float* input, void* output, const void* params,
                        int prepare_input_gradients, NeusContext** ctx_out) {
	return guard([&] {
		if (!ctx_out) throw std::runtime_error("neus_module_forward: null context output");
		HIP_CHECK(hipSetDevice(m->core.device));
		StreamSwap sw(m->core, stream);
		auto ctx = std::make_unique<NeusContext>();
		ctx->n = n;
		// the NerfNetwork's backward recomputes its forward; the encodings keep dy/dx for dL_dinput and second order
		(void)prepare_input_gradients;
		module_forward(m, m->core.stream, n, input, output, params, m->kind != NeusModule::Network ? ctx.get() : nullptr);
		*ctx_out = ctx.release();
	});
}

int neus_module_backward(NeusModule* m, void* stream, const NeusContext* ctx, uint32_t n, float* dL_dinput, const void* dL_doutput,
                         void* dL_dparams, const float* input, const void* output, const void* params, int gradient_mode) {
	return guard([&] {
		(void)output;
		if (!ctx || ctx->n != n) throw std::runtime_error("module backward: the context is not from a forward over n_elements");
		if (!input || !dL_doutput) throw std::runtime_error("module backward: null input / dL_doutput");
		m->check_n(n, true);
		HIP_CHECK(hipSetDevice(m->core.device));
		StreamSwap sw(m->core, stream);
		NeusTestbed& t = m->core;
		hipStream_t s = t.stream;
		float* g = m->grad_target(dL_dparams, gradient_mode);
		if (!g && !dL_dinput) return;
		if (m->kind == NeusModule::Mlp) {
			// FullyFusedMLP::backward_impl (fully_fused_mlp.cu:967-1085): the output activation's backward on dL/doutput, the
			// deltas through the hidden layers (activation derivative from the stored outputs), dW = D^T x per layer and
			// dL/dinput = W_0^T D_0 through the Identity encoding's backward (identity.h:86-104: x scale = 1)
			const FfNet& f = m->ff;
			if (!params) throw std::runtime_error("module: null params");
			if (!ctx->acts.p) throw std::runtime_error("module backward: the context is not from this module's forward");
			if (f.out_act != FF_NONE && !output) throw std::runtime_error("FullyFusedMLP backward: the forward output is needed for its output activation");
			const half_t* d = (const half_t*)dL_doutput;
			int pp = 0;
			if (f.out_act != FF_NONE) { launch_ff_out_delta(s, n, f.out_pad, f.out_act, d, (const half_t*)output, m->ff_d[0].p); d = m->ff_d[0].p; pp = 1; }
			uint32_t ldd = f.out_pad;
			for (uint32_t l = f.N + 1; l-- > 0;) {
				const half_t* x = l == 0 ? ctx->acts.p : ff_hidden(f, ctx->acts.p, n, l - 1);
				if (g) ff_wgrad(f, s, n, l, d, ldd, x, l == 0 ? f.in_pad : f.W, m->ff_partial.p);
				if (l > 0) {
					ff_back_through(f, s, n, params, l, d, ldd, ctx->acts.p, m->ff_d[pp].p);
					d = m->ff_d[pp].p; pp ^= 1; ldd = f.W;
				} else if (dL_dinput) {
					FfLayer L = ff_layer(ff_mat(f, params, 0), f.in_pad, f.W, true, d, ldd, n);
					L.mode = FF_MODE_F32; L.out_f = dL_dinput; L.ldo = f.n_in; L.o_lim = f.n_in; L.out_scale = f.in_scale;
					launch_ff_layer(s, L);
				}
			}
			if (g) {
				launch_mlp_grad_reduce(s, MlpGradReduce{m->ff_partial.p, ff_wgrad_blocks(n), f.P, g, nullptr, nullptr, 0, m->ff_dummy.p});
				m->finish_grad(dL_dparams, gradient_mode, s);
			}
			HIP_CHECK(hipGetLastError());
			return;
		}
		const uint32_t valid = m->valid();
		if (m->kind == NeusModule::GridMlp) {
			// NetworkWithInputEncoding::backward (network_with_input_encoding.h:126-156): the FullyFusedMLP's backward (weight
			// gradients, dL/d(its input) in fp16) and the HashGrid's backward of that (grid gradients, dL_dinput from dy/dx)
			const FfNet& f = m->ff;
			if (!params) throw std::runtime_error("module: null params");
			if (!ctx->acts.p || !ctx->dydx.p) throw std::runtime_error("module backward: the context is not from this module's forward");
			if (f.out_act != FF_NONE && !output) throw std::runtime_error("FullyFusedMLP backward: the forward output is needed for its output activation");
			const half_t* dX0 = ff_backward_chain(m, s, n, params, ctx->acts.p, (const half_t*)dL_doutput, (const half_t*)output, g != nullptr);
			launch_enc_from_rows(s, n, t.lay.L, dX0, f.in_pad, m->denc_tmp.p);
			if (g) {
				launch_mlp_grad_reduce(s, MlpGradReduce{m->ff_partial.p, ff_wgrad_blocks(n), f.P, g, nullptr, nullptr, 0, m->ff_dummy.p});
				launch_grid_scatter(s, nullptr, n, n, input, 3, t.gl, valid, (const half_t*)m->denc_tmp.p, m->zero_h.p, m->zero_v.p, g + f.P,
				                    t.swork, t.scan_tmp.p, t.scan_tmp_bytes);
			}
			if (dL_dinput) launch_enc_input_grad(s, n, n, t.lay.L, (const half_t*)m->denc_tmp.p, ctx->dydx.p, dL_dinput, 3);
			if (g) m->finish_grad(dL_dparams, gradient_mode, s);
			HIP_CHECK(hipGetLastError());
			return;
		}
		if (m->kind == NeusModule::DensityNet) {
			// NetworkWithInputEncoding::backward (network_with_input_encoding.h:113-156): the MLP backward gives its weight
			// gradients and dL/d(encoding); the encoding's backward the grid gradients and dL_dinput
			if (!params) throw std::runtime_error("module: null params");
			if (!ctx->enc.p || !ctx->dydx.p) throw std::runtime_error("module backward: the context is not from this module's forward");
			const half_t* ph = (const half_t*)params;
			DNetLaunch d{};
			d.w0 = ph; d.w1 = ph + (size_t)m->dn_width * m->dn_de; d.enc = ctx->enc.p; d.dL = (const half_t*)dL_doutput;
			d.denc = m->denc_tmp.p; d.wpartial = m->dn_partial.p;
			launch_dnet(s, t.lay.L, m->dn_width, 1, n, d);
			if (g) {
				launch_mlp_grad_reduce(s, MlpGradReduce{m->dn_partial.p, dnet_blocks(n), m->n_mlp, g, nullptr, nullptr, 0, m->dn_dummy.p});
				launch_grid_scatter(s, nullptr, n, n, input, 3, t.gl, valid, (const half_t*)m->denc_tmp.p, m->zero_h.p, m->zero_v.p, g + m->n_mlp,
				                    t.swork, t.scan_tmp.p, t.scan_tmp_bytes);
			}
			if (dL_dinput) launch_enc_input_grad(s, n, n, t.lay.L, (const half_t*)m->denc_tmp.p, ctx->dydx.p, dL_dinput, 3);
			if (g) m->finish_grad(dL_dparams, gradient_mode, s);
			HIP_CHECK(hipGetLastError());
			return;
		}
		if (m->f32) {  // GridEncoding<float>::backward: kernel_grid_backward (float atomics) and dL_dinput from dy/dx
			if (dL_dinput && !ctx->dydx.p) throw std::runtime_error("encoding backward: dL_dinput needs the forward's dy/dx");
			if (g) HIP_CHECK(hipMemsetAsync(g, 0, (size_t)m->n_params() * 4, s));
			launch_grid_f32_backward(s, n, t.gl, valid, input, (const float*)dL_doutput, m->layout, g, ctx->dydx.p, dL_dinput);
			if (g) m->finish_grad(dL_dparams, gradient_mode, s);
			HIP_CHECK(hipGetLastError());
			return;
		}
		m->load_params(params, s);
		if (m->kind == NeusModule::Network) {
			// NerfNetwork::backward (nerf_network.h:330-601): first and second order in one pass; the Testbed's
			// forward-recompute + backward writes every parameter gradient (Overwrite) into g
			float* gg = g ? g : m->gtmp.p;
			HIP_CHECK(hipMemsetAsync(gg, 0, (size_t)t.lay.P * 4, s));
			const float saved = t.tbuf.indeed_batch;
			t.tbuf.indeed_batch = (float)(m->indeed_batch ? m->indeed_batch : n);
			t.tbuf.dpos = dL_dinput ? m->dpos.p : nullptr;
			t.net_backward(nullptr, nullptr, n, input, valid, (const half_t*)dL_doutput, gg, s);
			t.tbuf.dpos = nullptr;
			t.tbuf.indeed_batch = saved;
			if (dL_dinput) {  // position columns; dt and direction columns are 0 (the direction gradient is not propagated)
				HIP_CHECK(hipMemset2DAsync(dL_dinput, COORD_W * 4, 0, COORD_W * 4, n, s));
				HIP_CHECK(hipMemcpy2DAsync(dL_dinput, COORD_W * 4, m->dpos.p, 16, 12, n, hipMemcpyDeviceToDevice, s));
			}
		} else {
			const half_t* dly = m->paired_in(dL_doutput, n, s);
			if (dL_dinput) {
				if (!ctx->dydx.p) throw std::runtime_error("encoding backward: dL_dinput needs the forward's dy/dx");
				launch_enc_input_grad(s, n, n, t.lay.L, dly, ctx->dydx.p, dL_dinput, 3);
			}
			if (g)  // kernel_grid_backward (grid.h:371-500) through the fused binned scatter, second-order term zero
				launch_grid_scatter(s, nullptr, n, n, input, 3, t.gl, valid, dly, m->zero_h.p, m->zero_v.p, g, t.swork,
				                    t.scan_tmp.p, t.scan_tmp_bytes);
		}
		if (g) m->finish_grad(dL_dparams, gradient_mode, s);
		HIP_CHECK(hipGetLastError());
	});
}

int neus_module_backward_backward_input(NeusModule* m, void* stream, const NeusContext* ctx, uint32_t n, const float* dL_ddLdinput,
                                        const float* input, const void* dL_doutput, void* dL_dparams, void* dL_ddLdoutput, float* dL_dinput,
                                        const void* params, int gradient_mode) {
	return guard([&] {
		if (m->kind == NeusModule::Network)
			throw std::runtime_error("NerfNetwork: the eikonal second-order term is part of backward (nerf_network.h:330-601); "
			                         "backward_backward_input is provided by the HashGrid and network-with-input-encoding modules "
			                         "(the reference's NerfNetwork does not implement it either: object.h:222-232)");
		if (m->kind == NeusModule::Mlp) {
			// NetworkWithInputEncoding::backward_backward_input (network_with_input_encoding.h:159-250) with the Identity
			// encoding: its backward_backward_input (identity.h:182-206) turns dL_ddLdinput into the network's dL_ddLdinput
			// (x scale; the padded rows, which the reference leaves uninitialised, are 0: the constant padding has no input
			// gradient); FullyFusedMLP::backward_backward_input_impl (fully_fused_mlp.cu:1088-1198): fronts f_0 = u,
			// f_i = act'(h_{i-1}) (W_{i-1} f_{i-1}); backs b_{N+2} = dL_doutput, b_i = act'(h_{i-2}) (W_{i-1}^T b_{i+1});
			// dW_{i-1} = b_{i+1} f_{i-1}^T. Like the reference, dL_ddLdoutput and dL_dinput are not produced.
			if (!ctx || ctx->n != n || !ctx->acts.p) throw std::runtime_error("backward_backward_input: needs the forward's context");
			if (!dL_ddLdinput || !dL_doutput || !params) throw std::runtime_error("backward_backward_input: null input");
			m->check_n(n, true);
			HIP_CHECK(hipSetDevice(m->core.device));
			StreamSwap sw(m->core, stream);
			hipStream_t s = m->core.stream;
			float* g = m->grad_target(dL_dparams, gradient_mode);
			if (!g) return;
			const FfNet& f = m->ff;
			half_t* fr = m->ff_front.p;
			auto front = [&](uint32_t i) { return i == 0 ? fr : fr + (size_t)n * f.in_pad + (size_t)(i - 1) * n * f.W; };
			launch_ff_input(s, n, f.n_in, f.in_pad, dL_ddLdinput, f.in_scale, 0.f, fr, true);
			for (uint32_t i = 1; i <= f.N; ++i) {
				FfLayer L = ff_layer(ff_mat(f, params, i - 1), f.rows[i - 1], f.cols[i - 1], false, front(i - 1), i == 1 ? f.in_pad : f.W, n);
				L.mode = FF_MODE_DACT; L.act = f.act; L.out = front(i); L.ldo = f.W;
				L.aux = ff_hidden(f, ctx->acts.p, n, i - 1); L.ldx = f.W;
				launch_ff_layer(s, L);
			}
			const half_t* b = (const half_t*)dL_doutput;
			uint32_t ldb = f.out_pad;
			int pp = 0;
			for (uint32_t l = f.N + 1; l-- > 0;) {  // dW_l = b_{l+2} f_l^T, then b_{l+1} through W_l
				ff_wgrad(f, s, n, l, b, ldb, front(l), l == 0 ? f.in_pad : f.W, m->ff_partial.p);
				if (l > 0) {
					ff_back_through(f, s, n, params, l, b, ldb, ctx->acts.p, m->ff_d[pp].p);
					b = m->ff_d[pp].p; pp ^= 1; ldb = f.W;
				}
			}
			launch_mlp_grad_reduce(s, MlpGradReduce{m->ff_partial.p, ff_wgrad_blocks(n), f.P, g, nullptr, nullptr, 0, m->ff_dummy.p});
			m->finish_grad(dL_dparams, gradient_mode, s);
			HIP_CHECK(hipGetLastError());
			return;
		}
		if (m->kind == NeusModule::GridMlp) {
			// NetworkWithInputEncoding::backward_backward_input (network_with_input_encoding.h:159-250): (1) the network's
			// backward gives dL/d(encoding) (parameter gradients ignored); (2) the HashGrid's backward_backward_input with it as
			// dL_doutput: the second-order grid gradient and pos_encoding_dy = dy/dx . dL_ddLdinput (grid.h:1697-1800); (3) the
			// FullyFusedMLP's backward_backward_input with pos_encoding_dy as its dL_ddLdinput (fully_fused_mlp.cu:1088-1198).
			// Like the reference, dL_ddLdoutput and dL_dinput are not produced.
			if (!ctx || ctx->n != n || !ctx->dydx.p || !ctx->acts.p) throw std::runtime_error("backward_backward_input: needs the forward's context");
			if (!input || !dL_ddLdinput || !dL_doutput || !params) throw std::runtime_error("backward_backward_input: null input");
			m->check_n(n, true);
			HIP_CHECK(hipSetDevice(m->core.device));
			StreamSwap sw(m->core, stream);
			NeusTestbed& t = m->core;
			hipStream_t s = t.stream;
			float* g = m->grad_target(dL_dparams, gradient_mode);
			if (!g) return;
			const FfNet& f = m->ff;
			const half_t* dX0 = ff_backward_chain(m, s, n, params, ctx->acts.p, (const half_t*)dL_doutput, nullptr, false);
			launch_enc_from_rows(s, n, t.lay.L, dX0, f.in_pad, m->denc_tmp.p);
			launch_enc_ddLdoutput(s, n, n, t.lay.L, dL_ddLdinput, ctx->dydx.p, (half_t*)m->u_tmp.p, m->v4.p);
			launch_grid_scatter(s, nullptr, n, n, input, 3, t.gl, m->valid(), m->zero_h.p, (const half_t*)m->denc_tmp.p, m->v4.p, g + f.P,
			                    t.swork, t.scan_tmp.p, t.scan_tmp_bytes);
			launch_enc_to_rows(s, n, t.lay.L, m->u_tmp.p, m->ff_front.p, f.in_pad);
			ff_bbi_chain(m, s, n, params, ctx->acts.p, (const half_t*)dL_doutput);
			launch_mlp_grad_reduce(s, MlpGradReduce{m->ff_partial.p, ff_wgrad_blocks(n), f.P, g, nullptr, nullptr, 0, m->ff_dummy.p});
			m->finish_grad(dL_dparams, gradient_mode, s);
			HIP_CHECK(hipGetLastError());
			return;
		}
		if (m->kind == NeusModule::DensityNet) {
			// NetworkWithInputEncoding::backward_backward_input (network_with_input_encoding.h:159-250): u = dy/dx . dL_ddLdinput
			// (kernel_grid_backward_input_backward_dLdoutput), the MLP's backward-backward (fully_fused_mlp.cu:1088-1198: b2 =
			// relu'(H0) W1^T dL, h1' = relu'(H0) W0 u; dW0 = b2 u^T, dW1 = dL h1'^T) and the encoding's second-order grid
			// gradient with dL/d(encoding) = W0^T b2. Like the reference, dL_ddLdoutput and dL_dinput are not produced.
			if (!ctx || ctx->n != n || !ctx->dydx.p || !ctx->enc.p) throw std::runtime_error("backward_backward_input: needs the forward's context");
			if (!input || !dL_ddLdinput || !dL_doutput || !params) throw std::runtime_error("backward_backward_input: null input");
			m->check_n(n, true);
			HIP_CHECK(hipSetDevice(m->core.device));
			StreamSwap sw(m->core, stream);
			NeusTestbed& t = m->core;
			hipStream_t s = t.stream;
			float* g = m->grad_target(dL_dparams, gradient_mode);
			if (!g) return;
			const half_t* ph = (const half_t*)params;
			launch_enc_ddLdoutput(s, n, n, t.lay.L, dL_ddLdinput, ctx->dydx.p, (half_t*)m->u_tmp.p, m->v4.p);
			DNetLaunch d{};
			d.w0 = ph; d.w1 = ph + (size_t)m->dn_width * m->dn_de; d.enc = ctx->enc.p; d.dL = (const half_t*)dL_doutput; d.u = m->u_tmp.p;
			d.denc = m->denc_tmp.p; d.wpartial = m->dn_partial.p;
			launch_dnet(s, t.lay.L, m->dn_width, 2, n, d);
			launch_mlp_grad_reduce(s, MlpGradReduce{m->dn_partial.p, dnet_blocks(n), m->n_mlp, g, nullptr, nullptr, 0, m->dn_dummy.p});
			launch_grid_scatter(s, nullptr, n, n, input, 3, t.gl, m->valid(), m->zero_h.p, (const half_t*)m->denc_tmp.p, m->v4.p, g + m->n_mlp,
			                    t.swork, t.scan_tmp.p, t.scan_tmp_bytes);
			m->finish_grad(dL_dparams, gradient_mode, s);
			HIP_CHECK(hipGetLastError());
			return;
		}
		if (dL_dinput) throw std::runtime_error("HashGrid backward_backward_input: dL_dinput (second derivative in x) is not provided");
		if (!ctx || ctx->n != n || !ctx->dydx.p) throw std::runtime_error("backward_backward_input: needs the forward's context (dy/dx)");
		if (!input || !dL_ddLdinput || !dL_doutput) throw std::runtime_error("backward_backward_input: null input");
		m->check_n(n, true);
		HIP_CHECK(hipSetDevice(m->core.device));
		StreamSwap sw(m->core, stream);
		NeusTestbed& t = m->core;
		hipStream_t s = t.stream;
		float* g = m->grad_target(dL_dparams, gradient_mode);
		if (m->f32) {  // GridEncoding<float>::backward_backward_input (grid.h:880-1007 with GRAD_T = float)
			if (g) HIP_CHECK(hipMemsetAsync(g, 0, (size_t)m->n_params() * 4, s));
			launch_grid_f32_bbi(s, n, t.gl, m->valid(), input, dL_ddLdinput, (const float*)dL_doutput, m->layout, g, ctx->dydx.p, (float*)dL_ddLdoutput);
			if (g) m->finish_grad(dL_dparams, gradient_mode, s);
			HIP_CHECK(hipGetLastError());
			return;
		}
		// dL_ddLdoutput (kernel_grid_backward_input_backward_dLdoutput) and dL_ddLdinput as float4 for the scatter
		const bool relay = m->layout != ENC_LAYOUT_PAIRED && dL_ddLdoutput;
		launch_enc_ddLdoutput(s, n, n, t.lay.L, dL_ddLdinput, ctx->dydx.p, relay ? (half_t*)m->enc_tmp.p : (half_t*)dL_ddLdoutput, m->v4.p);
		if (relay) launch_enc_to_layout(s, n, t.lay.L, m->enc_tmp.p, (half_t*)dL_ddLdoutput, m->layout);
		if (g) {
			m->load_params(params, s);
			const half_t* dly = m->paired_in(dL_doutput, n, s);
			// kernel_grid_backward_input_backward_grid (grid.h:880-1007): the fused scatter's second-order term with
			// g = dL_doutput, v = dL_ddLdinput, first-order term zero
			launch_grid_scatter(s, nullptr, n, n, input, 3, t.gl, m->valid(), m->zero_h.p, dly, m->v4.p, g, t.swork,
			                    t.scan_tmp.p, t.scan_tmp_bytes);
			m->finish_grad(dL_dparams, gradient_mode, s);
		}
		HIP_CHECK(hipGetLastError());
	});
}
