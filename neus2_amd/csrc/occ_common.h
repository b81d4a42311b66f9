// One density-grid sample of generate_grid_samples_nerf_nonuniform (testbed_nerf.cu:640-669): a cascade level from
// the sample's pcg32 stream (advanced by 4 per sample), a cell from the reference's hash of (i + step * n) that
// retries up to 10 times for a cell above `thresh`, a jittered position in it warped into the aabb. Shared by the
// separate sample pass (optim.hip) and the fused occupancy-density kernel (mlp.hip), so both give the same bits
// (no FMA contraction inside, whatever the including file's flags).
#pragma once
#include "kernels.h"

namespace neus {

// the cascade level and the cell (level * 128^3 + Morton index) of sample i, the rng advanced past the level draw
__device__ __forceinline__ uint32_t grid_sample_pick(uint32_t n_elements, uint32_t i, pcg32& rng, uint32_t step, const float* __restrict__ grid_in,
                                                     uint32_t n_cascades, float thresh) {
#pragma clang fp contract(off)
	const uint32_t level = (uint32_t)(rng.next_float() * n_cascades) % n_cascades;
	uint32_t idx = 0;
	for (uint32_t j = 0; j < 10; ++j) {
		idx = ((i + step * n_elements) * 56924617u + j * 19349663u + 96925573u) % GRID3;
		idx += level * GRID3;
		if (grid_in[idx] > thresh) break;
	}
	return idx;
}

__device__ __forceinline__ void grid_sample(uint32_t n_elements, uint32_t i, uint64_t rng_state, uint64_t rng_inc, uint32_t step,
                                            const float amin[3], const float diag[3], const float* __restrict__ grid_in, uint32_t n_cascades,
                                            float thresh, float pos[3], uint32_t& idx_out, const PcgJumpTable& jt) {
#pragma clang fp contract(off)  // the same bits in every translation unit (and as the oracle's restatement)
	pcg32 rng(rng_state, rng_inc);
	pcg_advance(rng, (uint64_t)(uint32_t)(i * 4), jt);
	const uint32_t idx = grid_sample_pick(n_elements, i, rng, step, grid_in, n_cascades, thresh);
	const uint32_t level = idx / GRID3;
	const uint32_t pi = idx % GRID3;
	const uint32_t x = morton3D_invert(pi >> 0), y = morton3D_invert(pi >> 1), z = morton3D_invert(pi >> 2);
	const float rx = rng.next_float(), ry = rng.next_float(), rz = rng.next_float();
	const float sc = scalbnf(1.0f, (int)level);
	const float px = (((float)x + rx) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f;
	const float py = (((float)y + ry) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f;
	const float pz = (((float)z + rz) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f;
	pos[0] = (px - amin[0]) / diag[0];
	pos[1] = (py - amin[1]) / diag[1];
	pos[2] = (pz - amin[2]) / diag[2];
	idx_out = idx;
}

// The same sample, addressed by its cell, for the all-cells uniform pass over one cascade (n = 128^3, thresh -0.01):
// there the first hash try is always taken (densities are >= 0) and (i + step n) * 56924617 + 96925573 mod 2^21 is a
// bijection (odd multiplier; n = 2^21 makes the step term vanish), so cell c holds exactly sample
// i = (c - 96925573) * 56924617^-1 mod 2^21 (the inverse is 53369). Walking cells in order gives coalesced grid
// reads / writes and spatially coherent hash-grid gathers; every sample's value is unchanged (a grid holding
// NaN would make the reference retry another cell - training has diverged then, see the non-finite loss flag).
__device__ __forceinline__ void grid_sample_cell(uint32_t c, uint64_t rng_state, uint64_t rng_inc, const float amin[3], const float diag[3],
                                                 float pos[3], const PcgJumpTable& jt) {
#pragma clang fp contract(off)
	const uint32_t i = ((c - 96925573u) * 53369u) & (GRID3 - 1);
	pcg32 rng(rng_state, rng_inc);
	pcg_advance(rng, (uint64_t)(uint32_t)(i * 4), jt);
	(void)rng.next_float();  // the cascade draw (one cascade: level 0)
	const uint32_t x = morton3D_invert(c >> 0), y = morton3D_invert(c >> 1), z = morton3D_invert(c >> 2);
	const float rx = rng.next_float(), ry = rng.next_float(), rz = rng.next_float();
	const float sc = 1.0f;
	const float px = (((float)x + rx) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f;
	const float py = (((float)y + ry) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f;
	const float pz = (((float)z + rz) / NERF_GRIDSIZE - 0.5f) * sc + 0.5f;
	pos[0] = (px - amin[0]) / diag[0];
	pos[1] = (py - amin[1]) / diag[1];
	pos[2] = (pz - amin[2]) / diag[2];
}

} // namespace neus
