// Marching cubes over an SDF grid on gfx950 (Testbed::marching_cubes -> marching_cubes_gpu,
// testbed_nerf.cu:4175-4226, marching_cubes.cu:276-420, 794-822).
//
// The reference runs gen_vertices / gen_faces twice (count with atomics, then emit with atomics), so
// its vertex and triangle order changes from run to run. Here the grid is cut into chunks of
// MC_CHUNK consecutive grid points (x fastest):
//   k_mc_count : per chunk, the number of crossing edges (vertices) and of triangles
//   exclusive scans of the two per-chunk counts (hipCUB)
//   k_mc_verts : per chunk, a workgroup-local scan gives each grid point its first vertex id; vertices are
//                written in (point, axis x<y<z) order and the point's first id is stored in vidx
//   k_mc_faces : per chunk, a local scan of triangle counts; every triangle edge resolves to
//                vidx[owner point] + (crossings of that point on lower axes)
// so the mesh is a deterministic function of the density grid. Vertex positions are the reference's
// expression ((x + dt) * scale + aabb.min with dt = (thresh - f0) / (f1 - f0)); compiled with
// -ffp-contract=off they are bit-identical to the CPU oracle. Indices are 64-bit in the grid (1024^3
// points and beyond) and 32-bit in the mesh.
//
// The triangle table is the reference's constant table (mc_tables.h, marching_cubes.cu:401-658), so every case,
// the ambiguous ones included, produces the reference's faces; only the vertex / triangle order differs
// (deterministic here, atomic-append order there).
#pragma clang fp contract(off)
#include "kernels.h"
#include "mc_tables.h"

#include <cmath>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace neus {

constexpr int MC_MAX_TRIS = 6;
constexpr int MC_ROW = 3 * MC_MAX_TRIS + 1;
__constant__ int8_t c_mc_table[256][MC_ROW];
__constant__ uint8_t c_mc_ntri[256];

// The case table is the reference's (mc_tables.h, marching_cubes.cu:401-658), re-laid out as rows of up to
// MC_MAX_TRIS edge triples, -1 terminated, plus the triangle count per case.
static void mc_build_table(int8_t table[256][MC_ROW], uint8_t ntri[256]) {
	for (int m = 0; m < 256; ++m) {
		for (int k = 0; k < MC_ROW; ++k) table[m][k] = -1;
		int n = 0;
		while (n < 15 && MC_TRIANGLE_TABLE[m][n] >= 0) { table[m][n] = MC_TRIANGLE_TABLE[m][n]; ++n; }
		if (n % 3 != 0) throw std::runtime_error("mc table: row not made of triangles");
		ntri[m] = (uint8_t)(n / 3);
	}
}

static void mc_upload_table() {
	static std::once_flag once;
	static int8_t table[256][MC_ROW];
	static uint8_t ntri[256];
	std::call_once(once, [] { mc_build_table(table, ntri); });
	// per device: the constant symbols live in each device's code object
	if (hipMemcpyToSymbol(HIP_SYMBOL(c_mc_table), table, sizeof(table)) != hipSuccess ||
	    hipMemcpyToSymbol(HIP_SYMBOL(c_mc_ntri), ntri, sizeof(ntri)) != hipSuccess)
		throw std::runtime_error("mc: table upload failed");
}

void mc_table_host(int8_t* out /* 256 * MC_ROW */) {
	static int8_t table[256][MC_ROW];
	static uint8_t ntri[256];
	mc_build_table(table, ntri);
	std::memcpy(out, table, sizeof(table));
}

struct McGrid { uint32_t rx, ry, rz; uint64_t n; float thresh; float scale[3], offset[3]; };

__device__ __forceinline__ void mc_xyz(const McGrid& g, uint64_t p, uint32_t& x, uint32_t& y, uint32_t& z) {
	const uint64_t rxy = (uint64_t)g.rx * g.ry;
	z = (uint32_t)(p / rxy);
	const uint64_t rem = p - (uint64_t)z * rxy;
	y = (uint32_t)(rem / g.rx);
	x = (uint32_t)(rem - (uint64_t)y * g.rx);
}
// crossing flags of the three edges owned by point p (+x, +y, +z), bits 0..2
__device__ __forceinline__ uint32_t mc_point_flags(const McGrid& g, const float* __restrict__ d, uint64_t p, uint32_t x, uint32_t y, uint32_t z) {
	const float f0 = d[p];
	const bool in0 = f0 > g.thresh;
	uint32_t f = 0;
	if (x + 1 < g.rx && in0 != (d[p + 1] > g.thresh)) f |= 1;
	if (y + 1 < g.ry && in0 != (d[p + g.rx] > g.thresh)) f |= 2;
	if (z + 1 < g.rz && in0 != (d[p + (uint64_t)g.rx * g.ry] > g.thresh)) f |= 4;
	return f;
}
__device__ __forceinline__ uint32_t mc_cube_mask(const McGrid& g, const float* __restrict__ d, uint64_t p, uint32_t x, uint32_t y, uint32_t z) {
	if (x + 1 >= g.rx || y + 1 >= g.ry || z + 1 >= g.rz) return 0;
	const uint64_t r1 = g.rx, r2 = (uint64_t)g.rx * g.ry;
	uint32_t m = 0;
	m |= (uint32_t)(d[p] > g.thresh);
	m |= (uint32_t)(d[p + 1] > g.thresh) << 1;
	m |= (uint32_t)(d[p + 1 + r1] > g.thresh) << 2;
	m |= (uint32_t)(d[p + r1] > g.thresh) << 3;
	m |= (uint32_t)(d[p + r2] > g.thresh) << 4;
	m |= (uint32_t)(d[p + 1 + r2] > g.thresh) << 5;
	m |= (uint32_t)(d[p + 1 + r1 + r2] > g.thresh) << 6;
	m |= (uint32_t)(d[p + r1 + r2] > g.thresh) << 7;
	return m;
}

constexpr uint32_t MC_THREADS = 256, MC_PER_THREAD = 8, MC_CHUNK = MC_THREADS * MC_PER_THREAD;

// Block-wide exclusive scan of one value per thread (wave prefix via DPP-free shuffles + LDS).
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wave, uint32_t& total) {
	const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	uint32_t inc = v;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t t = __shfl_up(inc, o, 64);
		if (lane >= (uint32_t)o) inc += t;
	}
	if (lane == 63) s_wave[wv] = inc;
	__syncthreads();
	uint32_t wbase = 0, tot = 0;
#pragma unroll
	for (uint32_t k = 0; k < MC_THREADS / 64; ++k) { const uint32_t s = s_wave[k]; wbase += k < wv ? s : 0; tot += s; }
	total = tot;
	__syncthreads();
	return wbase + inc - v;
}

__global__ void __launch_bounds__(MC_THREADS) k_mc_count(McGrid g, const float* __restrict__ d, uint32_t* __restrict__ cnt_v, uint32_t* __restrict__ cnt_t) {
	__shared__ uint32_t s_wave[2][MC_THREADS / 64];
	const uint64_t base = (uint64_t)blockIdx.x * MC_CHUNK;
	uint32_t nv = 0, nt = 0;
	for (uint32_t k = 0; k < MC_PER_THREAD; ++k) {
		const uint64_t p = base + (uint64_t)k * MC_THREADS + threadIdx.x;
		if (p >= g.n) break;
		uint32_t x, y, z; mc_xyz(g, p, x, y, z);
		nv += __popc(mc_point_flags(g, d, p, x, y, z));
		nt += c_mc_ntri[mc_cube_mask(g, d, p, x, y, z)];
	}
	uint32_t tv, tt;
	(void)block_exclusive_scan(nv, s_wave[0], tv);
	(void)block_exclusive_scan(nt, s_wave[1], tt);
	if (threadIdx.x == 0) { cnt_v[blockIdx.x] = tv; cnt_t[blockIdx.x] = tt; }
}

// Points of a chunk in thread-major order: thread t owns points base + t*8 .. base + t*8 + 7, so the
// workgroup-local scan over threads is the linear point order.
__global__ void __launch_bounds__(MC_THREADS) k_mc_verts(McGrid g, const float* __restrict__ d, const uint32_t* __restrict__ off_v,
                                                         float* __restrict__ verts, uint32_t* __restrict__ vidx) {
	__shared__ uint32_t s_wave[MC_THREADS / 64];
	const uint64_t base = (uint64_t)blockIdx.x * MC_CHUNK + (uint64_t)threadIdx.x * MC_PER_THREAD;
	uint32_t fl[MC_PER_THREAD], nv = 0;
#pragma unroll
	for (uint32_t k = 0; k < MC_PER_THREAD; ++k) {
		const uint64_t p = base + k;
		fl[k] = 0;
		if (p < g.n) { uint32_t x, y, z; mc_xyz(g, p, x, y, z); fl[k] = mc_point_flags(g, d, p, x, y, z); }
		nv += __popc(fl[k]);
	}
	uint32_t tot;
	uint32_t v = off_v[blockIdx.x] + block_exclusive_scan(nv, s_wave, tot);
#pragma unroll
	for (uint32_t k = 0; k < MC_PER_THREAD; ++k) {
		const uint64_t p = base + k;
		if (p >= g.n) break;
		vidx[p] = v;
		if (!fl[k]) continue;
		uint32_t x, y, z; mc_xyz(g, p, x, y, z);
		const float f0 = d[p];
		const uint64_t step[3] = {1, g.rx, (uint64_t)g.rx * g.ry};
#pragma unroll
		for (int a = 0; a < 3; ++a) {
			if (!((fl[k] >> a) & 1)) continue;
			const float f1 = d[p + step[a]];
			const float dt = (g.thresh - f0) / (f1 - f0);
			float q[3] = {(float)x, (float)y, (float)z};
			q[a] = q[a] + dt;
			float* o = verts + 3 * (size_t)v;
			// Vector3f{..}.cwiseProduct(scale) + offset: one FMA per component under nvcc --fmad=true
			o[0] = __builtin_fmaf(q[0], g.scale[0], g.offset[0]);
			o[1] = __builtin_fmaf(q[1], g.scale[1], g.offset[1]);
			o[2] = __builtin_fmaf(q[2], g.scale[2], g.offset[2]);
			++v;
		}
	}
}

__global__ void __launch_bounds__(MC_THREADS) k_mc_faces(McGrid g, const float* __restrict__ d, const uint32_t* __restrict__ off_t,
                                                         const uint32_t* __restrict__ vidx, uint32_t* __restrict__ tris) {
	__shared__ uint32_t s_wave[MC_THREADS / 64];
	const uint64_t base = (uint64_t)blockIdx.x * MC_CHUNK + (uint64_t)threadIdx.x * MC_PER_THREAD;
	uint32_t ms[MC_PER_THREAD], nt = 0;
#pragma unroll
	for (uint32_t k = 0; k < MC_PER_THREAD; ++k) {
		const uint64_t p = base + k;
		ms[k] = 0;
		if (p < g.n) { uint32_t x, y, z; mc_xyz(g, p, x, y, z); ms[k] = mc_cube_mask(g, d, p, x, y, z); }
		nt += c_mc_ntri[ms[k]];
	}
	uint32_t tot;
	uint32_t t = off_t[blockIdx.x] + block_exclusive_scan(nt, s_wave, tot);
	const uint64_t r1 = g.rx, r2 = (uint64_t)g.rx * g.ry;
	// owner point offset (in linear index) and axis of each cube edge (gen_faces local_edges order)
	const uint64_t eoff[12] = {0, 1, r1, 0, r2, 1 + r2, r1 + r2, r2, 0, 1, 1 + r1, r1};
	const uint8_t eax[12] = {0, 1, 0, 1, 0, 1, 0, 1, 2, 2, 2, 2};
#pragma unroll 1
	for (uint32_t k = 0; k < MC_PER_THREAD; ++k) {
		const uint32_t m = ms[k];
		const uint32_t n = c_mc_ntri[m];
		if (!n) continue;
		const uint64_t p = base + k;
		for (uint32_t q = 0; q < 3 * n; ++q) {
			const int e = c_mc_table[m][q];
			const uint64_t o = p + eoff[e];
			uint32_t ox, oy, oz; mc_xyz(g, o, ox, oy, oz);
			const uint32_t fl = mc_point_flags(g, d, o, ox, oy, oz);
			tris[3 * (size_t)t + q] = vidx[o] + __popc(fl & ((1u << eax[e]) - 1));
		}
		t += n;
	}
}

// generate_nerf_network_inputs_from_positions (testbed_nerf.cu:848-854): outward direction from the aabb centre,
// warped position / direction, dt = MIN_CONE_STEPSIZE.
__global__ void k_mesh_coords(uint32_t n, const float* __restrict__ verts, DevDataset ds, float* __restrict__ coords) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const float p[3] = {verts[3 * (size_t)i], verts[3 * (size_t)i + 1], verts[3 * (size_t)i + 2]};
	float d[3] = {p[0] - 0.5f, p[1] - 0.5f, p[2] - 0.5f};
	const float nrm = sqrtf((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
	float* c = coords + (size_t)i * COORD_W;
#pragma unroll
	for (int k = 0; k < 3; ++k) {
		d[k] = nrm > 0.f ? d[k] / nrm : d[k];
		c[k] = (p[k] - ds.aabb_min[k]) / (ds.aabb_max[k] - ds.aabb_min[k]);
		c[4 + k] = (d[k] + 1.0f) * 0.5f;
	}
	c[3] = 0.0f;  // warp_dt(MIN_CONE_STEPSIZE)
}
void launch_mesh_coords(hipStream_t s, uint32_t n, const float* verts, const DevDataset& ds, float* coords) {
	if (n) k_mesh_coords<<<(n + 255) / 256, 256, 0, s>>>(n, verts, ds, coords);
}

// transform_mesh_with_6d (testbed_nerf.cu:109-138): the mesh is extracted in the canonical frame; the
// accumulated movement maps it back to the current frame, v' = R^-1 (v - t) (R^-1 passed in, host-inverted).
__global__ void k_mesh_unmove(uint32_t n, RayMotion inv, float* __restrict__ verts) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	float* v = verts + 3 * (size_t)i;
	const float p[3] = {v[0] - inv.t[0], v[1] - inv.t[1], v[2] - inv.t[2]};
#pragma unroll
	for (int k = 0; k < 3; ++k) v[k] = (inv.R[3 * k] * p[0] + inv.R[3 * k + 1] * p[1]) + inv.R[3 * k + 2] * p[2];
}
void launch_mesh_unmove(hipStream_t s, uint32_t n, const RayMotion& m, float* verts) {
	if (!n || !m.on) return;
	// Eigen Matrix3f::inverse by cofactors
	const float* a = m.R;
	const float c00 = a[4] * a[8] - a[5] * a[7], c01 = a[5] * a[6] - a[3] * a[8], c02 = a[3] * a[7] - a[4] * a[6];
	const float id = 1.0f / ((a[0] * c00 + a[1] * c01) + a[2] * c02);
	RayMotion inv = m;
	inv.R[0] = c00 * id; inv.R[1] = (a[2] * a[7] - a[1] * a[8]) * id; inv.R[2] = (a[1] * a[5] - a[2] * a[4]) * id;
	inv.R[3] = c01 * id; inv.R[4] = (a[0] * a[8] - a[2] * a[6]) * id; inv.R[5] = (a[2] * a[3] - a[0] * a[5]) * id;
	inv.R[6] = c02 * id; inv.R[7] = (a[1] * a[6] - a[0] * a[7]) * id; inv.R[8] = (a[0] * a[4] - a[1] * a[3]) * id;
	k_mesh_unmove<<<(n + 255) / 256, 256, 0, s>>>(n, inv, verts);
}

static McGrid mc_grid(const uint32_t res[3], const float amin[3], const float amax[3], float thresh) {
	McGrid g{};
	g.rx = res[0]; g.ry = res[1]; g.rz = res[2];
	g.n = (uint64_t)res[0] * res[1] * res[2];
	g.thresh = thresh;
	for (int k = 0; k < 3; ++k) { g.scale[k] = (amax[k] - amin[k]) / (float)res[k]; g.offset[k] = amin[k]; }
	return g;
}

uint32_t mc_n_chunks(const uint32_t res[3]) {
	const uint64_t n = (uint64_t)res[0] * res[1] * res[2];
	return (uint32_t)((n + MC_CHUNK - 1) / MC_CHUNK);
}

void launch_mc_count(hipStream_t s, const uint32_t res[3], const float amin[3], const float amax[3], float thresh, const float* density,
                     uint32_t* cnt_v, uint32_t* cnt_t) {
	mc_upload_table();
	const McGrid g = mc_grid(res, amin, amax, thresh);
	k_mc_count<<<mc_n_chunks(res), MC_THREADS, 0, s>>>(g, density, cnt_v, cnt_t);
}
void launch_mc_emit(hipStream_t s, const uint32_t res[3], const float amin[3], const float amax[3], float thresh, const float* density,
                    const uint32_t* off_v, const uint32_t* off_t, float* verts, uint32_t* vidx, uint32_t* tris) {
	const McGrid g = mc_grid(res, amin, amax, thresh);
	k_mc_verts<<<mc_n_chunks(res), MC_THREADS, 0, s>>>(g, density, off_v, verts, vidx);
	k_mc_faces<<<mc_n_chunks(res), MC_THREADS, 0, s>>>(g, density, off_t, vidx, tris);
}

} // namespace neus
