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
// The triangle table is generated here (mc_build_table), not copied: per corner mask, crossing edges are
// joined face by face into segments (a face with four crossings cuts off each set corner separately, a
// symmetric rule, so neighbouring cubes agree and the mesh is watertight), segments are oriented with the
// set corners on their left seen from outside the cube, chained into loops and fanned from the loop's
// lowest edge id. oracle/mc_table.py restates the same construction for the parity tests.
#pragma clang fp contract(off)
#include "kernels.h"

#include <cmath>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace neus {

constexpr int MC_MAX_TRIS = 6;
constexpr int MC_ROW = 3 * MC_MAX_TRIS + 1;
__constant__ int8_t c_mc_table[256][MC_ROW];
__constant__ uint8_t c_mc_ntri[256];

// corner k -> offset bits (x, y, z); edge e -> corners; edge e -> owning grid point offset and axis
static const int CORNER[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};
static const int EDGE[12][2] = {{0, 1}, {1, 2}, {3, 2}, {0, 3}, {4, 5}, {5, 6}, {7, 6}, {4, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
static const int FACE[6][4] = {{0, 3, 7, 4}, {1, 2, 6, 5}, {0, 1, 5, 4}, {3, 2, 6, 7}, {0, 1, 2, 3}, {4, 5, 6, 7}};
static const int FACE_N[6][3] = {{-1, 0, 0}, {1, 0, 0}, {0, -1, 0}, {0, 1, 0}, {0, 0, -1}, {0, 0, 1}};

static int edge_of(int a, int b) {
	for (int e = 0; e < 12; ++e)
		if ((EDGE[e][0] == a && EDGE[e][1] == b) || (EDGE[e][0] == b && EDGE[e][1] == a)) return e;
	throw std::runtime_error("mc table: not an edge");
}

// Host: the case table (see the file comment); rows are edge triples terminated by -1.
static void mc_build_table(int8_t table[256][MC_ROW], uint8_t ntri[256]) {
	for (int m = 0; m < 256; ++m) {
		for (int k = 0; k < MC_ROW; ++k) table[m][k] = -1;
		ntri[m] = 0;
		if (m == 0 || m == 255) continue;
		int nxt[12];
		for (int e = 0; e < 12; ++e) nxt[e] = -1;
		auto in = [&](int c) { return (m >> c) & 1; };
		auto mid2 = [&](int e, int d) { return CORNER[EDGE[e][0]][d] + CORNER[EDGE[e][1]][d]; };  // 2 x midpoint
		auto add_seg = [&](int f, int a, int b, int c) {
			// cross(n, B - A) . (P - A) > 0 keeps the set corner P on the left (all in 2x units)
			float A[3], B[3], P[3], n[3];
			for (int d = 0; d < 3; ++d) { A[d] = (float)mid2(a, d); B[d] = (float)mid2(b, d); P[d] = 2.0f * CORNER[c][d]; n[d] = (float)FACE_N[f][d]; }
			const float u[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]};
			const float cr[3] = {n[1] * u[2] - n[2] * u[1], n[2] * u[0] - n[0] * u[2], n[0] * u[1] - n[1] * u[0]};
			const float s = cr[0] * (P[0] - A[0]) + cr[1] * (P[1] - A[1]) + cr[2] * (P[2] - A[2]);
			if (s < 0) std::swap(a, b);
			if (nxt[a] >= 0) throw std::runtime_error("mc table: edge with two successors");
			nxt[a] = b;
		};
		for (int f = 0; f < 6; ++f) {
			const int* cy = FACE[f];
			int n_set = 0, set_c[4];
			for (int i = 0; i < 4; ++i) if (in(cy[i])) set_c[n_set++] = cy[i];
			if (n_set == 0 || n_set == 4) continue;
			bool adjacent = false;
			for (int i = 0; i < 4; ++i) adjacent |= in(cy[i]) && in(cy[(i + 1) % 4]);
			if (n_set == 2 && !adjacent) {
				for (int q = 0; q < 2; ++q) {
					int i = 0;
					while (cy[i] != set_c[q]) ++i;
					add_seg(f, edge_of(set_c[q], cy[(i + 3) % 4]), edge_of(set_c[q], cy[(i + 1) % 4]), set_c[q]);
				}
			} else {
				int xs[2], nx = 0;
				for (int i = 0; i < 4; ++i) if (in(cy[i]) != in(cy[(i + 1) % 4])) xs[nx++] = edge_of(cy[i], cy[(i + 1) % 4]);
				if (nx != 2) throw std::runtime_error("mc table: face with odd crossings");
				add_seg(f, xs[0], xs[1], set_c[0]);
			}
		}
		bool seen[12] = {};
		int nt = 0;
		for (int st = 0; st < 12; ++st) {
			if (nxt[st] < 0 || seen[st]) continue;
			int loop[12], len = 0, v = st;
			do { loop[len++] = v; seen[v] = true; v = nxt[v]; } while (v != st);
			int k = 0;
			for (int i = 1; i < len; ++i) if (loop[i] < loop[k]) k = i;
			int r[12];
			for (int i = 0; i < len; ++i) r[i] = loop[(k + i) % len];
			for (int i = 1; i + 1 < len; ++i) {
				if (nt >= MC_MAX_TRIS) throw std::runtime_error("mc table: too many triangles");
				table[m][3 * nt] = (int8_t)r[0]; table[m][3 * nt + 1] = (int8_t)r[i]; table[m][3 * nt + 2] = (int8_t)r[i + 1];
				++nt;
			}
		}
		ntri[m] = (uint8_t)nt;
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
