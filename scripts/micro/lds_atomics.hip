// Microbenchmark: LDS atomic throughput on gfx950 for random addresses within an 8192-entry table
// (the grid-scatter accumulate pattern). Build: hipcc --offload-arch=gfx950 -O3 lds_atomics.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ void __launch_bounds__(256) k(const unsigned* __restrict__ idx, const float* __restrict__ val, float* out, int iters) {
	__shared__ float acc[2 * 8192];
	for (int i = threadIdx.x; i < 2 * 8192; i += blockDim.x) acc[i] = 0.f;
	__syncthreads();
	unsigned e = idx[blockIdx.x * 256 + threadIdx.x] & 8191;
	const float v = val[threadIdx.x];
	for (int it = 0; it < iters; ++it) {
		e = (e * 1664525u + 1013904223u) & 8191;  // lane-random addresses
		if (MODE == 0) { atomicAdd(&acc[e], v); atomicAdd(&acc[8192 + e], v); }                          // 2 x ds_add_f32
		if (MODE == 1) { __builtin_amdgcn_ds_atomic_fadd_v2f16((__attribute__((address_space(3))) h2v*)&acc[e], (h2v){(_Float16)v, (_Float16)v}); }
		if (MODE == 2) { atomicAdd((unsigned*)&acc[e], 3u); atomicAdd((unsigned*)&acc[8192 + e], 5u); }   // 2 x ds_add_u32
		if (MODE == 3) { atomicAdd(&acc[e], v); }                                                          // 1 x ds_add_f32
		if (MODE == 4) { acc[e] += v; acc[8192 + e] += v; }                                                 // plain RMW (racy; rate only)
		if (MODE == 6) { e ^= atomicAdd((unsigned*)&acc[e], 3u) & 1u; }                                  // 1 x ds_add_rtn_u32 (result used)
		if (MODE == 7) { e ^= atomicAdd((unsigned*)&acc[e & 127], 3u) & 1u; }                            // rtn, 128 counters
		if (MODE == 5) { atomicAdd((unsigned long long*)&acc[2 * (e & 4095)], 3ull); atomicAdd((unsigned long long*)&acc[8192 + 2 * (e & 4095)], 5ull); }  // 2 x ds_add_u64
	}
	__syncthreads();
	out[blockIdx.x * 256 + threadIdx.x] = acc[threadIdx.x];
}
int main() {
	const int blocks = 256 * 8, iters = 4096;
	unsigned* idx; float *val, *out;
	hipMalloc(&idx, blocks * 256 * 4); hipMalloc(&val, 256 * 4); hipMalloc(&out, blocks * 256 * 4);
	unsigned* h = new unsigned[blocks * 256];
	for (int i = 0; i < blocks * 256; ++i) h[i] = i * 2654435761u;
	hipMemcpy(idx, h, blocks * 256 * 4, hipMemcpyHostToDevice);
	hipMemset(val, 0, 256 * 4);
	hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
	const char* names[] = {"2x ds_add_f32", "1x ds_pk_add_f16", "2x ds_add_u32", "1x ds_add_f32", "2x plain rmw", "2x ds_add_u64", "1x ds_add_rtn_u32", "1x rtn_u32 128 ctr"};
	for (int m = 0; m < 8; ++m) {
		for (int rep = 0; rep < 2; ++rep) {
			hipEventRecord(a);
			switch (m) {
			case 0: k<0><<<blocks, 256>>>(idx, val, out, iters); break;
			case 1: k<1><<<blocks, 256>>>(idx, val, out, iters); break;
			case 2: k<2><<<blocks, 256>>>(idx, val, out, iters); break;
			case 3: k<3><<<blocks, 256>>>(idx, val, out, iters); break;
			case 4: k<4><<<blocks, 256>>>(idx, val, out, iters); break;
			case 5: k<5><<<blocks, 256>>>(idx, val, out, iters); break;
			case 6: k<6><<<blocks, 256>>>(idx, val, out, iters); break;
			case 7: k<7><<<blocks, 256>>>(idx, val, out, iters); break;
			}
			hipEventRecord(b); hipEventSynchronize(b);
			float ms; hipEventElapsedTime(&ms, a, b);
			const double recs = (double)blocks * 256 * iters;
			if (rep) printf("%-18s %8.3f ms  %7.2f G records/s  (%.2f records/clk/CU at 2.4 GHz)\n", names[m], ms, recs / ms / 1e6, recs / (ms * 1e-3) / 256 / 2.4e9);
		}
	}
	return 0;
}
