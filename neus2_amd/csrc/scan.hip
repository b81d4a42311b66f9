// Device-wide exclusive scans / sums (rocPRIM through hipCUB) for the deterministic
// ray/sample compaction (replacing the reference's atomicAdd appends, testbed_nerf.cu:1421-1428, 1682).
#include "kernels.h"
#include <hipcub/hipcub.hpp>

namespace neus {

size_t scan_temp_bytes(uint32_t n) {
	size_t a = 0, b = 0;
	(void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
	(void)hipcub::DeviceReduce::Sum(nullptr, b, (const float*)nullptr, (float*)nullptr, (int)n);
	return a > b ? a : b;
}
void launch_exclusive_scan(hipStream_t s, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n) {
	(void)hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, s);
}
void launch_sum_f32(hipStream_t s, void* temp, size_t temp_bytes, const float* in, float* out, uint32_t n) {
	(void)hipcub::DeviceReduce::Sum(temp, temp_bytes, in, out, (int)n, s);
}

} // namespace neus
