// calib_fetch.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for the access
// widths the vote kernel uses (MI355X_MICROARCH.md: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Kernels (each over a 4 GiB buffer, far past the 256 MiB Infinity Cache):
//   k_stream16   16 B/lane coalesced streaming read of 1 GiB   (known bytes)
//   k_gather4    M random u32 gathers (one per lane, distinct lines)
//   k_gather2    M random i16 gathers
//   k_gather4x8  M random runs of 8 consecutive u32 (one 32 B segment)
//   k_store4     M random u32 stores
// Run:  rocprofv3 --pmc FETCH_SIZE -d DIR -- ./calib_fetch
//       rocprofv3 --pmc WRITE_SIZE -d DIR -- ./calib_fetch
// FETCH_SIZE / M is then the counted bytes per random access of that width.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z)
{
	z += 0x9e3779b97f4a7c15ull;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

__global__ void k_stream16(const uint4 *a, uint64_t n16, uint32_t *out)
{
	uint32_t acc = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
		uint4 v = a[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u) out[0] = acc;
}

template <typename T, int RUN>
__global__ void k_gather(const T *a, uint64_t n, uint64_t m, uint32_t *out)
{
	uint32_t acc = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t j = (mix(i) % (n / 64)) * 64;   // distinct 128 B lines (for T=u32) with high probability
#pragma unroll
		for (int r = 0; r < RUN; r++) acc += (uint32_t)a[j + r];
	}
	if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_store4(uint32_t *a, uint64_t n, uint64_t m)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t j = (mix(i ^ 0x5555) % (n / 64)) * 64;
		a[j] = (uint32_t)i;
	}
}

int main()
{
	const uint64_t bytes = 4ull << 30;
	const uint64_t M = 16ull << 20;   // random accesses per gather kernel
	void *buf;
	uint32_t *out;
	CHK(hipMalloc(&buf, bytes));
	CHK(hipMalloc(&out, 64));
	CHK(hipMemset(buf, 1, bytes));
	CHK(hipDeviceSynchronize());
	dim3 g(256 * 16), b(256);
	hipLaunchKernelGGL(k_stream16, g, b, 0, 0, (const uint4 *)buf, (1ull << 30) / 16, out);
	hipLaunchKernelGGL((k_gather<uint32_t, 1>), g, b, 0, 0, (const uint32_t *)buf, bytes / 4, M, out);
	hipLaunchKernelGGL((k_gather<int16_t, 1>), g, b, 0, 0, (const int16_t *)buf, bytes / 2, M, out);
	hipLaunchKernelGGL((k_gather<uint32_t, 8>), g, b, 0, 0, (const uint32_t *)buf, bytes / 4, M, out);
	hipLaunchKernelGGL(k_store4, g, b, 0, 0, (uint32_t *)buf, bytes / 4, M);
	CHK(hipDeviceSynchronize());
	printf("calib_fetch: stream16 bytes=%llu, gathers M=%llu each\n", (unsigned long long)(1ull << 30),
	       (unsigned long long)M);
	CHK(hipFree(buf));
	CHK(hipFree(out));
	return 0;
}
