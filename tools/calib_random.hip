// calib_random.hip -- the random-line ceiling of MI355X HBM for the probe kernel's access shape:
// every lane reads whole L-byte lines at uniformly random L-aligned addresses of a buffer far
// larger than the Infinity Cache (8 GiB), F independent lines in flight per lane, 8 waves per
// SIMD (the probe kernel's occupancy).  Reports lines/s and GB/s per (L, F), timed with HIP
// events over repeated launches.  Also: a dependent chain (each address from the previous
// line's data), the one-line-at-a-time latency a serial probe pays.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/calib_random tools/calib_random.hip
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

template <int L, int F>
__global__ void __launch_bounds__(256, 8) k_rand(const uint4 *a, uint64_t nlines, uint32_t iters, uint32_t *out)
{
	constexpr int Q = L / 16;
	uint32_t acc = 0;
	const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
	for (uint32_t it = 0; it < iters; it++) {
		uint4 v[F][Q];
#pragma unroll
		for (int f = 0; f < F; f++) {
			const uint64_t line = mix(t * 1315423911ull + it * 2654435761ull + f) % nlines;
#pragma unroll
			for (int q = 0; q < Q; q++) v[f][q] = a[line * Q + q];
		}
#pragma unroll
		for (int f = 0; f < F; f++)
#pragma unroll
			for (int q = 0; q < Q; q++) acc ^= v[f][q].x ^ v[f][q].w;
	}
	if (acc == 0x12345678u) out[0] = acc;
}

// dependent chain: the next line index comes from the loaded data
__global__ void __launch_bounds__(256, 8) k_chain(const uint4 *a, uint64_t nlines, uint32_t iters, uint32_t *out)
{
	uint64_t line = mix(blockIdx.x * 256ull + threadIdx.x) % nlines;
	uint32_t acc = 0;
	for (uint32_t it = 0; it < iters; it++) {
		const uint4 v0 = a[line * 4], v3 = a[line * 4 + 3];
		acc ^= v3.w;
		line = mix(line ^ v0.x ^ it) % nlines;
	}
	if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint32_t *a, uint64_t n)
{
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) a[i] = (uint32_t)mix(i);
}

template <int L, int F>
static int run(const uint4 *a, uint64_t bytes, int ncu, uint32_t *out)
{
	const uint64_t nlines = bytes / L;
	const uint32_t iters = 64;
	dim3 g(ncu * 8), b(256);
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	hipLaunchKernelGGL((k_rand<L, F>), g, b, 0, 0, a, nlines, iters, out);
	CHK(hipEventRecord(e0, 0));
	const int reps = 5;
	for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k_rand<L, F>), g, b, 0, 0, a, nlines, iters, out);
	CHK(hipEventRecord(e1, 0));
	CHK(hipEventSynchronize(e1));
	float ms = 0;
	CHK(hipEventElapsedTime(&ms, e0, e1));
	const double lines = (double)reps * g.x * 256.0 * iters * F;
	printf("random %3d-B lines, %d in flight/lane: %6.2f G lines/s  %6.1f GB/s  (%.2f ms/launch)\n", L, F,
	       lines / (ms * 1e-3) / 1e9, lines * L / (ms * 1e-3) / 1e9, ms / reps);
	return 0;
}

int main()
{
	const uint64_t bytes = 8ull << 30;
	void *buf;
	uint32_t *out;
	hipDeviceProp_t prop;
	CHK(hipGetDeviceProperties(&prop, 0));
	const int ncu = prop.multiProcessorCount;
	CHK(hipMalloc(&buf, bytes));
	CHK(hipMalloc(&out, 64));
	hipLaunchKernelGGL(k_fill, dim3(ncu * 16), dim3(256), 0, 0, (uint32_t *)buf, bytes / 4);
	CHK(hipDeviceSynchronize());
	const uint4 *a = (const uint4 *)buf;
	run<32, 1>(a, bytes, ncu, out);
	run<64, 1>(a, bytes, ncu, out);
	run<64, 2>(a, bytes, ncu, out);
	run<64, 4>(a, bytes, ncu, out);
	run<128, 1>(a, bytes, ncu, out);
	run<128, 2>(a, bytes, ncu, out);
	{
		hipEvent_t e0, e1;
		CHK(hipEventCreate(&e0));
		CHK(hipEventCreate(&e1));
		const uint32_t iters = 64;
		dim3 g(ncu * 8), b(256);
		CHK(hipEventRecord(e0, 0));
		hipLaunchKernelGGL(k_chain, g, b, 0, 0, a, bytes / 64, iters, out);
		CHK(hipEventRecord(e1, 0));
		CHK(hipEventSynchronize(e1));
		float ms = 0;
		CHK(hipEventElapsedTime(&ms, e0, e1));
		printf("dependent chain of 64-B lines, 8 waves/SIMD: %.2f us per step, %.2f G lines/s\n", ms * 1e3 / iters,
		       (double)g.x * 256 * iters / (ms * 1e-3) / 1e9);
	}
	CHK(hipFree(buf));
	return 0;
}
