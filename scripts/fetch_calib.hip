// FETCH_SIZE / WRITE_SIZE calibration by access width (MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of the bytes of
// a 16-B-per-lane streaming read; other widths are uncalibrated).  Streams a 1 GiB array (past the 256 MiB Infinity
// Cache) with 4-, 8- and 16-B loads per lane and stores of the same widths; each kernel name carries its width, so
// rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE per dispatch against the known 1 GiB gives the factor for C1's 4-B-per-lane
// row kernels (k_f16a_*) and the fp64 8-B ones.
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/fetch_calib scripts/fetch_calib.hip
// run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace ... -- scripts/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename V>
__global__ void __launch_bounds__(256) k_read(const V* __restrict__ a, size_t n, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const V v = a[i];
    s += reinterpret_cast<const float*>(&v)[0];
  }
  if (s == 12345.f) out[blockIdx.x] = s;   // keeps the loads; never true for the zero-filled input
}

template <typename V>
__global__ void __launch_bounds__(256) k_write(V* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    V v;
    for (int k = 0; k < (int)(sizeof(V) / 4); ++k) reinterpret_cast<float*>(&v)[k] = (float)k;
    a[i] = v;
  }
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  void* buf = nullptr;
  float* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4096 * sizeof(float)) != hipSuccess) return 1;
  if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
  const dim3 g(4096), b(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_read<float>, g, b, 0, 0, (const float*)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_read<float2>, g, b, 0, 0, (const float2*)buf, bytes / 8, out);
    hipLaunchKernelGGL(k_read<float4>, g, b, 0, 0, (const float4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_write<float>, g, b, 0, 0, (float*)buf, bytes / 4);
    hipLaunchKernelGGL(k_write<float2>, g, b, 0, 0, (float2*)buf, bytes / 8);
    hipLaunchKernelGGL(k_write<float4>, g, b, 0, 0, (float4*)buf, bytes / 16);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("fetch_calib: %zu bytes per kernel, 3 repetitions\n", bytes);
  (void)hipFree(buf);
  (void)hipFree(out);
  return 0;
}
