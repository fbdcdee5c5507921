// d2h_copy.hip -- probe kernel for benchmarks/d2h_probe.py (not product code): copies n bytes (n % 16 == 0)
// from device memory to a pinned host buffer through its device mapping, 16 bytes per lane per step,
// `wgs` workgroups of 256 threads in a grid-stride loop; nontemporal stores when nt != 0.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void d2h_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       int64_t n16, int nt) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const u32x4 v = src[i];
    if (nt) __builtin_nontemporal_store(v, dst + i);
    else dst[i] = v;
  }
}

extern "C" int d2h_copy(const void* src, void* dst_dev, int64_t n, int wgs, int nt, void* stream) {
  if (n % 16) return -1;
  hipLaunchKernelGGL(d2h_copy_kernel, dim3(wgs), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src,
                     (u32x4*)dst_dev, n / 16, nt);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
