// Microbenchmark: sustained v_mfma_f64_16x16x4f64 rate on gfx950 (ceiling for autocorr_kernel).
// Build: hipcc -O3 --offload-arch=gfx950 benchmarks/mfma_f64_peak.hip -o /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(64) void k(const double* in, double* out, int iters) {
  dbl4 acc[NACC];
  for (int t = 0; t < NACC; ++t) acc[t] = dbl4{0, 0, 0, 0};
  double a = in[threadIdx.x], b = in[threadIdx.x + 64];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < NACC; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
  }
  double s = 0;
  for (int t = 0; t < NACC; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int NACC>
void run(int blocks, int iters) {
  double *in, *out;
  hipMalloc(&in, 128 * 8);
  hipMalloc(&out, (size_t)blocks * 64 * 8);
  double h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0.5 + 0.001 * ((i * 7919) % 997);  // non-trivial operands (DVFS)
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(64), 0, 0, in, out, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(64), 0, 0, in, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double flops = 5.0 * blocks * (double)iters * NACC * 2 * 16 * 16 * 4;
  printf("NACC=%d blocks=%d (waves/SIMD=%.1f): %.2f TFLOP/s\n", NACC, blocks, blocks / 1024.0, flops / (ms * 1e-3) / 1e12);
  hipFree(in);
  hipFree(out);
}

int main() {
  for (int b : {1024, 2048, 4096, 8192}) run<11>(b, 20000);
  run<4>(4096, 40000);
  run<1>(4096, 100000);
  return 0;
}
