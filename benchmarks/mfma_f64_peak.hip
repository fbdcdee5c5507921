// Microbenchmark: sustained v_mfma_f64_16x16x4f64 rate on gfx950 (ceiling for autocorr_kernel).
// Variants: (a) register operands; (b) operands re-read from LDS every k-step like autocorr_kernel.
// Build: hipcc -O3 --offload-arch=gfx950 benchmarks/mfma_f64_peak.hip -o benchmarks/mfma_f64_peak
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(64) void k_reg(const double* in, double* out, int iters) {
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

// distinct B registers per accumulator (the autocorr pattern: shared A, NACC different B)
template <int NACC>
__global__ __launch_bounds__(64) void k_regb(const double* in, double* out, int iters) {
  dbl4 acc[NACC];
  double b[NACC];
  for (int t = 0; t < NACC; ++t) {
    acc[t] = dbl4{0, 0, 0, 0};
    b[t] = in[(threadIdx.x + 7 * t) & 127];
  }
  double a = in[threadIdx.x];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < NACC; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[t], acc[t], 0, 0, 0);
    a = a * 0.999999;  // keep operands live and changing
  }
  double s = 0;
  for (int t = 0; t < NACC; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

// MFMA-only waves next to VALU-only fp64 FMA waves (is the VALU pipe free while MFMA runs?)
__global__ __launch_bounds__(64) void k_valu(const double* in, double* out, int iters) {
  double x0 = in[threadIdx.x], x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = in[threadIdx.x + 64];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      x0 = fma(x0, y, 1e-9); x1 = fma(x1, y, 1e-9); x2 = fma(x2, y, 1e-9); x3 = fma(x3, y, 1e-9);
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = x0 + x1 + x2 + x3;
}

template <int NACC>
__global__ __launch_bounds__(64, 4) void k_lds(const double* in, double* out, int iters) {
  __shared__ double xs[2048];
  for (int q = threadIdx.x; q < 2048; q += 64) xs[q] = in[q & 127] + 1e-3 * q;
  __syncthreads();
  dbl4 acc[NACC];
  for (int t = 0; t < NACC; ++t) acc[t] = dbl4{0, 0, 0, 0};
  const int l = threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    const double* w = xs + ((64 * it) & 1023) + l;
    const double a = w[0];
#pragma unroll
    for (int t = 0; t < NACC; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, w[16 * t], acc[t], 0, 0, 0);
  }
  double s = 0;
  for (int t = 0; t < NACC; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, int nacc, int blocks, int iters) {
  double *in, *out;
  (void)hipMalloc(&in, 128 * 8);
  (void)hipMalloc(&out, (size_t)blocks * 64 * 8);
  double h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0.5 + 0.001 * ((i * 7919) % 997);  // non-trivial operands (DVFS)
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, in, out, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, in, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  double flops = 5.0 * blocks * (double)iters * nacc * 2 * 16 * 16 * 4;
  printf("%s NACC=%d blocks=%d (waves/SIMD=%.1f): %.2f TFLOP/s  (%.2f ms/launch)\n", name, nacc, blocks,
         blocks / 1024.0, flops / (ms * 1e-3) / 1e12, ms / 5);
  (void)hipFree(in);
  (void)hipFree(out);
}

int main() {
  for (int b : {2048, 4096}) run("reg", k_reg<11>, 11, b, 20000);
  for (int b : {2048, 4096}) run("regb", k_regb<11>, 11, b, 20000);
  run("regb", k_regb<16>, 16, 4096, 15000);
  run("lds", k_lds<11>, 11, 4096, 20000);
  {
    // VALU fp64 FMA peak
    double *in, *out;
    (void)hipMalloc(&in, 128 * 8);
    (void)hipMalloc(&out, 8192 * 64 * 8);
    (void)hipMemset(in, 0, 128 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_valu, dim3(8192), dim3(64), 0, 0, in, out, 2000);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_valu, dim3(8192), dim3(64), 0, 0, in, out, 2000);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("valu fp64 fma: %.2f TFLOP/s\n", 8192.0 * 64 * 2000 * 64 * 2 / (ms * 1e-3) / 1e12);
    // concurrent: MFMA kernel on stream 1, VALU kernel on stream 2
    hipStream_t s1, s2;
    (void)hipStreamCreate(&s1);
    (void)hipStreamCreate(&s2);
    (void)hipEventRecord(e0, 0);
    (void)hipDeviceSynchronize();
    hipEvent_t a0, a1, b0, b1;
    (void)hipEventCreate(&a0); (void)hipEventCreate(&a1); (void)hipEventCreate(&b0); (void)hipEventCreate(&b1);
    (void)hipEventRecord(a0, s1);
    hipLaunchKernelGGL(k_regb<11>, dim3(2048), dim3(64), 0, s1, in, out, 20000);
    (void)hipEventRecord(a1, s1);
    (void)hipEventRecord(b0, s2);
    hipLaunchKernelGGL(k_valu, dim3(2048), dim3(64), 0, s2, in, out, 2000);
    (void)hipEventRecord(b1, s2);
    (void)hipDeviceSynchronize();
    float ma, mb;
    (void)hipEventElapsedTime(&ma, a0, a1);
    (void)hipEventElapsedTime(&mb, b0, b1);
    printf("concurrent: mfma %.2f ms (%.2f TF), valu %.2f ms (%.2f TF)\n", ma,
           2048.0 * 20000 * 11 * 2048 / (ma * 1e-3) / 1e12, mb, 2048.0 * 64 * 2000 * 64 * 2 / (mb * 1e-3) / 1e12);
  }
  return 0;
}
