// Microbenchmark: instruction mixes of ac_vsweep_kernel's inner block on gfx950 (one wave = 4 units of
// 16 lanes; per block 100 fp64 FMAs per lane into 10 accumulators).
//   fma   : broadcasts from registers (no DPP), window in registers
//   dpp   : 10 row_newbcast broadcasts per block (bound_ctrl), window in registers
//   lds   : dpp + the window's A new values and cur read from an LDS ring each block (two banks)
// Build: hipcc -O3 --offload-arch=gfx950 benchmarks/vsweep_mix.hip -o benchmarks/vsweep_mix
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int A = 10;
template <int K>
__device__ __forceinline__ double bc(double v) { return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + K, 0xF, 0xF, true); }
template <int V = 0>
__device__ __forceinline__ void bcast_all(double (&bb)[A], double cur) {
  if constexpr (V < A) { bb[V] = bc<V>(cur); bcast_all<V + 1>(bb, cur); }
}
__device__ __forceinline__ void block(double (&acc)[A], const double (&bb)[A], const double (&lo)[A], const double (&hi)[A]) {
#pragma unroll
  for (int v = 0; v < A; ++v)
#pragma unroll
    for (int u = 0; u < A; ++u) acc[u] = fma(bb[v], (v + u < A) ? lo[v + u] : hi[v + u - A], acc[u]);
}

template <int MODE>
__global__ __launch_bounds__(64, 2) void k(const double* in, double* out, int iters) {
  __shared__ double ring[4][528];
  const int l = threadIdx.x & 15, row = threadIdx.x >> 4;
  for (int q = l; q < 528; q += 16) ring[row][q] = in[(q + row) & 255] + 1e-3 * q;
  __syncthreads();
  double acc[A], X[A], Y[A], bb[A];
  for (int u = 0; u < A; ++u) { acc[u] = 0; X[u] = in[u + l]; Y[u] = in[u + 20 + l]; bb[u] = in[u + 40]; }
  double cur = in[l];
  for (int it = 0; it < iters; ++it) {
    const int n0 = (it * 2 * A) & 511;
    if constexpr (MODE == 2) {
      const int base = (n0 + A * l) & 510;
#pragma unroll
      for (int q = 0; q < A; ++q) X[q] = ring[row][base + q];
      cur = ring[row][(n0 + l) & 511];
    }
    if constexpr (MODE >= 1) bcast_all(bb, cur); else { cur = cur * 0.9999; bb[0] = cur; }
    block(acc, bb, X, Y);
    if constexpr (MODE == 2) {
      const int base = (n0 + A + A * l) & 510;
#pragma unroll
      for (int q = 0; q < A; ++q) Y[q] = ring[row][base + q];
      cur = ring[row][(n0 + A + l) & 511];
    }
    if constexpr (MODE >= 1) bcast_all(bb, cur); else { cur = cur * 0.9999; bb[1] = cur; }
    block(acc, bb, Y, X);
  }
  double s = 0;
  for (int u = 0; u < A; ++u) s += acc[u];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

// ldspf: as lds, but each block's window (and broadcast source) is read one block ahead into a third
// register bank, so the wait at a block head is for reads issued a whole block earlier
__global__ __launch_bounds__(64, 2) void kpf(const double* in, double* out, int iters) {
  __shared__ double ring[4][528];
  const int l = threadIdx.x & 15, row = threadIdx.x >> 4;
  for (int q = l; q < 528; q += 16) ring[row][q] = in[(q + row) & 255] + 1e-3 * q;
  __syncthreads();
  double acc[A], B0[A], B1[A], B2[A], bb[A];
  for (int u = 0; u < A; ++u) { acc[u] = 0; B0[u] = in[u + l]; B2[u] = in[u + 20 + l]; bb[u] = in[u + 40]; }
  double cur = in[l], curn;
  auto rd = [&](double (&dst)[A], double& c, int n0) {
    const int base = (n0 + A * l) & 510;
#pragma unroll
    for (int q = 0; q < A; ++q) dst[q] = ring[row][base + q];
    c = ring[row][(n0 + l) & 511];
  };
  for (int it = 0; it < iters; it += 3) {
    const int n0 = (it * A) & 511;
    rd(B1, curn, n0 + A);
    bcast_all(bb, cur);
    block(acc, bb, B0, B2);
    cur = curn;
    rd(B2, curn, n0 + 2 * A);
    bcast_all(bb, cur);
    block(acc, bb, B1, B0);
    cur = curn;
    rd(B0, curn, n0 + 3 * A);
    bcast_all(bb, cur);
    block(acc, bb, B2, B1);
    cur = curn;
  }
  double s = 0;
  for (int u = 0; u < A; ++u) s += acc[u];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

// dppwin: the window moves one lane down per block by DPP (row_shr:1, two v_mov_b32_dpp per double); only
// lane 0 of each row reads its 10 new values (and the broadcast source) from the LDS ring
template <int SH = 0>
__device__ __forceinline__ void shift_in(double (&dst)[A], const double (&src)[A], const double (&nv)[A]) {
#pragma unroll
  for (int q = 0; q < A; ++q) dst[q] = __builtin_amdgcn_update_dpp(nv[q], src[q], 0x111, 0xF, 0xF, false);
}
__global__ __launch_bounds__(64, 2) void kdw(const double* in, double* out, int iters) {
  __shared__ double ring[4][528];
  const int l = threadIdx.x & 15, row = threadIdx.x >> 4;
  for (int q = l; q < 528; q += 16) ring[row][q] = in[(q + row) & 255] + 1e-3 * q;
  __syncthreads();
  double acc[A], X[A], Y[A], bb[A], nv[A];
  for (int u = 0; u < A; ++u) { acc[u] = 0; X[u] = in[u + l]; Y[u] = in[u + 20 + l]; bb[u] = in[u + 40]; nv[u] = 0; }
  double cur = in[l];
  for (int it = 0; it < iters; ++it) {
    const int n0 = (it * 2 * A) & 511;
    if (l == 0) {
#pragma unroll
      for (int q = 0; q < A; ++q) nv[q] = ring[row][(n0 + q) & 510];
    }
    cur = ring[row][(n0 + l) & 511];
    shift_in(Y, X, nv);  // new lo (Y) from the old lo (X) of the lane below; X becomes hi
    bcast_all(bb, cur);
    block(acc, bb, Y, X);
    if (l == 0) {
#pragma unroll
      for (int q = 0; q < A; ++q) nv[q] = ring[row][(n0 + A + q) & 510];
    }
    cur = ring[row][(n0 + A + l) & 511];
    shift_in(X, Y, nv);
    bcast_all(bb, cur);
    block(acc, bb, X, Y);
  }
  double s = 0;
  for (int u = 0; u < A; ++u) s += acc[u];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int MODE>
static void launch(dim3 g, const double* in, double* out, int iters) {
  if constexpr (MODE == 4) hipLaunchKernelGGL(kdw, g, dim3(64), 0, 0, in, out, iters);
  else if constexpr (MODE == 3) hipLaunchKernelGGL(kpf, g, dim3(64), 0, 0, in, out, iters);
  else hipLaunchKernelGGL(k<MODE>, g, dim3(64), 0, 0, in, out, iters);
}
template <int MODE>
static void run(const char* name, const double* in, double* out, int waves, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  launch<MODE>(dim3(waves), in, out, 10);
  hipEventRecord(a);
  launch<MODE>(dim3(waves), in, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double flops = (MODE == 3 ? 1.0 : 2.0) * 2 * A * A * 64.0 * waves * (double)iters;  // kpf: one block per it
  printf("%-6s waves %5d  %.3f ms  %.1f TFLOP/s\n", name, waves, ms, flops / ms / 1e9);
}

int main() {
  double *in, *out;
  hipMalloc(&in, 4096 * sizeof(double));
  hipMalloc(&out, 65536 * 64 * sizeof(double));
  double h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = 1.0 + 1e-6 * i;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  for (int waves : {1024, 2048, 4096, 8192}) {
    run<0>("fma", in, out, waves, 20000);
    run<1>("dpp", in, out, waves, 20000);
    run<2>("lds", in, out, waves, 20000);
    run<3>("ldspf", in, out, waves, 40002);
    run<4>("dppwin", in, out, waves, 20000);
  }
  return 0;
}
