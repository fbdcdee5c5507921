// hip_init_probe.hip -- where a cold process's first HIP operations spend their time (the fixed cost of
// a compute-fdlp-feats JOB before its first batch, make_FDLPspectrum_feats.sh:126-172).  Each letter of
// argv[1] is one step, timed in order, in a fresh process:
//   c hipGetDeviceCount     m hipMalloc 1 MiB       p hipHostMalloc 4 MiB     P hipHostMalloc 128 MiB
//   h hipMemcpy H2D 4 KiB from pageable memory      a hipMemcpyAsync H2D 4 KiB from pinned + sync
//   d hipMemcpy D2H 4 KiB to pageable               s hipStreamCreate         k first kernel launch + sync
//   e hipEventCreate                                 f hipFuncSetAttribute (max dynamic LDS)
//   hipcc --offload-arch=gfx950 -O2 benchmarks/hip_init_probe.hip -o /tmp/hip_init_probe
//   /tmp/hip_init_probe cmhhpakPds
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <vector>

static double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

__global__ void touch(int* p) {
  if (threadIdx.x == 0) p[0] = 1;
}

int main(int argc, char** argv) {
  const char* seq = argc > 1 ? argv[1] : "cmhhpakPds";
  static char page[4096];
  void* d = nullptr;
  void* pin = nullptr;
  void* big = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  int n = 0, rc = 0;
  printf("{\"sequence\": \"%s\", \"steps\": [", seq);
  const double t_all = now_s();
  for (const char* q = seq; *q; ++q) {
    const double t0 = now_s();
    hipError_t e = hipSuccess;
    switch (*q) {
      case 'c': e = hipGetDeviceCount(&n); break;
      case 'm': e = hipMalloc(&d, 1 << 20); break;
      case 'p': e = hipHostMalloc(&pin, 4 << 20, hipHostMallocDefault); break;
      case 'P': e = hipHostMalloc(&big, (size_t)128 << 20, hipHostMallocDefault); break;
      case 'h': e = d ? hipMemcpy(d, page, sizeof page, hipMemcpyHostToDevice) : hipErrorInvalidValue; break;
      case 'd': e = d ? hipMemcpy(page, d, sizeof page, hipMemcpyDeviceToHost) : hipErrorInvalidValue; break;
      case 'a':
        e = d && pin ? hipMemcpyAsync(d, pin, 4096, hipMemcpyHostToDevice, s) : hipErrorInvalidValue;
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        break;
      case 's': e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking); break;
      case 'e': e = hipEventCreateWithFlags(&ev, hipEventDisableTiming); break;
      case 'f': e = hipFuncSetAttribute((const void*)touch, hipFuncAttributeMaxDynamicSharedMemorySize, 65536); break;
      case 'k':
        if (!d) { e = hipErrorInvalidValue; break; }
        touch<<<1, 64, 0, s>>>((int*)d);
        e = hipStreamSynchronize(s);
        break;
      default: e = hipErrorInvalidValue;
    }
    const double dt = now_s() - t0;
    printf("%s[\"%c\", %.5f, %d]", q == seq ? "" : ", ", *q, dt, (int)e);
    if (e != hipSuccess) rc = 1;
  }
  printf("], \"total_s\": %.5f}\n", now_s() - t_all);
  return rc;
}
