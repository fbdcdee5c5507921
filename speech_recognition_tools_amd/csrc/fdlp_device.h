// fdlp_device.h -- device-side helpers shared by the gfx950 kernel translation units
// (fdlp_dct.hip, fdlp_autocorr.hip, fdlp_lpc.hip, fdlp_misc.hip): complex arithmetic and the LDS
// Stockham DFT, the XCD-aware grid mapping, wave / DPP-row reductions, DPP-broadcast FMAs and the
// counted LDS loads.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "fdlp_internal.h"
#include "fdlp_mathtab.h"

namespace fdlp {

typedef double dbl4 __attribute__((ext_vector_type(4)));

// -----------------------------------------------------------------------------------------
// complex helpers
// -----------------------------------------------------------------------------------------
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }

// R-point forward DFT in registers; roots from the length-n table (omega_n^q), stride n/R.
template <int R>
__device__ __forceinline__ void small_dft(double2* v, const double2* __restrict__ om, int n) {
  if constexpr (R == 2) {
    double2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = make_double2(a.x - b.x, a.y - b.y);
  } else if constexpr (R == 4) {
    double2 a0 = cadd(v[0], v[2]), a1 = make_double2(v[0].x - v[2].x, v[0].y - v[2].y);
    double2 b0 = cadd(v[1], v[3]), b1 = make_double2(v[1].x - v[3].x, v[1].y - v[3].y);
    // forward: multiply b1 by -i
    double2 b1m = make_double2(b1.y, -b1.x);
    v[0] = cadd(a0, b0);
    v[2] = make_double2(a0.x - b0.x, a0.y - b0.y);
    v[1] = cadd(a1, b1m);
    v[3] = make_double2(a1.x - b1m.x, a1.y - b1m.y);
  } else {
    double2 out[R];
    const int st = n / R;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      double2 acc = v[0];
#pragma unroll
      for (int p = 1; p < R; ++p) acc = cadd(acc, cmul(v[p], om[((p * q) % R) * st]));
      out[q] = acc;
    }
#pragma unroll
    for (int q = 0; q < R; ++q) v[q] = out[q];
  }
}

// One Stockham autosort stage of radix R over `ncols` interleaved columns of length n.
// in/out index = pos * ncols + col.  Ns = product of the radices already applied.
template <int R>
__device__ inline void stockham_stage(const double2* __restrict__ in, double2* __restrict__ out,
                               const double2* __restrict__ om, int n, int ncols, int Ns) {
  const int nb = n / R;
  const int total = nb * ncols;
  const int tw0 = n / (Ns * R);
  const float inv_ns = 1.0f / (float)Ns;
  for (int b = threadIdx.x; b < total; b += blockDim.x) {
    const int col = b % ncols;
    const int j = b / ncols;
    // j / Ns without an integer division (j < 512: the float quotient is off by at most one)
    int jq = (int)((float)j * inv_ns);
    jq += (jq + 1) * Ns <= j;
    jq -= jq * Ns > j;
    const int k = j - jq * Ns;
    double2 v[R];
    const int twstep = tw0 * k;  // omega_{Ns*R}^{k*r} = omega_n^{k*r*n/(Ns*R)}; twstep * r < n
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double2 x = in[(j + r * nb) * ncols + col];
      v[r] = (r == 0) ? x : cmul(x, om[twstep * r]);
    }
    small_dft<R>(v, om, n);
    const int idxD = jq * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) out[(idxD + r * Ns) * ncols + col] = v[r];
  }
}

// Full length-n DFT of ncols columns resident in LDS (ping-pong a <-> b).  Returns the buffer
// holding the result.
__device__ inline double2* lds_dft(double2* a, double2* b, const double2* om, const DftPlan& d, int ncols) {
  int Ns = 1;
  for (int s = 0; s < d.nrad; ++s) {
    const int R = d.rad[s];
    switch (R) {
      case 2: stockham_stage<2>(a, b, om, d.n, ncols, Ns); break;
      case 3: stockham_stage<3>(a, b, om, d.n, ncols, Ns); break;
      case 4: stockham_stage<4>(a, b, om, d.n, ncols, Ns); break;
      case 5: stockham_stage<5>(a, b, om, d.n, ncols, Ns); break;
      case 7: stockham_stage<7>(a, b, om, d.n, ncols, Ns); break;
      default: break;  // rejected at plan creation
    }
    __syncthreads();
    Ns *= R;
    double2* t = a; a = b; b = t;
  }
  return a;
}

constexpr int kDftCols = 8;     // columns (rows) per workgroup in the two DFT passes

// Workgroup b is dispatched to XCD b % 8.  Giving every XCD a contiguous run of work items keeps
// the items that read the same frame (its D row) on one L2 instead of pulling the row into all
// eight.  Grid = 8 * ceil(total / 8); the padding workgroups get an index >= total.
__device__ __forceinline__ int xcd_item() {
  const int per = gridDim.x / kXcds;
  return (int)(blockIdx.x % kXcds) * per + (int)(blockIdx.x / kXcds);
}
static inline int xcd_grid(int total) { return (total + kXcds - 1) / kXcds * kXcds; }

// -----------------------------------------------------------------------------------------
// Device-side range checks ("HIP bounds-check debug build"): a library built with
// -DFDLP_DEVICE_CHECKS=1 (python _build.py --out lib/libfdlp_checks.so -DFDLP_DEVICE_CHECKS=1) evaluates
// FDLP_CHECK(cond) in the index-heavy kernels -- frame descriptors, reflected sample indices, LDS image
// and exchange indices, straddle windows, OLA slices -- and counts the violations in a per-translation-unit
// device counter (with the last failing source line) instead of trapping: a trap would end the process in
// the middle of a batch and leave nothing to read.  fdlp_device_checks() reads (and resets) the counters.
// In the default build FDLP_CHECK compiles to nothing.
// -----------------------------------------------------------------------------------------
#ifndef FDLP_DEVICE_CHECKS
#define FDLP_DEVICE_CHECKS 0
#endif
#if FDLP_DEVICE_CHECKS
static __device__ unsigned int fdlp_check_state[2];  // violations, largest failing line
#define FDLP_CHECK(cond)                                                   \
  do {                                                                     \
    if (!(cond)) {                                                         \
      atomicAdd(&fdlp_check_state[0], 1u);                                 \
      atomicMax(&fdlp_check_state[1], (unsigned int)__LINE__);             \
    }                                                                      \
  } while (0)
// host: this translation unit's counters (violations, line), optionally reset
static inline hipError_t fdlp_checks_local(unsigned int* v, bool reset) {
  hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(fdlp_check_state), 2 * sizeof(unsigned int));
  if (e == hipSuccess && reset) {
    const unsigned int z[2] = {0u, 0u};
    e = hipMemcpyToSymbol(HIP_SYMBOL(fdlp_check_state), z, 2 * sizeof(unsigned int));
  }
  return e;
}
#else
#define FDLP_CHECK(cond) \
  do {                   \
  } while (0)
static inline hipError_t fdlp_checks_local(unsigned int* v, bool) {
  v[0] = v[1] = 0u;
  return hipSuccess;
}
#endif

// -----------------------------------------------------------------------------------------
// wave-level helpers
// -----------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// -----------------------------------------------------------------------------------------
// 16-lane (one DPP row) helpers: an item is owned by a row of 16 lanes, 4 items per wave.
// -----------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  // every control used here has an in-row source for every lane, so no 'old' value is needed
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// sum over the 16 lanes of a DPP row; every lane gets the same (bitwise) value
__device__ __forceinline__ double row_sum16(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ void wave_lds_sync() {
  // LDS ops of one wave complete in order; this only stops the compiler from reordering
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 8-lane (half DPP row) sum; every lane of the half gets the same (bitwise) value
__device__ __forceinline__ double sum8(double v) {  // over the 8 lanes of a half DPP row
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror: lane i <-> 7-i inside each 8-lane half
  return v;
}

template <int K>
__device__ __forceinline__ double row_bcast(double v) {
  // row_newbcast:K; every lane has a source, and bound_ctrl spares the 'old' operand (no init, no nops)
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + K, 0xF, 0xF, true);
}

// acc += s[n0+V] * w with s[n0+V] read from lane V of the row by the FMA itself (DP ALU DPP:
// v_fmac_f64 takes row_newbcast on its first source), so a block costs A^2 FMAs and no moves
template <int V>
__device__ __forceinline__ void fmac_bcast(double& acc, double cur, double w) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(cur), "v"(w), "n"(V));
}

// LDS read of one double at a compile-time byte offset from a per-lane byte address.  Plain
// ds_read_b64 (2 LDS cycles per wave when conflict-free); the compiler would otherwise merge the
// window into ds_read2_b64 / ds_read_b128, which run at half rate or 2-way conflicted here.
// The caller waits with lds_wait() before using the values.
template <int OFF>
__device__ __forceinline__ double lds_ld(uint32_t addr) {
  double v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// 16 alpha values alpha[OFF - j] (j < 16, byte offsets from the lane's LDS address `addr`) as single
// ds_read_b64: 2 LDS cycles per wave-instruction, where the compiler's merged ds_read2_b64 takes 8 for
// two (MI355X_MICROARCH.md LDS table).  The asm results look ready to the compiler, so the caller
// waits (lgkm_wait) before the FMAs that read them.
template <int OFF, int J = 0>
__device__ __forceinline__ void lds_load16(double (&v)[16], uint32_t addr) {
  if constexpr (J < 16) {
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v[J]) : "v"(addr), "i"(8 * (OFF - J)) : "memory");
    lds_load16<OFF, J + 1>(v, addr);
  }
}
template <int N>
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }

// Radix-R butterfly (forward DFT) in registers with literal roots of unity (R = 2, 3, 4, 5)
template <int R>
__device__ __forceinline__ void bfly_c(double2 (&v)[R]) {
  if constexpr (R == 2) {
    const double2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = make_double2(a.x - b.x, a.y - b.y);
  } else if constexpr (R == 4) {
    const double2 a0 = cadd(v[0], v[2]), a1 = make_double2(v[0].x - v[2].x, v[0].y - v[2].y);
    const double2 b0 = cadd(v[1], v[3]), b1 = make_double2(v[1].x - v[3].x, v[1].y - v[3].y);
    const double2 b1m = make_double2(b1.y, -b1.x);  // -i b1
    v[0] = cadd(a0, b0);
    v[2] = make_double2(a0.x - b0.x, a0.y - b0.y);
    v[1] = cadd(a1, b1m);
    v[3] = make_double2(a1.x - b1m.x, a1.y - b1m.y);
  } else if constexpr (R == 3) {
    constexpr double c1 = -0.5, s1 = -0.86602540378443864676;  // e^{-2 pi i / 3}
    const double2 t = cadd(v[1], v[2]);
    const double2 d = make_double2(v[1].x - v[2].x, v[1].y - v[2].y);
    const double2 m = make_double2(v[0].x + c1 * t.x, v[0].y + c1 * t.y);
    const double2 u = make_double2(-s1 * d.y, s1 * d.x);  // i s1 d
    v[0] = cadd(v[0], t);
    v[1] = cadd(m, u);
    v[2] = make_double2(m.x - u.x, m.y - u.y);
  } else if constexpr (R == 5) {
    constexpr double c1 = 0.30901699437494742410, s1 = -0.95105651629515357212;  // e^{-2 pi i / 5}
    constexpr double c2 = -0.80901699437494742410, s2 = -0.58778525229247312917; // e^{-4 pi i / 5}
    const double2 t1 = cadd(v[1], v[4]), d1 = make_double2(v[1].x - v[4].x, v[1].y - v[4].y);
    const double2 t2 = cadd(v[2], v[3]), d2 = make_double2(v[2].x - v[3].x, v[2].y - v[3].y);
    const double2 m1 = make_double2(v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y);
    const double2 m2 = make_double2(v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y);
    // i (s1 d1 + s2 d2) and i (s2 d1 - s1 d2)
    const double2 u1 = make_double2(-(s1 * d1.y + s2 * d2.y), s1 * d1.x + s2 * d2.x);
    const double2 u2 = make_double2(-(s2 * d1.y - s1 * d2.y), s2 * d1.x - s1 * d2.x);
    v[0] = cadd(cadd(v[0], t1), t2);
    v[1] = cadd(m1, u1);
    v[4] = make_double2(m1.x - u1.x, m1.y - u1.y);
    v[2] = cadd(m2, u2);
    v[3] = make_double2(m2.x - u2.x, m2.y - u2.y);
  }
}


// -----------------------------------------------------------------------------------------
// Compact ark codes (ABI 7).  dict2Ark writes '%.3f' text (features.py:66) that copy-feats reads back
// as float32; on the device that value is (float)(k / 10^d) with k = nearbyint(v 10^d).  The integer k
// fits int16 for every log feature the recipes produce (log(1e-14) = -32.236 is the floor, full-scale
// int16 input peaks near +18), so the features can leave the device as 2-byte codes and be widened
// bit-exactly on the host (fdlp_q_widen): code = k, except -32768 = -0.0 (k = -0 keeps its sign through
// the division).  A value without a code (|k| > 32767, NaN) stores -32768 and sets *flag (plain vector
// store); the caller then takes that batch's float32 rows instead.
// -----------------------------------------------------------------------------------------
constexpr int16_t kQNegZero = -32768;
__device__ __forceinline__ int16_t q_code(double k, bool& bad) {
  if (k >= -32767.0 && k <= 32767.0) return (k == 0.0 && signbit(k)) ? kQNegZero : (int16_t)(int)k;
  bad = true;  // out of range or NaN
  return kQNegZero;
}

// One feature of the OLA output (computeFDLPSpectrogram.py:227-229): log(clip(acc, 1e-14)) keeping NaN,
// stored as fp64 (debug), float32 ('%.<d>f'-rounded when decimals >= 0) and / or compact code; the OLA
// kernel stores through this.
// np.log of the OLA sums (computeFDLPSpectrogram.py:227) in ~35 VALU operations instead of the ~65 of
// ocml's log: x = 2^e m with m in [sqrt(1/2), sqrt(2)) (so e = 0 around 1: no ln 2 cancellation),
// i = round(128 m), c = i / 128, u = m - c exactly (Sterbenz), r = u RN(1/c) (|r| < 2^-7.5),
// log x = e ln2 + log c + log1p(r), log1p(r) by its degree-8 Taylor polynomial (truncation < 1e-19 r);
// e ln2_hi (exact: 42-bit ln2_hi) + log(c)_hi summed error-free (TwoSum, kept out of FMA contraction by the
// _rn intrinsics), then the small terms once: within ~0.5 ulp (tests/test_device_log.py: <= 1 ulp against
// numpy's log over 1e-14 .. 1e12).  NaN and +inf pass through.  lt = kLogTable (fdlp_mathtab.h) or a copy
// of it in LDS.
__device__ __forceinline__ double ola_log(double x, const double* __restrict__ lt) {
  constexpr double kSqrtHalf = 0.70710678118654752440;
  int e = __builtin_amdgcn_frexp_exp(x);
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  if (m < kSqrtHalf) {
    m = 2.0 * m;
    --e;
  }
  const int i = min(max((int)fma(m, 128.0, 0.5), kLogBase), kLogBase + kLogTab - 1) - kLogBase;
  const double u = __dadd_rn(m, -(double)(i + kLogBase) * 0.0078125);
  const double r = u * lt[2 * kLogTab + i];
  double q = fma(r, -0.125, 1.0 / 7.0);
  q = fma(r, q, -1.0 / 6.0);
  q = fma(r, q, 0.2);
  q = fma(r, q, -0.25);
  q = fma(r, q, 1.0 / 3.0);
  q = fma(r, q, -0.5);
  const double lp = fma(r * r, q, r);
  const double ed = (double)e;
  const double a = __dmul_rn(ed, kLn2Hi);
  const double h = lt[i];
  const double sum = __dadd_rn(a, h);
  const double bb = __dadd_rn(sum, -a);
  const double err = __dadd_rn(__dadd_rn(a, -__dadd_rn(sum, -bb)), __dadd_rn(h, -bb));
  const double res = __dadd_rn(sum, lp + (fma(ed, kLn2Lo, lt[kLogTab + i]) + err));
  return x < __builtin_inf() ? res : x;
}

__device__ __forceinline__ void ola_store_feature(double acc, int64_t o, float* __restrict__ out,
                                                  double* __restrict__ out64, int16_t* __restrict__ outq,
                                                  int decimals, double scale10, bool& bad,
                                                  const double* __restrict__ lt = kLogTable) {
  const double v = ola_log(acc < 1e-14 ? 1e-14 : acc, lt);  // np.clip(a_min=1e-14) keeps NaN; :227
  if (out64) out64[o] = v;
  const double k = nearbyint(v * scale10);
  if (out) out[o] = decimals >= 0 ? (float)(k / scale10) : (float)v;
  if (outq) outq[o] = q_code(k, bad);
}

// numpy 'reflect' padding index (getFrames, features.py:146)
__device__ __forceinline__ int64_t reflect_idx(int64_t q, int64_t T) {
  // numpy 'reflect' pad == periodic reflection with period 2(T-1) (features.py:146); the 64-bit
  // modulo is only needed when the pad exceeds one period (utterances shorter than the padding)
  if (q >= 0 && q < T) return q;
  if (T == 1) return 0;
  const int64_t P = 2 * (T - 1);
  if (q < 0 && q > -T) return -q;
  if (q >= T && q < P) return P - q;
  q %= P;
  if (q < 0) q += P;
  return q < T ? q : P - q;
}

// the --add_noise diff filter (static: one copy per translation unit)
static __constant__ int kDiffTaps[13] = {1, 2, 3, 2, 0, -2, -5, -2, 0, 2, 3, 2, 1};  // :163

}  // namespace fdlp
