// fdlp_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the FDLP-spectrogram hot path.
//
// Reference path (sadhusamik/speech_recognition_tools):
//   src/featgen/computeFDLPSpectrogram.py getFeats :172-229 and src/featgen/features.py
//   getFrames :118-154, computeLpcFast :222-230, computeModSpecFromLpc :233-246.
//
// Everything up to and including Levinson is fp64 (fp32 anywhere before
// Levinson breaks the 1e-4 tolerance or diverges).  Stages:
//   1. frames_dft1  : int16/f64 PCM -> reflect pad -> Hamming -> Makhoul reorder -> column DFTs
//                     (length N1) of the four-step N = N1*N2 DFT, twiddled.       (:174-178)
//   2. dft2_dct     : row DFTs (length N2) -> Makhoul post-twiddle -> DCT-II/sqrt(2N). (:178)
//   3. autocorr     : per (frame, band): x = W_j (.) D_f on the band's tap support, circular
//                     autocorrelation lags 0..p+1 on MFMA f64 16x16x4 (lag-tiled Hankel GEMM,
//                     DESIGN.md "autocorrelation as MFMA tiles").           (features.py:223-225)
//   3+4 band_fused  : autocorrelation followed, on the same wave, by Durbin + cepstrum + envelope
//                     (64 lanes per item), so the VALU tail overlaps other waves' MFMAs.
//   4. lpc_env      : (unfused alternative) per (frame, band), 16 lanes per item: Durbin + gg
//                     (features.py:226-228) -> LPC cepstrum (features.py:233-246) -> weights ->
//                     exp(Re DFT_{2*fd*fr}(c .* w))[0:kk] * hann/hamm (:194-205).
//                     (levinson_kernel / cepstrum_kernel serve the per-stage entry points.)
//   7. ola_log      : deterministic gather OLA + floor + log -> float32 [L, B].  (:207-229)
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include "fdlp_internal.h"

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
__device__ void stockham_stage(const double2* __restrict__ in, double2* __restrict__ out,
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
__device__ double2* lds_dft(double2* a, double2* b, const double2* om, const DftPlan& d, int ncols) {
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


// -----------------------------------------------------------------------------------------
// 1. frames -> Makhoul-reordered real sequence -> column DFTs (length N1) + four-step twiddle
// -----------------------------------------------------------------------------------------
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

__constant__ int kDiffTaps[13] = {1, 2, 3, 2, 0, -2, -5, -2, 0, 2, 3, 2, 1};  // :163

// Windowed frame sample at Makhoul index n of v (v[n] = x[2n], v[N-1-n] = x[2n+1]).
__device__ __forceinline__ double makhoul_sample(const DevConsts& c, const FrameDesc& fd, int n, int f,
                                                 const void* __restrict__ pcm, int pcm_kind,
                                                 const int16_t* __restrict__ noise,
                                                 const double* __restrict__ dense_rows) {
  const int N = c.N;
  // Makhoul even/odd split; complex modulation: sample order (scipy.fftpack.ifft of the frame)
  const int m = c.natural ? n : ((2 * n < N) ? 2 * n : 2 * N - 1 - 2 * n);
  if (dense_rows) return dense_rows[(int64_t)f * N + m];
  const int64_t t = reflect_idx((int64_t)fd.k * c.hop + m - c.ext, fd.T);
  double s;
  if (pcm_kind == 0) {
    s = (double)((const int16_t*)pcm)[fd.pcm_off + t];
    if (fd.noise_off >= 0) {
      // sig + alp*ns, evaluated in fp64 without contraction (features.py:31)
      const double ns = (double)noise[fd.noise_off + t];
      s = __dadd_rn(s, __dmul_rn(fd.alpha, ns));
    }
  } else if (pcm_kind == 1) {
    s = ((const double*)pcm)[fd.pcm_off + t];
  } else {
    // pcm_kind 2: scipy.signal.convolve(int16 s, diff kernel, 'same') -> int64, exact
    // (computeFDLPSpectrogram.py:162-164); 'same' = full[6 : 6+T], zeros outside [0, T)
    const int16_t* x = (const int16_t*)pcm + fd.pcm_off;
    long long acc = 0;
#pragma unroll
    for (int q = 0; q < 13; ++q) {
      const int64_t idx = t + 6 - q;
      if (idx >= 0 && idx < fd.T) acc += (long long)kDiffTaps[q] * (long long)x[idx];
    }
    s = (double)acc;
  }
  return __dmul_rn(s, c.hamming[m]);  // frame * win (features.py:153)
}

// REAL (even N): the real sequence v of length N is packed as z[q] = v[2q] + i v[2q+1] and
// transformed with a length-N/2 complex FFT (dft2_dct_kernel<true> unpacks); otherwise v is
// transformed as a complex sequence of length N.  The four-step split is N1 x N2 of that length.
template <bool REAL>
__global__ __launch_bounds__(256) void frames_dft1_kernel(
    DevConsts c, DftPlan d1, int N2, const void* __restrict__ pcm, int pcm_kind,
    const int16_t* __restrict__ noise, const FrameDesc* __restrict__ frames,
    const double* __restrict__ dense_rows, const double2* __restrict__ om1,
    double2* __restrict__ z) {
  extern __shared__ double2 smem[];
  const int N1 = d1.n;
  double2* bufA = smem;
  double2* bufB = smem + N1 * kDftCols;
  double2* oms = smem + 2 * N1 * kDftCols;
  const int f = blockIdx.y;
  const int n2_0 = blockIdx.x * kDftCols;
  for (int q = threadIdx.x; q < N1; q += blockDim.x) oms[q] = om1[q];

  FrameDesc fd;
  if (!dense_rows) fd = frames[f];
  // load z[N2*n1 + n2] for n1 in [0,N1), n2 in [n2_0, n2_0+kDftCols)
  for (int e = threadIdx.x; e < N1 * kDftCols; e += blockDim.x) {
    const int col = e % kDftCols;
    const int n1 = e / kDftCols;
    const int n2 = n2_0 + col;
    double2 val = make_double2(0.0, 0.0);
    if (n2 < N2) {
      const int q = N2 * n1 + n2;
      if constexpr (REAL) {
        val.x = makhoul_sample(c, fd, 2 * q, f, pcm, pcm_kind, noise, dense_rows);
        val.y = makhoul_sample(c, fd, 2 * q + 1, f, pcm, pcm_kind, noise, dense_rows);
      } else {
        val.x = makhoul_sample(c, fd, q, f, pcm, pcm_kind, noise, dense_rows);
      }
    }
    bufA[n1 * kDftCols + col] = val;
  }
  __syncthreads();
  double2* res = lds_dft(bufA, bufB, oms, d1, kDftCols);
  // twiddle exp(-2 pi i n2 k1 / (N1 N2)) and store z[f][k1][n2]
  for (int e = threadIdx.x; e < N1 * kDftCols; e += blockDim.x) {
    const int col = e % kDftCols;
    const int k1 = e / kDftCols;
    const int n2 = n2_0 + col;
    if (n2 < N2) {
      const double2 tw = ((const double2*)c.tw1)[(int64_t)k1 * N2 + n2];
      z[((int64_t)f * N1 + k1) * N2 + n2] = cmul(res[k1 * kDftCols + col], tw);
    }
  }
}

// -----------------------------------------------------------------------------------------
// 2. row DFTs (length N2) + Makhoul post-twiddle -> DCT-II / sqrt(2N)
//    REAL: Z = FFT_{N/2}(z) is unpacked into V = FFT_N(v) with E = (Z_k + conj Z_{M-k})/2,
//    O = (Z_k - conj Z_{M-k})/(2i), V_k = E + w^k O, V_{k+M} = E - w^k O (w = e^{-2 pi i/N},
//    M = N/2).  A workgroup holds rows k1 and N1-k1 (4 such pairs), so Z_{M-k} is in its LDS.
// -----------------------------------------------------------------------------------------
template <bool REAL>
__global__ __launch_bounds__(256) void dft2_dct_kernel(DevConsts c, DftPlan d2, int N1,
                                                       const double2* __restrict__ z,
                                                       const double2* __restrict__ om2,
                                                       double inv_scale_div, double* __restrict__ dct) {
  extern __shared__ double2 smem[];
  const int N2 = d2.n;
  double2* bufA = smem;
  double2* bufB = smem + N2 * kDftCols;
  double2* oms = smem + 2 * N2 * kDftCols;
  const int f = blockIdx.y;
  const int N = c.N;
  constexpr int kHalf = kDftCols / 2;
  // slot -> row k1 (-1: unused).  REAL: slots r and r + 4 hold the rows of pair pp = 4 b + r,
  // (pp, N1 - pp); a self-paired row (pp = 0 or 2 pp = N1) occupies slot r only.
  auto slot_row = [&](int r) -> int {
    if constexpr (REAL) {
      const int pp = blockIdx.x * kHalf + (r % kHalf);
      if (2 * pp > N1) return -1;
      if (r < kHalf) return pp;
      const int m = N1 - pp;
      return (pp == 0 || m == pp) ? -1 : m;
    } else {
      const int k1 = blockIdx.x * kDftCols + r;
      return k1 < N1 ? k1 : -1;
    }
  };
  for (int q = threadIdx.x; q < N2; q += blockDim.x) oms[q] = om2[q];
  for (int e = threadIdx.x; e < N2 * kDftCols; e += blockDim.x) {
    const int row = e / N2;  // coalesced over n2
    const int n2 = e % N2;
    const int k1 = slot_row(row);
    double2 v = make_double2(0.0, 0.0);
    if (k1 >= 0) v = z[((int64_t)f * N1 + k1) * N2 + n2];
    bufA[n2 * kDftCols + row] = v;
  }
  __syncthreads();
  double2* res = lds_dft(bufA, bufB, oms, d2, kDftCols);
  const double2* post = (const double2*)c.post;
  for (int e = threadIdx.x; e < N2 * kDftCols; e += blockDim.x) {
    const int row = e % kDftCols;
    const int k2 = e / kDftCols;
    const int k1 = slot_row(row);
    if (k1 < 0) continue;
    const int k = k1 + N1 * k2;
    const double2 V = res[k2 * kDftCols + row];
    if constexpr (REAL) {
      const int M = N1 * N2;
      // km = M - k (Z_M = Z_0) split as k1m + N1 k2m without a division
      const int k1m = k1 == 0 ? 0 : N1 - k1;
      const int k2m = k1 == 0 ? (k2 == 0 ? 0 : N2 - k2) : N2 - 1 - k2;
      const int rm = k1m == k1 ? row : (row < kHalf ? row + kHalf : row - kHalf);
      const double2 W = res[k2m * kDftCols + rm];
      const double2 E = make_double2(0.5 * (V.x + W.x), 0.5 * (V.y - W.y));
      const double2 O = make_double2(0.5 * (V.y + W.y), -0.5 * (V.x - W.x));
      const double2 t = cmul(((const double2*)c.rtw)[k], O);
      const double2 V1 = make_double2(E.x + t.x, E.y + t.y);
      const double2 V2 = make_double2(E.x - t.x, E.y - t.y);
      const double2 w1 = post[k], w2 = post[k + M];
      dct[(int64_t)f * N + k] = 2.0 * (w1.x * V1.x - w1.y * V1.y) / inv_scale_div;
      dct[(int64_t)f * N + k + M] = 2.0 * (w2.x * V2.x - w2.y * V2.y) / inv_scale_div;
    } else if (c.natural) {
      // complex modulation: ifft(frame)[k] = conj(DFT_k) / N (real frame), bins k < int(N/2)
      // (computeModulationSpectrum.py:154-155); row f of N doubles holds them as double2
      if (k < N / 2) {
        const double inv = 1.0 / (double)N;
        ((double2*)(dct + (int64_t)f * N))[k] = make_double2(V.x * inv, -V.y * inv);
      }
    } else {
      const double2 w = post[k];
      const double y = 2.0 * (w.x * V.x - w.y * V.y);
      dct[(int64_t)f * N + k] = y / inv_scale_div;  // dct(.)/np.sqrt(2N)  (:178)
    }
  }
}

// Workgroup b is dispatched to XCD b % 8.  Giving every XCD a contiguous run of work items keeps
// the items that read the same frame (its D row) on one L2 instead of pulling the row into all
// eight.  Grid = 8 * ceil(total / 8); the padding workgroups get an index >= total.
constexpr int kXcds = 8;
__device__ __forceinline__ int xcd_item() {
  const int per = gridDim.x / kXcds;
  return (int)(blockIdx.x % kXcds) * per + (int)(blockIdx.x / kXcds);
}
static inline int xcd_grid(int total) { return (total + kXcds - 1) / kXcds * kXcds; }

// -----------------------------------------------------------------------------------------
// 1s/2s. The same two DCT passes specialised at compile time for the recipes' frame length
// (N = 24000: packed length-12000 complex FFT = 100 x 120; radices 4.5.5 and 8.3.5): constant
// butterflies (roots of unity as literals), constant Stockham strides, COLS interleaved columns
// (rows) per workgroup, and a branch-free sample gather for frames that need no reflect padding.
// Same arithmetic order per butterfly as the generic passes (Stockham DIT, twiddle then DFT).
// -----------------------------------------------------------------------------------------
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

// LDS slot of element (pos, col) of COLS = 8 interleaved columns.  SWZ: the column index XORed with
// g(pos mod 8) = ((pos & 1) << 2) | ((pos & 7) >> 1), so 8 consecutive positions of one column (the
// row pass's coalesced load order) land in 8 different 16-byte bank groups, while the 8 columns of one
// position still fill its 128 bytes (the stage reads' lane groups pair positions p and p + 2 on
// complementary column halves; g keeps bit 2 equal for p and p + 2, so they stay disjoint).
template <bool SWZ>
__device__ __forceinline__ int lslot(int pos, int col) {
  if constexpr (SWZ) return pos * 8 + (col ^ (((pos & 1) << 2) | ((pos & 7) >> 1)));
  else return pos * 8 + col;
}

// One Stockham stage (radix R, Ns = product of the radices before it) of COLS interleaved length-N
// columns in LDS; om = the N roots omega_N^q.  IP (in place, in == out): every thread reads and
// transforms all its butterflies first, then a barrier, then the writes; one buffer instead of two,
// so twice the workgroups fit a CU's LDS (same arithmetic, bit-identical results).
template <int N, int COLS, int NT, int Ns, int R, bool SWZ = false, bool IP = false>
__device__ __forceinline__ void st_stage_c(const double2* __restrict__ in, double2* __restrict__ out,
                                           const double2* __restrict__ om) {
  static_assert(!SWZ || COLS == 8, "swizzle of 8 columns");
  constexpr int NB = N / R, TOT = NB * COLS, ITER = (TOT + NT - 1) / NT, TW0 = N / (Ns * R);
  const double2* src = in;
  double2* dst = out;
  if constexpr (IP) src = out;  // the caller passes the one buffer as out
  auto slot = [&](int pos, int col) { return SWZ ? lslot<SWZ>(pos, col) : pos * COLS + col; };
  double2 v[IP ? ITER : 1][R];
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int b = (int)threadIdx.x + it * NT;
    if (TOT % NT != 0 && b >= TOT) break;
    const int col = b % COLS, j = b / COLS;
    const int k = j % Ns, jq = j / Ns;
    double2 (&w)[R] = v[IP ? it : 0];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double2 x = src[slot(j + r * NB, col)];
      w[r] = (r == 0 || Ns == 1) ? x : cmul(x, om[TW0 * k * r]);
    }
    bfly_c<R>(w);
    if constexpr (!IP) {
      const int idxD = jq * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) dst[slot(idxD + r * Ns, col)] = w[r];
    }
  }
  if constexpr (IP) {
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int b = (int)threadIdx.x + it * NT;
      if (TOT % NT != 0 && b >= TOT) break;
      const int col = b % COLS, j = b / COLS;
      const int k = j % Ns, jq = j / Ns;
      const int idxD = jq * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) dst[slot(idxD + r * Ns, col)] = v[it][r];
    }
  }
}

// full length-N DFT of COLS columns, radices R0 R1 ...; returns the buffer holding the result
// (IP: a only, b unused)
template <int N, int COLS, int NT, bool SWZ, bool IP, int Ns, int R0, int... Rs>
__device__ __forceinline__ double2* lds_dft_c(double2* a, double2* b, const double2* om) {
  if constexpr (IP) {
    st_stage_c<N, COLS, NT, Ns, R0, SWZ, true>(a, a, om);
    __syncthreads();
    if constexpr (sizeof...(Rs) > 0) return lds_dft_c<N, COLS, NT, SWZ, true, Ns * R0, Rs...>(a, b, om);
    else return a;
  } else {
    st_stage_c<N, COLS, NT, Ns, R0, SWZ>(a, b, om);
    __syncthreads();
    if constexpr (sizeof...(Rs) > 0) return lds_dft_c<N, COLS, NT, SWZ, false, Ns * R0, Rs...>(b, a, om);
    else return b;
  }
}

#ifndef FDLP_DCT_IP
#define FDLP_DCT_IP 1  // in-place Stockham stages in the specialised DCT kernels (0: ping-pong buffers)
#endif
constexpr bool kDctIP = FDLP_DCT_IP != 0;

template <int N1>
struct DctRadices1;
template <>
struct DctRadices1<100> {
  template <int COLS, int NT>
  __device__ static double2* run(double2* a, double2* b, const double2* om) {
    return lds_dft_c<100, COLS, NT, false, kDctIP, 1, 4, 5, 5>(a, b, om);
  }
};
template <int N2>
struct DctRadices2;
template <>
struct DctRadices2<120> {
  template <int COLS, int NT, bool SWZ = false>
  __device__ static double2* run(double2* a, double2* b, const double2* om) {
    return lds_dft_c<120, COLS, NT, SWZ, kDctIP, 1, 4, 2, 3, 5>(a, b, om);
  }
};

template <int N1, int N2, int COLS>
__global__ __launch_bounds__(256) void frames_dft1_c_kernel(DevConsts c, const void* __restrict__ pcm, int pcm_kind,
                                                            const int16_t* __restrict__ noise,
                                                            const FrameDesc* __restrict__ frames,
                                                            const double2* __restrict__ om1,
                                                            double2* __restrict__ z, int nframes) {
  constexpr int NT = 256;
  __shared__ double2 bufA[N1 * COLS], bufB[kDctIP ? 1 : N1 * COLS], oms[N1], twb[N2];
  // 1-D grid, XCD-mapped: the column blocks of a frame run on one XCD (their z rows share L2 lines)
  constexpr int NBX = (N2 + COLS - 1) / COLS;
  const int it0 = xcd_item();
  if (it0 >= nframes * NBX) return;
  const int f = it0 / NBX;
  const int n2_0 = (it0 - f * NBX) * COLS;
  for (int q = threadIdx.x; q < N1; q += NT) oms[q] = om1[q];
  // four-step twiddle W^{k1 n2} (W = e^{-2 pi i / (N1 N2)}) with k1 n2 = N2 a + b: W_{N1}^{a} W^{b}, i.e.
  // the N1 roots (oms) times row k1 = 1 of the tw1 table (W^{b}, b < N2)
  const double2* tw1 = (const double2*)c.tw1;
  for (int q = threadIdx.x; q < N2; q += NT) twb[q] = tw1[N2 + q];
  const FrameDesc fd = frames[f];
  const int N = c.N;
  const int64_t t0 = (int64_t)fd.k * c.hop - c.ext;
  // no reflect padding, plain int16, no mixing: sample m of the frame is pcm[pcm_off + t0 + m]
  const bool fast = pcm_kind == 0 && fd.noise_off < 0 && t0 >= 0 && t0 + N <= fd.T;
  const int16_t* xs = (const int16_t*)pcm + fd.pcm_off + t0;
  constexpr int TOT = N1 * COLS;
#pragma unroll
  for (int it = 0; it < (TOT + NT - 1) / NT; ++it) {
    const int e = (int)threadIdx.x + it * NT;
    if (TOT % NT != 0 && e >= TOT) break;
    const int col = e % COLS, n1 = e / COLS;
    const int q = N2 * n1 + n2_0 + col;  // packed z[q] = v[2q] + i v[2q+1] (Makhoul order v)
    const int m0 = 4 * q < N ? 4 * q : 2 * N - 1 - 4 * q;
    const int m1 = 4 * q + 2 < N ? 4 * q + 2 : 2 * N - 3 - 4 * q;
    double2 val;
    if (fast) {
      val.x = __dmul_rn((double)xs[m0], c.hamming[m0]);
      val.y = __dmul_rn((double)xs[m1], c.hamming[m1]);
    } else {
      val.x = makhoul_sample(c, fd, 2 * q, f, pcm, pcm_kind, noise, nullptr);
      val.y = makhoul_sample(c, fd, 2 * q + 1, f, pcm, pcm_kind, noise, nullptr);
    }
    bufA[n1 * COLS + col] = val;
  }
  __syncthreads();
  const double2* res = DctRadices1<N1>::template run<COLS, NT>(bufA, bufB, oms);
#pragma unroll
  for (int it = 0; it < (TOT + NT - 1) / NT; ++it) {
    const int e = (int)threadIdx.x + it * NT;
    if (TOT % NT != 0 && e >= TOT) break;
    const int col = e % COLS, k1 = e / COLS;
    const int n2 = n2_0 + col;
    const int q = k1 * n2;  // < N1 N2
    const double2 tw = cmul(oms[q / N2], twb[q % N2]);
    z[((int64_t)f * N1 + k1) * N2 + n2] = cmul(res[k1 * COLS + col], tw);
  }
}

// rows k1 of pair pp (pp, N1 - pp): slots r (< COLS/2) and r + COLS/2
template <int N1, int N2, int COLS, bool TWF = true, bool SWZ = true>
__global__ __launch_bounds__(256) void dft2_dct_c_kernel(DevConsts c, const double2* __restrict__ z,
                                                         const double2* __restrict__ om2, double scale2,
                                                         double* __restrict__ dct, int nframes) {
  // scale2 = 2 / sqrt(2N): dct(.) / np.sqrt(2N) (:178) as one multiplication (within an ulp of the
  // reference's division; no fp64 division per coefficient)
  constexpr int NT = 256, HALF = COLS / 2;
  __shared__ double2 bufA[N2 * COLS], bufB[kDctIP ? 1 : N2 * COLS], oms[N2];
  __shared__ double2 pw1[N1], pw2[N2], rw1[N1], rw2[N2];  // factored twiddles (TWF)
  // 1-D grid, XCD-mapped: the row-pair blocks of a frame run on one XCD, so the 32-B runs they store
  // into each D line (k = k1 + N1 k2: 4 consecutive k1 per block) merge in that XCD's L2
  constexpr int NBX = (N1 / 2 + 1 + HALF - 1) / HALF;
  const int it0 = xcd_item();
  if (it0 >= nframes * NBX) return;
  const int f = it0 / NBX;
  const int bx = it0 - f * NBX;
  const int N = c.N;
  auto slot_row = [&](int r) -> int {
    const int pp = bx * HALF + (r % HALF);
    if (2 * pp > N1) return -1;
    if (r < HALF) return pp;
    const int m = N1 - pp;
    return (pp == 0 || m == pp) ? -1 : m;
  };
  for (int q = threadIdx.x; q < N2; q += NT) oms[q] = om2[q];
  if (TWF) {  // post[k] = post[k1] post[N1 k2], rtw[k] = rtw[k1] rtw[N1 k2]  (k = k1 + N1 k2)
    const double2* post = (const double2*)c.post;
    const double2* rtw = (const double2*)c.rtw;
    for (int q = threadIdx.x; q < N1; q += NT) { pw1[q] = post[q]; rw1[q] = rtw[q]; }
    for (int q = threadIdx.x; q < N2; q += NT) { pw2[q] = post[N1 * q]; rw2[q] = rtw[N1 * q]; }
  }
  constexpr int TOT = N2 * COLS;
#pragma unroll
  for (int it = 0; it < (TOT + NT - 1) / NT; ++it) {
    const int e = (int)threadIdx.x + it * NT;
    if (TOT % NT != 0 && e >= TOT) break;
    const int row = e / N2, n2 = e % N2;  // coalesced over n2 (the row-fastest order measured slower)
    const int k1 = slot_row(row);
    double2 v = make_double2(0.0, 0.0);
    if (k1 >= 0) v = z[((int64_t)f * N1 + k1) * N2 + n2];
    bufA[lslot<SWZ>(n2, row)] = v;
  }
  __syncthreads();
  const double2* res = DctRadices2<N2>::template run<COLS, NT, SWZ>(bufA, bufB, oms);
  const double2* post = (const double2*)c.post;
  const double2* rtw = (const double2*)c.rtw;
  constexpr int M = N1 * N2;
#pragma unroll
  for (int it = 0; it < (TOT + NT - 1) / NT; ++it) {
    const int e = (int)threadIdx.x + it * NT;
    if (TOT % NT != 0 && e >= TOT) break;
    const int row = e % COLS, k2 = e / COLS;
    const int k1 = slot_row(row);
    if (k1 < 0) continue;
    const int k = k1 + N1 * k2;
    const double2 V = res[lslot<SWZ>(k2, row)];
    const int k1m = k1 == 0 ? 0 : N1 - k1;
    const int k2m = k1 == 0 ? (k2 == 0 ? 0 : N2 - k2) : N2 - 1 - k2;
    const int rm = k1m == k1 ? row : (row < HALF ? row + HALF : row - HALF);
    const double2 W = res[lslot<SWZ>(k2m, rm)];
    const double2 E = make_double2(0.5 * (V.x + W.x), 0.5 * (V.y - W.y));
    const double2 O = make_double2(0.5 * (V.y + W.y), -0.5 * (V.x - W.x));
    double2 rt, w1, w2;
    if (TWF) {
      rt = cmul(rw1[k1], rw2[k2]);
      w1 = cmul(pw1[k1], pw2[k2]);
      // post[k + M] = post[k] e^{-i pi M / (2N)} = post[k] e^{-i pi / 4}  (M = N / 2)
      constexpr double h = 0.70710678118654752440;
      w2 = make_double2(h * (w1.x + w1.y), h * (w1.y - w1.x));
    } else {
      rt = rtw[k];
      w1 = post[k];
      w2 = post[k + M];
    }
    const double2 t = cmul(rt, O);
    const double2 V1 = make_double2(E.x + t.x, E.y + t.y);
    const double2 V2 = make_double2(E.x - t.x, E.y - t.y);
    dct[(int64_t)f * N + k] = (w1.x * V1.x - w1.y * V1.y) * scale2;
    dct[(int64_t)f * N + k + M] = (w2.x * V2.x - w2.y * V2.y) * scale2;
  }
}

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

// -----------------------------------------------------------------------------------------
// 64-lane (one item per wave) LPC tail used by the fused band kernel: Durbin, cepstrum and
// envelope for ONE (frame, band) item right after its MFMA autocorrelation, so this VALU/LDS
// work of one wave overlaps the MFMA phases of the other waves on the SIMD.
// -----------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum64(double v) {
  v = row_sum16(v);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

struct LpcTail {
  int p, nlags, M, Me, kk, odd_zero;
  const double* weights;  // [3, M]
  const double* env_cos;  // [env_nfft]
  int env_nfft;
  const double* env_win;  // [kk, 2]: (hanning / hamming ratio, 1.0)
};

constexpr int kTS64 = 4;  // envelope samples per lane (kk <= 256)

// LDS: la[0..NAL) (a, zero beyond p), lr[0..max(nlags, M)) (r, then c).  Writes env[0..kk).
__device__ void lpc_tail64(const LpcTail& T, double* la, double* lr, double* env, int lane) {
  const int p = T.p, M = T.M;
  // Durbin (features.py:226-228) with the symmetric in-place update (see durbin16)
  double E = lr[0];
  for (int k = 1; k <= p; ++k) {
    double part = 0.0;
    for (int i = lane + 1; i < k; i += 64) part += la[i] * lr[k - i];
    const double acc = lr[k] + wave_sum64(part);
    const double kappa = -acc / E;
    wave_lds_sync();
    for (int i = lane + 1; 2 * i <= k; i += 64) {
      const int j = k - i;
      const double ai = la[i], aj = la[j];
      if (i == j) {
        la[i] = ai + kappa * ai;
      } else {
        la[i] = ai + kappa * aj;
        la[j] = aj + kappa * ai;
      }
    }
    if (lane == 0) la[k] = kappa;
    wave_lds_sync();
    E = E * (1.0 - kappa * kappa);
  }
  double part = 0.0;
  for (int i = lane; i <= p; i += 64) part += la[i] * lr[i + 1];
  const double gg = lr[0] + wave_sum64(part);
  wave_lds_sync();
  // cepstrum (features.py:233-246), alpha_n = -a_n; c overwrites r
  double* cs = lr;
  for (int b0 = 0; b0 < M; b0 += 64) {
    const int n = b0 + lane;
    const double inv_n = 1.0 / (double)(n > 0 ? n : 1);
    double acc = 0.0;
    const int kstart = max(1, b0 - p);
    double kd = (double)kstart;
    if (n < M)
      for (int k = kstart; k < b0; ++k, kd += 1.0) acc -= ((kd * inv_n) * la[n - k]) * cs[k];
    double mine = 0.0;
    for (int kk = 0; kk < 64; ++kk) {
      const int kg = b0 + kk;
      if (kg >= M) break;
      if (lane == kk) {
        if (kg == 0) mine = log(sqrt(gg));
        else if (kg == 1) mine = -la[1];
        else mine = acc - la[kg];
      }
      const double ck = __shfl(mine, kk, 64);
      if (kg >= 1 && lane > kk && n < M) acc -= (((double)kg * inv_n) * la[n - kg]) * ck;
    }
    wave_lds_sync();
    if (n < M) cs[n] = mine;
    wave_lds_sync();
  }
  // weights + envelope (computeFDLPSpectrogram.py:194-205)
  double* cw = la;
  for (int n = lane; n < T.Me; n += 64) {
    double v = cs[n];
    v = v * T.weights[n];
    v = v * T.weights[M + n];
    v = v * T.weights[2 * M + n];
    if (T.odd_zero && (n & 1)) v = 0.0;
    cw[n] = v;
  }
  wave_lds_sync();
  // one envelope sample at a time per lane keeps the tail's register footprint small (the
  // MFMA accumulators of this kernel already hold 88 AGPRs)
#pragma nounroll
  for (int t = lane; t < T.kk; t += 64) {
    const double c1 = T.env_cos[t % T.env_nfft];
    const double c2 = 2.0 * c1;
    double sum = cw[0], cprev = 1.0, ccur = c1;
    for (int n = 1; n < T.Me; ++n) {
      sum += cw[n] * ccur;
      const double nxt = c2 * ccur - cprev;
      cprev = ccur;
      ccur = nxt;
    }
    env[t] = exp(sum) * T.env_win[2 * t];
  }
}

// -----------------------------------------------------------------------------------------
// 3. circular autocorrelation, lags 0..nlags-1, on MFMA f64 16x16x4
//
// For one band signal x (support [lo,hi)), tile t (t = 0..NT-1) accumulates
//   C_t[i][jj] = sum_s sum_kk x[m] * x[m + 16t + jj - i],  m = base + 64 s + 16 kk + i
// with A[i][kk] = x[base + 64s + 16kk + i] and B_t[kk][jj] = x[base + 64s + 16(kk+t) + jj]:
// exactly one MFMA per tile per 64 positions.  r[l] = sum_i C_{t(i,l)}[i][(l+i) mod 16],
// t(i,l) = (l+i) div 16.  Indices past N wrap (circular, features.py:223 uses FFTs of length N).
// -----------------------------------------------------------------------------------------
// Staging: x = W_j (.) D_f is written into a mirrored LDS ring (every value at slot and
// slot + kRing, so window reads never wrap) one 256-position chunk at a time; the D/W loads of
// chunk c+2 are issued into registers before the MFMAs of chunk c and land in the ring after
// them, so global latency hides behind 44 MFMAs per chunk.
constexpr int kAcChunk = 256;   // positions per staged chunk (4 k-steps)
constexpr int kAcRing = 512;    // ring holds chunks c and c+1 (the window halo of c is <= 16*NT <= 256)
constexpr int kAcPer = kAcChunk / 64;

template <int NT, bool FUSE>
__global__ __launch_bounds__(64, 4) void autocorr_kernel(DevConsts c, const double* __restrict__ dct,
                                                      const double* __restrict__ dense,
                                                      double* __restrict__ rout, LpcTail tail,
                                                      double* __restrict__ env) {
  static_assert(16 * NT <= kAcChunk, "window halo must fit one chunk");
  constexpr int G = 2;                                  // tiles per epilogue group (LDS <= 8 KB)
  constexpr int kEpi = (16 * G + 15) * 17;              // padded lag-major epilogue buffer
  constexpr int kStage = 2 * kAcRing;
  constexpr int kLds = kStage > kEpi ? kStage : kEpi;
  constexpr int NLPL = (16 * NT + 63) / 64;             // owned lags per lane
  __shared__ double xs[kLds];

  const int item = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = c.N;
  int lo, hi;
  const double* drow;
  const double* wrow = nullptr;
  if (dense) {
    lo = 0;
    hi = N;
    drow = dense + (int64_t)item * N;
  } else {
    const int f = item / c.B, j = item % c.B;
    lo = c.lo[j];
    hi = c.hi[j];
    drow = dct + (int64_t)f * N;
    wrow = c.fbank + (int64_t)j * N;
  }
  const int i_lane = lane & 15;
  const int kk_lane = lane >> 4;

  dbl4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};

  const int span = hi - lo;
  const int nsteps = (span + 63) / 64;
  const int nchunks = (nsteps + kAcPer - 1) / kAcPer;
  double dv[kAcPer], wv[kAcPer];
  // positions lo + 256*ch + 64*q + lane; indices past N wrap once (plan guarantees N >= 1024)
  auto fetch = [&](int ch) {
#pragma unroll
    for (int q = 0; q < kAcPer; ++q) {
      int pos = lo + kAcChunk * ch + 64 * q + lane;
      if (pos >= N) pos -= N;
      const bool ok = pos >= lo && pos < hi;
      dv[q] = ok ? drow[pos] : 0.0;
      wv[q] = ok ? (wrow ? wrow[pos] : 1.0) : 0.0;
    }
  };
  auto store = [&](int ch) {
#pragma unroll
    for (int q = 0; q < kAcPer; ++q) {
      const int slot = (kAcChunk * ch + 64 * q + lane) & (kAcRing - 1);
      const double x = wv[q] * dv[q];  // filt * dct  (:191)
      xs[slot] = x;
      xs[slot + kAcRing] = x;
    }
  };
  if (nsteps > 0) {
    fetch(0);
    store(0);
    fetch(1);
    store(1);
    fetch(2);
  }
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    const int s_end = min(kAcPer, nsteps - kAcPer * ch);
    const int rbase = (kAcChunk * ch) & (kAcRing - 1);
    for (int st = 0; st < s_end; ++st) {
      const double* w = xs + rbase + 64 * st + 16 * kk_lane + i_lane;
      const double a = w[0];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, w[16 * t], acc[t], 0, 0, 0);
    }
    __syncthreads();
    store(ch + 2);  // overwrites chunk ch's slots
    if (ch + 3 <= nchunks) fetch(ch + 3);
    __syncthreads();
  }

  // epilogue: diagonal sums via a padded lag-major LDS image, G tiles at a time
  const int nlags = c.nlags;
  double mine[NLPL];
#pragma unroll
  for (int q = 0; q < NLPL; ++q) mine[q] = 0.0;
  const int col = lane & 15;
  const int row0 = lane >> 4;
#pragma unroll
  for (int tg = 0; tg < NT; tg += G) {
    const int lag_base = 16 * tg - 15;
#pragma unroll
    for (int t = tg; t < tg + G && t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * r;
        const int lag = 16 * t + col - row;
        xs[(lag - lag_base) * 17 + row] = acc[t][r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NLPL; ++q) {
      const int L = lane + 64 * q;
      if (L < nlags && L >= lag_base && L < 16 * (tg + G)) {
        double s = 0.0;
        for (int i = 0; i < 16; ++i) {
          const int t = (L + i) >> 4;
          if (t >= tg && t < tg + G && t < NT) s += xs[(L - lag_base) * 17 + i];
        }
        mine[q] += s;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < NLPL; ++q) {
    const int L = lane + 64 * q;
    if (L < nlags && rout) rout[(int64_t)item * nlags + L] = mine[q];
  }
  if constexpr (FUSE) {
    // LPC tail on the same wave (plan guarantees the region fits kLds)
    const int NAL = (tail.M > tail.p + 1 ? tail.M : tail.p + 1) + 64;
    double* la = xs;
    double* lr = xs + NAL;
    for (int q = lane; q < NAL; q += 64) la[q] = q == 0 ? 1.0 : 0.0;
#pragma unroll
    for (int q = 0; q < NLPL; ++q) {
      const int L = lane + 64 * q;
      if (L < nlags) lr[L] = mine[q];
    }
    wave_lds_sync();
    lpc_tail64(tail, la, lr, env + (int64_t)item * tail.kk, lane);
  }
}

// -----------------------------------------------------------------------------------------
// 3s. Structured autocorrelation for the cochlear filterbank with a fixed skirt slope
//     (createFbankCochlear, features.py:193-219, fixed == 1; DESIGN.md "Structured
//     autocorrelation").  Band j's taps are 10^(a(d+w/2)) on its lower skirt [0,m1), 1 on the
//     flat top [m1,m2) and 10^(-b(d-w/2)) on the upper skirt [m2,N), d = fw(m) - fc_j.  Inside
//     one skirt the product of two taps factorises, W[m] W[m'] = K_j E[m] E[m'], so the pairs of
//     r_j[l] with both ends on the lower (upper) skirt are K_j (K'_j) times a truncated
//     autocorrelation of the band-independent signal y = E.D (z = E'.D): ONE sweep per frame and
//     skirt, with a snapshot at every band's boundary, replaces 80 per-band passes.  The flat-top
//     pairs and the pairs that straddle a region boundary or the circular wrap are summed per band
//     with the true taps (ac_band_kernel).  No tap is truncated (support_eps does not apply).
// -----------------------------------------------------------------------------------------

// Diagonal sums r[L] = sum_i C_{(L+i)>>4}[i][(L+i)&15] of the NT lag tiles for the lags owned by
// this lane (L = lane + 64 q), through a padded lag-major LDS image, G tiles at a time.
// ep holds (16 G + 15) * 17 doubles.  Block = one wave.
template <int NT, int G, int NLPL>
__device__ __forceinline__ void diag_sums(const dbl4* acc, double* ep, int nlags, int lane, double* mine) {
#pragma unroll
  for (int q = 0; q < NLPL; ++q) mine[q] = 0.0;
  const int col = lane & 15;
  const int row0 = lane >> 4;
#pragma unroll
  for (int tg = 0; tg < NT; tg += G) {
    const int lag_base = 16 * tg - 15;
#pragma unroll
    for (int t = tg; t < tg + G && t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * r;
        ep[(16 * t + col - row - lag_base) * 17 + row] = acc[t][r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NLPL; ++q) {
      const int L = lane + 64 * q;
      if (L < nlags && L >= lag_base && L < 16 * (tg + G)) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int t = (L + i) >> 4;
          if (t >= tg && t < tg + G && t < NT) s += ep[(L - lag_base) * 17 + i];
        }
        mine[q] += s;
      }
    }
    __syncthreads();
  }
}

// Diagonal sums in lag blocks of LB lags (LB = 32 or 64), branch-free.  Block g covers lags
// [LB g, LB g + LB); its 16-term sums touch tiles LB/16 g .. LB/16 (g+1), which are written whole
// into a padded lag-major image (rows = lags LB g - 15 .. LB g + LB + 14, stride 17).  LPL = 64/LB
// lanes share a lag, each adding 16/LPL consecutive terms, and a DPP swap finishes the sum; the
// first lane of each group calls emit(L, r_L) (or emit(g, L, r_L) if emit takes the block index).  ep holds (LB + 31) * 17 doubles.  Block = one wave.
template <int NT, int LB, typename Emit>
__device__ __forceinline__ void diag_blocks(const dbl4* acc, double* ep, int nlags, int lane, Emit emit) {
  static_assert(LB == 32 || LB == 64, "lag block");
  constexpr int LPL = 64 / LB;
  constexpr int TPB = LB / 16;                       // tiles per block (+1 shared with the next)
  constexpr int NB = (16 * NT + LB - 1) / LB;
  const int col = lane & 15;
  const int row0 = lane >> 4;
  const int m = lane / LPL;
  const int part = lane % LPL;
#pragma unroll
  for (int g = 0; g < NB; ++g) {
    if (LB * g >= nlags) break;
#pragma unroll
    for (int u = 0; u <= TPB; ++u) {
      const int t = TPB * g + u;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * r;
        // lag 16 t + col - row -> image row (lag - LB g + 15)
        const double v = t < NT ? acc[t < NT ? t : 0][r] : 0.0;
        ep[(16 * u + col - row + 15) * 17 + row] = v;
      }
    }
    wave_lds_sync();
    const double* src = ep + (m + 15) * 17 + part * (16 / LPL);
    double v[16 / LPL];
#pragma unroll
    for (int i = 0; i < 16 / LPL; ++i) v[i] = src[i];
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < 16 / LPL; ++i) sum += v[i];
    if constexpr (LPL == 2) sum += dpp_f64<0xB1>(sum);  // quad_perm [1,0,3,2]: partner lane
    const int L = LB * g + m;
    if (part == 0 && L < nlags) {
      if constexpr (std::is_invocable_v<Emit, int, int, double>) emit(g, L, sum);
      else emit(L, sum);
    }
    wave_lds_sync();
  }
}

// One MFMA k-step of the lag tiles: A = x[P + 16 kk + i] (masked to [lo, hi)), B_t = x[P + 16(kk+t) + jj]
// read from a window w (w points at the lane's A element; B_t is w[16 t]).
template <int NT>
__device__ __forceinline__ void lag_step(dbl4* acc, const double* w, bool keep) {
  const double a = keep ? w[0] : 0.0;
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, w[16 * t], acc[t], 0, 0, 0);
}

// Skirt sweep: one wave per (frame, skirt).  Skirt 0 walks the reversed lower-skirt signal
// s[n] = E[N-1-n] D[N-1-n], skirt 1 the upper-skirt signal s[n] = E'[n] D[n] (s = 0 past N, no wrap).
// Positions are consumed from the top down, 64 per k-step, so after the steps covering [S, N) the
// tiles hold R(S)[l] = sum_{m >= S} s[m] s[m+l], the autocorrelation of s truncated to [S, N).
// For skirt 0, S = N - m1_j gives the lower-skirt pairs of band j; for skirt 1, S = m2_j the upper.
// A threshold inside a k-step splits it into two A-masked steps around the snapshot.
template <int NT, int G, bool SNAP = true>
__global__ __launch_bounds__(64, 2) void ac_sweep_kernel(DevConsts c, const double* __restrict__ dct,
                                                         double* __restrict__ rlow, double* __restrict__ rup,
                                                         int nwork) {
  static_assert(16 * NT <= kAcChunk, "window halo must fit one chunk");
  constexpr int kEpi = (G + 31) * 17;  // G = lag block of diag_blocks
  __shared__ double xs[2 * kAcRing];
  __shared__ double ep[kEpi];

  const int w = xcd_item();  // (frame, skirt) pairs of a frame stay on one XCD
  if (w >= nwork) return;
  const int f = w >> 1;
  const int sk = w & 1;
  const int lane = threadIdx.x;
  const int N = c.N, B = c.B, nlags = c.nlags;
  const double* drow = dct + (int64_t)f * N;
  const double* ew = c.sk_e + (int64_t)sk * N;
  const SkSnap* snaps = c.sk_snap + sk * B;
  double* out = (sk == 0 ? rlow : rup) + (int64_t)f * B * nlags;
  const int T0 = ((N + kAcChunk - 1) / kAcChunk) * kAcChunk;
  const int bmin = c.sk_min[sk] >> 6;
  const int nblk = (T0 >> 6) - bmin;
  const int nchunks = (nblk + kAcPer - 1) / kAcPer;
  const int i_lane = lane & 15;
  const int kk_lane = lane >> 4;

  dbl4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};

  // chunk ch = positions [T0 - 256 (ch+1), T0 - 256 ch); the loads land in registers and are
  // multiplied only when stored, one chunk later, so their latency hides behind 44 MFMAs
  double dv[kAcPer], ev[kAcPer];
  auto fetch = [&](int ch) {
#pragma unroll
    for (int q = 0; q < kAcPer; ++q) {
      const int n = T0 - kAcChunk * (ch + 1) + 64 * q + lane;
      const bool ok = n >= 0 && n < N;
      const int m = ok ? (sk == 0 ? N - 1 - n : n) : 0;
      dv[q] = drow[m];
      ev[q] = ok ? ew[m] : 0.0;
    }
  };
  auto store = [&](int ch) {
#pragma unroll
    for (int q = 0; q < kAcPer; ++q) {
      const int slot = (T0 - kAcChunk * (ch + 1) + 64 * q + lane) & (kAcRing - 1);
      const double v = ev[q] * dv[q];
      xs[slot] = v;
      xs[slot + kAcRing] = v;
    }
  };
  // snapshot records (threshold, band, K), consumed in order from an LDS copy
  extern __shared__ SkSnap tab[];
  for (int q = lane; q < B; q += 64) tab[q] = snaps[q];
  __syncthreads();
  int k = 0;
  SkSnap cur = tab[0];
  auto snapshot = [&]() {
    double* o = out + (int64_t)cur.band * nlags;
    const double K = cur.K;
    if constexpr (SNAP) {
      diag_blocks<NT, G>(acc, ep, nlags, lane, [&](int L, double v) { o[L] = K * v; });
    } else {  // timing experiment: keep every MFMA live through a cheap checksum
      double cs = 0.0;
#pragma unroll
      for (int t = 0; t < NT; ++t) cs += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
      if (lane < nlags) o[lane] = K * cs;
    }
    ++k;
    cur = k < B ? tab[k] : SkSnap{-1, 0, 0.0};
  };
  auto step = [&](int P, int lo, int hi) {
    const int pa = P + 16 * kk_lane + i_lane;
    lag_step<NT>(acc, xs + (P & (kAcRing - 1)) + 16 * kk_lane + i_lane, pa >= lo && pa < hi);
  };

#pragma unroll
  for (int q = 0; q < kAcPer; ++q) {  // chunk -1 (above T0) is zero
    const int slot = (T0 + 64 * q + lane) & (kAcRing - 1);
    xs[slot] = 0.0;
    xs[slot + kAcRing] = 0.0;
  }
  fetch(0);
  store(0);
  if (nchunks > 1) fetch(1);
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    for (int q = kAcPer - 1; q >= 0; --q) {
      const int P = T0 - kAcChunk * (ch + 1) + 64 * q;
      if ((P >> 6) < bmin) break;
      int hiM = P + 64;
      while (k < B && cur.S >= hiM) snapshot();
      while (k < B && cur.S > P) {
        step(P, cur.S, hiM);
        hiM = cur.S;
        snapshot();
      }
      step(P, P, hiM);
    }
    __syncthreads();
    if (ch + 1 < nchunks) store(ch + 1);  // into the slots of chunk ch-1
    if (ch + 2 < nchunks) fetch(ch + 2);
    __syncthreads();
  }
  while (k < B) snapshot();
}

// Per (frame, band): flat-top pairs (unit taps on [m1, m2)), the pairs straddling m1, m2 and the
// circular wrap at N (true taps W_j D), plus the two skirt snapshots from ac_sweep_kernel:
//   r_j[l] = K_j R_y(N-m1_j)[l] + flat + straddles + K'_j R_z(m2_j)[l]
// r holds the lower-skirt term on entry and r_j on exit.
// VS: the flat-top pairs come from ac_vsweep_kernel (rflat, right ends up to N), so the flat-top
// loop is skipped and the m2 straddle takes B = (W - 1) D on [m2, N) (W D past the wrap).
template <int NT, bool VS>
__global__ __launch_bounds__(64, 4) void ac_band_kernel(DevConsts c, const double* __restrict__ dct,
                                                        double* __restrict__ r, const double* __restrict__ rup,
                                                        const double* __restrict__ rflat,
                                                        const double* __restrict__ rpart, int items) {
  static_assert(16 * NT <= kAcChunk, "window halo must fit one chunk");
  constexpr int kEpi = (32 + 31) * 17;                   // diag_blocks<NT, 32> image
  constexpr int kWin = (16 * NT + 63) / 64 * 64;         // A window of a straddle (>= nlags - 1)
  constexpr int kLds = 2 * kAcRing > kEpi ? 2 * kAcRing : kEpi;
  static_assert(kEpi <= kLds && 2 * kWin + 16 * NT <= kLds, "LDS regions");
  __shared__ double xs[kLds];

  const int item = xcd_item();  // the B bands of a frame run on one XCD
  if (item >= items) return;
  const int lane = threadIdx.x;
  const int N = c.N, nlags = c.nlags;
  const int f = item / c.B, j = item % c.B;
  const int2 reg = c.sk_reg[j];
  const int m1 = reg.x, m2 = reg.y;
  const double* drow = dct + (int64_t)f * N;
  const double* wrow = c.fbank + (int64_t)j * N;
  const int i_lane = lane & 15;
  const int kk_lane = lane >> 4;

  dbl4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};

  // flat top: x = D on [m1, m2), 0 elsewhere
  if constexpr (!VS) {
    const int lo = m1, hi = m2;
    const int nsteps = (hi - lo + 63) / 64;
    const int nchunks = (nsteps + kAcPer - 1) / kAcPer;
    double dv[kAcPer];
    auto fetch = [&](int ch) {
#pragma unroll
      for (int q = 0; q < kAcPer; ++q) {
        const int pos = lo + kAcChunk * ch + 64 * q + lane;
        dv[q] = pos < hi ? drow[pos] : 0.0;
      }
    };
    auto store = [&](int ch) {
#pragma unroll
      for (int q = 0; q < kAcPer; ++q) {
        const int slot = (kAcChunk * ch + 64 * q + lane) & (kAcRing - 1);
        xs[slot] = dv[q];
        xs[slot + kAcRing] = dv[q];
      }
    };
    if (nsteps > 0) {
      fetch(0);
      store(0);
      fetch(1);
      store(1);
      fetch(2);
    }
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
      const int s_end = min(kAcPer, nsteps - kAcPer * ch);
      const int rbase = (kAcChunk * ch) & (kAcRing - 1);
      for (int st = 0; st < s_end; ++st)
        lag_step<NT>(acc, xs + rbase + 64 * st + 16 * kk_lane + i_lane, true);
      __syncthreads();
      store(ch + 2);
      if (ch + 3 <= nchunks) fetch(ch + 3);
      __syncthreads();
    }
  }

  // straddles: A = x[m], m in [lb, b) (the region just below boundary b, at most nlags-1 long),
  // B = x[(m + l) mod N] for m + l >= b, x = W_j D
  double* xa = xs;
  double* xb = xs + kWin;
#pragma unroll 1
  for (int e = 0; e < 3; ++e) {
    const int b = e == 0 ? m1 : (e == 1 ? m2 : N);
    int lb = e == 0 ? 0 : (e == 1 ? m1 : m2);
    lb = max(lb, b - (nlags - 1));
    if (lb >= b) continue;
    constexpr int kSt = (kWin + 16 * NT + 63) / 64;  // B reads reach xb[kWin - 1 + 16 NT - 1]
    double wv[kSt], dv[kSt];
#pragma unroll
    for (int u = 0; u < kSt; ++u) {  // all loads first: one exposed latency per boundary
      const int pos = b - kWin + 64 * u + lane;
      const int pm = pos < 0 ? 0 : (pos >= N ? pos - N : pos);
      wv[u] = wrow[pm];
      dv[u] = drow[pm];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kSt; ++u) {
      const int q = 64 * u + lane;
      const int pos = b - kWin + q;
      const double x = pos >= lb ? wv[u] * dv[u] : 0.0;
      if constexpr (VS) {
        if (q < kWin + 16 * NT) xb[q] = pos >= b ? (e == 1 && pos < N ? (wv[u] - 1.0) * dv[u] : x) : 0.0;
      } else {
        if (q < kWin + 16 * NT) xb[q] = pos >= b ? x : 0.0;
      }
      if (q < kWin) xa[q] = pos < b ? x : 0.0;
    }
    __syncthreads();
    // st unrolled, so each step's first live tile tmin is a constant: its MFMAs and their LDS reads are
    // branch-free (the reads issue together instead of one exposed LDS latency per MFMA)
    const int st0 = (lb - b + kWin) >> 6;
#pragma unroll
    for (int st = 0; st < kWin / 64; ++st) {
      if (st < st0) continue;
      const int w = 64 * st + 16 * kk_lane + i_lane;
      const double a = xa[w];
      // tile t reads B positions up to b - kWin + 64 st + 63 + 16 t; below b they are all zero
      const int tmin = (kWin - 64 * st - 48) >> 4;
      double bv[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (t >= tmin) bv[t] = xb[w + 16 * t];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (t >= tmin) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv[t], acc[t], 0, 0, 0);
    }
  }
  __syncthreads();
  double* ro = r + (int64_t)item * nlags;
  const double* uo = rup + (int64_t)item * nlags;
  if constexpr (VS) {
    // the diagonal sums first (kept in registers: acc is dead afterwards), then the rows they are added
    // to (lower / upper skirt snapshots, flat sum, partial chains of the flat parts above m1's) loaded
    // for all of the lane's lags at once: one exposed memory latency per item instead of one per block
    constexpr int kNB = (16 * NT + 31) / 32;
    double sums[kNB];
#pragma unroll
    for (int g = 0; g < kNB; ++g) sums[g] = 0.0;
    diag_blocks<NT, 32>(acc, xs, nlags, lane, [&](int g, int, double v) { sums[g] = v; });
    const double* fo = rflat + (int64_t)item * nlags;
    const int2 fb = c.fl_band[j];
    const int pmask = fb.y & ((1 << (c.fl_H - 1)) - 1);  // parts h < fl_H - 1 added in increasing h
    double rv[kNB], uv[kNB], fv[kNB];
#pragma unroll
    for (int g = 0; g < kNB; ++g) {
      const int L = min(32 * g + (lane >> 1), nlags - 1);  // clamped: the loads are unconditional
      rv[g] = ro[L];
      uv[g] = uo[L];
      fv[g] = fo[L];
    }
    if (pmask) {
      for (int rest = pmask; rest; rest &= rest - 1) {
        const double* po = rpart + (((int64_t)f * (c.fl_H - 1) + __builtin_ctz(rest)) * kMaxChains + fb.x) * nlags;
#pragma unroll
        for (int g = 0; g < kNB; ++g) fv[g] += po[min(32 * g + (lane >> 1), nlags - 1)];
      }
    }
#pragma unroll
    for (int g = 0; g < kNB; ++g) {
      const int L = 32 * g + (lane >> 1);
      if ((lane & 1) == 0 && L < nlags) ro[L] = sums[g] + rv[g] + uv[g] + fv[g];
    }
  } else {
    diag_blocks<NT, 32>(acc, xs, nlags, lane, [&](int L, double v) { ro[L] = v + ro[L] + uo[L]; });
  }
}

// -----------------------------------------------------------------------------------------
// 3t. The three sweeps of the structured autocorrelation on the fp64 VALU, lag-parallel.
//     Measured on MI355X: fp64 VALU FMA sustains ~75 TFLOP/s against ~51 for v_mfma_f64_16x16x4f64,
//     and with every lane owning whole lags a snapshot is a plain register store (the MFMA lag
//     tiles need a diagonal-sum epilogue per snapshot).
//     Unit = one 16-lane DPP row = one (frame, sweep); 4 frames of the same sweep per wave, so the
//     thresholds are wave-uniform.  Lane l owns lags A l .. A l + A - 1 (16 A >= nlags).  Sweep
//     signal s[n] (n in sweep order, 0 past N):
//       kind 0  lower skirt  s[n] = E[N-1-n] D[N-1-n]   snapshots K_j R(N - m1_j) -> rlow
//       kind 1  upper skirt  s[n] = E'[n] D[n]          snapshots K'_j R(m2_j)    -> rup
//       kind 2  flat tops    s[n] = D[n]                flat_j = sum_{m in [m1_j, m2_j)} D[m] D[m+l]
//                                                       (right ends up to N)       -> rflat
//     with R(S)[l] = sum_{n >= S} s[n] s[n+l].  Positions are consumed top-down in blocks of A:
//       acc[u] += sum_{v<A} s[n0+v] * s[n0+v+A l+u]
//     s[n0+v] comes from lane v of the row by DPP row_newbcast (one v_mov_b64_dpp per A FMAs), the
//     window s[n0 + A l + q], q < 2A-1, from the current block's A loads and the previous block's
//     (two register banks, so nothing is copied).  A threshold inside a block splits it into two
//     masked passes.  Flat tops: no subtraction of suffix sums (that cancels when the spectrum above
//     a band dominates it): the accumulator holds the positions since the last event and is added
//     into C chains at each event; band j owns chain j mod C from its restart at m2_j to its
//     emission at m1_j (C chosen on the host so that bands j and j - C never overlap).
//     s is staged per unit in an LDS ring of 512 (+16 mirrored) positions, 128 at a time, the next
//     128 prefetched into registers.
// -----------------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ double row_bcast(double v) {
  // row_newbcast:K; every lane has a source, and bound_ctrl spares the 'old' operand (no init, no nops)
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + K, 0xF, 0xF, true);
}

constexpr int kVsRing = 512;
constexpr int kVsMirror = 16;
// positions staged per chunk; the prefetch of the next chunk has to cover the HBM latency under load
// (64 positions, ~3000 cycles of FMAs, measured too short).  The flat sweep keeps its chains in
// registers, so it stages 128 at a time to stay at two waves per SIMD.
template <int A, int C>
constexpr int vs_chunk() { return (C == 0 && 18 * A < kVsRing - 256) ? 256 : 128; }
template <int C>
constexpr int vs_waves_per_simd() { return 2; }

template <int A, int V = 0>
__device__ __forceinline__ void vs_bcast_all(double (&bb)[A], double cur) {
  if constexpr (V < A) {
    bb[V] = row_bcast<V>(cur);
    vs_bcast_all<A, V + 1>(bb, cur);
  }
}
// acc += s[n0+V] * w with s[n0+V] read from lane V of the row by the FMA itself (DP ALU DPP:
// v_fmac_f64 takes row_newbcast on its first source), so a block costs A^2 FMAs and no moves
template <int V>
__device__ __forceinline__ void fmac_bcast(double& acc, double cur, double w) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(cur), "v"(w), "n"(V));
}
template <int A, int V = 0>
__device__ __forceinline__ void vs_fma_rows(double (&acc)[A], double cur, const double (&lo)[A], const double (&hi)[A]) {
  if constexpr (V < A) {
#pragma unroll
    for (int u = 0; u < A; ++u) fmac_bcast<V>(acc[u], cur, (V + u < A) ? lo[V + u] : hi[V + u - A]);
    vs_fma_rows<A, V + 1>(acc, cur, lo, hi);
  }
}
template <int A>
__device__ __forceinline__ void vs_fma_block(double (&acc)[A], double cur, const double (&lo)[A],
                                             const double (&hi)[A]) {
#ifdef FDLP_VSWEEP_DPP_MOV
  double bb[A];
  vs_bcast_all<A>(bb, cur);
#pragma unroll
  for (int v = 0; v < A; ++v)
#pragma unroll
    for (int u = 0; u < A; ++u) acc[u] = fma(bb[v], (v + u < A) ? lo[v + u] : hi[v + u - A], acc[u]);
#else
  // the DPP source must be two wait states past its VALU write (the compiler cannot see the DPP
  // inside the asm): copy it through one asm that ends in the wait
  double cm;
  asm volatile("v_mov_b64 %0, %1\n\ts_nop 1" : "=v"(cm) : "v"(cur));
  vs_fma_rows<A>(acc, cm, lo, hi);
#endif
}

template <int A, int C>
__global__ __launch_bounds__(64, vs_waves_per_simd<C>()) void ac_vsweep_kernel(DevConsts c, const double* __restrict__ dct,
                                                          double* __restrict__ rlow, double* __restrict__ rup,
                                                          double* __restrict__ rflat,
                                                          double* __restrict__ rpart,
                                                          const SkSnap* __restrict__ snaps,
                                                          const FlatEv* __restrict__ fev, int nframes,
                                                          int ngroups) {
  // snaps / fev (= c.sk_snap / c.fl_ev) as restrict parameters: not clobbered by the output stores,
  // so their wave-uniform reads become scalar loads
  constexpr int kVsChunk = vs_chunk<A, C>();
  static_assert(A % 2 == 0 && A <= 16 && 18 * A < kVsRing - kVsChunk && A <= kVsMirror + 1, "vsweep geometry");
  // row stride 544 doubles = 17 x 256 B: each ds_read_b128 lane group (lanes 0-3,12-15 of one row and
  // 4-11 of the next, MI355X_MICROARCH.md LDS) then covers the 64 banks exactly with the 10-double lane
  // stride of the window reads (A = 10; a 528 stride measured 9.4e7 conflict cycles per launch)
  __shared__ double ring_all[4][kVsRing + 32];
  static_assert(kVsMirror <= 32, "mirror fits the row padding");
  // C == 0: the two skirt sweeps, item = 2 group + skirt (a frame group's two sweeps adjacent on one
  // XCD, so its D rows are read from HBM once); C > 0: the flat-top sweep, item = group
  // (C > 0: item = H group + part, the parts of a frame group adjacent on one XCD)
  const int H = C == 0 ? 2 : c.fl_H;
  const int item = xcd_item();
  if (item >= H * ngroups) return;
  const int g = item / H;
  const int part = item - H * g;
  const int kind = C == 0 ? part : 2;
  const int lane = threadIdx.x;
  const int row = lane >> 4;
  const int l = lane & 15;
  const int f = 4 * g + row;
  const bool fvalid = f < nframes;
  const int N = c.N, B = c.B, nlags = c.nlags;
  const double* drow = dct + (int64_t)(fvalid ? f : 0) * N;
  const double* ew = c.sk_e + (int64_t)(kind == 1 ? N : 0);
  double* rg = ring_all[row];
  const int nlo = kind == 2 ? c.fl_part_lo[part] : c.sk_min[kind];
  const int nhi = kind == 2 ? c.fl_part_hi[part] : N;
  const int kbeg = kind == 2 ? c.fl_part_ev[part] : 0;
  const int kend = kind == 2 ? c.fl_part_ev[part + 1] : B;
  // chains left for the parts below (flat, part < H - 1)
  auto part_store = [&](auto&& value) {
    if (kind == 2 && part < H - 1) {
      for (int cc = 0; cc < C; ++cc) {
        double* o = rpart + (((int64_t)f * (H - 1) + part) * kMaxChains + cc) * nlags;
#pragma unroll
        for (int u = 0; u < A; ++u)
          if (fvalid && A * l + u < nlags) o[A * l + u] = value(cc, u);
      }
    }
  };
  if (nhi <= nlo) {  // nothing to sweep: every snapshot / emission is zero
    for (int k = kbeg; k < kend; ++k) {
      const int band = kind == 2 ? fev[k].band : snaps[kind * B + k].band;
      if (kind == 2 && fev[k].type == 0) continue;
      double* o = (kind == 0 ? rlow : (kind == 1 ? rup : rflat)) + ((int64_t)f * B + band) * nlags;
#pragma unroll
      for (int u = 0; u < A; ++u)
        if (fvalid && A * l + u < nlags) o[A * l + u] = 0.0;
    }
    part_store([](int, int) { return 0.0; });
    return;
  }

  // ---- staging: value at sweep position n, prefetched 128 positions ahead ----------------------
  constexpr int kPf = kVsChunk / 16;
  double pf[kPf], pe[C == 0 ? kPf : 1];
  // unconditional (clamped) loads: no branches around them, and their registers are read only in
  // commit, one chunk later, so the wait for them is not pulled into the FMA loop
  auto issue = [&](int base) {
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int n = min(max(base + 16 * q + l, 0), N - 1);
      const int m = kind == 0 ? N - 1 - n : n;
      pf[q] = __builtin_nontemporal_load(drow + m);
      if constexpr (C == 0) pe[q] = ew[m];
    }
  };
  auto commit = [&](int base) {
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int n = base + 16 * q + l;
      const int slot = n & (kVsRing - 1);
      double v = pf[q];
      if constexpr (C == 0) v = pe[q] * v;
      v = (n >= 0 && n < N) ? v : 0.0;
      rg[slot] = v;
      if (slot < kVsMirror) rg[kVsRing + slot] = v;
    }
  };
  const int b_top = (nhi - 1) / A;
  const int b_bot = nlo / A;

  double acc[A];
#pragma unroll
  for (int u = 0; u < A; ++u) acc[u] = 0.0;
  double ch[C > 0 ? C : 1][A];
#pragma unroll
  for (int k = 0; k < (C > 0 ? C : 1); ++k)
#pragma unroll
    for (int u = 0; u < A; ++u) ch[k][u] = 0.0;

  // ---- output rows: parked in registers nothing else uses and stored at the next chunk boundary,
  // right after the ring commit and before the next prefetch.  A VMEM store's data registers must
  // not be rewritten before the store completes (vmcnt, in order with the prefetch loads), so storing
  // from reused registers would put a wait for the prefetch at the head of every block.
  constexpr int P = C == 0 ? 2 : 1;
  double* const outb = kind == 0 ? rlow : (kind == 1 ? rup : rflat);
  double pend[P][A];
  int64_t prow[P];
  int npend = 0;
#pragma unroll
  for (int i = 0; i < P; ++i) {
    prow[i] = 0;
#pragma unroll
    for (int u = 0; u < A; ++u) pend[i][u] = 0.0;
  }
  auto flush = [&]() {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if (i < npend) {
        double* o = outb + prow[i];
#pragma unroll
        for (int u = 0; u < A; ++u)
          if (fvalid && A * l + u < nlags) o[A * l + u] = pend[i][u];
      }
    }
    npend = 0;
  };
  auto push = [&](const double (&v)[A], double K, int band) {
    if (npend == P) flush();
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if (i == npend) {
#pragma unroll
        for (int u = 0; u < A; ++u) pend[i][u] = K * v[u];
        prow[i] = ((int64_t)f * B + band) * nlags;
      }
    }
    ++npend;
  };

  // chunks [lo_loaded, lo_loaded + 512) resident; the top block needs up to A b_top + 17 A - 2
  int lo_loaded = ((A * b_top + 17 * A - 1 + kVsChunk - 1) / kVsChunk) * kVsChunk;
  issue(lo_loaded - kVsChunk);
  auto ensure = [&](int n0) {
    while (n0 < lo_loaded) {  // wave-uniform
      lo_loaded -= kVsChunk;
      commit(lo_loaded);
      flush();
      issue(lo_loaded - kVsChunk);
      wave_lds_sync();
    }
  };
  ensure(A * b_top);  // stages [lo_loaded, initial lo_loaded), which covers the top block's window

  // ---- events (wave-uniform) ------------------------------------------------------------------
  int k = kbeg;
  // event records are read with scalar loads: the index is wave-uniform, readfirstlane says so (a
  // vector load here would wait for the outstanding prefetch at every event)
  auto ev_S = [&](int kk) -> int {
    kk = __builtin_amdgcn_readfirstlane(kk);
    if (kk >= kend) return -1;
    return kind == 2 ? fev[kk].S : snaps[__builtin_amdgcn_readfirstlane(kind * B + kk)].S;
  };
  int evS = ev_S(k);
  // all events at position S (positions >= S consumed)
  auto handle_at = [&](int S) {
    if constexpr (C > 0) {  // flat: fold the positions since the last event into every chain
#pragma unroll
      for (int cc = 0; cc < C; ++cc)
#pragma unroll
        for (int u = 0; u < A; ++u) ch[cc][u] += acc[u];
#pragma unroll
      for (int u = 0; u < A; ++u) acc[u] = 0.0;
    }
    while (evS == S) {
      if constexpr (C > 0) {
        const FlatEv e = fev[__builtin_amdgcn_readfirstlane(k)];
#pragma unroll
        for (int cc = 0; cc < C; ++cc) {
          if (cc == e.chain) {
            if (e.type == 1) push(ch[cc], 1.0, e.band);
#pragma unroll
            for (int u = 0; u < A; ++u) ch[cc][u] = e.type == 0 ? 0.0 : ch[cc][u];
          }
        }
      } else {
        const SkSnap e = snaps[__builtin_amdgcn_readfirstlane(kind * B + k)];
        push(acc, e.K, e.band);
      }
      ++k;
      evS = ev_S(k);
    }
  };

  // one block [n0, n0 + A): positions at or above a pending event are consumed first (masked pass),
  // then the event is handled; usually a single unmasked pass
  auto block = [&](int n0, double (&lo)[A], const double (&hi)[A]) {
    ensure(n0);
    const int base = (n0 + A * l) & (kVsRing - 1);
#pragma unroll
    for (int q = 0; q < A; ++q) lo[q] = rg[base + q];
    const double cur = rg[(n0 + l) & (kVsRing - 1)];
    const int pos = n0 + l;
    int hi_m = min(n0 + A, nhi);
    for (;;) {
      while (evS >= hi_m) handle_at(evS);
      const int lo_m = max(max(evS, n0), nlo);
      vs_fma_block<A>(acc, (pos >= lo_m && pos < hi_m) ? cur : 0.0, lo, hi);
      if (lo_m <= n0 || lo_m <= nlo) break;
      hi_m = lo_m;
    }
  };

  double X[A], Y[A];
  {
    const int base = (A * b_top + A + A * l) & (kVsRing - 1);
#pragma unroll
    for (int q = 0; q < A; ++q) Y[q] = rg[base + q];
  }
  for (int b = b_top; b >= b_bot;) {
    block(A * b, X, Y);
    if (--b < b_bot) break;
    block(A * b, Y, X);
    --b;
  }
  while (k < kend) handle_at(evS);
  flush();
  if constexpr (C > 0) {
    part_store([&](int cc, int u) {
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < C; ++q)
        if (q == cc) v = ch[q][u] + acc[u];
      return v;
    });
  }
  // keep the parked rows' registers reserved for the whole sweep (see above)
#pragma unroll
  for (int i = 0; i < P; ++i)
#pragma unroll
    for (int u = 0; u < A; ++u) asm volatile("" ::"v"(pend[i][u]));
}

template <int NT>
constexpr int autocorr_lds_doubles() {
  constexpr int kEpi = (16 * 4 + 15) * 17;
  return 2 * kAcRing > kEpi ? 2 * kAcRing : kEpi;
}

// -----------------------------------------------------------------------------------------
// 3v. circular autocorrelation on the fp64 VALU (direct path, FDLP_AUTOCORR_VALU=1; MFMA is the default
//     there: the VALU variant clocks down under full fp64 FMA load, 27.1 vs 25.1 ms per batch).
//
// Measured on MI355X: v_fma_f64 sustains 75.8 TFLOP/s, v_mfma_f64_16x16x4f64 only ~51 TFLOP/s
// (benchmarks/mfma_f64_peak.hip), and the MFMA lag tiling above wastes 13.6 % of its MACs, so a
// register-blocked VALU kernel is the faster design for this fp64 path.
// One wave per (frame, band).  Lane = (lag group g, slice s), g = lane>>3, s = lane&7: lanes own
// LG consecutive lags [LG*g, LG*g+LG) and, in each 64-position super-block, the 8 positions
// 8s..8s+7.  Per super-block a lane loads its 8 x[m] and the LG+7 window values x[m+LG*g+...]
// from the LDS ring and issues 8*LG FMAs (152 FMAs per 34 LDS reads for p = 150).  The 8 slices of a
// lag group are summed with DPP at the end.
// -----------------------------------------------------------------------------------------
__device__ __forceinline__ double sum8(double v) {  // over the 8 lanes of a half DPP row
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror: lane i <-> 7-i inside each 8-lane half
  return v;
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

template <int MB, int WIN, int Q = 0>
__device__ __forceinline__ void load_window(double* a, double* b, uint32_t xa, uint32_t wa) {
  if constexpr (Q < MB) a[Q] = lds_ld<8 * Q>(xa);
  if constexpr (Q < WIN) b[Q] = lds_ld<8 * Q>(wa);
  if constexpr (Q + 1 < (MB > WIN ? MB : WIN)) load_window<MB, WIN, Q + 1>(a, b, xa, wa);
}

template <int LG>
__global__ __launch_bounds__(64, 4) void autocorr_valu_kernel(DevConsts c, const double* __restrict__ dct,
                                                              const double* __restrict__ dense,
                                                              double* __restrict__ rout) {
  constexpr int MB = 8;                 // positions per lane per super-block
  constexpr int WIN = MB + LG - 1;      // window values per lane
  static_assert(8 * LG + 64 <= kAcChunk + 64, "window halo must fit one chunk");
  __shared__ double xs[2 * kAcRing];

  const int item = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = c.N;
  int lo, hi;
  const double* drow;
  const double* wrow = nullptr;
  if (dense) {
    lo = 0;
    hi = N;
    drow = dense + (int64_t)item * N;
  } else {
    const int f = item / c.B, j = item % c.B;
    lo = c.lo[j];
    hi = c.hi[j];
    drow = dct + (int64_t)f * N;
    wrow = c.fbank + (int64_t)j * N;
  }
  // lane -> (lag group g, slice sl): slices 0-3 in lanes 0-31 and 4-7 in lanes 32-63, so each
  // 32-lane LDS service group reads 32 distinct banks for odd LG (offsets 8*sl + LG*g mod 32).
  const int sl = (lane & 3) + 4 * (lane >> 5);
  const int g = (lane >> 2) & 7;
  double acc[LG];
#pragma unroll
  for (int q = 0; q < LG; ++q) acc[q] = 0.0;

  const int span = hi - lo;
  const int nsb = (span + 63) / 64;                     // super-blocks of 64 positions
  const int nchunks = (nsb + kAcPer - 1) / kAcPer;
  double dv[kAcPer], wv[kAcPer];
  auto fetch = [&](int ch) {
#pragma unroll
    for (int q = 0; q < kAcPer; ++q) {
      int pos = lo + kAcChunk * ch + 64 * q + lane;
      if (pos >= N) pos -= N;
      const bool ok = pos >= lo && pos < hi;
      dv[q] = ok ? drow[pos] : 0.0;
      wv[q] = ok ? (wrow ? wrow[pos] : 1.0) : 0.0;
    }
  };
  auto store = [&](int ch) {
#pragma unroll
    for (int q = 0; q < kAcPer; ++q) {
      const int slot = (kAcChunk * ch + 64 * q + lane) & (kAcRing - 1);
      const double x = wv[q] * dv[q];  // filt * dct  (:191)
      xs[slot] = x;
      xs[slot + kAcRing] = x;
    }
  };
  if (nsb > 0) {
    fetch(0);
    store(0);
    fetch(1);
    store(1);
    fetch(2);
  }
  __syncthreads();
  // 32-bit LDS byte address of xs (address space 3), as ds_read expects
  const uint32_t xs_addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) double*)xs);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int sb_end = min(kAcPer, nsb - kAcPer * ch);
    const int rbase = (kAcChunk * ch) & (kAcRing - 1);
    for (int sb = 0; sb < sb_end; ++sb) {
      const uint32_t xa = xs_addr + 8u * (uint32_t)(rbase + 64 * sb + MB * sl);
      const uint32_t wa = xa + 8u * (uint32_t)(LG * g);
      double a[MB], b[WIN];
      load_window<MB, WIN>(a, b, xa, wa);
      lds_wait();
      // pin every loaded value behind the wait: the compiler does not know the asm loads are
      // asynchronous, so no use (or copy) of a/b may be scheduled before lgkmcnt(0)
#pragma unroll
      for (int q = 0; q < MB; ++q) asm volatile("" : "+v"(a[q]));
#pragma unroll
      for (int q = 0; q < WIN; ++q) asm volatile("" : "+v"(b[q]));
#pragma unroll
      for (int q = 0; q < MB; ++q)
#pragma unroll
        for (int t = 0; t < LG; ++t) acc[t] = fma(a[q], b[q + t], acc[t]);
    }
    __syncthreads();
    store(ch + 2);
    if (ch + 3 <= nchunks) fetch(ch + 3);
    __syncthreads();
  }
  const int nlags = c.nlags;
#pragma unroll
  for (int t = 0; t < LG; ++t) {
    double v = acc[t];
    v += dpp_f64<0xB1>(v);  // quad: lanes 4g..4g+3 hold slices 0-3 (or 4-7)
    v += dpp_f64<0x4E>(v);
    v += __shfl_xor(v, 32, 64);
    const int L = LG * g + t;
    if (lane < 32 && (lane & 3) == 0 && L < nlags) rout[(int64_t)item * nlags + L] = v;
  }
}

// -----------------------------------------------------------------------------------------
// 4. Levinson-Durbin (features.py:226-228): Toeplitz(r[0..p-1]) a' = -r[1..p]; a = [1, a'];
//    gg = r0 + sum_{l=0}^{p} a_l r_{l+1}.  Four items per wave: an item's a[] is spread over a
//    16-lane DPP row (lane l owns a_i, i = l + 16m); the per-order dot product is a 4-step DPP
//    reduction and the reversed operand a_{k-i} comes from a per-row LDS mirror.
// -----------------------------------------------------------------------------------------
template <int SL>
__global__ __launch_bounds__(64) void levinson_kernel(int p, int nlags, int items, const double* __restrict__ r,
                                                      double* __restrict__ aout,
                                                      double* __restrict__ ggout) {
  constexpr int RS = 16 * SL + 16;  // >= nlags
  constexpr int AS = 16 * SL;
  __shared__ double rs[4][RS];
  __shared__ double as[4][AS];
  const int g = threadIdx.x >> 4;
  const int l = threadIdx.x & 15;
  const int item = blockIdx.x * 4 + g;
  const bool valid = item < items;
  for (int q = l; q < RS; q += 16) rs[g][q] = (valid && q < nlags) ? r[(int64_t)item * nlags + q] : 0.0;
  wave_lds_sync();
  double a[SL];
#pragma unroll
  for (int m = 0; m < SL; ++m) a[m] = (l + 16 * m == 0) ? 1.0 : 0.0;
  double E = rs[g][0];
  for (int k = 1; k <= p; ++k) {
    double part = 0.0;
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const int i = l + 16 * m;
      if (16 * m < k && i >= 1 && i < k) part += a[m] * rs[g][k - i];
    }
    const double acc = rs[g][k] + row_sum16(part);
    const double kappa = -acc / E;
#pragma unroll
    for (int m = 0; m < SL; ++m)
      if (16 * m < k) as[g][l + 16 * m] = a[m];
    wave_lds_sync();
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const int i = l + 16 * m;
      if (16 * m <= k) {
        if (i >= 1 && i < k) a[m] = a[m] + kappa * as[g][k - i];
        else if (i == k) a[m] = kappa;
      }
    }
    wave_lds_sync();
    E = E * (1.0 - kappa * kappa);
  }
  double part = 0.0;
#pragma unroll
  for (int m = 0; m < SL; ++m) {
    const int i = l + 16 * m;
    if (i <= p) part += a[m] * rs[g][i + 1];
  }
  const double gg = rs[g][0] + row_sum16(part);
  if (valid) {
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const int i = l + 16 * m;
      if (i <= p) aout[(int64_t)item * (p + 1) + i] = a[m];
    }
    if (l == 0) ggout[item] = gg;
  }
}

// -----------------------------------------------------------------------------------------
// 5. LPC cepstrum (features.py:233-246): alpha_n = -a_n (0 beyond p); c0 = log(sqrt(gg));
//    c_n = alpha_n + sum_{k=1}^{n-1} ((k/n) alpha_{n-k}) c_k.  Block-parallel over 64 n at a
//    time: the part from finished blocks is a lane-parallel dot product, the in-block part a
//    64-step broadcast recurrence.
// -----------------------------------------------------------------------------------------
constexpr int kCepMaxM = 4096;
constexpr int kCepMaxP = 1024;
__global__ __launch_bounds__(64) void cepstrum_kernel(int p, int M, const double* __restrict__ a,
                                                      const double* __restrict__ gg,
                                                      double* __restrict__ cep) {
  extern __shared__ double sh[];
  const int item = blockIdx.x;
  const int lane = threadIdx.x;
  const int nal = max(M, p + 1) + 64;
  double* al = sh;        // alpha, zero padded
  double* cs = sh + nal;  // finished c_k
  for (int q = lane; q < nal; q += 64)
    al[q] = (q >= 1 && q <= p) ? -a[(int64_t)item * (p + 1) + q] : 0.0;
  __syncthreads();
  const double g = gg[item];
  for (int b0 = 0; b0 < M; b0 += 64) {
    const int n = b0 + lane;
    double acc = 0.0;
    if (n < M && n >= 2) {
      const int kstart = max(1, b0 - p);
      for (int k = kstart; k < b0; ++k) {
        const int d = n - k;
        if (d <= p) acc += (((double)k / (double)n) * al[d]) * cs[k];
      }
    }
    double mine = 0.0;
    for (int kk = 0; kk < 64; ++kk) {
      const int kg = b0 + kk;
      if (kg >= M) break;
      if (lane == kk) {
        if (kg == 0) mine = log(sqrt(g));
        else if (kg == 1) mine = al[1];
        else mine = acc + al[kg];
      }
      const double ck = __shfl(mine, kk, 64);
      if (kg >= 1 && lane > kk && n < M) {
        const int d = n - kg;
        if (d <= p) acc += (((double)kg / (double)n) * al[d]) * ck;
      }
    }
    if (n < M) {
      cs[n] = mine;
      cep[(int64_t)item * M + n] = mine;
    }
    __syncthreads();
  }
}

// -----------------------------------------------------------------------------------------
// 4-6 fused: Levinson -> gg -> LPC cepstrum -> modulation weights -> envelope, per (frame, band)
// item, 16 lanes (one DPP row) per item, 4 items per wave.  Only r is read and only the kk
// envelope samples are written (a/gg/cep optionally, for parity debugging).
//   Levinson   features.py:226-228          cepstrum   features.py:233-246
//   weights    computeFDLPSpectrogram.py:194-200
//   envelope   computeFDLPSpectrogram.py:201-205: exp(Re sum_n c'_n cos(2 pi n t / env_nfft))
//              * hanning(kk)[t] / hamming(kk)[t]  (fft(., env_nfft) truncates/zero-pads c')
// Per-item LDS region (doubles): [a: NAL, zero beyond p][r: nlags, later c: M]; phase 3 reuses the
// a slots for c'.  Envelope cosines come from a Chebyshev recurrence seeded with cos(2 pi t/env_nfft).
// -----------------------------------------------------------------------------------------
struct LpcEnvArgs {
  int p, nlags, M, Me, kk, env_nfft, odd_zero, items, region;
  int la_len;             // lattice kernel with a register cepstrum: doubles of the a area (cs follows, Me long)
  const double* r;
  const double* weights;  // [3, M]
  const double* env_cos;  // [env_nfft]
  const double* env_win;  // [kk, 2]: (hanning / hamming ratio, 1.0)
  double* env;            // [items, kk]
  double* a_out;          // nullable [items, p+1]
  double* gg_out;         // nullable [items]
  double* cep_out;        // nullable [items, M]
  const double* a_ext;    // DM = 2: a [items, a_stride] and gg [items] from durbin8_kernel
  const double* gg_ext;
  int a_stride;
};

// Durbin recursion with a[] resident in LDS (la[0..p], zero beyond) and r in LDS (lr): lane l of
// the 16-lane row sums a_i r_{k-i} over i = l+1, l+17, ... and updates the symmetric pairs
// (a_i, a_{k-i}) in place, so no mirror copy is needed.  Both loops run a uniform trip count: the
// a_i with i >= k are still zero and lr[-15..-1] is the zero tail of la, so the extra terms vanish.
// 1/E comes from v_rcp_f64 and two Newton steps.  Returns gg.
__device__ __forceinline__ double durbin16(double* la, const double* lr, int p, int l) {
  double E = lr[0];
  for (int k = 1; k <= p; ++k) {
    const int S = (k + 14) >> 4;
    double part = 0.0;
    for (int s = 0; s < S; ++s) {
      const int i = l + 1 + 16 * s;
      part = fma(la[i], lr[k - i], part);
    }
    const double acc = lr[k] + row_sum16(part);
    double rE = __builtin_amdgcn_rcp(E);
    rE = fma(rE, fma(-E, rE, 1.0), rE);
    rE = fma(rE, fma(-E, rE, 1.0), rE);
    const double kappa = -acc * rE;
    wave_lds_sync();
    const int S2 = (k + 31) >> 5;
    for (int s = 0; s < S2; ++s) {
      const int i = l + 1 + 16 * s;
      if (2 * i <= k) {  // i == k - i writes the same value twice
        const int j = k - i;
        const double ai = la[i], aj = la[j];
        la[i] = fma(kappa, aj, ai);
        la[j] = fma(kappa, ai, aj);
      }
    }
    if (l == 0) la[k] = kappa;
    wave_lds_sync();
    E = E * (1.0 - kappa * kappa);
  }
  double part = 0.0;
  for (int i = l; i <= p; i += 16) part = fma(la[i], lr[i + 1], part);
  return lr[0] + row_sum16(part);
}

// 16 finished-block terms of the cepstrum: acc += (k c_k from lane j) * alpha_{n-k} (alpha_{n-k} = al[-j]).
// The 16 LDS values are loaded first: the FMAs are inline asm, which the scheduler does not move loads
// across, so loads interleaved with them would each wait out their full LDS latency.
__device__ __forceinline__ void cep_terms16(double& a0, double& a1, double& a2, double& a3, double kc,
                                            const double* al) {
  double v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = al[-j];
  fmac_bcast<0>(a0, kc, v[0]);
  fmac_bcast<1>(a1, kc, v[1]);
  fmac_bcast<2>(a2, kc, v[2]);
  fmac_bcast<3>(a3, kc, v[3]);
  fmac_bcast<4>(a0, kc, v[4]);
  fmac_bcast<5>(a1, kc, v[5]);
  fmac_bcast<6>(a2, kc, v[6]);
  fmac_bcast<7>(a3, kc, v[7]);
  fmac_bcast<8>(a0, kc, v[8]);
  fmac_bcast<9>(a1, kc, v[9]);
  fmac_bcast<10>(a2, kc, v[10]);
  fmac_bcast<11>(a3, kc, v[11]);
  fmac_bcast<12>(a0, kc, v[12]);
  fmac_bcast<13>(a1, kc, v[13]);
  fmac_bcast<14>(a2, kc, v[14]);
  fmac_bcast<15>(a3, kc, v[15]);
}

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

__device__ __forceinline__ void cep_fma16(double& a0, double& a1, double& a2, double& a3, double kc,
                                          const double (&v)[16]) {
  fmac_bcast<0>(a0, kc, v[0]);
  fmac_bcast<1>(a1, kc, v[1]);
  fmac_bcast<2>(a2, kc, v[2]);
  fmac_bcast<3>(a3, kc, v[3]);
  fmac_bcast<4>(a0, kc, v[4]);
  fmac_bcast<5>(a1, kc, v[5]);
  fmac_bcast<6>(a2, kc, v[6]);
  fmac_bcast<7>(a3, kc, v[7]);
  fmac_bcast<8>(a0, kc, v[8]);
  fmac_bcast<9>(a1, kc, v[9]);
  fmac_bcast<10>(a2, kc, v[10]);
  fmac_bcast<11>(a3, kc, v[11]);
  fmac_bcast<12>(a0, kc, v[12]);
  fmac_bcast<13>(a1, kc, v[13]);
  fmac_bcast<14>(a2, kc, v[14]);
  fmac_bcast<15>(a3, kc, v[15]);
}

// The window blocks w = WI .. W-1 of one cepstrum block (CB < 0): block w's 16 alpha values were issued
// before this call (va); block w + 1's are issued before block w's FMAs (double buffer), and the wait
// before the FMAs leaves those 16 in flight (LDS operations complete in order).
template <int W, int WI>
__device__ __forceinline__ void cep_window(double& a0, double& a1, double& a2, double& a3, const double (&kc)[W],
                                           double (&va)[16], double (&vb)[16], uint32_t addr) {
  if constexpr (WI < W) {
    if constexpr (WI + 1 < W) {
      lds_load16<16 * (WI + 1) + 15>(vb, addr);
      lgkm_wait<15>();  // all of block WI's loads (and the first of WI + 1's) have landed
    } else {
      lgkm_wait<0>();
    }
    // the asm loads' results look ready to the compiler: tie them to the wait (a volatile asm that
    // "rewrites" them), so neither the FMAs nor a register copy can be scheduled above it
#pragma unroll
    for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(va[q]));
    cep_fma16(a0, a1, a2, a3, kc[WI], va);
    cep_window<W, WI + 1>(a0, a1, a2, a3, kc, vb, va, addr);
  }
}

// In-block part of the cepstrum recurrence for coefficient b0 + KK: lane KK finishes c_{b0+KK},
// DPP row_newbcast hands it to the row, the later lanes of the block fold it in.
// a_kg is read from la only up to amax (beyond it a is zero: the reference pads alpha with zeros).
template <int KK>
__device__ __forceinline__ void cep_block_step(int b0, int M, int l, double gg, double inv_n, const double* la,
                                               int n, double& acc, double& mine, int amax = 1 << 30) {
  const int kg = b0 + KK;
  if (kg >= M) return;
  if (l == KK) {
    if (kg == 0) mine = log(sqrt(gg));
    else if (kg == 1) mine = -la[1];
    else mine = -(kg <= amax ? la[kg] : 0.0) - acc * inv_n;
  }
  const double ck = dpp_f64<0x150 + KK>(mine);  // row_newbcast:KK
  if (kg >= 1 && l > KK) acc = fma((double)kg * ck, la[n - kg], acc);
  if constexpr (KK + 1 < 16) cep_block_step<KK + 1>(b0, M, l, gg, inv_n, la, n, acc, mine, amax);
}

#ifndef FDLP_LPC_PHASES
#define FDLP_LPC_PHASES 7  // bit 0 Durbin, 1 cepstrum, 2 envelope (benchmarks/lpc_env_phases.hip only)
#endif

// -----------------------------------------------------------------------------------------
// Durbin in lattice form, register-resident (no LDS traffic, no barriers).  Lane l of the 16-lane
// row owns positions m = l + 16 s (s < SL) of
//   A = a^(k)   (a_0 = 1)                      and   B = the reversed predictor, b_m = a_{k-1-m},
//   R1[m] = r_{m+1},
// so the order-k dot product  r_k + sum_{i=1}^{k-1} a_i r_{k-i} = sum_{m<k} b_m r_{m+1}  is lane-aligned,
// and the update  a_i <- a_i + kappa a_{k-i}  is  A <- A + kappa (z B),  B <- (z B) + kappa A  with z the
// shift by one position (DPP row_ror:1, lane 0 takes lane 15 of the previous slot).  This is the same
// arithmetic as the reference's recursion (features.py:226-228 via solve_toeplitz): fma(kappa, a_{k-i}, a_i)
// for both halves of every symmetric pair, so B stays the bitwise mirror of A.  Orders k in
// [16Q, 16Q+16) touch slots 0..Q only (positions > k are zero), hence the per-phase templates.
// -----------------------------------------------------------------------------------------
template <int SL, int Q>
__device__ __forceinline__ void lattice_phase(double (&A)[SL], double (&B)[SL], const double (&R1)[SL], double& E,
                                              int k0, int k1, bool lane0) {
  for (int k = k0; k < k1; ++k) {
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int s = 0; s <= Q; s += 2) p0 = fma(B[s], R1[s], p0);
#pragma unroll
    for (int s = 1; s <= Q; s += 2) p1 = fma(B[s], R1[s], p1);
    const double acc = row_sum16(p0 + p1);
    double rE = __builtin_amdgcn_rcp(E);
    rE = fma(rE, fma(-E, rE, 1.0), rE);
    rE = fma(rE, fma(-E, rE, 1.0), rE);
    const double kappa = -acc * rE;
    // zB without a select: lanes 1..15 take lane l-1 (row_shr:1); lane 0 takes 0 (slot 0, bound_ctrl)
    // or keeps the old value, a 64-bit row_newbcast:15 of the previous slot (one v_mov_b64_dpp)
    double bsh[Q + 1];
    bsh[0] = __builtin_amdgcn_update_dpp(0.0, B[0], 0x111, 0xF, 0xF, true);
#pragma unroll
    for (int s = 1; s <= Q; ++s) {
      const double prev15 = __builtin_amdgcn_update_dpp(0.0, B[s - 1], 0x15F, 0xF, 0xF, true);
      bsh[s] = __builtin_amdgcn_update_dpp(prev15, B[s], 0x111, 0xF, 0xF, false);
    }
#pragma unroll
    for (int s = 0; s <= Q; ++s) {
      // B first: its old value lives on in bsh[], so both updates are in place (no register copies)
      B[s] = fma(kappa, A[s], bsh[s]);
      A[s] = fma(kappa, bsh[s], A[s]);
    }
    E = E * (1.0 - kappa * kappa);
  }
}

template <int SL, int Q>
__device__ __forceinline__ void lattice_durbin(double (&A)[SL], double (&B)[SL], const double (&R1)[SL], double& E,
                                               int p, bool lane0) {
  const int k0 = Q == 0 ? 1 : 16 * Q;
  const int k1 = min(p + 1, 16 * Q + 16);
  if (k0 < k1) lattice_phase<SL, Q>(A, B, R1, E, k0, k1, lane0);
  if constexpr (Q + 1 < SL) lattice_durbin<SL, Q + 1>(A, B, R1, E, p, lane0);
}

// -----------------------------------------------------------------------------------------
// Durbin in lattice form with CONTIGUOUS chunks: in phase S (orders k < 16 S) lane l of the row owns
// positions l S .. l S + S - 1 of A = a^(k), of the mirror B (b_m = a^(k)_{k-m}) and of R1 (r_{m+1}).
// The one-position shift z B of the lattice update then moves data between lanes only at the chunk
// boundary: one DPP row_shr:1 of the last slot per order (bound_ctrl: lane 0 takes 0), and the
// in-lane part of the shift is free because B alternates between two register banks (the new B[j] is
// written from the old B[j-1]).  Per order: 3 S FMAs (update of A and B, next order's dot product)
// + the 16-lane reduction + the 1/E Newton steps, instead of the slot-major layout's 3 S FMAs + 3 S
// DPP moves.  Capacity grows with k: every 16 orders A and B are re-laid out through the item's LDS
// scratch (S -> S + 1 positions per lane) and R1 is reloaded for the new layout (prefetched from
// global memory one phase ahead).  Same recursion as lattice_phase (features.py:226-228): both halves
// of every symmetric pair are fma(kappa, a_{k-i}, a_i).
// -----------------------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void contig_step(double (&A)[S], const double (&Bs)[S], double (&Bd)[S],
                                            const double (&R1)[S], double& part, double& E) {
  const double acc = row_sum16(part);  // r_k + sum_i a_i r_{k-i} = sum_m b_m r_{m+1}
  double rE = __builtin_amdgcn_rcp(E);
  rE = fma(rE, fma(-E, rE, 1.0), rE);
  rE = fma(rE, fma(-E, rE, 1.0), rE);
  const double kappa = -acc * rE;
  // z B at slot 0: the last slot of lane l-1 (row_shr:1); lane 0 takes 0 (bound_ctrl)
  const double z0 = __builtin_amdgcn_update_dpp(0.0, Bs[S - 1], 0x111, 0xF, 0xF, true);
  double p0 = 0.0, p1 = 0.0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const double zb = j == 0 ? z0 : Bs[j - 1];
    Bd[j] = fma(kappa, A[j], zb);
    A[j] = fma(kappa, zb, A[j]);
    if (j & 1) p1 = fma(Bd[j], R1[j], p1);
    else p0 = fma(Bd[j], R1[j], p0);
  }
  part = p0 + p1;
  E = E * (1.0 - kappa * kappa);
}

// R1 of phase S for lane l: r_{lS+j+1} for positions <= p, 0 beyond (and for invalid items)
template <int S>
__device__ __forceinline__ void contig_load_r1(double (&R1)[S], const double* rr, int nlags, int p, int l, bool valid) {
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int m = l * S + j;
    const double v = rr[min(m + 1, nlags - 1)];
    R1[j] = (valid && m <= p) ? v : 0.0;
  }
}

// vec (S per lane, contiguous) -> la -> out (S + 1 per lane); positions >= 16 S read as 0
template <int S>
__device__ __forceinline__ void contig_relayout(const double (&v)[S], double (&out)[S + 1], double* la, int l) {
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j < S; ++j) la[l * S + j] = v[j];
  la[16 * S + l] = 0.0;
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j <= S; ++j) out[j] = la[l * (S + 1) + j];
}

// Orders k in [k0, k1) of phase S, then the next phase (or, after order p, the final A in place).
template <int SL, int S>
__device__ __forceinline__ void contig_durbin(double (&A)[S], double (&B)[S], double (&R1)[S], double& part,
                                              double& E, double* la, const double* rr, int nlags, int p, int l,
                                              bool valid, double& gg, double r0) {
  const int k0 = S == 1 ? 1 : 16 * (S - 1);
  const int k1 = min(p + 1, 16 * S);
  constexpr int SN = S < SL ? S + 1 : S;
  double R1n[SN];
  if constexpr (S < SL) {
    if (k1 <= p) contig_load_r1<SN>(R1n, rr, nlags, p, l, valid);  // next phase's R1, consumed after the loop
  }
  double B2[S];
  int k = k0;
  for (; k + 1 < k1; k += 2) {
    contig_step<S>(A, B, B2, R1, part, E);
    contig_step<S>(A, B2, B, R1, part, E);
  }
  if (k < k1) {
    contig_step<S>(A, B, B2, R1, part, E);
#pragma unroll
    for (int j = 0; j < S; ++j) B[j] = B2[j];
  }
  if constexpr (S < SL) {
    if (k1 <= p) {
      double An[S + 1], Bn[S + 1];
      contig_relayout<S>(A, An, la, l);
      contig_relayout<S>(B, Bn, la, l);
      contig_durbin<SL, S + 1>(An, Bn, R1n, part, E, la, rr, nlags, p, l, valid, gg, r0);
      return;
    }
  }
  // order p done: gg = r0 + sum_{m=0}^{p} a_m r_{m+1} (the reference's off-by-one, features.py:228);
  // A goes to la[0 .. 16 S) in position order for the cepstrum (zeros beyond p)
  double q0 = 0.0, q1 = 0.0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    if (j & 1) q1 = fma(A[j], R1[j], q1);
    else q0 = fma(A[j], R1[j], q0);
  }
  gg = r0 + row_sum16(q0 + q1);
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j < S; ++j) la[l * S + j] = A[j];
}

// -----------------------------------------------------------------------------------------
// The contiguous-chunk lattice Durbin with 8 lanes per item (each half of a DPP row is an item, 8 items
// per wave).  Per order the cross-lane part (the 8-lane sum, 1/E by rcp + two Newton steps, kappa, the
// E update: ~20 VALU instructions) is paid once for 8 items instead of 4, and the FMAs (3 per position)
// are the same, so the Durbin issues ~35 % fewer instructions per item than contig_durbin (p = 150).
// In phase S lane li (0..7) owns positions li S .. li S + S - 1 (capacity 8 S, orders < 8 S); the shift
// z B takes lane li - 1's last slot by row_shr:1, which would carry lane 7 of the first item into lane 8
// of the second: the first lane of each item takes 0 instead (a select).  Standalone kernel
// (durbin8_kernel): a [items, p + 1] and gg go to global memory for lpc_env_lattice_kernel's cepstrum and
// envelope phases (DM = 2), which then run at their own occupancy.  Same recursion as contig_step
// (features.py:226-228); only the summation order of the order-k dot product differs (8 lane partials).
// -----------------------------------------------------------------------------------------
#ifndef FDLP_D8_CHAINS
#define FDLP_D8_CHAINS 4  // 2 or 4
#endif
#ifndef FDLP_D8_NEWTON
#define FDLP_D8_NEWTON 2  // Newton steps after v_rcp_f64 for 1/E
#endif
template <int S>
__device__ __forceinline__ void c8_step(double (&A)[S], const double (&Bs)[S], double (&Bd)[S],
                                        const double (&R1)[S], double& part, double& E, bool first) {
  const double acc = sum8(part);  // r_k + sum_i a_i r_{k-i}
  double rE = __builtin_amdgcn_rcp(E);
#pragma unroll
  for (int it = 0; it < FDLP_D8_NEWTON; ++it) rE = fma(rE, fma(-E, rE, 1.0), rE);
  const double kappa = -acc * rE;
  const double zs = __builtin_amdgcn_update_dpp(0.0, Bs[S - 1], 0x111, 0xF, 0xF, true);  // row_shr:1
  const double z0 = first ? 0.0 : zs;
  // the next order's dot product in D independent chains (the chain, not the issue, bounds small S)
  constexpr int D = FDLP_D8_CHAINS;
  double pc[D];
#pragma unroll
  for (int d = 0; d < D; ++d) pc[d] = 0.0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const double zb = j == 0 ? z0 : Bs[j - 1];
    Bd[j] = fma(kappa, A[j], zb);
    A[j] = fma(kappa, zb, A[j]);
    pc[j % D] = fma(Bd[j], R1[j], pc[j % D]);
  }
  if constexpr (D == 4) part = (pc[0] + pc[1]) + (pc[2] + pc[3]);
  else part = pc[0] + pc[1];
  E = E * (1.0 - kappa * kappa);
}

// R1 of phase S for lane li from the item's staged r (rl[m] = r_{m+1}, 0 past p)
template <int S>
__device__ __forceinline__ void c8_load_r1(double (&R1)[S], const double* rl, int li) {
#pragma unroll
  for (int j = 0; j < S; ++j) R1[j] = rl[li * S + j];
}

// A (S per lane) -> sc -> An, Bn (S + 1 per lane).  B is the bitwise mirror of A: after order 8 S - 1,
// b_m = a_{8S-1-m} (both are fma(kappa, a_m, a_{k-m}) in c8_step), so B is read back mirrored from A's
// image instead of being written too; sc[8 S ..] and sc[-8 .. -1] are zeros (positions >= 8 S).
template <int S>
__device__ __forceinline__ void c8_relayout(const double (&A)[S], double (&An)[S + 1], double (&Bn)[S + 1],
                                            double* sc, int li) {
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j < S; ++j) sc[li * S + j] = A[j];
  sc[8 * S + li] = 0.0;
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j <= S; ++j) An[j] = sc[li * (S + 1) + j];
#pragma unroll
  for (int j = 0; j <= S; ++j) Bn[j] = sc[8 * S - 1 - li * (S + 1) - j];
}

template <int SL8, int S>
__device__ __forceinline__ void c8_durbin(double (&A)[S], double (&B)[S], double (&R1)[S], double& part, double& E,
                                          const double* rl, double* sc, int p, int li, bool valid, double r0,
                                          double* ao, double* go, int astride) {
  const int k0 = S == 1 ? 1 : 8 * (S - 1);
  const int k1 = min(p + 1, 8 * S);
  const bool first = li == 0;
  constexpr int SN = S < SL8 ? S + 1 : S;
  double R1n[SN];
  if constexpr (S < SL8) {
    if (k1 <= p) c8_load_r1<SN>(R1n, rl, li);  // next phase's R1 (LDS), consumed after the loop
  }
  double B2[S];
  int k = k0;
  for (; k + 1 < k1; k += 2) {
    c8_step<S>(A, B, B2, R1, part, E, first);
    c8_step<S>(A, B2, B, R1, part, E, first);
  }
  if (k < k1) {
    c8_step<S>(A, B, B2, R1, part, E, first);
#pragma unroll
    for (int j = 0; j < S; ++j) B[j] = B2[j];
  }
  if constexpr (S < SL8) {
    if (k1 <= p) {
      double An[S + 1], Bn[S + 1];
      c8_relayout<S>(A, An, Bn, sc, li);
      c8_durbin<SL8, S + 1>(An, Bn, R1n, part, E, rl, sc, p, li, valid, r0, ao, go, astride);
      return;
    }
  }
  // order p done: gg = r0 + sum_{m=0}^{p} a_m r_{m+1} (the reference's off-by-one, features.py:228)
  double q0 = 0.0, q1 = 0.0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    if (j & 1) q1 = fma(A[j], R1[j], q1);
    else q0 = fma(A[j], R1[j], q0);
  }
  const double gg = r0 + sum8(q0 + q1);
  if (valid) {  // the whole row: a_0 .. a_p, then zeros (A is exactly 0 past p) up to astride
#pragma unroll
    for (int j = 0; j < S; ++j) ao[li * S + j] = A[j];
    for (int m = 8 * S + li; m < astride; m += 8) ao[m] = 0.0;
    if (first) *go = gg;
  }
}

// one wave per 8 items (p + 1 <= 8 SL8 <= astride); a / gg: [items, astride] (zero past p) / [items].  The 8 items' r rows are
// staged in LDS first (one coalesced pass), so each phase's R1 is an LDS read, not a global load
// whose latency the short early phases cannot cover.  LDS per item: r_1 .. r_{8 SL8} and the relayout
// image (8 zeros + 8 SL8); 8 items = 19.5 KB at SL8 = 19, two waves per SIMD.
template <int SL8>
__global__ __launch_bounds__(64, 2) void durbin8_kernel(const double* __restrict__ r, int nlags, int p, int items,
                                                        double* __restrict__ a, double* __restrict__ gg, int astride) {
  constexpr int kR = 8 * SL8;
  constexpr int kItem = kR + 8 + 8 * SL8;
  __shared__ double lds[8 * kItem];
  const int lane = threadIdx.x;
  const int li = lane & 7;
  const int ii = lane >> 3;
  const int item0 = blockIdx.x * 8;
  for (int q = lane; q < 8 * kR; q += 64) {
    const int i = q / kR, m = q - i * kR;
    const int itm = item0 + i;
    double v = 0.0;
    if (itm < items && m <= p && m + 1 < nlags) v = r[(int64_t)itm * nlags + m + 1];
    lds[i * kItem + m] = v;
  }
  double* sc = lds + ii * kItem + kR + 8;
  sc[li - 8] = 0.0;
  wave_lds_sync();
  const int item = item0 + ii;
  const bool valid = item < items;
  const double r0 = valid ? r[(int64_t)item * nlags] : 1.0;
  const double* rl = lds + ii * kItem;
  double A1[1] = {li == 0 ? 1.0 : 0.0}, B1[1] = {li == 0 ? 1.0 : 0.0}, R11[1];
  c8_load_r1<1>(R11, rl, li);
  double part = li == 0 ? R11[0] : 0.0;  // order 1: b^(0) . R1 = r_1
  double E = r0;
  c8_durbin<SL8, 1>(A1, B1, R11, part, E, rl, sc, p, li, valid, r0, a + (int64_t)(valid ? item : 0) * astride,
                    gg + (valid ? item : 0), astride);
}

// lpc_env with the lattice Durbin: persistent waves (grid-stride over groups of 4 items), r read
// straight into registers, LDS only for a (cepstrum) and c (envelope).  Same outputs as lpc_env_kernel.
constexpr int kEnvChunk = 5;  // envelope slots held in registers at a time
// CB > 0 (M <= 16 CB): the cepstrum's finished blocks take c_k from the registers of the lane that
// computed it (v_fmac_f64_dpp row_newbcast, the broadcast is the FMA's source modifier) instead of an
// LDS read per term: one LDS read (alpha_{n-k}) and one FMA per term instead of two reads, a multiply
// and an FMA.  CB < 0: the same over a sliding register window of the last SL + 1 finished blocks
// (any M; the terms with n - k > p are zero).  CB = 0: the LDS form for any M.
// DM: the Durbin phase.  1: the contiguous-chunk Durbin (contig_durbin); 0: the slot-major lattice
// (lattice_durbin, FDLP_LPC_SLOTMAJOR=1); 2: none, a and gg come from durbin8_kernel (A.a_ext, A.gg_ext;
// default where durbin8_kernel is instantiated).
constexpr int kDmSlotMajor = 0, kDmContig = 1, kDmExt = 2;
template <int SL, int CB = 0, int DM = kDmContig>
#ifndef FDLP_LAT_WAVES
#define FDLP_LAT_WAVES 4  // waves per SIMD the lattice kernel is compiled for (register budget)
#endif
__global__ __launch_bounds__(64, FDLP_LAT_WAVES) void lpc_env_lattice_kernel(LpcEnvArgs A_) {
  extern __shared__ double sh[];
  const LpcEnvArgs& A = A_;
  const int ngroups = (A.items + 3) >> 2;
  // (prefetching the next group's r into registers before the envelope phase was measured: no gain,
  // it costs a wave per SIMD of occupancy)
  constexpr bool CONTIG = DM == kDmContig;
  double Rn[DM == kDmSlotMajor ? SL : 1], r0n;
  auto load_r = [&](int grp) {
    const int it = grp * 4 + (threadIdx.x >> 4);
    const double* rr = A.r + (int64_t)(it < A.items ? it : 0) * A.nlags;
    if constexpr (DM == kDmSlotMajor) {
#pragma unroll
      for (int s = 0; s < SL; ++s) Rn[s] = rr[min((int)(threadIdx.x & 15) + 16 * s + 1, A.nlags - 1)];
    }
    if constexpr (DM != kDmExt) r0n = rr[0];
  };
  // DM = 2 with a register cepstrum: the next group's a rows go global -> LDS by DMA (no registers)
  // while this group's envelope runs (it reads only cs, not la)
  auto dma_a = [&](int grp) {
    if constexpr (DM == kDmExt && CB != 0) {
#pragma unroll
      for (int g2 = 0; g2 < 4; ++g2) {
        const int it = min(grp * 4 + g2, A.items - 1);
        const double* src = A.a_ext + (int64_t)it * A.a_stride;  // la_len doubles, 16-B aligned rows
        double* dst = sh + g2 * A.region;
        for (int c0 = 0; c0 < A.la_len; c0 += 128) {  // 64 lanes x 16 B = 128 doubles per copy
          if (c0 + 2 * (int)threadIdx.x < A.la_len)
            __builtin_amdgcn_global_load_lds((const void*)(src + c0 + 2 * threadIdx.x),
                                             (__attribute__((address_space(3))) void*)(dst + c0), 16, 0, 0);
        }
      }
    }
  };
  if (blockIdx.x < ngroups) dma_a(blockIdx.x);
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    load_r(grp);
    // Everything below is re-derived per group from opaque copies, so the compiler cannot hoist
    // group-invariant addresses/tables out of the loop (they would stay live through the Durbin phase).
    int tid = threadIdx.x, p = A.p, M = A.M;
    asm volatile("" : "+v"(tid));
    asm volatile("" : "+s"(p), "+s"(M));
    const int g = tid >> 4;
    const int l = tid & 15;
    const bool lane0 = l == 0;
    // LDS per item: la = a_0..a_p and zeros, then cs = the cepstrum.  The register cepstra (CB != 0)
    // read la only below la_len and keep only the Me coefficients the envelope uses (compact: REVERB's
    // M = 450 would otherwise cut the occupancy to one wave per SIMD); the LDS cepstrum (CB == 0) reads
    // a and c up to M.
    const int NAL = CB != 0 ? A.la_len : (M > p + 1 ? M : p + 1) + 16;
    double* la = sh + g * A.region;
    double* cs = la + NAL;
    const int CSN = CB != 0 ? A.Me : M;  // coefficients kept in cs
    const int H = A.env_nfft >> 1;
    const int TS = (A.env_nfft / 4 + 1 + 15) / 16;
    const int item = grp * 4 + g;
    const bool valid = item < A.items;
    // ---- phase 1: Levinson-Durbin (features.py:226-228) in registers -------------------------
    double gg;
    if constexpr (DM == kDmExt) {
      if constexpr (CB != 0) {
        // la[0 .. la_len) = this group's a rows: LDS-DMA copies issued a group ahead (see below)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        const double* ai = A.a_ext + (int64_t)(valid ? item : 0) * A.a_stride;
        wave_lds_sync();  // the previous group's envelope reads of la are done
        for (int q = l; q < NAL; q += 16) la[q] = (valid && q <= p) ? ai[q] : 0.0;
      }
      gg = valid ? A.gg_ext[item] : 1.0;
    } else if constexpr (CONTIG) {
      const double* rr = A.r + (int64_t)(valid ? item : 0) * A.nlags;
      const double r0 = valid ? r0n : 1.0;
      gg = r0;
      {
        double A1[1] = {lane0 ? 1.0 : 0.0}, B1[1] = {lane0 ? 1.0 : 0.0}, R11[1];
        contig_load_r1<1>(R11, rr, A.nlags, p, l, valid);
        double part = lane0 ? R11[0] : 0.0;  // order 1: b^(0) . R1 = r_1
        double E = r0;
        if (FDLP_LPC_PHASES & 1) contig_durbin<SL, 1>(A1, B1, R11, part, E, la, rr, A.nlags, p, l, valid, gg, r0);
      }
      // la[0 .. 16 SL) holds a_0 .. a_p (zeros beyond p); zero the rest of the a region
      for (int q = l + 16 * SL; q < NAL; q += 16) la[q] = 0.0;
      wave_lds_sync();
      if (valid && A.a_out) {
        for (int m = l; m <= p; m += 16) A.a_out[(int64_t)item * (p + 1) + m] = la[m];
        if (lane0) A.gg_out[item] = gg;
      }
    } else {
      double Av[SL], Bv[SL], R1[SL];
#pragma unroll
      for (int s = 0; s < SL; ++s) {  // branch-free: clamped loads (load_r), then select
        const int m = l + 16 * s;
        R1[s] = (valid && m <= p) ? Rn[s] : 0.0;
        Av[s] = (m == 0) ? 1.0 : 0.0;
        Bv[s] = Av[s];
      }
      const double r0 = valid ? r0n : 1.0;
      double E = r0;
      if (FDLP_LPC_PHASES & 1) lattice_durbin<SL, 0>(Av, Bv, R1, E, p, lane0);
      double part = 0.0;
#pragma unroll
      for (int s = 0; s < SL; ++s) part = fma(Av[s], R1[s], part);
      gg = r0 + row_sum16(part);  // the reference's off-by-one gain (features.py:228)
      wave_lds_sync();  // the previous group's envelope reads of la are done
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const int m = l + 16 * s;
        if (m < NAL) la[m] = m <= p ? Av[s] : 0.0;
        if (valid && A.a_out && m <= p) A.a_out[(int64_t)item * (p + 1) + m] = Av[s];
      }
      for (int q = l + 16 * SL; q < NAL; q += 16) la[q] = 0.0;
      if (valid && A.a_out && lane0) A.gg_out[item] = gg;
    }
    wave_lds_sync();
    // ---- phase 2: cepstrum (features.py:233-246), as in lpc_env_kernel -------------------------
    if constexpr (CB > 0) {
      double kc[CB];  // lane l: n c_n for n = 16 b + l of every finished block b (0 for n = 0)
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        const int b0 = 16 * b;
        if (b0 >= ((FDLP_LPC_PHASES & 2) ? M : 0)) break;
        const int n = b0 + l;
        const double inv_n = 1.0 / (double)(n > 0 ? n : 1);
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        if (b > 0) asm volatile("s_nop 1");  // kc[b - 1] was just written: DPP reads need 2 wait states
#pragma unroll
        for (int bp = 0; bp < b; ++bp) {
          const double* al = la + n - 16 * bp;  // alpha_{n - k} = la[n - k], k = 16 bp + j
          cep_terms16(a0, a1, a2, a3, kc[bp], al);
        }
        double acc = (a0 + a1) + (a2 + a3);
        double mine = 0.0;
        cep_block_step<0>(b0, M, l, gg, inv_n, la, n, acc, mine, p);
        kc[b] = n == 0 ? 0.0 : (double)n * mine;
        if (n < CSN) cs[n] = mine;
        if (n < M && valid && A.cep_out) A.cep_out[(int64_t)item * M + n] = mine;
      }
      wave_lds_sync();
    } else if constexpr (CB < 0) {
      // any M (REVERB: 450): the same register broadcast over a sliding window of the last W finished
      // blocks.  alpha_{n-k} = 0 for n - k > p, and the window covers every k >= b0 - 16 W <= n - p, so
      // the terms it adds beyond the reference's range are exact zeros (la is zero past p).
      constexpr int W = SL;  // block w holds n - k >= 16 w + 1; w >= ceil(p / 16) <= SL is all zero terms
      double kc[W];              // kc[w]: n c_n (lane l) of block b - 1 - w; 0 before block 0
#pragma unroll
      for (int w = 0; w < W; ++w) kc[w] = 0.0;
      // only c_0 .. c_{Me-1} reach the envelope (fft(., env_nfft) truncates, :201); all M are computed
      // when the cepstra themselves are an output (debug / modulation-spectrum mode)
      const int Mc = A.cep_out ? M : A.Me;
      for (int b0 = 0; b0 < ((FDLP_LPC_PHASES & 2) ? Mc : 0); b0 += 16) {
        const int n = b0 + l;
        const double inv_n = 1.0 / (double)(n > 0 ? n : 1);
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        asm volatile("s_nop 1");  // kc[0] was just written: DPP reads need 2 wait states
        // k = b0 - 16 (w + 1) + j: alpha_{n-k} = la[n - b0 + 16 w + 16 - j]; the lane's base address is
        // la + n - b0 + 1, so window block w reads byte offsets 8 (16 w + 15 - j)
        double va[16], vb[16];
        const uint32_t aaddr =
            (uint32_t)(uintptr_t)((__attribute__((address_space(3))) double*)(la + n - b0 + 1));
        lgkm_wait<0>();  // nothing else (scalar loads complete out of order) may share the counted waits
        lds_load16<15>(va, aaddr);
        cep_window<W, 0>(a0, a1, a2, a3, kc, va, vb, aaddr);
        double acc = (a0 + a1) + (a2 + a3);
        double mine = 0.0;
        cep_block_step<0>(b0, Mc, l, gg, inv_n, la, n, acc, mine, p);
#pragma unroll
        for (int w = W - 1; w > 0; --w) kc[w] = kc[w - 1];
        kc[0] = n == 0 ? 0.0 : (double)n * mine;
        if (n < CSN) cs[n] = mine;
        if (n < M && valid && A.cep_out) A.cep_out[(int64_t)item * M + n] = mine;
      }
      wave_lds_sync();
    }
    for (int b0 = 0; b0 < ((CB == 0 && (FDLP_LPC_PHASES & 2)) ? M : 0); b0 += 16) {
      const int n = b0 + l;
      const double inv_n = 1.0 / (double)(n > 0 ? n : 1);
      // finished blocks: four independent FMA chains (the trip count is uniform across the wave)
      const int kstart = max(1, b0 - p);
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      int k = kstart;
      double kd = (double)kstart;
      for (; k + 3 < b0; k += 4, kd += 4.0) {
        a0 = fma(kd * cs[k], la[n - k], a0);
        a1 = fma((kd + 1.0) * cs[k + 1], la[n - k - 1], a1);
        a2 = fma((kd + 2.0) * cs[k + 2], la[n - k - 2], a2);
        a3 = fma((kd + 3.0) * cs[k + 3], la[n - k - 3], a3);
      }
      for (; k < b0; ++k, kd += 1.0) a0 = fma(kd * cs[k], la[n - k], a0);
      double acc = (a0 + a1) + (a2 + a3);
      double mine = 0.0;
      cep_block_step<0>(b0, M, l, gg, inv_n, la, n, acc, mine);
      if (n < M) {
        cs[n] = mine;
        if (valid && A.cep_out) A.cep_out[(int64_t)item * M + n] = mine;
      }
      wave_lds_sync();
    }
    if (grp + (int)gridDim.x < ngroups) dma_a(grp + gridDim.x);  // la is free until the next group
    // ---- phase 3: weights + envelope (computeFDLPSpectrogram.py:194-205) ---------------------
    double* cw = CB != 0 ? cs : la;  // compact layout: weighted in place
    const double* mask = A.weights;
    const double* lif = A.weights + M;
    const double* gam = A.weights + 2 * M;
    for (int n = l; n < A.Me; n += 16) {
      double v = cs[n];
      v = v * mask[n];
      v = v * lif[n];
      v = v * gam[n];
      if (A.odd_zero && (n & 1)) v = 0.0;
      cw[n] = v;
    }
    wave_lds_sync();
    // S(u) = Even(u) + Odd(u), S(H - u) = Even(u) - Odd(u); lane slots cover u = 0..H/2 (lpc_env_kernel)
    for (int q0 = 0; q0 < TS; q0 += kEnvChunk) {
      double se[kEnvChunk], so[kEnvChunk], cprev[kEnvChunk], ccur[kEnvChunk], c2[kEnvChunk];
#pragma unroll
      for (int q = 0; q < kEnvChunk; ++q) {
        const int u = l + 16 * (q0 + q);
        const double c1 = A.env_cos[u % A.env_nfft];
        se[q] = cw[0];
        so[q] = 0.0;
        cprev[q] = 1.0;
        ccur[q] = c1;
        c2[q] = 2.0 * c1;
      }
      int n = 1;
      for (; n + 1 < ((FDLP_LPC_PHASES & 4) ? A.Me : 0); n += 2) {
        const double wo = cw[n], we = cw[n + 1];
#pragma unroll
        for (int q = 0; q < kEnvChunk; ++q) {
          so[q] = fma(wo, ccur[q], so[q]);
          const double c_e = fma(c2[q], ccur[q], -cprev[q]);
          se[q] = fma(we, c_e, se[q]);
          cprev[q] = c_e;
          ccur[q] = fma(c2[q], c_e, -ccur[q]);
        }
      }
      if (n < A.Me) {
        const double wo = cw[n];
#pragma unroll
        for (int q = 0; q < kEnvChunk; ++q) so[q] = fma(wo, ccur[q], so[q]);
      }
      if (valid) {
        double* out = A.env + (int64_t)item * A.kk;
#pragma unroll
        for (int q = 0; q < kEnvChunk; ++q) {
          const int u = l + 16 * (q0 + q);
          if (2 * u > H) continue;
          if (u < A.kk) out[u] = exp(se[q] + so[q]) * A.env_win[2 * u];
          const int t2 = H - u;
          if (t2 != u && t2 < A.kk) out[t2] = exp(se[q] - so[q]) * A.env_win[2 * t2];
        }
      }
    }
  }
}
template <int TS>
__global__ __launch_bounds__(64) void lpc_env_kernel(LpcEnvArgs A) {
  extern __shared__ double sh[];
  const int g = threadIdx.x >> 4;
  const int l = threadIdx.x & 15;
  const int item = blockIdx.x * 4 + g;
  const bool valid = item < A.items;
  const int p = A.p, nlags = A.nlags, M = A.M;
  const int NAL = (M > p + 1 ? M : p + 1) + 16;
  double* la = sh + g * A.region;  // a_0..a_p, zeros up to NAL (alpha = -a in phase 2)
  double* lr = la + NAL;           // r (phase 1), then c (phase 2)
  // ---- phase 1: Levinson-Durbin (features.py:226-228) ---------------------------------------
  for (int q = l; q < nlags; q += 16) lr[q] = valid ? A.r[(int64_t)item * nlags + q] : 1.0;
  for (int q = l; q < NAL; q += 16) la[q] = q == 0 ? 1.0 : 0.0;
  wave_lds_sync();
  const double gg = (FDLP_LPC_PHASES & 1) ? durbin16(la, lr, p, l) : lr[0];
  if (valid && A.a_out) {
    for (int i = l; i <= p; i += 16) A.a_out[(int64_t)item * (p + 1) + i] = la[i];
    if (l == 0) A.gg_out[item] = gg;
  }
  wave_lds_sync();
  // ---- phase 2: cepstrum (features.py:233-246): c_n = -a_n - sum_{k<n} (k/n) c_k a_{n-k} --------
  // blocks of 16 coefficients: the finished blocks enter as a lane-parallel dot product, the block
  // itself as a 16-step recurrence with the new c_k broadcast along the row.
  double* cs = lr;
  for (int b0 = 0; b0 < ((FDLP_LPC_PHASES & 2) ? M : 0); b0 += 16) {
    const int n = b0 + l;
    const double inv_n = 1.0 / (double)(n > 0 ? n : 1);
    double acc = 0.0;
    const int kstart = max(1, b0 - p);
    double kd = (double)kstart;
    for (int k = kstart; k < b0; ++k, kd += 1.0) acc = fma(kd * cs[k], la[n - k], acc);
    double mine = 0.0;
    cep_block_step<0>(b0, M, l, gg, inv_n, la, n, acc, mine);
    if (n < M) {
      cs[n] = mine;
      if (valid && A.cep_out) A.cep_out[(int64_t)item * M + n] = mine;
    }
    wave_lds_sync();
  }
  // ---- phase 3: weights + envelope (computeFDLPSpectrogram.py:194-205) ---------------------
  double* cw = la;
  const double* mask = A.weights;
  const double* lif = A.weights + M;
  const double* gam = A.weights + 2 * M;
  for (int n = l; n < A.Me; n += 16) {
    double v = cs[n];
    v = v * mask[n];
    v = v * lif[n];
    v = v * gam[n];
    if (A.odd_zero && (n & 1)) v = 0.0;
    cw[n] = v;
  }
  wave_lds_sync();
  // S(t) = sum_n cw_n cos(n pi t / H), H = env_nfft / 2.  With u = min(t, H - t):
  //   S(u) = Even(u) + Odd(u),  S(H - u) = Even(u) - Odd(u)   (cos(n (pi - x)) = (-1)^n cos(n x)),
  // so lane slots cover u = 0..H/2 only; cos(n x) by the Chebyshev recurrence.
  const int H = A.env_nfft >> 1;
  double se[TS], so[TS], cprev[TS], ccur[TS], c2[TS];
#pragma unroll
  for (int q = 0; q < TS; ++q) {
    const int u = l + 16 * q;
    const double c1 = A.env_cos[u % A.env_nfft];
    se[q] = cw[0];
    so[q] = 0.0;
    cprev[q] = 1.0;
    ccur[q] = c1;
    c2[q] = 2.0 * c1;
  }
  int n = 1;
  for (; n + 1 < ((FDLP_LPC_PHASES & 4) ? A.Me : 0); n += 2) {
    const double wo = cw[n], we = cw[n + 1];
#pragma unroll
    for (int q = 0; q < TS; ++q) {
      so[q] = fma(wo, ccur[q], so[q]);                  // odd n
      const double c_e = fma(c2[q], ccur[q], -cprev[q]);
      se[q] = fma(we, c_e, se[q]);                      // even n + 1
      cprev[q] = c_e;
      ccur[q] = fma(c2[q], c_e, -ccur[q]);
    }
  }
  if (n < A.Me) {
    const double wo = cw[n];
#pragma unroll
    for (int q = 0; q < TS; ++q) so[q] = fma(wo, ccur[q], so[q]);
  }
  if (valid) {
    double* out = A.env + (int64_t)item * A.kk;
#pragma unroll
    for (int q = 0; q < TS; ++q) {
      const int u = l + 16 * q;
      if (2 * u > H) continue;
      if (u < A.kk) out[u] = exp(se[q] + so[q]) * A.env_win[2 * u];
      const int t2 = H - u;
      if (t2 != u && t2 < A.kk) out[t2] = exp(se[q] - so[q]) * A.env_win[2 * t2];
    }
  }
}

// -----------------------------------------------------------------------------------------
// 7. OLA gather + floor + log (computeFDLPSpectrogram.py:207-229).  Thread per (row, band);
//    contributions are summed in frame order, so 0 + e_a + e_b matches the reference exactly.
// -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ola_log_kernel(DevConsts c, const double* __restrict__ env,
                                                      const FrameDesc* __restrict__ frames,
                                                      const UttDesc* __restrict__ utts, float* __restrict__ out,
                                                      double* __restrict__ out64, int decimals, double scale10) {
  const int u = blockIdx.y;
  const UttDesc U = utts[u];
  const int B = c.B;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)U.L * B) return;
  const int t = (int)(e / B);
  const int j = (int)(e % B);
  // largest k with dst_k <= t (dst is non-decreasing in k)
  int lo = 0, hi = U.F - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (frames[U.frame0 + mid].dst <= t) lo = mid; else hi = mid - 1;
  }
  int kf = lo;
  while (kf > 0 && frames[U.frame0 + kf - 1].dst + c.kk > t) --kf;
  double acc = 0.0;
  for (int k = kf; k <= lo; ++k) {
    const FrameDesc& fd = frames[U.frame0 + k];
    if (t >= fd.dst && t < fd.dst + fd.cnt) {
      const int64_t item = (int64_t)(U.frame0 + k) * B + j;
      acc = acc + env[item * c.kk + fd.src + (t - fd.dst)];
    }
  }
  const double v = log(acc < 1e-14 ? 1e-14 : acc);  // np.clip(a_min=1e-14) keeps NaN; :227
  const int64_t o = (U.out_row + t) * (int64_t)B + j;
  if (out64) out64[o] = v;
  if (out) out[o] = decimals >= 0 ? (float)(nearbyint(v * scale10) / scale10) : (float)v;
}

// Tiled OLA: one workgroup per (utterance, kOlaRows output rows).  The frames overlapping the tile are
// added in frame order into an LDS tile [row][band] (0 + e_a + e_b, as above), reading each frame's
// envelope rows [band][t] with consecutive threads on consecutive t (coalesced; the per-thread gather
// above reads B bands kk doubles apart), then log + floor and row-major stores.
constexpr int kOlaRows = 32;
__global__ __launch_bounds__(256) void ola_log_tiled_kernel(DevConsts c, const double* __restrict__ env,
                                                            const FrameDesc* __restrict__ frames,
                                                            const UttDesc* __restrict__ utts, float* __restrict__ out,
                                                            double* __restrict__ out64, int decimals, double scale10) {
  extern __shared__ double tile[];  // [kOlaRows][B + 1]
  const int u = blockIdx.y;
  const UttDesc U = utts[u];
  const int t0 = blockIdx.x * kOlaRows;
  if (t0 >= U.L) return;
  const int nt = min(kOlaRows, U.L - t0);
  const int B = c.B, BS = c.B + 1, kk = c.kk;
  const int tid = threadIdx.x;
  for (int q = tid; q < kOlaRows * BS; q += blockDim.x) tile[q] = 0.0;
  // frames overlapping [t0, t0 + nt): dst is non-decreasing in k; the last one with dst < t0 + nt,
  // then down while a frame still reaches t0
  int lo = 0, hi = U.F - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (frames[U.frame0 + mid].dst < t0 + nt) lo = mid; else hi = mid - 1;
  }
  int kf = lo;
  while (kf > 0 && frames[U.frame0 + kf - 1].dst + kk > t0) --kf;
  __syncthreads();
  const int tt = tid % kOlaRows, jj = tid / kOlaRows;  // 8 band lanes x 32 rows
  for (int k = kf; k <= lo; ++k) {
    const FrameDesc fd = frames[U.frame0 + k];
    const int t = t0 + tt;
    if (t < t0 + nt && t >= fd.dst && t < fd.dst + fd.cnt) {
      const double* er = env + (int64_t)(U.frame0 + k) * B * kk + fd.src + (t - fd.dst);
      for (int j = jj; j < B; j += blockDim.x / kOlaRows) tile[tt * BS + j] = tile[tt * BS + j] + er[(int64_t)j * kk];
    }
    __syncthreads();
  }
  for (int q = tid; q < nt * B; q += blockDim.x) {
    const int t = q / B, j = q - t * B;
    const double acc = tile[t * BS + j];
    const double v = log(acc < 1e-14 ? 1e-14 : acc);  // np.clip(a_min=1e-14) keeps NaN; :227
    const int64_t o = (U.out_row + t0 + t) * (int64_t)B + j;
    if (out64) out64[o] = v;
    if (out) out[o] = decimals >= 0 ? (float)(nearbyint(v * scale10) / scale10) : (float)v;
  }
}

// -----------------------------------------------------------------------------------------
// launch wrappers
// -----------------------------------------------------------------------------------------
hipError_t launch_frames_dft1(const DevConsts& c, const DftPlan& d1, int N2, const void* pcm,
                              int pcm_kind, const int16_t* noise, const FrameDesc* frames,
                              const double* dense_rows, int nframes, double2* z, const double2* om1,
                              hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  dim3 grid((N2 + kDftCols - 1) / kDftCols, nframes);
  size_t lds = sizeof(double2) * (2 * d1.n * kDftCols + d1.n);
  if (c.real_fft && !c.dct_generic && d1.n == 100 && N2 == 120 && !dense_rows) {  // recipes: N = 24000
    hipLaunchKernelGGL((frames_dft1_c_kernel<100, 120, kDftCols>), dim3(xcd_grid(grid.x * nframes)), dim3(256), 0, s, c,
                       pcm, pcm_kind, noise, frames, om1, z, nframes);
    return hipGetLastError();
  }
  if (c.real_fft) {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)frames_dft1_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(frames_dft1_kernel<true>, grid, dim3(256), lds, s, c, d1, N2, pcm, pcm_kind, noise,
                       frames, dense_rows, om1, z);
  } else {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)frames_dft1_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(frames_dft1_kernel<false>, grid, dim3(256), lds, s, c, d1, N2, pcm, pcm_kind, noise,
                       frames, dense_rows, om1, z);
  }
  return hipGetLastError();
}

hipError_t launch_dft2_dct(const DevConsts& c, const DftPlan& d2, int N1, const double2* z,
                           int nframes, double* dct, const double2* om2, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  size_t lds = sizeof(double2) * (2 * d2.n * kDftCols + d2.n);
  const double div = sqrt((double)(2 * c.N));
  if (c.real_fft && !c.dct_generic && N1 == 100 && d2.n == 120) {  // recipes: N = 24000
    dim3 grid((N1 / 2 + 1 + kDftCols / 2 - 1) / (kDftCols / 2), nframes);
    static const bool table_tw = getenv("FDLP_DCT_TABLE_TW") != nullptr;  // A/B knob: full post/rtw tables
    const dim3 g1(xcd_grid(grid.x * nframes));
    const double sc2 = 2.0 / div;
    static const bool no_swz = getenv("FDLP_DCT_NOSWZ") != nullptr;  // A/B knob: unswizzled LDS columns
    if (table_tw)
      hipLaunchKernelGGL((dft2_dct_c_kernel<100, 120, kDftCols, false>), g1, dim3(256), 0, s, c, z, om2, sc2, dct, nframes);
    else if (no_swz)
      hipLaunchKernelGGL((dft2_dct_c_kernel<100, 120, kDftCols, true, false>), g1, dim3(256), 0, s, c, z, om2, sc2, dct,
                         nframes);
    else
      hipLaunchKernelGGL((dft2_dct_c_kernel<100, 120, kDftCols, true>), g1, dim3(256), 0, s, c, z, om2, sc2, dct, nframes);
    return hipGetLastError();
  }
  if (c.real_fft) {
    dim3 grid((N1 / 2 + 1 + kDftCols / 2 - 1) / (kDftCols / 2), nframes);  // row pairs (k1, N1-k1)
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)dft2_dct_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(dft2_dct_kernel<true>, grid, dim3(256), lds, s, c, d2, N1, z, om2, div, dct);
  } else {
    dim3 grid((N1 + kDftCols - 1) / kDftCols, nframes);
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)dft2_dct_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(dft2_dct_kernel<false>, grid, dim3(256), lds, s, c, d2, N1, z, om2, div, dct);
  }
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_ac_nt(const DevConsts& c, const double* dct, const double* dense, int items,
                               double* r, const LpcTail* tail, double* env, hipStream_t s) {
  if (tail) {
    hipLaunchKernelGGL((autocorr_kernel<NT, true>), dim3(items), dim3(64), 0, s, c, dct, dense, r, *tail, env);
  } else {
    LpcTail none{};
    hipLaunchKernelGGL((autocorr_kernel<NT, false>), dim3(items), dim3(64), 0, s, c, dct, dense, r, none, env);
  }
  return hipGetLastError();
}

int autocorr_tiles(int nlags) { return ((nlags + 14) >> 4) + 1; }

int band_fused_fits(int nlags, int p, int M, int kk) {
  const int NAL = (M > p + 1 ? M : p + 1) + 64;
  const int need = NAL + (nlags > M ? nlags : M);
  return need <= (16 * 4 + 15) * 17 && kk <= 64 * kTS64;
}

static hipError_t launch_autocorr_any(const DevConsts& c, const double* dct, const double* dense, int items,
                                      double* r, const LpcTail* tail, double* env, hipStream_t s) {
  if (items <= 0) return hipSuccess;
  switch (autocorr_tiles(c.nlags)) {
#define FDLP_AC_CASE(n) case n: return launch_ac_nt<n>(c, dct, dense, items, r, tail, env, s);
    FDLP_AC_CASE(1) FDLP_AC_CASE(2) FDLP_AC_CASE(3) FDLP_AC_CASE(4) FDLP_AC_CASE(5)
    FDLP_AC_CASE(6) FDLP_AC_CASE(7) FDLP_AC_CASE(8) FDLP_AC_CASE(9) FDLP_AC_CASE(10)
    FDLP_AC_CASE(11) FDLP_AC_CASE(12) FDLP_AC_CASE(13) FDLP_AC_CASE(14) FDLP_AC_CASE(15)
    FDLP_AC_CASE(16)
#undef FDLP_AC_CASE
    default: return hipErrorInvalidValue;
  }
}

template <int LG>
static hipError_t launch_acv_lg(const DevConsts& c, const double* dct, const double* dense, int items, double* r,
                                hipStream_t s) {
  hipLaunchKernelGGL(autocorr_valu_kernel<LG>, dim3(items), dim3(64), 0, s, c, dct, dense, r);
  return hipGetLastError();
}

int autocorr_valu_lags_per_group(int nlags) { return (nlags + 7) / 8; }

hipError_t launch_autocorr_valu(const DevConsts& c, const double* dct, const double* dense, int items, double* r,
                                hipStream_t s) {
  if (items <= 0) return hipSuccess;
  switch (autocorr_valu_lags_per_group(c.nlags)) {
#define FDLP_ACV_CASE(n) case n: return launch_acv_lg<n>(c, dct, dense, items, r, s);
    FDLP_ACV_CASE(1) FDLP_ACV_CASE(2) FDLP_ACV_CASE(3) FDLP_ACV_CASE(4) FDLP_ACV_CASE(5) FDLP_ACV_CASE(6)
    FDLP_ACV_CASE(7) FDLP_ACV_CASE(8) FDLP_ACV_CASE(9) FDLP_ACV_CASE(10) FDLP_ACV_CASE(11) FDLP_ACV_CASE(12)
    FDLP_ACV_CASE(13) FDLP_ACV_CASE(14) FDLP_ACV_CASE(15) FDLP_ACV_CASE(16) FDLP_ACV_CASE(17) FDLP_ACV_CASE(18)
    FDLP_ACV_CASE(19) FDLP_ACV_CASE(20) FDLP_ACV_CASE(21) FDLP_ACV_CASE(22) FDLP_ACV_CASE(23) FDLP_ACV_CASE(24)
    FDLP_ACV_CASE(25) FDLP_ACV_CASE(26) FDLP_ACV_CASE(27) FDLP_ACV_CASE(28) FDLP_ACV_CASE(29) FDLP_ACV_CASE(30)
#undef FDLP_ACV_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_autocorr(const DevConsts& c, const double* dct, const double* dense, int items,
                           double* r, hipStream_t s) {
  // MFMA is the default: measured 25.1 ms vs 27.1 ms (VALU) per 4096-frame batch on MI355X, the
  // VALU variant clocks down to ~1.95 GHz under full fp64 FMA load.  FDLP_AUTOCORR_VALU=1 selects it.
  static const bool use_valu = getenv("FDLP_AUTOCORR_VALU") != nullptr;
  if (use_valu && autocorr_valu_lags_per_group(c.nlags) <= 30)
    return launch_autocorr_valu(c, dct, dense, items, r, s);
  return launch_autocorr_any(c, dct, dense, items, r, nullptr, nullptr, s);
}

int vsweep_lanes_lags(int nlags) {
  // up to 160 lags (p <= 158): with more lags per lane the chains and the window no longer fit the
  // registers of two waves per SIMD (spills), and such plans keep the MFMA sweeps
  const int a = (nlags + 15) / 16;
  for (int v : {4, 8, 10})
    if (a <= v) return v;
  return 0;
}
int vsweep_chains(int C) {
  for (int v : {4, 5, 6, 8})
    if (C <= v) return v;
  return 0;
}

template <int A, int C>
static hipError_t launch_vsweep_ac(const DevConsts& c, const double* dct, int nframes, double* r, double* rup,
                                   double* rflat, double* rpart, hipStream_t s) {
  const int ngroups = (nframes + 3) / 4;
  hipLaunchKernelGGL((ac_vsweep_kernel<A, 0>), dim3(xcd_grid(2 * ngroups)), dim3(64), 0, s, c, dct, r, rup, rflat,
                     rpart, c.sk_snap, c.fl_ev, nframes, ngroups);
  hipLaunchKernelGGL((ac_vsweep_kernel<A, C>), dim3(xcd_grid(c.fl_H * ngroups)), dim3(64), 0, s, c, dct, r, rup,
                     rflat, rpart, c.sk_snap, c.fl_ev, nframes, ngroups);
  return hipGetLastError();
}
template <int A>
static hipError_t launch_vsweep_a(const DevConsts& c, const double* dct, int nframes, double* r, double* rup,
                                  double* rflat, double* rpart, hipStream_t s) {
  switch (vsweep_chains(c.fl_C)) {
    case 4: return launch_vsweep_ac<A, 4>(c, dct, nframes, r, rup, rflat, rpart, s);
    case 5: return launch_vsweep_ac<A, 5>(c, dct, nframes, r, rup, rflat, rpart, s);
    case 6: return launch_vsweep_ac<A, 6>(c, dct, nframes, r, rup, rflat, rpart, s);
    case 8: return launch_vsweep_ac<A, 8>(c, dct, nframes, r, rup, rflat, rpart, s);
    default: return hipErrorInvalidValue;
  }
}
static hipError_t launch_vsweep(const DevConsts& c, const double* dct, int nframes, double* r, double* rup,
                                double* rflat, double* rpart, hipStream_t s) {
  switch (vsweep_lanes_lags(c.nlags)) {
    case 4: return launch_vsweep_a<4>(c, dct, nframes, r, rup, rflat, rpart, s);
    case 8: return launch_vsweep_a<8>(c, dct, nframes, r, rup, rflat, rpart, s);
    case 10: return launch_vsweep_a<10>(c, dct, nframes, r, rup, rflat, rpart, s);
    default: return hipErrorInvalidValue;
  }
}

template <int NT>
static hipError_t launch_struct_nt(const DevConsts& c, const double* dct, int nframes, double* r, double* rup,
                                   double* rflat, double* rpart, hipStream_t s) {
  if (rflat) {  // lag-parallel VALU sweeps (flat tops included) + straddles
    const hipError_t e = launch_vsweep(c, dct, nframes, r, rup, rflat, rpart, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((ac_band_kernel<NT, true>), dim3(xcd_grid(nframes * c.B)), dim3(64), 0, s, c, dct, r, rup,
                       rflat, rpart, nframes * c.B);
    return hipGetLastError();
  }
  static const bool full = getenv("FDLP_SWEEP_FULL_EPI") != nullptr;
  static const bool nosnap = getenv("FDLP_SWEEP_NOSNAP") != nullptr;  // timing experiment only
  const size_t tab = sizeof(SkSnap) * (size_t)c.B;
  if (nosnap && full)
    hipLaunchKernelGGL((ac_sweep_kernel<NT, 64, false>), dim3(xcd_grid(2 * nframes)), dim3(64), tab, s, c, dct, r, rup, 2 * nframes);
  else if (nosnap)
    hipLaunchKernelGGL((ac_sweep_kernel<NT, 32, false>), dim3(xcd_grid(2 * nframes)), dim3(64), tab, s, c, dct, r, rup, 2 * nframes);
  else if (full)
    hipLaunchKernelGGL((ac_sweep_kernel<NT, 64>), dim3(xcd_grid(2 * nframes)), dim3(64), tab, s, c, dct, r, rup, 2 * nframes);
  else
    hipLaunchKernelGGL((ac_sweep_kernel<NT, 32>), dim3(xcd_grid(2 * nframes)), dim3(64), tab, s, c, dct, r, rup, 2 * nframes);
  hipLaunchKernelGGL((ac_band_kernel<NT, false>), dim3(xcd_grid(nframes * c.B)), dim3(64), 0, s, c, dct, r, rup,
                     nullptr, nullptr, nframes * c.B);
  return hipGetLastError();
}

hipError_t launch_autocorr_structured(const DevConsts& c, const double* dct, int nframes, double* r,
                                      double* rup, double* rflat, double* rpart, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  if (!c.sk_e || !c.sk_snap || !c.sk_reg) return hipErrorInvalidValue;
  if (rflat && (!c.fl_ev || !c.fl_band || (c.fl_H > 1 && !rpart))) return hipErrorInvalidValue;
  switch (autocorr_tiles(c.nlags)) {
#define FDLP_ST_CASE(n) case n: return launch_struct_nt<n>(c, dct, nframes, r, rup, rflat, rpart, s);
    FDLP_ST_CASE(1) FDLP_ST_CASE(2) FDLP_ST_CASE(3) FDLP_ST_CASE(4) FDLP_ST_CASE(5)
    FDLP_ST_CASE(6) FDLP_ST_CASE(7) FDLP_ST_CASE(8) FDLP_ST_CASE(9) FDLP_ST_CASE(10)
    FDLP_ST_CASE(11) FDLP_ST_CASE(12) FDLP_ST_CASE(13) FDLP_ST_CASE(14) FDLP_ST_CASE(15)
    FDLP_ST_CASE(16)
#undef FDLP_ST_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_band_fused(const DevConsts& c, int odd_zero, const double* dct, int items, double* r_dbg,
                             double* env, hipStream_t s) {
  LpcTail T;
  T.p = c.p; T.nlags = c.nlags; T.M = c.M; T.Me = c.Me; T.kk = c.kk; T.odd_zero = odd_zero;
  T.weights = c.weights; T.env_cos = c.env_cos; T.env_nfft = c.env_nfft; T.env_win = c.env_win;
  return launch_autocorr_any(c, dct, nullptr, items, r_dbg, &T, env, s);
}

template <int SL>
static hipError_t launch_lev_sl(int p, int nlags, const double* r, int items, double* a, double* gg,
                                hipStream_t s) {
  hipLaunchKernelGGL(levinson_kernel<SL>, dim3((items + 3) / 4), dim3(64), 0, s, p, nlags, items, r, a, gg);
  return hipGetLastError();
}

hipError_t launch_levinson(const DevConsts& c, const double* r, int items, double* a, double* gg,
                           hipStream_t s) {
  if (items <= 0) return hipSuccess;
  switch ((c.p + 1 + 15) / 16) {
#define FDLP_LEV_CASE(n) case n: return launch_lev_sl<n>(c.p, c.nlags, r, items, a, gg, s);
    FDLP_LEV_CASE(1) FDLP_LEV_CASE(2) FDLP_LEV_CASE(3) FDLP_LEV_CASE(4) FDLP_LEV_CASE(5)
    FDLP_LEV_CASE(6) FDLP_LEV_CASE(7) FDLP_LEV_CASE(8) FDLP_LEV_CASE(9) FDLP_LEV_CASE(10)
    FDLP_LEV_CASE(11) FDLP_LEV_CASE(12) FDLP_LEV_CASE(13) FDLP_LEV_CASE(14) FDLP_LEV_CASE(15)
#undef FDLP_LEV_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_cepstrum(int p, int M, const double* a, const double* gg, int items, double* cep,
                           hipStream_t s) {
  if (items <= 0) return hipSuccess;
  if (M > kCepMaxM || p > kCepMaxP) return hipErrorInvalidValue;
  size_t lds = sizeof(double) * ((size_t)(M > p + 1 ? M : p + 1) + 64 + M);
  hipLaunchKernelGGL(cepstrum_kernel, dim3(items), dim3(64), lds, s, p, M, a, gg, cep);
  return hipGetLastError();
}

template <int TS>
static hipError_t launch_lpc_env_t(const LpcEnvArgs& A, size_t lds, hipStream_t s) {
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)lpc_env_kernel<TS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((lpc_env_kernel<TS>), dim3((A.items + 3) / 4), dim3(64), lds, s, A);
  return hipGetLastError();
}

int lpc_env_region(int p, int M) {
  const int NAL = (M > p + 1 ? M : p + 1) + 16;
  const int need = NAL + (p + 2 > M ? p + 2 : M);
  return (need + 15) / 32 * 32 + 16;  // = 16 mod 32 doubles: the 4 items of a wave hit disjoint bank halves
}

// Lattice-kernel instantiation of a plan: calls fn(integral_constant<SL>, integral_constant<CB>) or
// returns hipErrorNotSupported when the plan runs the LDS Durbin (lpc_env_kernel).
template <class Fn>
static hipError_t lattice_dispatch_sl(const DevConsts& c, Fn&& fn) {
  using std::integral_constant;
  const int SL = (c.p + 1 + 15) / 16;
  if (SL > 16 || c.lpc_lds_durbin) return hipErrorNotSupported;
  if (!c.lpc_cep_lds && c.M <= 16 * 7 && SL >= 9 && SL <= 11) {  // register-broadcast cepstrum (recipes: p 150, M 100)
    switch (SL) {
      case 9: return fn(integral_constant<int, 9>{}, integral_constant<int, 7>{});
      case 10: return fn(integral_constant<int, 10>{}, integral_constant<int, 7>{});
      case 11: return fn(integral_constant<int, 11>{}, integral_constant<int, 7>{});
      default: break;
    }
  }
  if (!c.lpc_cep_lds && c.M > 16 * 7 && SL >= 9 && SL <= 11) {  // the same over a sliding window (REVERB: M 450)
    switch (SL) {
      case 9: return fn(integral_constant<int, 9>{}, integral_constant<int, -1>{});
      case 10: return fn(integral_constant<int, 10>{}, integral_constant<int, -1>{});
      case 11: return fn(integral_constant<int, 11>{}, integral_constant<int, -1>{});
      default: break;
    }
  }
  switch (SL) {
#define FDLP_SL_CASE(n) case n: return fn(integral_constant<int, n>{}, integral_constant<int, 0>{});
    FDLP_SL_CASE(1) FDLP_SL_CASE(2) FDLP_SL_CASE(3) FDLP_SL_CASE(4) FDLP_SL_CASE(5) FDLP_SL_CASE(6)
    FDLP_SL_CASE(7) FDLP_SL_CASE(8) FDLP_SL_CASE(9) FDLP_SL_CASE(10) FDLP_SL_CASE(11) FDLP_SL_CASE(12)
    FDLP_SL_CASE(13) FDLP_SL_CASE(14) FDLP_SL_CASE(15) FDLP_SL_CASE(16)
#undef FDLP_SL_CASE
    default: return hipErrorNotSupported;
  }
}

// durbin8_kernel instantiations: 8 SL8 >= p + 1 for the lattice range SL = 9..11 (p 128..175)
static bool durbin8_fits(int p) {
  const int sl8 = (p + 1 + 7) / 8;
  return sl8 >= 17 && sl8 <= 22;
}
template <class Fn>
static hipError_t durbin8_dispatch(int p, Fn&& fn) {
  using std::integral_constant;
  switch ((p + 1 + 7) / 8) {
    case 17: return fn(integral_constant<int, 17>{});
    case 18: return fn(integral_constant<int, 18>{});
    case 19: return fn(integral_constant<int, 19>{});
    case 20: return fn(integral_constant<int, 20>{});
    case 21: return fn(integral_constant<int, 21>{});
    case 22: return fn(integral_constant<int, 22>{});
    default: return hipErrorNotSupported;
  }
}

// fn(integral_constant<SL>, integral_constant<CB>, integral_constant<int, DM>)
template <class Fn>
static hipError_t lattice_dispatch(const DevConsts& c, Fn&& fn) {
  using std::integral_constant;
  return lattice_dispatch_sl(c, [&](auto sl, auto cb) -> hipError_t {
    if (c.lpc_slotmajor) return fn(sl, cb, integral_constant<int, kDmSlotMajor>{});
    if (c.lpc_split) return fn(sl, cb, integral_constant<int, kDmExt>{});
    return fn(sl, cb, integral_constant<int, kDmContig>{});
  });
}

// a-area length of the compact layout (register cepstra, CB != 0): the Durbin writes 16 SL positions,
// CB > 0 reads a below 16 CB, the window (CB < 0, W = SL blocks) below 16 SL + 16
static int lattice_la_len(const DevConsts& c, int CB, int SL) {
  int la = std::max(c.p + 2, 16 * SL);
  if (CB > 0) la = std::max(la, 16 * CB);
  if (CB < 0) la = std::max(la, 16 * SL + 16);
  return (la + 15) / 16 * 16;  // whole 128-B rows (the split Durbin's a rows are LDS-DMA copies)
}
static int lattice_region(const DevConsts& c, int CB, int SL) {
  const int need = CB != 0 ? lattice_la_len(c, CB, SL) + c.Me : (c.M > c.p + 1 ? c.M : c.p + 1) + 16 + c.M;
  return (need + 15) / 32 * 32 + 16;  // = 16 mod 32 doubles (disjoint bank halves per item)
}
static size_t lattice_lds(const DevConsts& c, int CB, int SL) {
  return sizeof(double) * 4 * (size_t)lattice_region(c, CB, SL);
}

hipError_t prepare_lpc_env(DevConsts& c) {
  c.lpc_lds_durbin = getenv("FDLP_LPC_LDS") != nullptr;
  c.lpc_cep_lds = getenv("FDLP_CEP_LDS") != nullptr;
  c.lpc_slotmajor = getenv("FDLP_LPC_SLOTMAJOR") != nullptr;
  // the Durbin as its own kernel (durbin8_kernel) unless FDLP_LPC_FUSED=1 or the slot-major A/B form
  c.lpc_split = !c.lpc_slotmajor && getenv("FDLP_LPC_FUSED") == nullptr && durbin8_fits(c.p);
  c.lpc_astride = 0;
  c.lpc_blocks = 0;
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  int per_cu = 0;
  e = lattice_dispatch(c, [&](auto sl, auto cb, auto ct) -> hipError_t {
    constexpr int SL = decltype(sl)::value, CB = decltype(cb)::value;
    constexpr int CT = decltype(ct)::value;
    const size_t lds = lattice_lds(c, CB, SL);
    if (CT == kDmExt) c.lpc_astride = CB != 0 ? lattice_la_len(c, CB, SL) : (c.p + 1 + 15) / 16 * 16;
    if (lds > 65536) {
      const hipError_t a = hipFuncSetAttribute((const void*)lpc_env_lattice_kernel<SL, CB, CT>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (a != hipSuccess) return a;
    }
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lpc_env_lattice_kernel<SL, CB, CT>, 64, lds);
  });
  if (e == hipErrorNotSupported) return hipSuccess;  // LDS Durbin: one block per item group, no setup
  if (e != hipSuccess) return e;
  c.lpc_blocks = std::max(1, per_cu) * std::max(1, cus);
  return hipSuccess;
}

hipError_t launch_lpc_env(const DevConsts& c, int odd_zero, const double* r, int items, double* env,
                          double* a_out, double* gg_out, double* cep_out, double* a_ws, double* gg_ws,
                          hipStream_t s) {
  if (items <= 0) return hipSuccess;
  LpcEnvArgs A;
  A.a_ext = nullptr;
  A.gg_ext = nullptr;
  A.a_stride = 0;
  if (c.lpc_blocks > 0 && c.lpc_split) {  // the Durbin first, into a_ws / gg_ws
    if (!a_ws || !gg_ws) return hipErrorInvalidValue;
    double* gd = gg_out ? gg_out : gg_ws;
    const hipError_t e = durbin8_dispatch(c.p, [&](auto sl8) -> hipError_t {
      constexpr int SL8 = decltype(sl8)::value;
      hipLaunchKernelGGL((durbin8_kernel<SL8>), dim3((items + 7) / 8), dim3(64), 0, s, r, c.nlags, c.p, items, a_ws, gd,
                         c.lpc_astride);
      return hipGetLastError();
    });
    if (e != hipSuccess) return e;
    if (a_out) {  // debug: the [items, p+1] layout
      const hipError_t e2 = hipMemcpy2DAsync(a_out, sizeof(double) * (c.p + 1), a_ws, sizeof(double) * c.lpc_astride,
                                             sizeof(double) * (c.p + 1), items, hipMemcpyDeviceToDevice, s);
      if (e2 != hipSuccess) return e2;
    }
    A.a_ext = a_ws;
    A.gg_ext = gd;
    A.a_stride = c.lpc_astride;
    a_out = nullptr;  // already written
    gg_out = nullptr;
  }
  A.p = c.p; A.nlags = c.nlags; A.M = c.M; A.Me = c.Me; A.kk = c.kk; A.env_nfft = c.env_nfft;
  A.odd_zero = odd_zero; A.items = items; A.region = lpc_env_region(c.p, c.M); A.la_len = 0;
  A.r = r; A.weights = c.weights; A.env_cos = c.env_cos; A.env_win = c.env_win; A.env = env;
  A.a_out = a_out; A.gg_out = gg_out; A.cep_out = cep_out;
  if (c.lpc_blocks > 0) {  // lattice Durbin in registers, persistent grid (prepare_lpc_env)
    const int grid = std::min((items + 3) / 4, c.lpc_blocks);
    return lattice_dispatch(c, [&](auto sl, auto cb, auto ct) -> hipError_t {
      constexpr int SL = decltype(sl)::value, CB = decltype(cb)::value;
      constexpr int CT = decltype(ct)::value;
      const size_t lds = lattice_lds(c, CB, SL);
      A.region = lattice_region(c, CB, SL);
      A.la_len = CB != 0 ? lattice_la_len(c, CB, SL) : 0;
      hipLaunchKernelGGL((lpc_env_lattice_kernel<SL, CB, CT>), dim3(grid), dim3(64), lds, s, A);
      return hipGetLastError();
    });
  }
  const size_t lds = sizeof(double) * (4 * (size_t)A.region);
  switch ((c.env_nfft / 4 + 1 + 15) / 16) {  // envelope slots: u = 0 .. env_nfft/4
#define FDLP_TS_CASE(n) case n: return launch_lpc_env_t<n>(A, lds, s);
    FDLP_TS_CASE(1) FDLP_TS_CASE(2) FDLP_TS_CASE(3) FDLP_TS_CASE(4) FDLP_TS_CASE(5) FDLP_TS_CASE(6)
    FDLP_TS_CASE(7) FDLP_TS_CASE(8) FDLP_TS_CASE(9) FDLP_TS_CASE(10) FDLP_TS_CASE(11) FDLP_TS_CASE(12)
    FDLP_TS_CASE(13) FDLP_TS_CASE(14) FDLP_TS_CASE(15) FDLP_TS_CASE(16)
#undef FDLP_TS_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_ola_log(const DevConsts& c, const double* env, const FrameDesc* frames, const UttDesc* utts,
                          int n_utt, int maxL, float* out, double* out_f64, int decimals, hipStream_t s) {
  if (n_utt <= 0 || maxL <= 0) return hipSuccess;
  double scale10 = 1.0;
  for (int i = 0; i < decimals; ++i) scale10 *= 10.0;
  static const bool gather = getenv("FDLP_OLA_GATHER") != nullptr;
  if (gather) {
    const int64_t per = (int64_t)maxL * c.B;
    dim3 grid((unsigned)((per + 255) / 256), n_utt);
    hipLaunchKernelGGL(ola_log_kernel, grid, dim3(256), 0, s, c, env, frames, utts, out, out_f64, decimals,
                       scale10);
  } else {
    dim3 grid((unsigned)((maxL + kOlaRows - 1) / kOlaRows), n_utt);
    const size_t lds = sizeof(double) * kOlaRows * (size_t)(c.B + 1);
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)ola_log_tiled_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(ola_log_tiled_kernel, grid, dim3(256), lds, s, c, env, frames, utts, out, out_f64, decimals,
                       scale10);
  }
  return hipGetLastError();
}

// -----------------------------------------------------------------------------------------
// 8. Global CMVN statistics: Kaldi compute-cmvn-stats (no --spk2utt) -> AccCmvnStats
//    (transform/cmvn.cc), the step after feature extraction in e2e/wsj/run_fdlp_e1.sh:280:
//      stats[0][d] += x_d,  stats[1][d] += x_d * x_d  (a BaseFloat product: float32, then double),
//      stats[0][D] += 1 per frame.
//    Deterministic: chunk partial sums in row order, then a fixed-order sum over chunks, so the
//    result does not depend on scheduling.  HBM-bound (4 bytes per feature read once).
// -----------------------------------------------------------------------------------------
constexpr int kCmvnRows = 256;  // rows per chunk

__global__ __launch_bounds__(128) void cmvn_partial_kernel(const float* __restrict__ x, int64_t rows, int D,
                                                           double* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * kCmvnRows;
  const int64_t r1 = min(rows, r0 + (int64_t)kCmvnRows);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    double s0 = 0.0, q0 = 0.0;
    const float* col = x + r0 * D + d;
    for (int64_t r = r0; r < r1; ++r, col += D) {
      const float v = *col;
      const float v2 = v * v;  // BaseFloat product, as Kaldi forms it
      s0 += (double)v;
      q0 += (double)v2;
    }
    part[((int64_t)blockIdx.x * 2) * D + d] = s0;
    part[((int64_t)blockIdx.x * 2 + 1) * D + d] = q0;
  }
}

__global__ __launch_bounds__(128) void cmvn_finish_kernel(const double* __restrict__ part, int nchunks, int D,
                                                          int64_t rows, double* __restrict__ stats) {
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    double s = 0.0, q = 0.0;
    for (int c = 0; c < nchunks; ++c) {
      s += part[((int64_t)c * 2) * D + d];
      q += part[((int64_t)c * 2 + 1) * D + d];
    }
    stats[d] += s;
    stats[(D + 1) + d] += q;
  }
  if (threadIdx.x == 0) stats[D] += (double)rows;
}

int cmvn_chunks(int64_t rows) { return (int)((rows + kCmvnRows - 1) / kCmvnRows); }

hipError_t launch_cmvn(const float* x, int64_t rows, int D, double* part, double* stats, hipStream_t s) {
  const int nch = cmvn_chunks(rows);
  if (nch > 0) {
    hipLaunchKernelGGL(cmvn_partial_kernel, dim3(nch), dim3(128), 0, s, x, rows, D, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(cmvn_finish_kernel, dim3(1), dim3(128), 0, s, part, nch, D, rows, stats);
  return hipGetLastError();
}

// -----------------------------------------------------------------------------------------
// 9. addReverb (features.py:110-115) after the optional diff / noise preprocessing
//    (computeFDLPSpectrogram.py:160-170), per utterance u of T samples and an RIR of R taps:
//      x = s | convolve(s, diff13, 'same') | s + alpha * noise[off:off+T]        (rev_pre_kernel)
//      y = convolve(x, rir), length T+R-1                                       (rev_conv_kernel)
//      xs[sh] = sum_n x[n] y[n+sh], sh < R  (np.correlate(x, y, 'valid') reversed) (rev_xcorr_kernel)
//      sh* = the LARGEST shift attaining max xs (numpy's first argmax over the reversed order),
//      out = y[sh*+1 : sh*+1+T] (shorter than T only when sh* = R-1)           (rev_select_kernel)
//    fp64 direct sums (numpy's convolve/correlate are direct too).  VALU, 4 outputs per thread.
// -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rev_pre_kernel(const RevUtt* __restrict__ U, const void* __restrict__ pcm,
                                                      int kind, int pre, const int16_t* __restrict__ noise,
                                                      double* __restrict__ x) {
  const RevUtt u = U[blockIdx.y];
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= u.T) return;
  double v;
  if (kind == 1) {
    v = ((const double*)pcm)[u.off + t];
  } else if (pre == 1) {  // scipy.signal.convolve(int16 s, diff kernel, 'same') -> int64, exact
    const int16_t* s = (const int16_t*)pcm + u.off;
    long long acc = 0;
#pragma unroll
    for (int q = 0; q < 13; ++q) {
      const int64_t idx = t + 6 - q;
      if (idx >= 0 && idx < u.T) acc += (long long)kDiffTaps[q] * (long long)s[idx];
    }
    v = (double)acc;
  } else {
    v = (double)((const int16_t*)pcm)[u.off + t];
    if (u.noff >= 0) v = __dadd_rn(v, __dmul_rn(u.alpha, (double)noise[u.noff + t]));  // features.py:31
  }
  x[u.off + t] = v;
}

constexpr int kRevTile = 256;

__global__ __launch_bounds__(256) void rev_conv_kernel(const RevUtt* __restrict__ U, const double* __restrict__ x,
                                                       const double* __restrict__ rir, int R, double* __restrict__ y) {
  __shared__ double rs[kRevTile];
  __shared__ double xw[4 * 256 + kRevTile];
  const RevUtt u = U[blockIdx.y];
  const int64_t ny = u.T + R - 1;
  const int64_t n0 = (int64_t)blockIdx.x * 1024;
  if (n0 >= ny) return;
  const int t4 = 4 * threadIdx.x;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  for (int k0 = 0; k0 < R; k0 += kRevTile) {
    __syncthreads();
    rs[threadIdx.x] = k0 + (int)threadIdx.x < R ? rir[k0 + threadIdx.x] : 0.0;
    // xw[i] = x[n0 - k0 - (kRevTile-1) + i]
    for (int i = threadIdx.x; i < 4 * 256 + kRevTile; i += 256) {
      const int64_t q = n0 - k0 - (kRevTile - 1) + i;
      xw[i] = (q >= 0 && q < u.T) ? x[u.off + q] : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < kRevTile; ++kk) {
      const double r = rs[kk];
      const int b = t4 + (kRevTile - 1) - kk;  // x[n - k] for n = n0 + t4, k = k0 + kk
      a0 = fma(r, xw[b], a0);
      a1 = fma(r, xw[b + 1], a1);
      a2 = fma(r, xw[b + 2], a2);
      a3 = fma(r, xw[b + 3], a3);
    }
  }
  double* yo = y + u.yoff;
  const int64_t n = n0 + t4;
  if (n < ny) yo[n] = a0;
  if (n + 1 < ny) yo[n + 1] = a1;
  if (n + 2 < ny) yo[n + 2] = a2;
  if (n + 3 < ny) yo[n + 3] = a3;
}

__global__ __launch_bounds__(256) void rev_xcorr_kernel(const RevUtt* __restrict__ U, const double* __restrict__ x,
                                                        const double* __restrict__ y, int R, double* __restrict__ xs) {
  __shared__ double xt[kRevTile];
  __shared__ double yw[4 * 256 + kRevTile];
  const RevUtt u = U[blockIdx.y];
  const int s0 = blockIdx.x * 1024;
  if (s0 >= R) return;
  const int64_t ny = u.T + R - 1;
  const int t4 = 4 * threadIdx.x;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  for (int64_t m0 = 0; m0 < u.T; m0 += kRevTile) {
    __syncthreads();
    xt[threadIdx.x] = m0 + threadIdx.x < u.T ? x[u.off + m0 + threadIdx.x] : 0.0;
    // yw[i] = y[m0 + s0 + i]
    for (int i = threadIdx.x; i < 4 * 256 + kRevTile; i += 256) {
      const int64_t q = m0 + s0 + i;
      yw[i] = q < ny ? y[u.yoff + q] : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int mm = 0; mm < kRevTile; ++mm) {
      const double xv = xt[mm];
      const int b = mm + t4;  // y[m + sh] for m = m0 + mm, sh = s0 + t4
      a0 = fma(xv, yw[b], a0);
      a1 = fma(xv, yw[b + 1], a1);
      a2 = fma(xv, yw[b + 2], a2);
      a3 = fma(xv, yw[b + 3], a3);
    }
  }
  double* o = xs + (int64_t)blockIdx.y * R;
  const int sh = s0 + t4;
  if (sh < R) o[sh] = a0;
  if (sh + 1 < R) o[sh + 1] = a1;
  if (sh + 2 < R) o[sh + 2] = a2;
  if (sh + 3 < R) o[sh + 3] = a3;
}

__global__ __launch_bounds__(256) void rev_select_kernel(const RevUtt* __restrict__ U, const double* __restrict__ y,
                                                         const double* __restrict__ xs, int R,
                                                         double* __restrict__ out, int64_t* __restrict__ out_len) {
  __shared__ double bv[256];
  __shared__ int bs[256];
  const RevUtt u = U[blockIdx.x];
  const double* o = xs + (int64_t)blockIdx.x * R;
  double best = -INFINITY;
  int bsh = -1;
  for (int sh = threadIdx.x; sh < R; sh += 256) {
    const double v = o[sh];
    if (v > best || (v == best && sh > bsh) || bsh < 0) { best = v; bsh = sh; }
  }
  bv[threadIdx.x] = best;
  bs[threadIdx.x] = bsh;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const double v2 = bv[threadIdx.x + w];
      const int s2 = bs[threadIdx.x + w];
      if (s2 >= 0 && (bs[threadIdx.x] < 0 || v2 > bv[threadIdx.x] || (v2 == bv[threadIdx.x] && s2 > bs[threadIdx.x]))) {
        bv[threadIdx.x] = v2;
        bs[threadIdx.x] = s2;
      }
    }
    __syncthreads();
  }
  const int64_t ind = (int64_t)bs[0] + 1;  // indM = R - argmax
  const int64_t ny = u.T + R - 1;
  const int64_t L = min(u.T, ny - ind);
  for (int64_t t = threadIdx.x; t < L; t += 256) out[u.off + t] = y[u.yoff + ind + t];
  if (threadIdx.x == 0) out_len[blockIdx.x] = L;
}

hipError_t launch_reverb(const RevUtt* U, int n_utt, int64_t maxT, const void* pcm, int kind, int pre,
                         const int16_t* noise, const double* rir, int R, double* x, double* y, double* xs,
                         double* out, int64_t* out_len, hipStream_t s) {
  if (n_utt <= 0) return hipSuccess;
  hipLaunchKernelGGL(rev_pre_kernel, dim3((unsigned)((maxT + 255) / 256), n_utt), dim3(256), 0, s, U, pcm, kind,
                     pre, noise, x);
  hipLaunchKernelGGL(rev_conv_kernel, dim3((unsigned)((maxT + R - 1 + 1023) / 1024), n_utt), dim3(256), 0, s, U, x,
                     rir, R, y);
  hipLaunchKernelGGL(rev_xcorr_kernel, dim3((unsigned)((R + 1023) / 1024), n_utt), dim3(256), 0, s, U, x, y, R, xs);
  hipLaunchKernelGGL(rev_select_kernel, dim3(n_utt), dim3(256), 0, s, U, y, xs, R, out, out_len);
  return hipGetLastError();
}

// -----------------------------------------------------------------------------------------
// 10. Mel spectrum (src/featgen/computeMelSpectrum.py:147-158, the run_melspec baseline feature):
//     frame = reflect-padded x[k*hop + i - ext] * hamming(L)[i] (getFrames, features.py:118-154),
//     |scipy.fftpack.fft(frame, nfft)[:nfft/2+1]| @ fbank.T, then log10 (or squared for 'power').
//     The real length-nfft FFT runs as a length-nfft/2 complex FFT of the packed frame (z[q] = x[2q] +
//     i x[2q+1]) in LDS with the real-FFT unpacking; kMelCols frames per workgroup.
// -----------------------------------------------------------------------------------------
constexpr int kMelCols = 2;

size_t mel_lds_bytes(int nh) { return sizeof(double2) * 2 * (size_t)nh * kMelCols; }

__global__ __launch_bounds__(256) void mel_kernel(MelConsts c, const MelFrame* __restrict__ frames, int nframes,
                                                  const void* __restrict__ pcm, int pcm_kind,
                                                  const int16_t* __restrict__ noise, float* __restrict__ out,
                                                  double* __restrict__ out64, int decimals, double scale10) {
  extern __shared__ double2 mel_sh[];
  double2* a = mel_sh;
  double2* b = mel_sh + (size_t)c.nh * kMelCols;
  const int f0 = blockIdx.x * kMelCols;
  const int nh = c.nh;
  const int Luse = c.L < c.nfft ? c.L : c.nfft;  // fft(x, n) truncates a longer frame
  // 1. packed windowed frames: a[q * kMelCols + col] = x[2q] + i x[2q+1]
  for (int e = threadIdx.x; e < nh * kMelCols; e += blockDim.x) {
    const int col = e % kMelCols, q = e / kMelCols;
    const int f = f0 + col;
    double v[2] = {0.0, 0.0};
    if (f < nframes) {
      const MelFrame fd = frames[f];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = 2 * q + h;
        if (i < Luse) {
          const int64_t t = reflect_idx((int64_t)fd.k * c.hop + i - c.ext, fd.T);
          double sv;
          if (pcm_kind == 0) {
            sv = (double)((const int16_t*)pcm)[fd.pcm_off + t];
            if (fd.noise_off >= 0) sv = __dadd_rn(sv, __dmul_rn(fd.alpha, (double)noise[fd.noise_off + t]));
          } else if (pcm_kind == 1) {
            sv = ((const double*)pcm)[fd.pcm_off + t];
          } else {  // convolve(int16 s, diff kernel, 'same') -> int64 (computeMelSpectrum.py:136-139)
            const int16_t* x = (const int16_t*)pcm + fd.pcm_off;
            long long acc = 0;
#pragma unroll
            for (int qq = 0; qq < 13; ++qq) {
              const int64_t idx = t + 6 - qq;
              if (idx >= 0 && idx < fd.T) acc += (long long)kDiffTaps[qq] * (long long)x[idx];
            }
            sv = (double)acc;
          }
          v[h] = __dmul_rn(sv, c.window[i]);
        }
      }
    }
    a[e] = make_double2(v[0], v[1]);
  }
  __syncthreads();
  double2* Z = lds_dft(a, b, c.om, c.dp, kMelCols);
  double* mag = (double*)(Z == a ? b : a);  // [kMelCols][nbins]
  // 2. real-FFT unpacking: X[k] = E[k] + W^k O[k], E = (Z[k] + conj Z[nh-k]) / 2, O = (Z[k] - conj Z[nh-k]) / 2i
  for (int e = threadIdx.x; e < c.nbins * kMelCols; e += blockDim.x) {
    const int col = e % kMelCols, k = e / kMelCols;
    const double2 zk = Z[(k % nh) * kMelCols + col];
    const double2 zc = Z[((nh - k) % nh) * kMelCols + col];
    const double2 E = make_double2(0.5 * (zk.x + zc.x), 0.5 * (zk.y - zc.y));
    const double2 O = make_double2(0.5 * (zk.y + zc.y), -0.5 * (zk.x - zc.x));
    const double2 w = c.rtw[k];
    const double2 X = make_double2(E.x + (w.x * O.x - w.y * O.y), E.y + (w.x * O.y + w.y * O.x));
    mag[col * c.nbins + k] = hypot(X.x, X.y);
  }
  __syncthreads();
  // 3. filterbank projection + log10 / power (computeMelSpectrum.py:150-158)
  for (int e = threadIdx.x; e < c.nfilters * kMelCols; e += blockDim.x) {
    const int col = e / c.nfilters, m = e % c.nfilters;
    const int f = f0 + col;
    if (f >= nframes) continue;
    const double* w = c.fbank + (size_t)m * c.nbins;
    const double* mg = mag + col * c.nbins;
    double acc = 0.0;
    for (int k = c.lo[m]; k < c.hi[m]; ++k) acc = fma(mg[k], w[k], acc);
    const double v = c.power ? acc * acc : log10(acc);
    const int64_t o = frames[f].out_row * c.nfilters + m;
    if (out64) out64[o] = v;
    if (out) out[o] = decimals >= 0 ? (float)(nearbyint(v * scale10) / scale10) : (float)v;
  }
}

hipError_t launch_mel(const MelConsts& c, const MelFrame* frames, int nframes, const void* pcm, int pcm_kind,
                      const int16_t* noise, float* out, double* out64, int decimals, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  double scale10 = 1.0;
  for (int i = 0; i < decimals; ++i) scale10 *= 10.0;
  const size_t lds = mel_lds_bytes(c.nh);
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)mel_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(mel_kernel, dim3((nframes + kMelCols - 1) / kMelCols), dim3(256), lds, s, c, frames, nframes,
                     pcm, pcm_kind, noise, out, out64, decimals, scale10);
  return hipGetLastError();
}

// -----------------------------------------------------------------------------------------
// 11. FDLP modulation spectrum output (src/featgen/computeModulationSpectrum.py:165-201): per frame and
//     band, np.real(computeModSpecFromLpc(gg, a, coeff_n)) [* faxis] [abs] sliced [coeff_0-1 : coeff_n]
//     (every other one with --keep_even), rows [frame, band * feat_len + i].  Thread per output value.
// -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void modspec_out_kernel(const double* __restrict__ cep,
                                                          const FrameDesc* __restrict__ frames,
                                                          const UttDesc* __restrict__ utts, int nframes, int B, int M,
                                                          int c0, int feat_len, int step, int first,
                                                          const double* __restrict__ faxis, int absval,
                                                          float* __restrict__ out, double* __restrict__ out64,
                                                          int decimals, double scale10) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)B * feat_len;
  if (e >= (int64_t)nframes * per) return;
  const int f = (int)(e / per);
  const int r = (int)(e % per);
  const int j = r / feat_len, i = r % feat_len;
  const int n = c0 + first + step * i;
  double v = cep[((int64_t)f * B + j) * M + n];
  if (faxis) v = v * faxis[n];
  if (absval) v = fabs(v);
  const FrameDesc fd = frames[f];
  const int64_t o = (utts[fd.utt].out_row + fd.k) * per + r;
  if (out64) out64[o] = v;
  if (out) out[o] = decimals >= 0 ? (float)(nearbyint(v * scale10) / scale10) : (float)v;
}

// -----------------------------------------------------------------------------------------
// Complex modulation spectrum (computeModulationSpectrum.py --complex_modulation, :153-180).
// cplx_autocorr_kernel: one wave per (frame, band) item, a lane per lag: with s = W_j X (the band's
// complex spectrum, bins [0, L)), y[l] = sum_n s[(n + l) mod L] conj(s[n]) -- the circular
// autocorrelation ifft(fft(s) conj(fft(s))) of computeLpcFast(keepreal=False) (features.py:223) as a
// direct sum over the band's non-zero taps [lo, hi).
// -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void cplx_autocorr_kernel(DevConsts c, int L, const double* __restrict__ X,
                                                           int items, double* __restrict__ y) {
  const int item = blockIdx.x;
  if (item >= items) return;
  const int f = item / c.B, j = item % c.B;
  const double2* Xr = (const double2*)(X + (int64_t)f * c.N);
  const double* W = c.fbank + (int64_t)j * c.N;
  const int lo = c.lo[j], hi = c.hi[j];
  for (int l0 = 0; l0 < c.nlags; l0 += 64) {
    const int l = l0 + (int)threadIdx.x;
    const int lc = l < c.nlags ? l : 0;
    double re = 0.0, im = 0.0;
    for (int n = lo; n < hi; ++n) {
      const double wn = W[n];
      const double2 xn = Xr[n];
      const double sr = wn * xn.x, si = wn * xn.y;  // s[n] = filt * cos_trans (features: band_dct)
      int m = n + lc;
      if (m >= L) m -= L;
      const double wm = W[m];
      const double2 xm = Xr[m];
      const double tr = wm * xm.x, ti = wm * xm.y;
      re = fma(tr, sr, fma(ti, si, re));     // Re s[m] conj(s[n])
      im = fma(ti, sr, fma(-tr, si, im));    // Im
    }
    if (l < c.nlags) {
      y[((int64_t)item * c.nlags + l) * 2] = re;
      y[((int64_t)item * c.nlags + l) * 2 + 1] = im;
    }
  }
}

__device__ __forceinline__ double2 wave_sum2(double2 v) { return make_double2(wave_sum(v.x), wave_sum(v.y)); }
__device__ __forceinline__ double2 cmul2(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// numpy's principal complex sqrt (npy_csqrt) and log
__device__ __forceinline__ double2 csqrt_np(double2 z) {
  if (z.x == 0.0 && z.y == 0.0) return make_double2(0.0, z.y);
  const double t = sqrt((fabs(z.x) + hypot(z.x, z.y)) * 0.5);
  if (z.x >= 0.0) return make_double2(t, z.y / (2.0 * t));
  return make_double2(fabs(z.y) / (2.0 * t), copysign(t, z.y));
}
__device__ __forceinline__ double2 clog_np(double2 z) { return make_double2(log(hypot(z.x, z.y)), atan2(z.y, z.x)); }

// cplx_lpc_out_kernel: one wave per item.  Levinson-Durbin on the Hermitian Toeplitz system of
// solve_toeplitz(y[0:p], -y[1:p+1]) (features.py:226; a_i += kappa conj(a_{k-i})), the complex gain
// gg = y[0] + sum a_i y[i+1] (:228), the complex cepstrum computeModSpecFromLpc (:233-246, c_0 =
// log(sqrt(gg)) on numpy's principal branches), then [* faxis], abs or (real, imag) of the slice
// [c0, coeff_n), keep_even (step 2 from `first`) into the item's output columns (:174-201).
__global__ __launch_bounds__(64) void cplx_lpc_out_kernel(const double* __restrict__ ycplx, int items, int B, int p,
                                                          int nlags, int coeff_n, const FrameDesc* __restrict__ frames,
                                                          const UttDesc* __restrict__ utts, int c0, int feat_len,
                                                          int step, int first, const double* __restrict__ faxis,
                                                          int absval, float* __restrict__ out, double* __restrict__ out64,
                                                          int decimals, double scale10) {
  extern __shared__ double2 csh[];
  const int item = blockIdx.x;
  if (item >= items) return;
  const int lane = threadIdx.x;
  const int NA = (p + 1 > coeff_n + 1 ? p + 1 : coeff_n + 1);
  double2* ys = csh;             // nlags
  double2* a = ys + nlags;       // NA: a_0 .. a_p, zeros beyond (alpha = -a past the order is 0)
  double2* cep = a + NA;         // coeff_n
  const double2* yi = (const double2*)ycplx + (int64_t)item * nlags;
  for (int l = lane; l < nlags; l += 64) ys[l] = yi[l];
  for (int i = lane; i < NA; i += 64) a[i] = make_double2(i == 0 ? 1.0 : 0.0, 0.0);
  __syncthreads();
  double E = ys[0].x;
  for (int k = 1; k <= p; ++k) {
    double2 part = make_double2(0.0, 0.0);
    for (int i = 1 + lane; i < k; i += 64) {
      const double2 t = cmul2(a[i], ys[k - i]);
      part.x += t.x;
      part.y += t.y;
    }
    const double2 acc = wave_sum2(part);
    const double2 yk = ys[k];
    const double2 kap = make_double2(-(yk.x + acc.x) / E, -(yk.y + acc.y) / E);
    double2 nv[4];
    int cnt = 0;
    for (int i = 1 + lane; i < k; i += 64, ++cnt) {
      const double2 am = a[k - i];
      const double2 t = cmul2(kap, make_double2(am.x, -am.y));
      nv[cnt & 3] = make_double2(a[i].x + t.x, a[i].y + t.y);
    }
    __syncthreads();
    cnt = 0;
    for (int i = 1 + lane; i < k; i += 64, ++cnt) a[i] = nv[cnt & 3];
    if (lane == 0) a[k] = kap;
    __syncthreads();
    E = E * (1.0 - (kap.x * kap.x + kap.y * kap.y));
  }
  // gg = y[0] + sum_{i=0}^{p} a_i y[i+1]
  double2 part = make_double2(0.0, 0.0);
  for (int i = lane; i <= p; i += 64) {
    const double2 t = cmul2(a[i], ys[i + 1]);
    part.x += t.x;
    part.y += t.y;
  }
  const double2 sg = wave_sum2(part);
  const double2 gg = make_double2(ys[0].x + sg.x, ys[0].y + sg.y);
  // cepstrum: alpha_i = -a_i
  if (lane == 0) {
    cep[0] = clog_np(csqrt_np(gg));
    if (coeff_n > 1) cep[1] = make_double2(-a[1].x, -a[1].y);
  }
  __syncthreads();
  for (int n = 2; n < coeff_n; ++n) {
    double2 q = make_double2(0.0, 0.0);
    for (int k = 1 + lane; k < n; k += 64) {
      const double w = (double)k / (double)n;                 // aa = arange(1, n) / n
      const double2 al = make_double2(-a[n - k].x, -a[n - k].y);  // bb = flipud(alpha[1:n])
      const double2 t = cmul2(make_double2(w * al.x, w * al.y), cep[k]);
      q.x += t.x;
      q.y += t.y;
    }
    const double2 sq = wave_sum2(q);
    if (lane == 0) cep[n] = make_double2(sq.x - a[n].x, sq.y - a[n].y);  // + alpha_n
    __syncthreads();
  }
  const int sel = coeff_n - c0;
  const int f = item / B, j = item % B;
  const FrameDesc fd = frames[f];
  const int64_t row = (utts[fd.utt].out_row + fd.k) * (int64_t)B * feat_len + (int64_t)j * feat_len;
  for (int i = lane; i < feat_len; i += 64) {
    const int qq = first + step * i;  // temp2 index
    double v;
    if (absval) {
      double2 z = cep[c0 + qq];
      if (faxis) z = make_double2(z.x * faxis[c0 + qq], z.y * faxis[c0 + qq]);
      v = hypot(z.x, z.y);
    } else {
      const int nn = qq < sel ? qq : qq - sel;
      double2 z = cep[c0 + nn];
      if (faxis) z = make_double2(z.x * faxis[c0 + nn], z.y * faxis[c0 + nn]);
      v = qq < sel ? z.x : z.y;
    }
    if (out64) out64[row + i] = v;
    if (out) out[row + i] = decimals >= 0 ? (float)(nearbyint(v * scale10) / scale10) : (float)v;
  }
}

hipError_t launch_cplx_modspec(const DevConsts& c, int L, const double* X, int nframes, double* ycplx,
                               const FrameDesc* frames, const UttDesc* utts, int c0, int coeff_n, int feat_len,
                               int step, int first, const double* faxis, int absval, float* out, double* out64,
                               int decimals, hipStream_t s) {
  const int items = nframes * c.B;
  if (items <= 0) return hipSuccess;
  hipLaunchKernelGGL(cplx_autocorr_kernel, dim3(items), dim3(64), 0, s, c, L, X, items, ycplx);
  double scale10 = 1.0;
  for (int i = 0; i < decimals; ++i) scale10 *= 10.0;
  const int NA = std::max(c.p + 1, coeff_n + 1);
  const size_t lds = sizeof(double2) * ((size_t)c.nlags + NA + coeff_n);
  hipLaunchKernelGGL(cplx_lpc_out_kernel, dim3(items), dim3(64), lds, s, ycplx, items, c.B, c.p, c.nlags, coeff_n,
                     frames, utts, c0, feat_len, step, first, faxis, absval, out, out64, decimals, scale10);
  return hipGetLastError();
}

hipError_t launch_modspec_out(const double* cep, const FrameDesc* frames, const UttDesc* utts, int nframes, int B,
                              int M, int c0, int feat_len, int step, int first, const double* faxis, int absval,
                              float* out, double* out64, int decimals, hipStream_t s) {
  const int64_t total = (int64_t)nframes * B * feat_len;
  if (total <= 0) return hipSuccess;
  double scale10 = 1.0;
  for (int i = 0; i < decimals; ++i) scale10 *= 10.0;
  hipLaunchKernelGGL(modspec_out_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, cep, frames, utts,
                     nframes, B, M, c0, feat_len, step, first, faxis, absval, out, out64, decimals, scale10);
  return hipGetLastError();
}

}  // namespace fdlp
