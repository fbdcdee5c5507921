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
//   4. levinson     : one wave per (frame, band), Durbin recursion + gg.     (features.py:226-228)
//   5. cepstrum     : one wave per item, LPC-cepstrum recursion, block-parallel. (features.py:233-246)
//   6. envelope     : exp(Re DFT_{2*fd*fr}(c .* w))[0:kk] * hann/hamm.          (:194-205)
//   7. ola_log      : deterministic gather OLA + floor + log -> float32 [L, B].  (:207-229)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

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
  for (int b = threadIdx.x; b < total; b += blockDim.x) {
    const int col = b % ncols;
    const int j = b / ncols;
    const int k = j % Ns;
    double2 v[R];
    const int twstep = (n / (Ns * R)) * k;  // omega_{Ns*R}^{k*r} = omega_n^{k*r*n/(Ns*R)}
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double2 x = in[(j + r * nb) * ncols + col];
      v[r] = (r == 0) ? x : cmul(x, om[(twstep * r) % n]);
    }
    small_dft<R>(v, om, n);
    const int idxD = (j / Ns) * Ns * R + k;
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
  // numpy 'reflect' pad == periodic reflection with period 2(T-1) (features.py:146)
  if (T == 1) return 0;
  const int64_t P = 2 * (T - 1);
  q %= P;
  if (q < 0) q += P;
  return q < T ? q : P - q;
}

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
  const int N = c.N;
  for (int q = threadIdx.x; q < N1; q += blockDim.x) oms[q] = om1[q];

  FrameDesc fd;
  if (!dense_rows) fd = frames[f];
  // load v[N2*n1 + n2] for n1 in [0,N1), n2 in [n2_0, n2_0+kDftCols)
  for (int e = threadIdx.x; e < N1 * kDftCols; e += blockDim.x) {
    const int col = e % kDftCols;
    const int n1 = e / kDftCols;
    const int n2 = n2_0 + col;
    double val = 0.0;
    if (n2 < N2) {
      const int n = N2 * n1 + n2;
      const int m = (2 * n < N) ? 2 * n : 2 * N - 1 - 2 * n;  // Makhoul even/odd split
      if (dense_rows) {
        val = dense_rows[(int64_t)f * N + m];
      } else {
        const int64_t t = reflect_idx((int64_t)fd.k * c.hop + m - c.ext, fd.T);
        double s;
        if (pcm_kind == 0) {
          s = (double)((const int16_t*)pcm)[fd.pcm_off + t];
          if (fd.noise_off >= 0) {
            // sig + alp*ns, evaluated in fp64 without contraction (features.py:31)
            const double ns = (double)noise[fd.noise_off + t];
            s = __dadd_rn(s, __dmul_rn(fd.alpha, ns));
          }
        } else {
          s = ((const double*)pcm)[fd.pcm_off + t];
        }
        val = __dmul_rn(s, c.hamming[m]);  // frame * win (features.py:153)
      }
    }
    bufA[n1 * kDftCols + col] = make_double2(val, 0.0);
  }
  __syncthreads();
  double2* res = lds_dft(bufA, bufB, oms, d1, kDftCols);
  // twiddle exp(-2 pi i n2 k1 / N) and store z[f][k1][n2]
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
// -----------------------------------------------------------------------------------------
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
  const int k1_0 = blockIdx.x * kDftCols;
  const int N = c.N;
  for (int q = threadIdx.x; q < N2; q += blockDim.x) oms[q] = om2[q];
  for (int e = threadIdx.x; e < N2 * kDftCols; e += blockDim.x) {
    const int row = e / N2;  // coalesced over n2
    const int n2 = e % N2;
    const int k1 = k1_0 + row;
    double2 v = make_double2(0.0, 0.0);
    if (k1 < N1) v = z[((int64_t)f * N1 + k1) * N2 + n2];
    bufA[n2 * kDftCols + row] = v;
  }
  __syncthreads();
  double2* res = lds_dft(bufA, bufB, oms, d2, kDftCols);
  for (int e = threadIdx.x; e < N2 * kDftCols; e += blockDim.x) {
    const int row = e % kDftCols;
    const int k2 = e / kDftCols;
    const int k1 = k1_0 + row;
    if (k1 < N1) {
      const int k = k1 + N1 * k2;
      const double2 V = res[k2 * kDftCols + row];
      const double2 w = ((const double2*)c.post)[k];
      const double y = 2.0 * (w.x * V.x - w.y * V.y);
      dct[(int64_t)f * N + k] = y / inv_scale_div;  // dct(.)/np.sqrt(2N)  (:178)
    }
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
constexpr int kAcChunk = 1024;  // positions staged per LDS chunk

template <int NT>
__global__ __launch_bounds__(64) void autocorr_kernel(DevConsts c, const double* __restrict__ dct,
                                                      const double* __restrict__ dense,
                                                      double* __restrict__ rout) {
  constexpr int G = 4;                                  // tiles per epilogue group
  constexpr int kEpi = (16 * G + 15) * 17;              // padded lag-major epilogue buffer
  constexpr int kStage = kAcChunk + 16 * NT;
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
  for (int s0 = 0; s0 < nsteps; s0 += kAcChunk / 64) {
    const int steps = min(kAcChunk / 64, nsteps - s0);
    const int base = lo + 64 * s0;
    const int extent = 64 * steps + 16 * NT;
    for (int q = lane; q < extent; q += 64) {
      int pos = base + q;
      while (pos >= N) pos -= N;  // circular
      double v = 0.0;
      if (pos >= lo && pos < hi) v = wrow ? wrow[pos] * drow[pos] : drow[pos];  // filt*dct (:191)
      xs[q] = v;
    }
    __syncthreads();
    for (int s = 0; s < steps; ++s) {
      const double* w = xs + 64 * s + 16 * kk_lane + i_lane;
      const double a = w[0];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, w[16 * t], acc[t], 0, 0, 0);
    }
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
    if (L < nlags) rout[(int64_t)item * nlags + L] = mine[q];
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
// 4. Levinson-Durbin (features.py:226-228): Toeplitz(r[0..p-1]) a' = -r[1..p]; a = [1, a'];
//    gg = r0 + sum_{l=0}^{p} a_l r_{l+1}.  One wave per item, a[] distributed over lanes.
// -----------------------------------------------------------------------------------------
template <int SL>
__global__ __launch_bounds__(64) void levinson_kernel(int p, int nlags, const double* __restrict__ r,
                                                      double* __restrict__ aout,
                                                      double* __restrict__ ggout) {
  __shared__ double rs[64 * SL + 64];
  __shared__ double as[64 * SL];
  const int item = blockIdx.x;
  const int lane = threadIdx.x;
  for (int q = lane; q < 64 * SL + 64; q += 64) rs[q] = q < nlags ? r[(int64_t)item * nlags + q] : 0.0;
  __syncthreads();
  double a[SL];
#pragma unroll
  for (int s = 0; s < SL; ++s) a[s] = (lane + 64 * s == 0) ? 1.0 : 0.0;
  double E = rs[0];
  for (int k = 1; k <= p; ++k) {
    double part = 0.0;
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      const int idx = lane + 64 * s;
      if (idx >= 1 && idx < k) part += a[s] * rs[k - idx];
    }
    const double acc = rs[k] + wave_sum(part);
    const double kappa = -acc / E;
#pragma unroll
    for (int s = 0; s < SL; ++s) as[lane + 64 * s] = a[s];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      const int idx = lane + 64 * s;
      if (idx >= 1 && idx < k) a[s] = a[s] + kappa * as[k - idx];
      else if (idx == k) a[s] = kappa;
    }
    __syncthreads();
    E = E * (1.0 - kappa * kappa);
  }
  double part = 0.0;
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    const int idx = lane + 64 * s;
    if (idx <= p) part += a[s] * rs[idx + 1];
  }
  const double gg = rs[0] + wave_sum(part);
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    const int idx = lane + 64 * s;
    if (idx <= p) aout[(int64_t)item * (p + 1) + idx] = a[s];
  }
  if (lane == 0) ggout[item] = gg;
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
// 6. envelope (computeFDLPSpectrogram.py:194-205):
//    ms = c * mask [* lifter] [* gamma]; odd coefficients := 0; fft(ms, env_nfft) truncates or
//    zero-pads; abs(exp(.)) = exp(Re); [0:kk] * hanning(kk) / hamming(kk).
// -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void envelope_kernel(DevConsts c, int odd_zero, const double* __restrict__ cep,
                                                      double* __restrict__ env) {
  extern __shared__ double sh[];
  double* cw = sh;                  // [Me]
  double* cq = sh + c.Me;           // [env_nfft]
  const int item = blockIdx.x;
  const int lane = threadIdx.x;
  const double* mask = c.weights;
  const double* lif = c.weights + c.M;
  const double* gam = c.weights + 2 * c.M;
  for (int n = lane; n < c.Me; n += 64) {
    double v = cep[(int64_t)item * c.M + n];
    v = v * mask[n];  // :194
    v = v * lif[n];   // :195-196 (1.0 when absent: exact)
    v = v * gam[n];   // :197-198 (1.0 when absent: exact)
    if (odd_zero && (n & 1)) v = 0.0;  // :199-200 assignment (NaN-safe like the reference)
    cw[n] = v;
  }
  for (int q = lane; q < c.env_nfft; q += 64) cq[q] = c.env_cos[q];
  __syncthreads();
  for (int t = lane; t < c.kk; t += 64) {
    double s = 0.0;
    int idx = 0;  // (n*t) mod env_nfft
    for (int n = 0; n < c.Me; ++n) {
      s += cw[n] * cq[idx];
      idx += t;
      if (idx >= c.env_nfft) idx -= c.env_nfft;
    }
    const double e = exp(s);
    env[(int64_t)item * c.kk + t] = (e * c.env_win[2 * t]) / c.env_win[2 * t + 1];
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
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)frames_dft1_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(frames_dft1_kernel, grid, dim3(256), lds, s, c, d1, N2, pcm, pcm_kind, noise,
                     frames, dense_rows, om1, z);
  return hipGetLastError();
}

hipError_t launch_dft2_dct(const DevConsts& c, const DftPlan& d2, int N1, const double2* z,
                           int nframes, double* dct, const double2* om2, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  dim3 grid((N1 + kDftCols - 1) / kDftCols, nframes);
  size_t lds = sizeof(double2) * (2 * d2.n * kDftCols + d2.n);
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)dft2_dct_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const double div = sqrt((double)(2 * c.N));
  hipLaunchKernelGGL(dft2_dct_kernel, grid, dim3(256), lds, s, c, d2, N1, z, om2, div, dct);
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_ac_nt(const DevConsts& c, const double* dct, const double* dense, int items,
                               double* r, hipStream_t s) {
  hipLaunchKernelGGL(autocorr_kernel<NT>, dim3(items), dim3(64), 0, s, c, dct, dense, r);
  return hipGetLastError();
}

int autocorr_tiles(int nlags) { return ((nlags + 14) >> 4) + 1; }

hipError_t launch_autocorr(const DevConsts& c, const double* dct, const double* dense, int items,
                           double* r, hipStream_t s) {
  if (items <= 0) return hipSuccess;
  switch (autocorr_tiles(c.nlags)) {
#define FDLP_AC_CASE(n) case n: return launch_ac_nt<n>(c, dct, dense, items, r, s);
    FDLP_AC_CASE(1) FDLP_AC_CASE(2) FDLP_AC_CASE(3) FDLP_AC_CASE(4) FDLP_AC_CASE(5)
    FDLP_AC_CASE(6) FDLP_AC_CASE(7) FDLP_AC_CASE(8) FDLP_AC_CASE(9) FDLP_AC_CASE(10)
    FDLP_AC_CASE(11) FDLP_AC_CASE(12) FDLP_AC_CASE(13) FDLP_AC_CASE(14) FDLP_AC_CASE(15)
    FDLP_AC_CASE(16) FDLP_AC_CASE(17) FDLP_AC_CASE(18) FDLP_AC_CASE(19) FDLP_AC_CASE(20)
    FDLP_AC_CASE(21) FDLP_AC_CASE(22) FDLP_AC_CASE(23) FDLP_AC_CASE(24)
#undef FDLP_AC_CASE
    default: return hipErrorInvalidValue;
  }
}

template <int SL>
static hipError_t launch_lev_sl(int p, int nlags, const double* r, int items, double* a, double* gg,
                                hipStream_t s) {
  hipLaunchKernelGGL(levinson_kernel<SL>, dim3(items), dim3(64), 0, s, p, nlags, r, a, gg);
  return hipGetLastError();
}

hipError_t launch_levinson(const DevConsts& c, const double* r, int items, double* a, double* gg,
                           hipStream_t s) {
  if (items <= 0) return hipSuccess;
  const int sl = (c.p + 1 + 63) / 64;
  switch (sl) {
    case 1: return launch_lev_sl<1>(c.p, c.nlags, r, items, a, gg, s);
    case 2: return launch_lev_sl<2>(c.p, c.nlags, r, items, a, gg, s);
    case 3: return launch_lev_sl<3>(c.p, c.nlags, r, items, a, gg, s);
    case 4: return launch_lev_sl<4>(c.p, c.nlags, r, items, a, gg, s);
    case 5: return launch_lev_sl<5>(c.p, c.nlags, r, items, a, gg, s);
    case 6: return launch_lev_sl<6>(c.p, c.nlags, r, items, a, gg, s);
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

hipError_t launch_envelope(const DevConsts& c, int odd_zero, const double* cep, int items, double* env,
                           hipStream_t s) {
  if (items <= 0) return hipSuccess;
  size_t lds = sizeof(double) * (c.Me + c.env_nfft);
  hipLaunchKernelGGL(envelope_kernel, dim3(items), dim3(64), lds, s, c, odd_zero, cep, env);
  return hipGetLastError();
}

hipError_t launch_ola_log(const DevConsts& c, const double* env, const FrameDesc* frames, const UttDesc* utts,
                          int n_utt, int maxL, float* out, double* out_f64, int decimals, hipStream_t s) {
  if (n_utt <= 0 || maxL <= 0) return hipSuccess;
  const int64_t per = (int64_t)maxL * c.B;
  dim3 grid((unsigned)((per + 255) / 256), n_utt);
  double scale10 = 1.0;
  for (int i = 0; i < decimals; ++i) scale10 *= 10.0;
  hipLaunchKernelGGL(ola_log_kernel, grid, dim3(256), 0, s, c, env, frames, utts, out, out_f64, decimals,
                     scale10);
  return hipGetLastError();
}

}  // namespace fdlp
