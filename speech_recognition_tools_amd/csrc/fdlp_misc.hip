// fdlp_misc.hip -- gfx950 kernels around the hot path: the OLA + log output stage
// (computeFDLPSpectrogram.py:207-229), global CMVN statistics, addReverb, the mel spectrum and the
// modulation-spectrum outputs.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include "fdlp_device.h"

namespace fdlp {

// -----------------------------------------------------------------------------------------
// OLA + floor + log (computeFDLPSpectrogram.py:207-229).  One workgroup per (utterance, kOlaRows output
// rows): the frames overlapping the tile are added in frame order into an LDS tile [row][band]
// (0 + e_a + e_b, bit-identical to the reference's in-place adds), reading each frame's envelope rows
// [band][t] with consecutive threads on consecutive t (coalesced), then log(clip(., 1e-14)) keeping
// NaN, float32 (optionally '%.3f'-rounded) row-major stores and the fp64 debug copy.
// -----------------------------------------------------------------------------------------
constexpr int kOlaRows = 32;
constexpr int kOlaFr = 3;   // frames on a tile summed in registers (kk <= 2 hops + 31 rows: every recipe)
constexpr int kOlaJ = 10;   // bands per thread in that path (B <= 80)
__global__ __launch_bounds__(256) void ola_log_tiled_kernel(DevConsts c, const double* __restrict__ env,
                                                            const FrameDesc* __restrict__ frames,
                                                            const UttDesc* __restrict__ utts, float* __restrict__ out,
                                                            double* __restrict__ out64, int16_t* __restrict__ outq,
                                                            uint32_t* __restrict__ qflag, int decimals, double scale10) {
  extern __shared__ double tile[];  // [kOlaRows][B + 1]
  __shared__ int fr_lo, fr_hi;      // the frames overlapping the tile
  __shared__ double ltab[3 * kLogTab];  // ola_log's table
  const int u = blockIdx.y;
  const UttDesc U = utts[u];
  const int t0 = blockIdx.x * kOlaRows;
  if (t0 >= U.L) return;
  const int nt = min(kOlaRows, U.L - t0);
  const int B = c.B, BS = c.B + 1, kk = c.kk;
  const int tid = threadIdx.x;
  for (int q = tid; q < kOlaRows * BS; q += blockDim.x) tile[q] = 0.0;
  for (int q = tid; q < 3 * kLogTab; q += blockDim.x) ltab[q] = kLogTable[q];
  // frames overlapping [t0, t0 + nt): dst is non-decreasing in k, so they are a range; every thread tests
  // its own frames at once (one memory round trip, not a binary search of dependent loads) and the range
  // ends are the smallest / largest frame that overlaps (a frame past t0 + nt or ending before t0 does not)
  if (tid == 0) {
    fr_lo = U.F;
    fr_hi = -1;
  }
  __syncthreads();
  for (int k = tid; k < U.F; k += blockDim.x) {
    const FrameDesc fd = frames[U.frame0 + k];
    if (fd.dst < t0 + nt && fd.dst + kk > t0) {
      atomicMin(&fr_lo, k);
      atomicMax(&fr_hi, k);
    }
  }
  __syncthreads();
  const int kf = fr_lo, lo = fr_hi;
  const int tt = tid % kOlaRows, jj = tid / kOlaRows;  // 8 band lanes x 32 rows
  // the cell (tt, j) of the tile belongs to one thread across the frames, so the usual case -- at most
  // kOlaFr frames on the tile, B <= 8 kOlaJ -- sums in registers with all envelope loads issued before the
  // first add (one exposed memory latency), in frame order, 0 + e_a + e_b as the reference's in-place adds
  if (lo - kf < kOlaFr && B <= 8 * kOlaJ) {
    const int t = t0 + tt;
    double v[kOlaFr][kOlaJ];
    bool cov[kOlaFr];
#pragma unroll
    for (int m = 0; m < kOlaFr; ++m) {
      const int k = min(kf + m, U.F - 1);
      const FrameDesc fd = frames[U.frame0 + k];
      cov[m] = kf + m <= lo && t < t0 + nt && t >= fd.dst && t < fd.dst + fd.cnt;
      const double* er = env + (int64_t)(U.frame0 + k) * B * kk + (cov[m] ? fd.src + (t - fd.dst) : 0);
#pragma unroll
      for (int i = 0; i < kOlaJ; ++i) {
        const int j = jj + 8 * i;
        v[m][i] = cov[m] && j < B ? er[(int64_t)j * kk] : 0.0;
      }
    }
#pragma unroll
    for (int i = 0; i < kOlaJ; ++i) {
      const int j = jj + 8 * i;
      double acc = 0.0;
#pragma unroll
      for (int m = 0; m < kOlaFr; ++m)
        if (cov[m]) acc = acc + v[m][i];
      if (j < B) tile[tt * BS + j] = acc;
    }
    __syncthreads();
  } else {
  for (int k = kf; k <= lo; ++k) {
    const FrameDesc fd = frames[U.frame0 + k];
    const int t = t0 + tt;
    if (t < t0 + nt && t >= fd.dst && t < fd.dst + fd.cnt) {
      FDLP_CHECK(fd.src + (t - fd.dst) >= 0 && fd.src + (t - fd.dst) < kk && k < U.F && t < U.L);
      const double* er = env + (int64_t)(U.frame0 + k) * B * kk + fd.src + (t - fd.dst);
      for (int j = jj; j < B; j += blockDim.x / kOlaRows) tile[tt * BS + j] = tile[tt * BS + j] + er[(int64_t)j * kk];
    }
    __syncthreads();
  }
  }
  // t = q / B by a float reciprocal: (q + 0.5) / B sits at least 0.5 / B from an integer, and two float
  // roundings move it by at most (q / B) 2^-22 <= kOlaRows 2^-22, far less for any B below 65536
  const float invB = 1.0f / (float)B;
  bool bad = false;
  for (int q = tid; q < nt * B; q += blockDim.x) {
    const int t = (int)(((float)q + 0.5f) * invB), j = q - t * B;
    FDLP_CHECK(t >= 0 && t < nt && j >= 0 && j < B);
    ola_store_feature(tile[t * BS + j], (U.out_row + t0 + t) * (int64_t)B + j, out, out64, outq, decimals, scale10,
                      bad, ltab);
  }
  if (bad) *qflag = 1u;
}


hipError_t launch_ola_log(const DevConsts& c, const double* env, const FrameDesc* frames, const UttDesc* utts,
                          int n_utt, int maxL, float* out, double* out_f64, int16_t* out_q, uint32_t* q_flag,
                          int decimals, hipStream_t s) {
  if (n_utt <= 0 || maxL <= 0) return hipSuccess;
  if (out_q && (decimals < 0 || !q_flag)) return hipErrorInvalidValue;
  double scale10 = 1.0;
  for (int i = 0; i < decimals; ++i) scale10 *= 10.0;
  dim3 grid((unsigned)((maxL + kOlaRows - 1) / kOlaRows), n_utt);
  const size_t lds = sizeof(double) * kOlaRows * (size_t)(c.B + 1);
  // the kernel's static LDS (log table, frame range) counts against the same 64 KB default limit
  constexpr size_t kStaticLds = sizeof(double) * 3 * kLogTab + 2 * sizeof(int);
  if (lds + kStaticLds > 160 * 1024) return hipErrorInvalidValue;  // B > ~620 bands: no tile fits a CU
  if (lds + kStaticLds > 65536)
    (void)hipFuncSetAttribute((const void*)ola_log_tiled_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(ola_log_tiled_kernel, grid, dim3(256), lds, s, c, env, frames, utts, out, out_f64, out_q, q_flag,
                     decimals, scale10);
  (void)kmark(kKOlaLog, s);
  return hipGetLastError();
}

// the path's log / exp on n values (fdlp_device_fn: accuracy tests of ola_log and the envelope's exp against numpy)
__global__ __launch_bounds__(256) void device_fn_kernel(int fn, const double* __restrict__ x, double* __restrict__ y,
                                                        int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = fn == 0 ? ola_log(x[i], kLogTable) : exp(x[i]);
}

hipError_t launch_device_fn(int fn, const double* x, double* y, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(device_fn_kernel, dim3((unsigned)blocks), dim3(256), 0, s, fn, x, y, n);
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


hipError_t checks_misc(unsigned int* v, bool reset) { return fdlp_checks_local(v, reset); }

}  // namespace fdlp
