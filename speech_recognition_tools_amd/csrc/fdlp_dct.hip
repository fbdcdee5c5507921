// fdlp_dct.hip -- gfx950 kernels of the DCT stage:
//   1. frames_dft1 : int16/f64 PCM -> reflect pad -> window -> Makhoul reorder -> column DFTs (length N1)
//                    of the four-step N = N1*N2 DFT, twiddled (getFrames features.py:118-154, :174-178)
//   2. dft2_dct    : row DFTs (length N2) -> Makhoul post-twiddle -> DCT-II/sqrt(2N) (:178)
// fp64 throughout.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <type_traits>
#include <vector>
#include <stdint.h>
#include <stdlib.h>

#include "fdlp_device.h"

namespace fdlp {

// -----------------------------------------------------------------------------------------
// 1. frames -> Makhoul-reordered real sequence -> column DFTs (length N1) + four-step twiddle
// -----------------------------------------------------------------------------------------
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
  FDLP_CHECK(dense_rows || (t >= 0 && t < fd.T));
  double s;
  if (pcm_kind == 0) {
    s = (double)((const int16_t*)pcm)[fd.pcm_off + t];
    if (fd.noise_off >= 0) {
      // sig + alp*ns, evaluated in fp64 without contraction (features.py:31)
      const double ns = (double)noise[fd.noise_off + t];
      s = __dadd_rn(s, __dmul_rn(fd.alpha, ns));
    }
  } else if (pcm_kind == 1) {
    // the double values of scipy's array for the other WAV formats (uint8 / int32 / int64 / float32 /
    // float64); noise mixing as for int16: sig + alp*ns in fp64 (features.py:31, any dtype + float64)
    s = ((const double*)pcm)[fd.pcm_off + t];
    if (fd.noise_off >= 0) s = __dadd_rn(s, __dmul_rn(fd.alpha, (double)noise[fd.noise_off + t]));
  } else if (pcm_kind == 2) {
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
  } else {
    // pcm_kind 3: the same 'same' convolution of a non-int16 signal (its double values): scipy takes the
    // direct route (np.convolve, float64 or int64 sums), here a float64 dot in increasing sample order; the
    // products tap x sample are exact and so are the sums of any integer or 16/24-bit-scaled signal
    const double* x = (const double*)pcm + fd.pcm_off;
    double acc = 0.0;
#pragma unroll
    for (int q = 12; q >= 0; --q) {
      const int64_t idx = t + 6 - q;
      if (idx >= 0 && idx < fd.T) acc = __dadd_rn(acc, __dmul_rn((double)kDiffTaps[q], x[idx]));
    }
    s = acc;
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

// -----------------------------------------------------------------------------------------
// 1s/2s. The same two DCT passes specialised at compile time for the recipes' frame length
// (N = 24000: packed length-12000 complex FFT = 100 x 120; radices 4.5.5 and 8.3.5): constant
// butterflies (roots of unity as literals), constant Stockham strides, COLS interleaved columns
// (rows) per workgroup, and a branch-free sample gather for frames that need no reflect padding.
// Same arithmetic order per butterfly as the generic passes (Stockham DIT, twiddle then DFT).
// -----------------------------------------------------------------------------------------
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
// columns in LDS, in place; om = the N roots omega_N^q.  Every thread reads and transforms all its
// butterflies first, then a barrier, then the writes: one buffer instead of two, so twice the workgroups
// fit a CU's LDS (round 2: 0.96 -> 0.87 ms for the DCT stage against ping-pong buffers).
template <int N, int COLS, int NT, int Ns, int R, bool SWZ = false>
__device__ __forceinline__ void st_stage_c(double2* __restrict__ buf, const double2* __restrict__ om) {
  static_assert(!SWZ || COLS == 8, "swizzle of 8 columns");
  constexpr int NB = N / R, TOT = NB * COLS, ITER = (TOT + NT - 1) / NT, TW0 = N / (Ns * R);
  auto slot = [&](int pos, int col) { return SWZ ? lslot<SWZ>(pos, col) : pos * COLS + col; };
  double2 v[ITER][R];
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int b = (int)threadIdx.x + it * NT;
    if (TOT % NT != 0 && b >= TOT) break;
    const int col = b % COLS, j = b / COLS;
    const int k = j % Ns;
    double2 (&w)[R] = v[it];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double2 x = buf[slot(j + r * NB, col)];
      w[r] = (r == 0 || Ns == 1) ? x : cmul(x, om[TW0 * k * r]);
    }
    bfly_c<R>(w);
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int b = (int)threadIdx.x + it * NT;
    if (TOT % NT != 0 && b >= TOT) break;
    const int col = b % COLS, j = b / COLS;
    const int k = j % Ns, jq = j / Ns;
    const int idxD = jq * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) buf[slot(idxD + r * Ns, col)] = v[it][r];
  }
}

// full length-N DFT of COLS columns in place in `a`, radices R0 R1 ...
template <int N, int COLS, int NT, bool SWZ, int Ns, int R0, int... Rs>
__device__ __forceinline__ double2* lds_dft_c(double2* a, const double2* om) {
  st_stage_c<N, COLS, NT, Ns, R0, SWZ>(a, om);
  __syncthreads();
  if constexpr (sizeof...(Rs) > 0) return lds_dft_c<N, COLS, NT, SWZ, Ns * R0, Rs...>(a, om);
  else return a;
}

template <int N1>
struct DctRadices1;
template <>
struct DctRadices1<100> {
  template <int COLS, int NT>
  __device__ static double2* run(double2* a, const double2* om) {
    return lds_dft_c<100, COLS, NT, false, 1, 4, 5, 5>(a, om);
  }
};
template <int N2>
struct DctRadices2;
template <>
struct DctRadices2<120> {
  template <int COLS, int NT, bool SWZ = false>
  __device__ static double2* run(double2* a, const double2* om) {
    return lds_dft_c<120, COLS, NT, SWZ, 1, 4, 2, 3, 5>(a, om);
  }
};

template <int N1, int N2, int COLS>
__global__ __launch_bounds__(256) void frames_dft1_c_kernel(DevConsts c, const void* __restrict__ pcm, int pcm_kind,
                                                            const int16_t* __restrict__ noise,
                                                            const FrameDesc* __restrict__ frames,
                                                            const double2* __restrict__ om1,
                                                            double2* __restrict__ z, int nframes) {
  constexpr int NT = 256;
  __shared__ double2 bufA[N1 * COLS], oms[N1], twb[N2];
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
  const double2* res = DctRadices1<N1>::template run<COLS, NT>(bufA, oms);
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
  __shared__ double2 bufA[N2 * COLS], oms[N2];
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
  const double2* res = DctRadices2<N2>::template run<COLS, NT, SWZ>(bufA, oms);
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
// 3. The recipes' DCT (N = 24000) in ONE kernel per frame: the packed length-M = 12000 complex FFT
//    as three in-register passes M = A x B x C = 20 x 24 x 25, q = BC q1 + C q2 + q3,
//    k = k1 + A k2a + AB k2b:
//      pass 1, thread (q2, q3): DFT_A over q1 of the gathered samples, twiddle W_M^{k1 (C q2 + q3)}
//      pass 2, thread (k1, q3): DFT_B over q2, twiddle W_BC^{k2a q3}
//      pass 3, thread (k1, k2a): DFT_C over q3 -> X[k]; real-FFT unpack with X[M - k] and the
//              Makhoul post-twiddle -> D[k], D[k + M]
//    The 12000 values stay in registers (one task per thread and pass); between passes they move
//    through a 12000-double LDS image, real parts first, then imaginary parts (96 KB instead of 192).
//    Pass-3 tasks are laid out so the task holding X[M - k] sits in the adjacent lane (lane ^ 1): the
//    unpack takes it by DPP quad_perm.  No Z intermediate in HBM: the frame is read once and D written
//    once (the four-step pair above moves Z = 384 KB per frame through HBM).
//    One workgroup per two frames, as straight-line code (frame 2 b, then 2 b + 1): the twiddle and
//    unpack tables are staged in LDS once for both.  The samples come by the single-bounce reflect fast
//    gather (int16 PCM straight into registers, noise-mixed frames included, the window pre-permuted into
//    16-byte pieces, dct1_fast); the diff filter, fp64 input and multi-bounce padding take the LDS-staged
//    general gather.  (No cross-frame prefetch: a persistent loop or a prefetch of the second frame spills,
//    see kDctFramesPerBlock.)
//    The LDS images are padded (exchange 1: k1 stride 601 = 25 mod 32; exchange 2: k2a stride 529) and
//    the twiddle tables laid out [k1][t mod 16] x [k1][t div 16] and [k2a][q3], so the lanes of an LDS
//    instruction spread over the banks (benchmarks/dct_lds_model.py).
// -----------------------------------------------------------------------------------------
namespace dct1 {
constexpr int kA = 20, kB = 24, kC = 25, kM = kA * kB * kC, kBC = kB * kC, kAC = kA * kC, kAB = kA * kB;
constexpr int kThreads = 640;  // >= max(BC, AC, AB) tasks
static_assert(kM == 12000 && kBC <= kThreads && kAC <= kThreads && kAB <= kThreads, "task layout");
constexpr int kT2N = (kBC + 15) / 16;  // t div 16 < 38
// table offsets (double2) in c.dct1_tw / LDS: T1[k1][u] = W_M^{k1 u} (u < 16), T2[k1][v] = W_M^{16 k1 v}
// (v < 38), T3[k2a][q3] = W_BC^{k2a q3}, rtw[lo], rtw[AB h], post[lo], post[AB h]  (lo < AB, h < C)
constexpr int kT1 = 0, kT2 = kT1 + kA * 16, kT3 = kT2 + kA * kT2N, kRtLo = kT3 + kB * kC, kRtHi = kRtLo + kAB,
              kPwLo = kRtHi + kC, kPwHi = kPwLo + kAB, kTabs = kPwHi + kC;
// exchange images (doubles): [k1][n2] with k1 stride kQ1, [k2a][k1][q3] with k2a stride kP2
constexpr int kQ1 = 601, kP2 = 529;
constexpr int kXch0 = kA * kQ1 > (kB - 1) * kP2 + kAC ? kA * kQ1 : (kB - 1) * kP2 + kAC;
constexpr int kXch = ((kXch0 > kM ? kXch0 : kM) + 15) / 16 * 16;

// cos / sin of 2 pi e / n, evaluated by the compiler (Taylor series on [0, pi/4] after an exact
// integer quadrant / octant reduction); used for the in-register radix twiddles
constexpr double kHalfPi = 1.57079632679489661923;
constexpr double tcos(double x) {
  double x2 = x * x, term = 1.0, s = 1.0;
  for (int i = 1; i < 16; ++i) { term *= -x2 / ((2.0 * i - 1.0) * (2.0 * i)); s += term; }
  return s;
}
constexpr double tsin(double x) {
  double x2 = x * x, term = x, s = x;
  for (int i = 1; i < 16; ++i) { term *= -x2 / ((2.0 * i) * (2.0 * i + 1.0)); s += term; }
  return s;
}
constexpr double qcos(long r, long n) {  // cos(pi/2 * r / n), 0 <= r <= n
  return 2 * r <= n ? tcos(kHalfPi * ((double)r / (double)n)) : tsin(kHalfPi * ((double)(n - r) / (double)n));
}
constexpr double root_re(long e, long n) {  // cos(2 pi e / n)
  e = ((e % n) + n) % n;
  const long q = (4 * e) / n, r = 4 * e - q * n;
  const double cr = qcos(r, n), sr = qcos(n - r, n);
  return q == 0 ? cr : q == 1 ? -sr : q == 2 ? -cr : sr;
}
constexpr double root_im(long e, long n) {  // -sin(2 pi e / n): forward-DFT root W_n^e
  e = ((e % n) + n) % n;
  const long q = (4 * e) / n, r = 4 * e - q * n;
  const double cr = qcos(r, n), sr = qcos(n - r, n);
  return -(q == 0 ? sr : q == 1 ? cr : q == 2 ? -sr : -cr);
}
template <int N>
struct Roots {
  double re[N], im[N];
  constexpr Roots() : re(), im() {
    for (int e = 0; e < N; ++e) { re[e] = root_re(e, N); im[e] = root_im(e, N); }
  }
};

template <int N>
__device__ __forceinline__ void rdft(double2 (&v)[N]);

// N = P Q: n = Q p + q, k = kp + P kq; P-point DFTs over p, twiddle W_N^{q kp}, Q-point DFTs over q
template <int P, int Q>
__device__ __forceinline__ void rdft_pq(double2 (&v)[P * Q]) {
  constexpr int N = P * Q;
  constexpr Roots<N> W{};
  double2 t[N];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    double2 w[P];
#pragma unroll
    for (int p = 0; p < P; ++p) w[p] = v[Q * p + q];
    rdft<P>(w);
#pragma unroll
    for (int kp = 0; kp < P; ++kp) {
      const int e = (q * kp) % N;
      t[q * P + kp] = e == 0 ? w[kp] : cmul(w[kp], make_double2(W.re[e], W.im[e]));
    }
  }
#pragma unroll
  for (int kp = 0; kp < P; ++kp) {
    double2 w[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) w[q] = t[q * P + kp];
    rdft<Q>(w);
#pragma unroll
    for (int kq = 0; kq < Q; ++kq) v[kp + P * kq] = w[kq];
  }
}

template <int N>
__device__ __forceinline__ void rdft(double2 (&v)[N]) {
  if constexpr (N == 2 || N == 3 || N == 4 || N == 5) bfly_c<N>(v);
  else if constexpr (N == 6) rdft_pq<2, 3>(v);
  else if constexpr (N == 20) rdft_pq<4, 5>(v);
  else if constexpr (N == 24) rdft_pq<4, 6>(v);
  else if constexpr (N == 25) rdft_pq<5, 5>(v);
  else static_assert(N == 2, "radix not instantiated");
}

__device__ __forceinline__ double2 swap_pair(double2 v) {  // value of lane ^ 1 (DPP quad_perm [1,0,3,2])
  return make_double2(dpp_f64<0xB1>(v.x), dpp_f64<0xB1>(v.y));
}

// pass-3 task of lane t (< AB): (k1, k2a) and its pairing mode (0: partner in lane ^ 1,
// 1: X[M - k] is its own register (C - k2b) mod C, 2: its own register C - 1 - k2b)
__device__ __forceinline__ void pass3_task(int t, int& k1, int& k2a, int& mode) {
  const int p = t >> 1, s = t & 1;
  mode = 0;
  if (p < 9 * kB) {                 // k1 in [1, 10) with (20 - k1, 23 - k2a)
    const int a = 1 + p % 9, b = p / 9;
    k1 = s ? kA - a : a;
    k2a = s ? kB - 1 - b : b;
  } else if (p < 9 * kB + kB / 2) {  // k1 = 10 with (10, 23 - k2a)
    const int b = p - 9 * kB;
    k1 = kA / 2;
    k2a = s ? kB - 1 - b : b;
  } else if (p < 9 * kB + kB - 1) {  // k1 = 0: (0, k2a) with (0, 24 - k2a), k2a in [1, 12)
    const int b = p - (9 * kB + kB / 2) + 1;
    k1 = 0;
    k2a = s ? kB - b : b;
  } else {                           // (0, 0) and (0, 12): their own partners
    k1 = 0;
    k2a = s ? kB / 2 : 0;
    mode = s ? 2 : 1;
  }
}
}  // namespace dct1

// Frames of the fast gather: int16 PCM (noise-mixed or not; not the diff filter) whose reflect padding
// (numpy 'reflect', features.py:146) is at most one bounce, sample u -> -u below 0 and 2(T-1) - u from T on
// (every frame of an utterance longer than the half window; the others take the general gather).
__device__ __forceinline__ bool dct1_fast(const DevConsts& c, const FrameDesc& fd, int pcm_kind) {
  const int64_t t0 = (int64_t)fd.k * c.hop - c.ext;
  return pcm_kind == 0 && fd.T >= 2 && t0 >= -(fd.T - 1) && t0 + 2 * dct1::kM - 1 <= 2 * (fd.T - 1);
}

// Two frames per workgroup (f = 2 b, 2 b + 1), as straight-line code: the tables are staged once per two
// frames.  (A persistent loop over frames spills: the register allocator keeps ~60 more registers live
// around the loop's back edge than through the same code twice; so does a prefetch of the second frame's
// gather into registers during the first frame, at 640 threads = 168 VGPRs.)
constexpr int kDctFramesPerBlock = 2;

__global__ __launch_bounds__(dct1::kThreads) void dct_frame_kernel(DevConsts c, const void* __restrict__ pcm,
                                                                   int pcm_kind, const int16_t* __restrict__ noise,
                                                                   const FrameDesc* __restrict__ frames,
                                                                   const double* __restrict__ dense_rows,
                                                                   int nframes, double scale2,
                                                                   double* __restrict__ dct) {
  using namespace dct1;
  __shared__ __attribute__((aligned(16))) double xch[kXch];
  __shared__ double2 tab[kTabs + kC];  // tables + the (0, 0) task's X (pass 3)
  const int t = threadIdx.x;
  constexpr int N = 2 * kM;
  const double2* hwin = c.dct1_tw + kTabs;  // the window in Makhoul order (dct_frame_tables)

  // the fast gather: thread n2 = C q2 + q3 takes the int16 pair (x[m0], x[m1]) of the packed samples
  // z[BC q1 + n2] = v[2q] + i v[2q+1] (v[2q] = x[4q], v[2q+1] = x[4q+2] in the first half, mirrored
  // (x[2N-1-4q], x[2N-3-4q]) after; frame positions reflected into the utterance) into one register (two
  // 16-bit loads), and the window pair (w[m0], w[m1]) (one coalesced 16-byte load)
  // (two int16 per register by 16-bit loads into the halves would halve the registers of a prefetch, but
  // gfx950 runs with SRAM ECC, where a D16 load does not preserve the other half of its register)
  auto load_samples = [&](int (&pk)[2 * kA], int fi) {
    const FrameDesc fd = frames[fi];
    const int16_t* xs = (const int16_t*)pcm + fd.pcm_off;  // the utterance
    const int t0 = (int)((int64_t)fd.k * c.hop - c.ext), T = fd.T;
#pragma unroll
    for (int q1 = 0; q1 < kA; ++q1) {
      const int q = kBC * q1 + t;
      int u0 = t0 + (4 * q1 < kA * 2 ? 4 * q : 2 * N - 1 - 4 * q);
      int u1 = t0 + (4 * q1 < kA * 2 ? 4 * q + 2 : 2 * N - 3 - 4 * q);
      u0 = u0 < 0 ? -u0 : (u0 >= T ? 2 * (T - 1) - u0 : u0);
      u1 = u1 < 0 ? -u1 : (u1 >= T ? 2 * (T - 1) - u1 : u1);
      FDLP_CHECK(u0 >= 0 && u0 < T && u1 >= 0 && u1 < T);
      pk[2 * q1] = xs[u0];
      pk[2 * q1 + 1] = xs[u1];
    }
  };
  auto load_window = [&](double2 (&wv)[kA]) {
#pragma unroll
    for (int q1 = 0; q1 < kA; ++q1) wv[q1] = hwin[kBC * q1 + t];
  };
  // noise-mixed frames (features.py:31, sig + alp * ns in fp64 without contraction, as makhoul_sample):
  // y1 holds the window; the samples and the noise at the same reflected positions arrive in two halves
  // (80 int registers for all of them at once would not fit next to y1)
  auto load_mixed = [&](double2 (&y)[kA], const FrameDesc& fd) {
    const int16_t* xs = (const int16_t*)pcm + fd.pcm_off;
    const int16_t* ns = noise + fd.noise_off;
    const int t0 = (int)((int64_t)fd.k * c.hop - c.ext), T = fd.T;
    constexpr int kHalf = kA / 2;
#pragma unroll
    for (int h = 0; h < kA; h += kHalf) {
      int px[2 * kHalf], pn[2 * kHalf];
#pragma unroll
      for (int q1 = h; q1 < h + kHalf; ++q1) {
        const int q = kBC * q1 + t;
        int u0 = t0 + (4 * q1 < kA * 2 ? 4 * q : 2 * N - 1 - 4 * q);
        int u1 = t0 + (4 * q1 < kA * 2 ? 4 * q + 2 : 2 * N - 3 - 4 * q);
        u0 = u0 < 0 ? -u0 : (u0 >= T ? 2 * (T - 1) - u0 : u0);
        u1 = u1 < 0 ? -u1 : (u1 >= T ? 2 * (T - 1) - u1 : u1);
        FDLP_CHECK(u0 >= 0 && u0 < T && u1 >= 0 && u1 < T);
        px[2 * (q1 - h)] = xs[u0];
        px[2 * (q1 - h) + 1] = xs[u1];
        pn[2 * (q1 - h)] = ns[u0];
        pn[2 * (q1 - h) + 1] = ns[u1];
      }
#pragma unroll
      for (int q1 = h; q1 < h + kHalf; ++q1) {
        const double s0 = __dadd_rn((double)px[2 * (q1 - h)], __dmul_rn(fd.alpha, (double)pn[2 * (q1 - h)]));
        const double s1 = __dadd_rn((double)px[2 * (q1 - h) + 1], __dmul_rn(fd.alpha, (double)pn[2 * (q1 - h) + 1]));
        y[q1].x = __dmul_rn(s0, y[q1].x);
        y[q1].y = __dmul_rn(s1, y[q1].y);
      }
    }
  };

  const int f0 = kDctFramesPerBlock * (int)blockIdx.x;
  for (int q = t; q < kTabs; q += kThreads) tab[q] = c.dct1_tw[q];
  __syncthreads();  // tables

  auto frame = [&](const int f) {
    FDLP_CHECK(f >= 0 && f < nframes);
    const bool fast = !dense_rows && dct1_fast(c, frames[f], pcm_kind);
    // ---- pass 1: thread n2 = C q2 + q3 holds z[BC q1 + n2] (Makhoul order) ----
    double2 y1[kA];
    if (fast) {
      if (t < kBC) {
        const FrameDesc fd = frames[f];
        if (fd.noise_off < 0) {
          int pk[2 * kA];
          load_samples(pk, f);
          load_window(y1);
#pragma unroll
          for (int q1 = 0; q1 < kA; ++q1) {
            y1[q1].x = __dmul_rn((double)pk[2 * q1], y1[q1].x);
            y1[q1].y = __dmul_rn((double)pk[2 * q1 + 1], y1[q1].y);
          }
        } else {
          load_window(y1);
          load_mixed(y1, fd);
        }
      }
    } else {
      // general frames (multi-bounce reflect padding, the diff filter, fp64 input, dense rows):
      // the samples are staged through xch by a rolled loop (the general gather is too large to unroll 40x),
      // real parts then imaginary parts; the branch is uniform over the workgroup
      FrameDesc fd;
      if (!dense_rows) fd = frames[f];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        for (int q = t; q < kM; q += kThreads) xch[q] = makhoul_sample(c, fd, 2 * q + h, f, pcm, pcm_kind, noise, dense_rows);
        __syncthreads();
        if (t < kBC) {
#pragma unroll
          for (int q1 = 0; q1 < kA; ++q1) {
            const double v = xch[kBC * q1 + t];
            if (h) y1[q1].y = v; else y1[q1].x = v;
          }
        }
        __syncthreads();
      }
    }
    if (t < kBC) {
      rdft<kA>(y1);
#pragma unroll
      for (int k1 = 1; k1 < kA; ++k1)  // W_M^{k1 n2} = W_M^{k1 (n2 mod 16)} W_M^{16 k1 (n2 div 16)}
        y1[k1] = cmul(y1[k1], cmul(tab[kT1 + 16 * k1 + (t & 15)], tab[kT2 + kT2N * k1 + (t >> 4)]));
    }
    // ---- exchange 1: [k1][n2] -> thread (k1, q3) reads q2 ----
    const int k1b = t / kC, q3 = t - kC * (t / kC);
    double2 y2[kB];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (t < kBC) {
#pragma unroll
        for (int k1 = 0; k1 < kA; ++k1) xch[k1 * kQ1 + t] = h ? y1[k1].y : y1[k1].x;
      }
      __syncthreads();
      if (t < kAC) {
#pragma unroll
        for (int q2 = 0; q2 < kB; ++q2) {
          const double v = xch[k1b * kQ1 + kC * q2 + q3];
          if (h) y2[q2].y = v; else y2[q2].x = v;
        }
      }
      __syncthreads();
    }
    // ---- pass 2: DFT_B over q2, twiddle W_BC^{k2a q3}; exchange 2: [k2a][k1][q3] ----
    if (t < kAC) {
      rdft<kB>(y2);
#pragma unroll
      for (int k2a = 1; k2a < kB; ++k2a) y2[k2a] = cmul(y2[k2a], tab[kT3 + kC * k2a + q3]);
    }
    int k1, k2a, mode;
    dct1::pass3_task(t < kAB ? t : 0, k1, k2a, mode);
    double2 y3[kC];
    const int a3 = k2a * kP2 + k1 * kC;
    FDLP_CHECK(a3 >= 0 && a3 + kC <= kXch && k1 < kA && k2a < kB);
    if (t < kAC) {
#pragma unroll
      for (int j = 0; j < kB; ++j) xch[j * kP2 + t] = y2[j].x;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kC; ++j) y3[j].x = xch[a3 + j];
    __syncthreads();
    if (t < kAC) {
#pragma unroll
      for (int j = 0; j < kB; ++j) xch[j * kP2 + t] = y2[j].y;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kC; ++j) y3[j].y = xch[a3 + j];
    // ---- pass 3: DFT_C over q3 -> X[k1 + A k2a + AB k2b]; unpack with X[M - k] ----
    // D leaves through LDS: the lanes' D[k] (k = lo + AB j: 8-byte pieces scattered over the row, 1.44x
    // the row's bytes in partial-line writes, r03e PMC) are staged in xch, then every thread of the
    // workgroup writes contiguous 16-byte pieces of the row; first D[0, M), then D[M, 2M) (held in
    // registers meanwhile).  The waves without pass-3 tasks stay for the barriers and the row writes.
    const bool task3 = t < kAB;
    if (task3) rdft<kC>(y3);
    const int lo = k1 + kA * k2a;
    FDLP_CHECK(lo >= 0 && lo < kAB);
    double2 rl = make_double2(0.0, 0.0), pl = rl;
    if (task3) {
      rl = tab[kRtLo + lo];
      pl = tab[kPwLo + lo];
    }
    double* drow = dct + (int64_t)f * N;
    double dhi[kC];  // D[k + M] of the lane's k = lo + AB j
#pragma unroll
    for (int j = 0; j < kC; ++j) dhi[j] = 0.0;
    // the one lane of task (0, 0) pairs X_k with its own X_{M-k} (register (C - j) mod C): it parks its X
    // in LDS, and 25 lanes of an otherwise idle wave (t = 512 ..) emit one output pair each (done by that
    // lane alone, its 25 outputs ran after everyone else's while the workgroup waited at the barrier)
    if (task3 && mode == 1) {
#pragma unroll
      for (int j = 0; j < kC; ++j) tab[kTabs + j] = y3[j];
    }
    const int hj = t - 8 * 64;
    const bool helper = hj >= 0 && hj < kC;
    static_assert(kThreads >= 8 * 64 + kC && kAB <= 8 * 64, "helper lanes of task (0, 0)");
    __syncthreads();  // every lane's pass-3 reads of xch are done; the (0, 0) values are parked
    // D[k], D[k + M] from V = X_k and W = X_{M-k} (E / O split of the packed FFT, Makhoul post-twiddle)
    auto emit_pair = [&](int j, double2 V, double2 W, double2 rlo, double2 plo, double& d1, double& d2) {
      const double2 E = make_double2(0.5 * (V.x + W.x), 0.5 * (V.y - W.y));
      const double2 O = make_double2(0.5 * (V.y + W.y), -0.5 * (V.x - W.x));
      const double2 rt = cmul(rlo, tab[kRtHi + j]);
      const double2 w1 = cmul(plo, tab[kPwHi + j]);
      constexpr double hr = 0.70710678118654752440;  // post[k + M] = post[k] e^{-i pi / 4}
      const double2 w2 = make_double2(hr * (w1.x + w1.y), hr * (w1.y - w1.x));
      const double2 tt = cmul(rt, O);
      const double2 V1 = make_double2(E.x + tt.x, E.y + tt.y);
      const double2 V2 = make_double2(E.x - tt.x, E.y - tt.y);
      d1 = (w1.x * V1.x - w1.y * V1.y) * scale2;
      d2 = (w2.x * V2.x - w2.y * V2.y) * scale2;
    };
    auto emit = [&](int j, double2 V, double2 W) {
      double d1, d2;
      emit_pair(j, V, W, rl, pl, d1, d2);
      xch[lo + kAB * j] = d1;
      dhi[j] = d2;
    };
    // pairs in lanes (2i, 2i+1) and the self-paired (0, 12) (mode 2): X_{M-k} is register C-1-j of the
    // partner lane, or of the lane itself
    const bool act = task3 && mode != 1;
    // j and C-1-j together, so both registers are dead after the pair (C odd: the middle one alone)
#pragma unroll
    for (int j = 0; j < (kC + 1) / 2; ++j) {
      const int jm = kC - 1 - j;
      const double2 a = y3[j], b = y3[jm];
      const double2 sa = swap_pair(a), sb = swap_pair(b);  // every lane of the wave takes part in the DPP
      if (act) {
        emit(j, a, mode == 2 ? b : sb);
        if (jm != j) emit(jm, b, mode == 2 ? a : sa);
      }
    }
    double dh_help = 0.0;
    if (helper) {  // task (0, 0), output pair hj: X_{AB hj} and X_{M - AB hj} = X_{AB ((C - hj) mod C)}
      double d1;
      emit_pair(hj, tab[kTabs + hj], tab[kTabs + (kC - hj) % kC], tab[kRtLo], tab[kPwLo], d1, dh_help);
      xch[kAB * hj] = d1;
    }
    // row writes: 16-byte pieces, consecutive threads on consecutive pieces (M / 2 = 6000 per half)
    double2* drow2 = reinterpret_cast<double2*>(drow);
    const double2* xch2 = reinterpret_cast<const double2*>(xch);
    __syncthreads();
    for (int q = t; q < kM / 2; q += kThreads) drow2[q] = xch2[q];
    __syncthreads();
    if (act) {
#pragma unroll
      for (int j = 0; j < kC; ++j) xch[lo + kAB * j] = dhi[j];
    }
    if (helper) xch[kAB * hj] = dh_help;
    __syncthreads();
    for (int q = t; q < kM / 2; q += kThreads) drow2[kM / 2 + q] = xch2[q];
  };

  frame(f0);
  if (f0 + 1 < nframes) {
    __syncthreads();  // the row reads of xch before the second frame's exchanges
    frame(f0 + 1);
  }
}

// host tables of dct_frame_kernel (double2 [dct1::kTabs]); empty unless N = 24000 with the real FFT
std::vector<double2> dct_frame_tables(int N, const std::vector<double>& window) {
  using namespace dct1;
  std::vector<double2> tab;
  if (N != 2 * kM || (int)window.size() != N) return tab;
  tab.resize(kTabs + kM);
  // after the tables: the analysis window in the fast gather's order, (w[m0(q)], w[m1(q)]) for the packed
  // sample q = v[2q] + i v[2q+1] (v = the Makhoul reorder), so pass 1 reads it coalesced
  for (int q = 0; q < kM; ++q) {
    const bool lo = q < kM / 2;
    tab[kTabs + q] = make_double2(window[lo ? 4 * q : 2 * N - 1 - 4 * q], window[lo ? 4 * q + 2 : 2 * N - 3 - 4 * q]);
  }
  const long double PI = 3.141592653589793238462643383279502884L;
  auto root = [&](long long e, long long n) {  // W_n^e = exp(-2 pi i e / n)
    const long double ang = -2.0L * PI * (long double)(e % n) / (long double)n;
    return make_double2((double)cosl(ang), (double)sinl(ang));
  };
  auto post = [&](long long k) {  // exp(-i pi k / (2N))
    const long double ang = -PI * (long double)k / (2.0L * (long double)N);
    return make_double2((double)cosl(ang), (double)sinl(ang));
  };
  for (int k1 = 0; k1 < kA; ++k1) {
    for (int u = 0; u < 16; ++u) tab[kT1 + 16 * k1 + u] = root((long long)k1 * u, kM);
    for (int v = 0; v < kT2N; ++v) tab[kT2 + kT2N * k1 + v] = root(16LL * k1 * v, kM);
  }
  for (int k2a = 0; k2a < kB; ++k2a)
    for (int q3 = 0; q3 < kC; ++q3) tab[kT3 + kC * k2a + q3] = root((long long)k2a * q3, kBC);
  for (int lo = 0; lo < kAB; ++lo) { tab[kRtLo + lo] = root(lo, N); tab[kPwLo + lo] = post(lo); }
  for (int h = 0; h < kC; ++h) { tab[kRtHi + h] = root((long long)kAB * h, N); tab[kPwHi + h] = post((long long)kAB * h); }
  return tab;
}

hipError_t launch_dct_frame(const DevConsts& c, const void* pcm, int pcm_kind, const int16_t* noise,
                            const FrameDesc* frames, const double* dense_rows, int nframes, double* dct,
                            hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  if (!c.dct1_tw || c.N != 2 * dct1::kM || !c.real_fft || c.natural) return hipErrorInvalidValue;
  const double sc2 = 2.0 / sqrt((double)(2 * c.N));
  const int grid = (nframes + kDctFramesPerBlock - 1) / kDctFramesPerBlock;
  hipLaunchKernelGGL(dct_frame_kernel, dim3(grid), dim3(dct1::kThreads), 0, s, c, pcm, pcm_kind, noise, frames,
                     dense_rows, nframes, sc2, dct);
  (void)kmark(kKDctFrame, s);
  return hipGetLastError();
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
  if (c.real_fft && d1.n == 100 && N2 == 120 && !dense_rows) {  // recipes: N = 24000
    hipLaunchKernelGGL((frames_dft1_c_kernel<100, 120, kDftCols>), dim3(xcd_grid(grid.x * nframes)), dim3(256), 0, s, c,
                       pcm, pcm_kind, noise, frames, om1, z, nframes);
    (void)kmark(kKFramesDft1, s);
    return hipGetLastError();
  }
  if (c.real_fft) {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)frames_dft1_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(frames_dft1_kernel<true>, grid, dim3(256), lds, s, c, d1, N2, pcm, pcm_kind, noise,
                       frames, dense_rows, om1, z);
    (void)kmark(kKFramesDft1, s);
  } else {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)frames_dft1_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(frames_dft1_kernel<false>, grid, dim3(256), lds, s, c, d1, N2, pcm, pcm_kind, noise,
                       frames, dense_rows, om1, z);
    (void)kmark(kKFramesDft1, s);
  }
  return hipGetLastError();
}

hipError_t launch_dft2_dct(const DevConsts& c, const DftPlan& d2, int N1, const double2* z,
                           int nframes, double* dct, const double2* om2, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  size_t lds = sizeof(double2) * (2 * d2.n * kDftCols + d2.n);
  const double div = sqrt((double)(2 * c.N));
  if (c.real_fft && N1 == 100 && d2.n == 120) {  // recipes: N = 24000
    dim3 grid((N1 / 2 + 1 + kDftCols / 2 - 1) / (kDftCols / 2), nframes);
    const dim3 g1(xcd_grid(grid.x * nframes));
    const double sc2 = 2.0 / div;
    hipLaunchKernelGGL((dft2_dct_c_kernel<100, 120, kDftCols, true>), g1, dim3(256), 0, s, c, z, om2, sc2, dct, nframes);
    (void)kmark(kKDft2Dct, s);
    return hipGetLastError();
  }
  if (c.real_fft) {
    dim3 grid((N1 / 2 + 1 + kDftCols / 2 - 1) / (kDftCols / 2), nframes);  // row pairs (k1, N1-k1)
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)dft2_dct_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(dft2_dct_kernel<true>, grid, dim3(256), lds, s, c, d2, N1, z, om2, div, dct);
    (void)kmark(kKDft2Dct, s);
  } else {
    dim3 grid((N1 + kDftCols - 1) / kDftCols, nframes);
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)dft2_dct_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(dft2_dct_kernel<false>, grid, dim3(256), lds, s, c, d2, N1, z, om2, div, dct);
    (void)kmark(kKDft2Dct, s);
  }
  return hipGetLastError();
}

hipError_t checks_dct(unsigned int* v, bool reset) { return fdlp_checks_local(v, reset); }

}  // namespace fdlp
