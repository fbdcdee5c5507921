// fdlp_lpc.hip -- gfx950 kernels of the LPC stage:
//   durbin8_kernel          : Levinson-Durbin (features.py:226-228) in lattice form, 8 lanes per item
//   lpc_env_lattice_kernel  : LPC cepstrum (features.py:233-246) + modulation weights + envelope
//                             exp(Re DFT_{2*fd*fr}(c .* w))[0:kk] * hann/hamm (computeFDLPSpectrogram.py:194-205)
//   lpc_env_kernel          : the LDS Durbin + cepstrum + envelope (large p, and the cross-check path)
//   levinson_kernel / cepstrum_kernel : the per-stage entry points (fdlp_lpc_rows / fdlp_cepstrum_rows)
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include "fdlp_device.h"

namespace fdlp {

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

// ---- FFT envelope (env_nfft = 300 with Me = 300: REVERB) -----------------------------------------
// Re(fft(c', 300))[t] (computeFDLPSpectrogram.py:201-205, scipy's own FFT route) from a 150-point complex
// FFT of z[q] = c'_{2q} + i c'_{2q+1} -- the weighted cepstrum buffer read as double2, so no packing --
// then the real-FFT unpacking Re X_t = (Z_t + conj Z_{-t}).x / 2 + Re(w^t (Z_t - conj Z_{-t}) / 2i),
// w = e^{-2 pi i / 300}.  One 16-lane row per item, Stockham stages in place in LDS (all butterflies of
// a stage read into registers, then written back; the row's LDS ops complete in order).  ~0.4k
// instructions per lane and item instead of the ~3k FMAs of the direct cosine sum.  Roots from the
// plan's cos(2 pi q / 300) table: w_150^e = cos(2 pi 2e/300) - i sin(.), sin x = cos(x - pi/2).
template <int N, int R, int Ns>
__device__ __forceinline__ void env_fft_stage(double2* buf, const double* __restrict__ cosT, int l) {
  constexpr int NB = N / R, IT = (NB + 15) / 16, TW0 = N / (Ns * R);
  double2 v[IT][R];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = l + 16 * it;
    if (j < NB) {
      const int k = j % Ns;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double2 x = buf[j + r * NB];
        if (r == 0 || Ns == 1) {
          v[it][r] = x;
        } else {
          const int e2 = 2 * TW0 * k * r;  // < 300
          const double2 w = make_double2(cosT[e2], -cosT[e2 >= 75 ? e2 - 75 : e2 + 225]);
          v[it][r] = cmul(x, w);
        }
      }
      bfly_c<R>(v[it]);
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = l + 16 * it;
    if (j < NB) {
      const int k = j % Ns, jq = j / Ns;
      const int idxD = jq * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) buf[idxD + r * Ns] = v[it][r];
    }
  }
  wave_lds_sync();
}

// env[t] = exp(Re X_t) * hann/hamm[t], t < 150, from the weighted cepstrum cw[0 .. 300) (16-B aligned),
// handed to emit(t, env[t]) (lane l: t = l + 16 it)
template <class Emit>
__device__ __forceinline__ void env_fft300(double* cw, const double* __restrict__ cosT,
                                           const double* __restrict__ win, int l, bool valid, Emit&& emit) {
  double2* z = reinterpret_cast<double2*>(cw);
  env_fft_stage<150, 2, 1>(z, cosT, l);
  env_fft_stage<150, 3, 2>(z, cosT, l);
  env_fft_stage<150, 5, 6>(z, cosT, l);
  env_fft_stage<150, 5, 30>(z, cosT, l);
  if (!valid) return;
#pragma unroll
  for (int it = 0; it < 10; ++it) {
    const int t = l + 16 * it;
    if (t < 150) {
      const int m = t == 0 ? 0 : 150 - t;
      const double2 Zt = z[t], Zm = z[m];
      const double c = cosT[t], s = cosT[t >= 75 ? t - 75 : t + 225];
      const double re = 0.5 * (Zt.x + Zm.x) + 0.5 * (c * (Zt.y + Zm.y) - s * (Zt.x - Zm.x));
      emit(t, exp(re) * win[2 * t]);
    }
  }
}

// ---- super-block cepstrum (CB < 0: any M, REVERB's 450) -----------------------------------------
// With d_n = n c_n the recursion of features.py:233-246 (alpha = -a) reads
//     d_n = -n a_n - sum_{1 <= k < n} d_k a_{n-k},      c_n = d_n / n  (n >= 1),  c_0 = log(sqrt(gg)).
// Blocks of 16 coefficients, lane l of the item's DPP row owning n = 16 b + l.  For lane l the vector
//     V_q[j] = a_{16 (q+1) + l - j}   (j < 16)
// multiplies the 16 d values of a finished block that lies q blocks behind the block being computed, and
// it does not depend on which block that is.  So a super-block of R consecutive blocks loads each V_q
// once and uses it for every block r of it (window block w = q - r): 4x fewer LDS reads than one window
// per block.  The in-block part is the unit lower-triangular Toeplitz system (I + T) d = y, T built from
// a_1 .. a_15; it is solved as d = H y, H = (I + T)^-1 = the lower Toeplitz matrix of h = the first 16
// terms of the impulse response of 1/a(z), computed once per item: 16 independent FMAs per block instead
// of a 16-step serial recurrence.

// acc[r] += kc[Q - r] (.) V_Q for the blocks r of the super-block whose window reaches V_Q (0 <= Q - r < W)
template <int W, int R, int Q, int J, int Rr>
__device__ __forceinline__ void sb_fma_r(double (&acc)[R][2], const double (&kc)[W], double v) {
  if constexpr (Rr < R) {
    if constexpr (Q - Rr >= 0 && Q - Rr < W) fmac_bcast<J>(acc[Rr][J & 1], kc[Q - Rr], v);
    sb_fma_r<W, R, Q, J, Rr + 1>(acc, kc, v);
  }
}
template <int W, int R, int Q, int J = 0>
__device__ __forceinline__ void sb_fma_q(double (&acc)[R][2], const double (&kc)[W], const double (&v)[16]) {
  if constexpr (J < 16) {
    sb_fma_r<W, R, Q, J, 0>(acc, kc, v[J]);
    sb_fma_q<W, R, Q, J + 1>(acc, kc, v);
  }
}

// The window phase of one super-block, V_Q .. V_{qmax-1}: V_Q was issued before this call (va), V_{Q+1}
// is issued before V_Q's FMAs (double buffer; the counted wait leaves those 16 in flight, LDS operations
// complete in order).  qmax (uniform) = the window blocks that reach a finished block (Q - r < s).
template <int W, int R, int Q>
__device__ __forceinline__ void sb_window(double (&acc)[R][2], const double (&kc)[W], double (&va)[16],
                                          double (&vb)[16], uint32_t addr, int qmax) {
  if constexpr (Q < W) {
    if (Q >= qmax) return;
    if constexpr (Q + 1 < W) {
      if (Q + 1 < qmax) {
        lds_load16<16 * (Q + 1) + 15>(vb, addr);
        lgkm_wait<15>();  // V_Q's 16 loads (and the first of V_{Q+1}'s) have landed (lgkmcnt holds <= 15)
      } else {
        lgkm_wait<0>();
      }
    } else {
      lgkm_wait<0>();
    }
    // the asm loads' results look ready to the compiler: tie them to the wait (a volatile asm that
    // "rewrites" them), so neither the FMAs nor a register copy can be scheduled above it
#pragma unroll
    for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(va[j]));
    sb_fma_q<W, R, Q>(acc, kc, va);
    sb_window<W, R, Q + 1>(acc, kc, vb, va, addr, qmax);
  }
}

// acc += kcnew[T0 - t] (.) V_t, t = 0 .. T0: the blocks of the current super-block before block T0 + 1
template <int R, int T0, int T = 0>
__device__ __forceinline__ void sb_local(double (&acc)[2], const double (&kcnew)[R], double (&va)[16],
                                         double (&vb)[16], uint32_t addr) {
  if constexpr (T <= T0) {
    if constexpr (T < T0) {
      lds_load16<16 * (T + 1) + 15>(vb, addr);
      lgkm_wait<15>();
    } else {
      lgkm_wait<0>();
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(va[j]));
    cep_fma16(acc[0], acc[1], acc[0], acc[1], kcnew[T0 - T], va);
    sb_local<R, T0, T + 1>(acc, kcnew, vb, va, addr);
  }
}

// d = H y for the block: lane l gets sum_m h_{l-m} y_m (y_m from lane m, Hrow[m] = h_{l-m}, 0 for m > l)
__device__ __forceinline__ double sb_solve(double y, const double (&Hrow)[16]) {
  double ym;
  asm volatile("v_mov_b64 %0, %1\n\ts_nop 1" : "=v"(ym) : "v"(y));  // DPP source: 2 wait states past its write
  double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
  fmac_bcast<0>(d0, ym, Hrow[0]);
  fmac_bcast<1>(d1, ym, Hrow[1]);
  fmac_bcast<2>(d2, ym, Hrow[2]);
  fmac_bcast<3>(d3, ym, Hrow[3]);
  fmac_bcast<4>(d0, ym, Hrow[4]);
  fmac_bcast<5>(d1, ym, Hrow[5]);
  fmac_bcast<6>(d2, ym, Hrow[6]);
  fmac_bcast<7>(d3, ym, Hrow[7]);
  fmac_bcast<8>(d0, ym, Hrow[8]);
  fmac_bcast<9>(d1, ym, Hrow[9]);
  fmac_bcast<10>(d2, ym, Hrow[10]);
  fmac_bcast<11>(d3, ym, Hrow[11]);
  fmac_bcast<12>(d0, ym, Hrow[12]);
  fmac_bcast<13>(d1, ym, Hrow[13]);
  fmac_bcast<14>(d2, ym, Hrow[14]);
  fmac_bcast<15>(d3, ym, Hrow[15]);
  return (d0 + d1) + (d2 + d3);
}

// Hrow[m] = h_{l-m} (0 for m > l) from hl = h_l: DPP row_shr:m with bound_ctrl (lanes l < m take 0)
template <int M0 = 1>
__device__ __forceinline__ void sb_hrow(double (&Hrow)[16], double hl) {
  if constexpr (M0 < 16) {
    Hrow[M0] = __builtin_amdgcn_update_dpp(0.0, hl, 0x110 + M0, 0xF, 0xF, true);
    sb_hrow<M0 + 1>(Hrow, hl);
  }
}

// h_1 .. h_15 of 1/a(z) (h_0 = 1, h_m = -sum_{k=1}^{m} a_k h_{m-k}): lane l ends with h_l
template <int M0 = 1>
__device__ __forceinline__ void sb_impulse(double& hl, double& t, const double* la, int l) {
  if constexpr (M0 < 16) {
    if (l == M0) hl = -t;
    const double hm = dpp_f64<0x150 + M0>(hl);  // row_newbcast:M0
    if (l > M0) t = fma(hm, la[l - M0], t);
    sb_impulse<M0 + 1>(hl, t, la, l);
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
// global memory one phase ahead).  Same recursion as the reference (features.py:226-228): both halves
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
constexpr int kD8Chains = 4;  // the next order's dot product in 4 chains (2: no difference, 1.13 vs 1.14 ms)
constexpr int kNewton = 1;    // Newton steps after v_rcp_f64 for 1/E: one (durbin4_kernel 0.693-0.711 ->
                              // 0.680-0.696 ms alternating, profiles/r04m_newton_ab.txt; per-item a within
                              // durbin8's accuracy against solve_toeplitz, test_durbin4_matches_durbin8)
template <int S>
__device__ __forceinline__ void c8_step(double (&A)[S], const double (&Bs)[S], double (&Bd)[S],
                                        const double (&R1)[S], double& part, double& E, bool first) {
  const double acc = sum8(part);  // r_k + sum_i a_i r_{k-i}
  double rE = __builtin_amdgcn_rcp(E);
#pragma unroll
  for (int it = 0; it < kNewton; ++it) rE = fma(rE, fma(-E, rE, 1.0), rE);
  const double kappa = -acc * rE;
  const double zs = __builtin_amdgcn_update_dpp(0.0, Bs[S - 1], 0x111, 0xF, 0xF, true);  // row_shr:1
  const double z0 = first ? 0.0 : zs;
  // the next order's dot product in D independent chains (the chain, not the issue, bounds small S)
  constexpr int D = kD8Chains;
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

// A (S per lane) -> sc -> An, Bn (S + 2 per lane).  B is the bitwise mirror of A: after order 8 S - 1,
// b_m = a_{8S-1-m} (both are fma(kappa, a_m, a_{k-m}) in c8_step), so B is read back mirrored from A's
// image instead of being written too; positions outside [0, 8 S) are zeros (a select, no zero pads).
// Only odd S occur (phases S = 1, 3, 5, ...): every lane stride of the image (S written, S + 2 read,
// -(S + 2) mirrored) is then odd, and with the item stride kItem = 8 mod 16 doubles the 32 lanes of a
// ds_read_b64 group (4 items x 8 lanes) and the 16 of a ds_write_b64 group hit distinct banks.
template <int S>
__device__ __forceinline__ void c8_relayout(const double (&A)[S], double (&An)[S + 2], double (&Bn)[S + 2],
                                            double* sc, int li) {
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j < S; ++j) sc[li * S + j] = A[j];
  wave_lds_sync();
  // positions outside [0, 8 S) are read unclamped and dropped by the select: m stays within
  // [-16, 8 (S + 2)) c [-16, 8 SL8), inside the item's LDS area (8 doubles of gap and r_{kR-8..} below sc).
  // Clamping them to sc[0] put those lanes on one bank beside the odd-stride lanes of the other items:
  // 1.15e7 bank-conflict cycles per launch (r03e PMC).
#pragma unroll
  for (int j = 0; j < S + 2; ++j) {
    const int m = li * (S + 2) + j;
    const double v = sc[m];
    An[j] = m < 8 * S ? v : 0.0;
  }
#pragma unroll
  for (int j = 0; j < S + 2; ++j) {
    const int m = 8 * S - 1 - li * (S + 2) - j;
    const double v = sc[m];
    Bn[j] = m >= 0 ? v : 0.0;
  }
}

// Orders [k0, k1) of phase S (capacity 8 S positions; phases S = 1, 3, 5, ... <= SL8, SL8 odd).
template <int SL8, int S>
__device__ __forceinline__ void c8_durbin(double (&A)[S], double (&B)[S], double (&R1)[S], double& part, double& E,
                                          const double* rl, double* sc, int p, int li, bool valid, double r0,
                                          double* ao, double* go, int astride) {
  static_assert(S % 2 == 1 && SL8 % 2 == 1, "odd phases only (conflict-free LDS strides)");
  const int k0 = S == 1 ? 1 : 8 * (S - 2);
  const int k1 = min(p + 1, 8 * S);
  const bool first = li == 0;
  constexpr int SN = S < SL8 ? S + 2 : S;
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
      double An[S + 2], Bn[S + 2];
      c8_relayout<S>(A, An, Bn, sc, li);
      c8_durbin<SL8, S + 2>(An, Bn, R1n, part, E, rl, sc, p, li, valid, r0, ao, go, astride);
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

// one wave per 8 items (p + 1 <= 8 SL8 <= astride, SL8 odd); a / gg: [items, astride] (zero past p) /
// [items].  The 8 items' r rows are staged in LDS first (one coalesced pass), so each phase's R1 is an LDS
// read, not a global load whose latency the short early phases cannot cover.  LDS per item (kItem
// doubles, = 8 mod 16 for conflict-free banks): r_1 .. r_{8 SL8}, then the relayout image (8 SL8) after
// an 8-double gap; 8 items = 19.5 KB at SL8 = 19, two waves per SIMD.
template <int SL8>
__global__ __launch_bounds__(64, 2) void durbin8_kernel(const double* __restrict__ r, int nlags, int p, int items,
                                                        double* __restrict__ a, double* __restrict__ gg, int astride) {
  constexpr int kR = 8 * SL8;
  constexpr int kItem = kR + 8 + 8 * SL8;
  static_assert(kItem % 16 == 8, "item stride must be 8 mod 16 doubles (bank-conflict-free image)");
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

// -----------------------------------------------------------------------------------------
// The same lattice Durbin with 4 lanes per item (a DPP quad is an item, 16 items per wave; the recipes'
// p = 150 and every p <= 4 SL4 - 2).  Per order a wave issues 3 S FMAs (A, B, the next order's dot
// product) and ~17 instructions of cross-lane work (the quad sum, kappa, the B shift, E and 1/E), so
// the cross-lane part is paid once per 16 items instead of 8: ~36 % fewer VALU instructions per item
// than durbin8_kernel at p = 150.  What makes it fit:
// * B is updated in place (slots in descending order: B[j-1] is still the previous order's when B[j]
//   and A[j] read it), so an order needs A, B and R1 only: 3 x 38 doubles at the last phase.
// * A phase S (S positions per lane, capacity 4 S) runs orders k <= 4 S - 2, so the last position
//   4 S - 1 of B is exactly 0 (b_m = a_{k-m}, m > k): the row_shr:1 of B's last slot then hands the next
//   item's first lane a 0 by itself (the quad boundaries are not row boundaries), no select.
// * 1/E for the next order (rcp + two Newton steps) is computed right after kappa, beside the order's
//   FMAs, so the serial part of an order is only the dot-product tail, the quad sum and kappa.
// * No r staging: R1 is re-laid out with A through the item's LDS image (R1 first, while B is already
//   dead), the 16 positions a phase adds come from global loads issued one phase ahead.  16 items x 156
//   doubles = 19.7 KB of LDS per wave, two waves per SIMD.
// Phases S = 1, 5, 9, ... (odd: the lane strides S and S + 4 with the item stride 156 = -4 mod 32 doubles
// put the 32 lanes of a ds_read_b64 group and the 16 of a ds_write_b64 group on distinct banks), then SL4
// = 38: the relayout into that last, even phase and its final A image put lanes li and li + 2 of an item
// on one bank (2-way), 304 extra cycles per wave, ~0.25 % of its time; no item stride avoids it
// (benchmarks/durbin4_lds_model.py), and an odd SL4 = 39 would cost registers and a larger image.
// Same recursion and the same kappa / E / 1/E arithmetic as c8_step (features.py:226-228); the order-k dot
// product is summed over 4 lane partials of 2 chains instead of 8 lanes of 4 chains.
// -----------------------------------------------------------------------------------------
__device__ __forceinline__ double sum4(double v) {  // over a DPP quad; every lane gets the same (bitwise) value
  v += dpp_f64<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);  // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ double rcp_newton(double E) {
  double rE = __builtin_amdgcn_rcp(E);
#pragma unroll
  for (int it = 0; it < kNewton; ++it) rE = fma(rE, fma(-E, rE, 1.0), rE);
  return rE;
}

// one chain for the next order's dot product: its FMA latency stays below the 3 FMAs a position issues
constexpr int kC4Chains = 1;
template <int S>
__device__ __forceinline__ void c4_step(double (&A)[S], double (&B)[S], const double (&R1)[S], double& part,
                                        double& E, double& rE) {
  const double acc = sum4(part);  // r_k + sum_i a_i r_{k-i}
  const double kappa = -acc * rE;
  // z B at slot 0: lane li - 1's last slot (row_shr:1; row edges take 0 from bound_ctrl, the other
  // quad edges the exact 0 of position 4 S - 1)
  const double z0 = __builtin_amdgcn_update_dpp(0.0, B[S - 1], 0x111, 0xF, 0xF, true);
  constexpr int D = kC4Chains;  // dot-product chains
  double pc[D];
#pragma unroll
  for (int d = 0; d < D; ++d) pc[d] = 0.0;
#pragma unroll
  for (int j = S - 1; j >= 0; --j) {
    const double zb = j == 0 ? z0 : B[j - 1];
    const double bn = fma(kappa, A[j], zb);
    A[j] = fma(kappa, zb, A[j]);
    B[j] = bn;
    pc[j % D] = fma(bn, R1[j], pc[j % D]);
  }
  if constexpr (D == 2) part = pc[0] + pc[1];
  else part = pc[0];
  E = fma(kappa, acc, E);  // E (1 - kappa^2) with kappa = -acc / E, one FMA
  rE = rcp_newton(E);
}

// Phases S = 1, 1 + kC4Step, ... (16 orders each), then SL4: a relayout every 16 orders (every 8 with
// step 2: 19 instead of 11 relayouts for p = 150, 1.8x the LDS instructions) for ~1 more padded slot
// per lane.  LDS doubles per item: the image of 4 SL4 positions, = 28 mod 32 (see above).
constexpr int kC4Step = 4;
__host__ __device__ constexpr int c4_item_stride(int SL4) {
  const int need = 4 * SL4;
  return need + ((28 - need % 32) + 32) % 32;
}
constexpr int kC4Guard = 24;  // doubles below item 0's image (the mirrored B reads reach index -4 kC4Step - 1)
// the phase that ends at order p holds it: p <= 4 S - 2 = cap - 2
__device__ __forceinline__ bool k_done_ok(int p, int cap) { return p <= cap - 2; }

// Orders [k0, min(p, 4 S - 2)] of phase S, then the next phase.  Returns (in cap) 4 S of the phase that
// ends at order p and leaves its A in img (positions < cap; exactly 0 past p), gg in g.
template <int SL4, int S>
__device__ __forceinline__ void c4_durbin(double (&A)[S], double (&B)[S], double (&R1)[S], double& part, double& E,
                                          double& rE, double* img, const double* rl1, int plim, int p, int li,
                                          double r0, int k0, int& cap, double& g) {
  const int k1 = min(p, 4 * S - 2);
  constexpr int SN = S + kC4Step <= SL4 ? S + kC4Step : SL4;
  constexpr int NA = SN > S ? SN - S : 1;  // positions per lane the next phase adds
  double rn[NA];  // R1 of the 4 NA positions the next phase adds: 4 S + li + 4 t (lanes on distinct banks)
#pragma unroll
  for (int t = 0; t < NA; ++t) rn[t] = 0.0;
  if constexpr (SN > S) {
    if (k1 < p) {
#pragma unroll
      for (int t = 0; t < NA; ++t)
        if (4 * S + 4 * t <= plim) rn[t] = rl1[4 * S + 4 * t];  // r_{m+1}, m = 4 S + li + 4 t <= p
    }
  }
  for (int k = k0; k <= k1; ++k) c4_step<S>(A, B, R1, part, E, rE);
  if constexpr (SN > S) {
    if (k1 < p) {
      // R1 first (B is dead: it is read back mirrored from A's image), then A
      double R1n[SN], An[SN], Bn[SN];
      wave_lds_sync();
      FDLP_CHECK(4 * SN <= c4_item_stride(SL4) && 4 * S + 4 * NA <= c4_item_stride(SL4));
#pragma unroll
      for (int j = 0; j < S; ++j) img[li * S + j] = R1[j];
#pragma unroll
      for (int t = 0; t < NA; ++t) img[4 * S + li + 4 * t] = rn[t];
      wave_lds_sync();
#pragma unroll
      for (int j = 0; j < SN; ++j) R1n[j] = img[li * SN + j];
      wave_lds_sync();
#pragma unroll
      for (int j = 0; j < S; ++j) img[li * S + j] = A[j];
#pragma unroll
      for (int t = 0; t < NA; ++t) img[4 * S + li + 4 * t] = 0.0;  // the staged R1 positions back to 0
      wave_lds_sync();
      // No selects: A past k1 = 4 S - 2 is exactly +0 in the image, [4 S, 4 SN) was just zeroed and
      // [4 SN, kItem) of every item is still the 0 of the kernel's first pass, so the An reads (< 4 SN) and
      // the mirrored Bn reads (b_m = a_{k1-m}, down to index -4 NA - 1, into the guard or the previous item's
      // [kItem - 4 NA - 1, kItem) c [4 SN, kItem)) see exact zeros wherever the recursion needs them.
      constexpr int k1c = 4 * S - 2;
      FDLP_CHECK(k1 == k1c);
#pragma unroll
      for (int j = 0; j < SN; ++j) An[j] = img[li * SN + j];
#pragma unroll
      for (int j = 0; j < SN; ++j) {
        FDLP_CHECK(k1c - li * SN - j >= -kC4Guard && k1c - li * SN - j < c4_item_stride(SL4));
        Bn[j] = img[k1c - li * SN - j];
      }
      c4_durbin<SL4, SN>(An, Bn, R1n, part, E, rE, img, rl1, plim, p, li, r0, k1 + 1, cap, g);
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
  g = r0 + sum4(q0 + q1);
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j < S; ++j) img[li * S + j] = A[j];
  cap = 4 * S;
}

// one wave per 16 items, p <= 4 SL4 - 2 <= astride; a / gg: [items, astride] (zero past p) / [items].
// The rows leave through the LDS images as coalesced 16-byte stores.
template <int SL4>
__global__ __launch_bounds__(64, 2) void durbin4_kernel(const double* __restrict__ r, int nlags, int p, int items,
                                                        double* __restrict__ a, double* __restrict__ gg, int astride) {
  constexpr int kItem = c4_item_stride(SL4);
  __shared__ double lds[kC4Guard + 16 * kItem];
  const int lane = threadIdx.x;
  const int li = lane & 3;
  const int ii = lane >> 2;
  const int item0 = blockIdx.x * 16;
  const int item = item0 + ii;
  const bool valid = item < items;
  const double* rrow = r + (int64_t)(valid ? item : 0) * nlags;
  double* img = lds + kC4Guard + ii * kItem;
  static_assert(4 * SL4 < kItem && kC4Guard >= 4 * kC4Step + 1, "zero margins of the select-free relayout");
  {  // every image and the guard start at +0 (c4_durbin's relayout reads them instead of selecting zeros)
    double2* z = reinterpret_cast<double2*>(lds);
    static_assert((kC4Guard + 16 * kItem) % 2 == 0, "");
    for (int q = lane; q < (kC4Guard + 16 * kItem) / 2; q += 64) z[q] = make_double2(0.0, 0.0);
  }
  const double r0 = valid ? rrow[0] : 1.0;
  double A[1] = {li == 0 ? 1.0 : 0.0}, B[1] = {li == 0 ? 1.0 : 0.0};
  double R1[1] = {valid && li <= p ? rrow[li + 1] : 0.0};
  double part = li == 0 ? R1[0] : 0.0;  // order 1: b^(0) . R1 = r_1
  double E = r0, rE = rcp_newton(r0);
  int cap = 0;
  double g = 0.0;
  // the lane's r_{li+1} and its limit: position m = 4 S + li + 4 t is loaded while 4 S + 4 t <= p - li
  const double* rl1 = rrow + 1 + li;
  const int plim = valid ? p - li : -1;
  c4_durbin<SL4, 1>(A, B, R1, part, E, rE, img, rl1, plim, p, li, r0, 1, cap, g);
  if (valid && li == 0) gg[item] = g;
  FDLP_CHECK(cap <= astride && cap <= c4_item_stride(SL4) && (cap & 1) == 0 && k_done_ok(p, cap));
  wave_lds_sync();
  constexpr int kRow = 4 * SL4;  // a full image row (p = 4 SL4 - 2, the recipes' 150)
  static_assert(kRow % 8 == 0 && kC4Guard % 2 == 0 && kItem % 2 == 0, "16-byte row pieces, 4 lanes per item");
  if (cap == kRow) {  // wave-uniform: each quad copies its own item with immediate offsets, then the zero tail
    FDLP_CHECK(astride >= kRow && (astride & 1) == 0);
    if (valid) {
      const double2* src = reinterpret_cast<const double2*>(img) + li;
      double2* dst = reinterpret_cast<double2*>(a + (int64_t)item * astride) + li;
#pragma unroll
      for (int j = 0; j < kRow / 8; ++j) dst[4 * j] = src[4 * j];
      for (int h = kRow / 2; h < (astride >> 1) - li; h += 4) dst[h] = make_double2(0.0, 0.0);
    }
    return;
  }
  const int half = astride >> 1;
  for (int i = 0; i < 16; ++i) {
    if (item0 + i >= items) break;
    const double* src = lds + kC4Guard + i * kItem;
    double2* dst = reinterpret_cast<double2*>(a + (int64_t)(item0 + i) * astride);
    for (int h = lane; h < half; h += 64) {
      const int m = 2 * h;
      double2 v = make_double2(0.0, 0.0);
      if (m < cap) v = *reinterpret_cast<const double2*>(src + m);  // cap is even: both or neither
      dst[h] = v;
    }
  }
}

// lpc_env with the lattice Durbin: persistent waves (grid-stride over groups of 4 items), r read
// straight into registers, LDS only for a (cepstrum) and c (envelope).  Same outputs as lpc_env_kernel.
constexpr int kEnvChunk = 5;  // envelope slots held in registers at a time
// CB > 0 (M <= 16 CB): the cepstrum's finished blocks take c_k from the registers of the lane that
// computed it (v_fmac_f64_dpp row_newbcast, the broadcast is the FMA's source modifier) instead of an
// LDS read per term: one LDS read (alpha_{n-k}) and one FMA per term instead of two reads, a multiply
// and an FMA.  CB < 0: the same over a sliding register window of the last SL + 1 finished blocks
// (any M; the terms with n - k > p are zero).  CB = 0: the LDS form for any M.
// DM: the Durbin phase.  1: the contiguous-chunk Durbin (contig_durbin, p outside durbin8_kernel's
// range); 2: none, a and gg come from durbin8_kernel (A.a_ext, A.gg_ext; default where it is instantiated).
constexpr int kDmContig = 1, kDmExt = 2;
// 1/n for a count n >= 1: v_rcp_f64 and two Newton steps, within an ulp of the quotient (the cepstrum's
// c_n = d_n / n once per coefficient; an IEEE division is ~10 instructions)
__device__ __forceinline__ double inv_count(int n) {
  const double x = (double)n;
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}
// waves per SIMD the lattice kernel is compiled for (register budget).  CB > 0: 4 (127 VGPRs and 12 spilled
// once per group: 0.62 ms per 327 680 items against 0.68 at 3 waves without spills, r04d); the super-block
// cepstrum (CB < 0) holds ~70 doubles of window, H rows and accumulators (spills at 3 waves per SIMD); its
// LDS allows 2.5 per SIMD anyway
template <int CB>
constexpr int lat_waves() { return CB < 0 ? 2 : 4; }
template <int SL, int CB = 0, int DM = kDmContig>
__global__ __launch_bounds__(64, lat_waves<CB>()) void lpc_env_lattice_kernel(LpcEnvArgs A_) {
  extern __shared__ double sh[];
  const LpcEnvArgs& A = A_;
  const int ngroups = (A.items + 3) >> 2;
  // (prefetching the next group's r into registers before the envelope phase was measured: no gain,
  // it costs a wave per SIMD of occupancy)
  double r0n;
  auto load_r = [&](int ibase) {
    const int it = ibase + (threadIdx.x >> 4);
    const double* rr = A.r + (int64_t)(it < A.items ? it : 0) * A.nlags;
    if constexpr (DM != kDmExt) r0n = rr[0];
  };
  // DM = 2 with a register cepstrum: the next group's a rows go global -> LDS by DMA (no registers)
  // while this group's envelope runs (it reads only cs, not la)
  auto dma_a = [&](int ibase) {
    if constexpr (DM == kDmExt && CB != 0) {
#pragma unroll
      for (int g2 = 0; g2 < 4; ++g2) {
        const int it = min(ibase + g2, A.items - 1);
        FDLP_CHECK(it >= 0 && A.la_len <= A.a_stride && A.la_len <= A.region);
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
  // ---- group sequence: groups blockIdx.x, + gridDim.x, ... of consecutive items (-1 at the end) ----
  auto next_group = [&](int ibase) -> int {
    return ibase + 4 * (int)gridDim.x < 4 * ngroups ? ibase + 4 * (int)gridDim.x : -1;
  };
  int cur = (int)blockIdx.x < ngroups ? 4 * (int)blockIdx.x : -1;
  if (cur >= 0) dma_a(cur);
  while (cur >= 0) {
    const int ibase = cur;
    load_r(ibase);
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
    const int item = ibase + g;
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
    } else {
      const double* rr = A.r + (int64_t)(valid ? item : 0) * A.nlags;
      const double r0 = valid ? r0n : 1.0;
      gg = r0;
      {
        double A1[1] = {lane0 ? 1.0 : 0.0}, B1[1] = {lane0 ? 1.0 : 0.0}, R11[1];
        contig_load_r1<1>(R11, rr, A.nlags, p, l, valid);
        double part = lane0 ? R11[0] : 0.0;  // order 1: b^(0) . R1 = r_1
        double E = r0;
        contig_durbin<SL, 1>(A1, B1, R11, part, E, la, rr, A.nlags, p, l, valid, gg, r0);
      }
      // la[0 .. 16 SL) holds a_0 .. a_p (zeros beyond p); zero the rest of the a region
      for (int q = l + 16 * SL; q < NAL; q += 16) la[q] = 0.0;
      wave_lds_sync();
      if (valid && A.a_out) {
        for (int m = l; m <= p; m += 16) A.a_out[(int64_t)item * (p + 1) + m] = la[m];
        if (lane0) A.gg_out[item] = gg;
      }
    }
    wave_lds_sync();
    // ---- phase 2: cepstrum (features.py:233-246), as in lpc_env_kernel -------------------------
    if constexpr (CB > 0) {
      // d_n = n c_n = y_n - sum_{k in the block, k < n} d_k a_{n-k}, y_n = -n a_n - (finished blocks' terms):
      // a unit lower-triangular Toeplitz system per block, solved by the first 16 terms of the impulse
      // response of 1/a(z) (h_0 = 1, h_m = -sum a_k h_{m-k}, once per item): d = H y, 16 broadcast FMAs in 4
      // chains instead of a 16-step serial recurrence (the form the REVERB super-blocks use, features.py:243-245)
      double kc[CB];  // lane l: d_n = n c_n for n = 16 b + l of every finished block b (0 for n = 0)
      double Hrow[16];
      {
        double t = l >= 1 ? la[l] : 0.0;  // sum_{i < l} h_i a_{l-i}, so far i = 0
        double hl = l == 0 ? 1.0 : 0.0;
        sb_impulse<1>(hl, t, la, l);
        Hrow[0] = hl;
        sb_hrow<1>(Hrow, hl);
      }
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        const int b0 = 16 * b;
        if (b0 >= M) break;
        const int n = b0 + l;
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        if (b > 0) asm volatile("s_nop 1");  // kc[b - 1] was just written: DPP reads need 2 wait states
#pragma unroll
        for (int bp = 0; bp < b; ++bp) {
          const double* al = la + n - 16 * bp;  // alpha_{n - k} = la[n - k], k = 16 bp + j
          cep_terms16(a0, a1, a2, a3, kc[bp], al);
        }
        const double an = n <= p ? la[min(n, p)] : 0.0;
        const double y = -(double)n * an - ((a0 + a1) + (a2 + a3));
        const double d = sb_solve(y, Hrow);
        const double mine = n == 0 ? log(sqrt(gg)) : d * inv_count(n > 0 ? n : 1);
        kc[b] = d;  // 0 for n = 0 (y_0 = 0)
        if (n < CSN) cs[n] = mine;
        if (n < M && valid && A.cep_out) A.cep_out[(int64_t)item * M + n] = mine;
      }
      wave_lds_sync();
    } else if constexpr (CB < 0) {
      // any M (REVERB: 450): super-blocks of R blocks (see sb_window above).  alpha_{n-k} = 0 for n - k > p,
      // and V_q, q < W = SL, covers every lag up to 16 SL + 15 >= p + 15, so the terms added beyond the
      // reference's range are exact zeros (la is zero from p + 1 to la_len).
      constexpr int W = SL;
      constexpr int R = 4;
      double kc[W];  // kc[w]: d (lane l) of block s - 1 - w of the current super-block s; 0 before block 0
#pragma unroll
      for (int w = 0; w < W; ++w) kc[w] = 0.0;
      // h and the H rows of this item (a_1 .. a_15 from la)
      double Hrow[16];
      {
        double t = l >= 1 ? la[l] : 0.0;  // sum_{i < l} h_i a_{l-i}, so far i = 0
        double hl = l == 0 ? 1.0 : 0.0;
        sb_impulse<1>(hl, t, la, l);
        Hrow[0] = hl;
        sb_hrow<1>(Hrow, hl);
      }
      // only c_0 .. c_{Me-1} reach the envelope (fft(., env_nfft) truncates, :201); all M are computed
      // when the cepstra themselves are an output (debug / modulation-spectrum mode)
      const int Mc = A.cep_out ? M : A.Me;
      const int NB = (Mc + 15) >> 4;
      // the lane's LDS byte address la + l + 1: V_q[j] = la[16 (q+1) + l - j] at byte offset 8 (16 q + 15 - j)
      const uint32_t aaddr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) double*)(la + l + 1));
      for (int sb = 0; sb < NB; sb += R) {
        double acc[R][2];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = 0.0;
        double va[16], vb[16];
        const int qmax = min(W, sb + R - 1);  // V_q reaches a finished block (q - r < sb) for some r
        asm volatile("s_nop 1");  // kc was just written: DPP reads need 2 wait states
        lgkm_wait<0>();  // nothing else (scalar loads complete out of order) may share the counted waits
        if (qmax > 0) {
          lds_load16<15>(va, aaddr);
          sb_window<W, R, 0>(acc, kc, va, vb, aaddr, qmax);
        }
        double kcnew[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int n = 16 * (sb + r) + l;
          if (r == 1) { lds_load16<15>(va, aaddr); sb_local<R, 0>(acc[1], kcnew, va, vb, aaddr); }
          if (r == 2) { lds_load16<15>(va, aaddr); sb_local<R, 1>(acc[2], kcnew, va, vb, aaddr); }
          if (r == 3) { lds_load16<15>(va, aaddr); sb_local<R, 2>(acc[3], kcnew, va, vb, aaddr); }
          const double an = n <= p ? la[min(n, p)] : 0.0;
          const double y = -(double)n * an - (acc[r][0] + acc[r][1]);
          const double d = sb_solve(y, Hrow);
          kcnew[r] = d;
          const double c = n == 0 ? log(sqrt(gg)) : d * inv_count(n > 0 ? n : 1);
          if (n < CSN) cs[n] = c;
          if (n < M && valid && A.cep_out) A.cep_out[(int64_t)item * M + n] = c;
          asm volatile("s_nop 1");  // kcnew[r] feeds the next block's DPP-broadcast FMAs
        }
#pragma unroll
        for (int w = W - 1; w >= 0; --w) kc[w] = w >= R ? kc[w - R] : kcnew[R - 1 - w];
      }
      wave_lds_sync();
    }
    for (int b0 = 0; b0 < (CB == 0 ? M : 0); b0 += 16) {
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
    cur = next_group(ibase);
    if (cur >= 0) dma_a(cur);  // la is free until the next group
    // ---- phase 3: weights + envelope (computeFDLPSpectrogram.py:194-205) ---------------------
    double* cw = CB != 0 ? cs : la;  // compact layout: weighted in place
    const double* mask = A.weights;
    const double* lif = A.weights + M;
    const double* gam = A.weights + 2 * M;
    // four coefficients per lane at a time: their 12 weight loads issue together (one exposed latency per
    // four, not per coefficient), the products in the reference's order
    for (int n0 = l; n0 < A.Me; n0 += 64) {
      double wm[4], wl[4], wg[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int n = min(n0 + 16 * k, A.Me - 1);  // clamped: the loads are unconditional
        wm[k] = mask[n];
        wl[k] = lif[n];
        wg[k] = gam[n];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int n = n0 + 16 * k;
        if (n < A.Me) {
          double v = cs[n];
          v = v * wm[k];
          v = v * wl[k];
          v = v * wg[k];
          if (A.odd_zero && (n & 1)) v = 0.0;
          cw[n] = v;
        }
      }
    }
    wave_lds_sync();
    // every envelope sample env[s] of this lane's item goes through emit
    const int kk = A.kk;
    double* const envp = A.env ? A.env + (int64_t)(valid ? item : 0) * kk : nullptr;
    auto emit = [&](int s_, double e) {
      if (valid && envp) envp[s_] = e;
    };
    bool env_done = false;
    if constexpr (CB < 0) {
      if (A.env_nfft == 300 && A.Me == 300 && A.kk == 150) {  // the recipes' REVERB envelope: FFT route
        env_fft300(cw, A.env_cos, A.env_win, l, valid, emit);
        env_done = true;
      }
    }
    // S(u) = Even(u) + Odd(u), S(H - u) = Even(u) - Odd(u); lane slots cover u = 0..H/2 (lpc_env_kernel)
    for (int q0 = 0; q0 < (env_done ? 0 : TS); q0 += kEnvChunk) {
      double se[kEnvChunk], so[kEnvChunk], cprev[kEnvChunk], ccur[kEnvChunk], c2[kEnvChunk];
      // slots u < 16 (q0 + kEnvChunk) <= env_nfft (every recipe: 80 <= 300) index the cosine table
      // directly; the modulo (~16 integer instructions per slot) is compiled only into the other branch
      auto setup = [&](auto direct) {
#pragma unroll
        for (int q = 0; q < kEnvChunk; ++q) {
          const int u = l + 16 * (q0 + q);
          const double c1 = A.env_cos[decltype(direct)::value ? u : u % A.env_nfft];
          se[q] = cw[0];
          so[q] = 0.0;
          cprev[q] = 1.0;
          ccur[q] = c1;
          c2[q] = 2.0 * c1;
        }
      };
      if (16 * (q0 + kEnvChunk) <= A.env_nfft) setup(std::true_type{});
      else setup(std::false_type{});
      int n = 1;
      for (; n + 1 < A.Me; n += 2) {
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
#pragma unroll
        for (int q = 0; q < kEnvChunk; ++q) {
          const int u = l + 16 * (q0 + q);
          if (2 * u > H) continue;
          if (u < A.kk) emit(u, exp(se[q] + so[q]) * A.env_win[2 * u]);
          const int t2 = H - u;
          if (t2 != u && t2 < A.kk) emit(t2, exp(se[q] - so[q]) * A.env_win[2 * t2]);
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
  const double gg = durbin16(la, lr, p, l);
  if (valid && A.a_out) {
    for (int i = l; i <= p; i += 16) A.a_out[(int64_t)item * (p + 1) + i] = la[i];
    if (l == 0) A.gg_out[item] = gg;
  }
  wave_lds_sync();
  // ---- phase 2: cepstrum (features.py:233-246): c_n = -a_n - sum_{k<n} (k/n) c_k a_{n-k} --------
  // blocks of 16 coefficients: the finished blocks enter as a lane-parallel dot product, the block
  // itself as a 16-step recurrence with the new c_k broadcast along the row.
  double* cs = lr;
  for (int b0 = 0; b0 < M; b0 += 16) {
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
  for (; n + 1 < A.Me; n += 2) {
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
  (void)kmark(kKLpcLds, s);
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
  if (SL > 16 || c.lpc_mode == 1) return hipErrorNotSupported;
  if (c.M <= 16 * 7 && SL >= 9 && SL <= 11) {  // register-broadcast cepstrum (recipes: p 150, M 100)
    switch (SL) {
      case 9: return fn(integral_constant<int, 9>{}, integral_constant<int, 7>{});
      case 10: return fn(integral_constant<int, 10>{}, integral_constant<int, 7>{});
      case 11: return fn(integral_constant<int, 11>{}, integral_constant<int, 7>{});
      default: break;
    }
  }
  if (c.M > 16 * 7 && SL >= 9 && SL <= 11) {  // the same over a sliding window (REVERB: M 450)
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

// durbin8_kernel instantiations: 8 SL8 >= p + 1, SL8 odd, for the lattice range SL = 9..11 (p 128..175)
static int durbin8_sl8(int p) { return ((p + 1 + 7) / 8) | 1; }
static bool durbin8_fits(int p) {
  const int sl8 = durbin8_sl8(p);
  return sl8 >= 17 && sl8 <= 23;
}
template <class Fn>
static hipError_t durbin8_dispatch(int p, Fn&& fn) {
  using std::integral_constant;
  switch (durbin8_sl8(p)) {
    case 17: return fn(integral_constant<int, 17>{});
    case 19: return fn(integral_constant<int, 19>{});
    case 21: return fn(integral_constant<int, 21>{});
    case 23: return fn(integral_constant<int, 23>{});
    default: return hipErrorNotSupported;
  }
}

// durbin4_kernel (4 lanes per item): one instantiation, SL4 = 38, for 128 <= p <= 150 (the recipes' 150)
constexpr int kDurbin4SL = 38;
static bool durbin4_fits(const DevConsts& c) {
  return c.lpc_mode == 0 && c.p >= 128 && c.p <= 4 * kDurbin4SL - 2;
}

// fn(integral_constant<SL>, integral_constant<CB>, integral_constant<int, DM>)
template <class Fn>
static hipError_t lattice_dispatch(const DevConsts& c, Fn&& fn) {
  using std::integral_constant;
  return lattice_dispatch_sl(c, [&](auto sl, auto cb) -> hipError_t {
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
  // c.lpc_mode (fdlp_set_lpc_path): 0 = the lattice kernels (durbin8_kernel where p fits it, then the
  // register cepstrum / envelope kernel), 1 = the LDS Durbin kernel (lpc_env_kernel) for every p
  // 2 = the lattice kernels with durbin8_kernel also where durbin4_kernel fits (cross-check)
  c.lpc_split = (c.lpc_mode == 0 || c.lpc_mode == 2) && durbin8_fits(c.p);
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
    if (CT == kDmExt)  // >= the durbin8 image (8 SL8 positions written per row) and the cepstrum's a area
      c.lpc_astride = (std::max({CB != 0 ? lattice_la_len(c, CB, SL) : c.p + 1, 8 * durbin8_sl8(c.p),
                                 durbin4_fits(c) ? 4 * kDurbin4SL : 0}) + 15) / 16 * 16;
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
    const hipError_t e = durbin4_fits(c) ? [&]() -> hipError_t {
      if (c.lpc_astride < 4 * kDurbin4SL) return hipErrorInvalidValue;
      hipLaunchKernelGGL((durbin4_kernel<kDurbin4SL>), dim3((items + 15) / 16), dim3(64), 0, s, r, c.nlags, c.p, items,
                         a_ws, gd, c.lpc_astride);
      (void)kmark(kKDurbin4, s);
      return hipGetLastError();
    }() : durbin8_dispatch(c.p, [&](auto sl8) -> hipError_t {
      constexpr int SL8 = decltype(sl8)::value;
      hipLaunchKernelGGL((durbin8_kernel<SL8>), dim3((items + 7) / 8), dim3(64), 0, s, r, c.nlags, c.p, items, a_ws, gd,
                         c.lpc_astride);
      (void)kmark(kKDurbin8, s);
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
    const hipError_t e = lattice_dispatch(c, [&](auto sl, auto cb, auto ct) -> hipError_t {
      constexpr int SL = decltype(sl)::value, CB = decltype(cb)::value;
      constexpr int CT = decltype(ct)::value;
      const size_t lds = lattice_lds(c, CB, SL);
      A.region = lattice_region(c, CB, SL);
      A.la_len = CB != 0 ? lattice_la_len(c, CB, SL) : 0;
      hipLaunchKernelGGL((lpc_env_lattice_kernel<SL, CB, CT>), dim3(grid), dim3(64), lds, s, A);
      (void)kmark(kKLattice, s);
      return hipGetLastError();
    });
    return e;
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

hipError_t checks_lpc(unsigned int* v, bool reset) { return fdlp_checks_local(v, reset); }

}  // namespace fdlp
