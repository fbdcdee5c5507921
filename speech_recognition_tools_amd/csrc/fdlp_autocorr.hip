// fdlp_autocorr.hip -- gfx950 kernels of the autocorrelation stage (SURVEY.md 8(a) a10-a11,
// features.py:223-225 on the band signal W_j (.) D_f, :190-191):
//   autocorr_kernel   : direct circular autocorrelation, lags 0..p+1, on MFMA f64 16x16x4 (any filterbank)
//   ac_vsweep_kernel  : structured path (cochlear, fixed skirt slope): lag-parallel VALU sweeps of the
//                       skirts and flat tops with per-band snapshots
//   ac_sweep_kernel   : the same skirt sweeps on MFMA (structured_mfma)
//   ac_band_kernel    : per-band boundary straddles (MFMA) + the combine into r
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include "fdlp_device.h"

namespace fdlp {

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
constexpr int kMaxWrapLags = 256;  // ac_wrap_kernel LDS edges (nlags <= 256)

template <int NT>
__global__ __launch_bounds__(64, 4) void autocorr_kernel(DevConsts c, const double* __restrict__ dct,
                                                      const double* __restrict__ dense,
                                                      double* __restrict__ rout) {
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
                                                        const double* __restrict__ rpart,
                                                        const double* __restrict__ rwrap, int items) {
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
  FDLP_CHECK(0 <= m1 && m1 <= m2 && m2 <= N && j < c.B);
  // the wrap straddle of a band whose first / last nlags - 1 taps are skirt taps is kw Wrap (ac_wrap_kernel)
  const double kw = (VS && rwrap) ? c.sk_wrap[j] : 0.0;
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
  constexpr int kSt = (kWin + 16 * NT + 63) / 64;  // B reads reach xb[kWin - 1 + 16 NT - 1]
  static_assert(kSt > kWin / 64 && kWin % 64 == 0, "window layout");
  // the MFMAs of one straddle from its staged windows xa / xb (B reads xb[kWin - 63, kWin + 16 NT))
  auto straddle = [&](const double* xa, const double* xb, int st0) {
    // st unrolled, so each step's first live tile tmin is a constant: its MFMAs and their LDS reads are
    // branch-free (the reads issue together instead of one exposed LDS latency per MFMA)
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
  };
  // Regular band (72 of the recipes' 80): both straddle windows [b - kWin, b + kSt 64 - kWin) lie inside
  // [0, N), the flat top is at least nlags - 1 wide (so the m1 straddle's B side is flat: x = D, and the m2
  // straddle's A side is flat: x = D) and the wrap straddle is the shared kw Wrap.  Then nothing is masked
  // or clamped: A positions below lb = b - (nlags - 1) pair only at lags >= nlags (their accumulator
  // elements are never emitted), B below b reads a zeroed 64-position block, and the staging is a product (or
  // a copy) per position with immediate-offset loads -- the same values the general staging writes at every
  // position an emitted lag reads, so r is bit-identical.  The loads of both boundaries are issued at once
  // into two compact LDS regions [A: kWin | zeros: 64 | B: 16 NT], so an item waits for memory once before
  // its straddles instead of once per boundary.
  constexpr int kReg = kWin + 64 + 16 * NT;  // one boundary's compact region
  constexpr bool kFits = 2 * kReg <= kLds;   // every order up to p = 190 (NT <= 12)
#ifdef FDLP_AB_BAND_GENERIC  // A/B build: every band through the general staging
  const bool fast = false;
#else
  const bool fast = kFits && VS && kw != 0.0 && m1 >= kWin && m2 - m1 >= nlags - 1 && m2 + (kSt * 64 - kWin) <= N;
#endif
  if constexpr (kFits) if (fast) {
    constexpr int kA = kWin / 64, kB = kSt - kWin / 64;  // staged A / B slots
    static_assert(kB <= kA + 1, "m2 B taps");
    double d1[kSt], w1[kA], d2[kSt], w2[kA];
    {
      const double* s1 = drow + (m1 - kWin) + lane;
      const double* t1 = wrow + (m1 - kWin) + lane;        // taps below m1
      const double* s2 = drow + (m2 - kWin) + lane;
      const double* t2 = wrow + m2 + lane;                 // taps from m2 on
      FDLP_CHECK(m1 - kWin >= 0 && m2 + 64 * kB <= N);
#pragma unroll
      for (int u = 0; u < kSt; ++u) d1[u] = s1[64 * u];
#pragma unroll
      for (int u = 0; u < kA; ++u) w1[u] = t1[64 * u];
#pragma unroll
      for (int u = 0; u < kSt; ++u) d2[u] = s2[64 * u];
#pragma unroll
      for (int u = 0; u < kA; ++u) w2[u] = t2[64 * u];
    }
    double* r1 = xs;
    double* r2 = xs + kReg;
#pragma unroll
    for (int u = 0; u < kA; ++u) {
      r1[64 * u + lane] = w1[u] * d1[u];  // lower-skirt taps x D below m1
      r2[64 * u + lane] = d2[u];          // flat top below m2
    }
    r1[kWin + lane] = 0.0;
    r2[kWin + lane] = 0.0;
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int q = 64 * u + lane;
      if (q < 16 * NT) {
        r1[kWin + 64 + q] = d1[kA + u];                                  // flat top from m1 on
        r2[kWin + 64 + q] = u < kA ? (w2[u] - 1.0) * d2[kA + u] : 0.0;  // (W - 1) D from m2 on
      }
    }
    __syncthreads();
    straddle(r1, r1 + 64, 0);  // xb index k -> region offset k + 64: xb[kWin - 64 + i] is the zero block
    straddle(r2, r2 + 64, 0);
  }
  if (!fast) {
    double* xa = xs;
    double* xb = xs + kWin;
#pragma unroll 1
    for (int e = 0; e < (kw != 0.0 ? 2 : 3); ++e) {
      const int b = e == 0 ? m1 : (e == 1 ? m2 : N);
      int lb = e == 0 ? 0 : (e == 1 ? m1 : m2);
      lb = max(lb, b - (nlags - 1));
      if (lb >= b) continue;
      double wv[kSt], dv[kSt];
#pragma unroll
      for (int u = 0; u < kSt; ++u) {  // all loads first: one exposed latency per boundary
        const int pos = b - kWin + 64 * u + lane;
        const int pm = pos < 0 ? 0 : (pos >= N ? pos - N : pos);
        FDLP_CHECK(pm >= 0 && pm < N);
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
      straddle(xa, xb, (lb - b + kWin) >> 6);
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
    double rv[kNB], uv[kNB], fv[kNB], wv[kNB];
    const double* wo = rwrap + (int64_t)f * nlags;
    // lag L = 32 g + lane / 2 from one lane pointer and immediate offsets: lags past the row end read the next
    // row (or the kRowSlack doubles every row buffer carries past its last row) and are never emitted
    static_assert(32 * kNB - (16 * (NT - 1) - 14) <= kRowSlack, "row slack covers the last lag block");
    const int lh = lane >> 1;
    FDLP_CHECK(32 * kNB <= nlags + kRowSlack);
#pragma unroll
    for (int g = 0; g < kNB; ++g) {
      rv[g] = ro[lh + 32 * g];
      uv[g] = uo[lh + 32 * g];
      fv[g] = fo[lh + 32 * g];
      wv[g] = kw != 0.0 ? wo[lh + 32 * g] : 0.0;
    }
    if (pmask) {
      for (int rest = pmask; rest; rest &= rest - 1) {
        FDLP_CHECK(__builtin_ctz(rest) < c.fl_H - 1 && fb.x >= 0 && fb.x < kMaxChains);
        const double* po = rpart + (((int64_t)f * (c.fl_H - 1) + __builtin_ctz(rest)) * kMaxChains + fb.x) * nlags + lh;
#pragma unroll
        for (int g = 0; g < kNB; ++g) fv[g] += po[32 * g];
      }
    }
#pragma unroll
    for (int g = 0; g < kNB; ++g) {
      const int L = 32 * g + (lane >> 1);
      if ((lane & 1) == 0 && L < nlags) {
        const double v = sums[g] + rv[g] + uv[g] + fv[g];
        ro[L] = kw != 0.0 ? v + kw * wv[g] : v;
      }
    }
  } else {
    diag_blocks<NT, 32>(acc, xs, nlags, lane, [&](int L, double v) { ro[L] = v + ro[L] + uo[L]; });
  }
}

// Wrap straddle shared by the bands of a frame whose first / last nlags - 1 taps are skirt taps: there
// x_j = sqrt(K_j) E D below m1_j and sqrt(K'_j) E' D above m2_j, so the pairs crossing the circular wrap
// at N give sqrt(K_j K'_j) Wrap[l] with one band-independent
//   Wrap[l] = sum_{i < l} z[N - l + i] y[i],   z = E' D (top nlags - 1 bins), y = E D (bottom ones)
// (ac_band_kernel adds it in place of the band's own wrap straddle).  One wave per frame, a lane per lag
// (l = lane, lane + 64, ...), the two edges staged in LDS, i ascending.
__global__ __launch_bounds__(64) void ac_wrap_kernel(DevConsts c, const double* __restrict__ dct,
                                                     double* __restrict__ rwrap, int nframes) {
  __shared__ double zt[kMaxWrapLags], yh[kMaxWrapLags];
  const int f = blockIdx.x;
  if (f >= nframes) return;
  const int N = c.N, nlags = c.nlags, L1 = nlags - 1;
  const double* drow = dct + (int64_t)f * N;
  for (int i = threadIdx.x; i < L1; i += 64) {
    const int mt = N - L1 + i;
    zt[i] = c.sk_e[N + mt] * drow[mt];
    yh[i] = c.sk_e[i] * drow[i];
  }
  __syncthreads();
  for (int l = threadIdx.x; l < nlags; l += 64) {
    double acc = 0.0;
    for (int i = 0; i < l; ++i) acc = fma(zt[L1 - l + i], yh[i], acc);
    rwrap[(int64_t)f * nlags + l] = acc;
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

constexpr int kVsMirror = 16;
// ring positions per unit (a power of two is not required: slots are taken modulo the ring) and the LDS
// row stride; rows of 544 doubles keep each ds_read_b128 lane group on 64 distinct banks for the
// 10-double lane stride of the window reads.  (Skirt sweeps at three waves per SIMD -- a 320-position
// ring, 128-position chunks, one parked row -- measured 1.56 -> 2.19 ms, r03s: not kept.)
template <int C>
constexpr int vs_ring() { return 512; }
template <int C>
constexpr int vs_row() { return 544; }
// positions staged per chunk; the prefetch of the next chunk has to cover the HBM latency under load
// (64 positions, ~3000 cycles of FMAs, measured too short).  The flat sweep keeps its chains in
// registers, so it stages 128 at a time to stay at two waves per SIMD.
template <int A, int C>
constexpr int vs_chunk() { return (C == 0 && 18 * A < vs_ring<C>() - 256) ? 256 : 128; }
template <int C>
constexpr int vs_waves_per_simd() { return 2; }

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
  // the DPP source must be two wait states past its VALU write (the compiler cannot see the DPP
  // inside the asm): copy it through one asm that ends in the wait.  (Broadcasting by v_mov_dpp into
  // registers first and plain FMAs: slower, r03.)
  double cm;
  asm volatile("v_mov_b64 %0, %1\n\ts_nop 1" : "=v"(cm) : "v"(cur));
  vs_fma_rows<A>(acc, cm, lo, hi);
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
  constexpr int kVsRing = vs_ring<C>();
  constexpr int kRow = vs_row<C>();
  static_assert(A % 2 == 0 && A <= 16 && 18 * A < kVsRing - kVsChunk && A <= kVsMirror + 1, "vsweep geometry");
  static_assert(kRow >= kVsRing + kVsMirror && kVsRing % 2 == 0, "ring row");
  // slot of sweep position n (n >= -kVsRing): n mod kVsRing (a mask when the ring is a power of two)
  auto slot_of = [](int n) {
    if constexpr ((kVsRing & (kVsRing - 1)) == 0) return n & (kVsRing - 1);
    else return (n + 8 * kVsRing) % kVsRing;
  };
  // wave-uniform base u (scalar modulo) plus a lane offset d < kVsRing
  auto slot_add = [&](int u, int d) {
    if constexpr ((kVsRing & (kVsRing - 1)) == 0) {
      return (u + d) & (kVsRing - 1);
    } else {
      const int b = slot_of(__builtin_amdgcn_readfirstlane(u)) + d;
      return b >= kVsRing ? b - kVsRing : b;
    }
  };
  // row stride 544 doubles = 17 x 256 B: each ds_read_b128 lane group (lanes 0-3,12-15 of one row and
  // 4-11 of the next, MI355X_MICROARCH.md LDS) then covers the 64 banks exactly with the 10-double lane
  // stride of the window reads (A = 10; a 528 stride measured 9.4e7 conflict cycles per launch)
  __shared__ double ring_all[4][kRow];
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
  // A skirt-sweep chunk that lies inside [0, N) (every chunk but the sweep's first and last) needs no clamping
  // or range selects: one lane pointer and immediate offsets (the general form spends ~10 integer VALU
  // instructions per load and per slot on the clamps, the reversed index and the mirror test).  Chunks start
  // at multiples of kVsChunk, so their ring slots are one aligned run and only the run at slot 0 writes the
  // mirror (slots < kVsMirror = its first 16 positions).  (The flat sweep, which holds its chains in
  // registers, spills with the second copy: 0.90 -> 1.18 ms; it keeps the general form.)
  static_assert((kVsRing & (kVsRing - 1)) == 0 && kVsRing % kVsChunk == 0 && kVsMirror == 16, "aligned chunk runs");
  auto inside = [&](int base) { return C == 0 && base >= 0 && base + kVsChunk <= N; };
  auto issue = [&](int base) __attribute__((always_inline)) {
    if (inside(base)) {  // wave-uniform
      if (kind == 0) {
        const double* pd = drow + (N - 1 - base - l);
        const double* pw = ew + (N - 1 - base - l);
#pragma unroll
        for (int q = 0; q < kPf; ++q) {
          pf[q] = __builtin_nontemporal_load(pd - 16 * q);
          if constexpr (C == 0) pe[q] = pw[-16 * q];
        }
      } else {
        const double* pd = drow + base + l;
        const double* pw = ew + base + l;
#pragma unroll
        for (int q = 0; q < kPf; ++q) {
          pf[q] = __builtin_nontemporal_load(pd + 16 * q);
          if constexpr (C == 0) pe[q] = pw[16 * q];
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < kPf; ++q) {
        const int n = min(max(base + 16 * q + l, 0), N - 1);
        const int m = kind == 0 ? N - 1 - n : n;
        pf[q] = __builtin_nontemporal_load(drow + m);
        if constexpr (C == 0) pe[q] = ew[m];
      }
    }
  };
  auto commit = [&](int base) __attribute__((always_inline)) {
    if (inside(base)) {  // wave-uniform
      const int sb = base & (kVsRing - 1);
      double* w = rg + sb + l;
#pragma unroll
      for (int q = 0; q < kPf; ++q) {
        double v = pf[q];
        if constexpr (C == 0) v = pe[q] * v;
        w[16 * q] = v;
      }
      if (sb == 0) {
        double v = pf[0];
        if constexpr (C == 0) v = pe[0] * v;
        rg[kVsRing + l] = v;
      }
    } else {
#pragma unroll
      for (int q = 0; q < kPf; ++q) {
        const int n = base + 16 * q + l;
        const int slot = slot_add(base, 16 * q + l);
        double v = pf[q];
        if constexpr (C == 0) v = pe[q] * v;
        v = (n >= 0 && n < N) ? v : 0.0;
        FDLP_CHECK(slot >= 0 && slot < kVsRing);
        rg[slot] = v;
        if (slot < kVsMirror) rg[kVsRing + slot] = v;
      }
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
        FDLP_CHECK(band >= 0 && band < B);
        prow[i] = ((int64_t)f * B + band) * nlags;
      }
    }
    ++npend;
  };

  // chunks [lo_loaded, lo_loaded + 512) resident; the top block needs up to A b_top + 17 A - 2
  int lo_loaded = ((A * b_top + 17 * A - 1 + kVsChunk - 1) / kVsChunk) * kVsChunk;
  issue(lo_loaded - kVsChunk);
  auto ensure = [&](int n0) __attribute__((always_inline)) {
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
    const int base = slot_add(n0, A * l);
    FDLP_CHECK(base >= 0 && base + A <= kVsRing + kVsMirror);
#pragma unroll
    for (int q = 0; q < A; ++q) lo[q] = rg[base + q];
    const double cur = rg[slot_add(n0, l)];
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
    const int base = slot_add(A * b_top + A, A * l);
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
static hipError_t launch_ac_nt(const DevConsts& c, const double* dct, const double* dense, int items,
                               double* r, hipStream_t s) {
  hipLaunchKernelGGL((autocorr_kernel<NT>), dim3(items), dim3(64), 0, s, c, dct, dense, r);
  (void)kmark(kKAutocorr, s);
  return hipGetLastError();
}

int autocorr_tiles(int nlags) { return ((nlags + 14) >> 4) + 1; }

static hipError_t launch_autocorr_any(const DevConsts& c, const double* dct, const double* dense, int items,
                                      double* r, hipStream_t s) {
  if (items <= 0) return hipSuccess;
  switch (autocorr_tiles(c.nlags)) {
#define FDLP_AC_CASE(n) case n: return launch_ac_nt<n>(c, dct, dense, items, r, s);
    FDLP_AC_CASE(1) FDLP_AC_CASE(2) FDLP_AC_CASE(3) FDLP_AC_CASE(4) FDLP_AC_CASE(5)
    FDLP_AC_CASE(6) FDLP_AC_CASE(7) FDLP_AC_CASE(8) FDLP_AC_CASE(9) FDLP_AC_CASE(10)
    FDLP_AC_CASE(11) FDLP_AC_CASE(12) FDLP_AC_CASE(13) FDLP_AC_CASE(14) FDLP_AC_CASE(15)
    FDLP_AC_CASE(16)
#undef FDLP_AC_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_autocorr(const DevConsts& c, const double* dct, const double* dense, int items,
                           double* r, hipStream_t s) {
  // MFMA: measured 25.1 ms per 4096-frame batch against 27.1 ms for a register-blocked fp64 VALU
  // variant (round 1; it clocked down to ~1.95 GHz under full fp64 FMA load, and was removed)
  return launch_autocorr_any(c, dct, dense, items, r, s);
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
  (void)kmark(kKVsweepSkirt, s);
  hipLaunchKernelGGL((ac_vsweep_kernel<A, C>), dim3(xcd_grid(c.fl_H * ngroups)), dim3(64), 0, s, c, dct, r, rup,
                     rflat, rpart, c.sk_snap, c.fl_ev, nframes, ngroups);
  (void)kmark(kKVsweepFlat, s);
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
                                   double* rflat, double* rpart, double* rwrap, hipStream_t s) {
  if (rflat) {  // lag-parallel VALU sweeps (flat tops included) + straddles
    const hipError_t e = launch_vsweep(c, dct, nframes, r, rup, rflat, rpart, s);
    if (e != hipSuccess) return e;
    const bool wrap = rwrap && c.sk_wrap && c.nlags <= kMaxWrapLags;
    if (wrap) {
      hipLaunchKernelGGL(ac_wrap_kernel, dim3(nframes), dim3(64), 0, s, c, dct, rwrap, nframes);
      (void)kmark(kKAcWrap, s);
    }
    hipLaunchKernelGGL((ac_band_kernel<NT, true>), dim3(xcd_grid(nframes * c.B)), dim3(64), 0, s, c, dct, r, rup,
                       rflat, rpart, wrap ? rwrap : nullptr, nframes * c.B);
    (void)kmark(kKAcBand, s);
    return hipGetLastError();
  }
  const size_t tab = sizeof(SkSnap) * (size_t)c.B;
  hipLaunchKernelGGL((ac_sweep_kernel<NT, 32>), dim3(xcd_grid(2 * nframes)), dim3(64), tab, s, c, dct, r, rup, 2 * nframes);
  (void)kmark(kKAcSweep, s);
  hipLaunchKernelGGL((ac_band_kernel<NT, false>), dim3(xcd_grid(nframes * c.B)), dim3(64), 0, s, c, dct, r, rup,
                     nullptr, nullptr, nullptr, nframes * c.B);
  (void)kmark(kKAcBand, s);
  return hipGetLastError();
}

hipError_t launch_autocorr_structured(const DevConsts& c, const double* dct, int nframes, double* r,
                                      double* rup, double* rflat, double* rpart, double* rwrap, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  if (!c.sk_e || !c.sk_snap || !c.sk_reg) return hipErrorInvalidValue;
  if (rflat && (!c.fl_ev || !c.fl_band || (c.fl_H > 1 && !rpart))) return hipErrorInvalidValue;
  switch (autocorr_tiles(c.nlags)) {
#define FDLP_ST_CASE(n) case n: return launch_struct_nt<n>(c, dct, nframes, r, rup, rflat, rpart, rwrap, s);
    FDLP_ST_CASE(1) FDLP_ST_CASE(2) FDLP_ST_CASE(3) FDLP_ST_CASE(4) FDLP_ST_CASE(5)
    FDLP_ST_CASE(6) FDLP_ST_CASE(7) FDLP_ST_CASE(8) FDLP_ST_CASE(9) FDLP_ST_CASE(10)
    FDLP_ST_CASE(11) FDLP_ST_CASE(12) FDLP_ST_CASE(13) FDLP_ST_CASE(14) FDLP_ST_CASE(15)
    FDLP_ST_CASE(16)
#undef FDLP_ST_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t checks_autocorr(unsigned int* v, bool reset) { return fdlp_checks_local(v, reset); }

}  // namespace fdlp
