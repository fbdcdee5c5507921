// fdlp_plan.cpp -- plan (setup of getFeats, computeFDLPSpectrogram.py:43-118), batch geometry,
// OLA tables and the kernel pipeline behind fdlp_compute (getFeats :159-229).
#ifndef FDLP_DEVICE_CHECKS
#define FDLP_DEVICE_CHECKS 0
#endif
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fdlp.h"
#include "fdlp_error.h"
#include "fdlp_internal.h"

namespace fdlp {
std::string& last_error_slot() {
  static thread_local std::string s;
  return s;
}
}  // namespace fdlp

using fdlp::fail;

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return fail(FDLP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));          \
  } while (0)

namespace {

// Makes `dev` current for the scope of an ABI call and restores the caller's device afterwards.
class DeviceGuard {
 public:
  explicit DeviceGuard(int dev) {
    if (dev < 0) return;
    if ((err_ = hipGetDevice(&prev_)) != hipSuccess) return;
    if (prev_ != dev) {
      err_ = hipSetDevice(dev);
      switched_ = err_ == hipSuccess;
    }
  }
  ~DeviceGuard() {
    if (switched_) (void)hipSetDevice(prev_);
  }
  hipError_t status() const { return err_; }

 private:
  int prev_ = -1;
  bool switched_ = false;
  hipError_t err_ = hipSuccess;
};

// numpy.linspace(start, stop, num): i*step + start, last element = stop exactly.
std::vector<double> linspace(double start, double stop, int num) {
  std::vector<double> y(num);
  if (num == 1) { y[0] = start; return y; }
  const double step = (stop - start) / (double)(num - 1);
  for (int i = 0; i < num; ++i) y[i] = (double)i * step + start;
  if (num > 1) y[num - 1] = stop;
  return y;
}

// numpy.hamming / numpy.hanning: c0 + c1*cos(pi*n/(M-1)), n = 1-M, 3-M, ..., M-1
std::vector<double> cos_window(int M, double c0, double c1) {
  std::vector<double> w(std::max(M, 0));
  if (M == 1) { w[0] = 1.0; return w; }
  for (int i = 0; i < M; ++i) {
    const double n = (double)(1 - M + 2 * i);
    w[i] = c0 + c1 * cos(M_PI * n / (double)(M - 1));
  }
  return w;
}

// createFbankCochlear (features.py:193-219)
std::vector<double> fbank_cochlear(int nf, int nfft, int srate, double om_w, double alp, int fixed, double bet,
                                   double wf, int* ncol_out) {
  auto bark = [wf](double x) { return 6.0 * asinh((x / wf) / 600.0); };
  const double fmax = (double)srate / 2.0;
  const std::vector<double> cf = linspace(0.0, bark(fmax), nf);
  const int ncol = (int)floor((double)nfft / 2.0 + 1.0);
  std::vector<double> fl = linspace(0.0, fmax, ncol);
  for (auto& v : fl) v = bark(v);
  std::vector<double> W((size_t)nf * ncol);
  auto rows = [&](int i0, int i1) {
    for (int i = i0; i < i1; ++i) {
      const double fc = cf[i];
      const double a = fixed == 1 ? alp : alp * exp(-0.1 * fc);
      for (int j = 0; j < ncol; ++j) {
        const double d = fl[j] - fc;
        double v;
        if (d <= -om_w / 2.0) v = pow(10.0, a * (d + om_w / 2.0));
        else if (d > -om_w / 2.0 && d < om_w / 2.0) v = 1.0;
        else v = pow(10.0, -bet * (d - om_w / 2.0));
        W[(size_t)i * ncol + j] = v;
      }
    }
  };
  // ~2M pow calls for the recipes' 80 x 24001 taps: rows on a few threads (same values per element)
  const int nt = std::max(1, std::min({8, nf, (int)std::thread::hardware_concurrency()}));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(rows, nf * t / nt, nf * (t + 1) / nt);
  rows(0, nf / nt);
  for (auto& x : th) x.join();
  *ncol_out = ncol;
  return W;
}

// createFbank (features.py:172-190)
std::vector<double> fbank_mel(int nf, int nfft, int srate, double wf, int* ncol_out) {
  const double mel_max = 2595.0 * log10(1.0 + ((double)srate / wf) / 1400.0);
  const std::vector<double> mels = linspace(0.0, mel_max, nf + 2);
  const int ncol = (int)floor((double)nfft / 2.0 + 1.0);
  std::vector<double> edge(nf + 2);
  for (int i = 0; i < nf + 2; ++i) {
    const double hz = wf * (700.0 * (pow(10.0, mels[i] / 2595.0) - 1.0));
    edge[i] = floor((double)(nfft + 1) * hz / (double)srate);
  }
  std::vector<double> W((size_t)nf * ncol, 0.0);
  for (int m = 1; m <= nf; ++m) {
    const int l = (int)edge[m - 1], c = (int)edge[m], r = (int)edge[m + 1];
    for (int k = l; k < c; ++k)
      if (k >= 0 && k < ncol) W[(size_t)(m - 1) * ncol + k] = ((double)k - edge[m - 1]) / (edge[m] - edge[m - 1]);
    for (int k = c; k < r; ++k)
      if (k >= 0 && k < ncol) W[(size_t)(m - 1) * ncol + k] = (edge[m + 1] - (double)k) / (edge[m + 1] - edge[m]);
  }
  *ncol_out = ncol;
  return W;
}

// Structured-autocorrelation tables (DESIGN.md "Structured autocorrelation") for
// createFbankCochlear with fixed == 1: every band's taps must follow the lower-skirt / flat-top /
// upper-skirt pattern along m (classified exactly like fbank_cochlear), and the skirt factors
// E, E', K, K' must stay well inside the fp64 range.  Returns false otherwise (direct path).
struct SkirtTables {
  std::vector<double> e;    // [2, N]
  std::vector<fdlp::SkSnap> snap;  // [2, B] in sweep order
  std::vector<int2> reg;    // [B]
  int smin[2] = {0, 0};
  // flat-top sweep of ac_vsweep_kernel: events and chain count (C = 0: not possible)
  std::vector<fdlp::FlatEv> fl;
  int fl_C = 0, fl_lo = 0, fl_hi = 0;
  int fl_H = 1;
  int part_lo[fdlp::kMaxFlatParts] = {0}, part_hi[fdlp::kMaxFlatParts] = {0}, part_ev[fdlp::kMaxFlatParts + 1] = {0};
  std::vector<int2> fl_band;  // [B] (chain, partial-part mask)
  // wrap straddle: band j whose last nlags-1 taps lie on its upper skirt and first nlags-1 on its lower
  // skirt has straddle_N,j[l] = sqrt(K_j K'_j) Wrap[l], Wrap[l] = sum_{i<l} z[N-l+i] y[i] (one per frame);
  // wrap_kw[j] = sqrt(K_j K'_j) for those bands, 0 for the others (ac_band_kernel computes theirs)
  std::vector<double> wrap_kw;
  bool wrap_any = false;
};

// Split the flat sweep [fl_lo, fl_hi) into H parts of equal work (more waves: the flat sweep has one unit
// per frame against two for the skirts): a position costs 1, an event (restart or emission: the fold into
// every chain, the masked extra pass of the block it splits) kFlatEventCost positions -- fitted to the
// recipes' sweep (A = 10 lags per lane, C = 5 chains) from per-wave timings, where equal position parts
// ran 858 / 1067 us (median) with 34 / 126 events.  Part h covers [P_{h+1}, P_h) and takes
// the events with P_{h+1} <= S < P_h (part 0 also S = fl_hi).  Band j needs the partial chain of part h
// when its flat top crosses the part's lower end: m1_j < P_{h+1} < m2_j.
constexpr double kFlatEventCost = 35.0;
void flat_parts(SkirtTables* T, int B, int H) {
  if (T->fl_hi - T->fl_lo < 1024 * H) H = 1;
  T->fl_H = H;
  std::vector<int> P(H + 1);
  {
    // cost above position n (sweep order: top down), then the cut points at h / H of the total
    const int lo = T->fl_lo, hi = T->fl_hi, len = hi - lo;
    std::vector<double> above(len + 1, 0.0);  // above[i]: cost of positions [hi - i, hi) and their events
    std::vector<int> ev_at(len + 1, 0);
    for (const auto& e : T->fl) ev_at[std::min(std::max(hi - e.S, 0), len)] += 1;
    for (int i = 1; i <= len; ++i) above[i] = above[i - 1] + 1.0 + kFlatEventCost * ev_at[i];
    P[0] = hi;
    P[H] = lo;
    for (int h = 1, i = 0; h < H; ++h) {
      const double target = above[len] * h / H;
      while (i < len && above[i] < target) ++i;
      P[h] = hi - i;
    }
  }
  for (int h = 0; h < H; ++h) { T->part_hi[h] = P[h]; T->part_lo[h] = P[h + 1]; }
  const int nev = (int)T->fl.size();
  T->part_ev[0] = 0;
  for (int h = 1; h <= H; ++h) {
    int k = T->part_ev[h - 1];
    if (h == H) k = nev;
    else while (k < nev && T->fl[k].S >= P[h]) ++k;
    T->part_ev[h] = k;
  }
  T->fl_band.assign(B, make_int2(0, 0));
  for (int j = 0; j < B; ++j) {
    int mask = 0;
    for (int h = 0; h + 1 < H; ++h)
      if (T->reg[j].x < P[h + 1] && P[h + 1] < T->reg[j].y) mask |= 1 << h;
    T->fl_band[j] = make_int2(j % std::max(T->fl_C, 1), mask);
  }
}

void flat_parts(SkirtTables* T, int B, int H);

// Events of the flat-top sweep: band j restarts chain j mod C at m2_j and emits it at m1_j.  Order:
// S descending; at equal S bands descending (band j emits before band j - C restarts) and a band's
// restart before its own emission.  C is the smallest count for which no chain is restarted while
// it still serves a band (checked by replaying the events).
void flat_events(SkirtTables* T, int B) {
  T->fl_C = 0;
  T->fl.clear();
  T->fl_lo = INT32_MAX;
  T->fl_hi = 0;
  for (int j = 0; j < B; ++j) {
    T->fl_lo = std::min(T->fl_lo, T->reg[j].x);
    T->fl_hi = std::max(T->fl_hi, T->reg[j].y);
  }
  for (int C = 1; C <= 8; ++C) {
    std::vector<fdlp::FlatEv> ev;
    for (int j = 0; j < B; ++j) {
      ev.push_back(fdlp::FlatEv{T->reg[j].y, j, 0, j % C});
      ev.push_back(fdlp::FlatEv{T->reg[j].x, j, 1, j % C});
    }
    std::sort(ev.begin(), ev.end(), [](const fdlp::FlatEv& a, const fdlp::FlatEv& b) {
      if (a.S != b.S) return a.S > b.S;
      if (a.band != b.band) return a.band > b.band;
      return a.type < b.type;
    });
    std::vector<int> owner(C, -1);
    bool ok = true;
    for (const auto& e : ev) {
      if (e.type == 0) {
        if (owner[e.chain] != -1) { ok = false; break; }
        owner[e.chain] = e.band;
      } else {
        if (owner[e.chain] != e.band) { ok = false; break; }
        owner[e.chain] = -1;
      }
    }
    if (ok) {
      T->fl = ev;
      T->fl_C = C;
      flat_parts(T, B, 2);  // two position parts (3 and 4 measured slower)
      return;
    }
  }
}

bool skirt_tables(const fdlp_config& c, int B, int N, int nfft, SkirtTables* T) {
  if (c.fbank_kind != FDLP_FBANK_COCHLEAR || c.fixed != 1) return false;
  const double wf = c.warp_fact, om = c.om_w, a = c.alp, b = c.bet;
  if (!std::isfinite(wf) || !std::isfinite(om) || !std::isfinite(a) || !std::isfinite(b)) return false;
  auto bark = [wf](double x) { return 6.0 * asinh((x / wf) / 600.0); };
  const double fmax = (double)c.srate / 2.0;
  const std::vector<double> cf = linspace(0.0, bark(fmax), B);
  const int ncol = (int)floor((double)nfft / 2.0 + 1.0);
  if (ncol - 1 != N) return false;
  std::vector<double> fl = linspace(0.0, fmax, ncol);
  for (auto& v : fl) v = bark(v);
  T->reg.resize(B);
  for (int j = 0; j < B; ++j) {
    int state = 0, m1 = 0, m2 = 0;
    for (int m = 0; m < N; ++m) {
      const double d = fl[m] - cf[j];
      const int cls = d <= -om / 2.0 ? 0 : ((d > -om / 2.0 && d < om / 2.0) ? 1 : 2);
      if (cls < state) return false;
      state = cls;
      if (cls == 0) m1 = m + 1;
      if (cls <= 1) m2 = m + 1;
    }
    if (m2 < m1) m2 = m1;
    T->reg[j] = make_int2(m1, m2);
  }
  const long double c0 = 0.5L * ((long double)fl[0] + (long double)fl[N - 1]);
  const long double span = std::max(fabsl((long double)fl[N - 1] - c0), fabsl((long double)fl[0] - c0));
  if (fabsl((long double)a) * span > 60.0L || fabsl((long double)b) * span > 60.0L) return false;
  T->e.resize(2 * (size_t)N);
  for (int m = 0; m < N; ++m) {
    const long double x = (long double)fl[m] - c0;
    T->e[m] = (double)powl(10.0L, (long double)a * x);
    T->e[(size_t)N + m] = (double)powl(10.0L, -(long double)b * x);
  }
  std::vector<double> K(2 * (size_t)B);
  for (int j = 0; j < B; ++j) {
    const long double ea = (long double)a * ((long double)om - 2.0L * cf[j] + 2.0L * c0);
    const long double eb = (long double)b * (2.0L * cf[j] + (long double)om - 2.0L * c0);
    if (fabsl(ea) > 150.0L || fabsl(eb) > 150.0L) return false;
    K[j] = (double)powl(10.0L, ea);
    K[(size_t)B + j] = (double)powl(10.0L, eb);
  }
  const int L1 = c.order + 1;  // nlags - 1: the longest straddle
  T->wrap_kw.assign(B, 0.0);
  T->wrap_any = false;
  for (int j = 0; j < B; ++j) {
    if (T->reg[j].x >= L1 && T->reg[j].y <= N - L1) {
      const long double ea = (long double)a * ((long double)om - 2.0L * cf[j] + 2.0L * c0);
      const long double eb = (long double)b * (2.0L * cf[j] + (long double)om - 2.0L * c0);
      T->wrap_kw[j] = (double)powl(10.0L, 0.5L * (ea + eb));
      T->wrap_any = true;
    }
  }
  T->snap.resize(2 * (size_t)B);
  for (int sk = 0; sk < 2; ++sk) {
    std::vector<fdlp::SkSnap> t(B);
    for (int j = 0; j < B; ++j)
      t[j] = fdlp::SkSnap{sk == 0 ? N - T->reg[j].x : T->reg[j].y, j, K[(size_t)sk * B + j]};
    std::stable_sort(t.begin(), t.end(), [](const fdlp::SkSnap& u, const fdlp::SkSnap& v) { return u.S > v.S; });
    for (int j = 0; j < B; ++j) T->snap[(size_t)sk * B + j] = t[j];
    T->smin[sk] = t[B - 1].S;
  }
  flat_events(T, B);
  return true;
}

// radix split of n over the supported radices (4s first, then 2, 3, 5, 7)
bool factor_radices(int n, fdlp::DftPlan* d) {
  d->n = n;
  d->nrad = 0;
  int m = n;
  auto push = [d](int r) {
    if (d->nrad >= fdlp::kMaxRadices) return false;
    d->rad[d->nrad++] = r;
    return true;
  };
  while (m % 4 == 0) { if (!push(4)) return false; m /= 4; }
  while (m % 2 == 0) { if (!push(2)) return false; m /= 2; }
  for (int r : {3, 5, 7})
    while (m % r == 0) { if (!push(r)) return false; m /= r; }
  return m == 1;
}

// split N = N1 * N2 with both sub-DFTs LDS-resident, N1 ~ sqrt(N)
bool split_four_step(int N, fdlp::DftPlan* d1, fdlp::DftPlan* d2) {
  int best = -1;
  for (int n1 = 1; n1 <= N; ++n1) {
    if (N % n1) continue;
    const int n2 = N / n1;
    if (n1 > fdlp::kDftMaxSub || n2 > fdlp::kDftMaxSub) continue;
    fdlp::DftPlan a, b;
    if (!factor_radices(n1, &a) || !factor_radices(n2, &b)) continue;
    if (best < 0 || std::abs(n1 - n2) < std::abs(best - N / best)) best = n1;
  }
  if (best < 0) return false;
  factor_radices(best, d1);
  factor_radices(N / best, d2);
  return true;
}

double gamma_pdf(double x, double a, double loc, double scale) {
  // scipy.stats.gamma.pdf = exp(xlogy(a-1, y) - y - gammaln(a)) / scale, y = (x-loc)/scale >= 0
  const double y = (x - loc) / scale;
  if (!(y >= 0.0)) return 0.0;
  const double xl = (a - 1.0 == 0.0) ? 0.0 : (a - 1.0) * log(y);
  return exp(xl - y - lgamma(a)) / scale;
}

struct StagingHost {
  std::vector<fdlp::FrameDesc> frames;
  std::vector<fdlp::UttDesc> utts;
};

}  // namespace

struct fdlp_plan {
  fdlp_config cfg{};
  int device = 0;
  double setup_s[5] = {0, 0, 0, 0, 0};  // creation phases: host tables, device open + uploads, LPC launch
                                        // setup, workspace, total (fdlp_plan_setup_times)
  // geometry (computeFDLPSpectrogram.py / features.py float expressions)
  int N = 0, nfft = 0, hop = 0, sp_b = 0, sp_f = 0, ext = 0, env_nfft = 0, kk = 0, kkb2 = 0, ola_hop = 0;
  int B = 0, p = 0, M = 0, nlags = 0, Me = 0, ncol = 0;
  bool real_fft = false;  // even N: packed length-N/2 complex FFT
  int nfft_c = 0;         // complex FFT length N1 * N2 (N/2 or N)
  fdlp::DftPlan d1{}, d2{};
  std::vector<double> fbank_host;  // [B, ncol]
  std::vector<int> lo, hi;
  std::vector<double> weights_host;  // [3, M]
  // device constants
  fdlp::DevConsts dc{};
  double *d_fbank = nullptr, *d_hamming = nullptr, *d_weights = nullptr, *d_env_cos = nullptr,
         *d_env_win = nullptr, *d_tw1 = nullptr, *d_post = nullptr, *d_rtw = nullptr;
  double2 *d_om1 = nullptr, *d_om2 = nullptr;
  double2* d_dct1 = nullptr;         // dct_frame_kernel tables (N = 24000)
  int dct_path = FDLP_DCT_AUTO;      // fdlp_set_dct_path
  int *d_lo = nullptr, *d_hi = nullptr;
  // workspace
  int max_frames = 0;
  fdlp::Workspace ws{};
  fdlp::FrameDesc* d_frames = nullptr;
  fdlp::UttDesc* d_utts = nullptr;
  fdlp::FrameDesc* h_frames = nullptr;  // pinned staging
  fdlp::UttDesc* h_utts = nullptr;
  hipEvent_t staging_done = nullptr;
  bool staging_pending = false;
  int last_frames = 0;
  bool env_valid = false;            // ws.env holds the last batch's envelopes (fdlp_debug_fetch)
  // optional per-stage HIP-event timing (fdlp_set_profiling / fdlp_stage_times)
  bool profiling = false;
  bool debug_intermediates = false;  // keep a/gg/cep of the fused LPC kernel for fdlp_debug_fetch
  int pipeline = 1;                  // sub-batches alternated over two streams (fdlp_set_pipeline)
  hipStream_t aux_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  bool sk_avail = false;             // structured autocorrelation possible for this filterbank
  int ac_path = FDLP_AC_DIRECT;      // FDLP_AC_DIRECT, FDLP_AC_STRUCTURED or FDLP_AC_STRUCTURED_MFMA
  bool vs_avail = false;             // lag-parallel VALU sweeps possible (flat chains, lag count)
  SkirtTables sk;
  double *d_sk_e = nullptr, *r_up = nullptr, *r_flat = nullptr, *r_flat_part = nullptr;
  double *d_sk_wrap = nullptr, *r_wrap = nullptr;  // wrap-straddle factors [B] / per-frame Wrap rows [F, nlags]
  fdlp::FlatEv* d_fl_ev = nullptr;
  int2* d_fl_band = nullptr;
  fdlp::SkSnap* d_sk_snap = nullptr;
  int2* d_sk_reg = nullptr;
  // modulation-spectrum mode (computeModulationSpectrum.py)
  bool modspec = false;
  bool cplx = false;      // modspec --complex_modulation (FDLP_MODE_MODSPEC_COMPLEX)
  int L = 0;              // cplx: int(fduration srate / 2) ifft bins (computeModulationSpectrum.py:155)
  int feat_len = 0, out_dim = 0;
  double* d_faxis = nullptr;  // [coeff_n] compensate_noise multipliers, null otherwise
  std::vector<std::vector<hipEvent_t>> prof_pending;
  double prof_ms[FDLP_NUM_STAGES] = {0};
  int prof_calls = 0;
  // per-kernel marks (profiling level 2): per call, the start event then one mark per kernel (one stream)
  bool kprofiling = false;
  std::vector<std::vector<fdlp::KMark>> kmark_pending;
  double kern_ms[FDLP_NUM_KERNELS] = {0};
  int64_t kern_launches[FDLP_NUM_KERNELS] = {0};
};

// the recipes' DCT as one kernel per frame (dct_frame_kernel) unless fdlp_set_dct_path chose the
namespace fdlp {
thread_local std::vector<KMark>* g_kmarks = nullptr;
hipError_t kmark(int id, hipStream_t s) {
  if (!g_kmarks) return hipSuccess;
  const hipError_t le = hipPeekAtLastError();  // a failed launch stays the caller's hipGetLastError()
  if (le != hipSuccess) return le;
  hipEvent_t ev = nullptr;
  hipError_t e = hipEventCreate(&ev);
  if (e == hipSuccess) e = hipEventRecord(ev, s);
  if (e != hipSuccess) {
    if (ev) (void)hipEventDestroy(ev);
    return e;
  }
  g_kmarks->push_back(KMark{id, ev});
  return hipSuccess;
}
}  // namespace fdlp

// two four-step kernels
static bool dct_fused(const fdlp_plan* p) { return p->dc.dct1_tw && p->dct_path == FDLP_DCT_AUTO; }

namespace {

int drain_kmarks(fdlp_plan* p) {
  for (auto& v : p->kmark_pending) {
    if (!v.empty()) HIP_TRY(hipEventSynchronize(v.back().ev));
    for (size_t i = 1; i < v.size(); ++i) {
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, v[i - 1].ev, v[i].ev));
      const int id = v[i].id >= 0 && v[i].id < FDLP_NUM_KERNELS ? v[i].id : fdlp::kKOther;
      p->kern_ms[id] += ms;
      p->kern_launches[id]++;
    }
    for (auto& m : v) (void)hipEventDestroy(m.ev);
  }
  p->kmark_pending.clear();
  return FDLP_OK;
}

int drain_profile(fdlp_plan* p) {
  const int krc = drain_kmarks(p);
  if (krc != FDLP_OK) return krc;
  // per call: 5 events per sub-batch (stage 0..3 boundaries on its stream) + 2 around the OLA
  for (auto& ev : p->prof_pending) {
    HIP_TRY(hipEventSynchronize(ev.back()));
    const size_t nsub = (ev.size() - 2) / 5;
    for (size_t i = 0; i < nsub; ++i)
      for (int k = 0; k < 4; ++k) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, ev[5 * i + k], ev[5 * i + k + 1]));
        p->prof_ms[k] += ms;
      }
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev[ev.size() - 2], ev[ev.size() - 1]));
    p->prof_ms[4] += ms;
    p->prof_calls++;
    for (auto e : ev) (void)hipEventDestroy(e);
  }
  p->prof_pending.clear();
  return FDLP_OK;
}

int free_plan(fdlp_plan* p) {
  if (!p) return FDLP_OK;
  for (auto& ev : p->prof_pending)
    for (auto e : ev) (void)hipEventDestroy(e);
  for (auto& v : p->kmark_pending)
    for (auto& m : v) (void)hipEventDestroy(m.ev);
  void* devs[] = {p->d_fbank, p->d_hamming, p->d_weights, p->d_env_cos, p->d_env_win, p->d_tw1, p->d_post, p->d_rtw,
                  p->d_om1, p->d_om2, p->d_dct1, p->d_lo, p->d_hi, p->ws.z, p->ws.dct, p->ws.r, p->ws.a, p->ws.gg,
                  p->ws.cep, p->ws.env, p->ws.a_pad, p->d_frames, p->d_utts, p->d_sk_e, p->r_up, p->d_sk_snap,
                  p->d_sk_reg, p->d_faxis, p->r_flat, p->d_fl_ev, p->r_flat_part, p->d_fl_band, p->d_sk_wrap,
                  p->r_wrap};
  for (void* d : devs)
    if (d) (void)hipFree(d);
  if (p->h_frames) (void)hipHostFree(p->h_frames);
  if (p->h_utts) (void)hipHostFree(p->h_utts);
  if (p->staging_done) (void)hipEventDestroy(p->staging_done);
  if (p->ev_fork) (void)hipEventDestroy(p->ev_fork);
  if (p->ev_join) (void)hipEventDestroy(p->ev_join);
  if (p->aux_stream) (void)hipStreamDestroy(p->aux_stream);
  delete p;
  return FDLP_OK;
}

template <typename T>
int upload(T** dst, const T* src, size_t n) {
  HIP_TRY(hipMalloc((void**)dst, sizeof(T) * std::max<size_t>(n, 1)));
  if (n) HIP_TRY(hipMemcpy(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice));
  return FDLP_OK;
}

int64_t frames_of(const fdlp_plan* p, int64_t T) {
  // getFrames: idx = sp_b + k*hop, yield while idx + sp_f < T + 2*ext  (features.py:151)
  const int64_t lim = T + 2 * (int64_t)p->ext - p->sp_b - p->sp_f;  // k*hop < lim
  if (lim <= 0) return 0;
  return (lim - 1) / p->hop + 1;
}

int64_t out_of(const fdlp_plan* p, int64_t T) {
  if (p->modspec) return frames_of(p, T);  // one row per analysis frame (computeModulationSpectrum.py:161)
  // int(np.ceil(T*frate/srate))  (computeFDLPSpectrogram.py:182)
  return (int64_t)ceil((double)(T * (int64_t)p->cfg.frate) / (double)p->cfg.srate);
}

// OLA slices of computeFDLPSpectrogram.py:207-225 (see oracle.ola_plan for the numpy rules)
int ola_table(const fdlp_plan* p, int F, int L, const uint8_t* jit, int32_t* dst, int32_t* src, int32_t* cnt) {
  int64_t ptr = 0;
  const int kk = p->kk, kkb2 = p->kkb2;
  for (int i = 0; i < F; ++i) {
    if (i == 0) {
      if (L < kkb2) {
        const int rhs = std::max(0, std::min(L, kk - kkb2));
        if (rhs != L) return fail(FDLP_E_BROADCAST, "reference OLA would fail to broadcast (frame 0)");
        dst[i] = 0; src[i] = kkb2; cnt[i] = L;
      } else {
        if (kk - kkb2 != kkb2) return fail(FDLP_E_BROADCAST, "reference OLA would fail to broadcast (frame 0)");
        dst[i] = 0; src[i] = kkb2; cnt[i] = kkb2;
      }
    } else if (i == F - 1 || i == F - 2) {
      const int64_t n = (int64_t)L - ptr;
      if (kk >= n) {
        const int64_t lhs = std::max<int64_t>(0, n);
        const int64_t rhs = n >= 0 ? n : std::max<int64_t>(0, kk + n);
        if (lhs != rhs) return fail(FDLP_E_BROADCAST, "reference OLA would fail to broadcast (tail frame)");
        dst[i] = (int32_t)ptr; src[i] = 0; cnt[i] = (int32_t)lhs;
      } else {
        dst[i] = (int32_t)ptr; src[i] = 0; cnt[i] = kk;
      }
    } else {
      if (ptr + kk > L) return fail(FDLP_E_BROADCAST, "reference OLA would fail to broadcast (middle frame)");
      dst[i] = (int32_t)ptr; src[i] = 0; cnt[i] = kk;
    }
    if (i == 0) ptr = ptr + p->ola_hop - kkb2;
    else ptr = ptr + p->ola_hop + (jit ? jit[i - 1] : 0);
  }
  return FDLP_OK;
}

}  // namespace

extern "C" {

const char* fdlp_last_error(void) { return fdlp::last_error_slot().c_str(); }
int fdlp_abi_version(void) { return FDLP_ABI_VERSION; }

int fdlp_mapped_ptr(void* host, void** dev) {
  if (!host || !dev) return fail(FDLP_E_INVALID, "fdlp_mapped_ptr: bad args");
  if (hipHostGetDevicePointer(dev, host, 0) != hipSuccess)
    return fail(FDLP_E_INVALID, "fdlp_mapped_ptr: not pinned host memory (hipHostMalloc / hipHostRegister)");
  return FDLP_OK;
}

int fdlp_plan_create(const fdlp_config* cfg, int device, fdlp_plan** out) {
  if (!cfg || !out) return fail(FDLP_E_INVALID, "fdlp_plan_create: null argument");
  *out = nullptr;
  const fdlp_config& c = *cfg;
  if (c.nfilters < 1 || c.order < 1 || c.coeff_num < 2 || c.srate < 1 || c.frate < 1 || !(c.fduration > 0))
    return fail(FDLP_E_INVALID, "invalid configuration (nfilters>=1, order>=1, coeff_num>=2 required)");
  if (c.max_frames < 1) return fail(FDLP_E_INVALID, "max_frames must be >= 1");
  auto* p = new (std::nothrow) fdlp_plan;
  if (!p) return fail(FDLP_E_NOMEM, "out of memory");
  const auto t_begin = std::chrono::steady_clock::now();
  auto t_last = t_begin;
  auto phase = [&](int k) {  // seconds since the previous phase boundary into setup_s[k]
    const auto t = std::chrono::steady_clock::now();
    p->setup_s[k] = std::chrono::duration<double>(t - t_last).count();
    p->setup_s[4] = std::chrono::duration<double>(t - t_begin).count();
    t_last = t;
  };
  p->cfg = c;
  p->cfg.lifter = nullptr;
  p->device = device;
  int rc;
#define PLAN_FAIL(code, msg) do { rc = fail(code, msg); free_plan(p); return rc; } while (0)
#define PLAN_TRY(expr) do { rc = (expr); if (rc != FDLP_OK) { std::string m_ = fdlp::last_error_slot(); free_plan(p); fdlp::last_error_slot() = m_; return rc; } } while (0)

  // geometry, same float expressions as the reference
  const double ov = 1.0 - c.overlap_fraction;                        // :104
  p->N = (int)((double)c.srate * c.fduration);                       // features.py:134
  const double lfr = 1.0 / (ov * c.fduration);                       // :174
  p->hop = (int)((double)c.srate / lfr);                             // features.py:135
  p->modspec = c.mode == FDLP_MODE_MODSPEC || c.mode == FDLP_MODE_MODSPEC_COMPLEX;
  p->cplx = c.mode == FDLP_MODE_MODSPEC_COMPLEX;
  if (c.mode != FDLP_MODE_SPECTROGRAM && !p->modspec) PLAN_FAIL(FDLP_E_INVALID, "unknown plan mode");
  p->L = (int)(c.fduration * (double)c.srate / 2.0);  // cos_trans[:, :int(fduration * srate / 2)] (:155)
  if (p->modspec) p->hop = (int)((double)c.srate / (double)c.frate);  // getFrames(.., frate, ..) (:150-151)
  if (p->N % 2 == 0) { p->sp_b = p->N / 2 - 1; p->sp_f = p->N / 2; p->ext = p->N / 2 - 1; }
  else { p->sp_b = p->sp_f = p->ext = (p->N - 1) / 2; }
  p->nfft = (int)(2.0 * c.fduration * (double)c.srate);              // :53, :59
  if (p->cplx) p->nfft = (int)(c.fduration * (double)c.srate);        // dur (computeModulationSpectrum.py:45-46)
  p->env_nfft = 2 * (int)(c.fduration * (double)c.frate);            // :201
  p->kk = (int)nearbyint(c.fduration * (double)c.frate);             // :203 (np.round: half-even)
  p->kkb2 = (int)nearbyint(c.fduration * (double)c.frate / 2.0);     // :204
  p->ola_hop = (int)nearbyint(c.fduration * (double)c.frate * ov);   // :220
  p->B = c.nfilters;
  p->p = c.order;
  p->M = c.coeff_num;
  p->nlags = c.order + 2;
  if (p->modspec) {  // no envelope / OLA: a minimal envelope for the shared LPC kernel, output = cepstra
    p->env_nfft = 2; p->kk = 1; p->kkb2 = 0; p->ola_hop = 1;
    if (c.coeff_0 < 1 || c.coeff_0 > c.coeff_num) PLAN_FAIL(FDLP_E_INVALID, "modspec needs 1 <= coeff_0 <= coeff_n");
    if (c.gamma_enabled || c.lifter || c.odd_mod_zero) PLAN_FAIL(FDLP_E_INVALID, "modspec takes no gamma/lifter/odd options");
    const int sel = c.coeff_num - c.coeff_0 + 1;                     // coeff_num (:64)
    p->feat_len = c.keep_even ? ((c.coeff_0 % 2 == 0) ? sel / 2 : (sel + 1) / 2)  // :66-80
                  : (p->cplx && !c.absolute_value ? 2 * sel : sel);
    if (p->feat_len < 1) PLAN_FAIL(FDLP_E_INVALID, "modspec selects no coefficient");
    if (p->cplx && c.keep_even && !c.absolute_value)  // temp2 has 2 sel values, feat_len ~ sel / 2 (:191-197)
      PLAN_FAIL(FDLP_E_INVALID, "complex_modulation with keep_even needs absolute_value (reference broadcast error)");
    if (p->cplx && c.coeff_num > 1024) PLAN_FAIL(FDLP_E_INVALID, "complex_modulation: coeff_n too large (max 1024)");
  }
  p->Me = std::min(p->M, p->env_nfft);
  p->out_dim = p->modspec ? c.nfilters * p->feat_len : c.nfilters;
  if (p->N < 2 || p->hop < 1) PLAN_FAIL(FDLP_E_INVALID, "frame length / hop too small");
  if (p->kk < 1 || p->env_nfft < 1 || p->kk > p->env_nfft) PLAN_FAIL(FDLP_E_INVALID, "fduration*frate too small");
  if (!p->modspec && p->ola_hop < p->kkb2) PLAN_FAIL(FDLP_E_INVALID, "unsupported: negative OLA pointer (overlap too large)");
  if (fdlp::autocorr_tiles(p->nlags) > 16) PLAN_FAIL(FDLP_E_INVALID, "order too large (max 238)");
  if (p->N < 1024) PLAN_FAIL(FDLP_E_INVALID, "frame length int(srate*fduration) must be >= 1024 samples");
  if ((p->p + 1 + 15) / 16 > 15) PLAN_FAIL(FDLP_E_INVALID, "order too large for the Levinson kernel");
  if (p->kk > 256) PLAN_FAIL(FDLP_E_INVALID, "fduration*frate too large (envelope > 256 samples)");
  if (p->M > 4096) PLAN_FAIL(FDLP_E_INVALID, "coeff_num too large (max 4096)");
  p->real_fft = !p->cplx && p->N % 2 == 0 && split_four_step(p->N / 2, &p->d1, &p->d2);
  p->nfft_c = p->real_fft ? p->N / 2 : p->N;  // complex FFT length of the DCT
  if (!p->real_fft && !split_four_step(p->nfft_c, &p->d1, &p->d2))
    PLAN_FAIL(FDLP_E_INVALID, "frame length int(srate*fduration) has no supported 2/3/5/7 four-step split");

  // skirt tables and the DFT twiddle tables need only the configuration: built on helper threads while
  // the filterbank is computed (plan creation is on the CLI's critical path)
  bool sk_ok = false;
  std::thread sk_thread([&] { sk_ok = !p->cplx && skirt_tables(c, p->B, p->N, p->nfft, &p->sk); });
  const int N1 = p->d1.n, N2 = p->d2.n, NC = p->nfft_c;
  std::vector<double> tw1(2 * (size_t)N1 * N2), post(2 * (size_t)p->N), rtw(2 * (size_t)std::max(1, p->N / 2));
  std::vector<double2> om1, om2;
  std::thread tw_thread([&] {
    const int N = p->N;
    const long double PI = 3.141592653589793238462643383279502884L;
    for (int k1 = 0; k1 < N1; ++k1)
      for (int n2 = 0; n2 < N2; ++n2) {
        const long long q = ((long long)k1 * n2) % NC;
        const long double ang = -2.0L * PI * (long double)q / (long double)NC;
        tw1[2 * ((size_t)k1 * N2 + n2)] = (double)cosl(ang);
        tw1[2 * ((size_t)k1 * N2 + n2) + 1] = (double)sinl(ang);
      }
    for (int k = 0; k < N / 2; ++k) {
      const long double ang = -2.0L * PI * (long double)k / (long double)N;
      rtw[2 * k] = (double)cosl(ang);
      rtw[2 * k + 1] = (double)sinl(ang);
    }
    for (int k = 0; k < N; ++k) {
      const long double ang = -PI * (long double)k / (2.0L * (long double)N);
      post[2 * k] = (double)cosl(ang);
      post[2 * k + 1] = (double)sinl(ang);
    }
    auto omega = [&](int n) {
      std::vector<double2> om(n);
      for (int q = 0; q < n; ++q) {
        const long double ang = -2.0L * PI * (long double)q / (long double)n;
        om[q] = make_double2((double)cosl(ang), (double)sinl(ang));
      }
      return om;
    };
    om1 = omega(N1);
    om2 = omega(N2);
  });
  auto join_helpers = [&] {
    if (sk_thread.joinable()) sk_thread.join();
    if (tw_thread.joinable()) tw_thread.join();
  };
  // filterbank (:49-63)
  if (c.fbank_kind == FDLP_FBANK_MEL) {
    p->fbank_host = fbank_mel(p->B, p->nfft, c.srate, c.warp_fact, &p->ncol);
  } else if (c.fbank_kind == FDLP_FBANK_COCHLEAR) {
    p->fbank_host = fbank_cochlear(p->B, p->nfft, c.srate, c.om_w, c.alp, c.fixed, c.bet, c.warp_fact, &p->ncol);
  } else {
    join_helpers();
    PLAN_FAIL(FDLP_E_INVALID, "Invalid type of filter bank, use mel or cochlear with proper configuration");
  }
  const int width = p->cplx ? p->L : p->N;  // taps of filt = fbank[j, :-1]
  if (p->ncol - 1 != width) {  // filt (ncol-1 taps) * cos_trans[i, :] (N, or L ifft bins) must broadcast (:190-191)
    join_helpers();
    PLAN_FAIL(FDLP_E_INVALID, "filterbank width nfft/2 does not match the frame length (reference broadcast error)");
  }
  if (p->cplx && p->nlags > p->L) {
    join_helpers();
    PLAN_FAIL(FDLP_E_INVALID, "complex_modulation: order + 2 exceeds the ifft bins");
  }
  std::vector<double> dense((size_t)p->B * p->N);  // rows of N (cplx: the L taps, zeros beyond)
  p->lo.assign(p->B, 0);
  p->hi.assign(p->B, 0);
  for (int j = 0; j < p->B; ++j) {
    const double* row = &p->fbank_host[(size_t)j * p->ncol];
    double peak = 0.0;
    for (int m = 0; m < width; ++m) peak = std::max(peak, std::fabs(row[m]));
    const double thr = c.support_eps > 0 && !p->cplx ? c.support_eps * peak : 0.0;
    int lo = p->N, hi = 0;
    for (int m = 0; m < width; ++m) {
      dense[(size_t)j * p->N + m] = row[m];
      const bool keep = thr > 0 ? std::fabs(row[m]) >= thr : row[m] != 0.0;
      if (keep) { lo = std::min(lo, m); hi = m + 1; }
    }
    if (hi <= lo) { lo = 0; hi = 0; }
    p->lo[j] = lo;
    p->hi[j] = hi;
  }

  join_helpers();
  p->sk_avail = sk_ok;
  p->vs_avail = p->sk_avail && p->sk.fl_C > 0 && fdlp::vsweep_chains(p->sk.fl_C) > 0 &&
                fdlp::vsweep_lanes_lags(p->nlags) > 0;
  // the other paths are selected explicitly (fdlp_set_autocorr_path), never from the environment
  p->ac_path = !p->sk_avail ? FDLP_AC_DIRECT : p->vs_avail ? FDLP_AC_STRUCTURED : FDLP_AC_STRUCTURED_MFMA;

  // modulation weights (:94-118)
  const int M = p->M;
  p->weights_host.assign((size_t)3 * M, 1.0);
  for (int i = 0; i < M; ++i) p->weights_host[i] = (p->modspec || (i >= c.coeff_lp && i <= c.coeff_hp)) ? 1.0 : 0.0;
  if (cfg->lifter) {
    if (cfg->lifter_len != M) PLAN_FAIL(FDLP_E_INVALID, "lifter_config must hold coeff_num values (reference broadcast)");
    for (int i = 0; i < M; ++i) p->weights_host[M + i] = cfg->lifter[i];
  }
  if (c.gamma_enabled) {
    if (c.order != M) PLAN_FAIL(FDLP_E_INVALID, "gamma_weight has length order and needs order == coeff_num (reference broadcast)");
    const std::vector<double> x = linspace(0.0, (double)(c.order - 1), c.order);  // :110
    const double scale = c.gamma_scale, shape = c.gamma_shape;
    const double pk_req = c.gamma_pk * (2.0 * c.fduration);                       // :114-115
    const double pk = (shape - 1.0) * scale;                                      // :116
    const double loc = -pk + pk_req;                                              // :117
    for (int i = 0; i < M; ++i) p->weights_host[2 * M + i] = gamma_pdf(x[i], shape, loc, scale) * 3.0 * scale;
  }

  // windows and tables
  // analysis window: np.hamming (spectrogram, :29), np.hanning (modspec default :30), ones (--no_window)
  std::vector<double> ham;
  if (c.window == FDLP_WIN_HAMMING) ham = cos_window(p->N, 0.54, 0.46);
  else if (c.window == FDLP_WIN_HANNING) ham = cos_window(p->N, 0.5, 0.5);
  else if (c.window == FDLP_WIN_RECT) ham.assign(p->N, 1.0);
  else PLAN_FAIL(FDLP_E_INVALID, "unknown analysis window");
  const std::vector<double> hann_k = cos_window(p->kk, 0.5, 0.5), hamm_k = cos_window(p->kk, 0.54, 0.46);
  std::vector<double> env_win(2 * (size_t)p->kk);
  // ms[0:kk] * np.hanning(kk) / window(kk) (computeFDLPSpectrogram.py:205) as one multiplication by the
  // ratio, rounded once here (a 1-ulp difference from the reference's two roundings; no fp64 division
  // per envelope sample on the device).  [2t + 1] stays 1.0 for the kernels that still divide.
  for (int t = 0; t < p->kk; ++t) { env_win[2 * t] = hann_k[t] / hamm_k[t]; env_win[2 * t + 1] = 1.0; }
  std::vector<double> env_cos(p->env_nfft);
  for (int q = 0; q < p->env_nfft; ++q)
    env_cos[q] = (double)cosl(2.0L * (long double)M_PI * (long double)q / (long double)p->env_nfft);
  const int N = p->N;

  p->max_frames = c.max_frames;
  if (device < 0) {  // host-only plan: geometry, filterbank, weights and OLA tables, no compute
    phase(0);
    *out = p;
    return FDLP_OK;
  }
  phase(0);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) PLAN_FAIL(FDLP_E_HIP, "no HIP device visible");
  if (device < 0 || device >= ndev) PLAN_FAIL(FDLP_E_INVALID, "device index out of range");
  DeviceGuard dg(device);  // restored when plan creation returns
  if (dg.status() != hipSuccess) PLAN_FAIL(FDLP_E_HIP, "hipSetDevice failed");
  PLAN_TRY(upload(&p->d_fbank, dense.data(), dense.size()));
  PLAN_TRY(upload(&p->d_lo, p->lo.data(), p->lo.size()));
  PLAN_TRY(upload(&p->d_hi, p->hi.data(), p->hi.size()));
  PLAN_TRY(upload(&p->d_hamming, ham.data(), ham.size()));
  if (p->modspec && c.compensate_noise) {  // faxis = linspace(0, coeff_num / (2 fduration), coeff_n) (:86-88)
    // complex: linspace(0, coeff_num / fduration, coeff_n) (:83-85)
    const double fmax = (double)(c.coeff_num - c.coeff_0 + 1) / ((p->cplx ? 1.0 : 2.0) * c.fduration);
    const std::vector<double> fax = linspace(0.0, fmax, c.coeff_num);
    PLAN_TRY(upload(&p->d_faxis, fax.data(), fax.size()));
  }
  PLAN_TRY(upload(&p->d_weights, p->weights_host.data(), p->weights_host.size()));
  PLAN_TRY(upload(&p->d_env_cos, env_cos.data(), env_cos.size()));
  PLAN_TRY(upload(&p->d_env_win, env_win.data(), env_win.size()));
  PLAN_TRY(upload(&p->d_tw1, tw1.data(), tw1.size()));
  PLAN_TRY(upload(&p->d_post, post.data(), post.size()));
  PLAN_TRY(upload(&p->d_rtw, rtw.data(), rtw.size()));
  PLAN_TRY(upload(&p->d_om1, om1.data(), om1.size()));
  PLAN_TRY(upload(&p->d_om2, om2.data(), om2.size()));
  if (p->real_fft && !p->cplx) {  // the recipes' N = 24000: one DCT kernel per frame
    const std::vector<double2> dct1 = fdlp::dct_frame_tables(N, ham);
    if (!dct1.empty()) PLAN_TRY(upload(&p->d_dct1, dct1.data(), dct1.size()));
  }

  fdlp::DevConsts& d = p->dc;
  d.B = p->B; d.N = N; d.hop = p->hop; d.ext = p->ext; d.p = p->p; d.nlags = p->nlags; d.M = M; d.Me = p->Me;
  d.kk = p->kk; d.env_nfft = p->env_nfft;
  d.fbank = p->d_fbank; d.lo = p->d_lo; d.hi = p->d_hi; d.hamming = p->d_hamming; d.weights = p->d_weights;
  d.env_cos = p->d_env_cos; d.env_win = p->d_env_win; d.tw1 = p->d_tw1; d.post = p->d_post;
  d.rtw = p->d_rtw; d.real_fft = p->real_fft ? 1 : 0; d.natural = p->cplx ? 1 : 0;
  d.dct1_tw = p->d_dct1;
  if (p->sk_avail) {
    PLAN_TRY(upload(&p->d_sk_e, p->sk.e.data(), p->sk.e.size()));
    PLAN_TRY(upload(&p->d_sk_snap, p->sk.snap.data(), p->sk.snap.size()));
    PLAN_TRY(upload(&p->d_sk_reg, p->sk.reg.data(), p->sk.reg.size()));
    d.sk_e = p->d_sk_e; d.sk_snap = p->d_sk_snap; d.sk_reg = p->d_sk_reg;
    d.sk_min[0] = p->sk.smin[0]; d.sk_min[1] = p->sk.smin[1];
    if (p->vs_avail) {
      PLAN_TRY(upload(&p->d_fl_ev, p->sk.fl.data(), p->sk.fl.size()));
      d.fl_ev = p->d_fl_ev; d.fl_nev = (int)p->sk.fl.size(); d.fl_C = p->sk.fl_C;
      d.fl_lo = p->sk.fl_lo; d.fl_hi = p->sk.fl_hi;
      PLAN_TRY(upload(&p->d_fl_band, p->sk.fl_band.data(), p->sk.fl_band.size()));
      d.fl_band = p->d_fl_band; d.fl_H = p->sk.fl_H;
      if (p->sk.wrap_any) {
        PLAN_TRY(upload(&p->d_sk_wrap, p->sk.wrap_kw.data(), p->sk.wrap_kw.size()));
        d.sk_wrap = p->d_sk_wrap;
      }
      for (int h = 0; h < fdlp::kMaxFlatParts; ++h) { d.fl_part_lo[h] = p->sk.part_lo[h]; d.fl_part_hi[h] = p->sk.part_hi[h]; }
      for (int h = 0; h <= fdlp::kMaxFlatParts; ++h) d.fl_part_ev[h] = p->sk.part_ev[h];
    }
  }

  phase(1);
  // launch geometry of the persistent LPC kernel for this device (occupancy, large-LDS attribute)
  if (fdlp::prepare_lpc_env(d) != hipSuccess) PLAN_FAIL(FDLP_E_HIP, "LPC kernel launch setup failed");
  phase(2);

  // workspace
  const size_t F = (size_t)c.max_frames, items = F * p->B;
  p->max_frames = c.max_frames;
  if ((!dct_fused(p) && hipMalloc((void**)&p->ws.z, sizeof(double2) * F * p->nfft_c) != hipSuccess) ||
      hipMalloc((void**)&p->ws.dct, sizeof(double) * F * N) != hipSuccess ||
      hipMalloc((void**)&p->ws.r, sizeof(double) * (items * p->nlags * (p->cplx ? 2 : 1) + fdlp::kRowSlack)) != hipSuccess ||
      hipMalloc((void**)&p->ws.gg, sizeof(double) * items) != hipSuccess ||
      (d.lpc_split && hipMalloc((void**)&p->ws.a_pad, sizeof(double) * items * d.lpc_astride) != hipSuccess) ||
      (p->modspec && hipMalloc((void**)&p->ws.cep, sizeof(double) * items * M) != hipSuccess) ||
      hipMalloc((void**)&p->ws.env, sizeof(double) * items * p->kk) != hipSuccess ||
      (p->sk_avail && hipMalloc((void**)&p->r_up, sizeof(double) * (items * p->nlags + fdlp::kRowSlack)) != hipSuccess) ||
      (p->vs_avail && hipMalloc((void**)&p->r_flat, sizeof(double) * (items * p->nlags + fdlp::kRowSlack)) != hipSuccess) ||
      (p->vs_avail && p->d_sk_wrap && hipMalloc((void**)&p->r_wrap, sizeof(double) * (F * p->nlags + fdlp::kRowSlack)) != hipSuccess) ||
      (p->vs_avail && p->sk.fl_H > 1 &&
       hipMalloc((void**)&p->r_flat_part, sizeof(double) * (F * (p->sk.fl_H - 1) * fdlp::kMaxChains * p->nlags + fdlp::kRowSlack)) !=
           hipSuccess) ||
      hipMalloc((void**)&p->d_frames, sizeof(fdlp::FrameDesc) * F) != hipSuccess ||
      hipMalloc((void**)&p->d_utts, sizeof(fdlp::UttDesc) * F) != hipSuccess ||
      hipHostMalloc((void**)&p->h_frames, sizeof(fdlp::FrameDesc) * F, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&p->h_utts, sizeof(fdlp::UttDesc) * F, hipHostMallocDefault) != hipSuccess ||
      hipEventCreateWithFlags(&p->staging_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&p->aux_stream, hipStreamNonBlocking) != hipSuccess)
    PLAN_FAIL(FDLP_E_NOMEM, "workspace allocation failed (reduce max_frames)");
  phase(3);
#undef PLAN_FAIL
#undef PLAN_TRY
  *out = p;
  return FDLP_OK;
}

int fdlp_plan_setup_times(const fdlp_plan* p, double* sec) {
  if (!p || !sec) return fail(FDLP_E_INVALID, "fdlp_plan_setup_times: bad args");
  for (int k = 0; k < 5; ++k) sec[k] = p->setup_s[k];
  return FDLP_OK;
}

int fdlp_plan_destroy(fdlp_plan* plan) {
  if (plan && plan->device >= 0) (void)hipDeviceSynchronize();
  return free_plan(plan);
}

int fdlp_geometry(const fdlp_plan* p, int64_t T, int32_t* F, int32_t* L) {
  if (!p || T < 0) return fail(FDLP_E_INVALID, "fdlp_geometry: bad args");
  if (F) *F = (int32_t)frames_of(p, T);
  if (L) *L = (int32_t)out_of(p, T);
  return FDLP_OK;
}

int fdlp_plan_out_dim(const fdlp_plan* p, int32_t* dim) {
  if (!p || !dim) return fail(FDLP_E_INVALID, "fdlp_plan_out_dim: bad args");
  *dim = p->out_dim;
  return FDLP_OK;
}

int fdlp_plan_info(const fdlp_plan* p, int32_t* N, int32_t* hop, int32_t* nlags, int32_t* kk, int32_t* ola_hop) {
  if (!p) return fail(FDLP_E_INVALID, "fdlp_plan_info: null plan");
  if (N) *N = p->N;
  if (hop) *hop = p->hop;
  if (nlags) *nlags = p->nlags;
  if (kk) *kk = p->kk;
  if (ola_hop) *ola_hop = p->ola_hop;
  return FDLP_OK;
}

int fdlp_plan_fbank(const fdlp_plan* p, double* fbank_out, int32_t* lo, int32_t* hi) {
  if (!p) return fail(FDLP_E_INVALID, "fdlp_plan_fbank: null plan");
  if (fbank_out) memcpy(fbank_out, p->fbank_host.data(), sizeof(double) * p->fbank_host.size());
  for (int j = 0; j < p->B; ++j) {
    if (lo) lo[j] = p->lo[j];
    if (hi) hi[j] = p->hi[j];
  }
  return FDLP_OK;
}

int fdlp_make_fbank(const fdlp_config* c, int32_t nfft, double* out, int32_t* ncol) {
  if (!c || !out || nfft < 2 || c->nfilters < 1 || c->srate < 1) return fail(FDLP_E_INVALID, "fdlp_make_fbank: bad args");
  int n = 0;
  std::vector<double> W;
  if (c->fbank_kind == FDLP_FBANK_MEL) W = fbank_mel(c->nfilters, nfft, c->srate, c->warp_fact, &n);
  else if (c->fbank_kind == FDLP_FBANK_COCHLEAR)
    W = fbank_cochlear(c->nfilters, nfft, c->srate, c->om_w, c->alp, c->fixed, c->bet, c->warp_fact, &n);
  else return fail(FDLP_E_INVALID, "Invalid type of filter bank, use mel or cochlear with proper configuration");
  memcpy(out, W.data(), sizeof(double) * W.size());
  if (ncol) *ncol = n;
  return FDLP_OK;
}

int fdlp_plan_weights(const fdlp_plan* p, double* w_out) {
  if (!p || !w_out) return fail(FDLP_E_INVALID, "fdlp_plan_weights: bad args");
  // folded product in the reference's multiplication order; odd zeroing applied after
  for (int i = 0; i < p->M; ++i) {
    double v = p->weights_host[i] * p->weights_host[p->M + i] * p->weights_host[2 * p->M + i];
    if (p->cfg.odd_mod_zero && (i & 1)) v = 0.0;
    w_out[i] = v;
  }
  return FDLP_OK;
}

int fdlp_ola_table(const fdlp_plan* p, int64_t T, const uint8_t* jitter, int32_t* dst, int32_t* src, int32_t* cnt) {
  if (!p || !dst || !src || !cnt) return fail(FDLP_E_INVALID, "fdlp_ola_table: bad args");
  return ola_table(p, (int)frames_of(p, T), (int)out_of(p, T), jitter, dst, src, cnt);
}

int fdlp_compute(fdlp_plan* p, const fdlp_batch* b, void* stream) {
  if (!p || !b) return fail(FDLP_E_INVALID, "fdlp_compute: null argument");
  if (b->n_utt < 0 || (b->n_utt > 0 && (!b->pcm_dev || !b->pcm_off || !b->utt_len || !b->out_row)))
    return fail(FDLP_E_INVALID, "fdlp_compute: missing batch arrays");
  if (b->pcm_kind != FDLP_PCM_I16 && b->pcm_kind != FDLP_PCM_F64) return fail(FDLP_E_INVALID, "bad pcm_kind");
  if (b->noise_dev && (!b->noise_off || !b->noise_alpha))
    return fail(FDLP_E_INVALID, "noise mixing needs noise_off and noise_alpha");
  if (b->preprocess != FDLP_PRE_NONE && b->preprocess != FDLP_PRE_DIFF) return fail(FDLP_E_INVALID, "bad preprocess");
  if (b->preprocess == FDLP_PRE_DIFF && b->noise_dev)
    return fail(FDLP_E_INVALID, "diff preprocessing and noise mixing are exclusive (computeFDLPSpectrogram.py:160-166)");
  if (!b->out_dev && !b->out_f64_dev && !b->out_q_dev) return fail(FDLP_E_INVALID, "fdlp_compute: no output buffer");
  if (b->out_q_dev && (b->ark_decimals < 0 || !b->out_q_flag_dev || p->modspec))
    return fail(FDLP_E_INVALID, "fdlp_compute: out_q_dev needs ark_decimals >= 0, out_q_flag_dev and a spectrogram plan");
  if (p->device < 0) return fail(FDLP_E_INVALID, "fdlp_compute: host-only plan (created with device < 0)");
  hipStream_t s = (hipStream_t)stream;
  DeviceGuard dg(p->device);  // the caller's current device is restored on return
  HIP_TRY(dg.status());
  // staging buffers may still feed the previous call's copies
  if (p->staging_pending) {
    HIP_TRY(hipEventSynchronize(p->staging_done));
    p->staging_pending = false;
  }
  int64_t nf = 0;
  int maxL = 0;
  const uint8_t* jit = b->jitter;
  std::vector<int32_t> dst, src, cnt;
  for (int u = 0; u < b->n_utt; ++u) {
    const int64_t T = b->utt_len[u];
    const int64_t F = frames_of(p, T), L = out_of(p, T);
    if (F < 1) return fail(FDLP_E_INVALID, "utterance too short: no analysis frame (scipy dct of an empty array)");
    if (L > INT32_MAX / 2) return fail(FDLP_E_INVALID, "utterance too long");
    if (nf + F > p->max_frames) return fail(FDLP_E_CAPACITY, "batch exceeds the plan's max_frames");
    if (b->noise_dev && b->noise_off[u] < 0) return fail(FDLP_E_INVALID, "negative noise offset");
    dst.assign(F, 0); src.assign(F, 0); cnt.assign(F, 0);
    if (!p->modspec) {
      int rc = ola_table(p, (int)F, (int)L, jit, dst.data(), src.data(), cnt.data());
      if (rc != FDLP_OK) return rc;
      if (jit) jit += F - 1;
    }
    for (int64_t k = 0; k < F; ++k) {
      fdlp::FrameDesc& fd = p->h_frames[nf + k];
      fd.pcm_off = b->pcm_off[u];
      fd.noise_off = b->noise_dev ? b->noise_off[u] : -1;
      fd.alpha = b->noise_dev ? b->noise_alpha[u] : 0.0;
      fd.T = (int32_t)T;
      fd.k = (int32_t)k;
      fd.dst = dst[k]; fd.src = src[k]; fd.cnt = cnt[k];
      fd.utt = u;
    }
    fdlp::UttDesc& ud = p->h_utts[u];
    ud.out_row = b->out_row[u];
    ud.L = (int32_t)L;
    ud.frame0 = (int32_t)nf;
    ud.F = (int32_t)F;
    ud.pad = 0;
    maxL = std::max(maxL, (int)L);
    nf += F;
  }
  p->last_frames = (int)nf;
  if (nf == 0) return FDLP_OK;
  // Sub-batches alternate between the caller's stream and the plan's second stream so that the
  // MFMA-bound autocorrelation of one overlaps the VALU-bound DFT / LPC kernels of the other.
  const int nsub = (int)std::max<int64_t>(1, std::min<int64_t>(p->pipeline, nf / 256));
  HIP_TRY(hipMemcpyAsync(p->d_frames, p->h_frames, sizeof(fdlp::FrameDesc) * nf, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(p->d_utts, p->h_utts, sizeof(fdlp::UttDesc) * b->n_utt, hipMemcpyHostToDevice, s));
  HIP_TRY(hipEventRecord(p->staging_done, s));
  p->staging_pending = true;
  p->env_valid = !p->modspec;

  std::vector<hipEvent_t> ev;
  if (p->profiling) {
    if (p->prof_pending.size() >= 64) {
      int rc = drain_profile(p);
      if (rc != FDLP_OK) return rc;
    }
    ev.resize(5 * (size_t)nsub + 2);
    for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
  }
  // per-kernel marks (one sub-batch: every kernel on stream s): a start event, then one per kernel launch
  std::vector<fdlp::KMark> kmarks;
  const bool kprof = p->profiling && p->kprofiling && nsub == 1;
  if (kprof) {
    hipEvent_t e0 = nullptr;
    HIP_TRY(hipEventCreate(&e0));
    kmarks.push_back(fdlp::KMark{-1, e0});
    HIP_TRY(hipEventRecord(e0, s));
    fdlp::g_kmarks = &kmarks;
  }
  struct KmarkScope {  // an early error return: stop collecting and free the marks of this call
    bool on;
    std::vector<fdlp::KMark>& v;
    ~KmarkScope() {
      if (!on) return;
      fdlp::g_kmarks = nullptr;
      for (auto& m : v) (void)hipEventDestroy(m.ev);
    }
  } kscope{kprof, kmarks};
  // frames [f0, f0 + n) of sub-batch i: everything up to the envelopes is independent per frame
  auto run_frames = [&](int i, int64_t f0, int n, hipStream_t st) -> int {
    auto mark = [&](int k) -> hipError_t { return p->profiling ? hipEventRecord(ev[5 * i + k], st) : hipSuccess; };
    const size_t N = (size_t)p->N, B = (size_t)p->B, nl = (size_t)p->nlags;
    const size_t it0 = (size_t)f0 * B;
    const int its = n * p->B;
    double* r = p->ws.r + it0 * nl;
    double* env = p->ws.env + it0 * p->kk;
    double* a_dbg = p->debug_intermediates ? p->ws.a + it0 * (p->p + 1) : nullptr;
    double* gg_dbg = p->debug_intermediates ? p->ws.gg + it0 : nullptr;
    double* cep_dbg = (p->debug_intermediates || p->modspec) ? p->ws.cep + it0 * p->M : nullptr;
    HIP_TRY(mark(0));
    // the sample gather's kinds: 0 int16, 1 float64 values of another WAV dtype, 2 / 3 the diff filter on them
    const int pcm_kind = b->preprocess == FDLP_PRE_DIFF ? (b->pcm_kind == FDLP_PCM_I16 ? 2 : 3) : b->pcm_kind;
    if (dct_fused(p)) {  // one kernel per frame; the second DCT stage mark follows it directly
      HIP_TRY(fdlp::launch_dct_frame(p->dc, b->pcm_dev, pcm_kind, b->noise_dev, p->d_frames + f0, nullptr, n,
                                     p->ws.dct + f0 * N, st));
      HIP_TRY(mark(1));
    } else {
      HIP_TRY(fdlp::launch_frames_dft1(p->dc, p->d1, p->d2.n, b->pcm_dev, pcm_kind, b->noise_dev, p->d_frames + f0,
                                       nullptr, n, p->ws.z + f0 * p->nfft_c, p->d_om1, st));
      HIP_TRY(mark(1));
      HIP_TRY(fdlp::launch_dft2_dct(p->dc, p->d2, p->d1.n, p->ws.z + f0 * p->nfft_c, n, p->ws.dct + f0 * N, p->d_om2, st));
    }
    HIP_TRY(mark(2));
    if (p->cplx) {  // complex modulation: autocorrelation, LPC, cepstrum and the output columns
      const fdlp_config& c = p->cfg;
      HIP_TRY(fdlp::launch_cplx_modspec(p->dc, p->L, p->ws.dct + f0 * N, n, p->ws.r + it0 * nl * 2, p->d_frames + f0,
                                        p->d_utts, c.coeff_0 - 1, p->M, p->feat_len, c.keep_even ? 2 : 1,
                                        c.keep_even && c.coeff_0 % 2 == 0 ? 1 : 0, p->d_faxis, c.absolute_value,
                                        b->out_dev, b->out_f64_dev, b->ark_decimals, st));
      HIP_TRY(mark(3));
      HIP_TRY(mark(4));
      return FDLP_OK;
    }
    if (p->ac_path == FDLP_AC_STRUCTURED || p->ac_path == FDLP_AC_STRUCTURED_MFMA) {
      double* rflat = p->ac_path == FDLP_AC_STRUCTURED ? p->r_flat + it0 * nl : nullptr;
      double* rpart = p->ac_path == FDLP_AC_STRUCTURED && p->r_flat_part
                          ? p->r_flat_part + (size_t)f0 * (p->sk.fl_H - 1) * fdlp::kMaxChains * nl
                          : nullptr;
      double* rwrap = p->ac_path == FDLP_AC_STRUCTURED && p->r_wrap ? p->r_wrap + (size_t)f0 * nl : nullptr;
      HIP_TRY(fdlp::launch_autocorr_structured(p->dc, p->ws.dct + f0 * N, n, r, p->r_up + it0 * nl, rflat, rpart,
                                               rwrap, st));
    } else {
      HIP_TRY(fdlp::launch_autocorr(p->dc, p->ws.dct + f0 * N, nullptr, its, r, st));
    }
    HIP_TRY(mark(3));
    HIP_TRY(fdlp::launch_lpc_env(p->dc, p->cfg.odd_mod_zero, r, its, env, a_dbg, gg_dbg, cep_dbg,
                                  p->ws.a_pad ? p->ws.a_pad + it0 * p->dc.lpc_astride : nullptr, p->ws.gg + it0,
                                  st));
    HIP_TRY(mark(4));
    return FDLP_OK;
  };
  if (nsub == 1) {
    int rc = run_frames(0, 0, (int)nf, s);
    if (rc != FDLP_OK) return rc;
  } else {
    HIP_TRY(hipEventRecord(p->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(p->aux_stream, p->ev_fork, 0));
    for (int i = 0; i < nsub; ++i) {
      const int64_t f0 = nf * i / nsub, f1 = nf * (i + 1) / nsub;
      int rc = run_frames(i, f0, (int)(f1 - f0), (i & 1) ? p->aux_stream : s);
      if (rc != FDLP_OK) return rc;
    }
    HIP_TRY(hipEventRecord(p->ev_join, p->aux_stream));
    HIP_TRY(hipStreamWaitEvent(s, p->ev_join, 0));
  }
  if (p->profiling) HIP_TRY(hipEventRecord(ev[ev.size() - 2], s));
  if (p->modspec && !p->cplx) {  // mod_spec[coeff_0-1 : coeff_n] per band (computeModulationSpectrum.py:182-201)
    const fdlp_config& c = p->cfg;
    const int keep_odd_slot = c.keep_even && c.coeff_0 % 2 == 0 ? 1 : 0;  // temp2[1::2] vs temp2[0::2]
    HIP_TRY(fdlp::launch_modspec_out(p->ws.cep, p->d_frames, p->d_utts, (int)nf, p->B, p->M, c.coeff_0 - 1,
                                     p->feat_len, c.keep_even ? 2 : 1, keep_odd_slot, p->d_faxis,
                                     c.absolute_value, b->out_dev, b->out_f64_dev, b->ark_decimals, s));
  } else if (!p->modspec) {  // (complex modulation: launch_cplx_modspec)
    HIP_TRY(fdlp::launch_ola_log(p->dc, p->ws.env, p->d_frames, p->d_utts, b->n_utt, maxL, b->out_dev,
                                 b->out_f64_dev, b->out_q_dev, b->out_q_flag_dev, b->ark_decimals, s));
  }
  if (p->profiling) {
    HIP_TRY(hipEventRecord(ev.back(), s));
    p->prof_pending.push_back(ev);
  }
  if (kprof) {
    fdlp::g_kmarks = nullptr;
    p->kmark_pending.push_back(kmarks);
    kmarks.clear();  // owned by kmark_pending now
  }
  return FDLP_OK;
}

int fdlp_set_autocorr_path(fdlp_plan* p, int32_t path) {
  if (!p) return fail(FDLP_E_INVALID, "fdlp_set_autocorr_path: null plan");
  if (path == FDLP_AC_AUTO) {
    p->ac_path = !p->sk_avail ? FDLP_AC_DIRECT : (p->vs_avail ? FDLP_AC_STRUCTURED : FDLP_AC_STRUCTURED_MFMA);
  } else if (path == FDLP_AC_DIRECT) {
    p->ac_path = FDLP_AC_DIRECT;
  } else if (path == FDLP_AC_STRUCTURED || path == FDLP_AC_STRUCTURED_MFMA) {
    if (!p->sk_avail)
      return fail(FDLP_E_INVALID, "structured autocorrelation needs the cochlear filterbank with fixed=1");
    p->ac_path = (path == FDLP_AC_STRUCTURED && p->vs_avail) ? FDLP_AC_STRUCTURED : FDLP_AC_STRUCTURED_MFMA;
  } else {
    return fail(FDLP_E_INVALID, "fdlp_set_autocorr_path: unknown path");
  }
  return FDLP_OK;
}

int fdlp_plan_flat_events(const fdlp_plan* p, int32_t* chains, int32_t* parts, int32_t* nev, int32_t* events,
                          int32_t cap) {
  if (!p) return fail(FDLP_E_INVALID, "fdlp_plan_flat_events: null plan");
  const bool ok = p->sk_avail && p->vs_avail;
  if (chains) *chains = ok ? p->sk.fl_C : 0;
  if (parts) *parts = ok ? p->sk.fl_H : 0;
  const int n = ok ? (int)p->sk.fl.size() : 0;
  if (nev) *nev = n;
  if (events)
    for (int k = 0; k < n && k < cap; ++k) {
      const fdlp::FlatEv& e = p->sk.fl[k];
      events[4 * k] = e.S; events[4 * k + 1] = e.band; events[4 * k + 2] = e.type; events[4 * k + 3] = e.chain;
    }
  return FDLP_OK;
}

int fdlp_plan_regions(const fdlp_plan* p, int32_t* m1, int32_t* m2) {
  if (!p) return fail(FDLP_E_INVALID, "fdlp_plan_regions: null plan");
  if (!p->sk_avail) return fail(FDLP_E_INVALID, "filterbank has no skirt/flat-top split (structured path unavailable)");
  for (int j = 0; j < p->B; ++j) {
    if (m1) m1[j] = p->sk.reg[j].x;
    if (m2) m2[j] = p->sk.reg[j].y;
  }
  return FDLP_OK;
}

int fdlp_set_lpc_path(fdlp_plan* p, int32_t path) {
  if (!p || (path != FDLP_LPC_AUTO && path != FDLP_LPC_LDS && path != FDLP_LPC_LATTICE8))
    return fail(FDLP_E_INVALID, "fdlp_set_lpc_path: need a plan and FDLP_LPC_AUTO, FDLP_LPC_LDS or FDLP_LPC_LATTICE8");
  if (p->device < 0) return fail(FDLP_E_INVALID, "fdlp_set_lpc_path: host-only plan");
  DeviceGuard dg(p->device);
  if (dg.status() != hipSuccess) return fail(FDLP_E_HIP, "hipSetDevice failed");
  p->dc.lpc_mode = path;
  if (fdlp::prepare_lpc_env(p->dc) != hipSuccess) return fail(FDLP_E_HIP, "LPC kernel launch setup failed");
  if (p->dc.lpc_split && !p->ws.a_pad &&
      hipMalloc((void**)&p->ws.a_pad, sizeof(double) * (size_t)p->max_frames * p->B * p->dc.lpc_astride) != hipSuccess)
    return fail(FDLP_E_NOMEM, "device workspace allocation failed");
  return FDLP_OK;
}

int fdlp_set_dct_path(fdlp_plan* p, int32_t path) {
  if (!p || (path != FDLP_DCT_AUTO && path != FDLP_DCT_FOUR_STEP))
    return fail(FDLP_E_INVALID, "fdlp_set_dct_path: need a plan and FDLP_DCT_AUTO or FDLP_DCT_FOUR_STEP");
  if (p->device < 0) return fail(FDLP_E_INVALID, "fdlp_set_dct_path: host-only plan");
  DeviceGuard dg(p->device);
  if (dg.status() != hipSuccess) return fail(FDLP_E_HIP, "hipSetDevice failed");
  p->dct_path = path;
  if (!dct_fused(p) && !p->ws.z &&
      hipMalloc((void**)&p->ws.z, sizeof(double2) * (size_t)p->max_frames * p->nfft_c) != hipSuccess)
    return fail(FDLP_E_NOMEM, "device workspace allocation failed");
  return FDLP_OK;
}

int fdlp_dct_path(const fdlp_plan* p) {
  if (!p) return fail(FDLP_E_INVALID, "fdlp_dct_path: null plan");
  return dct_fused(p) ? FDLP_DCT_FRAME : FDLP_DCT_FOUR_STEP;
}

int fdlp_set_pipeline(fdlp_plan* p, int32_t n_sub) {
  if (!p || n_sub < 1) return fail(FDLP_E_INVALID, "fdlp_set_pipeline: need a plan and n_sub >= 1");
  p->pipeline = n_sub;
  return FDLP_OK;
}

int fdlp_autocorr_path(const fdlp_plan* p) {
  if (!p) return fail(FDLP_E_INVALID, "fdlp_autocorr_path: null plan");
  return p->ac_path;
}

int fdlp_set_debug(fdlp_plan* p, int32_t keep_intermediates) {
  if (!p) return fail(FDLP_E_INVALID, "fdlp_set_debug: null plan");
  // a [items, p+1] and cep [items, M] exist only for debugging (and cep for the modspec output): allocated
  // here, not at plan creation (for REVERB's M = 450 the two are ~0.8 GB at 2048 frames).  The flag is set
  // only once both exist: fdlp_compute offsets them per sub-batch when it is set.
  if (keep_intermediates != 0 && p->device >= 0) {
    DeviceGuard dg(p->device);
    HIP_TRY(dg.status());
    const size_t items = (size_t)p->max_frames * p->B;
    if (!p->ws.a) HIP_TRY(hipMalloc((void**)&p->ws.a, sizeof(double) * items * (p->p + 1)));
    if (!p->ws.cep) HIP_TRY(hipMalloc((void**)&p->ws.cep, sizeof(double) * items * p->M));
  }
  p->debug_intermediates = keep_intermediates != 0;
  return FDLP_OK;
}

int fdlp_device_checks(int32_t* enabled, uint32_t* violations, uint32_t* last_line, int32_t reset) {
  unsigned int tot = 0, line = 0;
  hipError_t (*const fns[])(unsigned int*, bool) = {fdlp::checks_dct, fdlp::checks_autocorr, fdlp::checks_lpc,
                                                    fdlp::checks_misc};
  HIP_TRY(hipDeviceSynchronize());
  for (auto fn : fns) {
    unsigned int v[2] = {0u, 0u};
    HIP_TRY(fn(v, reset != 0));
    tot += v[0];
    line = std::max(line, v[1]);
  }
  if (enabled) *enabled = FDLP_DEVICE_CHECKS ? 1 : 0;
  if (violations) *violations = tot;
  if (last_line) *last_line = line;
  return FDLP_OK;
}

int fdlp_set_profiling(fdlp_plan* p, int32_t enable) {
  if (!p || p->device < 0) return fail(FDLP_E_INVALID, "fdlp_set_profiling: bad plan");
  int rc = drain_profile(p);
  if (rc != FDLP_OK) return rc;
  p->profiling = enable != 0;
  p->kprofiling = enable >= 2;
  for (double& v : p->prof_ms) v = 0.0;
  p->prof_calls = 0;
  for (double& v : p->kern_ms) v = 0.0;
  for (int64_t& v : p->kern_launches) v = 0;
  return FDLP_OK;
}

int fdlp_kernel_times(fdlp_plan* p, double* ms_sum, int64_t* launches) {
  if (!p || !ms_sum) return fail(FDLP_E_INVALID, "fdlp_kernel_times: bad args");
  int rc = drain_profile(p);
  if (rc != FDLP_OK) return rc;
  for (int k = 0; k < FDLP_NUM_KERNELS; ++k) {
    ms_sum[k] = p->kern_ms[k];
    if (launches) launches[k] = p->kern_launches[k];
  }
  return FDLP_OK;
}

const char* fdlp_kernel_name(int32_t id) {
  static const char* const names[FDLP_NUM_KERNELS] = {
      "fdlp::dct_frame_kernel", "fdlp::frames_dft1", "fdlp::dft2_dct", "fdlp::ac_vsweep_kernel<skirts>",
      "fdlp::ac_vsweep_kernel<flat>", "fdlp::ac_wrap_kernel", "fdlp::ac_band_kernel", "fdlp::ac_sweep_kernel",
      "fdlp::autocorr_kernel", "fdlp::durbin4_kernel", "fdlp::durbin8_kernel", "fdlp::lpc_env_lattice_kernel",
      "fdlp::lpc_env_kernel", "fdlp::ola_log_tiled_kernel", "other", ""};
  return id >= 0 && id < FDLP_NUM_KERNELS ? names[id] : "";
}

int fdlp_stage_times(fdlp_plan* p, double* ms_sum, int32_t* n_calls) {
  if (!p || !ms_sum) return fail(FDLP_E_INVALID, "fdlp_stage_times: bad args");
  int rc = drain_profile(p);
  if (rc != FDLP_OK) return rc;
  for (int k = 0; k < FDLP_NUM_STAGES; ++k) ms_sum[k] = p->prof_ms[k];
  if (n_calls) *n_calls = p->prof_calls;
  return FDLP_OK;
}

int fdlp_debug_fetch_range(fdlp_plan* p, int32_t f0, int32_t n, double* dct, double* r, double* a, double* gg,
                           double* cep, double* env) {
  if (!p || f0 < 0 || n < 0 || (int64_t)f0 + n > p->max_frames || p->device < 0)
    return fail(FDLP_E_INVALID, "fdlp_debug_fetch: bad args");
  DeviceGuard dg(p->device);
  HIP_TRY(dg.status());
  HIP_TRY(hipDeviceSynchronize());
  const size_t items = (size_t)n * p->B, it0 = (size_t)f0 * p->B;
  if ((a && !p->ws.a) || (cep && !p->ws.cep))
    return fail(FDLP_E_INVALID, "fdlp_debug_fetch: a / cep are kept only after fdlp_set_debug(plan, 1)");
  if (env && !p->env_valid)
    return fail(FDLP_E_INVALID, "fdlp_debug_fetch: no envelopes (modulation-spectrum plan or no compute yet)");
  if (dct) HIP_TRY(hipMemcpy(dct, p->ws.dct + (size_t)f0 * p->N, sizeof(double) * n * (size_t)p->N, hipMemcpyDeviceToHost));
  if (r) HIP_TRY(hipMemcpy(r, p->ws.r + it0 * p->nlags, sizeof(double) * items * p->nlags, hipMemcpyDeviceToHost));
  if (a) HIP_TRY(hipMemcpy(a, p->ws.a + it0 * (p->p + 1), sizeof(double) * items * (p->p + 1), hipMemcpyDeviceToHost));
  if (gg) HIP_TRY(hipMemcpy(gg, p->ws.gg + it0, sizeof(double) * items, hipMemcpyDeviceToHost));
  if (cep) HIP_TRY(hipMemcpy(cep, p->ws.cep + it0 * p->M, sizeof(double) * items * p->M, hipMemcpyDeviceToHost));
  if (env) HIP_TRY(hipMemcpy(env, p->ws.env + it0 * p->kk, sizeof(double) * items * p->kk, hipMemcpyDeviceToHost));
  return FDLP_OK;
}

int fdlp_debug_fetch(fdlp_plan* p, int32_t n, double* dct, double* r, double* a, double* gg, double* cep,
                     double* env) {
  return fdlp_debug_fetch_range(p, 0, n, dct, r, a, gg, cep, env);
}

int fdlp_dct_rows(fdlp_plan* p, const double* x, int32_t n, double* y, void* stream) {
  if (!p || !x || !y || n < 0 || p->device < 0) return fail(FDLP_E_INVALID, "fdlp_dct_rows: bad args or host-only plan");
  if (n > p->max_frames) return fail(FDLP_E_CAPACITY, "fdlp_dct_rows: more rows than max_frames");
  hipStream_t s = (hipStream_t)stream;
  if (dct_fused(p)) {
    HIP_TRY(fdlp::launch_dct_frame(p->dc, nullptr, 0, nullptr, nullptr, x, n, y, s));
    return FDLP_OK;
  }
  HIP_TRY(fdlp::launch_frames_dft1(p->dc, p->d1, p->d2.n, nullptr, 0, nullptr, nullptr, x, n, p->ws.z, p->d_om1, s));
  HIP_TRY(fdlp::launch_dft2_dct(p->dc, p->d2, p->d1.n, p->ws.z, n, y, p->d_om2, s));
  return FDLP_OK;
}

int fdlp_lpc_rows(fdlp_plan* p, const double* band, int32_t n, double* r, double* a, double* gg, void* stream) {
  if (!p || !band || !r || !a || !gg || n < 0 || p->device < 0) return fail(FDLP_E_INVALID, "fdlp_lpc_rows: bad args or host-only plan");
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(fdlp::launch_autocorr(p->dc, nullptr, band, n, r, s));
  HIP_TRY(fdlp::launch_levinson(p->dc, r, n, a, gg, s));
  return FDLP_OK;
}

int fdlp_cepstrum_rows(fdlp_plan* p, const double* a, const double* gg, int32_t n, int32_t order, int32_t lim,
                       double* cep, void* stream) {
  if (!p || !a || !gg || !cep || n < 0 || order < 1 || lim < 2) return fail(FDLP_E_INVALID, "fdlp_cepstrum_rows: bad args");
  HIP_TRY(fdlp::launch_cepstrum(order, lim, a, gg, n, cep, (hipStream_t)stream));
  return FDLP_OK;
}

// ---------------------------------------------------------------------------------------------
// mel spectrum plan (computeMelSpectrum.py:40-170)
// ---------------------------------------------------------------------------------------------
struct fdlp_mel_plan {
  fdlp_mel_config cfg{};
  int device = 0;
  int L = 0, hop = 0, sp_b = 0, sp_f = 0, ext = 0, nbins = 0;
  fdlp::MelConsts mc{};
  double *d_win = nullptr, *d_fb = nullptr;
  int *d_lo = nullptr, *d_hi = nullptr;
  double2 *d_om = nullptr, *d_rtw = nullptr;
  fdlp::MelFrame* d_frames = nullptr;
  fdlp::MelFrame* h_frames = nullptr;  // pinned staging
  hipEvent_t staging_done = nullptr;
  bool staging_pending = false;
};

static int free_mel_plan(fdlp_mel_plan* p) {
  if (!p) return FDLP_OK;
  void* devs[] = {p->d_win, p->d_fb, p->d_lo, p->d_hi, p->d_om, p->d_rtw, p->d_frames};
  for (void* d : devs)
    if (d) (void)hipFree(d);
  if (p->h_frames) (void)hipHostFree(p->h_frames);
  if (p->staging_done) (void)hipEventDestroy(p->staging_done);
  delete p;
  return FDLP_OK;
}

static int64_t mel_frames_of(const fdlp_mel_plan* p, int64_t T) {
  const int64_t lim = T + 2 * (int64_t)p->ext - p->sp_b - p->sp_f;  // getFrames: k*hop < lim
  if (lim <= 0) return 0;
  return (lim - 1) / p->hop + 1;
}

int fdlp_mel_plan_create(const fdlp_mel_config* cfg, int device, fdlp_mel_plan** out) {
  if (!cfg || !out) return fail(FDLP_E_INVALID, "fdlp_mel_plan_create: null argument");
  *out = nullptr;
  const fdlp_mel_config& c = *cfg;
  if (c.nfilters < 1 || c.srate < 1 || c.frate < 1 || !(c.fduration > 0) || c.max_frames < 1)
    return fail(FDLP_E_INVALID, "invalid mel configuration");
  if (c.nfft < 2 || c.nfft % 2 || c.nfft / 2 > 2048) return fail(FDLP_E_INVALID, "nfft must be even and <= 4096");
  auto* p = new (std::nothrow) fdlp_mel_plan;
  if (!p) return fail(FDLP_E_NOMEM, "out of memory");
  p->cfg = c;
  p->device = device;
  int rc;
#define MEL_FAIL(code, msg) do { rc = fail(code, msg); free_mel_plan(p); return rc; } while (0)
#define MEL_TRY(expr) do { rc = (expr); if (rc != FDLP_OK) { std::string m_ = fdlp::last_error_slot(); free_mel_plan(p); fdlp::last_error_slot() = m_; return rc; } } while (0)
  p->L = (int)((double)c.srate * c.fduration);       // features.py:134
  p->hop = (int)((double)c.srate / (double)c.frate);  // features.py:135
  if (p->L % 2 == 0) { p->sp_b = p->L / 2 - 1; p->sp_f = p->L / 2; p->ext = p->L / 2 - 1; }
  else { p->sp_b = p->sp_f = p->ext = (p->L - 1) / 2; }
  if (p->L < 2 || p->hop < 1) MEL_FAIL(FDLP_E_INVALID, "frame length / hop too small");
  const int nh = c.nfft / 2;
  fdlp::DftPlan dp{};
  if (!factor_radices(nh, &dp)) MEL_FAIL(FDLP_E_INVALID, "nfft/2 must factor into 2, 3, 5 and 7");
  std::vector<double> fb;
  int ncol = 0;
  if (c.fbank_kind == FDLP_FBANK_MEL) fb = fbank_mel(c.nfilters, c.nfft, c.srate, c.warp_fact, &ncol);  // :57
  else if (c.fbank_kind == FDLP_FBANK_COCHLEAR)
    fb = fbank_cochlear(c.nfilters, c.nfft, c.srate, c.om_w, c.alp, c.fixed, c.bet, c.warp_fact, &ncol);  // :63-65
  else MEL_FAIL(FDLP_E_INVALID, "Invalid type of filter bank, use mel or cochlear with proper configuration");
  if (ncol != nh + 1) MEL_FAIL(FDLP_E_INVALID, "filterbank width does not match nfft/2+1");
  p->nbins = ncol;
  std::vector<int> lo(c.nfilters, 0), hi(c.nfilters, 0);
  for (int m = 0; m < c.nfilters; ++m) {
    int a = ncol, b = 0;
    for (int k = 0; k < ncol; ++k)
      if (fb[(size_t)m * ncol + k] != 0.0) { a = std::min(a, k); b = k + 1; }
    if (b <= a) { a = 0; b = 0; }
    lo[m] = a;
    hi[m] = b;
  }
  const std::vector<double> win = cos_window(p->L, 0.54, 0.46);  // np.hamming (computeMelSpectrum.py:41)
  const long double PI = 3.141592653589793238462643383279502884L;
  std::vector<double2> om(nh), rtw(nh + 1);
  for (int q = 0; q < nh; ++q) {
    const long double ang = -2.0L * PI * (long double)q / (long double)nh;
    om[q] = make_double2((double)cosl(ang), (double)sinl(ang));
  }
  for (int k = 0; k <= nh; ++k) {
    const long double ang = -2.0L * PI * (long double)k / (long double)c.nfft;
    rtw[k] = make_double2((double)cosl(ang), (double)sinl(ang));
  }
  if (device < 0) {
    *out = p;
    return FDLP_OK;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) MEL_FAIL(FDLP_E_HIP, "no HIP device visible");
  if (device >= ndev) MEL_FAIL(FDLP_E_INVALID, "device index out of range");
  DeviceGuard dg(device);
  if (dg.status() != hipSuccess) MEL_FAIL(FDLP_E_HIP, "hipSetDevice failed");
  MEL_TRY(upload(&p->d_win, win.data(), win.size()));
  MEL_TRY(upload(&p->d_fb, fb.data(), fb.size()));
  MEL_TRY(upload(&p->d_lo, lo.data(), lo.size()));
  MEL_TRY(upload(&p->d_hi, hi.data(), hi.size()));
  MEL_TRY(upload(&p->d_om, om.data(), om.size()));
  MEL_TRY(upload(&p->d_rtw, rtw.data(), rtw.size()));
  if (hipMalloc((void**)&p->d_frames, sizeof(fdlp::MelFrame) * c.max_frames) != hipSuccess ||
      hipHostMalloc((void**)&p->h_frames, sizeof(fdlp::MelFrame) * c.max_frames, hipHostMallocDefault) != hipSuccess ||
      hipEventCreateWithFlags(&p->staging_done, hipEventDisableTiming) != hipSuccess)
    MEL_FAIL(FDLP_E_NOMEM, "mel plan workspace allocation failed");
  fdlp::MelConsts& m = p->mc;
  m.L = p->L; m.hop = p->hop; m.ext = p->ext; m.nfft = c.nfft; m.nh = nh; m.nbins = ncol;
  m.nfilters = c.nfilters; m.power = c.power ? 1 : 0;
  m.window = p->d_win; m.fbank = p->d_fb; m.lo = p->d_lo; m.hi = p->d_hi; m.om = p->d_om; m.rtw = p->d_rtw;
  m.dp = dp;
#undef MEL_FAIL
#undef MEL_TRY
  *out = p;
  return FDLP_OK;
}

int fdlp_mel_plan_destroy(fdlp_mel_plan* p) { return free_mel_plan(p); }

int fdlp_mel_geometry(const fdlp_mel_plan* p, int64_t T, int32_t* F) {
  if (!p || !F || T < 0) return fail(FDLP_E_INVALID, "fdlp_mel_geometry: bad args");
  *F = (int32_t)mel_frames_of(p, T);
  return FDLP_OK;
}

int fdlp_mel_compute(fdlp_mel_plan* p, const fdlp_batch* b, void* stream) {
  if (!p || !b || p->device < 0) return fail(FDLP_E_INVALID, "fdlp_mel_compute: bad args or host-only plan");
  if (b->n_utt < 0 || (b->n_utt > 0 && (!b->pcm_dev || !b->pcm_off || !b->utt_len || !b->out_row)) ||
      (!b->out_dev && !b->out_f64_dev))
    return fail(FDLP_E_INVALID, "fdlp_mel_compute: bad batch");
  if (b->noise_dev && (!b->noise_off || !b->noise_alpha)) return fail(FDLP_E_INVALID, "noise arrays missing");
  if (b->preprocess == FDLP_PRE_DIFF && (b->pcm_kind != FDLP_PCM_I16 || b->noise_dev))
    return fail(FDLP_E_INVALID, "diff preprocessing needs int16 PCM and no noise");
  hipStream_t s = (hipStream_t)stream;
  if (p->staging_pending) {
    HIP_TRY(hipEventSynchronize(p->staging_done));
    p->staging_pending = false;
  }
  int nf = 0;
  for (int u = 0; u < b->n_utt; ++u) {
    const int64_t T = b->utt_len[u];
    if (T < 1) return fail(FDLP_E_INVALID, "empty utterance");
    const int64_t F = mel_frames_of(p, T);
    if (nf + F > p->cfg.max_frames) return fail(FDLP_E_CAPACITY, "batch exceeds the mel plan's max_frames");
    for (int64_t k = 0; k < F; ++k) {
      fdlp::MelFrame& fd = p->h_frames[nf++];
      fd.pcm_off = b->pcm_off[u];
      fd.noise_off = b->noise_dev ? b->noise_off[u] : -1;
      fd.alpha = b->noise_dev ? b->noise_alpha[u] : 0.0;
      fd.out_row = b->out_row[u] + k;
      fd.T = (int32_t)T;
      fd.k = (int32_t)k;
    }
  }
  if (nf == 0) return FDLP_OK;
  HIP_TRY(hipMemcpyAsync(p->d_frames, p->h_frames, sizeof(fdlp::MelFrame) * nf, hipMemcpyHostToDevice, s));
  HIP_TRY(hipEventRecord(p->staging_done, s));
  p->staging_pending = true;
  const int kind = b->preprocess == FDLP_PRE_DIFF ? 2 : b->pcm_kind;
  HIP_TRY(fdlp::launch_mel(p->mc, p->d_frames, nf, b->pcm_dev, kind, b->noise_dev, b->out_dev, b->out_f64_dev,
                           b->ark_decimals, s));
  return FDLP_OK;
}

int fdlp_reverb(const fdlp_reverb_batch* b, void* stream) {
  if (!b || b->n_utt < 0 || !b->pcm_off || !b->utt_len || !b->rir_dev || b->rir_len < 1 || !b->out_dev ||
      !b->out_len || (b->n_utt > 0 && !b->pcm_dev) || (b->noise_dev && (!b->noise_off || !b->noise_alpha)) ||
      (b->pcm_kind != FDLP_PCM_I16 && b->pcm_kind != FDLP_PCM_F64) ||
      (b->pcm_kind == FDLP_PCM_F64 && (b->noise_dev || b->preprocess != FDLP_PRE_NONE)))
    return fail(FDLP_E_INVALID, "fdlp_reverb: bad args");
  if (b->n_utt == 0) return FDLP_OK;
  hipStream_t s = (hipStream_t)stream;
  const int R = b->rir_len;
  std::vector<fdlp::RevUtt> U(b->n_utt);
  int64_t extent = 0, ny = 0, maxT = 0;
  for (int i = 0; i < b->n_utt; ++i) {
    const int64_t T = b->utt_len[i];
    if (T < 1 || b->pcm_off[i] < 0) return fail(FDLP_E_INVALID, "fdlp_reverb: empty utterance");
    U[i].off = b->pcm_off[i];
    U[i].T = T;
    U[i].yoff = ny;
    U[i].noff = b->noise_dev ? b->noise_off[i] : -1;
    U[i].alpha = b->noise_dev ? b->noise_alpha[i] : 0.0;
    ny += T + R - 1;
    extent = std::max(extent, b->pcm_off[i] + T);
    maxT = std::max(maxT, T);
  }
  fdlp::RevUtt* dU = nullptr;
  double *x = nullptr, *y = nullptr, *xs = nullptr;
  int64_t* dlen = nullptr;
  HIP_TRY(hipMallocAsync((void**)&dU, sizeof(fdlp::RevUtt) * U.size(), s));
  HIP_TRY(hipMallocAsync((void**)&x, sizeof(double) * extent, s));
  HIP_TRY(hipMallocAsync((void**)&y, sizeof(double) * ny, s));
  HIP_TRY(hipMallocAsync((void**)&xs, sizeof(double) * (size_t)b->n_utt * R, s));
  HIP_TRY(hipMallocAsync((void**)&dlen, sizeof(int64_t) * b->n_utt, s));
  HIP_TRY(hipMemcpyAsync(dU, U.data(), sizeof(fdlp::RevUtt) * U.size(), hipMemcpyHostToDevice, s));
  const int pre = b->preprocess == FDLP_PRE_DIFF ? 1 : 0;
  HIP_TRY(fdlp::launch_reverb(dU, b->n_utt, maxT, b->pcm_dev, b->pcm_kind, pre, b->noise_dev, b->rir_dev, R, x, y,
                              xs, b->out_dev, dlen, s));
  HIP_TRY(hipMemcpyAsync(b->out_len, dlen, sizeof(int64_t) * b->n_utt, hipMemcpyDeviceToHost, s));
  for (void* d : {(void*)dU, (void*)x, (void*)y, (void*)xs, (void*)dlen}) HIP_TRY(hipFreeAsync(d, s));
  HIP_TRY(hipStreamSynchronize(s));
  return FDLP_OK;
}

int fdlp_device_fn(int32_t fn, const double* x, double* y, int64_t n, void* stream) {
  if ((fn != FDLP_FN_LOG && fn != FDLP_FN_EXP) || n < 0 || (n > 0 && (!x || !y)))
    return fail(FDLP_E_INVALID, "fdlp_device_fn: bad args");
  const hipError_t e = fdlp::launch_device_fn(fn, x, y, n, (hipStream_t)stream);
  if (e != hipSuccess) return fail(FDLP_E_HIP, std::string("device fn kernel: ") + hipGetErrorString(e));
  return FDLP_OK;
}

int fdlp_cmvn_accumulate(const float* feats, int64_t rows, int32_t dim, double* stats, void* stream) {
  if (rows < 0 || dim <= 0 || !stats || (rows > 0 && !feats)) return fail(FDLP_E_INVALID, "fdlp_cmvn_accumulate: bad args");
  hipStream_t s = (hipStream_t)stream;
  const size_t nch = (size_t)fdlp::cmvn_chunks(rows);
  double* part = nullptr;
  // stream-ordered scratch for the per-chunk partial sums [nch, 2, dim]
  HIP_TRY(hipMallocAsync((void**)&part, sizeof(double) * 2 * (size_t)dim * std::max<size_t>(nch, 1), s));
  hipError_t e = fdlp::launch_cmvn(feats, rows, dim, part, stats, s);
  hipError_t e2 = hipFreeAsync(part, s);
  if (e != hipSuccess) return fail(FDLP_E_HIP, std::string("cmvn kernels: ") + hipGetErrorString(e));
  if (e2 != hipSuccess) return fail(FDLP_E_HIP, std::string("hipFreeAsync: ") + hipGetErrorString(e2));
  return FDLP_OK;
}

}  // extern "C"
