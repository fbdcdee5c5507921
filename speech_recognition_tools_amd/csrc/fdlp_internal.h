// fdlp_internal.h -- structures shared by the host runtime (fdlp_plan.cpp) and the gfx950
// kernels (fdlp_*.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace fdlp {

constexpr int kMaxRadices = 16;
constexpr int kXcds = 8;  // XCDs of an MI355X; workgroup b is dispatched to XCD b mod 8

// A length-n complex DFT factored into radices (Stockham autosort, one LDS-resident pass).
struct DftPlan {
  int n;
  int nrad;
  int rad[kMaxRadices];
};

// One analysis frame of the batch (getFrames, features.py:118-154).
struct FrameDesc {
  int64_t pcm_off;     // first sample of the utterance in the batch PCM buffer
  int64_t noise_off;   // noise mixing offset (features.py:25), -1 = none
  double alpha;        // noise mixing gain (features.py:29)
  int32_t T;           // utterance length in samples
  int32_t k;           // frame index inside the utterance
  int32_t dst, src, cnt;  // OLA slice (computeFDLPSpectrogram.py:207-218)
  int32_t utt;         // utterance index in the batch
};

// One utterance of the batch (output side).
struct UttDesc {
  int64_t out_row;     // first output row
  int32_t L;           // output frames
  int32_t frame0;      // first analysis frame (global index in the batch)
  int32_t F;           // analysis frames
  int32_t pad;
};

// One snapshot of a skirt sweep: after the positions >= S are consumed, band `band` receives
// K times the truncated autocorrelation (structured autocorrelation, fdlp_autocorr.hip 3s).
struct SkSnap {
  int32_t S;
  int32_t band;
  double K;
};

constexpr int kMaxFlatParts = 4;
constexpr int kMaxChains = 8;
// doubles every autocorrelation row buffer (r, r_up, r_flat, r_wrap, r_flat_part) carries past its last row:
// ac_band_kernel reads its combine rows in whole 32-lag blocks (lags up to 32 ceil(nlags / 32) - 1)
constexpr int kRowSlack = 64;

// One event of the flat-top sweep (ac_vsweep_kernel): at sweep position S (after the positions >= S
// are consumed) restart (type 0) or emit (type 1) chain `chain`, which serves band `band`.
struct FlatEv {
  int32_t S, band, type, chain;
};

// Device-resident constants of a plan.
struct DevConsts {
  int B, N, hop, ext, p, nlags, M, Me, kk, env_nfft;
  const double* fbank;     // [B, N] dense taps (column N of the reference's nfft/2+1 dropped, :190)
  const int* lo;           // [B] first tap >= eps
  const int* hi;           // [B] one past the last tap >= eps
  const double* hamming;   // [N]   np.hamming(N)
  const double* weights;   // [3, M] mask (:94-103), lifter (:195-196), gamma (:197-198); 1.0 if absent
  const double* env_cos;   // [env_nfft] cos(2*pi*q/env_nfft)
  const double* env_win;   // [kk, 2] (hanning(kk)[t] / hamming(kk)[t], 1.0) interleaved (:205)
  const double* tw1;       // [N1 * N2] four-step twiddles exp(-2*pi*i*n2*k1/(N1*N2)) (complex)
  const double* post;      // [N] complex exp(-i*pi*k/(2N)) (Makhoul post-twiddle)
  const double* rtw;       // [N/2] complex exp(-2*pi*i*k/N) (real-FFT unpacking; real_fft only)
  int real_fft;            // N even: the DCT runs a length-N/2 complex FFT of the packed real sequence
  // structured autocorrelation (cochlear filterbank, fixed skirt slope); null when not used
  const double* sk_e;      // [2, N] E = 10^(a (fw - c0)) (lower skirt), E' = 10^(-b (fw - c0)) (upper)
  const SkSnap* sk_snap;   // [2, B] sorted by S descending: S = N - m1_j (lower) / m2_j (upper) with
                           // K_j = 10^(a (w - 2 fc_j + 2 c0)) / K'_j = 10^(b (2 fc_j + w - 2 c0))
  const int2* sk_reg;      // [B] (m1_j, m2_j): lower skirt [0,m1), flat top [m1,m2), upper skirt [m2,N)
  int sk_min[2];           // smallest threshold per skirt
  // lag-parallel VALU sweeps (ac_vsweep_kernel); fl_ev null when not used
  const FlatEv* fl_ev = nullptr;  // [fl_nev] flat-top events sorted by S descending
  int fl_nev = 0, fl_C = 0;       // event count, chains needed (bands j and j - C never overlap)
  int fl_lo = 0, fl_hi = 0;       // min m1, max m2
  // the flat sweep is split into fl_H position parts [fl_part_lo[h], fl_part_hi[h]) run by different
  // waves; part h takes the events fl_ev[fl_part_ev[h] .. fl_part_ev[h+1]) and, for h < fl_H - 1, leaves
  // every chain in rflat_part[f][h][chain] for the bands that continue below it
  int fl_H = 1;
  int fl_part_lo[kMaxFlatParts] = {0}, fl_part_hi[kMaxFlatParts] = {0}, fl_part_ev[kMaxFlatParts + 1] = {0};
  const int2* fl_band = nullptr;  // [B] (chain, bitmask of the parts h < fl_H - 1 it needs a partial from)
  // wrap straddle shared by the bands whose first / last nlags - 1 taps lie on their skirts: [B]
  // sqrt(K_j K'_j), 0 for the bands whose wrap straddle ac_band_kernel computes from the taps; null: none
  const double* sk_wrap = nullptr;
  // persistent LPC kernel: resident blocks on the plan's device (prepare_lpc_env, at plan creation)
  int lpc_blocks = 0;
  int lpc_mode = 0;        // fdlp_set_lpc_path: 0 lattice kernels (default), 1 the LDS Durbin (cross-check)
  int lpc_split = 0;       // the Durbin as durbin8_kernel (8 lanes per item), then the cepstrum/envelope
                           // kernel (set by prepare_lpc_env when p fits durbin8_kernel)
  int natural = 0;         // complex modulation: frames in sample order, dft2 writes X = conj(DFT_N)/N
                           // (scipy.fftpack.ifft of the real frame), bins [0, N/2), as double2 rows of N doubles
  int lpc_astride = 0;     // split Durbin: row stride of a_pad (the cepstrum kernel's a-area length,
                           // zero past p), so a row is one contiguous LDS-DMA copy
  const double2* dct1_tw = nullptr;  // dct_frame_kernel tables (N = 24000 only; see dct_frame_tables)
};

// Per-kernel HIP-event marks (fdlp_set_profiling(plan, 2), fdlp_kernel_times): while a profiled fdlp_compute
// issues its kernels, each launch site calls kmark(id, stream) after its launch, which records an event on
// that stream when marks are being collected on this thread (g_kmarks), and does nothing otherwise.
enum KernelId {
  kKDctFrame = 0, kKFramesDft1, kKDft2Dct, kKVsweepSkirt, kKVsweepFlat, kKAcWrap, kKAcBand, kKAcSweep,
  kKAutocorr, kKDurbin4, kKDurbin8, kKLattice, kKLpcLds, kKOlaLog, kKOther, kKCount
};
struct KMark {
  int id;
  hipEvent_t ev;
};
extern thread_local std::vector<KMark>* g_kmarks;
hipError_t kmark(int id, hipStream_t s);

}  // namespace fdlp

// Launch wrappers implemented in fdlp_{dct,autocorr,lpc,misc}.hip (host-callable).
namespace fdlp {
struct Workspace {
  double2* z;      // [F, N1, N2] complex (four-step intermediate)
  double* dct;     // [F, N]
  double* r;       // [F*B, nlags]
  double* a;       // [F*B, p+1]
  double* a_pad;   // [F*B, lpc_astride] (split Durbin only)
  double* gg;      // [F*B]
  double* cep;     // [F*B, M]
  double* env;     // [F*B, kk]
};

hipError_t launch_frames_dft1(const DevConsts& c, const DftPlan& d1, int N2, const void* pcm,
                              int pcm_kind, const int16_t* noise, const FrameDesc* frames,
                              const double* dense_rows, int nframes, double2* z,
                              const double2* om1, hipStream_t s);
hipError_t launch_dft2_dct(const DevConsts& c, const DftPlan& d2, int N1, const double2* z,
                           int nframes, double* dct, const double2* om2, hipStream_t s);
// the recipes' DCT (N = 24000, real FFT) as one kernel per frame; hipErrorInvalidValue otherwise
hipError_t launch_dct_frame(const DevConsts& c, const void* pcm, int pcm_kind, const int16_t* noise,
                            const FrameDesc* frames, const double* dense_rows, int nframes, double* dct,
                            hipStream_t s);
std::vector<double2> dct_frame_tables(int N, const std::vector<double>& window);
// FDLP_DEVICE_CHECKS builds: each kernel translation unit's violation counter and last failing line
hipError_t checks_dct(unsigned int* v, bool reset);
hipError_t checks_autocorr(unsigned int* v, bool reset);
hipError_t checks_lpc(unsigned int* v, bool reset);
hipError_t checks_misc(unsigned int* v, bool reset);
hipError_t launch_autocorr(const DevConsts& c, const double* dct, const double* dense_rows,
                           int nframes_or_items, double* r, hipStream_t s);
hipError_t launch_autocorr_structured(const DevConsts& c, const double* dct, int nframes, double* r,
                                      double* rup, double* rflat, double* rflat_part, double* rwrap, hipStream_t s);
int vsweep_lanes_lags(int nlags);   // lags per lane of ac_vsweep_kernel, 0 = unsupported
int vsweep_chains(int C);           // chain count instantiated for C needed chains, 0 = unsupported
hipError_t launch_levinson(const DevConsts& c, const double* r, int items, double* a,
                           double* gg, hipStream_t s);
hipError_t launch_cepstrum(int p, int M, const double* a, const double* gg, int items,
                           double* cep, hipStream_t s);
// a_ws / gg_ws: [items, c.lpc_astride] / [items] workspace of the split Durbin (durbin8_kernel,
// c.lpc_split); a_out / gg_out (debug, [items, p+1] / [items]) get copies
hipError_t launch_lpc_env(const DevConsts& c, int odd_zero, const double* r, int items, double* env,
                          double* a_out, double* gg_out, double* cep_out, double* a_ws, double* gg_ws,
                          hipStream_t s);
int lpc_env_region(int p, int M);
// Per-plan launch setup of launch_lpc_env for the current device: sets the kernel's large-LDS
// attribute and stores the resident block count in c.lpc_blocks.
hipError_t prepare_lpc_env(DevConsts& c);
int autocorr_tiles(int nlags);
constexpr int kDftMaxSub = 512;  // longest LDS-resident sub-DFT of the four-step DCT
// Complex modulation spectrum (computeModulationSpectrum.py --complex_modulation): per (frame, band) the
// complex circular autocorrelation of W_j X (lags 0..p+1), then Hermitian Levinson, complex gain and
// cepstrum, and the feature slice (real/imag or abs, keep_even, 1/f compensation) into the output rows.
hipError_t launch_cplx_modspec(const DevConsts& c, int L, const double* X, int nframes, double* ycplx,
                               const FrameDesc* frames, const UttDesc* utts, int c0, int coeff_n, int feat_len,
                               int step, int first, const double* faxis, int absval, float* out, double* out64,
                               int decimals, hipStream_t s);
hipError_t launch_ola_log(const DevConsts& c, const double* env, const FrameDesc* frames,
                          const UttDesc* utts, int n_utt, int maxL, float* out,
                          double* out_f64, int16_t* out_q, uint32_t* q_flag, int decimals, hipStream_t s);
// Mel spectrum (computeMelSpectrum.py): one analysis frame and the plan constants.
struct MelFrame {
  int64_t pcm_off, noise_off;  // noise_off < 0: no mixing
  double alpha;
  int64_t out_row;
  int32_t T, k;
};
struct MelConsts {
  int L, hop, ext, nfft, nh, nbins, nfilters, power;
  const double* window;  // [L]  np.hamming(L)
  const double* fbank;   // [nfilters, nbins]
  const int* lo;         // [nfilters] first non-zero tap
  const int* hi;         // [nfilters] one past the last non-zero tap
  const double2* om;     // [nh] exp(-2 pi i q / nh)
  const double2* rtw;    // [nh + 1] exp(-2 pi i k / nfft)
  DftPlan dp;            // length nh
};
hipError_t launch_mel(const MelConsts& c, const MelFrame* frames, int nframes, const void* pcm, int pcm_kind,
                      const int16_t* noise, float* out, double* out64, int decimals, hipStream_t s);
size_t mel_lds_bytes(int nh);

// One utterance of a reverb batch (fdlp_reverb): samples at pcm[off, off+T), y at [yoff, yoff+T+R-1).
struct RevUtt {
  int64_t off, T, yoff, noff;  // noff < 0: no noise mixing
  double alpha;
};
hipError_t launch_reverb(const RevUtt* U, int n_utt, int64_t maxT, const void* pcm, int kind, int pre,
                         const int16_t* noise, const double* rir, int R, double* x, double* y, double* xs,
                         double* out, int64_t* out_len, hipStream_t s);
hipError_t launch_modspec_out(const double* cep, const FrameDesc* frames, const UttDesc* utts, int nframes, int B,
                              int M, int c0, int feat_len, int step, int first, const double* faxis, int absval,
                              float* out, double* out64, int decimals, hipStream_t s);
int cmvn_chunks(int64_t rows);
hipError_t launch_cmvn(const float* x, int64_t rows, int D, double* part, double* stats, hipStream_t s);
hipError_t launch_device_fn(int fn, const double* x, double* y, int64_t n, hipStream_t s);
}  // namespace fdlp
