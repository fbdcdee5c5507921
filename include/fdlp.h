/*
 * fdlp.h -- C ABI of libfdlp_hip.so, the MI355X (gfx950) FDLP-spectrogram extractor.
 *
 * Drop-in boundary for the reference hot path
 *   sadhusamik/speech_recognition_tools  src/featgen/computeFDLPSpectrogram.py  getFeats :29-237
 *   (+ the helpers it imports from src/featgen/features.py).
 * The reference has no FFI of its own (it is pure Python calling numpy/scipy); the entry points
 * below are what a ctypes binding of that path needs (INTEGRATION.md shows the binding).
 * Each function names the reference interface it replaces.
 *
 * Conventions: plain C types, caller-owned buffers, no C++ exceptions across the boundary.
 * Every function returns 0 on success or a negative FDLP_E* code; fdlp_last_error() returns a
 * thread-local message for the last failure.  "dev" pointers are device (HBM) pointers,
 * everything else is host memory.  `stream` is a hipStream_t passed as void* (NULL = default).
 */
#ifndef FDLP_H
#define FDLP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FDLP_ABI_VERSION 9

enum {
  FDLP_OK = 0,
  FDLP_E_INVALID = -1,   /* bad argument / configuration the reference would reject      */
  FDLP_E_HIP = -2,       /* HIP runtime failure                                            */
  FDLP_E_NOMEM = -3,     /* allocation failure                                             */
  FDLP_E_CAPACITY = -4,  /* batch larger than the plan's max_frames                        */
  FDLP_E_IO = -5,        /* file read/write failure                                        */
  FDLP_E_BROADCAST = -6  /* the reference's numpy OLA slicing would raise ValueError here  */
};

enum { FDLP_FBANK_MEL = 0, FDLP_FBANK_COCHLEAR = 1 };
enum { FDLP_PCM_I16 = 0, FDLP_PCM_F64 = 1 };
enum { FDLP_PRE_NONE = 0, FDLP_PRE_DIFF = 1 };  /* --add_noise diff (computeFDLPSpectrogram.py:162-164) */

/* Frozen feature configuration.  Mirrors the argparse surface of
 * computeFDLPSpectrogram.py:240-262 after the parsing getFeats does (:43-118). */
typedef struct fdlp_config {
  int32_t nfilters;          /* --nfilters                                   (:245) */
  int32_t coeff_num;         /* --coeff_num  (M)                             (:246) */
  int32_t coeff_lp;          /* --coeff_range "lp,hp" -> mask lp<=i<=hp      (:94-103) */
  int32_t coeff_hp;
  int32_t order;             /* --order (p)                                  (:248) */
  int32_t frate;             /* --frate                                      (:250) */
  int32_t srate;             /* 16000 (getFeats default, :29)                       */
  int32_t fbank_kind;        /* FDLP_FBANK_MEL | FDLP_FBANK_COCHLEAR          (:49-63) */
  double fduration;          /* --fduration                                  (:249) */
  double overlap_fraction;   /* --overlap_fraction (before the 1-x at :104)  (:251) */
  double warp_fact;          /* mel "mel,wf" / cochlear 6th field                    */
  double om_w, alp, bet;     /* cochlear "cochlear,om_w,alp,fixed,bet,wf"    (:59-61) */
  int32_t fixed;
  int32_t odd_mod_zero;      /* --odd_mod_zero                               (:199-200) */
  int32_t gamma_enabled;     /* --gamma_weight "scale,shape,pk" (!= "None")  (:107-118) */
  double gamma_scale, gamma_shape, gamma_pk;
  const double* lifter;      /* nullable; coeff_num values (--lifter_config first line, :43-46) */
  int32_t lifter_len;
  double support_eps;        /* filter taps < eps*peak are skipped in the autocorrelation
                                (0 = every non-zero tap; DESIGN.md "support")            */
  int32_t max_frames;        /* workspace capacity: analysis frames per fdlp_compute call  */
  /* ---- sibling feature: FDLP modulation spectrum (src/featgen/computeModulationSpectrum.py) ---- */
  int32_t mode;              /* FDLP_MODE_SPECTROGRAM | FDLP_MODE_MODSPEC | FDLP_MODE_MODSPEC_COMPLEX */
  int32_t window;            /* analysis window: FDLP_WIN_HAMMING (spectrogram, :29) |
                                FDLP_WIN_HANNING (modspec default, :30) | FDLP_WIN_RECT (--no_window) */
  int32_t coeff_0;           /* modspec --coeff_0 (1-based first kept coefficient); --coeff_n = coeff_num */
  int32_t keep_even;         /* modspec --keep_even (:66-72, :191-195)                              */
  int32_t compensate_noise;  /* modspec --compensate_noise: x linspace(0, n/(2 fduration), coeff_n) (:82-88) */
  int32_t absolute_value;    /* modspec --absolute_value (:186-187)                                 */
} fdlp_config;
enum { FDLP_MODE_SPECTROGRAM = 0, FDLP_MODE_MODSPEC = 1,
       FDLP_MODE_MODSPEC_COMPLEX = 2 /* modspec --complex_modulation (computeModulationSpectrum.py:45-47,
                                        :74-88, :153-180): ifft frames, complex LPC and cepstrum */ };
enum { FDLP_WIN_HAMMING = 0, FDLP_WIN_HANNING = 1, FDLP_WIN_RECT = 2 };

typedef struct fdlp_plan fdlp_plan;

/* Per-call batch of utterances.  Replaces the per-utterance body of getFeats
 * (computeFDLPSpectrogram.py:159-229): signal -> frames -> DCT -> per-band LPC -> cepstrum ->
 * envelope -> OLA -> log.  Samples of all utterances are concatenated in one device buffer. */
typedef struct fdlp_batch {
  int32_t n_utt;
  int32_t pcm_kind;              /* FDLP_PCM_I16 (scipy wavfile int16, :139) | FDLP_PCM_F64    */
  const void* pcm_dev;           /* device: samples                                              */
  const int64_t* pcm_off;        /* host [n_utt]: first sample of each utterance                 */
  const int64_t* utt_len;        /* host [n_utt]: T (samples) of each utterance                  */
  const uint8_t* jitter;         /* host: concatenated randrange(2) draws, F_u-1 per utterance,
                                    in utterance order (:225); see fdlp_pyrandom_*               */
  /* optional on-device noise mixing  x = s + alpha*noise[off:off+T]  (features.py:24-31) */
  const int16_t* noise_dev;      /* nullable device noise samples                                */
  const int64_t* noise_off;      /* host [n_utt]                                                 */
  const double* noise_alpha;     /* host [n_utt]                                                 */
  float* out_dev;                /* device: [sum_u L_u, nfilters] float32, row-major (ark layout) */
  const int64_t* out_row;        /* host [n_utt]: first output row of each utterance             */
  double* out_f64_dev;           /* nullable device: same layout, fp64 log features (parity)     */
  int32_t ark_decimals;          /* >=0: round out_dev like '%.<d>f' text ark (dict2Ark
                                    features.py:66 uses 3); <0: keep full float32               */
  int32_t preprocess;            /* FDLP_PRE_DIFF: x = convolve(int16 s, [1,2,3,2,0,-2,-5,-2,0,2,3,
                                    2,1], 'same') on the device (int16 PCM only)                 */
  /* ABI 7: compact ark codes, half the bytes of out_dev for the device-to-host leg.  With
     ark_decimals = d >= 0 the ark value of a feature is the float32 (float)(k / 10^d) with
     k = nearbyint(v * 10^d) (dict2Ark's '%.3f' text read back by copy-feats, features.py:66).
     out_q_dev receives k as int16 (-32768 = -0.0), same layout as out_dev; fdlp_q_widen turns the
     codes into exactly the float32 values out_dev would hold.  A value without a code (|k| > 32767
     or NaN; log features of 16-bit audio stay within [-32.24, +19]) stores -32768 and writes 1 to
     *out_q_flag_dev, which the caller zeroes before the call: that batch's float32 rows (out_dev,
     when also given) are then the ones to use.  Spectrogram plans only.                          */
  int16_t* out_q_dev;            /* nullable device [sum_u L_u, nfilters] int16 codes               */
  uint32_t* out_q_flag_dev;      /* device word, required with out_q_dev                            */
} fdlp_batch;

/* ---- plan ------------------------------------------------------------------------------- */
/* Replaces getFeats setup (:43-118): filterbank (features.py:172-219), mask/lifter/gamma
 * weights, windows, DFT plans; uploads them to `device` and allocates the workspace.
 * device < 0 creates a host-only plan (geometry, filterbank, weights, OLA tables; no compute). */
int fdlp_plan_create(const fdlp_config* cfg, int device, fdlp_plan** out);
int fdlp_plan_destroy(fdlp_plan* plan);
const char* fdlp_last_error(void);
int fdlp_abi_version(void);
/* Device address of pinned host memory (hipHostMalloc / hipHostRegister): fdlp_batch.out_dev may point
 * there, the OLA kernel then stores the features straight into host memory (no D2H copy; ABI 4). */
int fdlp_mapped_ptr(void* host, void** dev);

/* Frame geometry of one utterance of T samples: F analysis frames (getFrames,
 * features.py:151) and L output frames (int(ceil(T*frate/srate)), :182; L = F for the modspec
 * mode, one feature row per analysis frame, computeModulationSpectrum.py:161). */
int fdlp_geometry(const fdlp_plan* plan, int64_t T, int32_t* F, int32_t* L);
/* Output feature dimension per row: nfilters (spectrogram) or nfilters * feat_len (modspec). */
int fdlp_plan_out_dim(const fdlp_plan* plan, int32_t* dim);
/* Plan constants: N (DCT length), nfft, hop, nlags (=order+2), kk (envelope length). */
int fdlp_plan_info(const fdlp_plan* plan, int32_t* N, int32_t* hop, int32_t* nlags, int32_t* kk,
                   int32_t* ola_hop);
/* Host copy of the filterbank [nfilters, nfft/2+1] fp64 (createFbank / createFbankCochlear,
 * features.py:172-219) and of the per-band tap support [lo, hi). */
int fdlp_plan_fbank(const fdlp_plan* plan, double* fbank_out, int32_t* lo, int32_t* hi);
/* createFbank / createFbankCochlear (features.py:172-219) for an arbitrary nfft, using the
 * fbank_kind / warp_fact / om_w / alp / fixed / bet / nfilters / srate fields of cfg.
 * out: [nfilters, floor(nfft/2+1)]; *ncol receives the column count. */
int fdlp_make_fbank(const fdlp_config* cfg, int32_t nfft, double* out, int32_t* ncol);
/* Host copy of the folded modulation weights w[coeff_num] (:94-118, :194-200). */
int fdlp_plan_weights(const fdlp_plan* plan, double* w_out);

/* OLA table of one utterance (computeFDLPSpectrogram.py:207-225): per frame (dst, src, cnt).
 * Returns FDLP_E_BROADCAST where the reference's numpy slicing raises. */
int fdlp_ola_table(const fdlp_plan* plan, int64_t T, const uint8_t* jitter, int32_t* dst,
                   int32_t* src, int32_t* cnt);

/* ---- compute ---------------------------------------------------------------------------- */
/* Whole pipeline for a batch (getFeats :159-229).  Enqueued on `stream`; host arrays are
 * consumed before return. */
int fdlp_compute(fdlp_plan* plan, const fdlp_batch* batch, void* stream);
/* Host: the float32 ark values of n compact codes (fdlp_batch.out_q_dev) with the batch's ark_decimals,
 * bit-identical to the float32 out_dev rows; `threads` > 1 splits the work (ABI 7). */
int fdlp_q_widen(const int16_t* q, int64_t n, int32_t decimals, float* out, int32_t threads);
/* Keep the fused LPC kernel's a/gg/cep in the workspace (off by default; needed by
 * fdlp_debug_fetch for those three arrays). */
int fdlp_set_debug(fdlp_plan* plan, int32_t keep_intermediates);
/* Device range checks (ABI 6): *enabled = 1 in a library built with -DFDLP_DEVICE_CHECKS=1, whose
 * index-heavy kernels count violated range assertions (descriptors, sample / LDS / exchange indices,
 * straddle windows, OLA slices) on the device instead of trapping; *violations and *last_line (the
 * largest failing source line of csrc/) since the last reset; reset != 0 zeroes them.  Synchronises the
 * current device.  The default build reports enabled = 0 and zeros. */
int fdlp_device_checks(int32_t* enabled, uint32_t* violations, uint32_t* last_line, int32_t reset);
/* Autocorrelation algorithm (stage 2).  FDLP_AC_DIRECT: per band, over the taps >= support_eps *
 * peak.  FDLP_AC_STRUCTURED: exact (no tap truncation) skirt-factorised algorithm for the cochlear
 * filterbank with a fixed slope (fbank_type cochlear,..,fixed=1,..; DESIGN.md "Structured
 * autocorrelation"), its three sweeps (lower skirt, flat tops, upper skirt) lag-parallel on the fp64
 * VALU; FDLP_AC_STRUCTURED_MFMA: the same algorithm with MFMA lag-tile skirt sweeps and per-band
 * flat tops (also used when the VALU sweeps do not fit: more than 160 lags or 8 overlapping flat
 * tops).  FDLP_AC_AUTO (plan default) picks the first available of STRUCTURED, STRUCTURED_MFMA,
 * DIRECT.  fdlp_set_autocorr_path returns FDLP_E_INVALID when the structured paths are not
 * available; fdlp_autocorr_path returns the path in use or a negative error code. */
#define FDLP_AC_AUTO 0
#define FDLP_AC_DIRECT 1
#define FDLP_AC_STRUCTURED 2
#define FDLP_AC_STRUCTURED_MFMA 3
int fdlp_set_autocorr_path(fdlp_plan* plan, int32_t path);
int fdlp_autocorr_path(const fdlp_plan* plan);
/* LPC stage (Levinson-Durbin + cepstrum + envelope).  FDLP_LPC_AUTO (plan default): the register-resident
 * lattice kernels (durbin4_kernel, 4 lanes per item, for 128 <= p <= 150; durbin8_kernel, 8 lanes per item,
 * for 150 < p <= 183; then the cepstrum / envelope kernel); FDLP_LPC_LATTICE8 (ABI 6): the same with
 * durbin8_kernel for every 128 <= p <= 183 (cross-check of durbin4_kernel); FDLP_LPC_LDS:
 * the LDS Durbin kernel for every p (the fallback for p > 255 and an independent cross-check; its
 * order-k dot products are summed in another order).  The only switches between kernel variants are
 * these explicit calls: nothing is read from the environment (ABI 4). */
#define FDLP_LPC_AUTO 0
#define FDLP_LPC_LDS 1
#define FDLP_LPC_LATTICE8 2
int fdlp_set_lpc_path(fdlp_plan* plan, int32_t path);
/* DCT stage (ABI 5).  FDLP_DCT_AUTO (plan default): for the recipes' frame length N = 24000 one kernel per
 * frame (dct_frame_kernel: the packed 12000-point FFT as three in-register passes with LDS exchanges,
 * D written once); other N, and FDLP_DCT_FOUR_STEP, the two four-step kernels through the Z workspace
 * (allocated when first needed).  fdlp_dct_path returns FDLP_DCT_FRAME or FDLP_DCT_FOUR_STEP. */
#define FDLP_DCT_AUTO 0
#define FDLP_DCT_FOUR_STEP 1
#define FDLP_DCT_FRAME 2
int fdlp_set_dct_path(fdlp_plan* plan, int32_t path);
int fdlp_dct_path(const fdlp_plan* plan);
/* Lower-skirt / flat-top / upper-skirt split of every band, [0,m1) [m1,m2) [m2,N), used by the
 * STRUCTURED path; FDLP_E_INVALID when the filterbank does not have it. */
int fdlp_plan_regions(const fdlp_plan* plan, int32_t* m1, int32_t* m2);
/* The flat-top sweep of FDLP_AC_STRUCTURED (DESIGN.md "Lag-parallel VALU sweeps"): number of chains
 * (0 when the VALU sweeps are not available), position parts, and for up to cap events (S, band, type
 * 0 restart / 1 emit, chain) in sweep order; *nev receives the event count. */
int fdlp_plan_flat_events(const fdlp_plan* plan, int32_t* chains, int32_t* parts, int32_t* nev, int32_t* events,
                          int32_t cap);
/* fdlp_compute splits a batch of F frames into min(n_sub, F/256) sub-batches that alternate
 * between the caller's stream and a second stream of the plan, so the MFMA-bound autocorrelation
 * of one sub-batch can overlap the VALU-bound kernels of the other (default 1 = serial: on MI355X
 * the fp64 MFMA and fp64 VALU work measured no net overlap). */
int fdlp_set_pipeline(fdlp_plan* plan, int32_t n_sub);
/* Reads back the intermediates of the most recent fdlp_compute (parity/debug; synchronous):
 * any pointer may be NULL.  Layouts: dct [F,N]; r [F,B,nlags]; a [F,B,order+1]; gg [F,B];
 * cep [F,B,coeff_num]; env [F,B,kk] (spectrogram plans).  ABI 9 removed the fused OLA stage
 * (fdlp_set_ola_path / fdlp_ola_path, measured slower than the separate OLA kernel). */
int fdlp_debug_fetch(fdlp_plan* plan, int32_t n_frames, double* dct, double* r, double* a,
                     double* gg, double* cep, double* env);
/* Same for the frames [first_frame, first_frame + n_frames) of the most recent batch (ABI 3).
 * a and cep need fdlp_set_debug(plan, 1) before that compute (their workspaces are allocated by it;
 * FDLP_E_INVALID otherwise); dct, r, gg and (spectrogram plans) env are always available. */
int fdlp_debug_fetch_range(fdlp_plan* plan, int32_t first_frame, int32_t n_frames, double* dct, double* r,
                           double* a, double* gg, double* cep, double* env);

/* Per-stage device time (HIP events on the stream each stage runs on) of every fdlp_compute since
 * profiling was (re)enabled.  Stages: 0 frames+column DFT, 1 row DFT+DCT, 2 autocorrelation,
 * 3 fused Levinson+cepstrum+envelope, 4 OLA+log.  With sub-batch pipelining the stage times are
 * summed over the sub-batches and overlap each other in wall time.  fdlp_stage_times
 * synchronises on the events. */
#define FDLP_NUM_STAGES 5
int fdlp_set_profiling(fdlp_plan* plan, int32_t enable);
int fdlp_stage_times(fdlp_plan* plan, double* ms_sum /* [FDLP_NUM_STAGES] */, int32_t* n_calls);
/* Per-kernel device time (ABI 9): with fdlp_set_profiling(plan, 2) every kernel launch of an fdlp_compute
 * (one sub-batch) is followed by a HIP event on the stream it runs on, and the time between consecutive
 * events -- one kernel each, the stage's launch gaps included -- is summed per kernel id.  fdlp_kernel_name
 * gives the id's kernel (the rocprofv3 name prefix, e.g. "fdlp::ac_band_kernel"); launches counts them. */
#define FDLP_NUM_KERNELS 16
int fdlp_kernel_times(fdlp_plan* plan, double* ms_sum /* [FDLP_NUM_KERNELS] */, int64_t* launches);
const char* fdlp_kernel_name(int32_t id);
/* Seconds fdlp_plan_create spent in: [0] host tables (filterbank, structured-autocorrelation tables,
 * weights), [1] device open + table uploads, [2] LPC kernel launch setup, [3] workspace allocation,
 * [4] total (a cold JOB's fixed cost, benchmarks/cold_start_probe.py; ABI 4). */
int fdlp_plan_setup_times(const fdlp_plan* plan, double* sec /* [5] */);

/* ---- stage entry points (the features.py helpers, batched on the device) --------------- */
/* scipy.fftpack.dct(x)/sqrt(2N) of n_rows windowed frames [n_rows, N] (computeFDLPSpectrogram
 * .py:178).  N is the plan's frame length. */
int fdlp_dct_rows(fdlp_plan* plan, const double* x_dev, int32_t n_rows, double* y_dev,
                  void* stream);
/* computeLpcFast (features.py:222-230) for n_items dense band signals [n_items, N]:
 * a [n_items, order+1] (a0=1), gg [n_items], and the lags r [n_items, order+2]. */
int fdlp_lpc_rows(fdlp_plan* plan, const double* band_dev, int32_t n_items, double* r_dev,
                  double* a_dev, double* gg_dev, void* stream);
/* computeModSpecFromLpc (features.py:233-246): cep [n_items, lim] from a [n_items, p+1], gg. */
int fdlp_cepstrum_rows(fdlp_plan* plan, const double* a_dev, const double* gg_dev,
                       int32_t n_items, int32_t p, int32_t lim, double* cep_dev, void* stream);

/* ---- sibling feature: mel spectrum (src/featgen/computeMelSpectrum.py, run_melspec) ----- */
/* Replaces compute_mel_spectrum (computeMelSpectrum.py:40-170): getFrames with np.hamming(L),
 * |scipy.fftpack.fft(frame, nfft)[:nfft/2+1]| @ fbank.T, log10 ('log') or squared ('power'). */
typedef struct fdlp_mel_config {
  int32_t nfilters;          /* --nfilters (23)                                        (:26)   */
  int32_t nfft;              /* --nfft (1024); even, nfft/2 a 2/3/5/7-smooth size <= 2048 (:29) */
  int32_t frate;             /* --frate (100)                                          (:28)   */
  int32_t srate;             /* 16000                                                  (:40)   */
  int32_t fbank_kind;        /* --fbank_type "mel,wf" | "cochlear,om_w,alp,fixed,bet,wf" (:53-67) */
  int32_t fixed;
  int32_t power;             /* --spectrum_type: 0 log (log10), 1 power (squared)      (:150-158) */
  double fduration;          /* --fduration (0.02)                                     (:27)   */
  double warp_fact, om_w, alp, bet;
  int32_t max_frames;        /* frames per fdlp_mel_compute call                             */
} fdlp_mel_config;
typedef struct fdlp_mel_plan fdlp_mel_plan;
int fdlp_mel_plan_create(const fdlp_mel_config* cfg, int device, fdlp_mel_plan** out);
int fdlp_mel_plan_destroy(fdlp_mel_plan* plan);
/* F frames of an utterance of T samples (getFrames, features.py:151). */
int fdlp_mel_geometry(const fdlp_mel_plan* plan, int64_t T, int32_t* F);
/* A batch (fdlp_batch: pcm, offsets, lengths, noise / diff preprocessing, out [sum F, nfilters] at
 * out_row, optional fp64 copy, ark_decimals; `jitter` is unused). */
int fdlp_mel_compute(fdlp_mel_plan* plan, const fdlp_batch* batch, void* stream);

/* ---- augmentation: addReverb (features.py:110-115) -------------------------------------- */
/* --add_reverb small_room|medium_room|large_room (computeFDLPSpectrogram.py:75-91, :168-170): after the
 * optional diff / noise preprocessing, every utterance is convolved with the RIR (channel 1 of
 * ./RIR/<room>.wav / 2^15) and re-aligned on the argmax of np.correlate(x, y, 'valid').  Writes the
 * fp64 signals to out_dev at the same offsets as the input (feed them to fdlp_compute as
 * FDLP_PCM_F64 with preprocess NONE and no noise) and their lengths to out_len (T, or T-1 in the
 * reference's edge case of a best shift of R-1).  Synchronous: waits for `stream` to return the
 * lengths. */
typedef struct fdlp_reverb_batch {
  int32_t n_utt;
  int32_t pcm_kind;              /* FDLP_PCM_I16 | FDLP_PCM_F64 (f64: no preprocessing)            */
  const void* pcm_dev;
  const int64_t* pcm_off;        /* host [n_utt] */
  const int64_t* utt_len;        /* host [n_utt] */
  int32_t preprocess;            /* FDLP_PRE_DIFF or FDLP_PRE_NONE (int16 input only)              */
  const int16_t* noise_dev;      /* nullable: x = s + alpha * noise[off:off+T] before the reverb    */
  const int64_t* noise_off;      /* host [n_utt] */
  const double* noise_alpha;     /* host [n_utt] */
  const double* rir_dev;         /* device [rir_len] */
  int32_t rir_len;
  double* out_dev;               /* device f64, indexed like pcm_dev                              */
  int64_t* out_len;              /* host [n_utt] */
} fdlp_reverb_batch;
int fdlp_reverb(const fdlp_reverb_batch* batch, void* stream);

/* ---- global CMVN statistics (the step after feature extraction) ------------------------- */
/* Kaldi `compute-cmvn-stats scp:feats.scp cmvn.ark` (e2e/wsj/run_fdlp_e1.sh:280; reverb :224,
 * chime4 :193): AccCmvnStats (Kaldi transform/cmvn.cc) over `rows` feature rows [rows, dim] float32
 * on the device, ADDED into stats_dev [2, dim+1] fp64 (row 0: sum x_d, then the frame count;
 * row 1: sum of the float32 products x_d*x_d, then 0).  Deterministic (fixed-order reduction). */
int fdlp_cmvn_accumulate(const float* feats_dev, int64_t rows, int32_t dim, double* stats_dev,
                         void* stream);

/* ---- the path's device transcendental functions (for accuracy tests) ------------------------ */
/* y_dev[i] = fn(x_dev[i]) for n fp64 values on the device, with the function the path itself uses:
 * FDLP_FN_LOG the OLA stage's log of its clipped sums (computeFDLPSpectrogram.py:227 np.log; x > 0, NaN /
 * +inf pass through; a table + polynomial form within ~0.5 ulp, fdlp_device.h ola_log), FDLP_FN_EXP the
 * envelope's exp (:204-205 np.exp; the device library's exp).  ABI 8. */
enum { FDLP_FN_LOG = 0, FDLP_FN_EXP = 1 };
int fdlp_device_fn(int32_t fn, const double* x_dev, double* y_dev, int64_t n, void* stream);

/* ---- host-side RNG replicas (no device work) --------------------------------------------- */
/* CPython `random` (MT19937, init_by_array seeding, randrange(2) = getrandbits(2) with
 * rejection) -- the jitter source of computeFDLPSpectrogram.py:21,225. */
typedef struct fdlp_pyrandom fdlp_pyrandom;
int fdlp_pyrandom_create(const uint32_t* key, int32_t key_len, fdlp_pyrandom** out);
int fdlp_pyrandom_randbits2(fdlp_pyrandom* rng, int64_t n, uint8_t* out);
int fdlp_pyrandom_destroy(fdlp_pyrandom* rng);
/* numpy legacy RandomState: seed(int) = init_genrand; rand() = 53-bit double
 * (features.py:25 noise offset). */
typedef struct fdlp_nprandom fdlp_nprandom;
int fdlp_nprandom_create(uint32_t seed, fdlp_nprandom** out);
int fdlp_nprandom_rand(fdlp_nprandom* rng, int64_t n, double* out);
int fdlp_nprandom_destroy(fdlp_nprandom* rng);
/* (offset, alpha) of add_noise_to_wav (features.py:24-31) given the uniform draw u:
 * energies from int16-wrapped squares exactly like the reference. */
int fdlp_noise_params(const int16_t* sig, int64_t T, const int16_t* noise, int64_t noise_len,
                      double snr, double u, int64_t* off, double* alpha);
/* scipy.io.wavfile.read's dtype of a WAV's samples (ABI 9; fdlp_wav_kind): 8-bit PCM -> uint8, 16 -> int16,
 * 24/32 -> int32 (24-bit left-justified), 40..64 -> int64, IEEE float 32 / 64. */
enum { FDLP_SIG_U8 = 1, FDLP_SIG_I16 = 2, FDLP_SIG_I32 = 3, FDLP_SIG_I64 = 4, FDLP_SIG_F32 = 5, FDLP_SIG_F64 = 6 };
/* The same for a signal of any of those dtypes, given as the double values of scipy's array (ABI 9): the
 * reference squares the signal in its own dtype (integer squares wrap, float32 squares round to float32) and
 * np.mean sums them like numpy (8192-element chunks, pairwise inside a chunk; float32 accumulated in float32),
 * features.py:27.  The noise is int16 (noises/<name>.wav of the recipes). */
int fdlp_noise_params_any(const double* sig, int64_t T, int32_t sig_kind, const int16_t* noise,
                          int64_t noise_len, double snr, double u, int64_t* off, double* alpha);

/* ---- native I/O (replaces scipy.io.wavfile.read :139 and dict2Ark + copy-feats :231) ---- */
/* Parse a RIFF/WAVE PCM16 mono buffer.  *samples points into `buf`. */
int fdlp_wav_parse(const uint8_t* buf, int64_t len, int32_t* srate, int32_t* channels,
                   const int16_t** samples, int64_t* n_samples);
/* Any RIFF/RIFX WAVE buffer scipy.io.wavfile.read accepts (PCM 1-64 bit, <= 8 bit unsigned, 3/5/6/7-byte
 * containers left-justified; IEEE float 32/64; WAVE_FORMAT_EXTENSIBLE): sample rate, channels, frames, and
 * *is_int16 = 1 when scipy would return little-endian int16 (the samples can be used in place, fdlp_wav_parse),
 * 2 for big-endian (RIFX) int16 (decode; the values are int16), 0 otherwise.  With out != NULL the interleaved samples are written as
 * the double values of scipy's array (ABI 3). */
int fdlp_wav_decode(const uint8_t* buf, int64_t len, int32_t* srate, int32_t* channels, int32_t* is_int16,
                    int64_t* n_samples, double* out);
/* FDLP_SIG_* kind of the samples scipy.io.wavfile.read returns for this buffer (ABI 9). */
int fdlp_wav_kind(const uint8_t* buf, int64_t len, int32_t* kind);
typedef struct fdlp_ark_writer fdlp_ark_writer;
/* Kaldi binary ark + scp ("<utt> <abs ark path>:<offset>") like `copy-feats ark,t:- ark,scp:`.  Written to
 * <path>.tmp and renamed to <path> by fdlp_ark_close (removed instead after a failed write). */
int fdlp_ark_open(const char* ark_path, const char* scp_path, fdlp_ark_writer** out);
int fdlp_ark_write(fdlp_ark_writer* w, const char* utt, const float* mat, int32_t rows,
                   int32_t cols);
int fdlp_ark_close(fdlp_ark_writer* w);
/* Closes the writer and deletes <path>.tmp without publishing: the failure path of a JOB, so its outputs
 * appear complete or not at all (ABI 4). */
int fdlp_ark_abort(fdlp_ark_writer* w);
/* Kaldi matrix reader for `compute-cmvn-stats`-style rspecifiers: "scp:<feats.scp>" (lines
 * "<utt> <ark path>:<offset>") or "ark:<file>" (binary ark, "-" = stdin).  Float ("FM") and double
 * ("DM") binary matrices; data is returned as float32 (double matrices are narrowed, as Kaldi's
 * Matrix<BaseFloat> reader does).  fdlp_mat_reader_next returns 1 with a matrix, 0 at the end,
 * <0 on error; *key and *data stay valid until the next call. */
typedef struct fdlp_mat_reader fdlp_mat_reader;
int fdlp_mat_reader_open(const char* rspecifier, fdlp_mat_reader** out);
int fdlp_mat_reader_next(fdlp_mat_reader* r, const char** key, int32_t* rows, int32_t* cols,
                         const float** data);
int fdlp_mat_reader_close(fdlp_mat_reader* r);
/* Write a double matrix as a Kaldi object file (WriteKaldiObject): binary = "\0B" + "DM " + sizes
 * + row-major fp64, or Kaldi text " [\n  v v ... \n  v v ... ]\n" (%g, the ostream default). */
int fdlp_kaldi_write_dmatrix(const char* path, const double* m, int32_t rows, int32_t cols,
                             int32_t binary);

/* ---- native JOB runner (getFeats' utterance loop, computeFDLPSpectrogram.py:119-237) --------- */
/* One scp shard end to end: reader threads (files, `<cmd> |` pipes, `<ark>:<offset>` wave entries,
 * scipy's WAV formats), the reference's skip / sample-rate semantics, noise offsets and hop jitter from
 * the RNG replicas, device batches of <= batch_frames frames through fdlp_compute (copies and kernels of
 * consecutive batches overlapped), and a writer thread for <outfile>.ark/.scp (and .len), each written
 * to <name>.tmp and renamed when complete.  Progress lines go to stdout like the reference's (:185). */
typedef struct fdlp_job_opts {
  int32_t scp_type;            /* 0 wav, 1 segment (both read natively; no wav-copy needed)           */
  int32_t write_len;           /* --write_utt2num_frames                                               */
  int32_t ark_decimals;        /* '%.3f' text-ark rounding of the reference (3); <0 keeps float32      */
  int32_t batch_frames;        /* analysis frames per device batch (a longer utterance grows the plan) */
  int32_t io_threads;          /* reader threads                                                       */
  int32_t preprocess;          /* FDLP_PRE_NONE | FDLP_PRE_DIFF (--add_noise diff)                     */
  const int16_t* noise;        /* nullable host noise samples (--add_noise <type>,<snr>)              */
  int64_t noise_len;
  double snr;
  uint32_t noise_seed;         /* numpy legacy seed of the noise offsets (np.random.rand, features.py:25) */
  const uint32_t* jitter_key;  /* CPython random.seed key words of the hop jitter (:225)              */
  int32_t jitter_key_len;
  int32_t srate;               /* the sample rate the reference asserts (16000, :144)                 */
  const char* progress_name;   /* non-NULL: "<name>: Computing Features for file: <utt>" per utterance */
  const char* cmvn_path;       /* non-NULL: global CMVN stats (Kaldi binary DM) of the written features */
  int32_t out_mapped;          /* 1: the OLA kernel stores the features straight into the pinned host
                                  slots (no D2H copy); 0 (default): device buffer + D2H copy (ABI 4)   */
  /* ---- ABI 8 ---- */
  int32_t out_codes;           /* D2H leg as int16 ark codes (fdlp_batch.out_q_dev), widened to the
                                  float32 ark values on the host by a thread pool: -1 auto (codes when
                                  0 <= ark_decimals <= 3 and not out_mapped), 0 float32, 1 codes.  A
                                  batch whose codes overflow is copied again as float32 (same arks)  */
  int32_t chunk_rows;          /* feature rows per D2H piece (0: 65536); the writer starts on a batch's
                                  first piece while the rest are still in flight                     */
  int32_t keep_warm;           /* 1: keep the plan, streams and pinned slots of this call for the next
                                  call in the process with the same config (fdlp_job_release frees
                                  them); 0: release them on return                                    */
  const char* trace_path;      /* non-NULL: JSON lines of the JOB's pipeline events (seconds since the
                                  call started; benchmarks/job_timeline.py summarises them)           */
} fdlp_job_opts;
typedef struct fdlp_job_stats {
  int64_t n_lines;             /* scp entries                                  */
  int64_t n_done;              /* utterances featurised                        */
  int64_t n_skipped;           /* unreadable entries skipped (:135-142)         */
  int64_t n_frames_out;        /* feature rows written                         */
  int64_t n_samples;           /* samples featurised                           */
  double seconds;              /* wall time of the call                        */
  double setup_seconds;        /* plan creation, buffers, output files          */
  double read_wait_seconds;    /* consumer waiting for the reader threads       */
  double write_seconds;        /* writer thread busy (ark/scp/len)              */
  double slot_wait_seconds;    /* consumer waiting for a free batch slot        */
  double plan_seconds;         /* fdlp_plan_create (part of setup)              */
  double pinned_seconds;       /* pinned host buffers of the first slot (setup); the
                                  other slots are pinned by a helper thread      */
  /* ---- ABI 8 ---- */
  double d2h_wait_seconds;     /* widening stage waiting for D2H pieces to land  */
  double widen_seconds;        /* widening stage busy (codes -> float32)        */
  int64_t n_batches;           /* device batches                               */
  int64_t n_code_fallbacks;    /* batches copied again as float32 (code overflow) */
  int32_t codes;               /* 1: the D2H leg carried int16 codes            */
  int32_t warm;                /* 1: plan and slots came from the previous call */
} fdlp_job_stats;
int fdlp_job_run(const fdlp_config* cfg, int device, const char* scp_path, const char* outfile,
                 const fdlp_job_opts* opts, fdlp_job_stats* stats);
/* Frees what a keep_warm call parked (plan, streams, pinned and device slots); a no-op when nothing
 * is parked.  Call before destroying the HIP context of the process. */
int fdlp_job_release(void);

#ifdef __cplusplus
}
#endif
#endif /* FDLP_H */
