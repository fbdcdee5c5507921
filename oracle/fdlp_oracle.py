"""CPU ORACLE for the FDLP-spectrogram path -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``speech_recognition_tools_amd``) never imports anything under
``oracle/`` and fails loudly when its HIP library is missing.

It is an fp64 numpy restatement of the reference algorithm, written from the
math in SURVEY.md Appendix A, with every step citing the reference line it follows
(paths relative to the reference root ``sadhusamik/speech_recognition_tools``):

* ``src/featgen/computeFDLPSpectrogram.py`` (getFeats :29-237, argparse :240-262)
* ``src/featgen/features.py`` (getFrames :118-154, createFbank :172-190,
  createFbankCochlear :197-219, computeLpcFast :222-230,
  computeModSpecFromLpc :233-246, add_noise_to_wav :24-31, dict2Ark :63-69)

Third-party arithmetic the reference leans on is called here the same way the
reference calls it (numpy.fft / scipy.fft DCT-II / scipy.linalg.solve_toeplitz,
numpy legacy RandomState, CPython ``random``).  Versions used to pin the oracle
(numpy 2.2.6, scipy 1.15.3, CPython 3.10) are recorded in the golden fixtures.

Parity pinning: ``tests/golden/make_golden.py`` imported the real reference in the
build container and stored its outputs; ``tests/test_oracle_golden.py`` checks this
restatement against them (max-abs <= 1e-6 on the log features).

Work is vectorised across bands and frames (same per-item arithmetic as the
reference: FFT autocorrelation, Levinson via solve_toeplitz, per-coefficient
cepstrum recursion), which makes the CPU baseline stronger, not weaker.
"""
from __future__ import annotations

import math
import random as _pyrandom
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import scipy.fft as _sfft
import scipy.linalg as _sla
import scipy.stats as _sstats

SRATE = 16000          # computeFDLPSpectrogram.py:29 (getFeats default srate)
FLOOR = 1e-14          # computeFDLPSpectrogram.py:227 (np.clip a_min)


# --------------------------------------------------------------------------------------
# configuration (computeFDLPSpectrogram.py:29-118, argparse :240-262)
# --------------------------------------------------------------------------------------
@dataclass
class FdlpConfig:
    nfilters: int = 20                 # :245
    coeff_num: int = 50                # :246
    coeff_range: str = "1,20"          # :247
    order: int = 50                    # :248
    fduration: float = 0.5             # :249
    frate: int = 100                   # :250
    overlap_fraction: float = 0.25     # :251
    fbank_type: str = "mel,1"          # :254
    odd_mod_zero: bool = False         # :256
    gamma_weight: str = "None"         # :257
    lifter: Optional[np.ndarray] = None  # :258 (parsed lifter_config first line, :43-46)
    srate: int = SRATE

    @staticmethod
    def wsj():
        """e2e/wsj/run_fdlp_e1.sh:54-95 recipe values."""
        return FdlpConfig(nfilters=80, coeff_num=100, coeff_range="0,100", order=150,
                          fduration=1.5, frate=100, overlap_fraction=0.25,
                          fbank_type="cochlear,1,1,1,2.5,1")

    @staticmethod
    def reverb():
        """e2e/reverb/run_fdlp_e1.sh:61-102 recipe values (coeff_num 450, range 1..450)."""
        return FdlpConfig(nfilters=80, coeff_num=450, coeff_range="1,450", order=150,
                          fduration=1.5, frate=100, overlap_fraction=0.25,
                          fbank_type="cochlear,1,1,1,2.5,1")

    @staticmethod
    def chime4():
        """e2e/chime4/run_fdlp_e1.sh:46-87 recipe values (range 1..100)."""
        return FdlpConfig(nfilters=80, coeff_num=100, coeff_range="1,100", order=150,
                          fduration=1.5, frate=100, overlap_fraction=0.25,
                          fbank_type="cochlear,1,1,1,2.5,1")


@dataclass
class Geometry:
    """Integer geometry derived exactly like the reference (float expressions kept)."""
    N: int            # frame / DCT length: int(srate*fduration)     (features.py:134; :178)
    nfft: int         # filterbank nfft: int(2*fduration*srate)       (:53, :59)
    hop: int          # int(srate/lfr), lfr = 1/(ov*fduration)        (:174; features.py:135)
    sp_b: int         # features.py:137-144
    sp_f: int
    ext: int
    env_nfft: int     # 2*int(fduration*frate)                        (:201)
    kk: int           # int(round(fduration*frate))                   (:203)
    kkb2: int         # int(round(fduration*frate/2))                 (:204)
    ola_hop: int      # int(round(fduration*frate*ov))                (:220)


def geometry(cfg: FdlpConfig) -> Geometry:
    sr = cfg.srate
    ov = 1 - cfg.overlap_fraction                                   # :104
    N = int(sr * cfg.fduration)                                     # features.py:134
    lfr = 1 / (ov * cfg.fduration)                                  # :174
    hop = int(sr / lfr)                                             # features.py:135
    if N % 2 == 0:                                                  # features.py:137-144
        sp_b, sp_f, ext = N // 2 - 1, N // 2, N // 2 - 1
    else:
        sp_b = sp_f = ext = (N - 1) // 2
    return Geometry(
        N=N, nfft=int(2 * cfg.fduration * sr), hop=hop, sp_b=sp_b, sp_f=sp_f, ext=ext,
        env_nfft=2 * int(cfg.fduration * cfg.frate),
        kk=int(np.round(cfg.fduration * cfg.frate)),
        kkb2=int(np.round(cfg.fduration * cfg.frate / 2)),
        ola_hop=int(np.round(cfg.fduration * cfg.frate * ov)))


def n_frames(T: int, g: Geometry) -> int:
    """#frames getFrames yields: idx = sp_b + k*hop while idx + sp_f < T + 2*ext (features.py:151)."""
    k = 0
    while g.sp_b + k * g.hop + g.sp_f < T + 2 * g.ext:
        k += 1
    return k


def n_out(T: int, cfg: FdlpConfig) -> int:
    """feats width int(ceil(T*frate/srate)) (computeFDLPSpectrogram.py:182)."""
    return int(np.ceil(T * cfg.frate / cfg.srate))


# --------------------------------------------------------------------------------------
# filterbanks (features.py:172-219), nfft = int(2*fduration*srate) (:53, :59)
# --------------------------------------------------------------------------------------
def fbank_cochlear(nfilters, nfft, srate, om_w=0.2, alp=2.5, fixed=1, bet=2.5, warp_fact=1.0):
    """Bark-warped flat-top filters (features.py:193-219), vectorised."""
    bark = lambda f: 6 * np.arcsinh((f / warp_fact) / 600)          # features.py:193-194
    fmax = srate / 2
    centres = np.linspace(0, bark(fmax), nfilters)                  # :200
    fw = bark(np.linspace(0, fmax, int(np.floor(nfft / 2 + 1))))    # :201-202
    out = np.zeros((nfilters, fw.size))
    for i, fc in enumerate(centres):
        a = alp if fixed == 1 else alp * np.exp(-0.1 * fc)          # :207-210
        d = fw - fc
        lo = d <= -om_w / 2                                          # :212
        mid = (~lo) & (d < om_w / 2)                                 # :214
        hi = ~(lo | mid)
        out[i, lo] = np.power(10, a * (d[lo] + om_w / 2))
        out[i, mid] = 1
        out[i, hi] = np.power(10, -bet * (d[hi] - om_w / 2))
    return out


def fbank_mel(nfilters, nfft, srate, warp_fact=1.0):
    """Triangular mel filters (features.py:172-190)."""
    mel_max = 2595 * np.log10(1 + (srate / warp_fact) / 1400)       # :173
    mels = np.linspace(0, mel_max, nfilters + 2)                     # :174
    out = np.zeros((nfilters, int(np.floor(nfft / 2 + 1))))
    hz = warp_fact * (700 * (10 ** (mels / 2595) - 1))               # :177
    edge = np.floor((nfft + 1) * hz / srate)                         # :178
    for m in range(1, nfilters + 1):
        l, c, r = int(edge[m - 1]), int(edge[m]), int(edge[m + 1])
        k = np.arange(l, c)
        out[m - 1, k] = (k - edge[m - 1]) / (edge[m] - edge[m - 1])  # :185-186
        k = np.arange(c, r)
        out[m - 1, k] = (edge[m + 1] - k) / (edge[m + 1] - edge[m])  # :187-188
    return out


def make_fbank(cfg: FdlpConfig) -> np.ndarray:
    """computeFDLPSpectrogram.py:49-63."""
    parts = cfg.fbank_type.strip().split(',')
    nfft = int(2 * cfg.fduration * cfg.srate)
    if parts[0] == "mel":
        if len(parts) < 2:
            raise ValueError('Mel filter bank not configured properly....')
        return fbank_mel(cfg.nfilters, nfft, cfg.srate, warp_fact=float(parts[1]))
    if parts[0] == "cochlear":
        if len(parts) < 6:
            raise ValueError('Cochlear filter bank not configured properly....')
        return fbank_cochlear(cfg.nfilters, nfft, cfg.srate, om_w=float(parts[1]),
                              alp=float(parts[2]), fixed=int(parts[3]), bet=float(parts[4]),
                              warp_fact=float(parts[5]))
    raise ValueError('Invalid type of filter bank, use mel or cochlear with proper configuration')


def modulation_weights(cfg: FdlpConfig) -> np.ndarray:
    """Per-coefficient multiplier: mask (:94-103) x lifter (:195-196) x gamma (:107-118,
    :197-198) x odd-zero (:199-200).  Broadcast failures of the reference raise here too."""
    M = cfg.coeff_num
    lp, hp = (int(v) for v in cfg.coeff_range.split(','))
    w = np.array([1.0 if lp <= i <= hp else 0.0 for i in range(M)])
    if cfg.lifter is not None:
        w = w * np.asarray(cfg.lifter, dtype=np.float64)
    gw = cfg.gamma_weight.strip().split(',')
    if gw[0] != "None":
        x = np.linspace(0, cfg.order - 1, cfg.order)                 # :110
        scale, shape, pk_req = float(gw[0]), float(gw[1]), float(gw[2])
        pk_req = pk_req * 2 * cfg.fduration                          # :114-115
        loc = -(shape - 1) * scale + pk_req                          # :116-117
        w = w * (_sstats.gamma.pdf(x, a=shape, loc=loc, scale=scale) * 3 * scale)
    if cfg.odd_mod_zero:
        w = w.copy()
        w[1::2] = 0                                                  # :199-200
    return w


# --------------------------------------------------------------------------------------
# per-utterance stages
# --------------------------------------------------------------------------------------
def reflect_index(q: np.ndarray, T: int) -> np.ndarray:
    """numpy 'reflect' padding as an index map (periodic with period 2(T-1); features.py:146)."""
    if T == 1:
        return np.zeros_like(q)
    P = 2 * (T - 1)
    q = np.mod(q, P)
    return np.where(q < T, q, P - q)


def frames(signal: np.ndarray, cfg: FdlpConfig, g: Geometry) -> np.ndarray:
    """getFrames (features.py:118-154) with np.hamming (computeFDLPSpectrogram.py:29,174-176)."""
    T = signal.shape[0]
    F = n_frames(T, g)
    n = np.arange(g.N)
    win = np.hamming(g.N)
    idx = (np.arange(F)[:, None] * g.hop + n[None, :]) - g.ext
    return signal[reflect_index(idx, T)].astype(np.float64) * win


def dct_frames(fr: np.ndarray, g: Geometry) -> np.ndarray:
    """scipy.fftpack.dct(frames) / sqrt(2*N)  (computeFDLPSpectrogram.py:178)."""
    return _sfft.dct(fr, type=2, axis=-1) / np.sqrt(2 * g.N)


def autocorr_fft(band: np.ndarray, nlags: int) -> np.ndarray:
    """Circular autocorrelation, real part, via FFT (features.py:223-225); lags [0, nlags)."""
    F = np.fft.fft(band, band.shape[-1], axis=-1)
    return np.real(np.fft.ifft(F * np.conj(F), axis=-1))[..., :nlags]


def lpc_from_autocorr(r: np.ndarray, order: int) -> Tuple[np.ndarray, float]:
    """features.py:226-228: solve_toeplitz(r[0:p], -r[1:p+1]); a=[1,a']; gg=r0+sum(a*r[1:p+2])."""
    a = np.append(1.0, _sla.solve_toeplitz(r[0:order], -r[1:order + 1]))
    gg = r[0] + np.sum(a * r[1:order + 2])
    return a, gg


def cepstrum_batch(a: np.ndarray, gg: np.ndarray, M: int) -> np.ndarray:
    """computeModSpecFromLpc (features.py:233-246) for a batch [B, p+1] of LPC vectors.

    alpha_n = -a_n (n>=1), zero beyond p; c0 = log(sqrt(gg)); c1 = alpha_1;
    c_n = alpha_n + sum_{k=1}^{n-1} (k/n) alpha_{n-k} c_k  for n = 2..M-1."""
    B, P1 = a.shape
    alpha = np.zeros((B, max(P1, M + 1)))
    alpha[:, 1:P1] = -a[:, 1:]
    c = np.zeros((B, M))
    c[:, 0] = np.log(np.sqrt(gg))
    c[:, 1] = alpha[:, 1]
    for n in range(2, M):
        kn = np.arange(1, n) / n
        acc = np.sum((kn[None, :] * alpha[:, n - 1:0:-1]) * c[:, 1:n], axis=1)
        c[:, n] = acc + alpha[:, n]
    return c


def envelope_batch(cw: np.ndarray, g: Geometry) -> np.ndarray:
    """fft(c*w, 2*int(fd*fr)) -> abs(exp(.)) -> [0:kk] * hanning(kk) / hamming(kk)
    (computeFDLPSpectrogram.py:201-205)."""
    spec = _sfft.fft(cw, n=g.env_nfft, axis=-1)
    e = np.abs(np.exp(spec))[..., :g.kk]
    return e * np.hanning(g.kk) / np.hamming(g.kk)


def ola_plan(F: int, L: int, g: Geometry, jitter: Sequence[int]) -> List[Tuple[int, int, int]]:
    """(dst, src, count) per analysis frame, replicating the slicing of
    computeFDLPSpectrogram.py:207-225 including its numpy broadcast failures.
    ``jitter`` holds randrange(2) draws for frames 1..F-1 (the reference draws after
    every frame i>=1, :225)."""
    plan = []
    ptr = 0
    kk, kkb2 = g.kk, g.kkb2
    if g.ola_hop < kkb2:
        raise ValueError("unsupported: negative OLA pointer (reference would wrap a negative slice)")
    for i in range(F):
        if i == 0:
            if L < kkb2:                                            # :208-209 feats[j,:] += ms[kkb2:kkb2+L]
                rhs = max(0, min(L, kk - kkb2))
                if rhs != L:
                    raise ValueError("could not broadcast (reference OLA, frame 0)")
                plan.append((0, kkb2, L))
            else:                                                   # :211 feats[j,0:kkb2] += ms[kkb2:]
                if kk - kkb2 != kkb2:
                    raise ValueError("could not broadcast (reference OLA, frame 0)")
                plan.append((0, kkb2, kkb2))
        elif i == F - 1 or i == F - 2:                              # :212-216
            n = L - ptr
            if kk >= n:                                             # feats[j,ptr:] += ms[:n]
                lhs = max(0, n)
                rhs = n if n >= 0 else max(0, kk + n)
                if lhs != rhs:
                    raise ValueError("could not broadcast (reference OLA, tail frame)")
                plan.append((ptr, 0, lhs))
            else:                                                   # feats[j,ptr:ptr+kk] += ms
                plan.append((ptr, 0, kk))
        else:                                                       # :217-218
            if ptr + kk > L:
                raise ValueError("could not broadcast (reference OLA, middle frame)")
            plan.append((ptr, 0, kk))
        if i == 0:                                                  # :220-225
            ptr = int(ptr + g.ola_hop - kkb2)
        else:
            ptr = int(ptr + g.ola_hop + jitter[i - 1])
    return plan


# --------------------------------------------------------------------------------------
# augmentation (features.py:24-31; computeFDLPSpectrogram.py:160-166)
# --------------------------------------------------------------------------------------
DIFF_KERNEL = np.array([1, 2, 3, 2, 0, -2, -5, -2, 0, 2, 3, 2, 1])   # :163


def diff_signal(sig: np.ndarray) -> np.ndarray:
    """scipy.signal.convolve(sig, a, 'same') (:162-164): integer input (int16 / int32 / uint8) -> int64, exact;
    float input -> float64 (scipy's direct route for a 13-tap kernel: np.convolve in float64)."""
    if not np.issubdtype(sig.dtype, np.integer):
        full = np.convolve(sig.astype(np.float64), DIFF_KERNEL.astype(np.float64))
        off = (DIFF_KERNEL.size - 1) // 2
        return full[off:off + sig.size]
    full = np.convolve(sig.astype(np.int64), DIFF_KERNEL)
    off = (DIFF_KERNEL.size - 1) // 2
    return full[off:off + sig.size]


def noise_mix_params(sig: np.ndarray, noise: np.ndarray, snr: float, u: float):
    """(offset, alpha) of add_noise_to_wav with the draw u = np.random.rand() (features.py:24-29).
    sig**2 and ns**2 stay in their own dtypes (int16 wraps) like the reference; sig may be any dtype
    scipy.io.wavfile returns (uint8, int16, int32, int64, float32, float64)."""
    off = int(np.floor(u * (len(noise) - len(sig))))
    ns = noise[off:off + len(sig)]
    Es = np.mean(sig ** 2)
    En = np.mean(ns ** 2)
    alp = np.sqrt(Es / (En * (10 ** (snr / 10))))
    return off, alp


def add_noise(sig, noise, snr, u):
    off, alp = noise_mix_params(sig, noise, snr, u)
    return sig + alp * noise[off:off + len(sig)]


def add_reverb(sig: np.ndarray, rir: np.ndarray) -> np.ndarray:
    """addReverb (features.py:110-115): full convolution with the RIR, then the T samples that start one
    past the best-correlated shift: np.correlate(sig, out, 'valid')[k] = sum_n sig[n] out[n + R-1-k], so
    indM = R - argmax = s* + 1 with s* the largest shift attaining the maximum."""
    out = np.convolve(sig, rir)
    xxc = np.correlate(sig, out, 'valid')
    indM = len(xxc) - np.argmax(xxc)
    return out[indM:indM + len(sig)]


def load_rir(stereo_int16: np.ndarray) -> np.ndarray:
    """RIR as the reference loads it (computeFDLPSpectrogram.py:75-87): channel 1 of the stereo WAV / 2**15."""
    return stereo_int16[:, 1] / np.power(2, 15)


# --------------------------------------------------------------------------------------
# whole pipeline
# --------------------------------------------------------------------------------------
@dataclass
class Intermediates:
    frames: np.ndarray = None
    dct: np.ndarray = None
    r: np.ndarray = None
    a: np.ndarray = None
    gg: np.ndarray = None
    cep: np.ndarray = None
    env: np.ndarray = None


class FdlpOracle:
    """Reusable CPU pipeline; state = precomputed filterbank and weights (getFeats :43-118)."""

    def __init__(self, cfg: FdlpConfig):
        self.cfg = cfg
        self.g = geometry(cfg)
        self.fbank = make_fbank(cfg)
        self.w = modulation_weights(cfg)
        if self.fbank.shape[1] - 1 != self.g.N:
            raise ValueError("filterbank width does not match the frame length (reference broadcast)")

    def band_envelopes(self, signal: np.ndarray, keep: Optional[Intermediates] = None) -> np.ndarray:
        """[F, B, kk] envelopes of one utterance (computeFDLPSpectrogram.py:172-205)."""
        cfg, g = self.cfg, self.g
        fr = frames(signal, cfg, g)
        if fr.shape[0] == 0:
            raise ValueError("invalid number of data points (0) specified")  # scipy dct on empty
        D = dct_frames(fr, g)
        F, B, p = D.shape[0], cfg.nfilters, cfg.order
        bands = self.fbank[None, :, :-1] * D[:, None, :]            # :190-191
        r = autocorr_fft(bands.reshape(F * B, -1), p + 2)
        a = np.empty((F * B, p + 1))
        gg = np.empty(F * B)
        for t in range(F * B):
            a[t], gg[t] = lpc_from_autocorr(r[t], p)
        cep = cepstrum_batch(a, gg, cfg.coeff_num)                  # :193
        env = envelope_batch(cep * self.w[None, :], g)              # :194-205
        if keep is not None:
            keep.frames, keep.dct, keep.r, keep.a, keep.gg, keep.cep, keep.env = \
                fr, D, r.reshape(F, B, -1), a.reshape(F, B, -1), gg.reshape(F, B), \
                cep.reshape(F, B, -1), env.reshape(F, B, -1)
        return env.reshape(F, B, -1)

    def utterance(self, signal: np.ndarray, rng: _pyrandom.Random,
                  keep: Optional[Intermediates] = None) -> np.ndarray:
        """log FDLP spectrogram [L, B] fp64 (computeFDLPSpectrogram.py:172-227).
        ``rng`` supplies the randrange(2) hop jitter (:225) in the reference's draw order."""
        cfg, g = self.cfg, self.g
        T = signal.shape[0]
        env = self.band_envelopes(signal, keep)
        F = env.shape[0]
        L = n_out(T, cfg)
        jit = [rng.randrange(2) for _ in range(F - 1)]
        feats = np.zeros((cfg.nfilters, L))
        for i, (dst, src, cnt) in enumerate(ola_plan(F, L, g, jit)):
            if cnt > 0:
                feats[:, dst:dst + cnt] += env[i, :, src:src + cnt]
        return np.log(np.clip(feats.T, a_max=None, a_min=FLOOR))    # :227


def compute_utterances(cfg: FdlpConfig, signals: Dict[str, np.ndarray], seed: int,
                       noise: Optional[np.ndarray] = None, snr: Optional[float] = None,
                       noise_seed: Optional[int] = None, diff: bool = False,
                       rir: Optional[np.ndarray] = None) -> Dict[str, np.ndarray]:
    """getFeats over an ordered dict of int16 signals with a seeded jitter stream
    (random.seed(seed), :21,:225) and optionally seeded noise mixing (np.random.seed)."""
    orc = FdlpOracle(cfg)
    rng = _pyrandom.Random(seed)
    nrng = np.random.RandomState(noise_seed) if noise is not None else None
    out = {}
    for utt, sig in signals.items():
        x = sig
        if diff:
            x = diff_signal(sig)
        elif noise is not None:
            x = add_noise(sig, noise, snr, nrng.rand())
        if rir is not None:                                            # :168-170
            x = add_reverb(x, rir)
        out[utt] = orc.utterance(x, rng)
    return out
