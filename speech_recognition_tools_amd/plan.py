"""FDLP plan: the reference's getFeats setup (computeFDLPSpectrogram.py:43-118) frozen into a
device-resident plan, plus batched compute over torch device tensors.

The plan owns its HBM workspace (sized by ``max_frames`` analysis frames per call) and is used
from one stream at a time.
"""
import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import FdlpBatchC, FdlpConfigC, check, lib, ptr

DEFAULT_SUPPORT_EPS = 1e-12


@dataclass
class FeatureConfig:
    """Parsed form of the reference argv (computeFDLPSpectrogram.py:240-262, :43-118)."""
    nfilters: int = 20
    coeff_num: int = 50
    coeff_range: str = "1,20"
    order: int = 50
    fduration: float = 0.5
    frate: int = 100
    overlap_fraction: float = 0.25
    fbank_type: str = "mel,1"
    odd_mod_zero: bool = False
    gamma_weight: str = "None"
    lifter: Optional[Sequence[float]] = None
    srate: int = 16000
    support_eps: float = DEFAULT_SUPPORT_EPS
    # modulation spectrum (computeModulationSpectrum.py): mode "modspec" ("modspec_complex" with
    # --complex_modulation), coeff_num = --coeff_n
    mode: str = "spectrogram"
    window: str = "hamming"           # "hamming" (:29) | "hanning" (modspec :30) | "rect" (--no_window)
    coeff_0: int = 1
    keep_even: bool = False
    compensate_noise: bool = False
    absolute_value: bool = False

    def to_c(self, max_frames: int):
        c = FdlpConfigC()
        c.nfilters, c.coeff_num, c.order = int(self.nfilters), int(self.coeff_num), int(self.order)
        lp, hp = (int(v) for v in self.coeff_range.split(','))               # :94-96
        c.coeff_lp, c.coeff_hp = lp, hp
        c.frate, c.srate = int(self.frate), int(self.srate)
        c.fduration, c.overlap_fraction = float(self.fduration), float(self.overlap_fraction)
        parts = self.fbank_type.strip().split(',')                            # :49-63
        if parts[0] == "mel":
            if len(parts) < 2:
                raise ValueError('Mel filter bank not configured properly....')
            c.fbank_kind, c.warp_fact = _lib.FDLP_FBANK_MEL, float(parts[1])
        elif parts[0] == "cochlear":
            if len(parts) < 6:
                raise ValueError('Cochlear filter bank not configured properly....')
            c.fbank_kind = _lib.FDLP_FBANK_COCHLEAR
            c.om_w, c.alp, c.fixed = float(parts[1]), float(parts[2]), int(parts[3])
            c.bet, c.warp_fact = float(parts[4]), float(parts[5])
        else:
            raise ValueError('Invalid type of filter bank, use mel or cochlear with proper configuration')
        c.odd_mod_zero = int(bool(self.odd_mod_zero))
        gw = self.gamma_weight.strip().split(',')                             # :107-118
        if gw[0] != "None":
            c.gamma_enabled = 1
            c.gamma_scale, c.gamma_shape, c.gamma_pk = float(gw[0]), float(gw[1]), float(gw[2])
        keep = None
        if self.lifter is not None:
            keep = np.ascontiguousarray(np.asarray(self.lifter, dtype=np.float64))
            c.lifter, c.lifter_len = ptr(keep, ctypes.c_double), keep.size
        c.support_eps = float(self.support_eps)
        c.max_frames = int(max_frames)
        c.mode = {"spectrogram": _lib.FDLP_MODE_SPECTROGRAM, "modspec": _lib.FDLP_MODE_MODSPEC,
                  "modspec_complex": _lib.FDLP_MODE_MODSPEC_COMPLEX}[self.mode]
        c.window = {"hamming": _lib.FDLP_WIN_HAMMING, "hanning": _lib.FDLP_WIN_HANNING,
                    "rect": _lib.FDLP_WIN_RECT}[self.window]
        c.coeff_0, c.keep_even = int(self.coeff_0), int(bool(self.keep_even))
        c.compensate_noise, c.absolute_value = int(bool(self.compensate_noise)), int(bool(self.absolute_value))
        return c, keep

    @staticmethod
    def from_args(args, support_eps=None):
        """From an argparse namespace with the reference's option names."""
        lifter = None
        if getattr(args, "lifter_config", None):
            with open(args.lifter_config, 'r') as fid:                        # :43-46
                lifter = [float(x) for x in fid.readline().strip().split(',')]
        eps = getattr(args, "support_eps", None) if support_eps is None else support_eps
        return FeatureConfig(
            nfilters=args.nfilters, coeff_num=args.coeff_num, coeff_range=args.coeff_range,
            order=args.order, fduration=args.fduration, frate=args.frate,
            overlap_fraction=args.overlap_fraction, fbank_type=args.fbank_type,
            odd_mod_zero=bool(args.odd_mod_zero), gamma_weight=args.gamma_weight, lifter=lifter,
            support_eps=DEFAULT_SUPPORT_EPS if eps is None else float(eps))

    @staticmethod
    def wsj():
        """e2e/wsj/run_fdlp_e1.sh:54-95."""
        return FeatureConfig(nfilters=80, coeff_num=100, coeff_range="0,100", order=150,
                             fduration=1.5, frate=100, overlap_fraction=0.25,
                             fbank_type="cochlear,1,1,1,2.5,1")

    @staticmethod
    def reverb():
        """e2e/reverb/run_fdlp_e1.sh:61-102."""
        return FeatureConfig(nfilters=80, coeff_num=450, coeff_range="1,450", order=150,
                             fduration=1.5, frate=100, overlap_fraction=0.25,
                             fbank_type="cochlear,1,1,1,2.5,1")

    @staticmethod
    def chime4():
        """e2e/chime4/run_fdlp_e1.sh:46-87."""
        return FeatureConfig(nfilters=80, coeff_num=100, coeff_range="1,100", order=150,
                             fduration=1.5, frate=100, overlap_fraction=0.25,
                             fbank_type="cochlear,1,1,1,2.5,1")


class FdlpPlan:
    """Device plan.  ``device=-1`` builds a host-only plan (geometry/filterbank/OLA tables)."""

    def __init__(self, cfg: FeatureConfig, device: int = 0, max_frames: int = 4096):
        self.cfg = cfg
        self.device = device
        self.max_frames = int(max_frames)
        c, self._keep = cfg.to_c(max_frames)
        h = ctypes.c_void_p()
        check(lib.fdlp_plan_create(ctypes.byref(c), int(device), ctypes.byref(h)))
        self._h = h
        v = [_lib.c_i32() for _ in range(5)]
        check(lib.fdlp_plan_info(h, *[ctypes.byref(x) for x in v]))
        self.N, self.hop, self.nlags, self.kk, self.ola_hop = (x.value for x in v)
        self.B = int(cfg.nfilters)
        d = _lib.c_i32()
        check(lib.fdlp_plan_out_dim(h, ctypes.byref(d)))
        self.out_dim = d.value  # nfilters, or nfilters * feat_len in the modspec mode

    @property
    def op_id(self) -> int:
        """Id of this plan for the torch.ops.fdlp.spectrogram operator (speech_recognition_tools_amd.ops)."""
        if getattr(self, "_op_id", None) is None:
            from .ops import register_plan
            self._op_id = register_plan(self)
        return self._op_id

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            lib.fdlp_plan_destroy(h)
            self._h = None

    def __del__(self):
        self.close()

    # ---- host-side plan queries --------------------------------------------------------
    def geometry(self, T: int):
        F, L = _lib.c_i32(), _lib.c_i32()
        check(lib.fdlp_geometry(self._h, int(T), ctypes.byref(F), ctypes.byref(L)))
        return F.value, L.value

    def fbank(self):
        ncol = self.N + 1
        fb = np.empty((self.B, ncol), dtype=np.float64)
        lo = np.empty(self.B, dtype=np.int32)
        hi = np.empty(self.B, dtype=np.int32)
        check(lib.fdlp_plan_fbank(self._h, ptr(fb, ctypes.c_double), ptr(lo, ctypes.c_int32),
                                  ptr(hi, ctypes.c_int32)))
        return fb, lo, hi

    def weights(self):
        w = np.empty(int(self.cfg.coeff_num), dtype=np.float64)
        check(lib.fdlp_plan_weights(self._h, ptr(w, ctypes.c_double)))
        return w

    def ola_table(self, T: int, jitter: np.ndarray):
        F, _ = self.geometry(T)
        jit = np.ascontiguousarray(jitter, dtype=np.uint8)
        if jit.size < max(F - 1, 0):
            raise ValueError("need F-1 jitter draws")
        d, s, c = (np.empty(F, dtype=np.int32) for _ in range(3))
        check(lib.fdlp_ola_table(self._h, int(T), ptr(jit, ctypes.c_uint8), ptr(d, ctypes.c_int32),
                                 ptr(s, ctypes.c_int32), ptr(c, ctypes.c_int32)))
        return d, s, c

    # ---- compute ---------------------------------------------------------------------------
    def compute(self, pcm: torch.Tensor, lengths: Sequence[int], jitter: np.ndarray,
                offsets: Optional[Sequence[int]] = None, noise: Optional[torch.Tensor] = None,
                noise_off: Optional[Sequence[int]] = None, noise_alpha: Optional[Sequence[float]] = None,
                ark_decimals: int = 3, want_f64: bool = False, out: Optional[torch.Tensor] = None,
                stream: Optional[torch.cuda.Stream] = None, preprocess: Optional[str] = None):
        """Features of a batch of utterances whose samples are concatenated in ``pcm`` (device).

        Returns (feats float32 [sum L, B], row offsets int64 [n_utt+1], feats_f64 or None)."""
        if not pcm.is_cuda:
            raise ValueError("pcm must be a device tensor")
        if pcm.dtype == torch.int16:
            kind = _lib.FDLP_PCM_I16
        elif pcm.dtype == torch.float64:
            kind = _lib.FDLP_PCM_F64
        else:
            raise TypeError("pcm must be int16 or float64")
        pcm = pcm.contiguous()
        lens = np.ascontiguousarray(np.asarray(lengths, dtype=np.int64))
        n = lens.size
        if offsets is None:
            offs = np.zeros(n, dtype=np.int64)
            if n:
                offs[1:] = np.cumsum(lens)[:-1]
        else:
            offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
        if n and int((offs + lens).max()) > pcm.numel():
            raise ValueError("utterance extends past the PCM buffer")
        Ls = np.array([self.geometry(int(T))[1] for T in lens], dtype=np.int64)
        rows = np.zeros(n + 1, dtype=np.int64)
        rows[1:] = np.cumsum(Ls)
        total = int(rows[-1])
        dev = pcm.device
        D = self.out_dim
        if out is None:
            out = torch.empty((total, D), dtype=torch.float32, device=dev)
        elif out.shape[0] < total or out.shape[1] != D or out.dtype != torch.float32:
            raise ValueError("out buffer too small")
        out64 = torch.empty((total, D), dtype=torch.float64, device=dev) if want_f64 else None
        jit = np.ascontiguousarray(np.zeros(1) if jitter is None else jitter, dtype=np.uint8)
        b = FdlpBatchC()
        b.n_utt, b.pcm_kind, b.pcm_dev = n, kind, pcm.data_ptr()
        b.pcm_off, b.utt_len, b.jitter = ptr(offs, ctypes.c_int64), ptr(lens, ctypes.c_int64), ptr(jit, ctypes.c_uint8)
        keep = []
        if noise is not None:
            if noise.dtype != torch.int16 or not noise.is_cuda:
                raise TypeError("noise must be an int16 device tensor")
            no = np.ascontiguousarray(np.asarray(noise_off, dtype=np.int64))
            na = np.ascontiguousarray(np.asarray(noise_alpha, dtype=np.float64))
            keep += [no, na]
            b.noise_dev, b.noise_off, b.noise_alpha = noise.data_ptr(), ptr(no, ctypes.c_int64), ptr(na, ctypes.c_double)
        b.out_dev = out.data_ptr()
        rows_c = np.ascontiguousarray(rows[:-1])
        b.out_row = ptr(rows_c, ctypes.c_int64)
        b.out_f64_dev = out64.data_ptr() if out64 is not None else None
        b.ark_decimals = int(ark_decimals)
        if preprocess not in (None, "diff"):
            raise ValueError("preprocess must be None or 'diff'")
        b.preprocess = _lib.FDLP_PRE_DIFF if preprocess == "diff" else _lib.FDLP_PRE_NONE
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        check(lib.fdlp_compute(self._h, ctypes.byref(b), ctypes.c_void_p(s.cuda_stream)))
        return out[:total], rows, out64

    AUTOCORR_PATHS = {"auto": 0, "direct": 1, "structured": 2, "structured_mfma": 3}

    @property
    def autocorr_path(self) -> str:
        """'direct' (per band over the taps >= support_eps*peak) or 'structured' (exact
        skirt-factorised algorithm, cochlear filterbank with fixed=1)."""
        v = lib.fdlp_autocorr_path(self._h)
        check(v if v < 0 else 0)
        return {1: "direct", 2: "structured", 3: "structured_mfma"}[v]

    def set_autocorr_path(self, path: str = "auto"):
        check(lib.fdlp_set_autocorr_path(self._h, self.AUTOCORR_PATHS[path]))

    LPC_PATHS = {"auto": 0, "lds": 1}

    def set_lpc_path(self, path: str = "auto"):
        """'auto': the lattice kernels (durbin8_kernel + register cepstrum / envelope); 'lds': the LDS
        Durbin kernel (the large-p fallback, an independent cross-check)."""
        check(lib.fdlp_set_lpc_path(self._h, self.LPC_PATHS[path]))

    def regions(self):
        """(m1, m2) int32 arrays: band j's lower skirt [0,m1), flat top [m1,m2), upper skirt [m2,N)."""
        m1 = np.empty(self.B, dtype=np.int32)
        m2 = np.empty(self.B, dtype=np.int32)
        check(lib.fdlp_plan_regions(self._h, ptr(m1, ctypes.c_int32), ptr(m2, ctypes.c_int32)))
        return m1, m2

    def flat_events(self):
        """(chains, parts, events[n, 4] = (S, band, type, chain)) of the flat-top sweep, sweep order;
        chains == 0 when the lag-parallel VALU sweeps are not available for this plan."""
        C, H, n = _lib.c_i32(), _lib.c_i32(), _lib.c_i32()
        check(lib.fdlp_plan_flat_events(self._h, ctypes.byref(C), ctypes.byref(H), ctypes.byref(n), None, 0))
        ev = np.zeros((n.value, 4), dtype=np.int32)
        check(lib.fdlp_plan_flat_events(self._h, None, None, ctypes.byref(n), ptr(ev, ctypes.c_int32), n.value))
        return C.value, H.value, ev

    def set_pipeline(self, n_sub: int):
        check(lib.fdlp_set_pipeline(self._h, int(n_sub)))

    def set_debug(self, keep_intermediates: bool = True):
        check(lib.fdlp_set_debug(self._h, int(bool(keep_intermediates))))

    def debug_fetch(self, n_frames: int, first_frame: int = 0, keys=("dct", "r", "a", "gg", "cep", "env")):
        """Intermediates of frames [first_frame, first_frame + n_frames) of the last batch; a/gg/cep
        need set_debug(True) before the compute."""
        F, B = int(n_frames), self.B
        p, M = int(self.cfg.order), int(self.cfg.coeff_num)
        shapes = dict(dct=(F, self.N), r=(F, B, self.nlags), a=(F, B, p + 1), gg=(F, B), cep=(F, B, M),
                      env=(F, B, self.kk))
        d = {k: np.empty(shapes[k]) for k in keys}
        check(lib.fdlp_debug_fetch_range(self._h, int(first_frame), F,
                                         *[ptr(d[k], ctypes.c_double) if k in d else None
                                           for k in ("dct", "r", "a", "gg", "cep", "env")]))
        return d

    def set_profiling(self, enable: bool = True):
        check(lib.fdlp_set_profiling(self._h, int(bool(enable))))

    def stage_times(self):
        """{stage: summed ms} over the profiled fdlp_compute calls, and the call count."""
        ms = np.zeros(_lib.FDLP_NUM_STAGES, dtype=np.float64)
        n = _lib.c_i32()
        check(lib.fdlp_stage_times(self._h, ptr(ms, ctypes.c_double), ctypes.byref(n)))
        return dict(zip(_lib.STAGE_NAMES, ms.tolist())), n.value

    # ---- stage entry points (features.py helpers, batched) ---------------------------------
    def dct_rows(self, x: torch.Tensor) -> torch.Tensor:
        x = x.contiguous()
        assert x.dtype == torch.float64 and x.is_cuda and x.shape[-1] == self.N
        y = torch.empty_like(x)
        s = torch.cuda.current_stream(x.device)
        check(lib.fdlp_dct_rows(self._h, x.data_ptr(), x.shape[0], y.data_ptr(), s.cuda_stream))
        return y

    def lpc_rows(self, band: torch.Tensor):
        band = band.contiguous()
        assert band.dtype == torch.float64 and band.is_cuda and band.shape[-1] == self.N
        n = band.shape[0]
        p = int(self.cfg.order)
        r = torch.empty((n, self.nlags), dtype=torch.float64, device=band.device)
        a = torch.empty((n, p + 1), dtype=torch.float64, device=band.device)
        gg = torch.empty((n,), dtype=torch.float64, device=band.device)
        s = torch.cuda.current_stream(band.device)
        check(lib.fdlp_lpc_rows(self._h, band.data_ptr(), n, r.data_ptr(), a.data_ptr(), gg.data_ptr(),
                                s.cuda_stream))
        return r, a, gg

    def cepstrum_rows(self, a: torch.Tensor, gg: torch.Tensor, lim: int) -> torch.Tensor:
        a = a.contiguous()
        gg = gg.contiguous()
        n, p1 = a.shape
        cep = torch.empty((n, int(lim)), dtype=torch.float64, device=a.device)
        s = torch.cuda.current_stream(a.device)
        check(lib.fdlp_cepstrum_rows(self._h, a.data_ptr(), gg.data_ptr(), n, p1 - 1, int(lim), cep.data_ptr(),
                                     s.cuda_stream))
        return cep
