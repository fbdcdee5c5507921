"""FDLP plan: the reference's getFeats setup (computeFDLPSpectrogram.py:43-118) frozen into a
device-resident plan, plus batched compute over torch device tensors.

The plan owns its HBM workspace (sized by ``max_frames`` analysis frames per call) and is used
from one stream at a time.
"""
import ctypes
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import FdlpBatchC, check, lib, ptr
from .config import DEFAULT_SUPPORT_EPS, FeatureConfig  # noqa: F401  (re-exported)
from . import ops  # noqa: F401,E402  (registers torch.ops.fdlp.spectrogram)

if not _lib.TORCH_RUNTIME:
    raise ImportError("libfdlp_hip.so was loaded without torch's HIP runtime (native CLI mode); FdlpPlan needs "
                      "torch imported before the library")

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
                stream: Optional[torch.cuda.Stream] = None, preprocess: Optional[str] = None,
                out_q: Optional[torch.Tensor] = None, q_flag: Optional[torch.Tensor] = None):
        """Features of a batch of utterances whose samples are concatenated in ``pcm`` (device).

        ``out_q`` (int16 [>= sum L, B], device or pinned host) receives the compact ark codes (ABI 7,
        include/fdlp.h): ``q_widen`` turns them into the float32 rows bit for bit; ``q_flag`` (int32
        device or pinned tensor, zeroed by the caller) becomes non-zero when a value has no code.  With
        ``out_q`` and no ``out`` no float32 rows are written.

        Returns (feats float32 [sum L, B] or None, row offsets int64 [n_utt+1], feats_f64 or None)."""
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
        if out is None and out_q is None:
            out = torch.empty((total, D), dtype=torch.float32, device=dev)
        elif out is not None and (out.shape[0] < total or out.shape[1] != D or out.dtype != torch.float32
                                  or not out.is_contiguous()):
            raise ValueError("out buffer too small")
        if out_q is not None:
            if (out_q.dtype != torch.int16 or out_q.dim() != 2 or out_q.shape[0] < total or out_q.shape[1] != D
                    or not out_q.is_contiguous()):
                raise ValueError("out_q must be a contiguous int16 [>= sum L, out_dim] tensor")
            if q_flag is None or q_flag.dtype != torch.int32 or q_flag.numel() < 1:
                raise ValueError("out_q needs q_flag (an int32 tensor of at least one element)")
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
        b.out_dev = _dev_ptr(out, "out") if out is not None else None
        if out_q is not None:
            b.out_q_dev, b.out_q_flag_dev = _dev_ptr(out_q, "out_q"), _dev_ptr(q_flag, "q_flag")
        rows_c = np.ascontiguousarray(rows[:-1])
        b.out_row = ptr(rows_c, ctypes.c_int64)
        b.out_f64_dev = out64.data_ptr() if out64 is not None else None
        b.ark_decimals = int(ark_decimals)
        if preprocess not in (None, "diff"):
            raise ValueError("preprocess must be None or 'diff'")
        b.preprocess = _lib.FDLP_PRE_DIFF if preprocess == "diff" else _lib.FDLP_PRE_NONE
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        check(lib.fdlp_compute(self._h, ctypes.byref(b), ctypes.c_void_p(s.cuda_stream)))
        return (out[:total] if out is not None else None), rows, out64

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

    LPC_PATHS = {"auto": 0, "lds": 1, "lattice8": 2}

    def set_lpc_path(self, path: str = "auto"):
        """'auto': the lattice kernels (durbin4_kernel for 128 <= p <= 150, durbin8_kernel above, then the
        register cepstrum / envelope kernel); 'lattice8': the same with durbin8_kernel for every p it
        covers (cross-check of durbin4_kernel); 'lds': the LDS Durbin kernel (the large-p fallback, an
        independent cross-check)."""
        check(lib.fdlp_set_lpc_path(self._h, self.LPC_PATHS[path]))

    DCT_PATHS = {"auto": 0, "four_step": 1}

    def set_dct_path(self, path: str = "auto"):
        """'auto': the recipes' N = 24000 DCT as one kernel per frame (dct_frame_kernel), other N the
        four-step pair; 'four_step': the two four-step kernels through the Z workspace."""
        check(lib.fdlp_set_dct_path(self._h, self.DCT_PATHS[path]))

    @property
    def dct_path(self) -> str:
        v = lib.fdlp_dct_path(self._h)
        if v < 0:
            check(v)
        return {1: "four_step", 2: "frame"}[v]

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

    def set_profiling(self, enable=True, kernels: bool = False):
        """Per-stage HIP events on every fdlp_compute; kernels=True also marks every kernel launch
        (kernel_times)."""
        check(lib.fdlp_set_profiling(self._h, (2 if kernels else 1) if enable else 0))

    def kernel_times(self):
        """{kernel name: (summed ms, launches)} of the profiled calls (set_profiling(kernels=True)): the time
        between consecutive HIP events on the kernels' stream, one kernel each."""
        ms = np.zeros(_lib.FDLP_NUM_KERNELS, dtype=np.float64)
        n = np.zeros(_lib.FDLP_NUM_KERNELS, dtype=np.int64)
        check(lib.fdlp_kernel_times(self._h, ptr(ms, ctypes.c_double), ptr(n, ctypes.c_int64)))
        return {lib.fdlp_kernel_name(k).decode(): (float(ms[k]), int(n[k]))
                for k in range(_lib.FDLP_NUM_KERNELS) if n[k] > 0}

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


def _dev_ptr(t: torch.Tensor, name: str) -> int:
    """Device address of a device tensor, or of a pinned host tensor through its device mapping (the
    kernel then stores straight into host memory)."""
    if t.is_cuda:
        return t.data_ptr()
    if t.is_pinned():
        dp = ctypes.c_void_p()
        check(lib.fdlp_mapped_ptr(ctypes.c_void_p(t.data_ptr()), ctypes.byref(dp)))
        return dp.value
    raise ValueError("%s must be a device tensor or a pinned host tensor" % name)


def q_widen(q, decimals: int = 3, threads: int = 1, out: Optional[np.ndarray] = None) -> np.ndarray:
    """float32 ark values of compact codes (host int16 array or CPU tensor; fdlp_q_widen): bitwise the
    float32 rows fdlp_compute writes to ``out`` with the same ark_decimals."""
    qa = np.ascontiguousarray(q.numpy() if isinstance(q, torch.Tensor) else q, dtype=np.int16)
    if out is None:
        out = np.empty(qa.shape, dtype=np.float32)
    elif out.dtype != np.float32 or out.size < qa.size or not out.flags.c_contiguous:
        raise ValueError("out must be a contiguous float32 array of at least q.size elements")
    check(lib.fdlp_q_widen(qa.ctypes.data, qa.size, int(decimals), out.ctypes.data, int(threads)))
    return out


def device_checks(reset: bool = False):
    """(enabled, violations, last_line) of the device range checks (fdlp_device_checks): enabled only in a
    library built with -DFDLP_DEVICE_CHECKS=1 (loaded through FDLP_LIB); synchronises the device."""
    en, v, ln = ctypes.c_int32(), ctypes.c_uint32(), ctypes.c_uint32()
    check(lib.fdlp_device_checks(ctypes.byref(en), ctypes.byref(v), ctypes.byref(ln), int(bool(reset))))
    return bool(en.value), int(v.value), int(ln.value)
