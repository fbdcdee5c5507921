"""Mel spectrum on the MI355X: the reference's sibling feature src/featgen/computeMelSpectrum.py
(compute_mel_spectrum :40-170, driven by recipes/timit/local_pyspeech/make_melspectrum_feats.sh), the
run_melspec baseline the FDLP features are compared with.

Per frame (getFrames, features.py:118-154, np.hamming window): log10(|fft(frame, nfft)[:nfft/2+1]| @ fbank.T)
('log') or its square ('power').  One plan per configuration (filterbank, window, FFT tables resident in
HBM); mel_kernel (fdlp_misc.hip) does frame gather, real FFT in LDS, magnitude, projection and log.
"""
import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import FdlpBatchC, FdlpMelConfigC, check, lib, ptr


@dataclass
class MelConfig:
    """Parsed argv of computeMelSpectrum.py (get_args :20-37)."""
    nfilters: int = 23
    fduration: float = 0.02
    frate: int = 100
    nfft: int = 1024
    fbank_type: str = "mel,1"
    spectrum_type: str = "log"
    srate: int = 16000

    def to_c(self, max_frames: int) -> FdlpMelConfigC:
        c = FdlpMelConfigC()
        c.nfilters, c.nfft, c.frate, c.srate = int(self.nfilters), int(self.nfft), int(self.frate), int(self.srate)
        c.fduration = float(self.fduration)
        parts = self.fbank_type.strip().split(',')                                  # :53-67
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
        if self.spectrum_type not in ("log", "power"):
            raise ValueError("Spectrum type not supported! ")
        c.power = 1 if self.spectrum_type == "power" else 0
        c.max_frames = int(max_frames)
        return c


class MelPlan:
    def __init__(self, cfg: MelConfig, device: int = 0, max_frames: int = 65536):
        self.cfg = cfg
        self.device = device
        self.max_frames = int(max_frames)
        c = cfg.to_c(max_frames)
        h = ctypes.c_void_p()
        check(lib.fdlp_mel_plan_create(ctypes.byref(c), int(device), ctypes.byref(h)))
        self._h = h
        self.B = int(cfg.nfilters)

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            lib.fdlp_mel_plan_destroy(h)
            self._h = None

    def __del__(self):
        self.close()

    def frames(self, T: int) -> int:
        F = _lib.c_i32()
        check(lib.fdlp_mel_geometry(self._h, int(T), ctypes.byref(F)))
        return F.value

    def compute(self, pcm: torch.Tensor, lengths: Sequence[int], offsets: Optional[Sequence[int]] = None,
                noise: Optional[torch.Tensor] = None, noise_off=None, noise_alpha=None, preprocess=None,
                ark_decimals: int = 3, want_f64: bool = False, stream=None):
        """(feats float32 [sum F, B], row offsets [n+1], feats_f64 or None) of a batch on the device."""
        if not pcm.is_cuda:
            raise ValueError("pcm must be a device tensor")
        kind = _lib.FDLP_PCM_I16 if pcm.dtype == torch.int16 else _lib.FDLP_PCM_F64
        if pcm.dtype not in (torch.int16, torch.float64):
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
        Fs = np.array([self.frames(int(T)) for T in lens], dtype=np.int64)
        rows = np.zeros(n + 1, dtype=np.int64)
        rows[1:] = np.cumsum(Fs)
        total = int(rows[-1])
        out = torch.empty((total, self.B), dtype=torch.float32, device=pcm.device)
        out64 = torch.empty((total, self.B), dtype=torch.float64, device=pcm.device) if want_f64 else None
        b = FdlpBatchC()
        b.n_utt, b.pcm_kind, b.pcm_dev = n, kind, pcm.data_ptr()
        b.pcm_off, b.utt_len = ptr(offs, ctypes.c_int64), ptr(lens, ctypes.c_int64)
        keep = []
        if noise is not None:
            no = np.ascontiguousarray(np.asarray(noise_off, dtype=np.int64))
            na = np.ascontiguousarray(np.asarray(noise_alpha, dtype=np.float64))
            keep += [no, na]
            b.noise_dev, b.noise_off, b.noise_alpha = noise.data_ptr(), ptr(no, ctypes.c_int64), ptr(na, ctypes.c_double)
        rows_c = np.ascontiguousarray(rows[:-1])
        b.out_dev, b.out_row = out.data_ptr(), ptr(rows_c, ctypes.c_int64)
        b.out_f64_dev = out64.data_ptr() if out64 is not None else None
        b.ark_decimals = int(ark_decimals)
        b.preprocess = _lib.FDLP_PRE_DIFF if preprocess == "diff" else _lib.FDLP_PRE_NONE
        s = stream if stream is not None else torch.cuda.current_stream(pcm.device)
        # the batch is split to respect the plan's frame capacity
        if total > self.max_frames:
            raise ValueError("batch of %d frames exceeds the plan's max_frames %d" % (total, self.max_frames))
        check(lib.fdlp_mel_compute(self._h, ctypes.byref(b), ctypes.c_void_p(s.cuda_stream)))
        return out, rows, out64
