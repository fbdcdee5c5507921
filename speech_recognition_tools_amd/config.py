"""Parsed form of the reference argv (computeFDLPSpectrogram.py:240-262, :43-118) and its C struct.

No torch import here: the native JOB runner (compute-fdlp-feats' default host path) needs only this and
the C ABI, so a cold JOB process does not pay for importing torch.
"""
import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import FdlpConfigC, ptr

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


