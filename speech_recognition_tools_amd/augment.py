"""Host-side parameters of the reference's augmentations (the mixing itself runs on the device).

add_noise_to_wav (features.py:24-31): offset = floor(rand()*(len(noise)-len(sig))),
alpha = sqrt(E_s / (E_n * 10**(snr/10))) with E = mean(x**2) over int16-wrapped squares.
"""
import ctypes

import numpy as np

from ._lib import check, lib, ptr

DIFF_KERNEL = (1, 2, 3, 2, 0, -2, -5, -2, 0, 2, 3, 2, 1)  # computeFDLPSpectrogram.py:163


def noise_params(sig: np.ndarray, noise: np.ndarray, snr: float, u: float):
    s = np.ascontiguousarray(sig, dtype=np.int16)
    n = np.ascontiguousarray(noise, dtype=np.int16)
    off = ctypes.c_int64()
    alpha = ctypes.c_double()
    check(lib.fdlp_noise_params(ptr(s, ctypes.c_int16), s.size, ptr(n, ctypes.c_int16), n.size, float(snr),
                                float(u), ctypes.byref(off), ctypes.byref(alpha)))
    return off.value, alpha.value
