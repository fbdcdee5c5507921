"""Host RNG replicas behind the C ABI.

* :class:`PyRandom` reproduces CPython ``random`` (``random.seed(int)`` + ``randrange(2)``),
  the OLA hop jitter source of computeFDLPSpectrogram.py:21,225.
* :class:`NpRandom` reproduces ``numpy.random`` legacy seeding + ``rand()``, the noise-offset
  source of features.py:25.

Unseeded (``seed=None``) both draw their seed material from ``os.urandom`` like the reference's
unseeded generators, so runs are non-deterministic unless a seed is given.
"""
import ctypes
import os

import numpy as np

from ._lib import check, lib, ptr


def _int_key(seed: int):
    """CPython random.seed(int): 32-bit little-endian words of |seed| ([0] for 0)."""
    n = abs(int(seed))
    words = []
    while n:
        words.append(n & 0xFFFFFFFF)
        n >>= 32
    return words or [0]


class PyRandom:
    def __init__(self, seed=None):
        if seed is None:
            key = list(np.frombuffer(os.urandom(624 * 4), dtype=np.uint32))
        else:
            key = _int_key(seed)
        k = np.asarray(key, dtype=np.uint32)
        h = ctypes.c_void_p()
        check(lib.fdlp_pyrandom_create(ptr(k, ctypes.c_uint32), len(k), ctypes.byref(h)))
        self._h = h

    def randbits2(self, n: int) -> np.ndarray:
        """n draws of random.randrange(2) as uint8."""
        out = np.empty(max(int(n), 0), dtype=np.uint8)
        if out.size:
            check(lib.fdlp_pyrandom_randbits2(self._h, out.size, ptr(out, ctypes.c_uint8)))
        return out

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.fdlp_pyrandom_destroy(h)
            self._h = None


class NpRandom:
    def __init__(self, seed=None):
        if seed is None:
            seed = int(np.frombuffer(os.urandom(4), dtype=np.uint32)[0])
        if not 0 <= int(seed) <= 0xFFFFFFFF:
            raise ValueError("Seed must be between 0 and 2**32 - 1")
        h = ctypes.c_void_p()
        check(lib.fdlp_nprandom_create(int(seed), ctypes.byref(h)))
        self._h = h

    def rand(self, n=None):
        m = 1 if n is None else int(n)
        out = np.empty(m, dtype=np.float64)
        check(lib.fdlp_nprandom_rand(self._h, m, ptr(out, ctypes.c_double)))
        return float(out[0]) if n is None else out

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.fdlp_nprandom_destroy(h)
            self._h = None
