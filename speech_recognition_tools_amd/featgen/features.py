"""Device-backed mirror of the FDLP-path helpers of
sadhusamik/speech_recognition_tools src/featgen/features.py (same names and argument meaning).

* createFbank / createFbankCochlear (features.py:172-219) -> host C++ in libfdlp_hip.so
* computeLpcFast (:222-230), computeModSpecFromLpc (:233-246) -> gfx950 kernels (batched: 1-D
  inputs behave like the reference, 2-D inputs are processed row by row on the device)
* load_noise (:34-44), add_noise_to_wav (:24-31) -> reference semantics (int16-wrapped energies);
  the mixing itself is done on the device inside fdlp_compute
* dict2Ark (:63-69) -> native Kaldi binary ark/scp writer (no copy-feats)
Nothing here falls back to a CPU implementation of the DSP.
"""
import ctypes
import os
import sys
from functools import lru_cache

import numpy as np

from .._lib import FdlpConfigC, FDLP_FBANK_COCHLEAR, FDLP_FBANK_MEL, check, lib, ptr


class WavSamples(np.ndarray):
    """float64 samples of a non-16-bit WAV with scipy's dtype kept as `scipy_kind` ('uint8', 'int32',
    'int64', 'float32', 'float64'): the reference squares the signal in that dtype when it mixes noise
    (features.py:27), so augment.noise_params needs it."""
    scipy_kind = None

    def __array_finalize__(self, obj):
        self.scipy_kind = getattr(obj, "scipy_kind", None)


_KIND_NAMES = {1: "uint8", 2: "int16", 3: "int32", 4: "int64", 5: "float32", 6: "float64"}


def read_wav_bytes(data: bytes):
    """(sr, samples) of a RIFF/WAVE buffer like scipy.io.wavfile.read (computeFDLPSpectrogram.py:133,:139):
    int16 for 16-bit PCM; the other formats scipy reads (8-bit unsigned, 24/32/64-bit integer, float32/64)
    come back as the float64 values of scipy's array (the reference only ever multiplies them by a float64
    window, features.py:153).  Multi-channel data is [T, channels]."""
    buf = np.frombuffer(data, dtype=np.uint8)
    sr, ch, i16, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    check(lib.fdlp_wav_decode(ptr(buf, ctypes.c_uint8), buf.size, ctypes.byref(sr), ctypes.byref(ch),
                              ctypes.byref(i16), ctypes.byref(n), None))
    if i16.value == 2:  # big-endian (RIFX) 16-bit PCM: scipy returns '>i2' values, i.e. int16 input
        x = np.empty(n.value * ch.value, dtype=np.float64)
        check(lib.fdlp_wav_decode(ptr(buf, ctypes.c_uint8), buf.size, None, None, None, None,
                                  ptr(x, ctypes.c_double)))
        x = x.astype(np.int16)
    elif i16.value:
        sp = ctypes.POINTER(ctypes.c_int16)()
        sr2, ch2, n2 = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        check(lib.fdlp_wav_parse(ptr(buf, ctypes.c_uint8), buf.size, ctypes.byref(sr2), ctypes.byref(ch2),
                                 ctypes.byref(sp), ctypes.byref(n2)))
        off = ctypes.cast(sp, ctypes.c_void_p).value - buf.ctypes.data
        x = np.frombuffer(data, dtype='<i2', count=n.value * ch.value, offset=off).astype(np.int16)
    else:
        x = np.empty(n.value * ch.value, dtype=np.float64)
        check(lib.fdlp_wav_decode(ptr(buf, ctypes.c_uint8), buf.size, None, None, None, None,
                                  ptr(x, ctypes.c_double)))
        kind = ctypes.c_int32()
        check(lib.fdlp_wav_kind(ptr(buf, ctypes.c_uint8), buf.size, ctypes.byref(kind)))
        x = x.view(WavSamples)
        x.scipy_kind = _KIND_NAMES[kind.value]
    if ch.value > 1:
        x = x.reshape(-1, ch.value)
    return sr.value, x


def read_wav(path):
    with open(path, 'rb') as f:
        return read_wav_bytes(f.read())


def load_noise(noise_type):
    """features.py:34-44: noises/<type>.wav relative to the working directory."""
    noise_file = "noises/" + noise_type + ".wav"
    if os.path.isfile(noise_file):
        sr, noise = read_wav(noise_file)
    else:
        print("Noise file " + noise_file + " not found!")
        sys.exit(1)  # the reference calls os.exit, which raises; either way the job fails
    return noise


def add_noise_to_wav_params(sig, noise, snr, u):
    """(offset, alpha) used by add_noise_to_wav for the uniform draw u (features.py:24-29)."""
    from ..augment import noise_params
    return noise_params(sig, noise, snr, u)


def _fbank(kind, nfilters, nfft, srate, **kw):
    c = FdlpConfigC()
    c.nfilters, c.srate, c.fbank_kind = int(nfilters), int(srate), kind
    c.warp_fact = float(kw.get("warp_fact", 1.0))
    c.om_w, c.alp, c.fixed, c.bet = (float(kw.get("om_w", 0.2)), float(kw.get("alp", 2.5)),
                                     int(kw.get("fixed", 1)), float(kw.get("bet", 2.5)))
    ncol = int(np.floor(nfft / 2 + 1))
    out = np.empty((int(nfilters), ncol), dtype=np.float64)
    n = ctypes.c_int32()
    check(lib.fdlp_make_fbank(ctypes.byref(c), int(nfft), ptr(out, ctypes.c_double), ctypes.byref(n)))
    return out


def createFbank(nfilters, nfft, srate, warp_fact=1):
    return _fbank(FDLP_FBANK_MEL, nfilters, nfft, srate, warp_fact=warp_fact)


def createFbankCochlear(nfilters, nfft, srate, om_w=0.2, alp=2.5, fixed=1, bet=2.5, warp_fact=1):
    return _fbank(FDLP_FBANK_COCHLEAR, nfilters, nfft, srate, om_w=om_w, alp=alp, fixed=fixed, bet=bet,
                  warp_fact=warp_fact)


@lru_cache(maxsize=8)
def _lpc_plan(N, order):
    from ..plan import FdlpPlan, FeatureConfig
    # fduration*srate = N with srate 16000; filterbank unused by the dense entry points
    cfg = FeatureConfig(nfilters=1, coeff_num=2, coeff_range="0,1", order=order, fduration=N / 16000.0,
                        frate=100, fbank_type="mel,1", support_eps=0.0)
    return FdlpPlan(cfg, device=0, max_frames=1)


def computeLpcFast(signal, order, keepreal=True):
    """features.py:222-230 on the device: (a[order+1], gg) for a 1-D band signal, or row-wise
    arrays for a 2-D input.  The circular autocorrelation is exact (not FFT-based)."""
    import torch
    if not keepreal:
        raise NotImplementedError("keepreal=False (complex autocorrelation) is not used by the FDLP path")
    x = np.asarray(signal, dtype=np.float64)
    one = x.ndim == 1
    x2 = np.atleast_2d(x)
    plan = _lpc_plan(int(x2.shape[1]), int(order))
    _, a, gg = plan.lpc_rows(torch.from_numpy(np.ascontiguousarray(x2)).cuda())
    a, gg = a.cpu().numpy(), gg.cpu().numpy()
    return (a[0], float(gg[0])) if one else (a, gg)


def computeModSpecFromLpc(gg, xlpc, lim):
    """features.py:233-246 on the device.  Like the reference it negates xlpc[1:] in place."""
    import torch
    a = np.asarray(xlpc, dtype=np.float64)
    one = a.ndim == 1
    a2 = np.atleast_2d(a)
    g = np.atleast_1d(np.asarray(gg, dtype=np.float64))
    plan = _lpc_plan(1024, max(int(a2.shape[1]) - 1, 1))
    cep = plan.cepstrum_rows(torch.from_numpy(np.ascontiguousarray(a2)).cuda(),
                             torch.from_numpy(np.ascontiguousarray(g)).cuda(), int(lim)).cpu().numpy()
    if isinstance(xlpc, np.ndarray) and xlpc.dtype == np.float64:
        xlpc[..., 1:] = -xlpc[..., 1:]
    return cep[0] if one else cep


def dict2Ark(feat_dict, outfile, kaldi_cmd=None):
    """features.py:63-69: <outfile>.ark + <outfile>.scp in Kaldi binary format, written natively
    (the values are already rounded like the reference's '%.3f' text ark when produced by
    getFeats).  Raises on I/O failure (the reference silently ignores copy-feats' status)."""
    h = ctypes.c_void_p()
    check(lib.fdlp_ark_open((outfile + '.ark').encode(), (outfile + '.scp').encode(), ctypes.byref(h)))
    try:
        for key, feat in feat_dict.items():
            m = np.ascontiguousarray(feat, dtype=np.float32)
            if m.ndim != 2:
                raise ValueError("feature matrix must be 2-D")
            check(lib.fdlp_ark_write(h, key.encode(), ptr(m, ctypes.c_float), m.shape[0], m.shape[1]))
    except BaseException:  # nothing is published under the final names (fdlp_ark_abort)
        lib.fdlp_ark_abort(h)
        raise
    check(lib.fdlp_ark_close(h))


def read_ark(path):
    """Minimal Kaldi binary float-matrix ark reader (tests / tooling)."""
    out = {}
    with open(path, 'rb') as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        sp = data.index(b' ', pos)
        key = data[pos:sp].decode()
        pos = sp + 1
        assert data[pos:pos + 2] == b'\0B', "not a binary ark"
        pos += 2
        tok = data[pos:pos + 3]
        assert tok == b'FM ', tok
        pos += 3
        assert data[pos] == 4
        rows = int.from_bytes(data[pos + 1:pos + 5], 'little', signed=True)
        assert data[pos + 5] == 4
        cols = int.from_bytes(data[pos + 6:pos + 10], 'little', signed=True)
        pos += 10
        n = rows * cols
        out[key] = np.frombuffer(data, dtype='<f4', count=n, offset=pos).reshape(rows, cols).copy()
        pos += 4 * n
    return out
