"""Host-side parameters of the reference's augmentations (the mixing itself runs on the device).

add_noise_to_wav (features.py:24-31): offset = floor(rand()*(len(noise)-len(sig))),
alpha = sqrt(E_s / (E_n * 10**(snr/10))) with E = mean(x**2) over the squares in the signal's own dtype
(int16 / int32 / uint8 squares wrap, float32 squares round and sum in float32; fdlp_noise_params_any).
"""
import ctypes

import numpy as np

from ._lib import check, lib, ptr

DIFF_KERNEL = (1, 2, 3, 2, 0, -2, -5, -2, 0, 2, 3, 2, 1)  # computeFDLPSpectrogram.py:163


# scipy.io.wavfile dtypes -> include/fdlp.h FDLP_SIG_*
SIG_KINDS = {"uint8": 1, "int16": 2, "int32": 3, "int64": 4, "float32": 5, "float64": 6}


def noise_params(sig: np.ndarray, noise: np.ndarray, snr: float, u: float, kind: str = None):
    """(offset, alpha) of add_noise_to_wav for the uniform draw u.  `kind` is scipy's dtype of the signal
    (default: sig's own dtype; a float64 array read from a non-16-bit WAV carries it as `scipy_kind`,
    featgen/features.read_wav_bytes)."""
    kind = kind or getattr(sig, "scipy_kind", None) or str(np.asarray(sig).dtype)
    if noise.dtype != np.int16:
        raise NotImplementedError("noise files other than 16-bit PCM (the recipes' noises/*.wav are 16-bit)")
    n = np.ascontiguousarray(noise, dtype=np.int16)
    if kind != "int16":
        if kind not in SIG_KINDS:
            raise ValueError("unsupported signal dtype %s" % kind)
        s = np.ascontiguousarray(np.asarray(sig), dtype=np.float64)
        off = ctypes.c_int64()
        alpha = ctypes.c_double()
        check(lib.fdlp_noise_params_any(ptr(s, ctypes.c_double), s.size, SIG_KINDS[kind], ptr(n, ctypes.c_int16),
                                        n.size, float(snr), float(u), ctypes.byref(off), ctypes.byref(alpha)))
        return off.value, alpha.value
    s = np.ascontiguousarray(sig, dtype=np.int16)
    off = ctypes.c_int64()
    alpha = ctypes.c_double()
    check(lib.fdlp_noise_params(ptr(s, ctypes.c_int16), s.size, ptr(n, ctypes.c_int16), n.size, float(snr),
                                float(u), ctypes.byref(off), ctypes.byref(alpha)))
    return off.value, alpha.value


ROOMS = {  # computeFDLPSpectrogram.py:75-87 (the reference's relative ./RIR paths)
    "small_room": "./RIR/RIR_SmallRoom1_near_AnglA.wav",
    "medium_room": "./RIR/RIR_MediumRoom1_far_AnglA.wav",
    "large_room": "./RIR/RIR_LargeRoom1_far_AnglA.wav",
}


def load_rir(room: str) -> np.ndarray:
    """RIR of --add_reverb <room> as the reference loads it: channel 1 of the stereo WAV / 2**15
    (computeFDLPSpectrogram.py:76-87).  Raises like the reference for an unknown room."""
    if room not in ROOMS:
        raise ValueError('Invalid type of reverberation!')
    from .featgen.features import read_wav
    sr, rir = read_wav(ROOMS[room])
    if rir.ndim != 2 or rir.shape[1] < 2:
        raise IndexError("RIR file %s must have at least two channels (the reference uses channel 1)" % ROOMS[room])
    return rir[:, 1] / np.power(2, 15)


def reverb(pcm, lengths, rir, offsets=None, noise=None, noise_off=None, noise_alpha=None, preprocess=None,
           stream=None):
    """addReverb (features.py:110-115) of a batch on the device, after the optional diff / noise
    preprocessing (computeFDLPSpectrogram.py:160-170).  pcm: int16 (or float64) device tensor of the
    concatenated utterances; rir: float64 device tensor.  Returns (float64 device tensor indexed like
    pcm, new lengths): feed it to FdlpPlan.compute without noise / preprocess."""
    import torch
    from ._lib import FdlpReverbBatchC, FDLP_PCM_F64, FDLP_PCM_I16, FDLP_PRE_DIFF, FDLP_PRE_NONE
    if not pcm.is_cuda or not rir.is_cuda or rir.dtype != torch.float64:
        raise TypeError("pcm and rir must be device tensors (rir float64)")
    kind = FDLP_PCM_I16 if pcm.dtype == torch.int16 else FDLP_PCM_F64
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
    out = torch.empty(pcm.numel(), dtype=torch.float64, device=pcm.device)
    out_len = np.zeros(n, dtype=np.int64)
    b = FdlpReverbBatchC()
    b.n_utt, b.pcm_kind, b.pcm_dev = n, kind, pcm.data_ptr()
    b.pcm_off, b.utt_len = ptr(offs, ctypes.c_int64), ptr(lens, ctypes.c_int64)
    b.preprocess = FDLP_PRE_DIFF if preprocess == "diff" else FDLP_PRE_NONE
    keep = []
    if noise is not None:
        no = np.ascontiguousarray(np.asarray(noise_off, dtype=np.int64))
        na = np.ascontiguousarray(np.asarray(noise_alpha, dtype=np.float64))
        keep += [no, na]
        b.noise_dev, b.noise_off, b.noise_alpha = noise.data_ptr(), ptr(no, ctypes.c_int64), ptr(na, ctypes.c_double)
    b.rir_dev, b.rir_len = rir.data_ptr(), int(rir.numel())
    b.out_dev, b.out_len = out.data_ptr(), ptr(out_len, ctypes.c_int64)
    s = stream if stream is not None else torch.cuda.current_stream(pcm.device)
    check(lib.fdlp_reverb(ctypes.byref(b), ctypes.c_void_p(s.cuda_stream)))
    return out, out_len
