"""CPU ORACLE for the mel-spectrum sibling feature -- TEST INFRASTRUCTURE ONLY (the checker, never the
product; only tests/ may import it).  fp64 numpy restatement of the reference's
src/featgen/computeMelSpectrum.py compute_mel_spectrum (:40-170):

* frames: features.py getFrames (:118-154) with np.hamming(int(srate*fduration)), hop int(srate/frate)
* spectrum: np.abs(scipy.fftpack.fft(frames, nfft, axis=1)[:, :int(nfft/2+1)])          (:151-155)
* projection: np.matmul(spectrum, fbank.T); log10 ('log') or squared ('power')           (:150-158)
* preprocessing (:133-145): diff convolution, add_noise_to_wav, addReverb (same helpers as the FDLP oracle)

Pinned by tests/golden/mel_*.npz, produced by tests/golden/make_golden.py from the real reference.
"""
import numpy as np
import scipy.fftpack as _fp

from .fdlp_oracle import fbank_cochlear, fbank_mel, reflect_index


def mel_fbank(nfilters, nfft, srate, fbank_type):
    parts = fbank_type.strip().split(',')
    if parts[0] == "mel":
        return fbank_mel(nfilters, nfft, srate, warp_fact=float(parts[1]))
    if parts[0] == "cochlear":
        return fbank_cochlear(nfilters, nfft, srate, om_w=float(parts[1]), alp=float(parts[2]),
                              fixed=int(parts[3]), bet=float(parts[4]), warp_fact=float(parts[5]))
    raise ValueError('Invalid type of filter bank, use mel or cochlear with proper configuration')


def get_frames(signal, srate, frate, flength, window=np.hamming):
    """features.py getFrames (:118-154) as an index map."""
    L = int(srate * flength)
    hop = int(srate / frate)
    if L % 2 == 0:
        sp_b, sp_f, ext = L // 2 - 1, L // 2, L // 2 - 1
    else:
        sp_b = sp_f = ext = (L - 1) // 2
    T = signal.shape[0]
    lim = T + 2 * ext - sp_b - sp_f
    F = 0 if lim <= 0 else (lim - 1) // hop + 1
    idx = np.arange(F)[:, None] * hop + np.arange(L)[None, :] - ext
    return signal[reflect_index(idx, T)].astype(np.float64) * window(L)


def mel_spectrum(signal, nfilters=23, fduration=0.02, frate=100, nfft=1024, fbank_type="mel,1",
                 spectrum_type="log", srate=16000):
    fb = mel_fbank(nfilters, nfft, srate, fbank_type)
    fr = get_frames(signal, srate, frate, fduration)
    mag = np.abs(_fp.fft(fr, nfft, axis=1)[:, :int(nfft / 2 + 1)])
    e = np.matmul(mag, np.transpose(fb))
    if spectrum_type == "log":
        return np.log10(e)
    if spectrum_type == "power":
        return np.power(e, 2)
    raise ValueError("Spectrum type not supported! ")
