"""CPU ORACLE for the FDLP modulation-spectrum sibling feature -- TEST INFRASTRUCTURE ONLY (the checker,
never the product; only tests/ may import it).  fp64 numpy restatement of the reference's
src/featgen/computeModulationSpectrum.py getFeats (:30-205), DCT branch (complex_modulation off):

* frames: features.py getFrames (:118-154) with np.hanning (getFeats default, :30) or ones (--no_window,
  :90-92), hop int(srate/frate), length int(srate*fduration)
* cos_trans = scipy.fftpack.dct(frames) / sqrt(2 N)                                          (:157)
* per band: filt = fbank[j, :-1] (createFbank/Cochlear with nfft = int(2 fduration srate), :46-61),
  computeLpcFast(filt * cos_trans[i], order) and np.real(computeModSpecFromLpc(gg, a, coeff_n)) (:168-183)
* [* linspace(0, coeff_num/(2 fduration), coeff_n)] (--compensate_noise :82-88), [abs] (:186-187),
  [coeff_0-1 : coeff_n], keep_even -> [1::2] if coeff_0 even else [0::2]                       (:184-197)
Pinned by tests/golden/modspec_*.npz (tests/golden/make_golden.py, real reference).
"""
import numpy as np
import scipy.fftpack as _fp

from .fdlp_oracle import autocorr_fft, cepstrum_batch, lpc_from_autocorr
from .mel_oracle import get_frames, mel_fbank


def modspec_features(signal, nfilters=15, coeff_0=5, coeff_n=30, order=50, fduration=0.5, frate=100,
                     fbank_type="mel,1", keep_even=False, no_window=False, compensate_noise=False,
                     absolute_value=False, srate=16000):
    N = int(srate * fduration)
    fb = mel_fbank(nfilters, int(2 * fduration * srate), srate, fbank_type)
    window = (lambda n: np.ones(n)) if no_window else np.hanning
    fr = get_frames(signal, srate, frate, fduration, window)
    D = _fp.dct(fr) / np.sqrt(2 * N)
    F, B = D.shape[0], nfilters
    bands = fb[None, :, :-1] * D[:, None, :]
    r = autocorr_fft(bands.reshape(F * B, -1), order + 2)
    a = np.empty((F * B, order + 1))
    gg = np.empty(F * B)
    for t in range(F * B):
        a[t], gg[t] = lpc_from_autocorr(r[t], order)
    mod = np.real(cepstrum_batch(a, gg, coeff_n))
    coeff_num = coeff_n - coeff_0 + 1
    if compensate_noise:
        mod = mod * np.linspace(0, coeff_num / (2 * fduration), coeff_n)
    if absolute_value:
        mod = np.abs(mod)
    sel = mod[:, coeff_0 - 1:coeff_n]
    if keep_even:
        sel = sel[:, 1::2] if coeff_0 % 2 == 0 else sel[:, 0::2]
    return sel.reshape(F, B * sel.shape[1])
