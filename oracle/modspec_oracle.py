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
Complex branch (--complex_modulation, :45-47, :74-88, :153-180), modspec_complex_features:
* fbank of nfft = int(fduration srate); cos_trans = scipy.fftpack.ifft(frames)[:, :int(fduration srate / 2)]
* per band: computeLpcFast(filt * cos_trans[i], order, keepreal=False) -- complex circular autocorrelation,
  solve_toeplitz on the Hermitian Toeplitz system, complex gain (features.py:222-230) -- and the complex
  cepstrum computeModSpecFromLpc (features.py:233-246, c_0 = log(sqrt(gg)) on the principal branches)
* [* linspace(0, coeff_num / fduration, coeff_n)], then abs, or real and imaginary parts appended
  (feat_len 2 coeff_num); keep_even as above (with real+imag it is the reference's broadcast error)
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


def complex_cepstrum(a, gg, lim):
    """computeModSpecFromLpc (features.py:233-246) for one complex LPC vector, in the reference's order."""
    x = np.array(a, dtype=np.complex128)
    x[1:] = -x[1:]
    cep = np.zeros(lim, dtype=np.complex128)
    cep[0] = np.log(np.sqrt(gg))
    cep[1] = x[1]
    if x.shape[0] < lim:
        x = np.append(x, np.zeros(int(lim - x.shape[0] + 1)))
    for n in range(2, lim):
        aa = np.arange(1, n) / n
        bb = np.flipud(x[1:n])
        cc = cep[1:n]
        cep[n] = np.sum(aa * bb * cc) + x[n]
    return cep


def modspec_complex_features(signal, nfilters=15, coeff_0=5, coeff_n=30, order=50, fduration=0.5, frate=100,
                             fbank_type="mel,1", keep_even=False, no_window=False, compensate_noise=False,
                             absolute_value=False, srate=16000):
    import scipy.linalg as _sla
    N = int(srate * fduration)
    L = int(fduration * srate / 2)
    fb = mel_fbank(nfilters, N, srate, fbank_type)
    window = (lambda n: np.ones(n)) if no_window else np.hanning
    fr = get_frames(signal, srate, frate, fduration, window)
    X = _fp.ifft(fr)[:, :L]
    F, B = X.shape[0], nfilters
    coeff_num = coeff_n - coeff_0 + 1
    faxis = np.linspace(0, coeff_num / fduration, coeff_n) if compensate_noise else None
    rows = []
    for i in range(F):
        feats = []
        for j in range(B):
            s = fb[j, 0:-1] * X[i, :]
            S = np.fft.fft(s, len(s))
            y = np.fft.ifft(S * np.conj(S))
            a = np.append(1, _sla.solve_toeplitz(y[0:order], -y[1:order + 1]))
            gg = y[0] + np.sum(a * y[1:order + 2])
            mod = complex_cepstrum(a, gg, coeff_n)
            if faxis is not None:
                mod = mod * faxis
            if absolute_value:
                t = np.abs(mod[coeff_0 - 1:coeff_n])
            else:
                t = np.append(np.real(mod[coeff_0 - 1:coeff_n]), np.imag(mod[coeff_0 - 1:coeff_n]))
            if keep_even:
                t = t[1::2] if coeff_0 % 2 == 0 else t[0::2]
            feats.append(t)
        rows.append(np.concatenate(feats))
    return np.array(rows).reshape(F, -1)
