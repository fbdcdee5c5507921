"""The path's device transcendental functions against numpy, through fdlp_device_fn:
* the OLA stage's log (fdlp_device.h ola_log: table + polynomial, used for every feature's
  np.log(np.clip(., 1e-14)), computeFDLPSpectrogram.py:227): within 1 ulp everywhere, and the same '%.3f'
  code (round(v * 1000)) as numpy's value for every input;
* the envelope's exp (np.exp of the log-magnitude, :204-205; the device library's exp -- a table form
  measured no faster, profiles/r05r_env_exp_ab.txt): within 1 ulp over the range the envelopes take and
  beyond, saturating to 0 / inf like np.exp, NaN kept."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _device_fn(fn, x):
    import torch
    from speech_recognition_tools_amd import _lib
    xd = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()
    yd = torch.empty_like(xd)
    s = torch.cuda.current_stream()
    _lib.check(_lib.lib.fdlp_device_fn(fn, xd.data_ptr(), yd.data_ptr(), xd.numel(), s.cuda_stream))
    torch.cuda.synchronize()
    return yd.cpu().numpy()


def _device_log(x):
    from speech_recognition_tools_amd import _lib
    return _device_fn(_lib.FDLP_FN_LOG, x)


def _device_exp(x):
    from speech_recognition_tools_amd import _lib
    return _device_fn(_lib.FDLP_FN_EXP, x)


def _ulps(y, ref):
    ulp = np.abs(y - ref) / np.spacing(np.abs(ref))
    zero = ref == 0
    ulp[zero] = np.abs(y[zero]) / np.finfo(np.float64).tiny
    return ulp


def _inputs():
    rng = np.random.default_rng(7)
    parts = [
        10.0 ** rng.uniform(-14, 12, 2_000_000),                  # the OLA sums' range (clip at 1e-14)
        1.0 + rng.uniform(-2e-3, 2e-3, 200_000),                    # around 1 (log near 0)
        1.0 + np.arange(-2000, 2001) * np.finfo(np.float64).eps,    # ulps next to 1
        np.ldexp(1.0, np.arange(-46, 40)).astype(np.float64),       # powers of two
        np.array([np.ldexp(i / 128.0, e) for i in range(128, 257) for e in (-20, -1, 0, 1, 7)]),  # table nodes
        np.nextafter(np.array([np.ldexp((i + 0.5) / 128.0, e) for i in range(128, 256) for e in (-3, 0, 5)]),
                     np.inf),                                       # the rounding edges of the table index
        np.array([1e-14, np.e, 10.0, 0.5, 2.0, 1.5, np.sqrt(2.0), 1e12]),
    ]
    return np.concatenate(parts)


def test_device_log_within_one_ulp_of_numpy():
    x = _inputs()
    y = _device_log(x)
    ref = np.log(x)
    ulp = _ulps(y, ref)
    assert np.isfinite(y).all()
    assert ulp.max() <= 1.0, (ulp.max(), x[np.argmax(ulp)])
    assert np.mean(y == ref) > 0.99, np.mean(y == ref)  # correctly rounded almost everywhere


def test_device_log_gives_numpys_ark_codes():
    x = _inputs()
    y = _device_log(x)
    ref = np.log(x)
    np.testing.assert_array_equal(np.rint(y * 1000.0), np.rint(ref * 1000.0))
    np.testing.assert_array_equal((np.rint(y * 1000.0) / 1000.0).astype(np.float32),
                                  (np.rint(ref * 1000.0) / 1000.0).astype(np.float32))


def test_device_log_special_values():
    y = _device_log(np.array([np.nan, np.inf, 1.0]))
    assert np.isnan(y[0]) and y[1] == np.inf and y[2] == 0.0


def test_device_exp_within_one_ulp_of_numpy():
    rng = np.random.default_rng(8)
    ln2_64 = np.log(2.0) / 64
    x = np.concatenate([
        rng.uniform(-80.0, 80.0, 2_000_000),                        # envelope log-magnitudes and beyond
        rng.uniform(-700.0, 700.0, 200_000),
        rng.uniform(-1e-3, 1e-3, 100_000),
        np.arange(-6400, 6401) * ln2_64,                            # the reduction's nodes k ln2 / 64
        (np.arange(-6400, 6400) + 0.5) * ln2_64,                    # and the rounding edges between them
        np.array([0.0, -0.0, 1.0, -1.0, 709.0, -708.0]),
    ])
    y = _device_exp(x)
    ref = np.exp(x)
    ulp = _ulps(y, ref)
    assert np.isfinite(y).all()
    assert ulp.max() <= 1.0, (ulp.max(), x[np.argmax(ulp)])
    assert np.mean(y == ref) > 0.9, np.mean(y == ref)


def test_device_exp_special_values():
    y = _device_exp(np.array([np.nan, 800.0, -800.0, np.inf, -np.inf, 0.0]))
    assert np.isnan(y[0]) and y[1] == np.inf and y[2] == 0.0 and y[3] == np.inf and y[4] == 0.0 and y[5] == 1.0
