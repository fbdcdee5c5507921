"""The OLA stage's device log (fdlp_device.h ola_log: table + polynomial, used for every feature's
np.log(np.clip(., 1e-14)), computeFDLPSpectrogram.py:227) against numpy's log, through fdlp_device_log:
within 1 ulp everywhere, and the same '%.3f' code (round(v * 1000)) as numpy's value for every input."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _device_log(x):
    import torch
    from speech_recognition_tools_amd import _lib
    xd = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()
    yd = torch.empty_like(xd)
    s = torch.cuda.current_stream()
    _lib.check(_lib.lib.fdlp_device_log(xd.data_ptr(), yd.data_ptr(), xd.numel(), s.cuda_stream))
    torch.cuda.synchronize()
    return yd.cpu().numpy()


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
    ulp = np.abs(y - ref) / np.spacing(np.abs(ref))
    ulp[ref == 0] = np.abs(y[ref == 0]) / np.finfo(np.float64).tiny
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
