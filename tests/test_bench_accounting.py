"""CPU tests of bench.py's algorithmic-FLOP accounting for the roofline (no GPU): the structured
autocorrelation counts the wrap straddle once per frame for the bands whose first / last p+1 taps are
skirt taps (ac_wrap_kernel) and per band for the others, and the band eligibility it assumes matches the
plan's skirt regions."""
import numpy as np

import bench
from speech_recognition_tools_amd import FdlpPlan, FeatureConfig


def _plan(**kw):
    return FdlpPlan(FeatureConfig(**kw) if kw else FeatureConfig.wsj(), device=-1)


def _tri(nl, n):
    lags = np.arange(nl)
    return float(np.minimum(lags, min(n, nl - 1)).sum())


def test_structured_flops_count_the_shared_wrap_once():
    p = _plan()
    assert p.autocorr_path == "structured"
    _, lo, hi = p.fbank()
    support = (hi - lo).astype(np.int64)
    nl, N = p.nlags, p.N
    m1, m2 = p.regions()
    shared = (m1 >= nl - 1) & (m2 <= N - (nl - 1))
    assert 60 <= int(shared.sum()) < p.B          # the recipes' bank: most bands, not the edge ones
    got = bench.autocorr_flops(p, support)
    # the same count with every band's wrap straddle per band (the round-2 accounting)
    per_band = got / 2.0 - _tri(nl, nl - 1) + sum(_tri(nl, int(N - m2[j])) for j in range(p.B) if shared[j])
    assert per_band * 2.0 > got
    assert abs(got / 1e6 - 24.92) < 0.05          # MFLOP per frame, DESIGN.md
    assert abs(per_band * 2.0 / 1e6 - 26.6) < 0.1


def test_no_shared_wrap_without_skirt_edges():
    # few wide bands: the first band's flat top starts at bin 0 and the last one's ends at N
    p = _plan(fbank_type="cochlear,1,1,1,2.5,1", nfilters=7, fduration=1.5, order=238, coeff_num=100)
    m1, m2 = p.regions()
    nl, N = p.nlags, p.N
    shared = (m1 >= nl - 1) & (m2 <= N - (nl - 1))
    assert not shared[0] and not shared[-1]
