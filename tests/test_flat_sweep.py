"""Host side of the lag-parallel flat-top sweep (ac_vsweep_kernel, DESIGN.md "Lag-parallel VALU sweeps"):
the plan's event table (fdlp_plan_flat_events) and a numpy emulation of the kernel's event handling --
segment accumulator folded into C chains at each event, restart at m2_j, emission at m1_j, position parts
with partial chains -- against the direct flat-top sums.  CPU only (host plan, device=-1)."""
import numpy as np
import pytest

from speech_recognition_tools_amd.plan import FdlpPlan, FeatureConfig

CFGS = [FeatureConfig.wsj(),
        FeatureConfig(fbank_type="cochlear,2,0.5,1,4,1.2", nfilters=20, fduration=0.5, order=30, coeff_num=40,
                      coeff_range="0,40")]


@pytest.mark.parametrize("cfg", CFGS, ids=["wsj", "wide"])
def test_flat_event_table(cfg):
    p = FdlpPlan(cfg, device=-1, max_frames=4)
    m1, m2 = p.regions()
    C, H, ev = p.flat_events()
    assert C >= 1 and H >= 1 and ev.shape == (2 * p.B, 4)
    S = ev[:, 0]
    assert np.all(np.diff(S) <= 0), "events in sweep order (S descending)"
    owner = [-1] * C
    for s_, band, typ, ch in ev:
        assert ch == band % C
        if typ == 0:
            assert s_ == m2[band] and owner[ch] == -1
            owner[ch] = band
        else:
            assert s_ == m1[band] and owner[ch] == band
            owner[ch] = -1
    # C is the smallest chain count: bands j and j - C never overlap, j and j - (C - 1) do somewhere
    if C > 1:
        assert any(m2[j - (C - 1)] > m1[j] for j in range(C - 1, p.B))


def _emulate(D, m1, m2, C, H, ev, nl):
    """The kernel's flat sweep in numpy: returns flat[j, l] = emission + partials."""
    N = D.size
    Dz = np.concatenate([D, np.zeros(nl)])
    B = len(m1)
    lo, hi = int(m1.min()), int(m2.max())
    P = [hi - (hi - lo) * h // H for h in range(H + 1)]
    flat = np.zeros((B, nl))
    for h in range(H):
        sel = [k for k in range(len(ev)) if P[h + 1] <= ev[k, 0] < P[h] or (h == 0 and ev[k, 0] == P[0])]
        chains = np.zeros((C, nl))
        acc = np.zeros(nl)
        k = 0
        for pos in range(P[h] - 1, P[h + 1] - 1, -1):
            while k < len(sel) and ev[sel[k], 0] > pos:       # events at S = pos + 1 and above
                S = ev[sel[k], 0]
                chains += acc
                acc[:] = 0
                while k < len(sel) and ev[sel[k], 0] == S:
                    _, band, typ, ch = ev[sel[k]]
                    if typ == 0:
                        chains[ch] = 0
                    else:
                        flat[band] += chains[ch]
                    k += 1
            acc += D[pos] * Dz[pos:pos + nl]
        chains += acc
        acc[:] = 0
        while k < len(sel):
            S = ev[sel[k], 0]
            while k < len(sel) and ev[sel[k], 0] == S:
                _, band, typ, ch = ev[sel[k]]
                if typ == 0:
                    chains[ch] = 0
                else:
                    flat[band] += chains[ch]
                k += 1
        if h < H - 1:  # partial chains of the bands continuing below this part
            for j in range(B):
                if m1[j] < P[h + 1] < m2[j]:
                    flat[j] += chains[j % C]
    return flat


@pytest.mark.parametrize("cfg", CFGS, ids=["wsj", "wide"])
def test_flat_chain_emulation_matches_direct_sums(cfg):
    p = FdlpPlan(cfg, device=-1, max_frames=4)
    m1, m2 = p.regions()
    C, H, ev = p.flat_events()
    nl, N = p.nlags, p.N
    D = np.random.default_rng(3).standard_normal(N)
    Dz = np.concatenate([D, np.zeros(nl)])
    got = _emulate(D, m1, m2, C, H, ev, nl)
    for j in range(p.B):
        want = np.array([np.dot(D[m1[j]:m2[j]], Dz[m1[j] + l:m2[j] + l]) for l in range(nl)])
        np.testing.assert_allclose(got[j], want, rtol=1e-9, atol=1e-9 * np.abs(want).max())
