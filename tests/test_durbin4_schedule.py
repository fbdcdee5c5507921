"""Host-side emulation of durbin4_kernel's data movement (csrc/fdlp_lpc.hip): 4 lanes
per item, phases S = 1, 5, 9, ... then SL4 = 38 with capacity 4 S and orders k <= 4 S - 2, B updated in place
from its row_shr:1 neighbour (the next item's first lane gets the exact 0 of position 4 S - 1, not a select),
R1 and A re-laid out through the item's LDS image with B read back mirrored, the 8 positions a phase adds
loaded one phase ahead.  The emulation keeps the kernel's per-lane slot arrays and checks a and gg against
the oracle's Levinson (features.py:226-228, scipy solve_toeplitz) -- the kernel's index logic, on the CPU."""
import numpy as np
import pytest

from oracle import fdlp_oracle as O

SL4 = 38
STEP = 4  # kC4Step
NQ = 4  # quads emulated side by side, so the row_shr:1 crosses item boundaries as on the device


def _c4_emulate(r_items, p):
    nq = len(r_items)
    nl = nq * 4
    r = np.zeros((nq, 160))
    for q, rr in enumerate(r_items):
        r[q, :rr.size] = rr
    li = np.arange(nl) % 4
    qi = np.arange(nl) // 4
    r0 = r[:, 0]
    S = 1
    A = np.where(li == 0, 1.0, 0.0)[:, None]
    B = A.copy()
    R1 = np.array([r[qi[x], li[x] + 1] if li[x] <= p else 0.0 for x in range(nl)])[:, None]
    part = np.where(li == 0, R1[:, 0], 0.0)
    E = r0.copy()
    k = 1
    checks = 0
    while True:
        k1 = min(p, 4 * S - 2)
        SN = min(S + STEP, SL4)
        NA = SN - S
        while k <= k1:
            acc = part.reshape(nq, 4).sum(1)
            kappa = -acc / E
            kap = kappa[qi]
            # row_shr:1 of B's last slot inside 16-lane rows; lane 0 of a row takes 0 (bound_ctrl)
            z0 = np.roll(B[:, S - 1], 1)
            z0[np.arange(nl) % 16 == 0] = 0.0
            # the quad boundaries receive the previous item's position 4 S - 1, which must be exactly 0
            assert np.all(z0[li == 0] == 0.0)
            checks += 1
            zb = np.concatenate([z0[:, None], B[:, :S - 1]], axis=1)
            Bn = kap[:, None] * A + zb
            A = A + kap[:, None] * zb
            B = Bn
            part = (B * R1).sum(1)
            E = E * (1.0 - kappa * kappa)
            k += 1
        if k1 == p or SN == S:
            break
        # relayout through the image: R1 (+ 8 new positions), then A; B mirrored from A's image
        img = np.zeros((nq, 160))
        for x in range(nl):
            img[qi[x], li[x] * S: li[x] * S + S] = R1[x]
            for t in range(NA):
                m = 4 * S + li[x] + 4 * t
                img[qi[x], m] = r[qi[x], m + 1] if m <= p else 0.0
        R1 = np.array([img[qi[x], li[x] * SN: li[x] * SN + SN] for x in range(nl)])
        img = np.zeros((nq, 160))
        for x in range(nl):
            img[qi[x], li[x] * S: li[x] * S + S] = A[x]
        An = np.zeros((nl, SN))
        Bm = np.zeros((nl, SN))
        for x in range(nl):
            for j in range(SN):
                m = li[x] * SN + j
                An[x, j] = img[qi[x], m] if m <= k1 else 0.0
                mb = k1 - li[x] * SN - j
                Bm[x, j] = img[qi[x], mb] if mb >= 0 else 0.0
        A, B, S = An, Bm, SN
    a = np.zeros((nq, 4 * S))
    for x in range(nl):
        a[qi[x], li[x] * S: li[x] * S + S] = A[x]
    gg = r0 + (A * R1).sum(1).reshape(nq, 4).sum(1)
    return a[:, :p + 1], gg, checks


@pytest.mark.parametrize("p", [150, 149, 147, 146, 139, 128])
def test_durbin4_schedule_matches_levinson(p):
    rng = np.random.default_rng(p)
    items = []
    for q in range(NQ):
        x = rng.standard_normal(2048) * np.exp(-np.arange(2048) / (200.0 + 300 * q))
        items.append(O.autocorr_fft(x, p + 2))
    a, gg, checks = _c4_emulate(items, p)
    assert checks == p
    for q in range(NQ):
        a_ref, g_ref = O.lpc_from_autocorr(items[q], p)
        np.testing.assert_allclose(a[q], a_ref, rtol=1e-6, atol=1e-9 * np.abs(a_ref).max())
        np.testing.assert_allclose(gg[q], g_ref, rtol=1e-8)
