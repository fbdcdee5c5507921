"""Host-side emulation of durbin4_kernel's data movement (csrc/fdlp_lpc.hip): one wave of
16 items x 4 lanes, phases S = 1, 5, 9, ... then SL4 = 38 with capacity 4 S and orders k <= 4 S - 2, B updated
in place from its row_shr:1 neighbour (the next item's first lane gets the exact 0 of position 4 S - 1, not a
select), R1 and A re-laid out through ONE persistent LDS array -- the guard plus 16 item images of kItem
doubles, zeroed once as the kernel does -- and read back without selects: A from [0, 4 SN), B mirrored from
A's image down to index -(4 NA + 1), i.e. into the guard (item 0) or the previous item's image tail.  The
emulation therefore checks the zero-margin invariant the kernel relies on (a stale value anywhere it reads
would corrupt a / gg), then the full-row or per-item copy of the rows (zero past p), against the oracle's
Levinson (features.py:226-228, scipy solve_toeplitz) -- the kernel's index logic, on the CPU."""
import numpy as np
import pytest

from oracle import fdlp_oracle as O

SL4 = 38
STEP = 4    # kC4Step
GUARD = 24  # kC4Guard
ITEMS = 16  # items per wave


def item_stride(sl4):  # c4_item_stride: 4 SL4 rounded up to 28 mod 32 doubles
    need = 4 * sl4
    return need + ((28 - need % 32) + 32) % 32


KITEM = item_stride(SL4)


def _c4_emulate(r_items, p, astride=160, guard_fill=0.0):
    """r_items: up to 16 autocorrelation rows (the rest of the wave's items are invalid: r0 = 1, R1 = 0).
    guard_fill: what the guard holds at the start (0 in the kernel; anything else models a broken margin)."""
    n_valid = len(r_items)
    lane = np.arange(64)
    li, ii = lane & 3, lane >> 2
    valid = ii < n_valid
    r = np.zeros((ITEMS, 200))
    for q, rr in enumerate(r_items):
        r[q, :rr.size] = rr
    lds = np.zeros(GUARD + ITEMS * KITEM)   # zeroed once per wave, never again
    lds[:GUARD] = guard_fill
    img0 = GUARD + ii * KITEM               # each lane's item image base
    r0 = np.where(valid, r[ii, 0], 1.0)
    S = 1
    A = np.where(li == 0, 1.0, 0.0)[:, None]
    B = A.copy()
    R1 = np.where(valid & (li <= p), r[ii, li + 1], 0.0)[:, None]
    part = np.where(li == 0, R1[:, 0], 0.0)
    E = r0.copy()
    plim = np.where(valid, p - li, -1)
    k = 1
    checks = 0
    while True:
        k1 = min(p, 4 * S - 2)
        SN = min(S + STEP, SL4)
        NA = SN - S if SN > S else 1
        rn = np.zeros((64, NA))
        if SN > S and k1 < p:  # the next phase's R1 positions, loaded one phase ahead
            for t in range(NA):
                ok = 4 * S + 4 * t <= plim
                rn[:, t] = np.where(ok, r[ii, np.minimum(li + 1 + 4 * S + 4 * t, 199)], 0.0)
        while k <= k1:
            acc = np.repeat(part.reshape(16, 4).sum(1), 4)
            kappa = -acc / E
            z0 = np.roll(B[:, S - 1], 1)
            z0[lane % 16 == 0] = 0.0           # row_shr:1, bound_ctrl
            assert np.all(z0[li == 0] == 0.0)  # quad edges inside a row: the previous item's exact 0
            checks += 1
            zb = np.concatenate([z0[:, None], B[:, :S - 1]], axis=1)
            Bn = kappa[:, None] * A + zb
            A = A + kappa[:, None] * zb
            B = Bn
            part = (B * R1).sum(1)
            E = E * (1.0 - kappa * kappa)
            k += 1
        if SN > S and k1 < p:
            # R1 first (positions li S + j, then the new 4 S + li + 4 t), read back at li SN + j
            for j in range(S):
                lds[img0 + li * S + j] = R1[:, j]
            for t in range(NA):
                lds[img0 + 4 * S + li + 4 * t] = rn[:, t]
            R1 = np.stack([lds[img0 + li * SN + j] for j in range(SN)], axis=1)
            # A, the staged R1 positions back to 0, then A and B (mirrored) read with no select
            for j in range(S):
                lds[img0 + li * S + j] = A[:, j]
            for t in range(NA):
                lds[img0 + 4 * S + li + 4 * t] = 0.0
            k1c = 4 * S - 2
            assert k1 == k1c
            An = np.stack([lds[img0 + li * SN + j] for j in range(SN)], axis=1)
            idx = np.stack([k1c - li * SN - j for j in range(SN)], axis=1)
            assert idx.min() >= -GUARD and idx.max() < KITEM
            Bm = lds[img0[:, None] + idx]
            A, B, S = An, Bm, SN
            continue
        break
    q = (A * R1).sum(1)
    gg = r0[::4] + q.reshape(16, 4).sum(1)
    for j in range(S):
        lds[img0 + li * S + j] = A[:, j]
    cap = 4 * S
    assert cap <= astride and cap <= KITEM and p <= cap - 2
    a_out = np.full((ITEMS, astride), np.nan)
    for i in range(n_valid):  # full-row copy (cap == 4 SL4) or per-item copy below cap; zeros past it
        base = GUARD + i * KITEM
        a_out[i, :cap] = lds[base:base + cap]
        a_out[i, cap:] = 0.0
    return a_out[:n_valid], gg[:n_valid], checks, cap


@pytest.mark.parametrize("p", [150, 149, 147, 146, 139, 130, 128])
@pytest.mark.parametrize("n_items", [16, 11])
def test_durbin4_schedule_matches_levinson(p, n_items):
    rng = np.random.default_rng(p + n_items)
    items = []
    for q in range(n_items):
        x = rng.standard_normal(2048) * np.exp(-np.arange(2048) / (150.0 + 60 * q))
        items.append(O.autocorr_fft(x, p + 2))
    a, gg, checks, cap = _c4_emulate(items, p)
    assert checks == p
    assert cap == (152 if p >= 147 else 4 * (1 + STEP * ((p + 2 - 4 + 4 * STEP - 1) // (4 * STEP))))
    for q in range(n_items):
        a_ref, g_ref = O.lpc_from_autocorr(items[q], p)
        np.testing.assert_allclose(a[q, :p + 1], a_ref, rtol=1e-6, atol=1e-9 * np.abs(a_ref).max())
        assert np.all(a[q, p + 1:] == 0.0)  # the rows the cepstrum kernel reads are exactly 0 past p
        np.testing.assert_allclose(gg[q], g_ref, rtol=1e-8)


def test_durbin4_schedule_detects_a_stale_margin():
    """The emulation reads the same LDS cells the kernel does: a non-zero left in the guard (what a missing
    zero pass would leave) changes a, so the test above would catch a broken zero margin."""
    rng = np.random.default_rng(7)
    x = rng.standard_normal(2048) * np.exp(-np.arange(2048) / 300.0)
    items = [O.autocorr_fft(x, 152)]
    a_ok, _, _, _ = _c4_emulate(items, 150)
    try:
        a_bad, _, _, _ = _c4_emulate(items, 150, guard_fill=1.0)
        detected = not np.allclose(a_bad[0, :151], a_ok[0, :151])
    except AssertionError:  # the stale value reached B's last slot and the next item's first lane
        detected = True
    assert detected
