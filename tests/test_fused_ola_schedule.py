"""CPU restatement of the fused OLA of lpc_env_lattice_kernel<..., OLA = true> (csrc/fdlp_lpc.hip) and of its
chunk tables (csrc/fdlp_plan.cpp build_ola_chunks): chunks of one utterance's frames cut every 8 frames
between two middle frames, each frame's envelope samples routed to the rows it owns (with the previous
frame's tail from the ring), to the next frame's tail (ring, or fb at a chunk edge) or to fa (a chunk's first
overlap rows), the uncovered owned rows, then ola_fixup_kernel's 0 + fb + fa.  Checked bit for bit against
the reference's in-place OLA (computeFDLPSpectrogram.py:207-229: out = 0, out[dst:dst+cnt] += env[src:src+cnt]
frame by frame, log(clip(out, 1e-14))) on the plan's own OLA tables."""
import numpy as np
import pytest

CHUNK = 8


def chunks_of(tab, kk):
    """build_ola_chunks for one utterance: [(k0, k1, bin, bout)], bounds [(dst of frame k1, len)]."""
    dst, src, cnt = tab
    F = dst.size
    out, bounds = [], []
    k0, bin_ = 0, -1
    while k0 < F:
        k1, bout = F, -1
        for kb in range(k0 + CHUNK, F - 2):
            ln = dst[kb - 1] + kk - dst[kb]
            if cnt[kb - 1] == kk and cnt[kb] == kk and src[kb - 1] == 0 and src[kb] == 0 and 0 < ln <= kk and kb >= 2:
                bounds.append((dst[kb], ln))
                bout = len(bounds) - 1
                k1 = kb
                break
        out.append((k0, k1, bin_, bout))
        bin_ = bout
        k0 = k1
    return out, bounds


def fused(env, tab, L, kk):
    """The kernel's routing for one utterance and all bands at once (env [F, B, kk] -> out [L, B])."""
    dst, src, cnt = tab
    F, B = env.shape[0], env.shape[1]
    out = np.full((L, B), np.nan)
    written = np.zeros(L, int)
    chunks, bounds = chunks_of(tab, kk)
    fa = np.full((len(bounds), B, kk), np.nan)
    fb = np.full((len(bounds), B, kk), np.nan)
    ring = np.full((2, B, kk), np.nan)

    def store(t, acc):
        out[t] = np.log(np.where(acc < 1e-14, 1e-14, acc))
        written[t] += 1
    for k0, k1, bin_, bout in chunks:
        for k in range(k0, k1):
            lo = 0 if k == 0 else min(dst[k], L)
            hi = min(dst[k + 1], L) if k + 1 < F else L
            tail = dst[k - 1] + cnt[k - 1] if k > 0 else 0
            b_in = bin_ if k == k0 else -1
            b_out = bout if k + 1 == k1 else -1
            rr, rw = ring[k & 1], ring[(k + 1) & 1]
            for s_ in range(kk):
                if s_ < src[k] or s_ >= src[k] + cnt[k]:
                    continue
                t = dst[k] + s_ - src[k]
                e = env[k, :, s_]
                if t >= hi:
                    assert t - hi < kk
                    if b_out >= 0:
                        fb[b_out, :, t - hi] = e
                    else:
                        rw[:, t - hi] = e
                    continue
                if b_in >= 0 and t < tail:
                    fa[b_in, :, t - dst[k]] = e
                    continue
                acc = np.zeros(B)
                if t < tail:
                    acc = acc + rr[:, t - dst[k]]
                store(t, acc + e)
            for t in list(range(lo, min(dst[k], hi))) + list(range(max(dst[k] + cnt[k], lo), hi)):
                acc = np.zeros(B)
                if t < tail:
                    acc = acc + rr[:, t - dst[k]]
                store(t, acc)
    for b, (d0, ln) in enumerate(bounds):
        for r in range(ln):
            store(d0 + r, (np.zeros(B) + fb[b, :, r]) + fa[b, :, r])
    assert (written == 1).all(), np.flatnonzero(written != 1)[:10]
    return out


def reference(env, tab, L):
    dst, src, cnt = tab
    out = np.zeros((L, env.shape[1]))
    for k in range(env.shape[0]):
        out[dst[k]:dst[k] + cnt[k]] += env[k, :, src[k]:src[k] + cnt[k]].T
    return np.log(np.clip(out, 1e-14, None))


@pytest.mark.parametrize("cfg_name", ["wsj", "reverb"])
@pytest.mark.parametrize("secs", [0.2, 1.0, 1.6, 4.0, 12.9, 13.0, 20.05, 30.0, 61.3])
def test_fused_ola_routing_matches_reference_ola(cfg_name, secs):
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, PyRandom
    plan = FdlpPlan(getattr(FeatureConfig, cfg_name)(), device=-1)
    T = int(secs * 16000)
    F, L = plan.geometry(T)
    tab = plan.ola_table(T, PyRandom(int(secs * 100)).randbits2(max(F - 1, 0)))
    kk = plan.kk
    for k in range(1, F - 1):  # the fused path's condition: at most two frames on a row
        assert tab[0][k + 1] >= tab[0][k - 1] + tab[2][k - 1]
    rng = np.random.default_rng(F)
    env = np.exp(rng.standard_normal((F, 4, kk)) * 3.0)
    env[:, :, 0] = 0.0  # the window's zero
    got = fused(env, tab, L, kk)
    ref = reference(env, tab, L)
    np.testing.assert_array_equal(got.view(np.uint64), ref.view(np.uint64))
    nb = len(chunks_of(tab, kk)[1])
    assert nb == (0 if F <= CHUNK + 2 else nb) and (F < 12 or nb >= 1)
