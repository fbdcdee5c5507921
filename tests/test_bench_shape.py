"""Parity at the exact benchmarked shapes (bench.py, N=1): the 1024 x 4 s WSJ batch (4096 analysis
frames, 327 680 LPC items: the persistent lattice kernel strides many item groups per block and the
XCD-mapped sweep grids are full) and one LibriSpeech-scale U(1,30) s batch (~4080 frames), built by
bench.py's own workload functions, against the CPU oracle at the north_star tolerance 1e-4 on the fp64
log features (computeFDLPSpectrogram.py:188-229) for utterances spread across the batch, plus the
autocorrelations and envelopes of the batch's last frames (stage parity on the last item groups of the
persistent grid).  The REVERB (M 450, range 1..450, U(2,15) s reverberant sets: the sliding-window cepstrum
over a multi-iteration persistent grid) and CHiME4 (range 1..100, babble mixed on the device at 20 dB) bench
workloads get the same checks, built by bench.py's own workload functions."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-4


class _Draws:
    """random.Random stand-in that replays a slice of the batch's jitter stream (randrange(2), :225)."""

    def __init__(self, bits):
        self._it = iter(int(b) for b in bits)

    def randrange(self, n):
        assert n == 2
        return next(self._it)


def _run_batch(entries, cfg_name="wsj", pcm=None, lens=None, mix=None, max_frames=None):
    import bench
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, PyRandom
    if pcm is None:
        lens = [t for _, t, _ in entries]
        pcm = bench.utterance_pcm(entries)
    cfg = getattr(FeatureConfig, cfg_name)()
    probe = FdlpPlan(cfg, device=-1)
    geo = [probe.geometry(t) for t in lens]
    frames = sum(g[0] for g in geo)
    plan = FdlpPlan(cfg, device=0, max_frames=max_frames or frames)
    plan.set_debug(True)  # (the envelopes are then kept whichever OLA stage runs)
    assert plan.autocorr_path == "structured"
    nj = sum(g[0] - 1 for g in geo)
    jit = PyRandom(7).randbits2(nj)
    _, rows, out64 = plan.compute(torch.from_numpy(pcm).cuda(), lens, jit, want_f64=True, **(mix or {}))
    torch.cuda.synchronize()
    offs = np.concatenate([[0], np.cumsum(lens)])
    jo = np.concatenate([[0], np.cumsum([g[0] - 1 for g in geo])])
    fo = np.concatenate([[0], np.cumsum([g[0] for g in geo])])
    return plan, pcm, offs, jit, jo, fo, rows, out64.cpu().numpy(), frames


def _check(entries, picks, cfg_name="wsj", pcm=None, lens=None, noise=None, draws=None):
    """Spread utterances vs the oracle at TOL, then r / env of the batch's last frames.  noise / draws: the
    babble and the per-utterance np.random.rand() draws of the CHiME4 mix (the oracle mixes on the host
    with numpy's RandomState, the GPU path takes (offset, alpha) from the NpRandom replica)."""
    from oracle import fdlp_oracle as O
    mix = None
    if noise is not None:
        import bench
        from speech_recognition_tools_amd import NpRandom
        if pcm is None:
            lens = [t for _, t, _ in entries]
            pcm = bench.utterance_pcm(entries)
        offs, alps = bench.noise_mix(pcm, lens, noise, bench.NOISE_SNR, NpRandom(draws))
        mix = dict(noise=torch.from_numpy(noise).cuda(), noise_off=offs, noise_alpha=alps)
    plan, pcm, offs, jit, jo, fo, rows, out64, frames = _run_batch(entries, cfg_name, pcm, lens, mix)
    orc = O.FdlpOracle(getattr(O.FdlpConfig, cfg_name)())
    us = np.random.RandomState(draws).rand(len(offs) - 1) if noise is not None else None

    def signal(i):
        x = pcm[offs[i]:offs[i + 1]]
        if noise is not None:  # add_noise_to_wav (features.py:24-31) on the host, numpy's own draws
            import bench
            x = O.add_noise(x, noise, bench.NOISE_SNR, us[i])
        return x

    worst = 0.0
    for i in picks:
        ref = orc.utterance(signal(i), _Draws(jit[jo[i]:jo[i + 1]]))
        got = out64[rows[i]:rows[i + 1]]
        assert got.shape == ref.shape, i
        err = float(np.abs(got - ref).max())
        worst = max(worst, err)
        assert err <= TOL, (i, err)
    # stage parity on the last frames of the batch: r (<= 1e-12 relative to r0) and the envelopes
    n = len(offs) - 1
    last = n - 1
    while fo[-1] - fo[last] < 8 and last > 0:
        last -= 1
    f0 = int(fo[last])
    d = plan.debug_fetch(frames - f0, first_frame=f0, keys=("r", "env"))
    keep_r, keep_e = [], []
    for i in range(last, n):
        k = O.Intermediates()
        orc.band_envelopes(signal(i), k)
        keep_r.append(k.r)
        keep_e.append(k.env)
    r_ref, e_ref = np.concatenate(keep_r), np.concatenate(keep_e)
    rel = np.abs(d["r"] - r_ref).max(axis=-1) / np.abs(r_ref[..., 0])
    assert rel.max() <= 1e-12, rel.max()
    assert np.abs(np.log(d["env"][..., 1:-1]) - np.log(e_ref[..., 1:-1])).max() <= 1e-5
    return worst


def test_wsj_bench_batch_vs_oracle():
    """bench.py default: 1024 utterances of 4 s, one 4096-frame batch; the first, every 32nd and the last."""
    import bench
    entries = bench.scp_list("wsj", 1, 1024, 4.0, 4096, None)
    picks = sorted(set(range(0, 1024, 32)) | {1023})
    _check(entries, picks)


def test_librispeech_bench_batch_vs_oracle():
    """bench.py --workload librispeech: U(1,30) s utterances filling 4096 frames; 32 spread utterances."""
    import bench
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig
    probe = FdlpPlan(FeatureConfig.wsj(), device=-1)
    entries = bench.scp_list("librispeech", 1, 0, 0.0, 4096, lambda t: probe.geometry(t)[0])
    n = len(entries)
    picks = sorted(set(np.linspace(0, n - 1, 32).astype(int).tolist()))
    _check(entries, picks)


def test_chime4_bench_batch_vs_oracle():
    """bench.py --config chime4: the 1024 x 4 s batch with CHiME4 params (range 1..100) and babble mixed on
    the device at 20 dB (frames_dft1_c_kernel's fused s + alpha * n) vs the oracle mixing on the host."""
    import bench
    entries = bench.scp_list("wsj", 1, 1024, 4.0, 4096, None)
    picks = sorted(set(range(0, 1024, 32)) | {1023})
    _check(entries, picks, "chime4", noise=bench.babble_noise(), draws=31)


def test_reverb_bench_batch_vs_oracle():
    """bench.py --config reverb: U(2,15) s utterances of the two synthetic reverberant sets (4096 frames,
    M 450: the sliding-window cepstrum on the persistent grid, many item groups per block), 32 spread
    utterances vs the oracle; r / env of the batch's last frames."""
    import bench
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig
    probe = FdlpPlan(FeatureConfig.reverb(), device=-1)
    entries = bench.scp_list("reverb", 1, 0, 0.0, 4096, lambda t: probe.geometry(t)[0])
    pcm, lens = bench.reverb_pcm(entries, torch.device("cuda", 0))
    assert sum(probe.geometry(t)[0] for t in lens) <= 4096
    n = len(entries)
    picks = sorted(set(np.linspace(0, n - 1, 32).astype(int).tolist()))
    _check(entries, picks, "reverb", pcm=pcm, lens=lens)


def test_reverb_workload_synthesis_matches_addreverb():
    """The REVERB workload's device reverberation (fdlp_reverb) equals the oracle's addReverb
    (features.py:110-115: np.convolve + np.correlate alignment) before the int16 rounding, for the two
    shortest utterances of each set."""
    import bench
    from oracle import fdlp_oracle as O
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig
    from speech_recognition_tools_amd.augment import reverb
    probe = FdlpPlan(FeatureConfig.reverb(), device=-1)
    entries = bench.scp_list("reverb", 1, 0, 0.0, 4096, lambda t: probe.geometry(t)[0])
    for k, kind in enumerate(bench.REVERB_SETS):
        idx = sorted((i for i in range(len(entries)) if (i & 1) == k), key=lambda i: entries[i][1])[:2]
        sub = [entries[i] for i in idx]
        h = bench.synthetic_rir(kind)
        x = bench.utterance_pcm(sub)
        y, ol = reverb(torch.from_numpy(x).cuda(), [t for _, t, _ in sub], torch.from_numpy(h).cuda())
        y = y.cpu().numpy()
        o = 0
        for j, (_, T, _) in enumerate(sub):
            ref = O.add_reverb(x[o:o + T].astype(np.float64), h)
            assert int(ol[j]) == ref.size
            np.testing.assert_allclose(y[o:o + ref.size], ref, rtol=0, atol=1e-9 * np.abs(ref).max())
            o += T
