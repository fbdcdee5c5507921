"""Parity at the exact benchmarked shapes (bench.py, N=1): the 1024 x 4 s WSJ batch (4096 analysis
frames, 327 680 LPC items: the persistent lattice kernel strides many item groups per block and the
XCD-mapped sweep grids are full) and one LibriSpeech-scale U(1,30) s batch (~4080 frames), built by
bench.py's own workload functions, against the CPU oracle at the north_star tolerance 1e-4 on the fp64
log features (computeFDLPSpectrogram.py:188-229) for utterances spread across the batch, plus the
autocorrelations and envelopes of the batch's last frames (stage parity on the last item groups of the
persistent grid)."""
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


def _run_batch(entries, max_frames=None):
    import bench
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, PyRandom
    lens = [t for _, t, _ in entries]
    pcm = bench.utterance_pcm(entries)
    probe = FdlpPlan(FeatureConfig.wsj(), device=-1)
    geo = [probe.geometry(t) for t in lens]
    frames = sum(g[0] for g in geo)
    plan = FdlpPlan(FeatureConfig.wsj(), device=0, max_frames=max_frames or frames)
    assert plan.autocorr_path == "structured"
    nj = sum(g[0] - 1 for g in geo)
    jit = PyRandom(7).randbits2(nj)
    _, rows, out64 = plan.compute(torch.from_numpy(pcm).cuda(), lens, jit, want_f64=True)
    torch.cuda.synchronize()
    offs = np.concatenate([[0], np.cumsum(lens)])
    jo = np.concatenate([[0], np.cumsum([g[0] - 1 for g in geo])])
    fo = np.concatenate([[0], np.cumsum([g[0] for g in geo])])
    return plan, pcm, offs, jit, jo, fo, rows, out64.cpu().numpy(), frames


def _check(entries, picks):
    from oracle import fdlp_oracle as O
    plan, pcm, offs, jit, jo, fo, rows, out64, frames = _run_batch(entries)
    orc = O.FdlpOracle(O.FdlpConfig.wsj())
    worst = 0.0
    for i in picks:
        x = pcm[offs[i]:offs[i + 1]]
        ref = orc.utterance(x, _Draws(jit[jo[i]:jo[i + 1]]))
        got = out64[rows[i]:rows[i + 1]]
        assert got.shape == ref.shape, i
        err = float(np.abs(got - ref).max())
        worst = max(worst, err)
        assert err <= TOL, (i, err)
    # stage parity on the last frames of the batch: r (<= 1e-12 relative to r0) and the envelopes
    last = len(entries) - 1
    while fo[-1] - fo[last] < 8 and last > 0:
        last -= 1
    f0 = int(fo[last])
    d = plan.debug_fetch(frames - f0, first_frame=f0, keys=("r", "env"))
    keep_r, keep_e = [], []
    for i in range(last, len(entries)):
        k = O.Intermediates()
        orc.band_envelopes(pcm[offs[i]:offs[i + 1]], k)
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
