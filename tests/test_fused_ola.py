"""OLA + log fused into the LPC kernel (ABI 7, include/fdlp.h FDLP_OLA_FUSED; computeFDLPSpectrogram.py:207-229):
every output -- fp64 log features, '%.3f' float32 rows, compact codes -- bit-identical to the separate
ola_log_tiled_kernel (FDLP_OLA_SEPARATE) on the golden sets, the bench batch, utterances long enough to be cut
into chunks (their edges finished by ola_fixup_kernel), short utterances with dead tails, and REVERB's FFT
envelope.  The separate kernel is itself pinned to the reference goldens (tests/test_gpu_parity.py)."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN_SETS, feature_cfg, load_golden

pytestmark = pytest.mark.gpu


def _both(cfg, pcm, lens, seed=11, **kw):
    """(fused, separate) runs of one batch: (f32, f64, codes, flag, plan.ola_path)."""
    from speech_recognition_tools_amd import FdlpPlan, PyRandom
    res = []
    for path in ("fused", "separate"):
        plan = FdlpPlan(cfg, device=0, max_frames=max(64, sum(FdlpPlan(cfg, device=-1).geometry(t)[0] for t in lens)))
        plan.set_ola_path(path)
        nj = sum(plan.geometry(t)[0] - 1 for t in lens)
        rows = sum(plan.geometry(t)[1] for t in lens)
        q = torch.full((rows, plan.out_dim), -32767, dtype=torch.int16, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        f32, _, f64 = plan.compute(torch.from_numpy(pcm).cuda(), lens, PyRandom(seed).randbits2(nj), want_f64=True,
                                   out_q=q, q_flag=flag, out=torch.empty((rows, plan.out_dim), device="cuda"), **kw)
        torch.cuda.synchronize()
        res.append((f32.cpu().numpy(), f64.cpu().numpy(), q.cpu().numpy(), int(flag.cpu()[0]), plan.ola_path))
    return res


def _same(a, b, what):
    (f32a, f64a, qa, fla, pa), (f32b, f64b, qb, flb, pb) = a, b
    assert pa == "fused" and pb == "separate", (what, pa, pb)
    np.testing.assert_array_equal(f64a.view(np.uint64), f64b.view(np.uint64), err_msg=what)
    np.testing.assert_array_equal(f32a.view(np.uint32), f32b.view(np.uint32), err_msg=what)
    np.testing.assert_array_equal(qa, qb, err_msg=what)
    assert fla == flb == 0
    assert (qa != -32767).all(), what  # every row written


@pytest.mark.parametrize("name", [n for n in GOLDEN_SETS if not n.startswith("reverb_rir")])
def test_fused_ola_bit_identical_on_golden_sets(name):
    meta, sig, ref, z = load_golden(name)
    if meta["opts"].get("add_noise", "clean") != "clean":
        pytest.skip("noise mixing: covered through the bench-shape CHiME-4 batch")
    pcm = np.concatenate([sig[u] for u in meta["utts"]])
    lens = [sig[u].size for u in meta["utts"]]
    kw = dict(preprocess="diff") if meta["opts"].get("add_noise") == "diff" else {}
    a, b = _both(feature_cfg(meta), pcm, lens, seed=meta["seed"], **kw)
    _same(a, b, name)


@pytest.mark.parametrize("cfg_name,secs", [("wsj", [4.0] * 64), ("wsj", [1.0, 13.0, 30.0, 29.99, 12.5, 0.3, 7.1]),
                                           ("reverb", [2.0, 15.0, 14.2, 3.3]), ("chime4", [4.0] * 8)])
def test_fused_ola_bit_identical_on_bench_shapes(cfg_name, secs):
    """4 s batches (one 4-frame chunk per utterance), long utterances cut into chunks (up to 26 frames: three
    chunk edges), a 0.3 s utterance (dead tail), REVERB's M = 450 / FFT envelope, CHiME-4 parameters."""
    import bench
    from speech_recognition_tools_amd import FeatureConfig
    lens = [int(s * 16000) for s in secs]
    pcm = bench.speech_like_batch(1, sum(lens), 77).reshape(-1)
    a, b = _both(getattr(FeatureConfig, cfg_name)(), pcm, lens)
    _same(a, b, "%s %s" % (cfg_name, secs))
