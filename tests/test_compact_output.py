"""Compact ark codes (ABI 7, include/fdlp.h fdlp_batch.out_q_dev): the features leave the device as int16
k = nearbyint(v * 10^d) and fdlp_q_widen turns them into the float32 ark values (float)(k / 10^d) that
dict2Ark's '%.3f' text + copy-feats produce (features.py:63-69).  The codes must widen to exactly the
float32 rows the device writes to out_dev -- bit for bit, -0.0 included."""
import numpy as np
import pytest
import torch

from conftest import feature_cfg, load_golden


def _ref_widen(q, decimals):
    sc = 1.0
    for _ in range(decimals):
        sc *= 10.0
    v = (q.astype(np.float64) / sc).astype(np.float32)
    v[q == -32768] = np.float32(-0.0)
    return v


@pytest.mark.parametrize("decimals", [0, 1, 3, 4])
@pytest.mark.parametrize("threads", [1, 5])
def test_q_widen_every_code(decimals, threads):
    from speech_recognition_tools_amd import q_widen
    q = np.tile(np.arange(-32768, 32768, dtype=np.int32).astype(np.int16), 3)
    got = q_widen(q, decimals, threads=threads)
    ref = _ref_widen(q, decimals)
    assert got.dtype == np.float32
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert got[0] == 0.0 and np.signbit(got[0])  # -32768 is -0.0


def test_q_widen_rejects_bad_args():
    from speech_recognition_tools_amd import q_widen
    from speech_recognition_tools_amd._lib import FdlpError
    with pytest.raises(FdlpError):
        q_widen(np.zeros(4, np.int16), -1)
    with pytest.raises(ValueError):
        q_widen(np.zeros(4, np.int16), 3, out=np.zeros(3, np.float32))


def _wsj_batch():
    meta, sig, _, _ = load_golden("wsj")
    utts = meta["utts"]
    return meta, [sig[u] for u in utts]


def _run(plan, pcm_list, **kw):
    from speech_recognition_tools_amd import PyRandom
    lens = [x.size for x in pcm_list]
    nj = sum(plan.geometry(T)[0] - 1 for T in lens)
    pcm = torch.from_numpy(np.concatenate(pcm_list)).cuda()
    return plan.compute(pcm, lens, PyRandom(5).randbits2(nj), **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["device", "pinned"])
def test_codes_widen_to_the_float32_rows(where):
    from speech_recognition_tools_amd import FdlpPlan, q_widen
    meta, pcm_list = _wsj_batch()
    plan = FdlpPlan(feature_cfg(meta), device=0, max_frames=512)
    rows = sum(plan.geometry(x.size)[1] for x in pcm_list)
    out = torch.empty((rows, plan.out_dim), dtype=torch.float32, device="cuda")
    if where == "device":
        q = torch.full((rows, plan.out_dim), -32767, dtype=torch.int16, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    else:  # the OLA kernel stores the codes straight into pinned host memory
        q = torch.full((rows, plan.out_dim), -32767, dtype=torch.int16).pin_memory()
        flag = torch.zeros(1, dtype=torch.int32).pin_memory()
    f, _, _ = _run(plan, pcm_list, out=out, out_q=q, q_flag=flag)
    torch.cuda.synchronize()
    fh = f.cpu().numpy()
    qh = q.cpu().numpy()
    assert int(flag.cpu()[0]) == 0
    w = q_widen(qh, 3, threads=4)
    np.testing.assert_array_equal(w.view(np.uint32), fh.view(np.uint32))
    assert (qh != -32767).all()  # every code written (-32.767 is below the log floor -32.236)
    # the codes alone (no float32 rows): the same codes
    q2 = torch.zeros((rows, plan.out_dim), dtype=torch.int16, device="cuda")
    flag.zero_()
    f2, _, _ = _run(plan, pcm_list, out_q=q2, q_flag=flag)
    assert f2 is None
    np.testing.assert_array_equal(q2.cpu().numpy(), qh)
    # the features exercise the sign of zero (log(acc) in (-0.0005, 0) rounds to -0.0)
    assert np.abs(fh).min() < 0.01


@pytest.mark.gpu
def test_values_without_a_code_set_the_flag():
    """fp64 PCM scaled far past 16-bit range drives the log features beyond +32.767: those values store
    -32768 and set the flag, and the float32 rows carry the values."""
    from speech_recognition_tools_amd import FdlpPlan, q_widen
    meta, pcm_list = _wsj_batch()
    plan = FdlpPlan(feature_cfg(meta), device=0, max_frames=512)
    x = [p.astype(np.float64) * 1e9 for p in pcm_list[:2]]
    rows = sum(plan.geometry(p.size)[1] for p in x)
    q = torch.zeros((rows, plan.out_dim), dtype=torch.int16, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    f, _, _ = _run(plan, x, out_q=q, q_flag=flag, out=torch.empty((rows, plan.out_dim), device="cuda"))
    torch.cuda.synchronize()
    fh, qh = f.cpu().numpy(), q.cpu().numpy()
    big = fh > 32.767
    assert big.any() and int(flag.cpu()[0]) == 1
    assert (qh[big] == -32768).all()
    ok = ~big & ~((fh == 0) & np.signbit(fh))
    np.testing.assert_array_equal(q_widen(qh[ok], 3).view(np.uint32), fh[ok].view(np.uint32))


@pytest.mark.gpu
def test_compact_codes_need_decimals_and_flag():
    from speech_recognition_tools_amd import FdlpPlan
    meta, pcm_list = _wsj_batch()
    plan = FdlpPlan(feature_cfg(meta), device=0, max_frames=512)
    rows = sum(plan.geometry(x.size)[1] for x in pcm_list)
    q = torch.zeros((rows, plan.out_dim), dtype=torch.int16, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    with pytest.raises(Exception):
        _run(plan, pcm_list, out_q=q, q_flag=flag, ark_decimals=-1)
    with pytest.raises(ValueError):
        _run(plan, pcm_list, out_q=q)
