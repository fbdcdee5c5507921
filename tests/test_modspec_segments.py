"""computeModulationSpectrum_segments.py drop-in (the segments sibling of §8f rank 4).

Goldens: tests/golden/modspec_segments*.npz, made by tests/golden/make_golden.py --modspec-segments-only
importing the real reference (two recordings, four segments out of recording order with fractional times;
default options, and --set_unity_gain with other sizes).  CPU: the segment slicing + oracle against the
goldens, argv defaults.  GPU: the FDLP plan's modspec mode on the segment signals (fp64, relative 1e-7 as
tests/test_modspec.py) and the CLI's ark ('%.3f', as dict2Ark)."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import modspec_oracle as MS

SETS = ["modspec_segments", "modspec_segments_unity"]
TOL = 1e-7


def _segments(name):
    meta, rec, _, z = load_golden(name)
    segs = meta["extra"]["segments"]
    ref = {s[0]: z["seg_" + s[0]] for s in segs}
    return meta, rec, segs, ref


def _oracle(sig, o):
    got = MS.modspec_features(sig, nfilters=o["nfilters"], coeff_0=1, coeff_n=o["nmodulations"], order=o["order"],
                              fduration=o["fduration"], frate=o["frate"], fbank_type="mel,1")
    if o.get("set_unity_gain"):  # gg = 1: c_0 = log(sqrt(1)) (computeModulationSpectrum_segments.py:108-110)
        got.reshape(got.shape[0], o["nfilters"], o["nmodulations"])[:, :, 0] = 0.0
    return got


@pytest.mark.parametrize("name", SETS)
def test_segments_oracle_matches_reference(name):
    from speech_recognition_tools_amd.featgen.computeModulationSpectrum_segments import segment_signal
    meta, rec, segs, ref = _segments(name)
    for s_id, r_id, t0, t1 in segs:
        got = _oracle(segment_signal(rec[r_id], 16000, t0, t1), meta["opts"])
        assert got.shape == ref[s_id].shape, s_id
        np.testing.assert_allclose(got, ref[s_id], rtol=1e-9, atol=1e-9)


def test_segment_signal_slicing():
    from speech_recognition_tools_amd.featgen.computeModulationSpectrum_segments import segment_signal
    x = np.arange(100, dtype=np.int16)
    y = segment_signal(x, 10, "1.05", "2.5")  # int(10.5) = 10 .. int(25.0) = 25
    assert y.dtype == np.float64 and y.shape == (15,) and y[0] == 10 / 32768.0
    assert segment_signal(x, 10, "9.5", "20").shape == (5,)  # numpy slicing clips at the end


def test_segments_cli_args(tmp_path):
    from speech_recognition_tools_amd.featgen.computeModulationSpectrum_segments import (feature_config, get_args,
                                                                                          read_scp, segments_of)
    a = get_args(["w.scp", "segs", "out"])
    assert (a.nfilters, a.nmodulations, a.order, a.fduration, a.frate, a.set_unity_gain) == (15, 12, 50, 0.5, 100, False)
    c = feature_config(a)
    assert c.mode == "modspec" and c.window == "hanning" and c.coeff_0 == 1 and c.coeff_num == 12
    scp = tmp_path / "w.scp"
    scp.write_text("r1 /x/a.wav\n\nr2 sph2pipe -f wav b.sph |\n")
    assert read_scp(str(scp)) == (["r1", "r2"], ["/x/a.wav", "sph2pipe -f wav b.sph |"])
    seg = tmp_path / "segs"
    seg.write_text("s1 r1 0.0 1.5\n\ns2 r2 1 2\n")
    assert list(segments_of(str(seg))) == [("s1", "r1", "0.0", "1.5"), ("s2", "r2", "1", "2")]


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_segments_gpu_vs_reference_golden(name):
    import torch
    from speech_recognition_tools_amd.featgen.computeModulationSpectrum_segments import (feature_config, get_args,
                                                                                          segment_signal)
    from speech_recognition_tools_amd.plan import FdlpPlan
    meta, rec, segs, ref = _segments(name)
    o = meta["opts"]
    argv = ["w.scp", "segs", "out", "--nfilters=%d" % o["nfilters"], "--nmodulations=%d" % o["nmodulations"],
            "--order=%d" % o["order"], "--fduration=%s" % o["fduration"], "--frate=%d" % o["frate"]]
    plan = FdlpPlan(feature_config(get_args(argv)), device=0, max_frames=2048)
    sigs = [np.ascontiguousarray(segment_signal(rec[r], 16000, t0, t1)) for _, r, t0, t1 in segs]
    out, rows, out64 = plan.compute(torch.from_numpy(np.concatenate(sigs)).cuda(), [s.size for s in sigs], None,
                                    want_f64=True)
    out64 = out64.cpu().numpy()
    for i, (s_id, _, _, _) in enumerate(segs):
        f64 = out64[rows[i]:rows[i + 1]].copy()
        if o.get("set_unity_gain"):
            f64.reshape(f64.shape[0], o["nfilters"], o["nmodulations"])[:, :, 0] = 0.0
        assert f64.shape == ref[s_id].shape, s_id
        scale = np.maximum(1.0, np.abs(ref[s_id]))
        assert np.max(np.abs(f64 - ref[s_id]) / scale) <= TOL, (name, s_id)


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_segments_cli_writes_reference_arks(tmp_path, name):
    from scipy.io import wavfile
    from speech_recognition_tools_amd.featgen.computeModulationSpectrum_segments import get_args, get_feats
    from speech_recognition_tools_amd.featgen.features import read_ark
    meta, rec, segs, ref = _segments(name)
    o = meta["opts"]
    scp = tmp_path / "wav.scp"
    with open(scp, "w") as f:
        for r, x in rec.items():
            p = tmp_path / (r + ".wav")
            wavfile.write(str(p), 16000, x)
            f.write("%s %s\n" % (r, p))
    seg = tmp_path / "segments"
    seg.write_text("".join("%s %s %s %s\n" % tuple(s) for s in segs))
    out = str(tmp_path / "ms")
    argv = [str(scp), str(seg), out, "--nfilters=%d" % o["nfilters"], "--nmodulations=%d" % o["nmodulations"],
            "--order=%d" % o["order"], "--fduration=%s" % o["fduration"], "--frate=%d" % o["frate"],
            "--kaldi_cmd=copy-feats"]
    if o.get("set_unity_gain"):
        argv.append("--set_unity_gain")
    get_feats(get_args(argv))
    ark = read_ark(out + ".ark")
    assert list(ark) == [s[0] for s in segs]
    for s_id in ark:
        q = np.round(ref[s_id], 3).astype(np.float32)
        assert ark[s_id].shape == q.shape
        assert np.abs(ark[s_id] - q).max() <= 1.0011e-3 * max(1.0, np.abs(ref[s_id]).max()), s_id
