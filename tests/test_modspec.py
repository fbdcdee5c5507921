"""FDLP modulation spectrum sibling feature: src/featgen/computeModulationSpectrum.py.

CPU: the oracle (oracle/modspec_oracle.py) against the real reference's outputs (tests/golden/modspec_*.npz,
made by tests/golden/make_golden.py --modspec-only), host-side geometry and option validation.  GPU: the FDLP
plan in its modspec mode against the goldens (fp64 cepstra, relative 1e-7: the reference computes in fp64, the
device differs only by summation order in the DCT/autocorrelation/Levinson), a reverberated batch against the
oracle, and the compute-modspec-feats CLI's ark ('%.3f' rounding, as dict2Ark)."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import fdlp_oracle as O
from oracle import mel_oracle as MO
from oracle import modspec_oracle as MS

MODSPEC_SETS = ["modspec_default", "modspec_even_comp_abs", "modspec_cochlear_rect"]
COMPLEX_SETS = ["modspec_complex", "modspec_complex_even_comp_abs", "modspec_complex_cochlear_rect"]
TOL = 1e-7


@pytest.mark.parametrize("name", MODSPEC_SETS)
def test_modspec_oracle_matches_reference(name):
    meta, sig, ref, _ = load_golden(name)
    for u in meta["utts"]:
        got = MS.modspec_features(sig[u].astype(np.float64), **meta["opts"])
        assert got.shape == ref[u].shape, u
        np.testing.assert_allclose(got, ref[u], rtol=1e-9, atol=1e-9)


def _opts(o):
    o = dict(o)
    o.pop("complex_modulation", None)
    return o


@pytest.mark.parametrize("name", COMPLEX_SETS)
def test_modspec_complex_oracle_matches_reference(name):
    meta, sig, ref, _ = load_golden(name)
    for u in meta["utts"]:
        got = MS.modspec_complex_features(sig[u].astype(np.float64), **_opts(meta["opts"]))
        assert got.shape == ref[u].shape, u
        np.testing.assert_allclose(got, ref[u], rtol=1e-9, atol=1e-9)


def test_modspec_complex_geometry_and_validation():
    from speech_recognition_tools_amd._lib import FdlpError
    from speech_recognition_tools_amd.plan import FdlpPlan, FeatureConfig
    for name in COMPLEX_SETS:
        meta, _, ref, _ = load_golden(name)
        plan = FdlpPlan(_cfg(meta["opts"]), device=-1, max_frames=16)
        assert plan.out_dim == ref[meta["utts"][0]].shape[1], name
    with pytest.raises(FdlpError):  # keep_even without abs: the reference's broadcast error
        FdlpPlan(FeatureConfig(mode="modspec_complex", nfilters=15, coeff_num=30, coeff_0=5, order=50,
                               keep_even=True), device=-1)


def _cfg(o):
    from speech_recognition_tools_amd.plan import FeatureConfig
    return FeatureConfig(mode="modspec_complex" if o.get("complex_modulation") else "modspec",
                         window="rect" if o.get("no_window") else "hanning",
                         nfilters=o["nfilters"], coeff_num=o["coeff_n"], coeff_0=o["coeff_0"], order=o["order"],
                         fduration=o["fduration"], frate=o["frate"], fbank_type=o["fbank_type"],
                         keep_even=bool(o.get("keep_even")), compensate_noise=bool(o.get("compensate_noise")),
                         absolute_value=bool(o.get("absolute_value")))


def test_modspec_geometry_and_width():
    from speech_recognition_tools_amd.plan import FdlpPlan
    for name in MODSPEC_SETS:
        meta, _, ref, _ = load_golden(name)
        o = meta["opts"]
        plan = FdlpPlan(_cfg(o), device=-1, max_frames=16)
        assert plan.out_dim == ref[meta["utts"][0]].shape[1]
        for T in (2, 100, 3999, 4000, 4001, 8000, 23457):
            F, L = plan.geometry(T)
            assert F == L == MO.get_frames(np.zeros(T), 16000, o["frate"], o["fduration"], np.hanning).shape[0]


def test_modspec_option_validation():
    from speech_recognition_tools_amd._lib import FdlpError
    from speech_recognition_tools_amd.plan import FdlpPlan, FeatureConfig
    for bad in (dict(coeff_0=0), dict(coeff_0=31), dict(gamma_weight="1,2,3"), dict(odd_mod_zero=True)):
        kw = dict(mode="modspec", nfilters=15, coeff_num=30, coeff_0=5, order=50)
        kw.update(bad)
        with pytest.raises(FdlpError):
            FdlpPlan(FeatureConfig(**kw), device=-1)


def test_modspec_cli_args():
    from speech_recognition_tools_amd.featgen.computeModulationSpectrum import feature_config, get_args
    a = get_args(["s.scp", "out"])
    assert (a.nfilters, a.coeff_0, a.coeff_n, a.order, a.fduration, a.frate, a.fbank_type) == \
        (15, 5, 30, 50, 0.5, 100, "mel,1")
    c = feature_config(get_args(["s.scp", "out", "--no_window", "--keep_even", "--coeff_0=2"]))
    assert c.mode == "modspec" and c.window == "rect" and c.keep_even and c.coeff_0 == 2
    assert feature_config(get_args(["s.scp", "out", "--complex_modulation"])).mode == "modspec_complex"


def _modspec_gpu(cfg, sig, utts, rir=None, max_frames=4096):
    import torch
    from speech_recognition_tools_amd.augment import reverb
    from speech_recognition_tools_amd.plan import FdlpPlan
    plan = FdlpPlan(cfg, device=0, max_frames=max_frames)
    lens = [sig[u].size for u in utts]
    pcm = torch.from_numpy(np.concatenate([sig[u] for u in utts])).cuda()
    offs = None
    if rir is not None:
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        pcm, lens = reverb(pcm, lens, torch.from_numpy(rir).cuda(), offsets=offs)
    out, rows, out64 = plan.compute(pcm, lens, None, offsets=offs, want_f64=True)
    out, out64 = out.cpu().numpy(), out64.cpu().numpy()
    return {u: (out64[rows[i]:rows[i + 1]], out[rows[i]:rows[i + 1]]) for i, u in enumerate(utts)}


@pytest.mark.gpu
@pytest.mark.parametrize("name", MODSPEC_SETS)
def test_modspec_gpu_vs_reference_golden(name):
    meta, sig, ref, _ = load_golden(name)
    res = _modspec_gpu(_cfg(meta["opts"]), sig, meta["utts"])
    for u in meta["utts"]:
        f64, f32 = res[u]
        assert f64.shape == ref[u].shape, u
        scale = np.maximum(1.0, np.abs(ref[u]))
        assert np.max(np.abs(f64 - ref[u]) / scale) <= TOL, (name, u, np.max(np.abs(f64 - ref[u]) / scale))
        np.testing.assert_allclose(f32, np.round(ref[u], 3).astype(np.float32), rtol=0, atol=1.0011e-3 * scale.max())


@pytest.mark.gpu
@pytest.mark.parametrize("name", COMPLEX_SETS)
def test_modspec_complex_gpu_vs_reference_golden(name):
    meta, sig, ref, _ = load_golden(name)
    res = _modspec_gpu(_cfg(meta["opts"]), sig, meta["utts"])
    for u in meta["utts"]:
        f64, f32 = res[u]
        assert f64.shape == ref[u].shape, u
        scale = np.maximum(1.0, np.abs(ref[u]))
        assert np.max(np.abs(f64 - ref[u]) / scale) <= TOL, (name, u, np.max(np.abs(f64 - ref[u]) / scale))
        np.testing.assert_allclose(f32, np.round(ref[u], 3).astype(np.float32), rtol=0, atol=1.0011e-3 * scale.max())


@pytest.mark.gpu
def test_modspec_gpu_reverb_vs_oracle():
    meta, sig, _, _ = load_golden("modspec_default")
    _, _, _, zr = load_golden("reverb_rir")
    rir = O.load_rir(zr["rir"])
    res = _modspec_gpu(_cfg(meta["opts"]), sig, meta["utts"], rir=rir)
    for u in meta["utts"]:
        want = MS.modspec_features(O.add_reverb(sig[u], rir), **meta["opts"])
        f64 = res[u][0]
        assert f64.shape == want.shape, u
        assert np.max(np.abs(f64 - want) / np.maximum(1.0, np.abs(want))) <= TOL, u


@pytest.mark.gpu
def test_modspec_cli_writes_reference_arks(tmp_path):
    from scipy.io import wavfile
    from speech_recognition_tools_amd.featgen.computeModulationSpectrum import get_args, get_feats
    from speech_recognition_tools_amd.featgen.features import read_ark
    meta, sig, ref, _ = load_golden("modspec_even_comp_abs")
    scp = tmp_path / "wav.scp"
    with open(scp, "w") as f:
        for u in meta["utts"]:
            p = tmp_path / (u + ".wav")
            wavfile.write(str(p), 16000, sig[u])
            f.write("%s %s\n" % (u, p))
    out = str(tmp_path / "modspec")
    get_feats(get_args([str(scp), out, "--keep_even", "--compensate_noise", "--absolute_value",
                        "--add_reverb=clean", "--kaldi_cmd=copy-feats"]))
    ark = read_ark(out + ".ark")
    assert list(ark) == meta["utts"]
    scp_keys = [l.split()[0] for l in open(out + ".scp")]
    assert scp_keys == meta["utts"]
    for u in meta["utts"]:
        q = np.round(ref[u], 3).astype(np.float32)
        assert ark[u].shape == q.shape
        assert np.abs(ark[u] - q).max() <= 1.0011e-3 * max(1.0, np.abs(ref[u]).max())


@pytest.mark.gpu
def test_modspec_complex_cli_writes_reference_arks(tmp_path):
    from scipy.io import wavfile
    from speech_recognition_tools_amd.featgen.computeModulationSpectrum import get_args, get_feats
    from speech_recognition_tools_amd.featgen.features import read_ark
    meta, sig, ref, _ = load_golden("modspec_complex")
    scp = tmp_path / "wav.scp"
    with open(scp, "w") as f:
        for u in meta["utts"]:
            p = tmp_path / (u + ".wav")
            wavfile.write(str(p), 16000, sig[u])
            f.write("%s %s\n" % (u, p))
    out = str(tmp_path / "modspec_c")
    get_feats(get_args([str(scp), out, "--complex_modulation"]))
    ark = read_ark(out + ".ark")
    assert list(ark) == meta["utts"]
    for u in meta["utts"]:
        q = np.round(ref[u], 3).astype(np.float32)
        assert ark[u].shape == q.shape
        assert np.abs(ark[u] - q).max() <= 1.0011e-3 * max(1.0, np.abs(ref[u]).max())
