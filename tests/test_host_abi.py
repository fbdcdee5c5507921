"""CPU-only tests of the C ABI host side (no compute calls): symbol table, RNG replicas, host-only
plan geometry / filterbanks / weights / OLA tables, noise parameters, WAV parser, ark writer and
the CLI's argparse surface against the reference's."""
import argparse
import json
import os
import random
import re
import struct

import numpy as np
import pytest
from scipy.io import wavfile

from conftest import GOLDEN, ROOT, load_golden, oracle_cfg, feature_cfg
from oracle import fdlp_oracle as O


def header_symbols():
    src = open(os.path.join(ROOT, "include", "fdlp.h")).read()
    return sorted(set(re.findall(r"\b(fdlp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from speech_recognition_tools_amd import _lib
    syms = header_symbols()
    assert len(syms) >= 25
    for name in syms:
        assert hasattr(_lib.lib, name), name
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)
    assert _lib.lib.fdlp_abi_version() == 9


@pytest.mark.parametrize("seed", [0, 1, 7, 1234, 2 ** 40 + 5, 2 ** 64 + 3])
def test_pyrandom_matches_cpython_randrange(seed):
    from speech_recognition_tools_amd import PyRandom
    r = random.Random(seed)
    ref = np.array([r.randrange(2) for _ in range(4000)], dtype=np.uint8)
    got = PyRandom(seed).randbits2(4000)
    np.testing.assert_array_equal(got, ref)


def test_pyrandom_stream_continues_across_calls():
    from speech_recognition_tools_amd import PyRandom
    r = random.Random(99)
    ref = [r.randrange(2) for _ in range(300)]
    g = PyRandom(99)
    got = np.concatenate([g.randbits2(n) for n in (3, 0, 100, 197)])
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("seed", [0, 42, 2 ** 32 - 1])
def test_nprandom_matches_numpy_legacy(seed):
    from speech_recognition_tools_amd import NpRandom
    np.testing.assert_array_equal(NpRandom(seed).rand(2000), np.random.RandomState(seed).rand(2000))


def test_unseeded_generators_differ():
    from speech_recognition_tools_amd import NpRandom, PyRandom
    assert not np.array_equal(PyRandom().randbits2(256), PyRandom().randbits2(256))
    assert NpRandom().rand() != NpRandom().rand()


def _host_plan(cfg):
    from speech_recognition_tools_amd import FdlpPlan
    return FdlpPlan(cfg, device=-1)


@pytest.mark.parametrize("name", ["wsj", "reverb", "cli_default_mel", "gamma_lifter_odd"])
def test_host_plan_geometry_matches_oracle(name):
    meta, sig, ref, z = load_golden(name)
    plan = _host_plan(feature_cfg(meta))
    ocfg = oracle_cfg(meta)
    g = O.geometry(ocfg)
    assert (plan.N, plan.hop, plan.kk, plan.ola_hop) == (g.N, g.hop, g.kk, g.ola_hop)
    for T in [2, 100, 7999, 8000, 16000, 17999, 18000, 18001, 18002, 35555, 64000, 72000, 160000, 480000]:
        F, L = plan.geometry(T)
        assert (F, L) == (O.n_frames(T, g), O.n_out(T, ocfg)), T
    for u, x in sig.items():
        F, L = plan.geometry(x.size)
        assert L == ref[u].shape[0]


def test_ola_tables_match_oracle_including_edges():
    from speech_recognition_tools_amd import PyRandom
    for cfg_name in ("wsj", "cli_default_mel"):
        meta, _, _, _ = load_golden(cfg_name)
        plan = _host_plan(feature_cfg(meta))
        ocfg = oracle_cfg(meta)
        g = O.geometry(ocfg)
        rng = PyRandom(5)
        for T in [2, 50, 1000, 8000, 11999, 12001, 16000, 18000, 18002, 36001, 64000, 72000, 160000, 1600000]:
            F, L = plan.geometry(T)
            jit = rng.randbits2(max(F - 1, 0))
            try:
                want = O.ola_plan(F, L, g, [int(v) for v in jit])
            except ValueError:
                # e.g. the CLI default config (fduration 0.5) drifts its OLA pointer by ~0.5-1.5
                # frames per hop, so long utterances overrun feats: the reference raises there too
                with pytest.raises(ValueError):
                    plan.ola_table(T, jit)
                continue
            d, s, c = plan.ola_table(T, jit)
            assert [tuple(v) for v in zip(d.tolist(), s.tolist(), c.tolist())] == want, (cfg_name, T)


def test_ola_table_raises_like_numpy_broadcast():
    # an all-ones jitter stream over a very long utterance pushes the middle frames past the end
    plan = _host_plan(feature_cfg(load_golden("wsj")[0]))
    T = 16000 * 600
    F, L = plan.geometry(T)
    with pytest.raises(ValueError):
        plan.ola_table(T, np.ones(F - 1, dtype=np.uint8))
    g = O.geometry(O.FdlpConfig.wsj())
    with pytest.raises(ValueError):
        O.ola_plan(F, L, g, [1] * (F - 1))


def test_filterbanks_match_reference_fixture():
    from speech_recognition_tools_amd.featgen import features as F
    z = np.load(os.path.join(GOLDEN, "stages_wsj.npz"))
    fb = F.createFbankCochlear(80, 48000, 16000, om_w=1.0, alp=1.0, fixed=1, bet=2.5, warp_fact=1.0)
    np.testing.assert_allclose(fb[[0, 37, 79]], z["fb_rows"], rtol=1e-12, atol=0)
    fbm = F.createFbank(80, 48000, 16000, warp_fact=1.0)
    np.testing.assert_array_equal(fbm, z["fbm"])
    # against the oracle for other shapes / non-fixed alpha
    np.testing.assert_allclose(F.createFbankCochlear(40, 16000, 16000, om_w=0.5, alp=2.0, fixed=0, bet=3.0,
                                                     warp_fact=1.1),
                               O.fbank_cochlear(40, 16000, 16000, 0.5, 2.0, 0, 3.0, 1.1), rtol=1e-12, atol=0)
    np.testing.assert_array_equal(F.createFbank(20, 16000, 16000, 1.0), O.fbank_mel(20, 16000, 16000, 1.0))


@pytest.mark.parametrize("name", ["wsj", "reverb", "chime4_noise", "gamma_lifter_odd"])
def test_modulation_weights_match_oracle(name):
    meta, _, _, _ = load_golden(name)
    plan = _host_plan(feature_cfg(meta))
    np.testing.assert_allclose(plan.weights(), O.modulation_weights(oracle_cfg(meta)), rtol=1e-13, atol=1e-300)


def test_supports_cover_every_tap_above_eps():
    from speech_recognition_tools_amd import FeatureConfig
    for eps in (0.0, 1e-12, 1e-20):
        cfg = FeatureConfig.wsj()
        cfg.support_eps = eps
        fb, lo, hi = _host_plan(cfg).fbank()
        dense = fb[:, :-1]
        for j in range(80):
            keep = dense[j] >= eps * dense[j].max() if eps > 0 else dense[j] != 0
            idx = np.nonzero(keep)[0]
            assert lo[j] == idx[0] and hi[j] == idx[-1] + 1


def test_plan_rejects_what_the_reference_rejects():
    from speech_recognition_tools_amd import FdlpError, FeatureConfig
    with pytest.raises(ValueError, match="Invalid type of filter bank"):
        _host_plan(FeatureConfig(fbank_type="gammatone,1"))
    with pytest.raises(ValueError, match="Cochlear filter bank not configured"):
        _host_plan(FeatureConfig(fbank_type="cochlear,1,1"))
    with pytest.raises(FdlpError, match="gamma_weight"):
        _host_plan(FeatureConfig(order=50, coeff_num=60, coeff_range="0,59", gamma_weight="20,1.5,3"))
    with pytest.raises(FdlpError, match="lifter"):
        _host_plan(FeatureConfig(coeff_num=50, lifter=[1.0] * 49))


def test_noise_params_match_reference_arithmetic():
    from speech_recognition_tools_amd.augment import noise_params
    rng = np.random.default_rng(3)
    sig = (rng.standard_normal(30000) * 4000).astype(np.int16)
    finite = 0
    for scale in (100.0, 9000.0):  # 9000: the int16-wrapped energies go negative -> alpha NaN
        noise = (rng.standard_normal(200000) * scale).astype(np.int16)
        for snr in (20.0, 40.0, -5.0):
            u = rng.random()
            off, alp = noise_params(sig, noise, snr, u)
            off2, alp2 = O.noise_mix_params(sig, noise, snr, u)
            assert off == off2
            np.testing.assert_equal(alp, alp2)
            finite += np.isfinite(alp)
    assert finite >= 3


def test_wav_parser_matches_scipy(tmp_path):
    from speech_recognition_tools_amd.featgen.features import read_wav
    x = (np.random.default_rng(0).standard_normal(12345) * 3000).astype(np.int16)
    p = str(tmp_path / "a.wav")
    wavfile.write(p, 16000, x)
    sr, y = read_wav(p)
    assert sr == 16000 and np.array_equal(y, x)
    # extra chunk before data + odd-sized chunk padding
    raw = open(p, "rb").read()
    fmt_end = raw.index(b"data")
    extra = b"LIST" + struct.pack("<I", 3) + b"abc" + b"\0"
    raw2 = raw[:fmt_end] + extra + raw[fmt_end:]
    raw2 = raw2[:4] + struct.pack("<I", len(raw2) - 8) + raw2[8:]
    open(p, "wb").write(raw2)
    sr, y = read_wav(p)
    assert np.array_equal(y, x)


def test_wav_decoder_matches_scipy_formats(tmp_path):
    """fdlp_wav_decode returns scipy.io.wavfile.read's values for every format scipy reads (the
    reference featurises them unscaled, computeFDLPSpectrogram.py:139,:156-157): 8-bit unsigned, 16/32-bit
    int, 24-bit (left-justified int32), float32/64, WAVE_FORMAT_EXTENSIBLE, big-endian RIFX, stereo."""
    from scipy.io.wavfile import read
    from speech_recognition_tools_amd.featgen.features import read_wav_bytes
    rng = np.random.default_rng(3)
    x = np.clip(rng.standard_normal(777) * 5000, -32768, 32767).astype(np.int16)
    cases = {"u8": (x // 256 + 128).astype(np.uint8), "i32": x.astype(np.int32) * 65537,
             "f32": (x / 32768.0).astype(np.float32), "f64": x / 7.0, "i16": x,
             "stereo": np.stack([x, -x], axis=1)}
    for name, v in cases.items():
        p = str(tmp_path / (name + ".wav"))
        wavfile.write(p, 16000, v)
        raw = open(p, "rb").read()
        sr, got = read_wav_bytes(raw)
        sr2, want = read(p)
        assert sr == sr2 == 16000 and got.shape == want.shape, name
        assert (got.dtype == np.int16) == (want.dtype == np.int16), name
        np.testing.assert_array_equal(got, want.astype(got.dtype), err_msg=name)
    # 24-bit PCM, plain and WAVE_FORMAT_EXTENSIBLE, little- and big-endian
    v = x.astype(np.int32) * 256 + 5
    for ext in (False, True):
        for big in (False, True):
            e = ">" if big else "<"
            raw = b"".join(struct.pack(e + "i", int(s))[1:] if big else struct.pack("<i", int(s))[:3] for s in v)
            if ext:
                tail = (b"\x00\x00\x00\x10" if big else b"\x00\x00\x10\x00") + b"\x80\x00\x00\xAA\x00\x38\x9B\x71"
                fmt = struct.pack(e + "HHIIHHHHII", 0xFFFE, 1, 16000, 48000, 3, 24, 22, 24, 4, 1) + tail
            else:
                fmt = struct.pack(e + "HHIIHH", 1, 1, 16000, 48000, 3, 24)
            body = b"WAVE" + b"fmt " + struct.pack(e + "I", len(fmt)) + fmt + b"data" + struct.pack(e + "I", len(raw)) + raw
            blob = (b"RIFX" if big else b"RIFF") + struct.pack(e + "I", len(body)) + body
            p = str(tmp_path / ("i24_%d_%d.wav" % (ext, big)))
            open(p, "wb").write(blob)
            sr, got = read_wav_bytes(blob)
            sr2, want = read(p)
            assert want.dtype.kind == "i" and want.dtype.itemsize == 4
            np.testing.assert_array_equal(got, want.astype(np.float64))
    # big-endian 16-bit PCM: scipy returns '>i2', i.e. int16 input (noise mixing / diff apply to it)
    fmt = struct.pack(">HHIIHH", 1, 1, 16000, 32000, 2, 16)
    raw = x.astype(">i2").tobytes()
    body = b"WAVE" + b"fmt " + struct.pack(">I", len(fmt)) + fmt + b"data" + struct.pack(">I", len(raw)) + raw
    blob = b"RIFX" + struct.pack(">I", len(body)) + body
    p = str(tmp_path / "i16_be.wav")
    open(p, "wb").write(blob)
    sr, got = read_wav_bytes(blob)
    sr2, want = read(p)
    assert want.dtype.kind == "i" and want.dtype.itemsize == 2 and got.dtype == np.int16
    np.testing.assert_array_equal(got, want)


def test_wav_parser_rejects_garbage():
    from speech_recognition_tools_amd import FdlpError
    from speech_recognition_tools_amd.featgen.features import read_wav_bytes
    with pytest.raises(FdlpError):
        read_wav_bytes(b"not a wav file at all")


def test_ark_writer_roundtrip_and_scp_offsets(tmp_path):
    from speech_recognition_tools_amd.featgen.features import dict2Ark, read_ark
    feats = {"utt1": np.arange(12, dtype=np.float32).reshape(3, 4) - 5.5,
             "u2": np.full((1, 4), -32.236, dtype=np.float32)}
    out = str(tmp_path / "melspec_x.1")
    dict2Ark(feats, out, "copy-feats")
    back = read_ark(out + ".ark")
    assert list(back) == ["utt1", "u2"]
    for k in feats:
        np.testing.assert_array_equal(back[k], feats[k])
    data = open(out + ".ark", "rb").read()
    for line in open(out + ".scp"):
        key, loc = line.split()
        path, off = loc.rsplit(":", 1)
        assert os.path.isabs(path) and os.path.samefile(path, out + ".ark")
        assert data[int(off):int(off) + 2] == b"\0B"
        assert data[int(off) - len(key) - 1:int(off)] == (key + " ").encode()
    assert not any(f.endswith(".tmp") for f in os.listdir(str(tmp_path)))  # written to .tmp, renamed on close


def test_ark_writer_is_atomic(tmp_path):
    """Until fdlp_ark_close the ark/scp exist only as <name>.tmp (a JOB's outputs appear complete or not
    at all), and the scp already names the final ark path."""
    import ctypes
    from speech_recognition_tools_amd._lib import check, lib
    h = ctypes.c_void_p()
    out = str(tmp_path / "j.1")
    check(lib.fdlp_ark_open((out + ".ark").encode(), (out + ".scp").encode(), ctypes.byref(h)))
    m = np.ones((2, 3), dtype=np.float32)
    check(lib.fdlp_ark_write(h, b"u", m.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 2, 3))
    assert sorted(os.listdir(str(tmp_path))) == ["j.1.ark.tmp", "j.1.scp.tmp"]
    check(lib.fdlp_ark_close(h))
    assert sorted(os.listdir(str(tmp_path))) == ["j.1.ark", "j.1.scp"]
    line = open(out + ".scp").read().split()
    assert line[1].rsplit(":", 1)[0] == os.path.realpath(out + ".ark")


def test_ark_writer_abort_publishes_nothing(tmp_path):
    """fdlp_ark_abort (a JOB's failure path) deletes the temporaries: no ark/scp under any name."""
    import ctypes
    from speech_recognition_tools_amd._lib import check, lib
    from speech_recognition_tools_amd.io_pipeline import ArkStream
    h = ctypes.c_void_p()
    out = str(tmp_path / "j.1")
    check(lib.fdlp_ark_open((out + ".ark").encode(), (out + ".scp").encode(), ctypes.byref(h)))
    m = np.ones((2, 3), dtype=np.float32)
    check(lib.fdlp_ark_write(h, b"u", m.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 2, 3))
    check(lib.fdlp_ark_abort(h))
    assert os.listdir(str(tmp_path)) == []
    with pytest.raises(RuntimeError):
        with ArkStream(out) as ark:
            ark.write("u", m)
            raise RuntimeError("JOB failed")
    assert os.listdir(str(tmp_path)) == []


def test_cli_argparse_surface_matches_reference():
    from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import build_parser
    ref = json.load(open(os.path.join(GOLDEN, "cli_options.json")))
    ours = {a.option_strings[0] if a.option_strings else a.dest: a for a in build_parser()._actions}
    for o in ref:
        a = ours[o["name"]]
        if "default" in o:
            assert a.default == o["default"], o
        if "type" in o:
            assert a.type.__name__ == o["type"], o
        if o.get("action") == "store_true":
            assert isinstance(a, argparse._StoreTrueAction), o
    # the driver's "--opt=value" forms parse identically
    args = build_parser().parse_args(["a.scp", "out", "--fbank_type=cochlear,1,1,1,2.5,1", "--nfilters=80",
                                      "--coeff_range=0,100", "--order=150", "--add_noise=clean"])
    assert args.nfilters == 80 and args.fbank_type.startswith("cochlear") and args.order == 150


def test_autocorr_path_selection():
    from speech_recognition_tools_amd import FdlpError, FeatureConfig
    p = _host_plan(FeatureConfig.wsj())
    assert p.autocorr_path == "structured"
    p.set_autocorr_path("direct")
    assert p.autocorr_path == "direct"
    p.set_autocorr_path("auto")
    assert p.autocorr_path == "structured"
    for cfg in (FeatureConfig(), FeatureConfig(fbank_type="cochlear,1,1,0,2.5,1"),   # mel; alpha not fixed
                FeatureConfig(fbank_type="cochlear,1,9,1,2.5,1")):                    # skirt exponents too wide
        q = _host_plan(cfg)
        assert q.autocorr_path == "direct"
        with pytest.raises(FdlpError, match="structured"):
            q.set_autocorr_path("structured")


@pytest.mark.parametrize("fb", ["cochlear,1,1,1,2.5,1", "cochlear,0.5,2.5,1,1.5,1", "cochlear,2,0.5,1,4,1.2"])
def test_structured_regions_match_filterbank_branches(fb):
    """m1/m2 split every band exactly where createFbankCochlear (features.py:212-217) switches
    branch: d <= -om/2 (lower skirt), -om/2 < d < om/2 (flat top), else upper skirt."""
    from speech_recognition_tools_amd import FeatureConfig
    cfg = FeatureConfig(fbank_type=fb, nfilters=40, fduration=1.5, order=60, coeff_num=60, coeff_range="0,60")
    plan = _host_plan(cfg)
    m1, m2 = plan.regions()
    _, om, alp, fixed, bet, wf = fb.split(",")
    om, wf = float(om), float(wf)
    bark = lambda f: 6 * np.arcsinh((f / wf) / 600)
    fw = bark(np.linspace(0, 8000, plan.N + 1))[:plan.N]
    for j, fc in enumerate(np.linspace(0, bark(8000), 40)):
        d = fw - fc
        lo = d <= -om / 2
        mid = (~lo) & (d < om / 2)
        assert m1[j] == lo.sum() and lo[:m1[j]].all()
        assert m2[j] == m1[j] + mid.sum() and mid[m1[j]:m2[j]].all()
    with pytest.raises(Exception):
        _host_plan(FeatureConfig()).regions()


def test_torch_op_is_registered():
    """torch.ops.fdlp.spectrogram (speech_recognition_tools_amd.ops) wraps fdlp_compute on tensors."""
    import torch
    import speech_recognition_tools_amd  # noqa: F401
    schema = str(torch.ops.fdlp.spectrogram.default._schema)
    assert schema.startswith("fdlp::spectrogram(") and "Tensor pcm" in schema and schema.endswith("-> Tensor")
