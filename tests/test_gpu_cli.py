"""End-to-end CLI (compute-fdlp-feats == computeFDLPSpectrogram.py argv) on the GPU: WAV files
and pipes in, Kaldi ark/scp/len out, compared with the reference's golden features after the
reference's own '%.3f' text-ark rounding (one 0.001 step allowed at rounding boundaries)."""
import os

import numpy as np
import pytest
from scipy.io import wavfile

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _args(extra):
    from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import build_parser
    return build_parser().parse_args(extra)


def _run(extra, runner):
    """The CLI's getFeats (no feature dict returned) through the native JOB runner (fdlp_job_run) or the
    Python loop."""
    from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import getFeats
    getFeats(_args(extra + ["--host_runner=" + runner]), return_feats=False)


RUNNERS = pytest.mark.parametrize("runner", ["native", "python"])


def _write_scp(tmp, sig, utts, pipe=()):
    scp = os.path.join(tmp, "wav.scp")
    with open(scp, "w") as f:
        for u in utts:
            p = os.path.join(tmp, u + ".wav")
            wavfile.write(p, 16000, sig[u])
            f.write("%s cat %s |\n" % (u, p) if u in pipe else "%s %s\n" % (u, p))
    return scp


def _opts(meta):
    o = meta["opts"]
    return ["--nfilters=%d" % o["nfilters"], "--coeff_num=%d" % o["coeff_num"], "--coeff_range=" + o["coeff_range"],
            "--order=%d" % o["order"], "--fduration=%s" % o["fduration"], "--frate=%d" % o["frate"],
            "--overlap_fraction=%s" % o["overlap_fraction"], "--fbank_type=" + o["fbank_type"],
            "--seed=%d" % meta["seed"], "--write_utt2num_frames"]


def _check(out, meta, ref, utts):
    from speech_recognition_tools_amd.featgen.features import read_ark
    ark = read_ark(out + ".ark")
    assert list(ark) == list(utts)
    lens = dict(l.split() for l in open(out + ".len"))
    for u in utts:
        q = np.round(ref[u], 3).astype(np.float32)
        assert ark[u].shape == q.shape
        tol = 2.1e-3 if u == "short2" else 1.0011e-3
        assert np.abs(ark[u] - q).max() <= tol, u
        assert int(lens[u]) == q.shape[0]
    for line in open(out + ".scp"):
        assert line.split()[0] in utts


def test_cli_wsj_files_and_pipes_return_feats(tmp_path):
    """getFeats returning the feature dict (the Python loop) equals the ark it writes."""
    from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import getFeats
    from speech_recognition_tools_amd.featgen.features import read_ark
    meta, sig, ref, z = load_golden("wsj")
    utts = meta["utts"]
    scp = _write_scp(str(tmp_path), sig, utts, pipe=("s4p0", "white10"))
    out = str(tmp_path / "melspec_test.1")
    feats = getFeats(_args([scp, out] + _opts(meta) + ["--batch_frames=16"]))
    _check(out, meta, ref, utts)
    ark = read_ark(out + ".ark")
    for u in utts:
        np.testing.assert_array_equal(feats[u], ark[u])


@RUNNERS
def test_cli_wsj_files_and_pipes(tmp_path, runner):
    meta, sig, ref, z = load_golden("wsj")
    utts = meta["utts"]
    scp = _write_scp(str(tmp_path), sig, utts, pipe=("s4p0", "white10"))
    out = str(tmp_path / "melspec_test.1")
    _run([scp, out] + _opts(meta) + ["--batch_frames=16"], runner)
    _check(out, meta, ref, utts)
    assert not any(f.endswith(".tmp") for f in os.listdir(str(tmp_path)))  # renamed when complete


@RUNNERS
def test_cli_skips_unreadable_utterances(tmp_path, runner, capfd):
    meta, sig, ref, z = load_golden("reverb")
    utts = meta["utts"]
    scp = _write_scp(str(tmp_path), sig, utts)
    with open(scp, "a") as f:
        f.write("missing_utt %s\n" % str(tmp_path / "nope.wav"))
        f.write("garbage_utt %s\n" % scp)  # not a WAV
    out = str(tmp_path / "o")
    _run([scp, out] + _opts(meta), runner)
    _check(out, meta, ref, utts)
    assert "skipped 2 of %d utterances" % (len(utts) + 2) in capfd.readouterr().out
    # a failing FIRST utterance leaves the reference's `sr` undefined -> NameError (:144)
    bad = str(tmp_path / "bad.scp")
    with open(bad, "w") as f:
        f.write("missing_utt %s\n" % str(tmp_path / "nope.wav"))
    with pytest.raises(NameError):
        _run([bad, out] + _opts(meta), runner)
    # every entry of a segment scp unreadable: the JOB fails (the reference would write nothing)
    with pytest.raises(RuntimeError, match="every utterance"):
        _run([bad, str(tmp_path / "seg")] + _opts(meta) + ["--scp_type=segment"], runner)


@RUNNERS
def test_cli_rejects_other_sample_rates(tmp_path, runner):
    p = str(tmp_path / "a.wav")
    wavfile.write(p, 8000, np.zeros(16000, dtype=np.int16))
    scp = str(tmp_path / "w.scp")
    open(scp, "w").write("u %s\n" % p)
    with pytest.raises(AssertionError, match="different sampling rate"):
        _run([scp, str(tmp_path / "o")], runner)


@RUNNERS
def test_cli_failure_leaves_no_partial_outputs(tmp_path, runner):
    """An scp whose second entry is 8 kHz fails the JOB after the first utterance was featurised: the
    reference raises before dict2Ark and writes nothing, so no .ark / .scp may appear (not even the
    first utterance's), and no .tmp is left behind."""
    a, b = str(tmp_path / "a.wav"), str(tmp_path / "b.wav")
    wavfile.write(a, 16000, (np.random.default_rng(0).standard_normal(40000) * 1000).astype(np.int16))
    wavfile.write(b, 8000, np.zeros(16000, dtype=np.int16))
    scp = str(tmp_path / "w.scp")
    open(scp, "w").write("u1 %s\nu2 %s\n" % (a, b))
    with pytest.raises(AssertionError, match="different sampling rate"):
        _run([scp, str(tmp_path / "o"), "--write_utt2num_frames"], runner)
    left = sorted(f for f in os.listdir(str(tmp_path)) if f.startswith("o"))
    assert left == [], left


def _write_formats(tmp, x):
    """The int16 signal x in the WAV formats scipy reads, and the values scipy returns for each."""
    import struct
    files = {}
    p = os.path.join(tmp, "f32.wav")
    wavfile.write(p, 16000, (x / 32768.0).astype(np.float32))
    files["f32"] = p
    p = os.path.join(tmp, "f64.wav")
    wavfile.write(p, 16000, x.astype(np.float64) * 0.5)
    files["f64"] = p
    p = os.path.join(tmp, "i32.wav")
    wavfile.write(p, 16000, x.astype(np.int32) * 65536)
    files["i32"] = p
    p = os.path.join(tmp, "u8.wav")
    wavfile.write(p, 16000, (x // 256 + 128).astype(np.uint8))
    files["u8"] = p
    # 24-bit PCM (scipy returns it left-justified in int32)
    v = x.astype(np.int32) * 256 + 17
    raw = b"".join(struct.pack("<i", int(s))[:3] for s in v)
    hdr = (b"RIFF" + struct.pack("<I", 36 + len(raw)) + b"WAVEfmt " + struct.pack("<IHHIIHH", 16, 1, 1, 16000,
           16000 * 3, 3, 24) + b"data" + struct.pack("<I", len(raw)))
    p = os.path.join(tmp, "i24.wav")
    open(p, "wb").write(hdr + raw)
    files["i24"] = p
    return files


@RUNNERS
def test_cli_scipy_wav_formats(tmp_path, runner):
    """Every format scipy.io.wavfile.read returns (the reference featurises its values as they are, no
    scaling, :156-157) gives the oracle's features of scipy's values; int16 and other-format utterances
    in one scp go to separate device batches."""
    import random
    from scipy.io.wavfile import read
    from oracle import fdlp_oracle as O
    from speech_recognition_tools_amd.featgen.features import read_ark
    rng = np.random.default_rng(11)
    x = np.clip(rng.standard_normal(30000) * 3000, -32768, 32767).astype(np.int16)
    files = _write_formats(str(tmp_path), x)
    p16 = str(tmp_path / "i16.wav")
    wavfile.write(p16, 16000, x)
    order = ["f32", "i16", "i24", "u8", "f64", "i32"]
    files["i16"] = p16
    scp = str(tmp_path / "w.scp")
    with open(scp, "w") as f:
        for k in order:
            f.write("%s %s\n" % (k, files[k]))
    out = str(tmp_path / "fmt")
    cfg = O.FdlpConfig.wsj()
    opts = ["--nfilters=80", "--coeff_num=100", "--coeff_range=0,100", "--order=150", "--fduration=1.5",
            "--frate=100", "--overlap_fraction=0.25", "--fbank_type=cochlear,1,1,1,2.5,1", "--seed=4",
            "--ark_precision=-1"]
    _run([scp, out] + opts, runner)
    ark = read_ark(out + ".ark")
    assert list(ark) == order
    orc = O.FdlpOracle(cfg)
    r = random.Random(4)
    for k in order:
        sr, v = read(files[k])
        want = orc.utterance(v.astype(np.float64) if v.dtype != np.int16 else v, r)
        assert np.abs(ark[k] - want.astype(np.float32)).max() <= 1e-4 * max(1.0, np.abs(want).max()), k


def test_native_and_python_runners_write_identical_arks(tmp_path):
    """Same scp (files, a pipe, an unreadable entry, a long utterance that outgrows the batch) through
    both host runners: byte-identical .ark / .len and identical scp keys and offsets."""
    meta, sig, ref, z = load_golden("wsj")
    utts = meta["utts"]
    scp = _write_scp(str(tmp_path), sig, utts, pipe=("s4p0",))
    with open(scp, "a") as f:
        f.write("missing_utt %s\n" % str(tmp_path / "nope.wav"))
    outs = {}
    for runner in ("native", "python"):
        out = str(tmp_path / runner)
        _run([scp, out] + _opts(meta) + ["--batch_frames=8"], runner)
        outs[runner] = out
    a, b = outs["native"], outs["python"]
    assert open(a + ".ark", "rb").read() == open(b + ".ark", "rb").read()
    assert open(a + ".len").read() == open(b + ".len").read()
    ka = [(l.split()[0], l.split()[1].rsplit(":", 1)[1]) for l in open(a + ".scp")]
    kb = [(l.split()[0], l.split()[1].rsplit(":", 1)[1]) for l in open(b + ".scp")]
    assert ka == kb


def test_native_runner_batch_ramp_matches_python(tmp_path):
    """300 utterances of 1-6 s through 1024-frame batches: the native runner's ramp (64, 128, ..., 1024
    frames) and its three-slot rotation write the same bytes as the Python loop."""
    meta, _, _, _ = load_golden("wsj")
    rng = np.random.default_rng(11)
    utts = ["r%04d" % i for i in range(300)]
    sig = {u: np.clip(rng.standard_normal(int(rng.integers(16000, 96000))) * 2000, -32768, 32767).astype(np.int16)
           for u in utts}
    scp = _write_scp(str(tmp_path), sig, utts)
    outs = {}
    for runner in ("native", "python"):
        out = str(tmp_path / runner)
        _run([scp, out] + _opts(meta) + ["--batch_frames=1024"], runner)
        outs[runner] = out
    a, b = outs["native"], outs["python"]
    assert open(a + ".ark", "rb").read() == open(b + ".ark", "rb").read()
    assert open(a + ".len").read() == open(b + ".len").read()
    assert len(open(a + ".len").read().split("\n")) == 301


def test_native_runner_d2h_legs_write_identical_arks(tmp_path):
    """The native runner's device-to-host leg in every form writes the Python loop's bytes: float32 rows,
    int16 ark codes widened on the host (in one piece and in many small pieces), codes that overflow
    (--ark_precision 4 leaves most log values outside int16: every batch is copied again as float32),
    the mapped-output path, and a second call that reuses the first one's plan and pinned slots."""
    from speech_recognition_tools_amd.featgen import computeFDLPSpectrogram as cli
    meta, _, _, _ = load_golden("wsj")
    rng = np.random.default_rng(5)
    utts = ["d%04d" % i for i in range(90)]
    sig = {u: np.clip(rng.standard_normal(int(rng.integers(16000, 80000))) * 3000, -32768, 32767).astype(np.int16)
           for u in utts}
    scp = _write_scp(str(tmp_path), sig, utts)
    base = [scp] + _opts(meta) + ["--batch_frames=256"]

    def run(name, extra, runner="native"):
        out = str(tmp_path / name)
        _run([base[0], out] + base[1:] + extra, runner)
        return (open(out + ".ark", "rb").read(), open(out + ".len").read(),
                [(l.split()[0], l.split()[1].rsplit(":", 1)[1]) for l in open(out + ".scp")])

    for prec in (3, 4):
        want = run("py%d" % prec, ["--ark_precision=%d" % prec], "python")
        cases = {"off": ["--d2h_codes=off"], "on": ["--d2h_codes=on"],
                 "on_pieces": ["--d2h_codes=on", "--chunk_rows=300"], "mapped": ["--mapped_output"]}
        for name, extra in cases.items():
            got = run("n%d_%s" % (prec, name), ["--ark_precision=%d" % prec] + extra)
            assert got == want, (prec, name)
            st = cli.LAST_JOB_STATS
            assert st["codes"] == (1 if name.startswith("on") else 0), (prec, name)
            if name == "on_pieces":
                assert st["n_batches"] >= 3
            if name.startswith("on"):
                fb = st["n_code_fallbacks"]
                assert (fb >= 1) if prec == 4 else fb == 0, (prec, name, fb, st["n_batches"])
    # keep_warm: the second call takes the parked plan and slots and writes the same bytes
    trace = str(tmp_path / "trace.jsonl")
    a = run("w1", ["--keep_warm"])
    assert cli.LAST_JOB_STATS["warm"] == 0
    b = run("w2", ["--keep_warm", "--job_trace=" + trace])
    assert cli.LAST_JOB_STATS["warm"] == 1 and a == b
    from speech_recognition_tools_amd import _lib
    _lib.lib.fdlp_job_release()
    import json
    ev = [json.loads(l)["ev"] for l in open(trace)]
    for e in ("plan", "setup", "flush", "launched", "landed", "widened", "written", "end"):
        assert e in ev, e


@RUNNERS
def test_cli_diff_and_noise(tmp_path, monkeypatch, runner):
    meta, sig, ref, z = load_golden("wsj_diff")
    scp = _write_scp(str(tmp_path), sig, meta["utts"])
    out = str(tmp_path / "d")
    _run([scp, out] + _opts(meta) + ["--add_noise=diff"], runner)
    _check(out, meta, ref, meta["utts"])

    meta, sig, ref, z = load_golden("chime4_noise")
    d = tmp_path / "n"
    d.mkdir()
    (d / "noises").mkdir()
    wavfile.write(str(d / "noises" / "babble.wav"), 16000, z["noise_babble"])
    scp = _write_scp(str(d), sig, meta["utts"])
    monkeypatch.chdir(str(d))
    out = str(d / "nz")
    _run([scp, out] + _opts(meta) + ["--add_noise=babble,20", "--noise_seed=%d" % meta["extra"]["noise_seed"]],
         runner)
    _check(out, meta, ref, meta["utts"])


def test_driver_script_two_jobs(tmp_path):
    """scripts/make_FDLPspectrum_feats.sh (the Kaldi-style driver) splits wav.scp into JOBs and
    concatenates feats.scp / utt2num_frames in JOB order."""
    import subprocess
    import sys
    from conftest import ROOT
    from speech_recognition_tools_amd.featgen.features import read_ark
    meta, sig, ref, z = load_golden("reverb")
    data = tmp_path / "data" / "test_set"
    data.mkdir(parents=True)
    _write_scp(str(data), sig, meta["utts"])
    os.rename(str(data / "wav.scp"), str(data / "wav.scp"))
    o = meta["opts"]
    cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", "2", "--ngpu", "1",
           "--nfilters", str(o["nfilters"]), "--order", str(o["order"]), "--fduration", str(o["fduration"]),
           "--frate", str(o["frate"]), "--coeff_range", o["coeff_range"], "--coeff_num", str(o["coeff_num"]),
           "--overlap_fraction", str(o["overlap_fraction"]), "--fbank_type", o["fbank_type"],
           "--write_utt2num_frames", "true", "--compute_cmvn", "true", str(data), str(tmp_path / "fbank")]
    r = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    feats = [l.split() for l in open(str(data / "feats.scp"))]
    assert [f[0] for f in feats] == meta["utts"]
    lens = dict(l.split() for l in open(str(data / "utt2num_frames")))
    for u in meta["utts"]:
        assert int(lens[u]) == ref[u].shape[0]
    arks = {}
    for n in (1, 2):
        arks.update(read_ark(str(tmp_path / "fbank" / ("melspec_test_set.%d.ark" % n))))
    for u in meta["utts"]:
        assert arks[u].shape == ref[u].shape
    # fused global CMVN: the JOB stats summed into data_dir/cmvn.ark == Kaldi semantics over the arks
    from oracle import cmvn_oracle as CO
    from speech_recognition_tools_amd.cmvn import read_kaldi_dmatrix
    got = read_kaldi_dmatrix(str(data / "cmvn.ark"))
    want = CO.global_stats(arks[u] for u in meta["utts"])
    assert got[0, -1] == want[0, -1]
    assert np.max(np.abs(got - want) / np.maximum(np.abs(want), 1.0)) <= 1e-12


def test_driver_chained_jobs_write_cold_jobs_bytes(tmp_path):
    """The driver's warm JOB chains (--chain_jobs true: 5 JOBs in 2 processes, a plan and slots reused and
    the jitter generator re-seeded per JOB) write every JOB's .ark / .len and the data dir's feats.scp /
    utt2num_frames byte for byte as one cold process per JOB does (--chain_jobs false).  --seed is given:
    unseeded, the OLA jitter draws from OS entropy per JOB, as the reference's random module does, and
    two runs of either mode differ (benchmarks/job_determinism.py, profiles/r06x_job_determinism.jsonl)."""
    import subprocess
    from conftest import ROOT
    meta, _, _, _ = load_golden("wsj")
    rng = np.random.default_rng(23)
    utts = ["c%03d" % i for i in range(25)]
    sig = {u: np.clip(rng.standard_normal(int(rng.integers(16000, 64000))) * 2500, -32768, 32767).astype(np.int16)
           for u in utts}
    o = meta["opts"]
    got = {}
    for chain in ("true", "false"):
        data = tmp_path / chain / "data"
        data.mkdir(parents=True)
        _write_scp(str(data), sig, utts)
        fb = tmp_path / chain / "fbank"
        cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", "5", "--ngpu", "1",
               "--jobs_per_gpu", "2", "--chain_jobs", chain, "--seed", "7", "--nfilters", str(o["nfilters"]),
               "--order", str(o["order"]), "--fduration", str(o["fduration"]), "--frate", str(o["frate"]),
               "--coeff_range", o["coeff_range"], "--coeff_num", str(o["coeff_num"]),
               "--overlap_fraction", str(o["overlap_fraction"]), "--fbank_type", o["fbank_type"],
               "--write_utt2num_frames", "true", str(data), str(fb)]
        r = subprocess.run(cmd, cwd=str(tmp_path / chain), capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout + r.stderr
        files = {}
        for n in range(1, 6):
            for ext in (".ark", ".len"):
                p = fb / ("melspec_data.%d%s" % (n, ext))
                files[p.name] = p.read_bytes()
        feats = [l.split() for l in open(str(data / "feats.scp"))]
        files["feats.scp"] = [(k, v.rsplit("/", 1)[1]) for k, v in feats]  # paths differ by the run dir
        files["utt2num_frames"] = (data / "utt2num_frames").read_text()
        got[chain] = files
    assert [k for k, _ in got["true"]["feats.scp"]] == utts
    assert got["true"].keys() == got["false"].keys()
    for k in got["true"]:
        assert got["true"][k] == got["false"][k], k


@pytest.mark.parametrize("name", ["reverb_rir", "reverb_rir_noise"])
def test_cli_add_reverb(tmp_path, monkeypatch, name):
    """--add_reverb small_room reads ./RIR/RIR_SmallRoom1_near_AnglA.wav (channel 1 / 2^15) and
    convolves + re-aligns on the device (after the noise mixing when both are given)."""
    from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import getFeats
    meta, sig, ref, z = load_golden(name)
    d = tmp_path / "r"
    (d / "RIR").mkdir(parents=True)
    wavfile.write(str(d / "RIR" / "RIR_SmallRoom1_near_AnglA.wav"), 16000, z["rir"])
    extra = ["--add_reverb=small_room"]
    if "noise_babble" in z.files:
        (d / "noises").mkdir()
        wavfile.write(str(d / "noises" / "babble.wav"), 16000, z["noise_babble"])
        extra += ["--add_noise=" + meta["opts"]["add_noise"], "--noise_seed=%d" % meta["extra"]["noise_seed"]]
    scp = _write_scp(str(d), sig, meta["utts"])
    monkeypatch.chdir(str(d))
    out = str(d / "rv")
    getFeats(_args([scp, out] + _opts(meta) + extra))
    _check(out, meta, ref, meta["utts"])


@RUNNERS
@pytest.mark.parametrize("name", ["wav_kinds_noise", "wav_kinds_diff"])
def test_cli_noise_and_diff_on_other_wav_formats(tmp_path, monkeypatch, runner, name):
    """--add_noise babble,20 and --add_noise diff on float32, 24-bit, 32-bit and 8-bit WAVs
    (the reference mixes / convolves whatever dtype scipy.io.wavfile.read returns, features.py:24-31,
    computeFDLPSpectrogram.py:160-166), the WAV files themselves as the reference read them, against the
    reference's features (tests/golden/make_golden.py wav_kinds_fixtures)."""
    meta, sig, ref, z = load_golden(name)
    (tmp_path / "noises").mkdir()
    if "noise_babble" in z.files:
        wavfile.write(str(tmp_path / "noises" / "babble.wav"), 16000, z["noise_babble"])
    scp = str(tmp_path / "wav.scp")
    with open(scp, "w") as f:
        for u in meta["utts"]:
            p = tmp_path / (u + ".wav")
            p.write_bytes(z["wav_" + u].tobytes())
            f.write("%s %s\n" % (u, p))
    monkeypatch.chdir(str(tmp_path))
    out = str(tmp_path / "k")
    extra = ["--add_noise=" + meta["opts"]["add_noise"]]
    if "noise_seed" in meta["extra"]:
        extra.append("--noise_seed=%d" % meta["extra"]["noise_seed"])
    _run([scp, out] + _opts(meta) + extra, runner)
    _check(out, meta, ref, meta["utts"])
