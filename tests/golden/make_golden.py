"""Generate the golden fixtures by running the REAL reference in the build container.

Run once, here (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports ``src/featgen/computeFDLPSpectrogram.py`` / ``features.py`` from the read-only
reference tree, replaces ``dict2Ark`` (Kaldi ``copy-feats`` is absent here, and the real
writer would silently write nothing: features.py:63-69) with a capture of the fp64 feature
dict, seeds ``random`` (jitter, computeFDLPSpectrogram.py:225) and ``np.random`` (noise
offset, features.py:25) right before each ``getFeats`` call, and stores inputs + outputs as
small ``.npz`` fixtures next to this script.  Only data is stored (int16 inputs, fp64
outputs, seeds, versions); no reference source.

Inputs: seeded synthetic speech-like signals (AR(2)-coloured noise x syllabic envelope),
white noise, edge lengths from SURVEY.md Appendix B, and two PESQ conformance clips shipped
in the reference (e2e/reverb/local/PESQ_sources/P862/Software/Conform/*.wav, 8 kHz) upsampled
2x to 16 kHz with scipy.signal.resample_poly and cropped.
"""
import argparse
import json
import os
import random
import sys
import tempfile
from collections import OrderedDict

import numpy as np
import scipy
from scipy.io import wavfile
from scipy.signal import lfilter, resample_poly

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
PESQ_DIR = os.path.join(REF, "e2e/reverb/local/PESQ_sources/P862/Software/Conform")


def speech_like(T, seed, rms=2000.0):
    rng = np.random.default_rng(seed)
    e = rng.standard_normal(T + 400)
    # AR(2) resonance around 500-1500 Hz, random per utterance
    f0 = rng.uniform(400, 1500)
    rad = rng.uniform(0.90, 0.98)
    a1, a2 = -2 * rad * np.cos(2 * np.pi * f0 / 16000), rad * rad
    x = lfilter([1.0], [1.0, a1, a2], e)[400:]
    t = np.arange(T) / 16000
    env = 0.55 + 0.45 * np.sin(2 * np.pi * rng.uniform(3, 5) * t + rng.uniform(0, 6.28))
    x = x * env
    x = x / (np.sqrt(np.mean(x ** 2)) + 1e-12) * rms
    return np.clip(np.round(x), -32768, 32767).astype(np.int16)


def white(T, seed, scale=3000.0):
    x = np.random.default_rng(seed).standard_normal(T) * scale
    return np.clip(np.round(x), -32768, 32767).astype(np.int16)


def pesq_clip(name, seconds):
    sr, x = wavfile.read(os.path.join(PESQ_DIR, name))
    assert sr == 8000
    y = resample_poly(x.astype(np.float64), 2, 1)
    y = np.clip(np.round(y), -32768, 32767).astype(np.int16)
    return y[: int(seconds * 16000)]


def synthetic_rir(R, seed, t60=0.25):
    """Stereo int16 RIR: a direct path + exponentially decaying noise tail (channel 1 is the one used)."""
    rng = np.random.default_rng(seed)
    t = np.arange(R) / 16000.0
    h = rng.standard_normal((R, 2)) * np.exp(-6.9 * t / t60)[:, None] * 0.3
    h[0] = [0.9, 0.8]
    h[37] += [0.4, -0.35]
    return np.clip(np.round(h * 32767), -32768, 32767).astype(np.int16)


def wav24_bytes(v, sr=16000):
    """A mono 24-bit PCM RIFF file of the int32 values v (|v| < 2**23): scipy.io.wavfile.write has no 24-bit
    writer; scipy reads it back as int32 v << 8 (left-justified)."""
    import struct
    v = np.asarray(v, dtype=np.int64)
    data = bytearray()
    for x in v:
        data += int(x & 0xFFFFFF).to_bytes(3, "little")
    fmt = struct.pack("<HHIIHH", 1, 1, sr, sr * 3, 3, 24)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(data)) + bytes(data)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def run_reference(signals, opts, seed, noise_seed=None, noise=None, noise_name=None, rir=None, raw=None):
    """Write WAVs + scp, call getFeats with an argparse Namespace, capture the dict.  raw: {utt: file bytes}
    written as they are instead of wavfile.write(signals[utt])."""
    sys.path.insert(0, os.path.join(REF, "src/featgen"))
    import computeFDLPSpectrogram as cf  # noqa: E402

    captured = {}

    def capture(feat_dict, outfile, kaldi_cmd):
        captured.update({k: np.array(v) for k, v in feat_dict.items()})

    cf.dict2Ark = capture
    with tempfile.TemporaryDirectory() as td:
        scp = os.path.join(td, "wav.scp")
        with open(scp, "w") as f:
            for utt, x in signals.items():
                p = os.path.join(td, utt + ".wav")
                if raw and utt in raw:
                    with open(p, "wb") as fw:
                        fw.write(raw[utt])
                else:
                    wavfile.write(p, 16000, x)
                f.write("%s %s\n" % (utt, p))
        cwd = os.getcwd()
        if noise is not None:
            os.makedirs(os.path.join(td, "noises"), exist_ok=True)
            wavfile.write(os.path.join(td, "noises", noise_name + ".wav"), 16000, noise)
        if rir is not None:  # computeFDLPSpectrogram.py:76: ./RIR/RIR_SmallRoom1_near_AnglA.wav
            os.makedirs(os.path.join(td, "RIR"), exist_ok=True)
            wavfile.write(os.path.join(td, "RIR", "RIR_SmallRoom1_near_AnglA.wav"), 16000, rir)
        os.chdir(td)
        try:
            ns = argparse.Namespace(
                scp=scp, outfile=os.path.join(td, "out"), scp_type="wav",
                nfilters=opts["nfilters"], coeff_num=opts["coeff_num"],
                coeff_range=opts["coeff_range"], order=opts["order"],
                fduration=opts["fduration"], frate=opts["frate"],
                overlap_fraction=opts["overlap_fraction"], kaldi_cmd="true",
                add_reverb=opts.get("add_reverb", "clean"), fbank_type=opts["fbank_type"],
                odd_mod_zero=opts.get("odd_mod_zero", False),
                gamma_weight=opts.get("gamma_weight", "None"),
                lifter_config=opts.get("lifter_config"),
                write_utt2num_frames=True, add_noise=opts.get("add_noise", "clean"))
            random.seed(seed)
            if noise_seed is not None:
                np.random.seed(noise_seed)
            cf.getFeats(ns)
        finally:
            os.chdir(cwd)
    return captured


WSJ = dict(nfilters=80, coeff_num=100, coeff_range="0,100", order=150, fduration=1.5,
           frate=100, overlap_fraction=0.25, fbank_type="cochlear,1,1,1,2.5,1")
REVERB = dict(WSJ, coeff_num=450, coeff_range="1,450")
CHIME4 = dict(WSJ, coeff_range="1,100")
CLI_DEFAULT = dict(nfilters=20, coeff_num=50, coeff_range="1,20", order=50, fduration=0.5,
                   frate=100, overlap_fraction=0.25, fbank_type="mel,1")
MEL80 = dict(WSJ, fbank_type="mel,1")


def save(name, signals, opts, seed, feats, extra=None, more=None):
    arrays = dict(more or {})
    meta = dict(opts=opts, seed=seed, utts=list(signals.keys()),
                numpy=np.__version__, scipy=scipy.__version__,
                python=sys.version.split()[0], extra=extra or {})
    for utt, x in signals.items():
        arrays["in_" + utt] = x
        arrays["out_" + utt] = feats[utt]
    arrays["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, sum(v.nbytes for v in arrays.values()) // 1024, "KiB raw")


def stage_fixture():
    """Per-stage intermediates for one frame x 3 bands (WSJ cfg), via reference primitives."""
    sys.path.insert(0, os.path.join(REF, "src/featgen"))
    import features as fe  # noqa: E402
    import scipy.fftpack as fp
    x = speech_like(30000, 11)
    fr = np.array([f for f in fe.getFrames(x, 16000, 1 / (0.75 * 1.5), 1.5, np.hamming)])
    dct = fp.dct(fr) / np.sqrt(2 * 24000)
    fb = fe.createFbankCochlear(80, 48000, 16000, om_w=1.0, alp=1.0, fixed=1, bet=2.5, warp_fact=1.0)
    fbm = fe.createFbank(80, 48000, 16000, warp_fact=1.0)
    out = dict(x=x, frames0=fr[0], dct=dct, fb_rows=fb[[0, 37, 79]], fbm=fbm)
    for tag, j in (("b0", 0), ("b37", 37), ("b79", 79)):
        band = fb[j, :-1] * dct[1]
        y = np.real(np.fft.ifft(np.fft.fft(band) * np.conj(np.fft.fft(band))))
        a, gg = fe.computeLpcFast(band.copy(), 150)
        cep100 = fe.computeModSpecFromLpc(gg, a.copy(), 100)
        cep450 = fe.computeModSpecFromLpc(gg, a.copy(), 450)
        out.update({tag + "_r": y[:152], tag + "_a": a, tag + "_gg": np.array(gg),
                    tag + "_c100": cep100, tag + "_c450": cep450})
    path = os.path.join(HERE, "stages_wsj.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


def cli_options_fixture():
    """The reference's argparse table (computeFDLPSpectrogram.py:240-261), read from its source
    text with ast (names, defaults, types, actions) -> cli_options.json."""
    import ast
    src = open(os.path.join(REF, "src/featgen/computeFDLPSpectrogram.py")).read()
    opts = []
    for node in ast.walk(ast.parse(src)):
        if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "add_argument":
            name = ast.literal_eval(node.args[0])
            kw = {}
            for k in node.keywords:
                if k.arg in ("default", "action"):
                    kw[k.arg] = ast.literal_eval(k.value)
                elif k.arg == "type":
                    kw["type"] = k.value.id
            opts.append(dict(name=name, **kw))
    with open(os.path.join(HERE, "cli_options.json"), "w") as f:
        json.dump(opts, f, indent=1)
    print("wrote cli_options.json", len(opts))


def run_reference_mel(signals, opts, noise_seed=None, noise=None, noise_name=None, rir=None):
    """computeMelSpectrum.compute_mel_spectrum with get_kaldi_ark captured (copy-feats is absent)."""
    sys.path.insert(0, os.path.join(REF, "src/featgen"))
    import computeMelSpectrum as cm  # noqa: E402
    captured = {}
    cm.get_kaldi_ark = lambda feat_dict, outfile, kaldi_cmd='copy-feats': captured.update(
        {k: np.array(v) for k, v in feat_dict.items()})
    with tempfile.TemporaryDirectory() as td:
        scp = os.path.join(td, "wav.scp")
        with open(scp, "w") as f:
            for utt, x in signals.items():
                p = os.path.join(td, utt + ".wav")
                wavfile.write(p, 16000, x)
                f.write("%s %s\n" % (utt, p))
        if noise is not None:
            os.makedirs(os.path.join(td, "noises"), exist_ok=True)
            wavfile.write(os.path.join(td, "noises", noise_name + ".wav"), 16000, noise)
        if rir is not None:
            os.makedirs(os.path.join(td, "RIR"), exist_ok=True)
            wavfile.write(os.path.join(td, "RIR", "RIR_SmallRoom1_near_AnglA.wav"), 16000, rir)
        cwd = os.getcwd()
        os.chdir(td)
        try:
            ns = argparse.Namespace(scp=scp, outfile=os.path.join(td, "out"), scp_type="wav",
                                    spectrum_type=opts.get("spectrum_type", "log"), nfilters=opts["nfilters"],
                                    fduration=opts["fduration"], frate=opts["frate"], nfft=opts["nfft"],
                                    add_reverb=opts.get("add_reverb", "clean"), fbank_type=opts["fbank_type"],
                                    write_utt2num_frames=False, add_noise=opts.get("add_noise", "clean"))
            if noise_seed is not None:
                np.random.seed(noise_seed)
            cm.compute_mel_spectrum(ns)
        finally:
            os.chdir(cwd)
    return captured


MEL_DEFAULT = dict(nfilters=23, fduration=0.02, frate=100, nfft=1024, fbank_type="mel,1", spectrum_type="log")


def mel_fixtures():
    """computeMelSpectrum.py (run_melspec baseline): default log-mel, recipe nfilters=15, power spectrum with
    a cochlear filterbank, diff, and noise + reverb."""
    sig = OrderedDict()
    sig["m1"] = speech_like(16000, 81)
    sig["m2"] = speech_like(23457, 82)
    sig["mwhite"] = white(8000, 83)
    sig["mshort"] = speech_like(700, 84)
    save("mel_default", sig, MEL_DEFAULT, 0, run_reference_mel(sig, MEL_DEFAULT))
    opts = dict(MEL_DEFAULT, nfilters=15)
    save("mel_recipe15", sig, opts, 0, run_reference_mel(sig, opts))
    opts = dict(MEL_DEFAULT, nfilters=40, nfft=512, fduration=0.025, fbank_type="cochlear,1,1,1,2.5,1",
                spectrum_type="power")
    save("mel_cochlear_power", sig, opts, 0, run_reference_mel(sig, opts))
    opts = dict(MEL_DEFAULT, add_noise="diff")
    save("mel_diff", sig, opts, 0, run_reference_mel(sig, opts))
    rir = synthetic_rir(1200, 85)
    noise = white(16000 * 3, 86, scale=1000.0)
    opts = dict(MEL_DEFAULT, add_noise="babble,10", add_reverb="small_room")
    save("mel_noise_reverb", sig, opts, 0,
         run_reference_mel(sig, opts, noise_seed=7, noise=noise, noise_name="babble", rir=rir),
         extra=dict(noise_seed=7), more={"rir": rir, "noise_babble": noise})


def run_reference_modspec(signals, opts):
    """computeModulationSpectrum.getFeats with dict2Ark captured (copy-feats is absent)."""
    sys.path.insert(0, os.path.join(REF, "src/featgen"))
    import computeModulationSpectrum as cms  # noqa: E402
    captured = {}
    cms.dict2Ark = lambda feat_dict, outfile, kaldi_cmd: captured.update({k: np.array(v) for k, v in feat_dict.items()})
    with tempfile.TemporaryDirectory() as td:
        scp = os.path.join(td, "wav.scp")
        with open(scp, "w") as f:
            for utt, x in signals.items():
                p = os.path.join(td, utt + ".wav")
                wavfile.write(p, 16000, x)
                f.write("%s %s\n" % (utt, p))
        ns = argparse.Namespace(scp=scp, outfile=os.path.join(td, "out"), scp_type="wav", add_reverb="clean",
                                coeff_0=opts["coeff_0"], coeff_n=opts["coeff_n"], order=opts["order"],
                                fduration=opts["fduration"], frate=opts["frate"], nfilters=opts["nfilters"],
                                kaldi_cmd="true", fbank_type=opts["fbank_type"],
                                complex_modulation=opts.get("complex_modulation", False),
                                keep_even=opts.get("keep_even", False),
                                compensate_noise=opts.get("compensate_noise", False),
                                no_window=opts.get("no_window", False),
                                absolute_value=opts.get("absolute_value", False), set_unity_gain=False)
        cms.getFeats(ns)
    return captured


MODSPEC_DEFAULT = dict(nfilters=15, coeff_0=5, coeff_n=30, order=50, fduration=0.5, frate=100, fbank_type="mel,1")


def modspec_fixtures():
    """computeModulationSpectrum.py (make_modspec_feats.sh defaults) and its option variants."""
    sig = OrderedDict()
    sig["q1"] = speech_like(9000, 91)
    sig["q2"] = speech_like(4100, 92)
    sig["qwhite"] = white(3000, 93)
    save("modspec_default", sig, MODSPEC_DEFAULT, 0, run_reference_modspec(sig, MODSPEC_DEFAULT))
    opts = dict(MODSPEC_DEFAULT, keep_even=True, compensate_noise=True, absolute_value=True)
    save("modspec_even_comp_abs", sig, opts, 0, run_reference_modspec(sig, opts))
    opts = dict(MODSPEC_DEFAULT, nfilters=20, coeff_0=2, coeff_n=24, order=40, fduration=0.4, frate=50,
                fbank_type="cochlear,1,1,1,2.5,1", keep_even=True, no_window=True)
    save("modspec_cochlear_rect", sig, opts, 0, run_reference_modspec(sig, opts))
    modspec_complex_fixtures()


def modspec_complex_fixtures():
    """--complex_modulation (computeModulationSpectrum.py:45-47, :74-88, :153-180): real+imag, and
    abs + compensate_noise + keep_even; a cochlear filterbank with abs and a rectangular window."""
    sig = OrderedDict()
    sig["q1"] = speech_like(9000, 91)
    sig["q2"] = speech_like(4100, 92)
    sig["qwhite"] = white(3000, 93)
    opts = dict(MODSPEC_DEFAULT, complex_modulation=True)
    save("modspec_complex", sig, opts, 0, run_reference_modspec(sig, opts))
    opts = dict(MODSPEC_DEFAULT, complex_modulation=True, keep_even=True, compensate_noise=True,
                absolute_value=True)
    save("modspec_complex_even_comp_abs", sig, opts, 0, run_reference_modspec(sig, opts))
    opts = dict(MODSPEC_DEFAULT, nfilters=20, coeff_0=2, coeff_n=24, order=40, fduration=0.4, frate=50,
                fbank_type="cochlear,1,1,1,2.5,1", complex_modulation=True, absolute_value=True, no_window=True)
    save("modspec_complex_cochlear_rect", sig, opts, 0, run_reference_modspec(sig, opts))


def run_reference_modspec_segments(recordings, segments, opts):
    """computeModulationSpectrum_segments.getFeats (:24-116) with dict2Ark captured."""
    sys.path.insert(0, os.path.join(REF, "src/featgen"))
    import computeModulationSpectrum_segments as cmss  # noqa: E402
    captured = {}
    cmss.dict2Ark = lambda feat_dict, outfile, kaldi_cmd: captured.update(
        {k: np.array(v) for k, v in feat_dict.items()})
    with tempfile.TemporaryDirectory() as td:
        scp = os.path.join(td, "wav.scp")
        with open(scp, "w") as f:
            for rec, x in recordings.items():
                p = os.path.join(td, rec + ".wav")
                wavfile.write(p, 16000, x)
                f.write("%s %s\n" % (rec, p))
        seg = os.path.join(td, "segments")
        with open(seg, "w") as f:
            for s_id, rec, t0, t1 in segments:
                f.write("%s %s %s %s\n" % (s_id, rec, t0, t1))
        ns = argparse.Namespace(scp=scp, segment=seg, outfile=os.path.join(td, "out"), add_reverb=None,
                                set_unity_gain=opts.get("set_unity_gain", False),
                                nmodulations=opts["nmodulations"], order=opts["order"],
                                fduration=opts["fduration"], frate=opts["frate"], nfilters=opts["nfilters"],
                                kaldi_cmd="true")
        cmss.getFeats(ns)
    return captured


MODSPEC_SEG_DEFAULT = dict(nfilters=15, nmodulations=12, order=50, fduration=0.5, frate=100)


def modspec_segments_fixtures():
    """computeModulationSpectrum_segments.py: segments of two recordings (out of order, overlapping,
    fractional times), default options and --set_unity_gain with other sizes."""
    rec = OrderedDict()
    rec["recA"] = speech_like(40000, 95)
    rec["recB"] = speech_like(26000, 96)
    segs = [("recA-000", "recA", "0.00", "0.75"), ("recA-001", "recA", "0.5", "1.9371"),
            ("recB-000", "recB", "0.1", "1.6"), ("recA-002", "recA", "2.0", "2.5")]
    meta_segs = [list(x) for x in segs]
    feats = run_reference_modspec_segments(rec, segs, MODSPEC_SEG_DEFAULT)
    save("modspec_segments", rec, MODSPEC_SEG_DEFAULT, 0, _seg_feats(feats, rec), extra=dict(segments=meta_segs),
         more=_seg_more(feats))
    opts = dict(MODSPEC_SEG_DEFAULT, nfilters=20, nmodulations=40, order=30, fduration=0.4, frate=50,
                set_unity_gain=True)
    feats = run_reference_modspec_segments(rec, segs, opts)
    save("modspec_segments_unity", rec, opts, 0, _seg_feats(feats, rec), extra=dict(segments=meta_segs),
         more=_seg_more(feats))


def _seg_feats(feats, rec):  # save() stores out_<recording>; the per-segment outputs go in `more`
    return {r: np.zeros((0,)) for r in rec}


def _seg_more(feats):
    return {"seg_" + k: v for k, v in feats.items()}


def reverb_rir_fixture():
    """--add_reverb small_room (features.py:110-115) with a synthetic stereo RIR, clean and with noise."""
    rir = synthetic_rir(4000, 5)
    sig = OrderedDict()
    sig["v1p2"] = speech_like(19200, 51)
    sig["v3p0"] = speech_like(48000, 52)
    sig["vwhite"] = white(30000, 53)
    opts = dict(WSJ, add_reverb="small_room")
    save("reverb_rir", sig, opts, 99, run_reference(sig, opts, 99, rir=rir), more={"rir": rir})
    noise = white(16000 * 6, 54, scale=1500.0)
    opts_n = dict(CHIME4, add_reverb="small_room", add_noise="babble,20")
    save("reverb_rir_noise", sig, opts_n, 98,
         run_reference(sig, opts_n, 98, noise_seed=4, noise=noise, noise_name="babble", rir=rir),
         extra=dict(noise_seed=4), more={"rir": rir, "noise_babble": noise})


def wav_kinds_fixtures():
    """Noise mixing (--add_noise babble,20) and the diff filter (--add_noise diff) on the WAV formats scipy
    reads as other dtypes than int16 (features.py:24-31 squares the signal in its own dtype; :162-164 convolves
    it): float32 (a 16-bit-scaled signal and an unscaled one), 24-bit PCM (int32, left-justified), 32-bit PCM
    (int32, squares that wrap) and 8-bit unsigned PCM.  The WAV bytes are stored (wav_<utt>) with scipy's
    array (in_<utt>) and the reference's features (out_<utt>)."""
    import io
    sig, raw = OrderedDict(), {}
    sig["f32"] = (speech_like(24000, 61).astype(np.float64) / 32768.0).astype(np.float32)
    sig["f32big"] = (speech_like(20000, 62).astype(np.float64) * 0.37).astype(np.float32)
    # 24/32-bit squares wrap in int32, so the reference's mean energy can come out negative (alpha NaN, and
    # solve_toeplitz raises): the first seeds whose wrapped mean is positive are used
    seed = 63
    while True:
        v24 = np.clip(speech_like(40000, seed).astype(np.int64) * 211, -(2 ** 23), 2 ** 23 - 1)
        if np.mean((v24 << 8).astype(np.int32) ** 2) > 0:
            break
        seed += 100
    raw["i24"] = wav24_bytes(v24)
    sig["i24"] = wavfile.read(io.BytesIO(raw["i24"]))[1]
    assert sig["i24"].dtype == np.int32 and np.array_equal(sig["i24"], (v24 << 8).astype(np.int32))
    seed = 64
    while True:
        sig["i32"] = (speech_like(30000, seed).astype(np.int64) * 12).astype(np.int32)
        if np.mean(sig["i32"] ** 2) > 0:
            break
        seed += 100
    sig["u8"] = np.clip(speech_like(17000, 65).astype(np.int64) // 64 + 128, 0, 255).astype(np.uint8)
    for u, x in sig.items():
        if u not in raw:
            b = io.BytesIO()
            wavfile.write(b, 16000, x)
            raw[u] = b.getvalue()
        assert wavfile.read(io.BytesIO(raw[u]))[1].dtype == x.dtype
    more = {"wav_" + u: np.frombuffer(raw[u], dtype=np.uint8) for u in sig}
    noise = white(16000 * 5, 66, scale=1200.0)
    opts = dict(CHIME4, add_noise="babble,20")
    save("wav_kinds_noise", sig, opts, 77,
         run_reference(sig, opts, 77, noise_seed=5, noise=noise, noise_name="babble", raw=raw),
         extra=dict(noise_seed=5), more=dict(more, noise_babble=noise))
    opts = dict(WSJ, add_noise="diff")
    save("wav_kinds_diff", sig, opts, 78, run_reference(sig, opts, 78, raw=raw), more=more)


def main():
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    if "--wav-kinds-only" in sys.argv:
        wav_kinds_fixtures()
        return
    if "--reverb-only" in sys.argv:
        reverb_rir_fixture()
        return
    if "--mel-only" in sys.argv:
        mel_fixtures()
        return
    if "--modspec-only" in sys.argv:
        modspec_fixtures()
        return
    if "--modspec-complex-only" in sys.argv:
        modspec_complex_fixtures()
        return
    if "--modspec-segments-only" in sys.argv:
        modspec_segments_fixtures()
        return
    cli_options_fixture()
    if "--cli-only" in sys.argv:
        return
    stage_fixture()

    wsj = OrderedDict()
    wsj["short2"] = speech_like(2, 1)
    wsj["s0p5"] = speech_like(8000, 2)
    wsj["s1p0"] = speech_like(16000, 3)
    wsj["s18000"] = speech_like(18000, 4)
    wsj["s18002"] = speech_like(18002, 5)
    wsj["s4p0"] = speech_like(64000, 6)
    wsj["s4p5"] = speech_like(72000, 7)
    wsj["white10"] = white(160000, 0)
    wsj["pesq_or109"] = pesq_clip("or109.wav", 6.0)
    wsj["pesq_u_af1s02"] = pesq_clip("u_af1s02.wav", 5.3)
    save("wsj", wsj, WSJ, 1234, run_reference(wsj, WSJ, 1234))

    rev = OrderedDict()
    rev["r1p0"] = speech_like(16000, 21)
    rev["r4p0"] = speech_like(64000, 22)
    rev["pesq_dg149"] = pesq_clip("dg149.wav", 3.0)
    save("reverb", rev, REVERB, 7, run_reference(rev, REVERB, 7))

    noise = white(16000 * 20, 99, scale=2500.0)
    noise[::7] = (noise[::7].astype(np.int32) * 3).clip(-32768, 32767).astype(np.int16)
    ch = OrderedDict()
    ch["c1"] = speech_like(40000, 31)
    ch["c2"] = speech_like(27000, 32, rms=300.0)
    ch["c3"] = speech_like(52000, 33)
    opts = dict(CHIME4, add_noise="babble,20")
    save("chime4_noise", ch, opts, 5, run_reference(ch, opts, 5, noise_seed=42, noise=noise,
                                                    noise_name="babble"),
         extra=dict(noise_seed=42), more=dict(noise_babble=noise))

    cli = OrderedDict()
    cli["m1"] = speech_like(20000, 41)
    cli["m2"] = speech_like(35555, 42)
    save("cli_default_mel", cli, CLI_DEFAULT, 3, run_reference(cli, CLI_DEFAULT, 3))

    mel = OrderedDict()
    mel["k1"] = speech_like(50000, 51)
    save("mel80", mel, MEL80, 9, run_reference(mel, MEL80, 9))

    dif = OrderedDict()
    dif["d1"] = speech_like(30000, 61)
    dif["d2"] = white(19000, 62)
    opts = dict(WSJ, add_noise="diff")
    save("wsj_diff", dif, opts, 11, run_reference(dif, opts, 11))

    # gamma weight + odd-mod-zero + lifter file need p == M (computeFDLPSpectrogram.py:110,198)
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        lif = np.round(1.0 + 0.5 * np.cos(np.arange(120) / 7.0), 6)
        f.write(",".join("%.6f" % v for v in lif) + "\n")
        lifpath = f.name
    gw = OrderedDict()
    gw["g1"] = speech_like(33000, 71)
    opts = dict(WSJ, coeff_num=120, order=120, coeff_range="0,119", gamma_weight="20,1.5,3",
                odd_mod_zero=True, lifter_config=lifpath)
    feats = run_reference(gw, opts, 13)
    opts = dict(opts, lifter_config=None)
    save("gamma_lifter_odd", gw, opts, 13, feats, extra=dict(lifter=lif.tolist()))
    os.unlink(lifpath)
    reverb_rir_fixture()
    mel_fixtures()
    modspec_fixtures()
    modspec_segments_fixtures()


if __name__ == "__main__":
    main()
