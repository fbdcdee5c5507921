#!/usr/bin/env python3
"""End-to-end throughput of compute-fdlp-feats (WAV files in, Kaldi ark/scp out) on one MI355X, i.e.
including the host side the device-resident bench.py excludes: WAV read + parse, jitter RNG, H2D,
D2H and the ark writer.  Synthetic speech-like 4 s WAVs (bench.speech_like_batch) in a temp dir.

    python benchmarks/cli_throughput.py [--utts 512] [--workers 1 4 8] [--batch-frames 8192]
                                        [--runners native python]
Prints one JSON line per (host runner, worker count).
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
from scipy.io import wavfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=512)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--workers", type=int, nargs="+", default=[1, 4, 8])
    ap.add_argument("--batch-frames", type=int, default=8192)
    ap.add_argument("--profile", default=None, help="write cProfile stats of the last run to this file")
    ap.add_argument("--runners", nargs="+", default=["native", "python"], choices=["native", "native_mapped", "python"])
    ap.add_argument("--variants", nargs="+", default=["-"],
                    help="extra CLI flags (without the leading --) per run of the native runner, e.g. "
                         "'d2h_codes=off' 'keep_warm chunk_rows=32768'; '-' for none")
    ap.add_argument("--repeat", type=int, default=1, help="runs per (runner, workers, variant)")
    ap.add_argument("--trace-dir", default=None, help="native: write each run's --job_trace here")
    a = ap.parse_args()
    from bench import speech_like_batch
    from speech_recognition_tools_amd.featgen import computeFDLPSpectrogram as cli
    from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import build_parser, getFeats
    T = int(a.seconds * 16000)
    with tempfile.TemporaryDirectory() as d:
        sig = speech_like_batch(a.utts, T, 77)
        with open(os.path.join(d, "wav.scp"), "w") as f:
            for i in range(a.utts):
                p = os.path.join(d, "u%05d.wav" % i)
                wavfile.write(p, 16000, sig[i])
                f.write("u%05d %s\n" % (i, p))
        opts = ["--nfilters=80", "--coeff_num=100", "--coeff_range=0,100", "--order=150", "--fduration=1.5",
                "--frate=100", "--overlap_fraction=0.25", "--fbank_type=cochlear,1,1,1,2.5,1", "--seed=1",
                "--batch_frames=%d" % a.batch_frames]
        devnull = open(os.devnull, "w")
        # warm-up (plan build, kernel load)
        so = sys.stdout
        sys.stdout = devnull
        getFeats(build_parser().parse_args([os.path.join(d, "wav.scp"), os.path.join(d, "warm")] + opts),
                 return_feats=False)
        sys.stdout = so
        runs = [(r, w, v, k) for r in a.runners for w in a.workers
                for v in (a.variants if r.startswith("native") else [""]) for k in range(a.repeat)]
        for runner, w, variant, rep in runs:
            extra = ["--" + f for f in variant.split() if f != "-"]
            if a.trace_dir and runner.startswith("native"):
                os.makedirs(a.trace_dir, exist_ok=True)
                tag = "%s_w%d_%s_%d" % (runner, w, "".join(ch if ch.isalnum() else "_" for ch in variant), rep)
                extra = extra + ["--job_trace=" + os.path.join(a.trace_dir, tag + ".jsonl")]
            # a fresh output name per run, the previous run's outputs deleted before the clock starts (replacing
            # a 1 GB ark frees its page-cache pages inside the JOB's final rename: ~0.18 s on the box)
            for f in os.listdir(d):
                if f.startswith("o_"):
                    os.remove(os.path.join(d, f))
            oname = os.path.join(d, "o_%d_%d" % (w, rep))
            args = build_parser().parse_args([os.path.join(d, "wav.scp"), oname,
                                              "--io_workers=%d" % w, "--host_runner=" + runner.split("_")[0]] +
                                             (["--mapped_output"] if runner == "native_mapped" else []) + opts + extra)
            sys.stdout = devnull
            prof = None
            if a.profile:
                import cProfile
                prof = cProfile.Profile()
                prof.enable()
            t0 = time.perf_counter()
            getFeats(args, return_feats=False)
            el = time.perf_counter() - t0
            sys.stdout = so
            if prof is not None:
                import pstats
                prof.disable()
                with open(a.profile, "w") as fh:
                    pstats.Stats(prof, stream=fh).sort_stats("cumulative").print_stats(40)
                    pstats.Stats(prof, stream=fh).sort_stats("tottime").print_stats(30)
            audio_h = a.utts * T / 16000.0 / 3600.0
            print(json.dumps({"metric": "compute-fdlp-feats end-to-end audio-hours/s (WAV in, ark out)",
                              "value": audio_h / el, "unit": "audio-hours/s", "io_workers": w,
                              "host_runner": runner, "variant": variant, "repeat": rep,
                              "batch_frames": a.batch_frames,
                              "utts": a.utts, "utt_seconds": a.seconds, "seconds": el,
                              "ark_bytes": os.path.getsize(oname + ".ark"),
                              "job_stats": cli.LAST_JOB_STATS if runner.startswith("native") else None}))
            sys.stdout.flush()


if __name__ == "__main__":
    main()
