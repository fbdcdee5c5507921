#!/usr/bin/env python3
"""Recipe-level end-to-end time of stage 1 (features) as e2e/wsj/run_fdlp_e1.sh:189-209 runs it: the
drop-in driver scripts/make_FDLPspectrum_feats.sh (reference recipes/timit/local_pyspeech/
make_FDLPspectrum_feats.sh:126-172) with the WSJ recipe's options, `--nj` cold JOB processes of
compute-fdlp-feats (each: interpreter start, imports, HIP initialisation, plan build, WAV reads, kernels,
ark/scp/len writes), the scp split and the feats.scp / utt2num_frames concatenation.  Wall time runs from
the driver's start to its exit (feats.scp complete).  The GPU count is the driver's own default (every
visible GPU, counted without touching HIP), as an unchanged recipe would get.

Synthetic data dir: --utts speech-like WAVs (bench.speech_like, 16 kHz int16) of U(lo, hi) seconds
written to a temp dir first (page-cached, as a recipe's second stage-1 pass would find them; the WAV
synthesis and writes are not timed).

    python benchmarks/driver_e2e.py [--utts 1800] [--nj 8] [--lengths 4 4] [--jobs-per-gpu 2]
Prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
from scipy.io import wavfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WSJ_OPTS = ["--nfilters", "80", "--order", "150", "--fduration", "1.5", "--frate", "100", "--coeff_num", "100",
            "--coeff_range", "0,100", "--overlap_fraction", "0.25", "--fbank_type", "cochlear,1,1,1,2.5,1",
            "--write_utt2num_frames", "true",  # e2e/wsj/run_fdlp_e1.sh:54-95
            "--add_opts", "--job_stats"]       # per-JOB phase timings into the JOB logs
# the same features as the CLI's own options (a JOB the driver would start)
WSJ_OPTS_CLI = ["--nfilters=80", "--order=150", "--fduration=1.5", "--frate=100", "--coeff_num=100",
                "--coeff_range=0,100", "--overlap_fraction=0.25", "--fbank_type=cochlear,1,1,1,2.5,1",
                "--write_utt2num_frames"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=1800)
    ap.add_argument("--lengths", type=float, nargs=2, default=[4.0, 4.0], help="U(lo, hi) seconds")
    ap.add_argument("--nj", type=int, default=8)
    ap.add_argument("--jobs-per-gpu", type=int, default=2)
    ap.add_argument("--ngpu", type=int, default=None, help="default: the driver's visible-GPU count")
    ap.add_argument("--keep", default=None, help="write the data dir here instead of a temp dir")
    ap.add_argument("--trace-dir", default=None, help="the single cold JOB's --job_trace files go here")
    a = ap.parse_args()
    from bench import speech_like
    rs = np.random.RandomState(11)
    lens = [int(rs.uniform(a.lengths[0], a.lengths[1]) * 16000) for _ in range(a.utts)]
    with tempfile.TemporaryDirectory() as tmp:
        base = a.keep or tmp
        data = os.path.join(base, "data", "train_si284")
        wavd = os.path.join(base, "wav")
        os.makedirs(data, exist_ok=True)
        os.makedirs(wavd, exist_ok=True)
        with open(os.path.join(data, "wav.scp"), "w") as f:
            for i, T in enumerate(lens):
                p = os.path.join(wavd, "u%06d.wav" % i)
                wavfile.write(p, 16000, speech_like(T, np.random.default_rng(500 + i)))
                f.write("u%06d %s\n" % (i, p))
        cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", str(a.nj),
               "--jobs_per_gpu", str(a.jobs_per_gpu)] + (["--ngpu", str(a.ngpu)] if a.ngpu else []) + WSJ_OPTS + [
               data, os.path.join(base, "fbank")]
        t0 = time.perf_counter()
        r = subprocess.run(cmd, cwd=base, capture_output=True, text=True)
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
            for n in range(1, a.nj + 1):
                lp = os.path.join(data, "log", "feats_train_si284.%d.log" % n)
                if os.path.exists(lp):
                    sys.stderr.write("--- %s\n%s\n" % (lp, open(lp).read()[-2000:]))
            sys.exit(r.returncode)
        n_feats = sum(1 for _ in open(os.path.join(data, "feats.scp")))
        frames = sum(int(l.split()[1]) for l in open(os.path.join(data, "utt2num_frames")))
        job_s, stats = [], []
        for n in range(1, a.nj + 1):
            for line in open(os.path.join(data, "log", "feats_train_si284.%d.log" % n)):
                if line.startswith("Execution Time:"):
                    job_s.append(float(line.split()[2]))
                if ": job stats " in line:
                    stats.append(json.loads(line.split(": job stats ", 1)[1]))
        audio_h = sum(lens) / 16000.0 / 3600.0
        # one cold JOB process timed from outside (interpreter start to exit) on a shard of the same size
        shard = os.path.join(base, "one_job.scp")
        lines = open(os.path.join(data, "wav.scp")).read().splitlines(True)
        with open(shard, "w") as f:
            f.writelines(lines[:max(1, len(lines) // a.nj)])
        cli = os.path.join(ROOT, "speech_recognition_tools_amd", "featgen", "computeFDLPSpectrogram.py")
        one = {}
        if a.trace_dir:
            a.trace_dir = os.path.abspath(a.trace_dir)
            os.makedirs(a.trace_dir, exist_ok=True)
        for k in range(2):
            t1 = time.perf_counter()
            tr = os.path.join(a.trace_dir, "cold_job_%d.jsonl" % k) if a.trace_dir else None
            r1 = subprocess.run(["python3", cli, shard, os.path.join(base, "one_job_%d" % k)] + WSJ_OPTS_CLI + ["--job_stats"]
                                + (["--job_trace=" + tr] if tr else []),
                                cwd=base, capture_output=True, text=True)
            w1 = time.perf_counter() - t1
            if r1.returncode != 0:
                sys.stderr.write(r1.stdout[-2000:] + r1.stderr[-2000:])
                sys.exit(r1.returncode)
            ex = [float(l.split()[2]) for l in r1.stdout.splitlines() if l.startswith("Execution Time:")]
            js = [json.loads(l.split(": job stats ", 1)[1]) for l in r1.stdout.splitlines() if ": job stats " in l]
            one.setdefault("process_wall_s", []).append(round(w1, 4))
            one.setdefault("execution_time_s", []).append(ex[0] if ex else None)
            if js:
                one.setdefault("early_hip_start_s", []).append(js[0].get("early_hip_start_s"))
                one.setdefault("early_hip_done_s", []).append(js[0].get("early_hip_done_s"))
                one.setdefault("plan_s", []).append(js[0].get("plan_seconds"))
        from speech_recognition_tools_amd.shard import visible_gpu_count
        ngpu = a.ngpu or max(1, visible_gpu_count())  # the driver's own rule
        print(json.dumps({"metric": "recipe stage-1 end-to-end audio-hours/s (make_FDLPspectrum_feats.sh, cold JOBs)",
                          "value": audio_h / wall, "unit": "audio-hours/s", "wall_s": wall, "audio_hours": audio_h,
                          "utts": a.utts, "utt_seconds": "U(%g,%g)" % tuple(a.lengths), "nj": a.nj,
                          "jobs_per_gpu": a.jobs_per_gpu, "ngpu": ngpu, "feats_scp_lines": n_feats,
                          "frames": frames, "job_execution_s": job_s, "one_cold_job": one,
                          "job_execution_s_mean": float(np.mean(job_s)) if job_s else None,
                          "job_stats_mean": {k: float(np.mean([s[k] for s in stats if s.get(k) is not None]))
                                             for k in stats[0] if any(s.get(k) is not None for s in stats)} if stats else None,
                          "note": "wall from the driver's start to feats.scp; every JOB is a cold process "
                                  "(interpreter, imports, HIP init, plan build, reads, kernels, writes)"}))


if __name__ == "__main__":
    main()
