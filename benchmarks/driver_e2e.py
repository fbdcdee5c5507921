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


def _write_wav(path, T, i):
    from bench import speech_like
    wavfile.write(path, 16000, speech_like(T, np.random.default_rng(500 + i)))


def _read_feats(scp):
    """{utt: matrix} of a feats.scp (every ark it names read once), in scp order."""
    from speech_recognition_tools_amd.featgen.features import read_ark
    arks, order = {}, []
    for line in open(scp):
        utt, rx = line.split()
        ark = rx.rsplit(":", 1)[0]
        if ark not in arks:
            arks[ark] = read_ark(ark)
        order.append((utt, ark))
    return [(u, arks[k][u]) for u, k in order]


def _check_single(a, base, data):
    """The same data dir through the driver with --nj 1: keys, order, frame counts and matrix shapes must
    match; the values differ only by the unseeded hop jitter (random.randrange, computeFDLPSpectrogram.py:
    225), whose draws depend on each utterance's position in its JOB -- reported, not asserted."""
    d1 = os.path.join(base, "data_single", "train_si284")
    os.makedirs(d1, exist_ok=True)
    with open(os.path.join(d1, "wav.scp"), "w") as f:
        f.write(open(os.path.join(data, "wav.scp")).read())
    cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", "1"] + \
        (["--ngpu", str(a.ngpu)] if a.ngpu else []) + WSJ_OPTS + [d1, os.path.join(base, "fbank_single")]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=base, capture_output=True, text=True)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
        sys.exit(r.returncode)
    many = _read_feats(os.path.join(data, "feats.scp"))
    one = _read_feats(os.path.join(d1, "feats.scp"))
    u2n_many = open(os.path.join(data, "utt2num_frames")).read()
    u2n_one = open(os.path.join(d1, "utt2num_frames")).read()
    keys_same = [u for u, _ in many] == [u for u, _ in one]
    shapes_same = keys_same and all(x.shape == y.shape for (_, x), (_, y) in zip(many, one))
    def moments(feats):  # global mean / std of every feature value (the jitter moves values, not these)
        n = sum(x.size for _, x in feats)
        m = sum(float(x.sum(dtype=np.float64)) for _, x in feats) / n
        v = sum(float(((x.astype(np.float64) - m) ** 2).sum()) for _, x in feats) / n
        return round(m, 6), round(v ** 0.5, 6)
    ok = keys_same and shapes_same and u2n_many == u2n_one
    if not ok:
        sys.stderr.write("single-JOB check failed: keys %s shapes %s utt2num_frames %s\n"
                         % (keys_same, shapes_same, u2n_many == u2n_one))
        sys.exit(3)
    return {"nj": 1, "wall_s": wall, "feats_scp_keys_and_order_equal": keys_same, "shapes_equal": shapes_same,
            "utt2num_frames_equal": u2n_many == u2n_one,
            "mean_std_nj": moments(many), "mean_std_single": moments(one),
            "note": "values are not compared one to one: the unseeded hop jitter (randrange, as the reference) "
                    "draws differently per JOB layout; the global moments show the same features"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=1800)
    ap.add_argument("--lengths", type=float, nargs=2, default=[4.0, 4.0], help="U(lo, hi) seconds")
    ap.add_argument("--nj", type=int, default=8)
    ap.add_argument("--jobs-per-gpu", type=int, default=2)
    ap.add_argument("--ngpu", type=int, default=None, help="default: the driver's visible-GPU count")
    ap.add_argument("--keep", default=None, help="write the data dir here instead of a temp dir")
    ap.add_argument("--trace-dir", default=None, help="the single cold JOB's --job_trace files go here")
    ap.add_argument("--check-single", action="store_true",
                    help="run the driver again with --nj 1 on the same data dir and compare feats.scp keys and order, "
                         "utt2num_frames and every utterance's matrix (VERDICT r5 item 6)")
    ap.add_argument("--workers", type=int, default=8, help="processes synthesising the WAVs (not timed)")
    ap.add_argument("--chain-jobs", choices=("true", "false"), default="true",
                    help="the driver's --chain_jobs: warm JOB chains (true) or one cold process per JOB")
    a = ap.parse_args()
    rs = np.random.RandomState(11)
    lens = [int(rs.uniform(a.lengths[0], a.lengths[1]) * 16000) for _ in range(a.utts)]
    with tempfile.TemporaryDirectory() as tmp:
        base = a.keep or tmp
        data = os.path.join(base, "data", "train_si284")
        wavd = os.path.join(base, "wav")
        os.makedirs(data, exist_ok=True)
        os.makedirs(wavd, exist_ok=True)
        import concurrent.futures
        paths = [os.path.join(wavd, "u%06d.wav" % i) for i in range(len(lens))]
        with concurrent.futures.ProcessPoolExecutor(max(1, a.workers)) as ex:
            list(ex.map(_write_wav, paths, lens, range(len(lens)), chunksize=64))
        with open(os.path.join(data, "wav.scp"), "w") as f:
            for i, p in enumerate(paths):
                f.write("u%06d %s\n" % (i, p))
        cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", str(a.nj),
               "--jobs_per_gpu", str(a.jobs_per_gpu), "--chain_jobs", a.chain_jobs] + \
            (["--ngpu", str(a.ngpu)] if a.ngpu else []) + WSJ_OPTS + [
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
        single = _check_single(a, base, data) if a.check_single else None
        from speech_recognition_tools_amd.shard import visible_gpu_count
        ngpu = a.ngpu or max(1, visible_gpu_count())  # the driver's own rule
        print(json.dumps({"metric": "recipe stage-1 end-to-end audio-hours/s (make_FDLPspectrum_feats.sh, %s)"
                          % ("warm JOB chains" if a.chain_jobs == "true" else "a cold process per JOB"),
                          "value": audio_h / wall, "unit": "audio-hours/s", "wall_s": wall, "audio_hours": audio_h,
                          "utts": a.utts, "utt_seconds": "U(%g,%g)" % tuple(a.lengths), "nj": a.nj,
                          "jobs_per_gpu": a.jobs_per_gpu, "chain_jobs": a.chain_jobs == "true", "ngpu": ngpu,
                          "feats_scp_lines": n_feats,
                          "frames": frames, "job_execution_s": job_s, "one_cold_job": one,
                          "job_execution_s_mean": float(np.mean(job_s)) if job_s else None,
                          "job_stats_mean": {k: float(np.mean([s[k] for s in stats if s.get(k) is not None]))
                                             for k in stats[0] if any(s.get(k) is not None for s in stats)} if stats else None,
                          "single_job_check": single,
                          "note": "wall from the driver's start to feats.scp; every JOB is a cold process "
                                  "(interpreter, imports, HIP init, plan build, reads, kernels, writes)"}))


if __name__ == "__main__":
    main()
