#!/usr/bin/env python3
"""Run scripts/make_FDLPspectrum_feats.sh over one synthetic data dir in several modes (and repeats of a
mode) and compare every JOB's ark value by value: which modes write the same features, and where the
others differ (utterance, frame, dimension, both values).

    python3 benchmarks/job_determinism.py [--modes chain,cold,cold] [--nj 5] [--utts 25] [--seed 23] [--extra '--seed 7']
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
from scipy.io import wavfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="chain,cold,cold")
    ap.add_argument("--nj", type=int, default=5)
    ap.add_argument("--jobs_per_gpu", type=int, default=2)
    ap.add_argument("--utts", type=int, default=25)
    ap.add_argument("--seed", type=int, default=23)
    ap.add_argument("--extra", default="--seed 7", help="more driver options, space separated (unseeded, the OLA "
                    "jitter comes from OS entropy per JOB and every run differs)")
    a = ap.parse_args()
    from speech_recognition_tools_amd.featgen.features import read_ark
    rng = np.random.default_rng(a.seed)
    utts = ["c%03d" % i for i in range(a.utts)]
    sig = {u: np.clip(rng.standard_normal(int(rng.integers(16000, 64000))) * 2500, -32768, 32767).astype(np.int16)
           for u in utts}
    tmp = tempfile.mkdtemp(prefix="jobdet_")
    runs = []
    for i, mode in enumerate(a.modes.split(",")):
        d = os.path.join(tmp, "%d_%s" % (i, mode))
        data = os.path.join(d, "data")
        os.makedirs(data)
        with open(os.path.join(data, "wav.scp"), "w") as f:
            for u in utts:
                p = os.path.join(data, u + ".wav")
                wavfile.write(p, 16000, sig[u])
                f.write("%s %s\n" % (u, p))
        cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", str(a.nj), "--ngpu", "1",
               "--jobs_per_gpu", str(a.jobs_per_gpu), "--chain_jobs", "true" if mode == "chain" else "false",
               "--write_utt2num_frames", "true"] + a.extra.split() + [data, os.path.join(d, "fbank")]
        r = subprocess.run(cmd, cwd=d, capture_output=True, text=True, timeout=600)
        if r.returncode:
            print(r.stdout[-3000:], r.stderr[-3000:])
            return 1
        arks = {}
        for n in range(1, a.nj + 1):
            arks[n] = read_ark(os.path.join(d, "fbank", "melspec_data.%d.ark" % n))
        runs.append((i, mode, arks))
    base_i, base_mode, base = runs[0]
    for i, mode, arks in runs[1:]:
        for n in range(1, a.nj + 1):
            diffs = []
            for u, x in base[n].items():
                y = arks[n][u]
                if x.shape != y.shape:
                    diffs.append({"utt": u, "shape": [list(x.shape), list(y.shape)]})
                    continue
                idx = np.argwhere(x != y)
                for fr, dim in idx[:5]:
                    diffs.append({"utt": u, "frame": int(fr), "dim": int(dim), "a": float(x[fr, dim]),
                                  "b": float(y[fr, dim]), "n_frames": int(x.shape[0])})
                if len(idx) > 5:
                    diffs.append({"utt": u, "more": int(len(idx) - 5)})
            print(json.dumps({"a": "%d_%s" % (base_i, base_mode), "b": "%d_%s" % (i, mode), "job": n,
                              "utts": len(base[n]), "n_diffs": len(diffs), "diffs": diffs[:12]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
