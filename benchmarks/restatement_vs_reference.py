#!/usr/bin/env python3
"""Calibration of the CPU baseline: the oracle (oracle/fdlp_oracle.py, the
reference-equivalent numpy restatement that bench.py times on the GPU box as `cpu_baseline`) against the
REAL reference getFeats (src/featgen/computeFDLPSpectrogram.py:29-237) on the same utterances, one core
each, in THIS container (the reference never travels to the GPU box).

Steady state: the reference's getFeats builds its filterbank per call (features.py:197-219, seconds of pure
Python), so each side is timed on k utterances and on 1 utterance and the difference is divided by k - 1.
Also checks the two agree (max-abs of the log features).

    PYTHONDONTWRITEBYTECODE=1 OMP_NUM_THREADS=1 python benchmarks/restatement_vs_reference.py [--utts 6]
Prints one JSON line.
"""
import argparse
import json
import os
import random
import sys
import time
from collections import OrderedDict

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=6)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--config", default="wsj", choices=["wsj", "reverb"])
    a = ap.parse_args()
    import numpy as np
    import make_golden as G  # run_reference: the real getFeats with dict2Ark captured
    from oracle import fdlp_oracle as O
    T = int(a.seconds * 16000)
    sig = OrderedDict(("u%d" % i, G.speech_like(T, 300 + i)) for i in range(a.utts))
    opts = G.WSJ if a.config == "wsj" else G.REVERB
    ocfg = O.FdlpConfig.wsj() if a.config == "wsj" else O.FdlpConfig.reverb()

    def t_ref(signals):
        t0 = time.perf_counter()
        out = G.run_reference(signals, opts, 11)
        return time.perf_counter() - t0, out

    def t_orc(signals):
        t0 = time.perf_counter()
        out = O.compute_utterances(ocfg, signals, 11)
        return time.perf_counter() - t0, out

    one = OrderedDict(list(sig.items())[:1])
    r1, _ = t_ref(one)
    rk, ref = t_ref(sig)
    o1, _ = t_orc(one)
    ok, orc = t_orc(sig)
    audio_s = (a.utts - 1) * a.seconds
    ref_rate = audio_s / (rk - r1)
    orc_rate = audio_s / (ok - o1)
    err = max(float(np.abs(ref[u] - orc[u]).max()) for u in sig)
    print(json.dumps({"config": a.config, "utts": a.utts, "utt_seconds": a.seconds, "cores": 1,
                      "reference_audio_s_per_s": ref_rate, "restatement_audio_s_per_s": orc_rate,
                      "restatement_over_reference": orc_rate / ref_rate,
                      "reference_setup_s": r1 - (rk - r1) / (a.utts - 1),
                      "max_abs_restatement_vs_reference": err,
                      "numpy": np.__version__}))


if __name__ == "__main__":
    main()
