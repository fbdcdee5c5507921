#!/usr/bin/env python3
"""Phase timeline of dct_frame_kernel: builds the timing variant (-DFDLP_DCT_PHASES=1: thread 0 of each
workgroup overwrites D[f][0..6] with s_memrealtime stamps, 100 MHz) at a side path, runs one 4096-frame
WSJ batch and prints the mean duration of each phase per frame and the frames in flight per CU.
Timing build only (its D rows are overwritten).

    python benchmarks/dct_phases.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VAR = os.path.join(ROOT, "variants", "libfdlp_dct_phases.so")  # built here, shipped with the tree


def main():
    if os.environ.get("FDLP_LIB") != VAR:
        if not os.path.exists(VAR):
            from speech_recognition_tools_amd import _build
            _build.build(out=VAR, defines=["-DFDLP_DCT_PHASES=2"])
        env = dict(os.environ, FDLP_LIB=VAR)
        sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)], env=env))
    import numpy as np
    import torch
    import bench
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, PyRandom
    cfg = FeatureConfig.wsj()
    T = 64000
    probe = FdlpPlan(cfg, device=-1)
    F, L = probe.geometry(T)
    n = 1024
    pcm = torch.from_numpy(bench.speech_like_batch(n, T, 1000).reshape(-1)).cuda()
    plan = FdlpPlan(cfg, device=0, max_frames=F * n)
    plan.set_debug(True)
    out = torch.empty((L * n, cfg.nfilters), dtype=torch.float32, device="cuda")
    rng = PyRandom(7)
    for _ in range(2):
        plan.compute(pcm, [T] * n, rng.randbits2(n * (F - 1)), out=out)
    torch.cuda.synchronize()
    dd = plan.debug_fetch(F * n, keys=("dct",))["dct"]
    ts = dd[:, :7].astype(np.int64)
    tg = dd[:, 7:10].astype(np.int64)
    dur = np.diff(ts, axis=1) * 10.0  # ns
    names = ["descriptor+gather+tables+radix20", "twiddle1+exchange1", "radix24+twiddle2", "exchange2+radix25",
             "unpack+post-twiddle", "D rows out"]
    t0, t1 = ts[:, 0].min(), ts[:, 6].max()
    res = {"frames": int(ts.shape[0]), "kernel_span_us": (t1 - t0) / 100.0,
           "frame_us_mean": float((ts[:, 6] - ts[:, 0]).mean()) / 100.0,
           "phase_us_mean": {k: round(float(v) / 1000.0, 3) for k, v in zip(names, dur.mean(axis=0))},
           "frames_in_flight_mean": float((ts[:, 6] - ts[:, 0]).sum()) / float(t1 - t0)}
    if tg[:, 0].min() > 0:  # the gather / tables / radix-20 split of the first phase (thread 0's view)
        g = np.stack([tg[:, 0] - ts[:, 0], tg[:, 1] - tg[:, 0], tg[:, 2] - tg[:, 1], ts[:, 1] - tg[:, 2]], axis=1)
        res["phase0_split_us_mean"] = {k: round(float(v) / 100.0, 3) for k, v in
                                       zip(["descriptor+gather", "tables", "radix20+twiddle", "barrier wait"],
                                           g.mean(axis=0))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
