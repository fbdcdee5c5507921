#!/usr/bin/env python3
"""Device batches in flight per process: K independent FdlpPlans (own workspaces) on K HIP streams, each
featurising its own 1024 x 4 s batch every step; stream k starts k/K of a step late (it waits on an
event recorded after plan 0's first step), so the streams do not run the same kernel at the same time.
Prints audio-hours/s for K = 1, 2, 3 alternating.  An experiment for DESIGN.md §6, not the bench line.

    python benchmarks/inflight_probe.py [--steps 10] [--rounds 2]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--ks", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--stagger-cycles", type=int, default=0,
                    help="stream k first spins k * this / K GPU cycles (torch.cuda._sleep) inside the timed region")
    a = ap.parse_args()
    import torch
    from bench import scp_list, utterance_pcm
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, PyRandom
    cfg = FeatureConfig.wsj()
    probe = FdlpPlan(cfg, device=-1)
    full = scp_list("wsj", 1, 1024, 4.0, 4096, lambda t: probe.geometry(t)[0])
    lens = [t for _, t, _ in full]
    geo = [probe.geometry(t) for t in lens]
    frames, rows, nj = sum(g[0] for g in geo), sum(g[1] for g in geo), sum(g[0] - 1 for g in geo)
    audio_h = sum(lens) / 16000.0 / 3600.0
    dev = torch.device("cuda", 0)
    pcm = torch.from_numpy(utterance_pcm(full)).to(dev)
    kmax = max(a.ks)
    plans = [FdlpPlan(cfg, device=0, max_frames=frames) for _ in range(kmax)]
    outs = [torch.empty((rows, cfg.nfilters), dtype=torch.float32, device=dev) for _ in range(kmax)]
    streams = [torch.cuda.Stream(dev) for _ in range(kmax)]
    rng = PyRandom(7)
    jit = rng.randbits2(nj)
    for _ in range(a.rounds):
        for K in a.ks:
            for k in range(K):  # warm-up
                with torch.cuda.stream(streams[k]):
                    plans[k].compute(pcm, lens, jit, out=outs[k])
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            if a.stagger_cycles:
                for k in range(1, K):
                    with torch.cuda.stream(streams[k]):
                        torch.cuda._sleep(a.stagger_cycles * k // K)
            for s in range(a.steps):
                for k in range(K):
                    with torch.cuda.stream(streams[k]):
                        plans[k].compute(pcm, lens, jit, out=outs[k])
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            print("K=%d  %.1f audio-h/s  (%.3f ms per batch)" % (K, K * a.steps * audio_h / el, el / (K * a.steps) * 1e3),
                  flush=True)


if __name__ == "__main__":
    main()
