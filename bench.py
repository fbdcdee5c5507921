#!/usr/bin/env python3
"""Benchmark: audio-hours/s of 80-band, p=150 FDLP-spectrogram features on MI355X.

One step = one fdlp_compute over a batch of synthetic 16 kHz utterances already resident in HBM
(BASELINE.json configs[1]: WSJ si284-like 4 s utterances, 80 bands, p=150, coeff_num=100,
cochlear filterbank; DESIGN.md "Measurement").  Every rank processes its own batch (utterances
shard across GPUs with no collective; scaling is weak).  Prints ONE JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config wsj|reverb]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix (= vector) dense peak, AMD spec
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec


def speech_like_batch(n_utt, T, seed):
    """AR(2)-coloured Gaussian noise x 3-5 Hz syllabic envelope, RMS ~2000, int16."""
    from scipy.signal import lfilter
    rng = np.random.default_rng(seed)
    out = np.empty((n_utt, T), dtype=np.int16)
    t = np.arange(T) / 16000.0
    for i in range(n_utt):
        e = rng.standard_normal(T + 400)
        f0, rad = rng.uniform(400, 1500), rng.uniform(0.90, 0.98)
        x = lfilter([1.0], [1.0, -2 * rad * np.cos(2 * np.pi * f0 / 16000), rad * rad], e)[400:]
        x *= 0.55 + 0.45 * np.sin(2 * np.pi * rng.uniform(3, 5) * t + rng.uniform(0, 6.28))
        x *= 2000.0 / (np.sqrt(np.mean(x * x)) + 1e-12)
        out[i] = np.clip(np.round(x), -32768, 32767).astype(np.int16)
    return out


def _cpu_worker(args):
    cfg_name, utts, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    import random
    from oracle import fdlp_oracle as O
    orc = O.FdlpOracle(getattr(O.FdlpConfig, cfg_name)())
    rng = random.Random(seed)
    t0 = time.perf_counter()
    for x in utts:
        orc.utterance(x, rng)
    return time.perf_counter() - t0


def cpu_baseline(cfg_name, T, workers, per_worker):
    """The oracle (reference-equivalent fp64 numpy restatement) on a bounded sample."""
    sig = speech_like_batch(workers * per_worker, T, 4242)
    jobs = [(cfg_name, [sig[w * per_worker + i] for i in range(per_worker)], 100 + w) for w in range(workers)]
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        times = pool.map(_cpu_worker, jobs)
    audio_h = workers * per_worker * T / 16000.0 / 3600.0
    return dict(value=audio_h / max(times), unit="audio-hours/s", cores=workers, kind="port",
                sample="%d x %.1f s synthetic utterances (%d per process), oracle/fdlp_oracle.py, "
                       "OMP_NUM_THREADS=1, steady state (plan setup excluded)" %
                       (workers * per_worker, T / 16000.0, per_worker))


def _latest_pmc():
    """The newest committed PMC summary (profiles/rNN*_pmc.json, written by scripts/round_evidence.sh)."""
    import glob
    c = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_pmc.json")))
    return c[-1] if c else None


PMC_FILE = _latest_pmc()
AC_KERNEL_PREFIX = {"structured": ("fdlp::ac_vsweep_kernel", "fdlp::ac_band_kernel"),
                    "structured_mfma": ("fdlp::ac_sweep_kernel", "fdlp::ac_band_kernel"),
                    "direct": ("fdlp::autocorr_kernel",)}


def stage_traffic(path):
    """HBM bytes per launch of the autocorrelation stage from the committed rocprofv3 PMC summary
    of this same bench command (scripts/round_evidence.sh -> scripts/pmc_report.py): FETCH_SIZE x 2
    (gfx950 correction, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, KiB -> bytes.  None if absent."""
    try:
        rows = json.load(open(PMC_FILE))
    except (OSError, ValueError, TypeError):
        return None
    tot, seen = 0.0, set()
    for name, m in rows.items():
        short = name.replace("void ", "")
        for pre in AC_KERNEL_PREFIX[path]:
            if short.startswith(pre) and "fetch_bytes_x2" in m and "write_bytes" in m:
                tot += m["fetch_bytes_x2"] + m["write_bytes"]
                seen.add(pre)
    return tot if len(seen) == len(AC_KERNEL_PREFIX[path]) else None


AC_KERNELS = {"structured": "autocorr stage: ac_vsweep_kernel x2 (fp64 VALU FMA, lag-parallel sweeps) + "
                            "ac_band_kernel (v_mfma_f64_16x16x4f64 straddles); the 78.6 TFLOP/s fp64 peak is "
                            "shared by the VALU and matrix pipes",
              "structured_mfma": "autocorr stage: ac_sweep_kernel + ac_band_kernel (v_mfma_f64_16x16x4f64)",
              "direct": "autocorr stage: autocorr_kernel (v_mfma_f64_16x16x4f64)"}


def autocorr_flops(plan, support):
    """Useful fp64 FLOPs of the autocorrelation stage per analysis frame (2 per MAC) for the
    algorithm the path runs.  direct: nlags MACs per tap of every band support (circular).
    structured_mfma: the two skirt sweeps, the per-band flat tops and the boundary straddles;
    structured: the same with the flat tops as one sweep over [min m1, max m2) whose products run to N
    (DESIGN.md "Structured autocorrelation")."""
    nl, N = plan.nlags, plan.N
    lags = np.arange(nl)
    trunc = lambda n: float(np.maximum(n - lags, 0).sum())      # truncated autocorrelation
    path = plan.autocorr_path
    if path == "direct":
        return 2.0 * nl * float(support.sum())
    m1, m2 = plan.regions()
    macs = trunc(int(m1.max())) + trunc(N - int(m2.min()))
    if path == "structured":
        pos = np.arange(int(m1.min()), int(m2.max()))
        macs += float(np.minimum(nl, N - pos).sum())
    for j in range(plan.B):
        if path != "structured":
            macs += trunc(int(m2[j] - m1[j]))
        for b, lb in ((m1[j], 0), (m2[j], m1[j]), (N, m2[j])):
            macs += float(np.minimum(lags, min(int(b - lb), nl - 1)).sum())
    return 2.0 * macs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="wsj", choices=["wsj", "reverb"])
    ap.add_argument("--utts", type=int, default=1024, help="utterances per step per GPU")
    ap.add_argument("--seconds", type=float, default=4.0, help="utterance length")
    ap.add_argument("--support-eps", type=float, default=None)
    ap.add_argument("--cpu-workers", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--cpu-per-worker", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", type=int, default=None, help="sub-batches over two streams (plan default 2)")
    ap.add_argument("--workload", default="wsj", choices=["wsj", "librispeech"],
                    help="wsj: --utts utterances of --seconds (BASELINE configs[1]); librispeech: U(1,30) s "
                         "utterances filling --frames analysis frames per step (configs[4], per GPU)")
    ap.add_argument("--frames", type=int, default=4096, help="analysis frames per step (librispeech workload)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    T = int(round(args.seconds * 16000))

    # CPU baseline first (fork before any GPU initialisation in this process)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, T, args.cpu_workers, args.cpu_per_worker)

    import torch
    import torch.distributed as dist
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, PyRandom
    from speech_recognition_tools_amd.shard import timed_steps

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfg = getattr(FeatureConfig, args.config)()
    if args.support_eps is not None:
        cfg.support_eps = args.support_eps
    probe = FdlpPlan(cfg, device=-1)
    if args.workload == "wsj":
        lens = [T] * args.utts
    else:  # LibriSpeech-960h scale: lengths U(1, 30) s, a fresh draw per rank
        rs = np.random.RandomState(2000 + rank)
        lens, fr = [], 0
        while True:
            t = int(rs.uniform(1.0, 30.0) * 16000)
            if fr + probe.geometry(t)[0] > args.frames:
                break
            lens.append(t)
            fr += probe.geometry(t)[0]
    geo = [probe.geometry(t) for t in lens]
    frames = sum(g[0] for g in geo)
    plan = FdlpPlan(cfg, device=local, max_frames=frames)
    if args.pipeline is not None:
        plan.set_pipeline(args.pipeline)
    _, lo, hi = probe.fbank()
    support = (hi - lo).astype(np.int64)

    if args.workload == "wsj":
        pcm_host = speech_like_batch(args.utts, T, 1000 + rank).reshape(-1)
    else:
        pcm_host = speech_like_batch(1, sum(lens), 1000 + rank).reshape(-1)
    pcm = torch.from_numpy(pcm_host).to(dev)
    out = torch.empty((sum(g[1] for g in geo), cfg.nfilters), dtype=torch.float32, device=dev)
    rng = PyRandom(7 + rank)
    nj = sum(g[0] - 1 for g in geo)

    def step():
        plan.compute(pcm, lens, rng.randbits2(nj), out=out)

    # warmup, barrier + sync, exactly K steps, sync + barrier, max over ranks (speech_recognition_tools_amd.shard)
    elapsed = timed_steps(step, args.steps, args.warmup, lambda: torch.cuda.synchronize(dev),
                          dist if world > 1 else None, dev, before_timed=lambda: plan.set_profiling(True))
    stages, ncalls = plan.stage_times()

    audio_h = world * args.steps * sum(lens) / 16000.0 / 3600.0
    value = audio_h / elapsed
    # dominant stage: the MFMA autocorrelation (DESIGN.md "Roofline": useful MACs only)
    flops_per_launch = autocorr_flops(plan, support) * frames
    ac_ms = stages["autocorr"] / max(ncalls, 1)
    achieved = flops_per_launch / (ac_ms * 1e-3) / 1e12
    res = {
        "metric": "audio-hours/sec FDLP featurized (16 kHz, 80-band)",
        "value": value,
        "unit": "audio-hours/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": ("librispeech_960h_scale_u1_30s" if args.workload == "librispeech" else
                                "wsj_si284_4s_batches" if args.config == "wsj" else "reverb_et_4s_batches"),
                   "utts_per_step_per_gpu": len(lens),
                   "utt_seconds": args.seconds if args.workload == "wsj" else "U(1,30), mean %.2f" % (
                       sum(lens) / 16000.0 / len(lens)),
                   "frames_per_step_per_gpu": frames, "nfilters": cfg.nfilters, "order": cfg.order,
                   "coeff_num": cfg.coeff_num, "fbank": cfg.fbank_type, "support_eps": cfg.support_eps,
                   "autocorr_path": plan.autocorr_path,
                   "parallelism": "scp-shard x%d (no collective)" % world},
        "roofline": {"bound": "mfma", "kernel": AC_KERNELS[plan.autocorr_path],
                     "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": stage_traffic(plan.autocorr_path),
                     "traffic_unit": "bytes/launch (rocprofv3 PMC, %s)" % os.path.relpath(PMC_FILE or "none", ROOT),
                     "avg_launch_ms": ac_ms, "algorithmic_flops_per_launch": flops_per_launch},
        "stage_ms_per_step": {k: v / max(ncalls, 1) for k, v in stages.items()},
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
