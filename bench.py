#!/usr/bin/env python3
"""Benchmark: audio-hours/s of 80-band, p=150 FDLP-spectrogram features on MI355X.

One step = one fdlp_compute over this rank's batch of synthetic 16 kHz utterances already resident
in HBM (BASELINE.json configs[1]: WSJ si284-like 4 s utterances, 80 bands, p=150, coeff_num=100,
cochlear filterbank; DESIGN.md "Measurement").  The utterance list is a synthetic scp of
N x --utts entries (or U(1,30) s LibriSpeech-like entries, configs[4]) split into contiguous
shards like utils/split_scp.pl (make_FDLPspectrum_feats.sh:135-157): every rank featurises its own
shard with no collective (scaling is weak).  Prints ONE JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config wsj|reverb|chime4] [--workload wsj|librispeech|reverb]

Configs (BASELINE.json configs[1..4]):
  wsj      WSJ params (M 100, range 0..100), 4 s speech-like utterances (workload wsj, the headline);
           --workload librispeech: U(1,30) s lengths (configs[4])
  reverb   REVERB params (M 450, range 1..450), U(2,15) s utterances of two synthetic reverberant sets,
           "1ch" (T60 0.7 s) and "8ch_beamformit" (T60 0.35 s, stronger direct path): speech-like signals
           reverberated on the device by fdlp_reverb (addReverb, features.py:110-115) and stored as int16 PCM
           like the recorded et_real WAVs (input synthesis, outside the timed region)
  chime4   CHiME4 params (M 100, range 1..100), 4 s utterances mixed on the device with a synthetic babble
           noise at 20 dB inside the timed kernels (--add_noise babble,20: features.py:24-31; the per-utterance
           (offset, alpha) come from the numpy-legacy rand() replica like the reference's draws)
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no launcher environment (WORLD_SIZE unset) bench.py starts the N rank processes
itself (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE set, before anything touches a GPU).  Ranks meet over
gloo on the host for the barrier and the max-of-elapsed reduction only.  --dry-run keeps the launcher,
the sharding and the reduction and skips all device work (CPU test of the N > 1 path).
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= matrix) dense peak, AMD spec
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "audio-hours/sec FDLP featurized (16 kHz, 80-band)"


def speech_like(T, rng):
    """AR(2)-coloured Gaussian noise x 3-5 Hz syllabic envelope, RMS ~2000, int16."""
    from scipy.signal import lfilter
    t = np.arange(T) / 16000.0
    e = rng.standard_normal(T + 400)
    f0, rad = rng.uniform(400, 1500), rng.uniform(0.90, 0.98)
    x = lfilter([1.0], [1.0, -2 * rad * np.cos(2 * np.pi * f0 / 16000), rad * rad], e)[400:]
    x *= 0.55 + 0.45 * np.sin(2 * np.pi * rng.uniform(3, 5) * t + rng.uniform(0, 6.28))
    x *= 2000.0 / (np.sqrt(np.mean(x * x)) + 1e-12)
    return np.clip(np.round(x), -32768, 32767).astype(np.int16)


def speech_like_batch(n_utt, T, seed):
    """n_utt speech-like utterances of T samples from one seeded stream, [n_utt, T] int16."""
    rng = np.random.default_rng(seed)
    return np.stack([speech_like(T, rng) for _ in range(n_utt)]) if n_utt else np.zeros((0, T), np.int16)


def utterance_pcm(entries):
    """Concatenated int16 PCM of scp entries (utt, T, seed): every utterance from its own seed, so a
    rank's shard is the same whatever the world size."""
    return np.concatenate([speech_like(T, np.random.default_rng(seed)) for _, T, seed in entries])


def scp_list(workload, world, utts, seconds, frames, frames_of):
    """The synthetic scp of the whole job: [(utt_id, T, seed)].
    wsj: world * utts utterances of `seconds` (configs[1]).  librispeech: lengths U(1, 30) s (seeded,
    SURVEY.md 8(d) config 5); reverb: lengths U(2, 15) s (8(d) config 3), entries alternating between the
    "1ch" and "8ch_beamformit" sets.  The U(a, b) lists grow until they hold world * frames analysis frames
    (so every rank's contiguous shard is about `frames` frames, one device batch)."""
    if workload == "wsj":
        T = int(round(seconds * 16000))
        return [("wsj%06d" % i, T, 1000 + i) for i in range(world * utts)]
    lo, hi, rseed, seed0 = {"librispeech": (1.0, 30.0, 2000, 5000), "reverb": (2.0, 15.0, 3000, 9000)}[workload]
    rs = np.random.RandomState(rseed)
    out, fr = [], 0
    while True:
        t = int(rs.uniform(lo, hi) * 16000)
        f = frames_of(t)
        if fr + f > world * frames:
            return out
        i = len(out)
        name = "libri%06d" % i if workload == "librispeech" else "et_%s_%06d" % (REVERB_SETS[i & 1], i)
        out.append((name, t, seed0 + i))
        fr += f


REVERB_SETS = ("1ch", "8ch_beamformit")


def synthetic_rir(kind, fs=16000):
    """Synthetic room impulse response of a REVERB set: a unit direct path after
    2.5 ms and an exponentially decaying Gaussian tail (60 dB over T60) whose energy sits `drr` dB below
    the direct path, normalised to unit energy.  "1ch": T60 0.7 s, DRR 0 dB (a distant single
    microphone); "8ch_beamformit": T60 0.35 s, DRR +8 dB (the beamformed array output is drier)."""
    t60, drr_db, seed = {"1ch": (0.7, 0.0, 11), "8ch_beamformit": (0.35, 8.0, 12)}[kind]
    rng = np.random.default_rng(seed)
    R = int(t60 * fs)
    d0 = int(0.0025 * fs)
    n = np.arange(R, dtype=np.float64)
    tail = rng.standard_normal(R) * np.exp(-6.907755278982137 * (n - d0) / (t60 * fs))
    tail[:d0 + 16] = 0.0
    tail *= np.sqrt(10.0 ** (-drr_db / 10.0) / np.sum(tail * tail))
    h = tail
    h[d0] = 1.0
    return h / np.sqrt(np.sum(h * h))


def reverb_pcm(entries, device):
    """int16 PCM of REVERB-like entries: each set's speech-like signals go through fdlp_reverb on the device
    with the set's synthetic RIR (full convolution + the reference's xcorr alignment, features.py:110-115),
    then round/clip to int16 like a recorded WAV.  Returns (concatenated int16 numpy, lengths)."""
    import torch
    from speech_recognition_tools_amd.augment import reverb
    parts = [None] * len(entries)
    lens = [0] * len(entries)
    for k, kind in enumerate(REVERB_SETS):
        idx = [i for i in range(len(entries)) if (i & 1) == k]
        if not idx:
            continue
        rir = torch.from_numpy(synthetic_rir(kind)).to(device)
        for c0 in range(0, len(idx), 128):  # bounded device scratch (the convolution output is T + R - 1)
            sub = [entries[i] for i in idx[c0:c0 + 128]]
            sl = [t for _, t, _ in sub]
            x = torch.from_numpy(utterance_pcm(sub)).to(device)
            y, ol = reverb(x, sl, rir)
            y = torch.clamp(torch.round(y), -32768, 32767).to(torch.int16).cpu().numpy()
            off = np.concatenate([[0], np.cumsum(sl)])
            for j, i in enumerate(idx[c0:c0 + 128]):
                parts[i] = y[off[j]:off[j] + int(ol[j])]
                lens[i] = int(ol[j])
    return np.concatenate(parts), lens


NOISE_SNR = 20.0


def babble_noise(seconds=240.0, seed=77):
    """Synthetic noises/babble.wav stand-in (the reference's noises/*.wav are absent):
    six overlapped speech-like talkers, int16."""
    T = int(seconds * 16000)
    rng = np.random.default_rng(seed)
    acc = np.zeros(T)
    for _ in range(6):
        acc += speech_like(T, rng).astype(np.float64)
    acc *= 2500.0 / np.sqrt(np.mean(acc * acc))
    return np.clip(np.round(acc), -32768, 32767).astype(np.int16)


def noise_mix(pcm_host, lens, noise, snr, nprandom):
    """(offsets, alphas) of add_noise_to_wav (features.py:24-31) for every utterance of a batch in scp
    order, each offset from one np.random.rand() draw of `nprandom` (NpRandom: the numpy legacy stream)."""
    from speech_recognition_tools_amd.augment import noise_params
    offs = np.empty(len(lens), dtype=np.int64)
    alps = np.empty(len(lens), dtype=np.float64)
    o = 0
    for i, T in enumerate(lens):
        offs[i], alps[i] = noise_params(pcm_host[o:o + T], noise, snr, nprandom.rand())
        o += T
    return offs, alps


def _cpu_worker(args):
    cfg_name, utts, seed, noise, noise_seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    import random
    from oracle import fdlp_oracle as O
    orc = O.FdlpOracle(getattr(O.FdlpConfig, cfg_name)())
    rng = random.Random(seed)
    nrng = np.random.RandomState(noise_seed)
    t0 = time.perf_counter()
    for x in utts:
        if noise is not None:  # add_noise_to_wav (features.py:24-31), as the timed GPU path mixes
            x = O.add_noise(x, noise, NOISE_SNR, nrng.rand())
        orc.utterance(x, rng)
    return time.perf_counter() - t0


def cpu_baseline(cfg_name, lens, workers, per_worker, noise=None):
    """The oracle (reference-equivalent fp64 numpy restatement, cpu_baseline kind "port") on a bounded
    sample of the same workload (the first workers x per_worker utterance lengths of it), one process per
    core."""
    n = workers * per_worker
    lens = [lens[i % len(lens)] for i in range(n)]
    rng = np.random.default_rng(4242)
    sig = [speech_like(T, rng) for T in lens]
    jobs = [(cfg_name, sig[w * per_worker:(w + 1) * per_worker], 100 + w, noise, 300 + w) for w in range(workers)]
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        times = pool.map(_cpu_worker, jobs)
    audio_h = sum(lens) / 16000.0 / 3600.0
    return dict(value=audio_h / max(times), unit="audio-hours/s", cores=workers, kind="port",
                sample="%d synthetic utterances of the %s workload (%.1f audio-s, %d per process%s), "
                       "oracle/fdlp_oracle.py, OMP_NUM_THREADS=1, steady state (plan setup excluded), %.1f s wall" %
                       (n, cfg_name, sum(lens) / 16000.0, per_worker,
                        ", babble mixed at %g dB" % NOISE_SNR if noise is not None else "", max(times)))


def _latest_pmc(config="wsj"):
    """The newest committed PMC summary of a config (profiles/rNN*_pmc.json for wsj,
    profiles/rNN*_<config>_pmc.json otherwise; written by scripts/round_evidence.sh)."""
    import glob

    def order(f):  # rNN<letters>: round, then a..z before aa..zz (the evidence tags of a round)
        tag = os.path.basename(f).split("_")[0]
        return int(tag[1:3]), len(tag[3:]), tag[3:]
    c = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_pmc.json")), key=order)
    tagged = lambda f: any(("_%s_pmc" % k) in os.path.basename(f) for k in ("reverb", "chime4", "librispeech"))
    c = [f for f in c if ((("_%s_pmc" % config) in os.path.basename(f)) if config != "wsj" else not tagged(f))]
    return c[-1] if c else None


PMC_FILE = _latest_pmc()
# kernels of each timed stage (fdlp_stage_times), as rocprofv3 names them
STAGE_KERNELS = {"dct": ("fdlp::dct_frame", "fdlp::frames_dft1", "fdlp::dft2_dct"),
                 "autocorr": {"structured": ("fdlp::ac_vsweep_kernel", "fdlp::ac_wrap_kernel", "fdlp::ac_band_kernel"),
                              "structured_mfma": ("fdlp::ac_sweep_kernel", "fdlp::ac_band_kernel"),
                              "direct": ("fdlp::autocorr_kernel",)},
                 "lpc_env": ("fdlp::durbin4_kernel", "fdlp::durbin8_kernel", "fdlp::lpc_env_lattice_kernel",
                             "fdlp::lpc_env_kernel"),
                 "ola_log": ("fdlp::ola_log",)}


def stage_kernel_prefixes(stage, path):
    k = STAGE_KERNELS[stage]
    return k[path] if isinstance(k, dict) else k


def pmc_rows(pmc_file=None):
    try:
        return {k.replace("void ", ""): m for k, m in json.load(open(pmc_file or PMC_FILE)).items()}
    except (OSError, ValueError, TypeError):
        return {}


def stage_pmc(prefixes, pmc_file=None):
    """(HBM bytes per launch, bound) of a stage's kernels from the committed rocprofv3 PMC summary of the
    same bench command (scripts/round_evidence.sh -> scripts/pmc_report.py).  Bytes: FETCH_SIZE x 2 (gfx950
    correction, MI355X_MICROARCH.md "HBM") + WRITE_SIZE.  Bound: the fp64 pipe that is busier, time-weighted
    over the stage's kernels (SQ_ACTIVE_INST_VALU vs SQ_VALU_MFMA_BUSY_CYCLES); (None, None) without data."""
    tot, seen, valu, mfma = 0.0, 0, 0.0, 0.0
    for name, m in pmc_rows(pmc_file).items():
        if any(name.startswith(pre) for pre in prefixes) and "fetch_bytes_x2" in m and "write_bytes" in m:
            tot += m["fetch_bytes_x2"] + m["write_bytes"]
            seen += 1
            valu += m.get("valu_active_pct_per_simd", 0.0) * m.get("avg_ms", 0.0)
            mfma += m.get("mfma_busy_pct", 0.0) * m.get("avg_ms", 0.0)
    if not seen:
        return None, None
    return tot, ("fp64-valu" if valu >= mfma else "fp64-mfma")


def step_pmc_bytes(pmc_file=None):
    """HBM bytes of one batch: every fdlp kernel of the PMC summary, FETCH_SIZE x 2 + WRITE_SIZE per
    launch (one launch of each per batch, default pipeline)."""
    rows = pmc_rows(pmc_file)
    tot = [m["fetch_bytes_x2"] + m["write_bytes"] for k, m in rows.items()
           if k.startswith("fdlp::") and "fetch_bytes_x2" in m and "write_bytes" in m]
    return sum(tot) if tot else None


STAGE_DESC = {"dct": "DCT stage: dct_frame_kernel (one workgroup per frame, Makhoul DCT-II over a 20x24x25 "
                     "in-register FFT, fp64 VALU; frames_dft1 + dft2_dct with --dct-path four_step)",
              "autocorr": {"structured": "autocorr stage: ac_vsweep_kernel x2 (fp64 VALU FMA, lag-parallel sweeps) + "
                                         "ac_wrap_kernel (the wrap straddle shared by the bands) + ac_band_kernel "
                                         "(v_mfma_f64_16x16x4f64 straddles); the 78.6 TFLOP/s fp64 peak is shared "
                                         "by the VALU and matrix pipes",
                           "structured_mfma": "autocorr stage: ac_sweep_kernel + ac_band_kernel (v_mfma_f64_16x16x4f64)",
                           "direct": "autocorr stage: autocorr_kernel (v_mfma_f64_16x16x4f64)"},
              "lpc_env": "LPC stage: durbin4_kernel (Levinson-Durbin) + cepstrum + envelope kernels (fp64)",
              "ola_log": "OLA + log stage: ola_log_tiled_kernel"}


def lpc_flops(p, M, Me, kk):
    """Useful fp64 FLOPs of the LPC stage per (frame, band) item, 2 per MAC: the Durbin recursion (order k:
    a k-term dot product and k - 1 updates, sum = p^2 MACs) and the off-by-one gain (p + 1), the LPC
    cepstrum c_n, n < Me (features.py:233-246: min(n - 1, p) terms each; only the Me = min(M, env_nfft)
    coefficients the envelope uses are computed), the envelope sum_n c'_n cos(2 pi n t / env_nfft) for
    kk samples (Me x kk MACs) and its exp x window (2 per sample)."""
    cep = sum(min(n - 1, p) for n in range(2, Me))
    return 2.0 * (p * p + p + 1) + 2.0 * cep + 2.0 * Me * kk + 2.0 * kk


def dct_flops(N):
    """DCT-II of one frame as the FFT route counts it (2.5 N log2 N) plus the window (N)."""
    return 2.5 * N * np.log2(N) + N


def autocorr_flops(plan, support):
    """Useful fp64 FLOPs of the autocorrelation stage per analysis frame (2 per MAC) for the
    algorithm the path runs.  direct: nlags MACs per tap of every band support (circular).
    structured_mfma: the two skirt sweeps, the per-band flat tops and the boundary straddles;
    structured: the same with the flat tops as one sweep over [min m1, max m2) whose products run to N,
    and the wrap straddle shared by the bands with skirt taps at both edges (DESIGN.md "Structured
    autocorrelation")."""
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
    # structured: the wrap straddle of a band whose first / last nlags - 1 taps are skirt taps is one
    # band-independent Wrap row per frame (ac_wrap_kernel) times sqrt(K_j K'_j): counted once per frame
    shared = (m1 >= nl - 1) & (m2 <= N - (nl - 1)) if path == "structured" else np.zeros(plan.B, bool)
    if shared.any():
        macs += float(np.minimum(lags, nl - 1).sum())
    for j in range(plan.B):
        if path != "structured":
            macs += trunc(int(m2[j] - m1[j]))
        for b, lb in ((m1[j], 0), (m2[j], m1[j]), (N, m2[j])):
            if b == N and shared[j]:
                continue
            macs += float(np.minimum(lags, min(int(b - lb), nl - 1)).sum())
    return 2.0 * macs


def canonical_flops(N, B, p, M, kk, env_nfft):
    """FLOPs per analysis frame of the reference's own (FFT-based) algorithm:
    (autocorrelation stage, whole path)."""
    lg = np.log2(N)
    Me = min(M, env_nfft)
    ac = B * (5.0 * N * lg + 1.5 * N)
    whole = (2.5 * N * lg + N + B * N + ac + B * 2.0 * p * p + B * 1.5 * (M - 1) * (M - 2)
             + B * (2.0 * Me * kk + 3.0 * kk) + 2.0 * B * 112.5)
    return ac, whole


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """One child process per GPU (RANK = LOCAL_RANK = r), started before anything in this process
    touches a GPU; rank 0 prints the JSON line.  Returns the first non-zero exit code (or 0)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


RANK_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
            "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")


def xfer_child_spec(args, world, rank, local, argv=None, environ=None):
    """argv and environment of the PCIe-pass child of one rank (started before the rank touches the GPU):
    a single-process bench.py --xfer-only over the rank's own shard (--xfer-shard rank/world), on the rank's
    GPU only (HIP_VISIBLE_DEVICES narrowed to it), with GPU_MAX_HW_QUEUES = --xfer-hw-queues (read once per
    process, so the rank's own timed steps keep the default), and no rendezvous variables."""
    argv = list(sys.argv[1:] if argv is None else argv)
    environ = os.environ if environ is None else environ
    out, skip = [], False
    for a in argv:  # drop the launcher-level options the child must not inherit
        if skip:
            skip = False
            continue
        if a in ("--xfer-only", "--dry-run"):
            continue
        if a in ("--gpus", "--xfer-shard"):
            skip = True
            continue
        if a.startswith("--gpus=") or a.startswith("--xfer-shard="):
            continue
        out.append(a)
    out += ["--xfer-only", "--no-cpu-baseline", "--gpus", "1", "--xfer-shard", "%d/%d" % (rank, world)]
    env = {k: v for k, v in environ.items() if k not in RANK_ENV}
    env["GPU_MAX_HW_QUEUES"] = str(args.xfer_hw_queues)
    if world > 1:
        # the rank's GPU among the visible ones: HIP_VISIBLE_DEVICES wins over CUDA_VISIBLE_DEVICES in HIP, so
        # the list comes from the first that is set, and the child sees only HIP_VISIBLE_DEVICES
        vis = environ.get("HIP_VISIBLE_DEVICES") or environ.get("CUDA_VISIBLE_DEVICES")
        ids = [v.strip() for v in vis.split(",") if v.strip()] if vis else None
        env["HIP_VISIBLE_DEVICES"] = ids[local % len(ids)] if ids else str(local)
        env.pop("CUDA_VISIBLE_DEVICES", None)
    return out, env


def combine_xfer_children(got):
    """The ranks' PCIe-pass children -> one with_transfers block: total audio over the union of their timed
    regions, first start to last end on absolute clocks (the children run concurrently, one per GPU, but
    without a shared barrier, so a child that starts late lengthens the wall instead of hiding in a max of
    per-child times); None if any child failed."""
    if any(g is None or "audio_h" not in g for g in got):
        return None
    x = dict(got[0])
    if all("t_go" in g for g in got):
        t0 = min(g["t_go"] for g in got)
        wall = max(g["t_go"] + g["elapsed_s"] for g in got) - t0
        x["start_spread_s"] = max(g["t_go"] for g in got) - t0
    else:
        wall = max(g["elapsed_s"] for g in got)
    x["value"] = sum(g["audio_h"] for g in got) / wall
    steps = max(1, round(got[0]["elapsed_s"] * 1e3 / got[0]["ms_per_step"]))
    x["ms_per_step"] = wall / steps * 1e3
    x["audio_h"] = sum(g["audio_h"] for g in got)
    x["elapsed_s"] = wall
    x["per_rank_value"] = [g["value"] for g in got]
    x.pop("t_go", None)
    x["note"] = (x.get("note", "") + "; one child process per rank on its own GPU, started before the rank "
                 "touches it, all at once: value = total audio / first start to last end")
    return x


def run_xfer_child(args, world=1, rank=0, local=0):
    """bench.py --xfer-only in a child process (xfer_child_spec); its with_transfers block, or None (with
    the child's tail on stderr) when it fails."""
    argv, env = xfer_child_spec(args, world, rank, local)
    try:
        p = subprocess.run([sys.executable, os.path.abspath(__file__)] + argv, env=env, capture_output=True,
                           text=True, timeout=900)
    except subprocess.TimeoutExpired:
        print("bench.py: PCIe-pass child timed out, measuring in-process", file=sys.stderr)
        return None
    lines = [l for l in p.stdout.strip().splitlines() if l.startswith("{")]
    if p.returncode != 0 or not lines:
        print("bench.py: PCIe-pass child failed (rc %d), measuring in-process:\n%s" % (p.returncode, p.stderr[-2000:]),
              file=sys.stderr)
        return None
    return json.loads(lines[-1])["with_transfers"]


CPU_WORKERS_CAP = 16  # without OMP_NUM_THREADS: one oracle process holds ~1 GB on REVERB-sized utterances


def host_cores(with_rule=False):
    """The host cores this process may use: its CPU affinity, capped at the CPU share a pool gives a job
    (OMP_NUM_THREADS, which the GPU pool sets to a one-GPU job's share; os.cpu_count() there counts every
    CPU of the machine, most of them other jobs'), or at CPU_WORKERS_CAP when OMP_NUM_THREADS is unset.
    with_rule: also return how the count was chosen (recorded in the cpu_baseline block)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        v, rule = max(1, min(n, int(share))), "min(affinity %d, OMP_NUM_THREADS %s)" % (n, share)
    else:
        v, rule = max(1, min(n, CPU_WORKERS_CAP)), "min(affinity %d, cap %d; OMP_NUM_THREADS unset)" % (
            n, CPU_WORKERS_CAP)
    return (v, rule) if with_rule else v


def pcie_pass(args, plans, streams, pcms, outs, pcm_host, lens, nj, rng, mix, audio_s, world, dd, sync, dev, B):
    """SURVEY.md 8(d) wall, first H2D to last D2H: every batch's PCM copied in from pinned host memory and
    its features copied back to pinned host memory, every batch of every step.  Every batch in flight has
    two device buffer sets used on alternate steps, so step s + 1's copy-in runs while step s computes and
    step s's copy-out while step s + 1 computes (with one set per batch, every step's four copy-ins queued
    behind the previous step's kernels on the one H2D stream: 31.9 ms per step against 23.4 computing,
    r03f).  One H2D stream, --xfer-d2h-streams D2H streams; the compute of batch b stays on its own stream.

    The features leave the device as the compact ark codes (ABI 7, include/fdlp.h out_q_dev): int16
    k = nearbyint(v 10^3) per value, the ark's float32 (float)(k / 10^3) restored bit for bit on the host by
    fdlp_q_widen (the flag word of the batch, copied back with the codes, says whether every value had a
    code; otherwise the batch's float32 rows, also written in HBM, are the ones to fetch).  The widening of
    every step's codes to the ark's float32 runs inside the timed region on a host thread pool, overlapped
    with the next steps' copies and kernels (the float32 values an ark writer needs); the pass ends when the
    last step's codes are widened.  (Schedules measured at or below this one and removed in round 6: 3-4
    buffer sets, one grouped copy stream, host issue threads, per-batch H2D streams, float32 D2H, mapped
    codes, several processes per GPU)"""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from speech_recognition_tools_amd import q_widen
    out = outs[0]
    rows, D = out.shape
    nq = rows * D
    pin_in = torch.from_numpy(pcm_host).pin_memory()
    S = 2                                            # device buffer sets per batch, used in turn
    NB = S * B                                       # (batch, step mod S)
    pcm_d = [pcms[i // S] if i % S == 0 else torch.empty_like(pcms[0]) for i in range(NB)]
    out_d = [outs[i // S] if i % S == 0 else torch.empty_like(out) for i in range(NB)]
    # codes + the flag word in one buffer: [nq int16 codes | int32 flag], one D2H copy per batch
    q_d = [torch.empty(nq + 2, dtype=torch.int16, device=dev) for _ in range(NB)]
    q_h = [torch.empty(nq + 2, dtype=torch.int16).pin_memory() for _ in range(NB)]
    f_h = [np.empty(nq, dtype=np.float32) for _ in range(NB)]  # the widened ark values
    s_in = torch.cuda.Stream(dev)
    nd = args.xfer_d2h_streams or (2 if args.xfer_only else 1)
    s_outs = [torch.cuda.Stream(dev) for _ in range(nd)]
    comp = [torch.cuda.current_stream(dev)] if B == 1 else [streams[b] for b in range(B)]
    ev_in = [torch.cuda.Event() for _ in range(NB)]
    ev_done = [torch.cuda.Event() for _ in range(NB)]
    ev_out = [torch.cuda.Event() for _ in range(NB)]
    for i in range(NB):
        ev_done[i].record(comp[(i // S) % len(comp)])
        ev_out[i].record(comp[(i // S) % len(comp)])
    it = [0]
    widen_pool = ThreadPoolExecutor(1)               # one widening job at a time, each on 16 threads
    widen_jobs = [None] * NB
    widen_s = [0.0]
    host_issue = args.xfer_d2h_issue == "host"
    issue_pool = ThreadPoolExecutor(1) if host_issue else None
    issue_jobs = [None] * NB

    def issue_d2h(i, so):                            # --xfer-d2h-issue host: no device-side wait before the copy
        ev_done[i].synchronize()
        with torch.cuda.stream(so):
            q_h[i].copy_(q_d[i], non_blocking=True)
            ev_out[i].record(so)

    def widen(i):
        if issue_jobs[i] is not None:
            issue_jobs[i].result()                   # ev_out[i] is recorded
        ev_out[i].synchronize()                      # the codes of buffer set i are on the host
        t0 = time.perf_counter()
        q_widen(q_h[i][:nq], 3, threads=16, out=f_h[i])
        widen_s[0] += time.perf_counter() - t0

    def xbatch(b, i):
        cs = comp[b % len(comp)]
        if widen_jobs[i] is not None:                # q_h[i] is read by the previous widening of set i
            widen_jobs[i].result()
        s_in.wait_event(ev_done[i])                  # pcm_d[i] no longer read by its previous compute
        with torch.cuda.stream(s_in):
            pcm_d[i].copy_(pin_in, non_blocking=True)
            ev_in[i].record(s_in)
        cs.wait_event(ev_in[i])
        cs.wait_event(ev_out[i])                     # q_d[i] copied out by its previous D2H
        with torch.cuda.stream(cs):
            flag = q_d[i][nq:].view(torch.int32)
            flag.zero_()
            plans[b].compute(pcm_d[i], lens, rng.randbits2(nj), out=out_d[i], out_q=q_d[i][:nq].view(rows, D),
                             q_flag=flag, **mix[b])
            ev_done[i].record(cs)
        so = s_outs[b % nd]
        if host_issue:
            issue_jobs[i] = issue_pool.submit(issue_d2h, i, so)
        else:
            so.wait_event(ev_done[i])
            with torch.cuda.stream(so):
                q_h[i].copy_(q_d[i], non_blocking=True)
                ev_out[i].record(so)
        widen_jobs[i] = widen_pool.submit(widen, i)

    def xstep():
        par = it[0] % S
        it[0] += 1
        for b in range(B):
            xbatch(b, S * b + par)

    def xsync():                                     # the wall ends when the last codes are widened
        for j in widen_jobs:
            if j is not None:
                j.result()
        sync()

    cpu_dev = torch.device("cpu")
    from speech_recognition_tools_amd.shard import timed_steps
    t_go = [time.time()]

    def mark_start():
        widen_s[0] = 0.0
        t_go[0] = time.time()  # absolute start of the timed region (the ranks' children combine on the union)
    el_x = timed_steps(xstep, args.steps, args.warmup, xsync, dd, cpu_dev, before_timed=mark_start)
    widen_pool.shutdown()
    if issue_pool is not None:
        issue_pool.shutdown()
    flags = [int(q[nq:].view(torch.int32)[0]) for q in q_h]
    # the last step's widened codes equal the float32 rows still in HBM (bit-identical)
    par = (it[0] - 1) % S
    same = bool(np.array_equal(f_h[par].view(np.uint32), out_d[par].cpu().numpy().reshape(-1).view(np.uint32)))
    ah = world * args.steps * B * audio_s / 3600.0
    return {"value": ah / el_x, "ms_per_step": el_x / args.steps * 1e3, "audio_h": ah, "elapsed_s": el_x,
            "t_go": t_go[0],
            "h2d_bytes_per_step": int(B * pcm_host.nbytes), "d2h_bytes_per_step": int(B * (nq + 2) * 2),
            "d2h_encoding": "compact ark codes: int16 nearbyint(v * 1e3) + an int32 flag per batch (ABI 7)",
            "codes_flagged_batches": sum(1 for f in flags if f), "codes_widen_bit_identical": same,
            "host_widen_ms_per_step": widen_s[0] / args.steps * 1e3,
            "host_widen_note": "fdlp_q_widen of every batch's codes to the ark's float32 on 16 host threads, inside "
                               "the timed region (overlapped with the next steps' copies and kernels)",
            "note": "every batch's PCM copied in from pinned host memory, its compact feature codes copied back "
                    "and widened to float32 on the host, every step (%d batch(es) in flight on %d compute "
                    "stream(s), %d device buffer sets per batch used in turn, one H2D stream, %d D2H stream(s))"
                    % (B, len(comp), S, nd)}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="wsj", choices=["wsj", "reverb", "chime4"])
    ap.add_argument("--utts", type=int, default=1024, help="utterances per step per GPU (wsj workload)")
    ap.add_argument("--seconds", type=float, default=4.0, help="utterance length (wsj workload)")
    ap.add_argument("--support-eps", type=float, default=None)
    ap.add_argument("--cpu-workers", type=int, default=host_cores(),
                    help="CPU-baseline processes (default: every host core this process may use)")
    ap.add_argument("--cpu-per-worker", type=int, default=None,
                    help="utterances per CPU-baseline process (default: about 10 s of oracle time)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-transfers", action="store_true", help="skip the PCIe-inclusive timed pass")
    ap.add_argument("--xfer-d2h-streams", type=int, default=0,
                    help="PCIe pass: device-to-host copy streams (0: two in the child process that has its own "
                         "hardware queues, one in-process, where more streams share queues with the kernels)")
    ap.add_argument("--xfer-d2h-issue", choices=["stream", "host"], default="host",
                    help="PCIe pass: a batch's D2H copy is issued by a host thread once the batch's event has "
                         "completed (host, the default: no device-side wait) or waits for its kernels on the D2H "
                         "stream (stream: the copy's span falls into a 5.14 ms quantum as soon as two batches are in "
                         "flight, profiles/r06l_d2h_inflight.jsonl; ratio 0.79-0.85 against 0.91-0.93, r06s)")
    ap.add_argument("--xfer-hw-queues", type=int, default=8,
                    help="PCIe pass: every rank runs it in a child process (started before the rank touches the "
                         "GPU) with GPU_MAX_HW_QUEUES set to this (the compute, H2D and D2H streams then get hardware "
                         "queues of their own; 0: in-process, with the process default of 4)")
    ap.add_argument("--xfer-only", action="store_true", help=argparse.SUPPRESS)  # the PCIe-pass child
    ap.add_argument("--xfer-shard", default=None, help=argparse.SUPPRESS)  # rank/world of the child's shard
    ap.add_argument("--dct-path", default="auto", choices=["auto", "four_step"],
                    help="DCT stage: auto (one dct_frame_kernel per frame at N = 24000) or the four-step pair")
    ap.add_argument("--lpc-path", default="auto", choices=["auto", "lattice8", "lds"],
                    help="Durbin kernel (A/B): auto = durbin4_kernel for the recipes' p = 150")
    ap.add_argument("--inflight", type=int, default=4,
                    help="device batches in flight per GPU: independent plans on their own HIP streams, each "
                         "featurising its own batch every step (their kernels overlap on the device)")
    ap.add_argument("--workload", default=None, choices=["wsj", "librispeech", "reverb"],
                    help="wsj: --utts utterances of --seconds per GPU (configs[1], [3]); librispeech: U(1,30) s "
                         "(configs[4]); reverb: U(2,15) s reverberant sets (configs[2]); default from --config")
    ap.add_argument("--frames", type=int, default=4096, help="analysis frames per step per GPU (U(a,b) workloads)")
    ap.add_argument("--dry-run", action="store_true", help="launcher + sharding + reduction only, no device work")
    a = ap.parse_args(argv)
    if a.workload is None:
        a.workload = {"wsj": "wsj", "reverb": "reverb", "chime4": "wsj"}[a.config]
    return a


WORKLOAD_NAME = {("wsj", "wsj"): "wsj_si284_4s_batches", ("wsj", "librispeech"): "librispeech_960h_scale_u1_30s",
                 ("reverb", "reverb"): "reverb_et_real_1ch_8ch_u2_15s", ("chime4", "wsj"): "chime4_tr05_4s_babble20db"}


def workload_name(a):
    return WORKLOAD_NAME.get((a.config, a.workload), "%s_params_%s_lengths" % (a.config, a.workload))


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: --gpus %d, WORLD_SIZE %d: running %d ranks" % (args.gpus, world, world), file=sys.stderr)
    noise_host = babble_noise() if args.config == "chime4" else None

    import torch
    import torch.distributed as dist
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, NpRandom, PyRandom
    from speech_recognition_tools_amd.shard import shard_of, split_counts, timed_steps

    cfg = getattr(FeatureConfig, args.config)()
    if args.support_eps is not None:
        cfg.support_eps = args.support_eps
    probe = FdlpPlan(cfg, device=-1)
    # the PCIe-pass child of rank r of W measures that rank's shard (same utterances as its parent)
    s_rank, s_world = (int(v) for v in args.xfer_shard.split("/")) if args.xfer_shard else (rank, world)
    full = scp_list(args.workload, s_world, args.utts, args.seconds, args.frames, lambda t: probe.geometry(t)[0])
    mine = shard_of(full, s_rank, s_world)
    first = sum(split_counts(len(full), s_world)[:s_rank])

    # CPU baseline first (fork before any GPU initialisation in this process), rank 0 at N=1 only
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry_run:
        per = args.cpu_per_worker or (10 if args.config == "reverb" else 24)
        cpu = cpu_baseline(args.config, [t for _, t, _ in mine], args.cpu_workers, per, noise_host)
        cpu["workers_rule"] = ("--cpu-workers %d" % args.cpu_workers if args.cpu_workers != host_cores()
                               else "default: " + host_cores(with_rule=True)[1])

    # PCIe-inclusive pass of every rank in a child process (before this process touches the GPU):
    # GPU_MAX_HW_QUEUES is read once per process, and the headline keeps the process default.  The ranks'
    # children run at the same time, each on its own GPU, as the JOBs of a recipe run do.
    xfer_child = None
    use_child = not args.no_transfers and not args.xfer_only and args.xfer_hw_queues > 0
    if use_child and not args.dry_run:
        xfer_child = run_xfer_child(args, world, rank, local)

    if world > 1:  # host-side rendezvous: the only cross-rank traffic is a barrier and a max (no RCCL)
        dist.init_process_group("gloo", rank=rank, world_size=world)

    if args.dry_run:
        lens = [t for _, t, _ in mine]
        frames = sum(probe.geometry(t)[0] for t in lens)

        def step():
            pass
        sync = lambda: None
        elapsed = timed_steps(step, args.steps, args.warmup, sync, dist if world > 1 else None, torch.device("cpu"))
        shards = [None] * world
        child = None
        if use_child:
            cargv, cenv = xfer_child_spec(args, world, rank, local)
            child = {"argv": cargv, "env": {k: cenv.get(k) for k in ("GPU_MAX_HW_QUEUES", "HIP_VISIBLE_DEVICES")},
                     "rank_env_dropped": not any(k in cenv for k in RANK_ENV),
                     "before_gpu_init": "torch.cuda" not in sys.modules or not torch.cuda.is_initialized()}
        children = [None] * world
        if world > 1:
            dist.all_gather_object(shards, [first, first + len(mine), frames])
            dist.all_gather_object(children, child)
        else:
            shards = [[first, first + len(mine), frames]]
            children = [child]
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "audio-hours/s", "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                              "config": {"workload": workload_name(args)},
                              "scp_entries": len(full), "shards": shards, "elapsed_s": elapsed,
                              "xfer_children": children}))
        if world > 1:
            dist.destroy_process_group()
        return

    # one rank per GPU; more ranks than visible GPUs share them round-robin (a correctness check of the
    # N > 1 path on a small box, not a scaling measurement)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    # input synthesis (untimed): speech-like int16 PCM; REVERB: reverberated on the device, back as int16
    if args.workload == "reverb":
        pcm_host, lens = reverb_pcm(mine, dev)
    else:
        pcm_host = utterance_pcm(mine)
        lens = [t for _, t, _ in mine]
    geo = [probe.geometry(t) for t in lens]
    frames = sum(g[0] for g in geo)
    rows_out = sum(g[1] for g in geo)
    nj = sum(g[0] - 1 for g in geo)
    audio_s = sum(lens) / 16000.0

    plan = FdlpPlan(cfg, device=dev.index, max_frames=frames)
    _, lo, hi = probe.fbank()
    support = (hi - lo).astype(np.int64)

    pcm = torch.from_numpy(pcm_host).to(dev)
    out = torch.empty((rows_out, cfg.nfilters), dtype=torch.float32, device=dev)
    rng = PyRandom(7 + rank)
    sync = lambda: torch.cuda.synchronize(dev)
    dd = dist if world > 1 else None
    cpu_dev = torch.device("cpu")

    # B batches in flight: plan b (own workspace) featurises its own batch on its own stream every step;
    # the streams' kernels overlap on the device (the DCT and band kernels are latency-bound, the sweeps
    # VALU-bound).  Batch b holds the same utterance lengths with its own samples (the concatenated
    # signals rotated), and its own output buffer.
    B = max(1, args.inflight)
    plans = [plan] + [FdlpPlan(cfg, device=dev.index, max_frames=frames) for _ in range(B - 1)]
    for pl in plans:
        pl.set_dct_path(args.dct_path)
        pl.set_lpc_path(args.lpc_path)
    shifts = [7919 * b for b in range(B)]
    pcms = [pcm] + [torch.roll(pcm, shifts[b]) for b in range(1, B)]
    outs = [out] + [torch.empty_like(out) for _ in range(B - 1)]
    streams = [torch.cuda.Stream(dev) for _ in range(B)]
    # CHiME4: --add_noise babble,20 mixed inside the timed kernels; the per-utterance (offset, alpha) are
    # host-side descriptors of the batch (like its lengths), drawn once per batch in scp order
    mix = [{} for _ in range(B)]
    if noise_host is not None:
        noise_dev = torch.from_numpy(noise_host).to(dev)
        nr = NpRandom(31 + rank)
        for b in range(B):
            offs, alps = noise_mix(np.roll(pcm_host, shifts[b]), lens, noise_host, NOISE_SNR, nr)
            mix[b] = dict(noise=noise_dev, noise_off=offs, noise_alpha=alps)

    def step():
        plan.compute(pcm, lens, rng.randbits2(nj), out=out, **mix[0])

    def step_inflight():
        for b in range(B):
            with torch.cuda.stream(streams[b]):
                plans[b].compute(pcms[b], lens, rng.randbits2(nj), out=outs[b], **mix[b])

    # 1) headline: device-resident input and output, no profiling events.  warmup, barrier + sync,
    #    exactly K steps, sync + barrier, max over ranks (speech_recognition_tools_amd.shard)
    if args.xfer_only:
        elapsed = elapsed_one = elapsed_prof = None
    else:
        elapsed = timed_steps(step_inflight, args.steps, args.warmup, sync, dd, cpu_dev)

    # 1b) one batch in flight (the same steps with B = 1), reported beside the headline
    if not args.xfer_only:
        elapsed_one = timed_steps(step, args.steps, 1, sync, dd, cpu_dev) if B > 1 else elapsed

    # 2) one batch per step with per-stage HIP events on the stream the kernels run on (roofline: the
    #    kernels alone, not overlapped with another batch's)
    if not args.xfer_only:
        plan.set_profiling(True, kernels=True)
        elapsed_prof = timed_steps(step, args.steps, 0, sync, dd, cpu_dev)
        stages, ncalls = plan.stage_times()
        kern = plan.kernel_times()
        plan.set_profiling(False)

    # 3) PCIe-inclusive: PCM copied in from pinned host memory and float32 features back to pinned host
    #    memory, every batch of every step.  Every batch in flight has two device buffer sets used on
    #    alternate steps, so step s + 1's copy-in runs while step s computes and step s's copy-out while
    #    step s + 1 computes (with one set per batch, every step's four copy-ins queued behind the previous
    #    step's kernels on the one H2D stream: 31.9 ms per step against 23.4 computing, r03f).  One H2D
    #    and one D2H stream (--xfer-d2h-streams); the compute of batch b stays on its own stream.
    #    `mapped` = the OLA kernel stores the features straight into the pinned host buffer through its
    #    device mapping instead of a D2H copy (measured slower: reported, not used).
    if world > 1 and use_child:  # every rank's child result, or the in-process pass on every rank
        got = [None] * world
        dist.all_gather_object(got, xfer_child)
        xfer_child = combine_xfer_children(got)
    xfer = xfer_child
    if not args.no_transfers and xfer_child is None:
        xfer = pcie_pass(args, plans, streams, pcms, outs, pcm_host, lens, nj, rng, mix, audio_s, world, dd,
                         sync, dev, B)

    if args.xfer_only:
        xfer["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES", "default")
        print(json.dumps({"with_transfers": xfer}))
        return
    audio_h = world * args.steps * B * audio_s / 3600.0
    value = audio_h / elapsed
    ms_step = elapsed / args.steps * 1e3
    # dominant stage of the one-batch profiled pass (fdlp_stage_times: HIP events on the kernels' stream);
    # its algorithmic FLOPs are the useful work of the algorithm that stage runs (DESIGN.md "Measurement")
    sms = {k: v / max(ncalls, 1) for k, v in stages.items()}
    stage_ms = {"dct": sms["frames_dft1"] + sms["dft2_dct"], "autocorr": sms["autocorr"],
                "lpc_env": sms["lpc_env"], "ola_log": sms["ola_log"]}
    dom = max(stage_ms, key=stage_ms.get)
    # per-kernel HIP events of the same profiled pass: ms per launch of every kernel, and the dominant stage's
    # kernels summed (the roofline's time: the kernels themselves, comparable kernel by kernel with a rocprofv3
    # trace of the same command)
    kernel_ms = {k: ms / max(n, 1) for k, (ms, n) in kern.items()}
    kernel_launches_per_batch = {k: n / max(ncalls, 1) for k, (ms, n) in kern.items()}
    dom_prefixes = stage_kernel_prefixes(dom, plan.autocorr_path)
    dom_kernels = {k: v * kernel_launches_per_batch[k] for k, v in kernel_ms.items()
                   if any(k.startswith(pre) for pre in dom_prefixes)}
    items = frames * plan.B
    Me = min(cfg.coeff_num, 2 * plan.kk)
    stage_flops = {"dct": dct_flops(plan.N) * frames, "autocorr": autocorr_flops(plan, support) * frames,
                   "lpc_env": lpc_flops(cfg.order, cfg.coeff_num, Me, plan.kk) * items,
                   "ola_log": 2.0 * items * plan.kk}
    pmc_file = _latest_pmc(args.config if args.workload != "librispeech" else "librispeech") or PMC_FILE
    path = plan.autocorr_path
    traffic, bound = stage_pmc(stage_kernel_prefixes(dom, path), pmc_file)
    dom_ms = sum(dom_kernels.values()) if dom_kernels else stage_ms[dom]
    achieved = stage_flops[dom] / (dom_ms * 1e-3) / 1e12
    ac_can, whole_can = canonical_flops(plan.N, plan.B, cfg.order, cfg.coeff_num, plan.kk, 2 * plan.kk)
    # algorithmic HBM bytes (north_star / SURVEY 8(d)): int16 PCM in + float32 features out
    alg_bytes = float(B * (pcm_host.nbytes + out.numel() * 4))
    pmc_step = step_pmc_bytes(pmc_file)
    pmc_step = B * pmc_step if pmc_step else pmc_step  # B batches per step
    hbm = {"algorithmic_bytes_per_step": alg_bytes,
           "algorithmic_GBps": alg_bytes / (ms_step * 1e-3) / 1e9,
           "algorithmic_frac": alg_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "counter_bytes_per_step": pmc_step,
           "counter_GBps": pmc_step / (ms_step * 1e-3) / 1e9 if pmc_step else None,
           "counter_frac": pmc_step / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS if pmc_step else None,
           "peak_GBps": HBM_PEAK_GBS,
           "counter_source": "FETCH_SIZE x 2 + WRITE_SIZE summed over every kernel of one step, rocprofv3 PMC "
                             "passes of this command, %s" % os.path.relpath(pmc_file or "none", ROOT),
           "note": "the path is fp64-compute-bound; HBM does not bound it (SURVEY.md 8(d))"}
    desc = STAGE_DESC[dom]
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "audio-hours/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": workload_name(args),
                   "params": args.config,
                   "scp_entries_total": len(full),
                   "utts_per_step_per_gpu": B * len(lens),
                   "batches_in_flight": B,
                   "utts_per_batch": len(lens),
                   "utt_seconds": args.seconds if args.workload == "wsj" else "%s, mean %.2f" % (
                       "U(1,30)" if args.workload == "librispeech" else "U(2,15)", audio_s / max(len(lens), 1)),
                   "frames_per_step_per_gpu": B * frames, "nfilters": cfg.nfilters, "order": cfg.order,
                   "coeff_num": cfg.coeff_num, "coeff_range": cfg.coeff_range, "fbank": cfg.fbank_type,
                   "support_eps": cfg.support_eps, "autocorr_path": path, "dct_path": plan.dct_path,
                   "add_noise": "babble,%g (on the device, in the timed kernels)" % NOISE_SNR
                   if noise_host is not None else "clean",
                   "reverb_sets": ("1ch T60 0.7 s / 8ch_beamformit T60 0.35 s, synthetic RIRs applied by "
                                   "fdlp_reverb before timing" if args.workload == "reverb" else None),
                   "parallelism": "scp-shard x%d (contiguous split_scp shards, no collective)" % world},
        "roofline": {"bound": bound or "fp64-valu", "stage": dom,
                     "kernel": desc[path] if isinstance(desc, dict) else desc,
                     "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_unit": "bytes/launch (rocprofv3 PMC, %s)" % os.path.relpath(pmc_file or "none", ROOT),
                     "avg_launch_ms": dom_ms, "algorithmic_flops_per_launch": stage_flops[dom],
                     "timing": ("avg_launch_ms = the sum of the stage's kernels (kernel_ms_per_batch), each timed by "
                                "the HIP events recorded right before and after it on the stream it runs on "
                                "(fdlp_set_profiling(plan, 2) / fdlp_kernel_times), one batch in flight, mean over "
                                "the %d profiled steps of this run; achieved = algorithmic_flops_per_launch / "
                                "avg_launch_ms.  scripts/round_evidence.sh compares these kernel by kernel with a "
                                "rocprofv3 trace of the same command (<tag>_frac_check.json); stage_span_ms is the "
                                "per-stage event span (launch gaps included)" % args.steps),
                     "stage_kernels": list(stage_kernel_prefixes(dom, path)),
                     "kernel_ms_per_batch": dom_kernels,
                     "stage_span_ms": stage_ms[dom],
                     "stage_fracs": {k: stage_flops[k] / (stage_ms[k] * 1e-3) / 1e12 / FP64_PEAK_TFLOPS
                                     for k in stage_ms if stage_ms[k] > 0},
                     "canonical_frac": ac_can * frames / (sms["autocorr"] * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                     "canonical_frac_whole_step": whole_can * B * frames / (ms_step * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                     "canonical_note": "canonical = SURVEY.md 8(d) FFT-route FLOPs (%.1f MFLOP/frame autocorr, %.1f "
                                       "whole path); the exact structured algorithm runs ~5x fewer FLOPs than the FFT "
                                       "route, so canonical fractions can exceed 1 and are not a kernel-quality "
                                       "measure; frac uses the FLOPs the path actually runs" %
                                       (ac_can / 1e6, whole_can / 1e6)},
        "hbm": hbm,
        "stage_ms_per_step": sms,
        "kernel_ms_per_launch": kernel_ms,
        "ms_per_batch_profiled": elapsed_prof / args.steps * 1e3,
        "one_batch_in_flight": {"value": world * args.steps * audio_s / 3600.0 / elapsed_one,
                                "ms_per_step": elapsed_one / args.steps * 1e3,
                                "note": "the same steps with one batch per step (stage_ms_per_step and the "
                                        "roofline are per batch, from a one-batch profiled pass)"},
        "with_transfers": xfer,
        # SURVEY.md 8(d)'s wall "from the first H2D to the last D2H": the with_transfers pass; `value` above is
        # the task contract's figure (PCM and features resident in HBM)
        "sect8d_first_h2d_to_last_d2h": ({"value": xfer["value"], "unit": "audio-hours/s",
                                          "ratio_to_value": xfer["value"] / value} if xfer else None),
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
