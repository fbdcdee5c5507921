#!/usr/bin/env python3
"""compute-fdlp-feats: argv-compatible drop-in for
sadhusamik/speech_recognition_tools src/featgen/computeFDLPSpectrogram.py (argparse :240-262,
getFeats :29-237), running the FDLP pipeline on an MI355X through libfdlp_hip.so.

Same positional arguments, options, defaults, outputs (<outfile>.ark/.scp[/.len]) and
skip/abort semantics as the reference.  Differences (DESIGN.md "CLI"):
  * the ark/scp are written natively in Kaldi binary format (no copy-feats; --kaldi_cmd is
    accepted and ignored) with the reference's '%.3f' text-ark rounding (--ark_precision);
  * --seed / --noise_seed make the hop jitter (random.randrange) and noise offsets
    (np.random.rand) reproducible; unseeded runs draw seeds from os.urandom like the reference;
  * a failure to write the ark exits non-zero (the reference ignores copy-feats' status).
"""
import collections
import os
import sys
import time
from collections import OrderedDict

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if __name__ == "__main__":  # a cold JOB: the HIP runtime starts on a helper thread while numpy imports
    from speech_recognition_tools_amd.featgen import _early_hip
    _early_hip.start(sys.argv[1:])

import numpy as np

from speech_recognition_tools_amd.featgen._fdlp_args import (  # noqa: E402,F401  (the CLI's public names)
    build_parser, native_eligible, narrow_visible_devices, resolve_device)


def _read_scp_entry(line, scp_type):
    """(uttid, int16 samples, sr) or (uttid, None, None) on a read failure (skip, :129-154)."""
    from speech_recognition_tools_amd.io_pipeline import read_rx
    return read_rx(line, scp_type)


def getFeats(args, srate=16000, window=np.hamming, return_feats=True):
    """computeFDLPSpectrogram.py:29-237 on the device.  Returns {utt: features} (float32, as written to
    the ark) unless return_feats is False (the CLI: features are streamed to the ark only)."""
    if window is not np.hamming:
        raise ValueError("only the reference's np.hamming analysis window is supported")
    from speech_recognition_tools_amd.config import FeatureConfig
    from speech_recognition_tools_amd.featgen.features import add_noise_to_wav_params, load_noise

    wavs, scp_type, outfile = args.scp, args.scp_type, args.outfile
    add_noise, add_reverb = args.add_noise, args.add_reverb
    cfg = FeatureConfig.from_args(args)                                     # :43-63 (+ValueErrors)
    fbank_type = args.fbank_type.strip().split(',')
    if fbank_type[0] == "cochlear" and int(fbank_type[3]) == 1:
        print('%s: Alpha is fixed and will not change as a function of the center frequency...' % sys.argv[0])
    if args.odd_mod_zero:
        print('%s: Ignoring odd modulations... ' % sys.argv[0])
    noise = None
    diff = False
    if add_noise:                                                           # :68-73
        if add_noise == "clean" or add_noise == "diff":
            print('%s: No noise added!' % sys.argv[0])
            diff = add_noise == "diff"
        else:
            noise_info = add_noise.strip().split(',')
            noise = load_noise(noise_info[0])
            snr = float(noise_info[1])
    rir = None
    if add_reverb:                                                          # :75-91
        if add_reverb == 'clean':
            print('%s: No reverberation added!' % sys.argv[0])
        else:
            from speech_recognition_tools_amd.augment import load_rir
            rir = load_rir(add_reverb)                                      # ValueError for unknown rooms
    if not args.gamma_weight.strip().split(',')[0] == "None":
        print('%s: Adding gamma filter on modulation frequencies...' % sys.argv[0])
    if scp_type not in ('wav', 'segment'):
        raise ValueError('Invalid type of scp type, it should be either wav or segment')

    device = resolve_device(args)
    if getattr(args, 'host_runner', 'python') == 'native' and rir is None and not return_feats:
        return _run_native(args, cfg, device, noise, snr if noise is not None else 0.0, diff)
    import torch
    from speech_recognition_tools_amd import FdlpPlan, NpRandom, PyRandom
    torch.cuda.set_device(device)
    plan = FdlpPlan(cfg, device=device, max_frames=max(int(args.batch_frames), 1))
    jit_rng = PyRandom(args.seed)
    noise_rng = NpRandom(args.noise_seed) if noise is not None else None
    noise_dev = torch.from_numpy(np.ascontiguousarray(noise)).cuda(device) if noise is not None else None
    rir_dev = torch.from_numpy(np.ascontiguousarray(rir, dtype=np.float64)).cuda(device) if rir is not None else None
    cmvn = None
    if args.cmvn_stats:  # fused e2e/*/run_fdlp_e1.sh `compute-cmvn-stats` (speech_recognition_tools_amd.cmvn)
        from speech_recognition_tools_amd.cmvn import CmvnAccumulator
        cmvn = CmvnAccumulator(cfg.nfilters, device)
    from speech_recognition_tools_amd.io_pipeline import ArkStream, PrefetchReader

    all_feats = OrderedDict() if return_feats else None
    all_lens = OrderedDict()
    ark = ArkStream(outfile)                                                # :231 (streamed)
    # Two batches in flight: while the device works on one, the host reads/parses the next
    # (PrefetchReader threads) and writes the ark entries of the previous one.
    inflight = collections.deque()  # (entries, rows, host_out, event)
    pending = []  # (uttid, samples, F, noise_off, alpha)
    pending_frames = 0

    def complete(job):
        entries, rows, host, ev = job
        ev.synchronize()
        for i, x in enumerate(entries):
            feat = host[rows[i]:rows[i + 1]]
            ark.write(x[0], feat)
            if all_feats is not None:
                all_feats[x[0]] = feat.copy()                              # :227
            if args.write_utt2num_frames:
                all_lens[x[0]] = int(rows[i + 1] - rows[i])               # :228-229

    def flush():
        nonlocal pending, pending_frames
        if not pending:
            return
        sys.stdout.flush()
        lens = [x[1].shape[0] for x in pending]
        pcm_host = torch.from_numpy(np.concatenate([x[1] for x in pending])).pin_memory()
        pcm = pcm_host.to(torch.device("cuda", device), non_blocking=True)
        kw = {}
        if noise is not None:
            kw = dict(noise=noise_dev, noise_off=[x[3] for x in pending], noise_alpha=[x[4] for x in pending])
        pre = "diff" if diff else None
        offs = None
        if rir_dev is not None:  # :168-170 on the device; lengths can shrink by one (edge case)
            from speech_recognition_tools_amd.augment import reverb
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            pcm, lens = reverb(pcm, lens, rir_dev, offsets=offs, preprocess=pre, **kw)
            kw, pre = {}, None
        jit = np.concatenate([jit_rng.randbits2(plan.geometry(int(T))[0] - 1) for T in lens])
        out, rows, _ = plan.compute(pcm, lens, jit, offsets=offs, ark_decimals=args.ark_precision,
                                    preprocess=pre, **kw)
        if cmvn is not None:
            cmvn.add(out[:int(rows[-1])])
        host = torch.empty(out.shape, dtype=out.dtype, pin_memory=True)
        host.copy_(out, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        inflight.append((pending, rows, host.numpy(), ev))
        pending, pending_frames = [], 0
        while len(inflight) > 1:
            complete(inflight.popleft())

    sr = None
    n_lines = n_skipped = 0
    workers = max(1, int(getattr(args, 'io_workers', 4) or 1))
    try:
        for uttid, sig, sr_new in PrefetchReader(wavs, scp_type, workers=workers):   # :125
            n_lines += 1
            skip = sig is None
            if not skip:
                sr = sr_new
            if scp_type == 'wav':
                if sr is None:  # the reference hits a NameError on 'sr' here (:144)
                    raise NameError("name 'sr' is not defined")
                assert sr == srate, 'Input file has different sampling rate.'  # :144
            if skip:
                n_skipped += 1
                continue
            if sig.ndim != 1:
                raise ValueError("multi-channel WAV input is not supported (the reference expects mono)")
            if pending and pending[-1][1].dtype != sig.dtype:
                flush()  # a device batch holds one sample type (int16 or the float64 of other formats)
            T = sig.shape[0]
            F, _ = plan.geometry(T)
            if F < 1:
                raise ValueError("invalid number of data points (0) specified")
            off, alpha = 0, 0.0
            if noise is not None:                                           # :166
                off, alpha = add_noise_to_wav_params(sig, noise, snr, noise_rng.rand())
            # the reference's progress line; flushed once per device batch (flush()) rather than per
            # utterance, which cost ~20 us per line on 4 s utterances
            print('%s: Computing Features for file: %s' % (sys.argv[0], uttid))
            if pending_frames + F > plan.max_frames:
                flush()
            if F > plan.max_frames:
                while inflight:
                    complete(inflight.popleft())
                plan = FdlpPlan(cfg, device=device, max_frames=F)
            pending.append((uttid, sig, F, off, alpha))
            pending_frames += F
        flush()
        while inflight:
            complete(inflight.popleft())
    except BaseException:  # a failed JOB publishes no partial ark/scp (fdlp_ark_abort)
        ark.abort()
        raise
    finally:
        ark.close()
    if args.write_utt2num_frames:                                           # :232-237
        with open(outfile + '.len.tmp', 'w+') as file:
            for key, lens in all_lens.items():
                file.write("{:s} {:d}".format(key, lens))
                file.write("\n")
        os.replace(outfile + '.len.tmp', outfile + '.len')
    if cmvn is not None:
        from speech_recognition_tools_amd.cmvn import write_kaldi_dmatrix
        write_kaldi_dmatrix(args.cmvn_stats, cmvn.numpy(), binary=True)
    _report_skips(n_lines, n_skipped)
    return all_feats


def _report_skips(n_lines, n_skipped):
    """The reference skips unreadable entries silently (:135-142); here they are counted and reported,
    and a JOB in which every entry was skipped fails."""
    if n_skipped:
        print('%s: skipped %d of %d utterances (unreadable)' % (sys.argv[0], n_skipped, n_lines))
        sys.stdout.flush()
    if n_lines and n_skipped == n_lines:
        raise RuntimeError('every utterance of the scp was skipped (unreadable)')


def _seed_words(seed, n_random=624):
    """CPython random.seed key words (rng._int_key), or OS entropy like an unseeded random."""
    from speech_recognition_tools_amd.rng import _int_key
    if seed is None:
        return np.frombuffer(os.urandom(n_random * 4), dtype=np.uint32).copy()
    return np.asarray(_int_key(seed), dtype=np.uint32)


def _run_native(args, cfg, device, noise, snr, diff):
    """The JOB loop in libfdlp_hip.so (fdlp_job_run): reader threads, pinned batches with the copies and
    kernels of consecutive batches overlapped, writer thread; same outputs and semantics as the Python loop."""
    import ctypes
    from speech_recognition_tools_amd import _lib
    c, keep = cfg.to_c(max(int(args.batch_frames), 1))
    o = _lib.FdlpJobOptsC()
    o.scp_type = 0 if args.scp_type == 'wav' else 1
    o.write_len = int(bool(args.write_utt2num_frames))
    o.ark_decimals = int(args.ark_precision)
    o.batch_frames = max(int(args.batch_frames), 1)
    o.io_threads = max(1, int(getattr(args, 'io_workers', 4) or 1))
    o.preprocess = _lib.FDLP_PRE_DIFF if diff else _lib.FDLP_PRE_NONE
    hold = []
    if noise is not None:
        nz = np.ascontiguousarray(noise, dtype=np.int16)
        hold.append(nz)
        o.noise, o.noise_len, o.snr = _lib.ptr(nz, ctypes.c_int16), nz.size, float(snr)
        seed = args.noise_seed
        if seed is None:
            seed = int(np.frombuffer(os.urandom(4), dtype=np.uint32)[0])
        if not 0 <= int(seed) <= 0xFFFFFFFF:
            raise ValueError("Seed must be between 0 and 2**32 - 1")
        o.noise_seed = int(seed)
    key = _seed_words(args.seed)
    hold.append(key)
    o.jitter_key, o.jitter_key_len = _lib.ptr(key, ctypes.c_uint32), key.size
    o.srate = 16000
    # the reference's progress lines, from the C runtime's stdout (only when Python's stdout is the process's)
    o.progress_name = sys.argv[0].encode() if sys.stdout is sys.__stdout__ else None
    o.cmvn_path = args.cmvn_stats.encode() if args.cmvn_stats else None
    o.out_mapped = int(bool(getattr(args, 'mapped_output', False)))
    o.out_codes = {'auto': -1, 'on': 1, 'off': 0}[getattr(args, 'd2h_codes', 'auto')]
    o.chunk_rows = int(getattr(args, 'chunk_rows', 0) or 0)
    o.keep_warm = int(bool(getattr(args, 'keep_warm', False)))
    if o.keep_warm:
        _register_job_release()
    trace = getattr(args, 'job_trace', None)
    o.trace_path = trace.encode() if trace else None
    st = _lib.FdlpJobStatsC()
    sys.stdout.flush()
    t_call = time.time()
    rc = _lib.lib.fdlp_job_run(ctypes.byref(c), int(device), args.scp.encode(), args.outfile.encode(),
                               ctypes.byref(o), ctypes.byref(st))
    if rc != _lib.FDLP_OK:
        msg = _lib.lib.fdlp_last_error().decode("utf-8", "replace")
        if msg == "name 'sr' is not defined":
            raise NameError(msg)                                            # :144 before any read
        if msg == 'Input file has different sampling rate.':
            raise AssertionError(msg)                                       # :144
        _lib.check(rc)
    global LAST_JOB_STATS
    LAST_JOB_STATS = {k: getattr(st, k) for k, _ in st._fields_}
    LAST_JOB_STATS["call_seconds"] = time.time() - t_call  # includes the HIP runtime start of a cold process
    from speech_recognition_tools_amd.featgen import _early_hip
    if _early_hip.T_START is not None:  # the helper's runtime start, relative to the JOB call
        t0 = time.perf_counter() - LAST_JOB_STATS["call_seconds"]
        LAST_JOB_STATS["early_hip_start_s"] = _early_hip.T_START - t0
        LAST_JOB_STATS["early_hip_done_s"] = (_early_hip.T_DONE - t0) if _early_hip.T_DONE else None
    if getattr(args, 'job_stats', False):
        import json
        print('%s: job stats %s' % (sys.argv[0], json.dumps(LAST_JOB_STATS)))
    _report_skips(st.n_lines, st.n_skipped)
    return None


def _register_job_release():
    """--keep_warm parks the plan, streams and pinned slots in the library; include/fdlp.h asks for
    fdlp_job_release before the HIP runtime is torn down, so the process releases them at exit."""
    import atexit
    from speech_recognition_tools_amd import _lib
    # the flag lives in the library module: a JOB chain (featgen/job_chain.py) re-runs this file per JOB
    if getattr(_lib, "_job_release_registered", False):
        return
    atexit.register(_lib.lib.fdlp_job_release)
    _lib._job_release_registered = True


LAST_JOB_STATS = None  # fdlp_job_stats of the last native run (benchmarks/cli_throughput.py reports it)


def main(argv=None):
    from speech_recognition_tools_amd.featgen import _early_hip
    try:
        # inside the try: a usage error (SystemExit 2) still joins the helper thread first
        args = build_parser().parse_args(argv)
        if native_eligible(args) and "torch" not in sys.modules:
            from speech_recognition_tools_amd import _hip_runtime
            _hip_runtime.TORCH = False  # before anything loads libfdlp_hip.so: a cold JOB skips importing torch
            if _early_hip.NARROWED:  # _early_hip.start already narrowed HIP_VISIBLE_DEVICES to this JOB's GPU
                args.device, args.device_rr = 0, None
            elif "CUDA_VISIBLE_DEVICES" not in os.environ:
                args = narrow_visible_devices(args)
        start_time = time.time()
        print('%s: Extracting features....' % sys.argv[0])
        sys.stdout.flush()
        getFeats(args, return_feats=False)
        print('Execution Time: {t:.3f} seconds'.format(t=time.time() - start_time))
        sys.stdout.flush()
    finally:
        _early_hip.join()  # never leave the process while the helper is inside the HIP runtime start


if __name__ == '__main__':
    main()
