#!/usr/bin/env python3
"""compute-mel-feats: argv-compatible drop-in for sadhusamik/speech_recognition_tools
src/featgen/computeMelSpectrum.py (get_args :20-37, compute_mel_spectrum :40-170), the mel-spectrum
baseline feature of recipes/timit/local_pyspeech/make_melspectrum_feats.sh, running on an MI355X
(speech_recognition_tools_amd.melspec, mel_kernel).

Same positional arguments, options, defaults and outputs (<outfile>.ark/.scp[/.len]); the ark is written
natively with the reference's '%.3f' rounding (get_kaldi_ark, features.py:15-21).  Additions:
--noise_seed (np.random seed of the noise offsets), --device, --batch_frames, --io_workers, --ark_precision.
"""
import argparse
import collections
import os
import sys

import numpy as np

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def get_args(argv=None):
    parser = argparse.ArgumentParser('Extract Mel Energy Features')
    parser.add_argument('scp', help='scp file')
    parser.add_argument('outfile', help='output file')
    parser.add_argument("--scp_type", default='wav', help="scp type can be 'wav' or 'segment'")
    parser.add_argument("--spectrum_type", default="log", help="log/power For log spectrum or energy spectrum")
    parser.add_argument('--nfilters', type=int, default=23, help='number of filters (30)')
    parser.add_argument('--fduration', type=float, default=0.02, help='Window length (0.02 sec)')
    parser.add_argument('--frate', type=int, default=100, help='Frame rate (100 Hz)')
    parser.add_argument('--nfft', type=int, default=1024, help='Number of points of computing FFT')
    parser.add_argument('--add_reverb', help='input "clean" OR "small_room" OR "large_room"')
    parser.add_argument('--fbank_type', type=str, default='mel,1',
                        help='mel,warp_fact OR cochlear,om_w,alpa,fixed,beta,warp_fact')
    parser.add_argument("--write_utt2num_frames", action="store_true", help="Set to write utt2num_frames")
    parser.add_argument('--add_noise',
                        help='Specify "type of noise, snr", types: babble, buccaneer1, buccaneer2, car, destroyerops, '
                             'f16, factory1, factory2, m109, machinegun, pink, street, volvo, white')
    # MI355X additions (all optional)
    parser.add_argument('--noise_seed', type=int, default=None, help='seed of the noise offsets (np.random.seed)')
    parser.add_argument('--device', type=int, default=None, help='HIP device (default: LOCAL_RANK or 0)')
    parser.add_argument('--batch_frames', type=int, default=65536, help='frames per GPU batch')
    parser.add_argument('--io_workers', type=int, default=4, help='threads reading `<cmd> |` scp entries ahead (plain files are read inline)')
    parser.add_argument('--ark_precision', type=int, default=3, help="decimals of the text ark ('%%.3f')")
    return parser.parse_args(argv)


def compute_mel_spectrum(args, srate=16000, window=np.hamming, return_feats=False):
    """computeMelSpectrum.py:40-170 on the device."""
    if window is not np.hamming:
        raise ValueError("only the reference's np.hamming analysis window is supported")
    import torch
    from speech_recognition_tools_amd import NpRandom
    from speech_recognition_tools_amd.augment import load_rir, reverb
    from speech_recognition_tools_amd.featgen.features import add_noise_to_wav_params, load_noise
    from speech_recognition_tools_amd.io_pipeline import ArkStream, PrefetchReader
    from speech_recognition_tools_amd.melspec import MelConfig, MelPlan

    cfg = MelConfig(nfilters=args.nfilters, fduration=args.fduration, frate=args.frate, nfft=args.nfft,
                    fbank_type=args.fbank_type, spectrum_type=args.spectrum_type, srate=srate)
    cfg.to_c(1)                                                              # :53-67 ValueErrors up front
    add_noise, add_reverb = args.add_noise, args.add_reverb
    noise = None
    if add_noise and add_noise not in ("clean", "diff"):                    # :69-72
        noise_info = add_noise.strip().split(',')
        noise = load_noise(noise_info[0])
        snr = float(noise_info[1])
    rir = None
    if add_reverb:                                                           # :74-90
        if add_reverb == 'clean':
            print('%s: No reverberation added!' % sys.argv[0])
        else:
            rir = load_rir(add_reverb)
    device = args.device if args.device is not None else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(device)
    plan = MelPlan(cfg, device=device, max_frames=max(int(args.batch_frames), 1))
    dev = torch.device("cuda", device)
    noise_rng = NpRandom(args.noise_seed) if noise is not None else None
    noise_dev = torch.from_numpy(np.ascontiguousarray(noise)).to(dev) if noise is not None else None
    rir_dev = torch.from_numpy(np.ascontiguousarray(rir, dtype=np.float64)).to(dev) if rir is not None else None
    diff = add_noise == "diff"

    feats_out = collections.OrderedDict() if return_feats else None
    all_lens = collections.OrderedDict()
    ark = ArkStream(args.outfile)
    pending, pending_frames = [], 0

    def flush():
        nonlocal pending, pending_frames
        if not pending:
            return
        lens = [x[1].shape[0] for x in pending]
        pcm = torch.from_numpy(np.concatenate([x[1] for x in pending])).pin_memory().to(dev, non_blocking=True)
        kw = {}
        if noise is not None:
            kw = dict(noise=noise_dev, noise_off=[x[2] for x in pending], noise_alpha=[x[3] for x in pending])
        pre = "diff" if diff else None
        offs = None
        if rir_dev is not None:                                              # :143-145
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            pcm, lens = reverb(pcm, lens, rir_dev, offsets=offs, preprocess=pre, **kw)
            kw, pre = {}, None
        out, rows, _ = plan.compute(pcm, lens, offsets=offs, preprocess=pre, ark_decimals=args.ark_precision, **kw)
        host = out.cpu().numpy()
        for i, x in enumerate(pending):
            m = host[rows[i]:rows[i + 1]]
            ark.write(x[0], m)
            if feats_out is not None:
                feats_out[x[0]] = m.copy()
            all_lens[x[0]] = int(rows[i + 1] - rows[i])
        pending, pending_frames = [], 0

    try:
        for uttid, sig, sr in PrefetchReader(args.scp, args.scp_type, workers=args.io_workers):   # :98-130
            print('%s: Computing Features for file: %s' % (sys.argv[0], uttid))
            sys.stdout.flush()
            if args.scp_type == 'wav' and sig is not None:
                assert sr == srate, 'Input file has different sampling rate.'   # :120
            if sig is None:
                continue
            if sig.ndim != 1:
                raise ValueError("multi-channel WAV input is not supported (the reference expects mono)")
            off, alpha = 0, 0.0
            if noise is not None:                                            # :141
                off, alpha = add_noise_to_wav_params(sig, noise, snr, noise_rng.rand())
            F = plan.frames(sig.shape[0])
            if pending_frames + F > plan.max_frames:
                flush()
            if F > plan.max_frames:
                plan = MelPlan(cfg, device=device, max_frames=F)
            pending.append((uttid, sig, off, alpha))
            pending_frames += F
        flush()
    except BaseException:  # a failed JOB publishes no partial ark/scp (fdlp_ark_abort)
        ark.abort()
        raise
    finally:
        ark.close()
    if args.write_utt2num_frames:                                            # :165-170
        with open(args.outfile + '.len', 'w+') as file:
            for key, lens in all_lens.items():
                file.write("{:s} {:d}".format(key, lens))
                file.write("\n")
    return feats_out


if __name__ == '__main__':
    compute_mel_spectrum(get_args())
