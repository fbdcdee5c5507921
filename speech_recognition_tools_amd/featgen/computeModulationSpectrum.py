#!/usr/bin/env python3
"""compute-modspec-feats: argv-compatible drop-in for sadhusamik/speech_recognition_tools
src/featgen/computeModulationSpectrum.py (argparse :214-236, getFeats :30-205), the FDLP modulation-spectrum
feature, running on an MI355X: the FDLP plan in its modspec mode (fdlp_config.mode = FDLP_MODE_MODSPEC) shares
the frame/DCT/autocorrelation/lattice-LPC kernels of compute-fdlp-feats and ends in modspec_out_kernel
(cepstrum slice [coeff_0-1, coeff_n), keep_even, 1/f compensation, abs) instead of the envelope/OLA stage.

Same positional arguments, options, defaults and outputs (<outfile>.ark/.scp, '%.3f' rounding of dict2Ark,
features.py:63-69); the ark is written natively, --kaldi_cmd is accepted and ignored.  --complex_modulation
(the ifft/complex-LPC branch, :45-47/:74-88/:152-180) runs as the plan's FDLP_MODE_MODSPEC_COMPLEX (ifft
frames, complex autocorrelation + Hermitian Levinson + complex cepstrum kernels); with --keep_even it needs
--absolute_value (otherwise the reference fails with a broadcast error, and so does this).  --set_unity_gain
is accepted and, as in the reference, has no effect.  Additions: --device, --batch_frames, --io_workers,
--ark_precision.
"""
import argparse
import collections
import os
import sys
import time

import numpy as np

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def get_args(argv=None):
    parser = argparse.ArgumentParser('Extract FDLP Modulation Spectral Features.')
    parser.add_argument('scp', help='"scp" list')
    parser.add_argument('outfile', help='output file')
    parser.add_argument("--scp_type", default='wav', help="scp type can be 'wav' or 'segment'")
    parser.add_argument('--nfilters', type=int, default=15, help='number of filters (15)')
    parser.add_argument('--coeff_0', type=int, default=5, help='starting coefficient')
    parser.add_argument('--coeff_n', type=int, default=30, help='ending coefficient')
    parser.add_argument('--keep_even', action='store_true', help='Keep only even coefficients')
    parser.add_argument('--order', type=int, default=50, help='LPC filter order (50)')
    parser.add_argument('--fduration', type=float, default=0.5, help='Window length (0.5 sec)')
    parser.add_argument('--frate', type=int, default=100, help='Frame rate (100 Hz)')
    parser.add_argument('--add_reverb', help='input "clean" OR "small_room" OR "large_room"')
    parser.add_argument('--fbank_type', type=str, default='mel,1',
                        help='mel,warp_fact OR cochlear,om_w,alpa,fixed,beta,warp_fact')
    parser.add_argument('--set_unity_gain', action='store_true', help='Set LPC gain to 1 (True)')
    parser.add_argument('--no_window', action='store_true', help='Keeps the square window')
    parser.add_argument('--complex_modulation', action='store_true', help='Computes modulation by fft and not dct')
    parser.add_argument('--compensate_noise', action='store_true', help='Compensate 1/f noise in modulation spectrum')
    parser.add_argument('--absolute_value', action='store_true', help='Compute absolute value of modulation spectrum')
    parser.add_argument('--kaldi_cmd', help='Kaldi command to use to get ark files (ignored: the ark is written natively)')
    # MI355X additions (all optional)
    parser.add_argument('--device', type=int, default=None, help='HIP device (default: LOCAL_RANK or 0)')
    parser.add_argument('--batch_frames', type=int, default=8192, help='analysis frames per GPU batch')
    parser.add_argument('--io_workers', type=int, default=4, help='threads reading `<cmd> |` scp entries ahead (plain files are read inline)')
    parser.add_argument('--ark_precision', type=int, default=3, help="decimals of the text ark ('%%.3f')")
    return parser.parse_args(argv)


def feature_config(args, srate=16000):
    """getFeats :30-92 as a plan configuration."""
    from speech_recognition_tools_amd.plan import FeatureConfig
    return FeatureConfig(mode="modspec_complex" if args.complex_modulation else "modspec",
                         window="rect" if args.no_window else "hanning",
                         nfilters=args.nfilters, coeff_num=args.coeff_n, coeff_0=args.coeff_0, order=args.order,
                         fduration=args.fduration, frate=args.frate, fbank_type=args.fbank_type,
                         keep_even=bool(args.keep_even), compensate_noise=bool(args.compensate_noise),
                         absolute_value=bool(args.absolute_value), srate=srate)


def get_feats(args, srate=16000, return_feats=False):
    """computeModulationSpectrum.getFeats on the device; returns {uttid: feats} when return_feats."""
    import torch
    from speech_recognition_tools_amd.augment import load_rir, reverb
    from speech_recognition_tools_amd.io_pipeline import ArkStream, PrefetchReader
    from speech_recognition_tools_amd.plan import FdlpPlan

    cfg = feature_config(args, srate)
    fb = cfg.fbank_type.strip().split(',')
    if fb[0] == "cochlear" and len(fb) >= 6 and int(fb[3]) == 1:
        print('%s: Alpha is fixed and will not change as a function of the center frequency...' % sys.argv[0])
    if args.no_window:
        print('%s: Using square windows' % sys.argv[0])
    rir = None
    if args.add_reverb:                                                        # :94-106
        if args.add_reverb == 'clean':
            print('%s: No reverberation added!' % sys.argv[0])
        elif args.add_reverb in ('small_room', 'large_room'):
            rir = load_rir(args.add_reverb)
        else:
            raise ValueError('Invalid type of reverberation!')
    device = args.device if args.device is not None else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    max_frames = max(int(args.batch_frames), 1)
    plan = FdlpPlan(cfg, device=device, max_frames=max_frames)
    rir_dev = torch.from_numpy(np.ascontiguousarray(rir, dtype=np.float64)).to(dev) if rir is not None else None

    feats_out = collections.OrderedDict() if return_feats else None
    ark = ArkStream(args.outfile)
    pending, pending_frames = [], 0

    def frames_of(T):
        return plan.geometry(int(T))[0]

    def flush():
        nonlocal pending, pending_frames
        if not pending:
            return
        lens = [x[1].shape[0] for x in pending]
        pcm = torch.from_numpy(np.concatenate([x[1] for x in pending])).pin_memory().to(dev, non_blocking=True)
        offs = None
        if rir_dev is not None:                                                # :146-148
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            pcm, lens = reverb(pcm, lens, rir_dev, offsets=offs)
        out, rows, _ = plan.compute(pcm, lens, None, offsets=offs, ark_decimals=args.ark_precision)
        host = out.cpu().numpy()
        for i, x in enumerate(pending):
            m = host[rows[i]:rows[i + 1]]
            ark.write(x[0], m)
            if feats_out is not None:
                feats_out[x[0]] = m.copy()
        pending, pending_frames = [], 0

    try:
        for uttid, sig, sr in PrefetchReader(args.scp, args.scp_type, workers=args.io_workers):   # :108-140
            if args.scp_type == 'wav' and sig is not None:
                assert sr == srate, 'Input file has different sampling rate.'  # :130
            if sig is None:
                continue
            if sig.ndim != 1:
                raise ValueError("multi-channel WAV input is not supported (the reference expects mono)")
            F = frames_of(sig.shape[0])                                        # addReverb keeps <= T samples
            print('%s: Computing Features for file: %s, also %d' % (sys.argv[0], uttid, F))
            sys.stdout.flush()
            if pending_frames + F > plan.max_frames:
                flush()
            if F > plan.max_frames:
                plan = FdlpPlan(cfg, device=device, max_frames=F)
            pending.append((uttid, sig))
            pending_frames += F
        flush()
    except BaseException:  # a failed JOB publishes no partial ark/scp (fdlp_ark_abort)
        ark.abort()
        raise
    finally:
        ark.close()
    return feats_out


if __name__ == '__main__':
    args = get_args()
    start_time = time.time()
    print('%s: Extracting features....' % sys.argv[0])
    sys.stdout.flush()
    get_feats(args)
    print('Execution Time: {t:.3f} seconds'.format(t=time.time() - start_time))
    sys.stdout.flush()
