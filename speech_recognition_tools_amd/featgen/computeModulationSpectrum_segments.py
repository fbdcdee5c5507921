#!/usr/bin/env python3
"""compute-modspec-segment-feats: argv-compatible drop-in for sadhusamik/speech_recognition_tools
src/featgen/computeModulationSpectrum_segments.py (argparse :119-132, getFeats :24-116): FDLP modulation
spectra of the Kaldi segments of a recording scp, on an MI355X through the FDLP plan's modspec mode
(the same kernels as compute-modspec-feats).

What the reference does, and what this does the same way:
  * reads the whole wav.scp first (:57-63) and the segments file line by line (:66-71); a recording is
    re-read only when the segment's recording differs from the previous one (:73-82); a `<cmd> |` entry is
    not checked against 16 kHz, a file entry is (:82, the reference's own asymmetry);
  * segment samples signal_big[int(t_beg sr) : int(t_end sr)] / 2^15 (:84-86, numpy slicing), optional
    room reverberation (:88-90), Hanning frames (:24, :92-93), DCT / sqrt(2N) (:95), the mel filterbank
    of createFbank(nfilters, 2 fduration srate, srate) (:38), LPC of --order per band and the cepstrum
    c_0 .. c_{nmodulations-1} (:102-111, features.py:222-246), written band-major (:112);
  * --set_unity_gain sets the gain to 1 (:108-109): only c_0 = log(sqrt(gg)) depends on it, so c_0 = 0;
  * read errors are not caught (no skip, unlike computeModulationSpectrum.py).
Outputs <outfile>.ark/.scp ('%.3f' rounding of dict2Ark, features.py:63-69); --kaldi_cmd is accepted and
ignored.  Additions: --device, --batch_frames, --ark_precision.
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
    parser = argparse.ArgumentParser('Extract FDLP Modulation Spectral Features with segment files')
    parser.add_argument('scp', help='"scp" list')
    parser.add_argument('segment', help='segment file')
    parser.add_argument('outfile', help='output file')
    parser.add_argument('--nfilters', type=int, default=15, help='number of filters (15)')
    parser.add_argument('--nmodulations', type=int, default=12,
                        help='number of modulations of the modulation spectrum (12)')
    parser.add_argument('--order', type=int, default=50, help='LPC filter order (50)')
    parser.add_argument('--fduration', type=float, default=0.5, help='Window length (0.5 sec)')
    parser.add_argument('--frate', type=int, default=100, help='Frame rate (100 Hz)')
    parser.add_argument('--add_reverb', help='input "clean" OR "small_room" OR "large_room"')
    parser.add_argument('--set_unity_gain', action='store_true', help='Set LPC gain to 1 (True)')
    parser.add_argument('--kaldi_cmd', help='Kaldi command to use to get ark files (ignored: the ark is written natively)')
    # MI355X additions (all optional)
    parser.add_argument('--device', type=int, default=None, help='HIP device (default: LOCAL_RANK or 0)')
    parser.add_argument('--batch_frames', type=int, default=8192, help='analysis frames per GPU batch')
    parser.add_argument('--ark_precision', type=int, default=3, help="decimals of the text ark ('%%.3f')")
    return parser.parse_args(argv)


def feature_config(args, srate=16000):
    """getFeats :24-38 as a plan configuration: cepstrum slice [0, nmodulations), Hanning window, mel."""
    from speech_recognition_tools_amd.plan import FeatureConfig
    return FeatureConfig(mode="modspec", window="hanning", nfilters=args.nfilters, coeff_num=args.nmodulations,
                         coeff_0=1, order=args.order, fduration=args.fduration, frate=args.frate,
                         fbank_type="mel,1", keep_even=False, compensate_noise=False, absolute_value=False,
                         srate=srate)


def read_scp(path):
    """:57-63: recording ids and rxspecifiers, in order (blank lines ignored)."""
    ids, locs = [], []
    with open(path, 'r') as fid:
        for line in fid:
            tokens = line.strip().split()
            if not tokens:
                continue
            ids.append(tokens[0])
            locs.append(' '.join(tokens[1:]))
    return ids, locs


def segments_of(path):
    """(seg_id, recording_id, t_beg, t_end) of every non-blank segments line (:68-71, :84)."""
    with open(path, 'r') as fid:
        for line in fid:
            t = line.strip().split()
            if t:
                yield t[0], t[1], t[2], t[3]


def segment_signal(signal_big, sr, t_beg, t_end):
    """:84-86: samples [int(t_beg sr), int(t_end sr)) (numpy slicing) scaled by 2^-15, float64."""
    b, e = int(float(t_beg) * sr), int(float(t_end) * sr)
    return signal_big[b:e] / np.power(2, 15)


def get_feats(args, srate=16000, return_feats=False):
    """computeModulationSpectrum_segments.getFeats on the device; returns {seg_id: feats} when return_feats."""
    import torch
    from speech_recognition_tools_amd.augment import load_rir, reverb
    from speech_recognition_tools_amd.featgen.features import read_wav_bytes
    from speech_recognition_tools_amd.io_pipeline import ArkStream, read_rx_bytes
    from speech_recognition_tools_amd.plan import FdlpPlan

    cfg = feature_config(args, srate)
    rir = None
    if args.add_reverb:                                                        # :40-52
        if args.add_reverb == 'clean':
            print('%s: No reverberation added!' % sys.argv[0])
        elif args.add_reverb in ('small_room', 'large_room'):
            rir = load_rir(args.add_reverb)
        else:
            raise ValueError('Invalid type of reverberation!')
    wav_ids, wav_locs = read_scp(args.scp)
    device = args.device if args.device is not None else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    plan = FdlpPlan(cfg, device=device, max_frames=max(int(args.batch_frames), 1))
    rir_dev = torch.from_numpy(np.ascontiguousarray(rir, dtype=np.float64)).to(dev) if rir is not None else None
    B, nmod = args.nfilters, args.nmodulations

    feats_out = collections.OrderedDict() if return_feats else None
    ark = ArkStream(args.outfile)
    pending, pending_frames = [], 0

    def flush():
        nonlocal pending, pending_frames
        if not pending:
            return
        lens = [x[1].shape[0] for x in pending]
        pcm = torch.from_numpy(np.concatenate([x[1] for x in pending])).pin_memory().to(dev, non_blocking=True)
        offs = None
        if rir_dev is not None:                                                # :88-90
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            pcm, lens = reverb(pcm, lens, rir_dev, offsets=offs)
        out, rows, _ = plan.compute(pcm, lens, None, offsets=offs, ark_decimals=args.ark_precision)
        if args.set_unity_gain:                                                # :108-109: c_0 = log(sqrt(1))
            out.view(out.shape[0], B, nmod)[:, :, 0] = 0.0
        host = out.cpu().numpy()
        for i, x in enumerate(pending):
            m = host[rows[i]:rows[i + 1]]
            ark.write(x[0], m)
            if feats_out is not None:
                feats_out[x[0]] = m.copy()
        pending, pending_frames = [], 0

    try:
        wav_in_buffer, signal_big, sr = '', None, None
        for seg_id, wav_id, t_beg, t_end in segments_of(args.segment):
            if wav_in_buffer != wav_id:                                        # :73-82
                wav_in_buffer = wav_id
                inwav = wav_locs[wav_ids.index(wav_id)]
                sr, signal_big = read_wav_bytes(read_rx_bytes(inwav))
                if inwav[-1] != '|':
                    assert sr == srate, 'Input file has different sampling rate.'
            signal = np.ascontiguousarray(segment_signal(signal_big, sr, t_beg, t_end), dtype=np.float64)
            if signal.ndim != 1:
                raise ValueError("multi-channel WAV input is not supported (the reference expects mono)")
            F = plan.geometry(signal.shape[0])[0]
            print('%s: Computing Features for file: %s and segment: %s' % (sys.argv[0], wav_id, seg_id))
            sys.stdout.flush()
            if pending_frames + F > plan.max_frames:
                flush()
            if F > plan.max_frames:
                plan = FdlpPlan(cfg, device=device, max_frames=F)
            pending.append((seg_id, signal))
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
