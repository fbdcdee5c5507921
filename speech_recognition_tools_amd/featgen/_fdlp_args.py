"""Argument surface of compute-fdlp-feats (computeFDLPSpectrogram.py argparse :240-262 plus the MI355X
options) and the device choice, importable without numpy so a cold JOB can parse its argv and start
the HIP runtime (featgen/_early_hip.py) before the interpreter imports the heavy modules."""
import argparse
import os


def build_parser():
    parser = argparse.ArgumentParser('Extract FDLP Spectrogram.')
    parser.add_argument('scp', help='"scp" list')
    parser.add_argument('outfile', help='output file')
    parser.add_argument("--scp_type", default='wav', help="scp type can be 'wav' or 'segment'")
    parser.add_argument('--nfilters', type=int, default=20, help='number of filters (15)')
    parser.add_argument('--coeff_num', type=int, default=50, help='Total Number of coefficients to compute')
    parser.add_argument('--coeff_range', type=str, default='1,20', help="Range of Modulation coefficients to keep")
    parser.add_argument('--order', type=int, default=50, help='LPC filter order (50)')
    parser.add_argument('--fduration', type=float, default=0.5, help='Window length (0.5 sec)')
    parser.add_argument('--frate', type=int, default=100, help='Frame rate (100 Hz)')
    parser.add_argument('--overlap_fraction', type=float, default=0.25, help='Fraction of Overlap for OLA')
    parser.add_argument('--kaldi_cmd', default='copy-feats', help='Kaldi command to use to get ark files')
    parser.add_argument('--add_reverb', help='input "clean" OR "small_room" OR "large_room"')
    parser.add_argument('--fbank_type', type=str, default='mel,1',
                        help='mel,warp_fact OR cochlear,om_w,alpa,fixed,beta,warp_fact')
    parser.add_argument('--odd_mod_zero', action='store_true', help='Ignore the odd modulation coefficients')
    parser.add_argument('--gamma_weight', type=str, default='None', help='Configured as scale,shape,pk')
    parser.add_argument('--lifter_config', type=str, default=None, help='Configuration for general liftering')
    parser.add_argument("--write_utt2num_frames", action="store_true", help="Set to write utt2num_frames")
    parser.add_argument('--add_noise',
                        help='Specify "type of noise, snr", types: babble, buccaneer1, buccaneer2, car, '
                             'destroyerops, f16, factory1, factory2, m109, machinegun, pink, street, volvo, white')
    # MI355X additions (all optional)
    parser.add_argument('--seed', type=int, default=None, help='seed of the OLA hop jitter (random.seed)')
    parser.add_argument('--noise_seed', type=int, default=None, help='seed of the noise offsets (np.random.seed)')
    parser.add_argument('--device', type=int, default=None, help='HIP device (default: LOCAL_RANK or 0)')
    parser.add_argument('--device_rr', type=str, default=None,
                        help='"JOB,N": run on device (JOB-1) mod N (what make_FDLPspectrum_feats.sh --ngpu N '
                             'passes, so Kaldi $cmd array jobs spread over the GPUs)')
    parser.add_argument('--batch_frames', type=int, default=2048, help='analysis frames per GPU batch')
    parser.add_argument('--job_stats', action='store_true',
                        help='native runner: print the fdlp_job_stats of the JOB (timings of its phases) to stdout')
    parser.add_argument('--mapped_output', action='store_true',
                        help='native runner: the features go from the kernel straight into pinned host memory '
                             '(no D2H copy)')
    parser.add_argument('--ark_precision', type=int, default=3,
                        help="decimals of the reference's text ark ('%%.3f'); -1 keeps full float32")
    parser.add_argument('--support_eps', type=float, default=None,
                        help='filter taps below eps*peak are skipped in the autocorrelation (0 = exact)')
    parser.add_argument('--io_workers', type=int, default=4,
                        help='threads reading `<cmd> |` scp entries ahead of the device (plain files are read inline)')
    parser.add_argument('--cmvn_stats', type=str, default=None,
                        help='also write the global CMVN stats of the written features (Kaldi compute-cmvn-stats '
                             'format, accumulated on the device) to this file')
    parser.add_argument('--d2h_codes', choices=('auto', 'on', 'off'), default='auto',
                        help='native runner: features leave the device as int16 ark codes widened on the host '
                             '(auto: when --ark_precision is 0..3); the arks are byte-identical either way')
    parser.add_argument('--chunk_rows', type=int, default=0,
                        help='native runner: feature rows per device-to-host piece (0: 65536)')
    parser.add_argument('--keep_warm', action='store_true',
                        help='native runner: keep the plan and pinned buffers for the next getFeats call of '
                             'this process (same options)')
    parser.add_argument('--job_trace', type=str, default=None,
                        help='native runner: write the JOB pipeline events (JSON lines) to this file')
    parser.add_argument('--host_runner', choices=('native', 'python'), default='native',
                        help='native: the C++ JOB runner of libfdlp_hip.so (fdlp_job_run: reader threads, '
                             'pinned double-buffered batches, writer thread); python: the same loop in Python '
                             '(always used with --add_reverb)')
    return parser


def resolve_device(args):
    """--device, else --device_rr "JOB,N" -> (JOB-1) mod N, folded into the GPUs this process can see
    (a scheduler that gives each JOB its own GPU leaves it one: device 0), else LOCAL_RANK, else 0."""
    if args.device is not None:
        return int(args.device)
    if getattr(args, 'device_rr', None):
        from speech_recognition_tools_amd.shard import visible_gpu_count
        job, n = (int(v) for v in args.device_rr.split(','))
        if job < 1 or n < 1:
            raise ValueError('--device_rr needs JOB >= 1 and N >= 1')
        vis = visible_gpu_count()
        return (job - 1) % n % vis if vis > 0 else (job - 1) % n
    return int(os.environ.get("LOCAL_RANK", "0"))


def native_eligible(args, return_feats=False):
    """getFeats runs the native JOB runner (no torch object anywhere): the default host runner, no
    --add_reverb (its device convolution goes through torch tensors), features streamed to the ark."""
    return args.host_runner == 'native' and args.add_reverb in (None, '', 'clean') and not return_feats


def narrow_visible_devices(args, env=os.environ):
    """Before the HIP runtime starts: make the JOB's one GPU the only visible one (HIP_VISIBLE_DEVICES) and
    address it as device 0, so a cold JOB process on an 8-GPU node initialises one device instead of
    eight.  HIP_VISIBLE_DEVICES, if set, lists the candidates (its entries are kept, one is chosen); it
    indexes into ROCR_VISIBLE_DEVICES when that is set.  Returns the narrowed args (device = 0)."""
    dev = resolve_device(args)
    hip = env.get("HIP_VISIBLE_DEVICES")
    if hip is not None:
        ids = [x.strip() for x in hip.split(",") if x.strip()]
        if dev >= len(ids):
            return args  # out of range: let HIP report it
        env["HIP_VISIBLE_DEVICES"] = ids[dev]
    else:
        env["HIP_VISIBLE_DEVICES"] = str(dev)
    args.device, args.device_rr = 0, None
    return args
