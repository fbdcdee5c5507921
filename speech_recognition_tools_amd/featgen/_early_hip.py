"""Start the HIP runtime of a cold compute-fdlp-feats JOB on a helper thread.

A cold JOB process (make_FDLPspectrum_feats.sh:126-172 starts `nj` of them) spends ~0.2-0.25 s in the
HIP runtime's first calls (device enumeration, queues, the first copy; benchmarks/hip_init_probe.hip)
and ~0.1 s importing numpy and the package.  computeFDLPSpectrogram.py calls start(argv) before its
heavy imports: the argv is parsed with the real parser (featgen/_fdlp_args.py, no numpy), the JOB's GPU
is made the only visible one exactly as main() would do it, and a daemon thread loads the HIP runtime
(the libamdhip64.so.7 libfdlp_hip.so binds to) and makes one small allocation and copy ON THAT GPU, so
the runtime start overlaps the imports.  The ctypes calls release the GIL.  main() joins the thread
before exit.  Nothing happens unless the native JOB runner will run (no torch in the process, no
--add_reverb) and the argv parses cleanly (a usage error is main()'s to report, with no helper running).
"""
import ctypes
import os
import sys
import threading
import time

NARROWED = False   # HIP_VISIBLE_DEVICES was narrowed here (main() then addresses the GPU as device 0)
DEVICE = None      # the device index the helper warms (the JOB's own GPU among the visible ones)
T_START = None     # time.perf_counter() when the helper started / finished (the JOB's job_stats report them)
T_DONE = None
_thread = None


def _warm(dev):
    global T_DONE
    try:
        hip = ctypes.CDLL("libamdhip64.so.7")
        n = ctypes.c_int(0)
        if hip.hipGetDeviceCount(ctypes.byref(n)) != 0 or not 0 <= dev < n.value:
            return  # out of range: the JOB reports it from its own first HIP call
        if hip.hipSetDevice(dev) != 0:
            return
        p = ctypes.c_void_p()
        if hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(256)) != 0:
            return
        buf = ctypes.create_string_buffer(256)
        hip.hipMemcpy(p, buf, ctypes.c_size_t(256), 1)  # hipMemcpyHostToDevice
        hip.hipFree(p)
    except (OSError, AttributeError):
        pass  # no runtime here: the JOB reports it from its own first HIP call
    T_DONE = time.perf_counter()


def warm_target(argv, env=os.environ):
    """(device index the helper would warm, whether HIP_VISIBLE_DEVICES gets narrowed), or None when no
    helper runs (torch present, a usage error or unknown option, a non-native runner, a bad --device_rr).
    With CUDA_VISIBLE_DEVICES set the visible set is left alone (main() does the same) and the helper warms
    the device main() will use, resolve_device(args): never device 0 for a JOB that runs elsewhere."""
    if "torch" in sys.modules:
        return None
    from speech_recognition_tools_amd.featgen._fdlp_args import build_parser, native_eligible, resolve_device
    import contextlib
    import io
    try:
        with contextlib.redirect_stderr(io.StringIO()), contextlib.redirect_stdout(io.StringIO()):
            args, rest = build_parser().parse_known_args(argv)
    except SystemExit:
        return None  # -h or a usage error: main() prints it (once)
    if rest:
        return None  # unknown options: main()'s parse_args exits with status 2 before any GPU work
    try:
        if not native_eligible(args):
            return None
        dev = resolve_device(args)  # validates --device_rr like main() would
        if "CUDA_VISIBLE_DEVICES" in env:
            return dev, False
        return 0, True  # narrowed: the JOB's GPU is the only visible one, device 0
    except ValueError:
        return None  # main() raises it


def start(argv):
    global NARROWED, DEVICE, _thread, T_START
    if _thread is not None:
        return
    t = warm_target(argv)
    if t is None:
        return
    DEVICE, narrow = t
    if narrow:
        from speech_recognition_tools_amd.featgen._fdlp_args import build_parser, narrow_visible_devices
        args, _ = build_parser().parse_known_args(argv)
        narrow_visible_devices(args)  # the JOB's GPU becomes device 0 of this process
        NARROWED = True
    T_START = time.perf_counter()
    _thread = threading.Thread(target=_warm, args=(DEVICE,), name="hip-runtime-start", daemon=True)
    _thread.start()


def join():
    if _thread is not None:
        _thread.join()
