"""ctypes binding of libfdlp_hip.so (include/fdlp.h).

torch is imported first on purpose: torch-ROCm ships its own libamdhip64.so.7 and the
dynamic linker then resolves this library's libamdhip64.so.7 dependency to that same copy,
so the process has ONE HIP runtime shared by torch tensors/streams and our kernels.

There is no fallback: if the library is missing the import raises.
"""
import ctypes
import os
import sys

from . import _hip_runtime

if _hip_runtime.TORCH or "torch" in sys.modules:
    import torch  # noqa: F401  (must precede the CDLL load, see module docstring)
TORCH_RUNTIME = "torch" in sys.modules  # the library shares torch's HIP runtime

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FDLP_LIB", os.path.join(_PKG, "lib", "libfdlp_hip.so"))

FDLP_OK = 0
FDLP_E_INVALID = -1
FDLP_E_HIP = -2
FDLP_E_NOMEM = -3
FDLP_E_CAPACITY = -4
FDLP_E_IO = -5
FDLP_E_BROADCAST = -6
FDLP_FBANK_MEL = 0
FDLP_FBANK_COCHLEAR = 1
FDLP_PCM_I16 = 0
FDLP_PCM_F64 = 1
FDLP_PRE_NONE = 0
FDLP_PRE_DIFF = 1
FDLP_NUM_STAGES = 5
FDLP_NUM_KERNELS = 16
FDLP_MODE_SPECTROGRAM = 0
FDLP_MODE_MODSPEC = 1
FDLP_MODE_MODSPEC_COMPLEX = 2
FDLP_WIN_HAMMING = 0
FDLP_WIN_HANNING = 1
FDLP_WIN_RECT = 2
ABI_VERSION = 9
FDLP_FN_LOG, FDLP_FN_EXP = 0, 1  # fdlp_device_fn
STAGE_NAMES = ("frames_dft1", "dft2_dct", "autocorr", "lpc_env", "ola_log")

c_i32, c_i64, c_dbl, c_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
P_i32 = ctypes.POINTER(c_i32)
P_i64 = ctypes.POINTER(c_i64)
P_dbl = ctypes.POINTER(c_dbl)
P_u8 = ctypes.POINTER(ctypes.c_uint8)
P_u32 = ctypes.POINTER(ctypes.c_uint32)
P_i16 = ctypes.POINTER(ctypes.c_int16)


class FdlpConfigC(ctypes.Structure):
    _fields_ = [
        ("nfilters", c_i32), ("coeff_num", c_i32), ("coeff_lp", c_i32), ("coeff_hp", c_i32),
        ("order", c_i32), ("frate", c_i32), ("srate", c_i32), ("fbank_kind", c_i32),
        ("fduration", c_dbl), ("overlap_fraction", c_dbl), ("warp_fact", c_dbl),
        ("om_w", c_dbl), ("alp", c_dbl), ("bet", c_dbl), ("fixed", c_i32),
        ("odd_mod_zero", c_i32), ("gamma_enabled", c_i32),
        ("gamma_scale", c_dbl), ("gamma_shape", c_dbl), ("gamma_pk", c_dbl),
        ("lifter", P_dbl), ("lifter_len", c_i32), ("support_eps", c_dbl), ("max_frames", c_i32),
        ("mode", c_i32), ("window", c_i32), ("coeff_0", c_i32), ("keep_even", c_i32),
        ("compensate_noise", c_i32), ("absolute_value", c_i32),
    ]


class FdlpBatchC(ctypes.Structure):
    _fields_ = [
        ("n_utt", c_i32), ("pcm_kind", c_i32), ("pcm_dev", c_p), ("pcm_off", P_i64),
        ("utt_len", P_i64), ("jitter", P_u8), ("noise_dev", c_p), ("noise_off", P_i64),
        ("noise_alpha", P_dbl), ("out_dev", c_p), ("out_row", P_i64), ("out_f64_dev", c_p),
        ("ark_decimals", c_i32), ("preprocess", c_i32), ("out_q_dev", c_p), ("out_q_flag_dev", c_p),
    ]


class FdlpMelConfigC(ctypes.Structure):
    _fields_ = [
        ("nfilters", c_i32), ("nfft", c_i32), ("frate", c_i32), ("srate", c_i32), ("fbank_kind", c_i32),
        ("fixed", c_i32), ("power", c_i32), ("fduration", c_dbl), ("warp_fact", c_dbl), ("om_w", c_dbl),
        ("alp", c_dbl), ("bet", c_dbl), ("max_frames", c_i32),
    ]


class FdlpReverbBatchC(ctypes.Structure):
    _fields_ = [
        ("n_utt", c_i32), ("pcm_kind", c_i32), ("pcm_dev", c_p), ("pcm_off", P_i64), ("utt_len", P_i64),
        ("preprocess", c_i32), ("noise_dev", c_p), ("noise_off", P_i64), ("noise_alpha", P_dbl),
        ("rir_dev", c_p), ("rir_len", c_i32), ("out_dev", c_p), ("out_len", P_i64),
    ]


class FdlpJobOptsC(ctypes.Structure):
    _fields_ = [
        ("scp_type", c_i32), ("write_len", c_i32), ("ark_decimals", c_i32), ("batch_frames", c_i32),
        ("io_threads", c_i32), ("preprocess", c_i32), ("noise", P_i16), ("noise_len", c_i64), ("snr", c_dbl),
        ("noise_seed", ctypes.c_uint32), ("jitter_key", P_u32), ("jitter_key_len", c_i32), ("srate", c_i32),
        ("progress_name", ctypes.c_char_p), ("cmvn_path", ctypes.c_char_p), ("out_mapped", c_i32),
        ("out_codes", c_i32), ("chunk_rows", c_i32), ("keep_warm", c_i32), ("trace_path", ctypes.c_char_p),
    ]


class FdlpJobStatsC(ctypes.Structure):
    _fields_ = [
        ("n_lines", c_i64), ("n_done", c_i64), ("n_skipped", c_i64), ("n_frames_out", c_i64),
        ("n_samples", c_i64), ("seconds", c_dbl), ("setup_seconds", c_dbl), ("read_wait_seconds", c_dbl),
        ("write_seconds", c_dbl), ("slot_wait_seconds", c_dbl), ("plan_seconds", c_dbl),
        ("pinned_seconds", c_dbl), ("d2h_wait_seconds", c_dbl), ("widen_seconds", c_dbl),
        ("n_batches", c_i64), ("n_code_fallbacks", c_i64), ("codes", c_i32), ("warm", c_i32),
    ]


# name -> (restype, argtypes); every function declared in include/fdlp.h
SIGNATURES = {
    "fdlp_plan_create": (c_i32, [ctypes.POINTER(FdlpConfigC), c_i32, ctypes.POINTER(c_p)]),
    "fdlp_plan_destroy": (c_i32, [c_p]),
    "fdlp_last_error": (ctypes.c_char_p, []),
    "fdlp_abi_version": (c_i32, []),
    "fdlp_mapped_ptr": (c_i32, [c_p, ctypes.POINTER(c_p)]),
    "fdlp_geometry": (c_i32, [c_p, c_i64, P_i32, P_i32]),
    "fdlp_plan_info": (c_i32, [c_p, P_i32, P_i32, P_i32, P_i32, P_i32]),
    "fdlp_plan_out_dim": (c_i32, [c_p, P_i32]),
    "fdlp_plan_fbank": (c_i32, [c_p, P_dbl, P_i32, P_i32]),
    "fdlp_plan_weights": (c_i32, [c_p, P_dbl]),
    "fdlp_make_fbank": (c_i32, [ctypes.POINTER(FdlpConfigC), c_i32, P_dbl, P_i32]),
    "fdlp_ola_table": (c_i32, [c_p, c_i64, P_u8, P_i32, P_i32, P_i32]),
    "fdlp_compute": (c_i32, [c_p, ctypes.POINTER(FdlpBatchC), c_p]),
    "fdlp_q_widen": (c_i32, [c_p, c_i64, c_i32, c_p, c_i32]),
    "fdlp_debug_fetch": (c_i32, [c_p, c_i32, P_dbl, P_dbl, P_dbl, P_dbl, P_dbl, P_dbl]),
    "fdlp_debug_fetch_range": (c_i32, [c_p, c_i32, c_i32, P_dbl, P_dbl, P_dbl, P_dbl, P_dbl, P_dbl]),
    "fdlp_set_profiling": (c_i32, [c_p, c_i32]),
    "fdlp_set_debug": (c_i32, [c_p, c_i32]),
    "fdlp_set_autocorr_path": (c_i32, [c_p, c_i32]),
    "fdlp_autocorr_path": (c_i32, [c_p]),
    "fdlp_plan_regions": (c_i32, [c_p, c_p, c_p]),
    "fdlp_plan_flat_events": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_i32]),
    "fdlp_set_lpc_path": (c_i32, [c_p, c_i32]),
    "fdlp_device_checks": (c_i32, [c_p, c_p, c_p, c_i32]),
    "fdlp_set_dct_path": (c_i32, [c_p, c_i32]),
    "fdlp_dct_path": (c_i32, [c_p]),
    "fdlp_set_pipeline": (c_i32, [c_p, c_i32]),
    "fdlp_stage_times": (c_i32, [c_p, P_dbl, P_i32]),
    "fdlp_kernel_times": (c_i32, [c_p, P_dbl, P_i64]),
    "fdlp_kernel_name": (ctypes.c_char_p, [c_i32]),
    "fdlp_plan_setup_times": (c_i32, [c_p, P_dbl]),
    "fdlp_dct_rows": (c_i32, [c_p, c_p, c_i32, c_p, c_p]),
    "fdlp_lpc_rows": (c_i32, [c_p, c_p, c_i32, c_p, c_p, c_p, c_p]),
    "fdlp_cepstrum_rows": (c_i32, [c_p, c_p, c_p, c_i32, c_i32, c_i32, c_p, c_p]),
    "fdlp_pyrandom_create": (c_i32, [P_u32, c_i32, ctypes.POINTER(c_p)]),
    "fdlp_pyrandom_randbits2": (c_i32, [c_p, c_i64, P_u8]),
    "fdlp_pyrandom_destroy": (c_i32, [c_p]),
    "fdlp_nprandom_create": (c_i32, [ctypes.c_uint32, ctypes.POINTER(c_p)]),
    "fdlp_nprandom_rand": (c_i32, [c_p, c_i64, P_dbl]),
    "fdlp_nprandom_destroy": (c_i32, [c_p]),
    "fdlp_noise_params": (c_i32, [P_i16, c_i64, P_i16, c_i64, c_dbl, c_dbl, P_i64, P_dbl]),
    "fdlp_noise_params_any": (c_i32, [P_dbl, c_i64, c_i32, P_i16, c_i64, c_dbl, c_dbl, P_i64, P_dbl]),
    "fdlp_wav_kind": (c_i32, [P_u8, c_i64, P_i32]),
    "fdlp_wav_parse": (c_i32, [P_u8, c_i64, P_i32, P_i32, ctypes.POINTER(P_i16), P_i64]),
    "fdlp_wav_decode": (c_i32, [P_u8, c_i64, P_i32, P_i32, P_i32, P_i64, P_dbl]),
    "fdlp_job_run": (c_i32, [ctypes.POINTER(FdlpConfigC), c_i32, ctypes.c_char_p, ctypes.c_char_p,
                             ctypes.POINTER(FdlpJobOptsC), ctypes.POINTER(FdlpJobStatsC)]),
    "fdlp_job_release": (c_i32, []),
    "fdlp_ark_open": (c_i32, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(c_p)]),
    "fdlp_ark_write": (c_i32, [c_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_float), c_i32, c_i32]),
    "fdlp_ark_close": (c_i32, [c_p]),
    "fdlp_ark_abort": (c_i32, [c_p]),
    "fdlp_device_fn": (c_i32, [c_i32, c_p, c_p, c_i64, c_p]),
    "fdlp_cmvn_accumulate": (c_i32, [c_p, c_i64, c_i32, c_p, c_p]),
    "fdlp_reverb": (c_i32, [ctypes.POINTER(FdlpReverbBatchC), c_p]),
    "fdlp_mel_plan_create": (c_i32, [ctypes.POINTER(FdlpMelConfigC), c_i32, ctypes.POINTER(c_p)]),
    "fdlp_mel_plan_destroy": (c_i32, [c_p]),
    "fdlp_mel_geometry": (c_i32, [c_p, c_i64, P_i32]),
    "fdlp_mel_compute": (c_i32, [c_p, ctypes.POINTER(FdlpBatchC), c_p]),
    "fdlp_mat_reader_open": (c_i32, [ctypes.c_char_p, ctypes.POINTER(c_p)]),
    "fdlp_mat_reader_next": (c_i32, [c_p, ctypes.POINTER(ctypes.c_char_p), P_i32, P_i32,
                                     ctypes.POINTER(ctypes.POINTER(ctypes.c_float))]),
    "fdlp_mat_reader_close": (c_i32, [c_p]),
    "fdlp_kaldi_write_dmatrix": (c_i32, [ctypes.c_char_p, P_dbl, c_i32, c_i32, c_i32]),
}


class FdlpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (fdlp code %d)" % (msg, code))
        self.code = code


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libfdlp_hip.so not built (%s); run __graft_entry__.build() or "
                          "python speech_recognition_tools_amd/_build.py" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fdlp_abi_version() != ABI_VERSION:
        raise ImportError("libfdlp_hip.so ABI mismatch")
    return lib


lib = _load()


def check(rc):
    if rc != FDLP_OK:
        msg = lib.fdlp_last_error()
        msg = msg.decode("utf-8", "replace") if msg else "unknown error"
        if rc == FDLP_E_BROADCAST:
            raise ValueError(msg)
        raise FdlpError(rc, msg)
    return rc


def ptr(arr, ctype):
    """numpy array -> ctypes pointer (arr must stay alive)."""
    return arr.ctypes.data_as(ctypes.POINTER(ctype))
