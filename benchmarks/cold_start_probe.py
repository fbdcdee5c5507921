#!/usr/bin/env python3
"""Where a cold compute-fdlp-feats JOB process spends its fixed cost (the recipe driver starts `nj` of
them, make_FDLPspectrum_feats.sh:126-172): interpreter + imports (no torch on the native path), loading
libfdlp_hip.so, HIP runtime start (first HIP call), plan creation (filterbank, tables, workspace), and the
first batch (kernel code-object loading) against a second, warm batch of the same utterances.

    python benchmarks/cold_start_probe.py      # run as its own (cold) process; prints one JSON line
"""
import time

T0 = time.perf_counter()
import ctypes  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import sys  # noqa: E402

import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    t = {"python_numpy_s": time.perf_counter() - T0}
    t1 = time.perf_counter()
    from speech_recognition_tools_amd import _hip_runtime
    _hip_runtime.TORCH = False
    from speech_recognition_tools_amd import _lib
    from speech_recognition_tools_amd.config import FeatureConfig
    t["import_lib_s"] = time.perf_counter() - t1
    hip = ctypes.CDLL("libamdhip64.so.7")
    t1 = time.perf_counter()
    n = ctypes.c_int()
    hip.hipGetDeviceCount(ctypes.byref(n))
    t["hip_runtime_start_s"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    hip.hipSetDevice(0)
    p = ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(p), 1 << 20)
    hip.hipDeviceSynchronize()
    t["device_open_s"] = time.perf_counter() - t1
    cfg = FeatureConfig.wsj()
    for key, mf, dev in (("plan_host_only_s", 2048, -1), ("plan_create_64_frames_s", 64, 0),
                         ("plan_create_s", 2048, 0)):
        t1 = time.perf_counter()
        c, keep = cfg.to_c(mf)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.fdlp_plan_create(ctypes.byref(c), dev, ctypes.byref(h)))
        t[key] = time.perf_counter() - t1
        ph = np.zeros(5)
        _lib.check(_lib.lib.fdlp_plan_setup_times(h, _lib.ptr(ph, ctypes.c_double)))
        t[key + "_phases(host,upload,lpc_setup,workspace,total)"] = [round(float(v), 4) for v in ph]
        if key != "plan_create_s":
            _lib.lib.fdlp_plan_destroy(h)
    # one batch of 64 x 4 s utterances, twice (the first one loads the kernels' code objects)
    from bench import utterance_pcm
    entries = [("u%d" % i, 64000, 10 + i) for i in range(64)]
    pcm = np.ascontiguousarray(utterance_pcm(entries))
    lens = np.full(64, 64000, dtype=np.int64)
    offs = np.arange(64, dtype=np.int64) * 64000
    F, L = ctypes.c_int32(), ctypes.c_int32()
    _lib.check(_lib.lib.fdlp_geometry(h, 64000, ctypes.byref(F), ctypes.byref(L)))
    rows = np.arange(64, dtype=np.int64) * L.value
    jit = np.zeros(64 * (F.value - 1), dtype=np.uint8)
    d_pcm, d_out = ctypes.c_void_p(), ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(d_pcm), pcm.nbytes)
    hip.hipMalloc(ctypes.byref(d_out), 64 * L.value * 80 * 4)
    hip.hipMemcpy(d_pcm, pcm.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(pcm.nbytes), 1)
    for key in ("first_batch_s", "warm_batch_s"):
        b = _lib.FdlpBatchC()
        b.n_utt, b.pcm_kind, b.pcm_dev = 64, _lib.FDLP_PCM_I16, d_pcm.value
        b.pcm_off, b.utt_len = _lib.ptr(offs, ctypes.c_int64), _lib.ptr(lens, ctypes.c_int64)
        b.jitter = _lib.ptr(jit, ctypes.c_uint8)
        b.out_dev, b.out_row, b.ark_decimals = d_out.value, _lib.ptr(rows, ctypes.c_int64), 3
        t1 = time.perf_counter()
        _lib.check(_lib.lib.fdlp_compute(h, ctypes.byref(b), None))
        hip.hipDeviceSynchronize()
        t[key] = time.perf_counter() - t1
    _lib.lib.fdlp_plan_destroy(h)
    t["total_s"] = time.perf_counter() - T0
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in t.items()}))


if __name__ == "__main__":
    main()
