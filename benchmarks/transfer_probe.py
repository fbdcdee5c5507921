#!/usr/bin/env python3
"""Host<->device copy rates behind bench.py's PCIe-inclusive pass (`with_transfers`).

Times, on one GPU, with the bench's buffer sizes (1024 x 4 s int16 PCM in, float32 features out):
  h2d       pinned host -> device, alone
  d2h       device -> pinned host, alone
  both      one of each at once, on two streams
  compute   plan.compute on device-resident buffers
  xstep     bench.py's double-buffered copy-in / compute / copy-out step
Prints one JSON line (GB/s per copy kind, ms per step).

    python benchmarks/transfer_probe.py [--utts 1024] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=1024)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only-xstep", action="store_true", help="time only the double-buffered step (for traces)")
    ap.add_argument("--split-probe", action="store_true",
                    help="D2H / H2D rates with each copy split into K chunks on K streams (K = 1, 2, 4, 8), "
                         "alone and with both directions at once")
    ap.add_argument("--d2h-variants", action="store_true",
                    help="device->host copy into differently allocated host buffers (hipMemcpyAsync): alone, "
                         "and overlapped with one compute step")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, PyRandom

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = FeatureConfig.wsj()
    T = int(round(a.seconds * 16000))
    probe = FdlpPlan(cfg, device=-1)
    F, L = probe.geometry(T)
    lens = [T] * a.utts
    pcm_host = bench.speech_like_batch(a.utts, T, 1000).reshape(-1)
    plan = FdlpPlan(cfg, device=0, max_frames=F * a.utts)
    pin_in = torch.from_numpy(pcm_host).pin_memory()
    pcm_d = [pin_in.to(dev), pin_in.to(dev)]
    out_d = [torch.empty((L * a.utts, cfg.nfilters), dtype=torch.float32, device=dev) for _ in range(2)]
    out_h = [torch.empty(out_d[0].shape, dtype=torch.float32).pin_memory() for _ in range(2)]
    rng = PyRandom(7)
    nj = a.utts * (F - 1)
    s_in, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    comp = torch.cuda.current_stream(dev)

    def timeit(fn, reps):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps

    def h2d():
        with torch.cuda.stream(s_in):
            pcm_d[1].copy_(pin_in, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s_out):
            out_h[1].copy_(out_d[1], non_blocking=True)

    def both():
        h2d()
        d2h()

    def compute():
        plan.compute(pcm_d[0], lens, rng.randbits2(nj), out=out_d[0])

    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_done = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]
    for e in ev_done + ev_out:
        e.record(comp)
    it = [0]

    def xstep():  # the same schedule as bench.py's PCIe-inclusive pass
        b = it[0] & 1
        it[0] += 1
        s_in.wait_event(ev_done[b])
        with torch.cuda.stream(s_in):
            pcm_d[b].copy_(pin_in, non_blocking=True)
            ev_in[b].record(s_in)
        comp.wait_event(ev_in[b])
        comp.wait_event(ev_out[b])
        plan.compute(pcm_d[b], lens, rng.randbits2(nj), out=out_d[b])
        ev_done[b].record(comp)
        s_out.wait_event(ev_done[b])
        with torch.cuda.stream(s_out):
            out_h[b].copy_(out_d[b], non_blocking=True)
            ev_out[b].record(s_out)

    nb_in = pin_in.numel() * pin_in.element_size()
    nb_out = out_d[0].numel() * 4
    if a.split_probe:
        res = {"sdma": os.environ.get("HSA_ENABLE_SDMA", "default")}
        so = [torch.cuda.Stream(dev) for _ in range(8)]
        si = [torch.cuda.Stream(dev) for _ in range(8)]
        src_o, dst_o = out_d[1].view(-1), out_h[1].view(-1)
        src_i, dst_i = pin_in.view(-1), pcm_d[1].view(-1)

        def chunks(n, k):
            step = (n + k - 1) // k
            return [(i, min(n, i + step)) for i in range(0, n, step)]

        for k in (1, 2, 4, 8):
            def d2h_k():
                for q, (lo, hi) in enumerate(chunks(src_o.numel(), k)):
                    with torch.cuda.stream(so[q]):
                        dst_o[lo:hi].copy_(src_o[lo:hi], non_blocking=True)

            def h2d_k():
                for q, (lo, hi) in enumerate(chunks(src_i.numel(), k)):
                    with torch.cuda.stream(si[q]):
                        dst_i[lo:hi].copy_(src_i[lo:hi], non_blocking=True)

            def both_k():
                h2d_k()
                d2h_k()

            t_o, t_i, t_b = timeit(d2h_k, a.reps), timeit(h2d_k, a.reps), timeit(both_k, a.reps)
            res["k%d" % k] = {"d2h_GBps": round(nb_out / t_o / 1e9, 2), "h2d_GBps": round(nb_in / t_i / 1e9, 2),
                              "both_GBps": round((nb_in + nb_out) / t_b / 1e9, 2)}
        print(json.dumps(res))
        return
    if a.d2h_variants:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
        hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        res = {}
        keep = []
        for name, how, flags in (("hostmalloc_default", "malloc", 0x0), ("hostmalloc_noncoherent", "malloc", 0x80000000),
                                 ("hostmalloc_coherent", "malloc", 0x40000000), ("register", "register", 0x0)):
            if how == "malloc":
                ptr = ctypes.c_void_p()
                if hip.hipHostMalloc(ctypes.byref(ptr), nb_out, flags) != 0:
                    res[name] = "alloc failed"
                    continue
                hp = ptr.value
            else:
                buf = np.empty(nb_out, np.uint8)
                keep.append(buf)
                if hip.hipHostRegister(buf.ctypes.data, nb_out, flags) != 0:
                    res[name] = "register failed"
                    continue
                hp = buf.ctypes.data

            def d2h_v():
                hip.hipMemcpyAsync(hp, out_d[1].data_ptr(), nb_out, 2, ctypes.c_void_p(s_out.cuda_stream))

            def overl():
                d2h_v()
                compute()

            t_alone = timeit(d2h_v, a.reps)
            t_ov = timeit(overl, a.reps)
            res[name] = {"d2h_GBps": nb_out / t_alone / 1e9, "d2h_plus_compute_ms": t_ov * 1e3}
        res["compute_ms"] = timeit(compute, a.reps) * 1e3
        print(json.dumps(res))
        return
    if a.only_xstep:
        t_x = timeit(xstep, a.reps)
        print(json.dumps({"xstep_ms": t_x * 1e3}))
        return
    t_h2d = timeit(h2d, a.reps)
    t_d2h = timeit(d2h, a.reps)
    t_both = timeit(both, a.reps)
    t_comp = timeit(compute, a.reps)
    t_x = timeit(xstep, a.reps)
    audio_h = a.utts * a.seconds / 3600.0
    print(json.dumps({
        "h2d_bytes": nb_in, "d2h_bytes": nb_out,
        "h2d_GBps": nb_in / t_h2d / 1e9, "d2h_GBps": nb_out / t_d2h / 1e9,
        "both_ms": t_both * 1e3, "both_GBps": (nb_in + nb_out) / t_both / 1e9,
        "compute_ms": t_comp * 1e3, "xstep_ms": t_x * 1e3,
        "compute_audio_h_per_s": audio_h / t_comp, "xstep_audio_h_per_s": audio_h / t_x}))


if __name__ == "__main__":
    main()
