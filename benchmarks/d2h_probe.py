#!/usr/bin/env python3
"""Device-to-host copy rate of one batch's features under the PCIe pass's background load (an experiment
for DESIGN.md §6 "PCIe pass", not the bench line).  The copy (the compact codes of one 1024 x 4 s batch,
65.5 MB, or its float32 rows, 131 MB) is timed by HIP events on its own stream while the device runs:
  idle      nothing else
  h2d       a 131 MB host-to-device copy on another stream
  compute   four batches of fdlp_compute on four streams (the bench's batches in flight)
  both      compute + h2d
for the runtime's hipMemcpyAsync and for a copy kernel (benchmarks/d2h_copy.hip: device buffer -> pinned
host buffer through its device mapping, 16 bytes per lane) with W workgroups.  One JSON line per case.

    hipcc -O3 --offload-arch=gfx950 -shared -fPIC benchmarks/d2h_copy.hip -o benchmarks/libd2h_copy.so
    GPU_MAX_HW_QUEUES=8 python benchmarks/d2h_probe.py [--pipeline [--k=K] VARIANT...]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import scp_list, utterance_pcm
    from speech_recognition_tools_amd import FdlpPlan, FeatureConfig, PyRandom
    from speech_recognition_tools_amd._lib import lib
    kern = ctypes.CDLL(os.path.join(ROOT, "benchmarks", "libd2h_copy.so"))
    kern.d2h_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                              ctypes.c_void_p]
    cfg = FeatureConfig.wsj()
    probe = FdlpPlan(cfg, device=-1)
    full = scp_list("wsj", 1, 1024, 4.0, 4096, lambda t: probe.geometry(t)[0])
    lens = [t for _, t, _ in full]
    geo = [probe.geometry(t) for t in lens]
    frames, rows, nj = sum(g[0] for g in geo), sum(g[1] for g in geo), sum(g[0] - 1 for g in geo)
    dev = torch.device("cuda", 0)
    pcm_h = torch.from_numpy(utterance_pcm(full)).pin_memory()
    pcm = pcm_h.to(dev)
    K = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--k=")), 4))  # batches in flight
    plans = [FdlpPlan(cfg, device=0, max_frames=frames) for _ in range(K)]
    outs = [torch.empty((rows, cfg.nfilters), dtype=torch.float32, device=dev) for _ in range(K)]
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    rng = PyRandom(7)
    s_in, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    pcm_d2 = torch.empty_like(pcm)
    src = {"codes": torch.empty(rows * cfg.nfilters, dtype=torch.int16, device=dev).random_(-30000, 20000),
           "float32": outs[0].view(-1)}
    dst = {k: torch.empty(v.shape, dtype=v.dtype).pin_memory() for k, v in src.items()}

    def mapped(t):
        p = ctypes.c_void_p()
        assert lib.fdlp_mapped_ptr(ctypes.c_void_p(t.data_ptr()), ctypes.byref(p)) == 0
        return p.value

    def background(kind):
        if kind in ("h2d", "both"):
            with torch.cuda.stream(s_in):
                pcm_d2.copy_(pcm_h, non_blocking=True)
        if kind in ("compute", "both"):
            for b in range(K):
                with torch.cuda.stream(streams[b]):
                    plans[b].compute(pcm, lens, rng.randbits2(nj), out=outs[b])

    def one(kind, what, how, wgs=0, nt=1, reps=6, delay_ms=3.0, start="sleep"):
        rates = []
        for r in range(reps + 1):
            torch.cuda.synchronize(dev)
            background(kind)
            with torch.cuda.stream(s_out):
                if start == "sleep" and kind != "idle":
                    torch.cuda._sleep(int(delay_ms * 2.0e6))  # start the copy inside the background work
                elif start == "wait":  # after the first background kernels, like the PCIe pass's event waits
                    ev = torch.cuda.Event()
                    ev.record(streams[0])
                    s_out.wait_event(ev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s_out)
                if how == "runtime":
                    dst[what].copy_(src[what], non_blocking=True)
                else:
                    n = src[what].numel() * src[what].element_size()
                    assert kern.d2h_copy(src[what].data_ptr(), mapped(dst[what]), n, wgs, nt, s_out.cuda_stream) == 0
                e1.record(s_out)
            torch.cuda.synchronize(dev)
            if r:
                rates.append(src[what].numel() * src[what].element_size() / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        rates.sort()
        return dict(load=kind, data=what, copy=how, wgs=wgs, nt=nt, start=start, GBps_median=round(rates[len(rates) // 2], 2),
                    GBps_min=round(rates[0], 2), GBps_max=round(rates[-1], 2))

    if "--schedules" in sys.argv:
        schedules(torch, dev, plans, streams, pcm_h, lens, nj, rng, rows, cfg,
                  [v for v in sys.argv[1:] if not v.startswith("-")])
        return
    if "--pipeline" in sys.argv:
        pipeline(torch, dev, plans, streams, pcm_h, lens, nj, rng, rows, cfg, kern, mapped)
        return
    background("compute")
    torch.cuda.synchronize(dev)
    if "--starts" in sys.argv:
        for kind in ("idle", "compute", "both"):
            for start in ("none", "sleep", "wait"):
                print(json.dumps(one(kind, "codes", "runtime", start=start)), flush=True)
        return
    for kind in ("idle", "h2d", "compute", "both"):
        for what in ("codes", "float32"):
            print(json.dumps(one(kind, what, "runtime")), flush=True)
        for wgs in (16, 64, 256):
            print(json.dumps(one(kind, "codes", "kernel", wgs=wgs)), flush=True)
    print(json.dumps(one("both", "codes", "kernel", wgs=64, nt=0)), flush=True)
    # is the copy's result right (kernel path)
    assert torch.equal(dst["codes"], src["codes"].cpu())


def pipeline(torch, dev, plans, streams, pcm_h, lens, nj, rng, rows, cfg, kern, mapped, steps=10):
    """bench.py's PCIe pass (codes) with per-copy HIP events: where does the D2H go slow?  Variants of where
    the D2H is issued: 'stream' (bench: its own stream after an event wait), 'compute' (on the compute
    stream right after the batch), 'kernel64' (the copy kernel on the compute stream, 64 workgroups).
    A prefix 'h2dk<W>+' issues the host-to-device PCM copy as the copy kernel with W workgroups reading the
    pinned host buffer through its device mapping (on the H2D stream), so it leaves the SDMA engines to the
    device-to-host leg; 'h2dk<W>+none' is that H2D with no D2H."""
    import time
    K = len(plans)
    nq = rows * cfg.nfilters
    NB = 2 * K
    pcm_d = [torch.empty(pcm_h.shape, dtype=pcm_h.dtype, device=dev) for _ in range(NB)]
    out_d = [torch.empty((rows, cfg.nfilters), dtype=torch.float32, device=dev) for _ in range(NB)]
    nqa = (nq + 2 + 7) // 8 * 8  # codes + flag, padded to 16 bytes for the copy kernel
    q_d = [torch.empty(nqa, dtype=torch.int16, device=dev) for _ in range(NB)]
    q_h = [torch.empty(nqa, dtype=torch.int16).pin_memory() for _ in range(NB)]
    s_in = torch.cuda.Stream(dev)
    s_out = [torch.cuda.Stream(dev) for _ in range(8)]
    audio_h = sum(lens) / 16000.0 / 3600.0
    variants = [v for v in sys.argv[1:] if not v.startswith("-")] or ["stream", "compute", "kernel64"]
    same_stream = "--same-stream" in sys.argv  # every batch's kernels on one compute stream (serialised)
    for variant in variants + variants:
        ev_done = [torch.cuda.Event() for _ in range(NB)]
        ev_out = [torch.cuda.Event() for _ in range(NB)]
        ev_in = [torch.cuda.Event() for _ in range(NB)]
        for i in range(NB):
            ev_done[i].record(streams[i // 2])
            ev_out[i].record(streams[i // 2])
        marks = []
        it = [0]
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(1)
        issued = [None] * NB

        h2d, variant = variant.split("+", 1) if "+" in variant else ("", variant)
        h2d_wgs = int(h2d[4:]) if h2d.startswith("h2dk") else 0
        pcm_bytes = pcm_h.numel() * pcm_h.element_size()
        assert pcm_bytes % 16 == 0

        def xstep():
            par = it[0] & 1
            it[0] += 1
            for b in range(K):
                i = 2 * b + par
                cs = streams[0 if same_stream else b]
                s_in.wait_event(ev_done[i])
                with torch.cuda.stream(s_in):
                    if h2d_wgs:
                        assert kern.d2h_copy(mapped(pcm_h), pcm_d[i].data_ptr(), pcm_bytes, h2d_wgs, 1,
                                             s_in.cuda_stream) == 0
                    else:
                        pcm_d[i].copy_(pcm_h, non_blocking=True)
                    ev_in[i].record(s_in)
                cs.wait_event(ev_in[i])
                if issued[i] is not None:  # 'host': the copy-out of set i's last use was issued by the host thread
                    issued[i].result()
                cs.wait_event(ev_out[i])
                with torch.cuda.stream(cs):
                    flag = q_d[i][nq:nq + 2].view(torch.int32)
                    flag.zero_()
                    plans[b].compute(pcm_d[i], lens, rng.randbits2(nj), out=out_d[i], out_q=q_d[i][:nq].view(rows, -1),
                                     q_flag=flag)
                    ev_done[i].record(cs)
                if variant == "none":  # compute + H2D only: the floor
                    ev_out[i].record(cs)
                    continue
                sep = variant.startswith(("stream", "split")) or variant.endswith("s")
                nso = int(variant[6:]) if variant.startswith("stream") and variant[6:] else 2
                so = s_out[b % nso] if sep else cs
                if variant.startswith("hyb"):  # hyb<W>_<P>: the first P % by the copy kernel (W workgroups) on one
                    # stream, the rest by the runtime's copy (SDMA) on another, both after the batch
                    w_s, p_s = variant[3:].split("_")
                    nk = (nqa * int(p_s) // 100) // 8 * 8  # int16 elements, 16-byte pieces for the kernel
                    es, ee = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s_k, s_d = s_out[2 + (b % 2)], s_out[b % 2]
                    for sj in (s_k, s_d):
                        sj.wait_event(ev_done[i])
                    es.record(s_d)
                    if nk > 0:
                        assert kern.d2h_copy(q_d[i].data_ptr(), mapped(q_h[i]), nk * 2, int(w_s), 1, s_k.cuda_stream) == 0
                    with torch.cuda.stream(s_d):
                        q_h[i][nk:].copy_(q_d[i][nk:], non_blocking=True)
                    ek = torch.cuda.Event()
                    ek.record(s_k)
                    s_d.wait_event(ek)
                    ee.record(s_d)
                    ev_out[i].record(s_d)
                    marks.append((es, ee))
                    continue
                if variant.startswith("split"):  # each copy in k chunks on k streams
                    k = int(variant[5:])
                    es, ee = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    n = q_d[i].numel()
                    c = (n + k - 1) // k
                    parts = []
                    for j in range(k):
                        sj = s_out[j]
                        sj.wait_event(ev_done[i])
                        if j == 0:
                            es.record(sj)
                        with torch.cuda.stream(sj):
                            q_h[i][j * c:(j + 1) * c].copy_(q_d[i][j * c:(j + 1) * c], non_blocking=True)
                            e = torch.cuda.Event()
                            e.record(sj)
                            parts.append(e)
                    for e in parts:
                        s_out[0].wait_event(e)
                    ee.record(s_out[0])
                    ev_out[i].record(s_out[0])
                    marks.append((es, ee))
                    continue
                if variant == "host":  # a host thread waits for the batch, then issues the copy: no device-side wait
                    def copy_out(i=i, so=s_out[b % 2]):
                        ev_done[i].synchronize()
                        with torch.cuda.stream(so):
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record(so)
                            q_h[i].copy_(q_d[i], non_blocking=True)
                            e1.record(so)
                            ev_out[i].record(so)
                        marks.append((e0, e1))
                    issued[i] = pool.submit(copy_out)
                    continue
                if sep:
                    so.wait_event(ev_done[i])
                with torch.cuda.stream(so):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(so)
                    if variant.startswith("kernel"):
                        wgs = int(variant[6:].rstrip("s"))
                        assert kern.d2h_copy(q_d[i].data_ptr(), mapped(q_h[i]), nqa * 2, wgs, 1, so.cuda_stream) == 0
                    elif variant.startswith("dst"):  # D2H into the first k host buffers only (page reuse)
                        q_h[i % int(variant[3:].rstrip("s"))].copy_(q_d[i], non_blocking=True)
                    else:
                        q_h[i].copy_(q_d[i], non_blocking=True)
                    e1.record(so)
                    ev_out[i].record(so)
                    marks.append((e0, e1))

        def drain():
            for f in issued:
                if f is not None:
                    f.result()
            torch.cuda.synchronize(dev)

        for _ in range(2):
            xstep()
        drain()
        marks.clear()
        t0 = time.perf_counter()
        for _ in range(steps):
            xstep()
        drain()
        el = time.perf_counter() - t0
        pool.shutdown()
        ms = sorted(a.elapsed_time(b) for a, b in marks) or [0.0]
        if h2d_wgs:
            assert torch.equal(pcm_d[0].cpu(), pcm_h)
        print(json.dumps(dict(variant=(h2d + "+" if h2d else "") + variant, audio_h_per_s=round(steps * K * audio_h / el, 1),
                              ms_per_step=round(el / steps * 1e3, 2), d2h_ms_median=round(ms[len(ms) // 2], 3),
                              d2h_ms_max=round(ms[-1], 3), d2h_GBps_median=round(nq * 2 / max(ms[len(ms) // 2], 1e-6) / 1e6, 1))),
              flush=True)


def schedules(torch, dev, plans, streams, pcm_h, lens, nj, rng, rows, cfg, specs, steps=10):
    """The PCIe pass with other copy schedules: spec "h<H>d<D>s<S>" = H host-to-device streams (batch b on
    b mod H), D device-to-host streams (b mod D), S device buffer sets per batch in rotation (a batch's copy-in
    for step s + S - 1 can start while step s computes).  Codes out.  Prints audio-h/s per spec."""
    import re
    import time
    K = len(plans)
    nq = rows * cfg.nfilters
    audio_h = sum(lens) / 16000.0 / 3600.0
    S_max = 3
    pcm_d = [[torch.empty(pcm_h.shape, dtype=pcm_h.dtype, device=dev) for _ in range(S_max)] for _ in range(K)]
    out_d = [[torch.empty((rows, cfg.nfilters), dtype=torch.float32, device=dev) for _ in range(S_max)] for _ in range(K)]
    q_d = [[torch.empty(nq + 2, dtype=torch.int16, device=dev) for _ in range(S_max)] for _ in range(K)]
    q_h = [[torch.empty(nq + 2, dtype=torch.int16).pin_memory() for _ in range(S_max)] for _ in range(K)]
    s_in = [torch.cuda.Stream(dev) for _ in range(K)]
    s_out = [torch.cuda.Stream(dev) for _ in range(K)]
    for spec in specs + specs:
        H, D, S = (int(x) for x in re.match(r"h(\d+)d(\d+)s(\d+)", spec).groups())
        ev_in = [[torch.cuda.Event() for _ in range(S)] for _ in range(K)]
        ev_done = [[torch.cuda.Event() for _ in range(S)] for _ in range(K)]
        ev_out = [[torch.cuda.Event() for _ in range(S)] for _ in range(K)]
        for b in range(K):
            for j in range(S):
                ev_done[b][j].record(streams[b])
                ev_out[b][j].record(streams[b])
        it = [0]

        def xstep():
            j = it[0] % S
            it[0] += 1
            for b in range(K):
                si, so, cs = s_in[b % H], s_out[b % D], streams[b]
                si.wait_event(ev_done[b][j])
                with torch.cuda.stream(si):
                    pcm_d[b][j].copy_(pcm_h, non_blocking=True)
                    ev_in[b][j].record(si)
                cs.wait_event(ev_in[b][j])
                cs.wait_event(ev_out[b][j])
                with torch.cuda.stream(cs):
                    flag = q_d[b][j][nq:].view(torch.int32)
                    flag.zero_()
                    plans[b].compute(pcm_d[b][j], lens, rng.randbits2(nj), out=out_d[b][j],
                                     out_q=q_d[b][j][:nq].view(rows, -1), q_flag=flag)
                    ev_done[b][j].record(cs)
                so.wait_event(ev_done[b][j])
                with torch.cuda.stream(so):
                    q_h[b][j].copy_(q_d[b][j], non_blocking=True)
                    ev_out[b][j].record(so)

        for _ in range(2):
            xstep()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            xstep()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        print(json.dumps(dict(spec=spec, audio_h_per_s=round(steps * K * audio_h / el, 1),
                              ms_per_step=round(el / steps * 1e3, 2))), flush=True)


if __name__ == "__main__":
    main()
