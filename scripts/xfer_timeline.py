#!/usr/bin/env python3
"""Copy/compute timeline of the last part of a rocprofv3 --kernel-trace --memory-copy-trace database (the
bench's PCIe pass): every memory copy (direction, size, rate), every blit kernel (__amd_rocclr_*), and per
compute batch its span from the first kernel (the DCT) to the last (OLA + log) with its queue, then a
summary: busy time of the copy directions and of the compute queues over the window.

    python scripts/xfer_timeline.py <run_results.db> [window_ms]
"""
import sqlite3
import sys


def union_ms(iv):
    iv = sorted(iv)
    tot, cs, ce = 0.0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot / 1e6


def main(db, win_ms=120.0):
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    view = next(v for v in ("memory_copies", "memory_copy") if v in names)
    cols = [r[1] for r in c.execute("pragma table_info(%s)" % view)]
    size = next(k for k in ("size", "bytes") if k in cols)
    dirk = next((k for k in ("name", "kind", "direction") if k in cols), None)
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    q = next((k for k in ("queue_id", "stream_id") if k in kcols), None)
    kern = list(c.execute("select start, end, name, %s from kernels" % (q or "0")))
    copies = list(c.execute("select start, end, %s, %s from %s" % (size, dirk or "'?'", view)))
    end = max([e for _, e, *_ in kern] + [e for _, e, *_ in copies])
    t0 = end - win_ms * 1e6
    ev = []
    for s, e, z, d in copies:
        if e > t0:
            d = str(d).replace("MEMORY_COPY_", "")
            ev.append((s, e, "COPY %-14s %7.1f MB %6.1f GB/s" % (d, z / 1e6, z / max(e - s, 1))))
    for s, e, n, qq in kern:
        if e > t0 and "rocclr" in n:
            ev.append((s, e, "BLIT %s q%s" % (n[:40], qq)))
    # compute batches: a dct kernel opens one, the next ola_log on the same queue closes it
    open_ = {}
    spans = []
    for s, e, n, qq in sorted(kern):
        if "dct_frame" in n or "frames_dft1" in n:
            open_[qq] = s
        elif "ola_log" in n and qq in open_:
            spans.append((open_.pop(qq), e, qq))
    for s, e, qq in spans:
        if e > t0:
            ev.append((s, e, "BATCH compute q%s" % qq))
    for s, e, what in sorted(ev):
        print("%9.3f %8.3f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, what))
    w = lambda iv: [(max(s, t0), e) for s, e in iv if e > t0]
    h2d = w([(s, e) for s, e, z, d in copies if "HOST_TO_DEVICE" in str(d)])
    d2h = w([(s, e) for s, e, z, d in copies if "DEVICE_TO_HOST" in str(d)])
    comp = w([(s, e) for s, e, _ in spans])
    print("window %.1f ms: H2D busy %.2f ms, D2H busy %.2f ms, any compute batch running %.2f ms, "
          "compute batches closed in window %d" % (win_ms, union_ms(h2d), union_ms(d2h), union_ms(comp),
                                                  sum(1 for s, e, _ in spans if s > t0)))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 120.0)
