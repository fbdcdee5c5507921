#!/usr/bin/env python3
"""Timeline of the last part of a rocprofv3 --kernel-trace --memory-copy-trace database: every memory-copy
record and every blit kernel (__amd_rocclr_*) with start (ms, relative), duration and size, plus per
stream-queue counts of the compute kernels in the same window.

    python scripts/xfer_timeline.py <run_results.db> [window_ms]
"""
import sqlite3
import sys


def main(db, win_ms=120.0):
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    view = next(v for v in ("memory_copies", "memory_copy") if v in names)
    cols = [r[1] for r in c.execute("pragma table_info(%s)" % view)]
    size = next(k for k in ("size", "bytes") if k in cols)
    dirk = next((k for k in ("name", "kind", "direction") if k in cols), None)
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    extra = [k for k in ("grid_size", "grid_x", "workgroup_size", "queue_id", "stream_id") if k in kcols]
    kern = list(c.execute("select start, end, name%s from kernels" % "".join(", " + e for e in extra)))
    copies = list(c.execute("select start, end, %s, %s from %s" % (size, dirk or "'?'", view)))
    end = max(e for _, e, *_ in kern)
    t0 = end - win_ms * 1e6
    ev = [(s, e, "COPY %s %.1f MB" % (d, z / 1e6)) for s, e, z, d in copies if e > t0]
    ev += [(s, e, "BLIT %s %s" % (n[:40], r)) for s, e, n, *r in kern if e > t0 and "rocclr" in n]
    big = [(s, e, n) for s, e, n, *r in kern if e > t0 and "rocclr" not in n and "dct_frame" in n]
    ev += [(s, e, "kern %s" % n[:30]) for s, e, n in big]
    print("extra kernel columns:", extra)
    for s, e, what in sorted(ev):
        print("%9.3f %8.3f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, what))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 120.0)
