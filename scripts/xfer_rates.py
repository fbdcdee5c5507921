#!/usr/bin/env python3
"""Per-direction copy rates and kernel slow-down under copies, from a rocprofv3 --kernel-trace
--memory-copy-trace database of bench.py: each copy's GB/s (count, median, 10th percentile), the wall time
with at least one copy active, and per kernel name the mean duration of launches that overlap a copy
against those that do not.

    python scripts/xfer_rates.py <run_results.db>
"""
import sqlite3
import statistics
import sys


def main(db):
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    view = next(v for v in ("memory_copies", "memory_copy") if v in names)
    cols = [r[1] for r in c.execute("pragma table_info(%s)" % view)]
    size = next(k for k in ("size", "bytes") if k in cols)
    dirk = next((k for k in ("name", "kind", "direction") if k in cols), None)
    copies = list(c.execute("select start, end, %s, %s from %s" % (size, dirk or "'?'", view)))
    kern = list(c.execute("select start, end, name from kernels"))
    big = [cp for cp in copies if cp[2] >= 1 << 20]
    by = {}
    for s, e, z, d in big:
        by.setdefault(d, []).append(z / max(e - s, 1))  # bytes/ns = GB/s
    for d, v in by.items():
        v.sort()
        print("%-28s n=%4d median %6.1f GB/s  p10 %6.1f  max %6.1f" % (d, len(v), statistics.median(v),
                                                                     v[len(v) // 10], v[-1]))
    iv = sorted((s, e) for s, e, _, _ in big)
    merged = []
    for s, e in iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    if merged:
        span = merged[-1][1] - merged[0][0]
        print("copy-active %.2f ms of %.2f ms span" % (sum(e - s for s, e in merged) / 1e6, span / 1e6))

    def overl(s, e):
        import bisect
        i = bisect.bisect_right([m[0] for m in merged], e) - 1
        return i >= 0 and merged[i][1] > s

    agg = {}
    for s, e, n in kern:
        key = n.replace("void ", "")[:48]
        a = agg.setdefault(key, [[], []])
        a[1 if overl(s, e) else 0].append((e - s) / 1e6)
    for k, (no, yes) in sorted(agg.items(), key=lambda kv: -sum(kv[1][0] + kv[1][1])):
        if len(no) + len(yes) < 4:
            continue
        print("%-48s alone %3d x %7.3f ms   under copies %3d x %7.3f ms" % (
            k, len(no), statistics.mean(no) if no else 0, len(yes), statistics.mean(yes) if yes else 0))


if __name__ == "__main__":
    main(sys.argv[1])
