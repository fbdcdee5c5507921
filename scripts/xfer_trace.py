#!/usr/bin/env python3
"""Timeline of bench.py's PCIe-inclusive step from a rocprofv3 kernel + memory-copy trace database:
per step, the compute kernels' span, the gaps between consecutive kernels, and the copies that overlap.

    python scripts/xfer_trace.py <run_results.db>
"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
kern = sorted(c.execute("select start, end, name from kernels"))
copies = []
for t in tabs:
    if "memory_copies" in t or t == "memory_copy":
        try:
            copies = sorted(c.execute("select start, end, src_agent_type, dst_agent_type, size from %s" % t))
        except sqlite3.Error:
            copies = sorted((r[0], r[1], "?", "?", 0) for r in c.execute("select start, end from %s" % t))
        break
big = [k for k in kern if "lattice" in k[2] or "frames_dft1" in k[2]]
print("kernels", len(kern), "copies", len(copies))
# gaps between consecutive kernels longer than 20 us
prev = None
for s, e, n in kern[-80:]:
    if prev is not None and s - prev[1] > 20000:
        ov = [(cs, ce, a, b, z) for cs, ce, a, b, z in copies if cs < s and ce > prev[1]]
        print("gap %8.3f ms before %-40s copies overlapping: %s" % ((s - prev[1]) / 1e6, n[:40],
              ["%s->%s %.1fMB %.2fms" % (a, b, z / 1e6, (ce - cs) / 1e6) for cs, ce, a, b, z in ov]))
    prev = (s, e, n)
for cs, ce, a, b, z in copies[-12:]:
    print("copy %s->%s %.1f MB %.3f ms at %.3f" % (a, b, z / 1e6, (ce - cs) / 1e6, (cs - kern[0][0]) / 1e6))
for s, e, n in kern[-24:]:
    print("kern %-50s %.3f ms at %.3f" % (n[:50], (e - s) / 1e6, (s - kern[0][0]) / 1e6))

# host API calls longer than 0.5 ms (needs --hip-trace)
for t in tabs:
    if t in ("regions", "hip_api", "api") or "region" in t:
        try:
            rows = list(c.execute("select start, end, name from %s" % t))
        except sqlite3.Error:
            continue
        long_ = [(s, e, n) for s, e, n in rows if e - s > 500000]
        print("table", t, "calls", len(rows), "long", len(long_))
        for s, e, n in sorted(long_)[-30:]:
            print("api %-40s %.3f ms at %.3f" % (n[:40], (e - s) / 1e6, (s - kern[0][0]) / 1e6))
        break
