#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (kernel-trace --stats run) as CSV:
kernel, calls, total_us, avg_us, pct  (+ PMC counter means per kernel when present)."""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    # durations in the kernels view are ns
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration), 0 from kernels group by name "
                          "order by sum(duration) desc"))
    tot_all = sum(r[2] for r in rows) or 1
    rows = [(n, k, t, a, 100.0 * t / tot_all) for n, k, t, a, _ in rows]
    pmc = {}
    try:
        for name, counter, val in c.execute(
                "select kernel_name, counter_name, avg(value) from counters_collection "
                "group by kernel_name, counter_name"):
            pmc.setdefault(name, {})[counter] = val
    except sqlite3.Error:
        pass
    counters = sorted({k for d in pmc.values() for k in d})
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_ms", "pct"] + counters)
        for name, n, tot, avg, pct in rows:
            w.writerow([name, n, "%.4f" % (tot / 1e6), "%.4f" % (avg / 1e6), "%.2f" % pct] +
                       [pmc.get(name, {}).get(k, "") for k in counters])
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
