#!/usr/bin/env python3
"""Merge rocpd PMC databases (one counter group each) into a per-kernel table + derived metrics."""
import collections
import glob
import json
import sqlite3
import sys


def load(paths):
    data = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for p in paths:
        c = sqlite3.connect(p)
        for k, did, cn, v, dur in c.execute("select kernel_name, dispatch_id, counter_name, value, duration "
                                            "from counters_collection"):
            data[k][cn].append(v)
        for k, dur in c.execute("select name, duration from kernels"):
            durs[k].append(dur)
    return data, durs


def main(pattern, out=None):
    data, durs = load(sorted(glob.glob(pattern)))
    rows = {}
    for k, cs in data.items():
        if k.startswith("__amd"):
            continue
        m = {cn: sum(v) / len(v) for cn, v in cs.items()}
        d = sum(durs[k]) / len(durs[k]) if durs[k] else 0
        m["avg_ms"] = d / 1e6
        g = m.get("GRBM_GUI_ACTIVE")
        if g and d:
            m["clock_GHz"] = g / 8 / (d * 1e-9) / 1e9
            cyc = g / 8
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                m["mfma_busy_pct"] = 100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
            if "SQ_ACTIVE_INST_VALU" in m:
                # quad-cycle units per the microarch guide
                m["valu_active_pct_per_simd"] = 100 * 4 * m["SQ_ACTIVE_INST_VALU"] / (cyc * 1024)
        if "FETCH_SIZE" in m:
            m["fetch_bytes_x2"] = 2 * 1024 * m["FETCH_SIZE"]
        if "WRITE_SIZE" in m:
            m["write_bytes"] = 1024 * m["WRITE_SIZE"]
        rows[k.split("(")[0]] = m
    for k, m in rows.items():
        print(k)
        for cn in sorted(m):
            print("   %-28s %.6g" % (cn, m[cn]))
    if out:
        json.dump(rows, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
