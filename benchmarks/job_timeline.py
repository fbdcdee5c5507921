#!/usr/bin/env python3
"""Summarise a native JOB runner trace (compute-fdlp-feats --job_trace, fdlp_job_opts.trace_path):
per batch, when the consumer flushed it, when its D2H pieces were issued, landed, widened and written,
and how busy the writer was.

    python benchmarks/job_timeline.py trace.jsonl [...]
"""
import collections
import json
import sys


def summarise(path):
    ev = [json.loads(line) for line in open(path)]
    first = {}
    for e in ev:
        first.setdefault(e["ev"], e["t"])
    batches = collections.defaultdict(dict)
    written = []
    for e in ev:
        b = batches[e["a"]] if e["ev"] in ("flush", "copies", "launched", "landed", "widened", "written") else None
        if b is None:
            continue
        if e["ev"] == "flush":
            b["flush"], b["frames"] = e["t"], e["b"]
        elif e["ev"] == "launched":
            b["launched"], b["pieces"] = e["t"], e["b"]
        elif e["ev"] == "copies":
            b["copies"] = e["t"]
        else:
            b.setdefault(e["ev"] + "_first", e["t"])
            b[e["ev"] + "_last"] = e["t"]
        if e["ev"] == "written":
            written.append(e["t"])
    end = max(e["t"] for e in ev)
    out = {"file": path, "plan_s": first.get("plan"), "setup_s": first.get("setup"),
           "first_flush_s": first.get("flush"), "first_written_s": first.get("written"),
           "last_launch_s": max((b.get("launched", 0) for b in batches.values()), default=None),
           "end_s": end, "batches": len(batches)}
    rows = []
    for k in sorted(batches):
        b = batches[k]
        rows.append({"batch": k, "frames": b.get("frames"), "pieces": b.get("pieces"),
                     "flush": round(b.get("flush", -1), 4), "copies": round(b.get("copies", -1), 4),
                     "launched": round(b.get("launched", -1), 4),
                     "landed": [round(b.get("landed_first", -1), 4), round(b.get("landed_last", -1), 4)],
                     "written": [round(b.get("written_first", -1), 4), round(b.get("written_last", -1), 4)]})
    out["per_batch"] = rows
    return out


def main():
    for p in sys.argv[1:]:
        s = summarise(p)
        rows = s.pop("per_batch")
        print(json.dumps(s))
        for r in rows:
            print("  ", json.dumps(r))


if __name__ == "__main__":
    main()
