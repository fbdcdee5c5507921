#!/usr/bin/env python3
"""The bench line's roofline frac, recomputed from a kernel trace of the same run.

    python3 scripts/frac_check.py <bench line .json> <kernel_trace_stats.csv>

The line's `roofline.avg_launch_ms` is HIP events around the dominant stage's kernels (one batch in flight,
`fdlp_stage_times`); the trace gives each kernel's own average duration.  Per batch, the stage's kernel time
is the sum over its kernels (`roofline.stage_kernels` name prefixes) of total_ms / batches, batches = the
profiled steps of the line (every kernel of the stage runs once per batch; the trace also holds the warmup
and the timed steps of the other passes, so calls are counted from the CSV and divided evenly).
Prints one JSON object: both times and both fracs.
"""
import csv
import json
import sys


def main():
    line = [json.loads(x) for x in open(sys.argv[1]) if x.lstrip().startswith("{") and '"roofline"' in x][-1]
    rf = line["roofline"]
    pre = rf.get("stage_kernels") or []
    flops, peak = rf["algorithmic_flops_per_launch"], rf["peak"]
    per_kernel = {}
    for row in csv.DictReader(open(sys.argv[2])):
        name = row["kernel"].replace("void ", "")
        if any(name.startswith(p) for p in pre):
            per_kernel[name[:60]] = {"calls": int(row["calls"]), "avg_ms": float(row["avg_ms"])}
    # kernels of one stage launch once per batch each (the sweeps: two instantiations, each once)
    trace_ms = sum(k["avg_ms"] for k in per_kernel.values())
    out = {"stage": rf["stage"], "stage_kernels": pre, "hip_event_ms_per_batch": rf["avg_launch_ms"],
           "trace_kernel_ms_per_batch": trace_ms, "frac_hip_events": rf["frac"],
           "frac_trace": flops / (trace_ms * 1e-3) / 1e12 / peak if trace_ms else None,
           "algorithmic_flops_per_launch": flops, "peak_tflops": peak, "kernels": per_kernel,
           "timing": rf.get("timing")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
