#!/usr/bin/env python3
"""One line per benchmarks/cli_throughput.py result: audio-h/s and the native runner's job stats."""
import json
import sys

for line in open(sys.argv[1]):
    d = json.loads(line)
    s = d.get("job_stats") or {}
    print(round(d["value"], 1), {k: round(v, 4) for k, v in s.items() if k.endswith("seconds")})
