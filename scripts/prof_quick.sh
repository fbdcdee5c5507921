#!/usr/bin/env bash
# Kernel-trace summary of a short bench run: prof_quick.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q_$tag -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/q_$tag.log 2>&1 || { tail -20 gpurun_out/q_$tag.log; exit 3; }
python3 scripts/rocpd_summary.py gpurun_out/q_$tag/run_results.db gpurun_out/q_$tag.csv > /dev/null
python3 -c "import csv,sys; [print(r[0][:48].ljust(48), *r[2:4]) for r in csv.reader(open(sys.argv[1]))]" gpurun_out/q_$tag.csv
grep -o "\"value\": [0-9.]*" gpurun_out/q_$tag.log || true
