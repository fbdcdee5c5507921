#!/usr/bin/env bash
# One iteration on a GPU box: GPU parity suite + smoke + bench (gpu_check.sh), a kernel trace of the
# bench (ab_trace.sh), and the end-to-end CLI throughput at the CLI default and an 8192-frame batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS="tests -m gpu -x -q --timeout 300 --timeout-method thread" BENCH_ARGS="--no-cpu-baseline" \
  bash scripts/gpu_check.sh || exit $?
bash scripts/ab_trace.sh - || exit $?
[ -n "${SKIP_CLI:-}" ] && exit 0
for bf in 2048 8192; do
  timeout -k 10 300 python benchmarks/cli_throughput.py --utts 8192 --workers 4 8 --runners native \
    --batch-frames $bf > gpurun_out/cli_$bf.jsonl 2>&1 || { tail -20 gpurun_out/cli_$bf.jsonl; exit 5; }
  grep -o '"value": [0-9.]*\|"io_workers": [0-9]*\|"seconds": [0-9.]*' gpurun_out/cli_$bf.jsonl | paste -sd' '
done
