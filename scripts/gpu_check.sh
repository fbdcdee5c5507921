#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, short bench.  Stops at the first crash/timeout
# (exit codes >= 2 from pytest, or any non-zero from smoke/bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -x -q"}
timeout -k 10 900 python -m pytest $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 4; }
tail -3 gpurun_out/bench.log
