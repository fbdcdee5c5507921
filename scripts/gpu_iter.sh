#!/usr/bin/env bash
# One GPU iteration: pytest -m gpu (all, or -k "$PYTEST_K"), the default bench line without the CPU baseline,
# and a rocprofv3 kernel trace of the one-batch bench command (per-kernel averages).  Every GPU step under its
# own time limit, stopping at the first failure.  Outputs under gpurun_out/$TAG/.
#   TAG=r06c [PYTEST_K=band] [NO_PYTEST=1] [BENCH_EXTRA="--config reverb"] bash scripts/gpu_iter.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-it}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "${NO_PYTEST:-}" ]; then
  K=()
  [ -n "${PYTEST_K:-}" ] && K=(-k "$PYTEST_K")
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit $rc; }
fi
timeout -k 10 400 python3 bench.py --no-cpu-baseline ${BENCH_EXTRA:-} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 4; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; x=d.get('with_transfers') or {}
print(round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), 'xfer', round(x.get('value',0) or 0,1), r['stage'], round(r['frac'],3))
print({k: round(v,3) for k,v in d['kernel_ms_per_launch'].items()})" $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers ${BENCH_EXTRA:-} > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 5; }
python3 scripts/rocpd_summary.py $O/tr/run_results.db $O/kernel_trace_stats.csv > /dev/null || true
rm -rf $O/tr
cut -c1-70,200- $O/kernel_trace_stats.csv | head -14
