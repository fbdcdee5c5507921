#!/usr/bin/env bash
# Round-3 GPU session: parity tests (incl. the REVERB / CHiME4 bench-shape tests), smoke, then the
# bench lines of the three configs.  Stops at the first crash / timeout of a GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03
mkdir -p $O
PT=${PYTEST_SEL:-"tests -m gpu"}
timeout -k 10 900 python -u -m pytest $PT -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 3; }
cat $O/smoke.log
for c in ${BENCH_CONFIGS:-chime4 reverb wsj}; do
  timeout -k 10 400 python bench.py --config $c ${BENCH_ARGS:---no-cpu-baseline} > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -30 $O/bench_$c.log; exit 4; }
  tail -1 $O/bench_$c.log > $O/bench_$c.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), r['stage'], round(r['frac'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})" $O/bench_$c.json $c
done
