#!/usr/bin/env bash
# Quick GPU iteration: selected parity tests, one bench line, and the kernel trace + one PMC pass
# (FETCH_SIZE / WRITE_SIZE by default) of the bench command with one batch in flight.
#   TAG=r03i PYTEST_K="dct" PMC="WRITE_SIZE" bash scripts/gpu_quick.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-q}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_SEL:-tests} -k "$PYTEST_K" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
fi
timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_EXTRA:-} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 4; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; x=d.get('with_transfers') or {}; print(round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), 'xfer', round(x.get('value',0),1), r['stage'], round(r['frac'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})" $O/bench.json
BARGS="--steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers ${BENCH_EXTRA:-}"
for pmc in ${PMC:-FETCH_SIZE WRITE_SIZE}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${pmc//+/ } -d $O/pmc_$pmc -o run -- python3 bench.py $BARGS > $O/pmc_$pmc.log 2>&1 || { echo "pmc $pmc failed"; tail -5 $O/pmc_$pmc.log; exit 5; }
done
python3 scripts/pmc_report.py "$O/pmc_*/*.db" $O/pmc.json > $O/pmc.txt 2>&1
python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
for k,m in d.items():
    if 'fdlp' not in k: continue
    print('%-46s %6.3f ms  GB %.3f  %s' % (k.replace('void ','')[:46], m.get('avg_ms',0), (m.get('fetch_bytes_x2',0)+m.get('write_bytes',0))/1e9, {c: '%.3g' % v for c, v in m.items() if c.startswith(('SQ_','TCC','TCP','GRBM'))}))
" $O/pmc.json
find $O -name "*.db" -delete
