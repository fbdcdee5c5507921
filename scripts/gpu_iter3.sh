#!/usr/bin/env bash
# One iteration on a GPU box: selected parity tests, bench lines of the given configs, and optionally a
# kernel trace (+ PMC passes) of one config's bench command.  Big rocpd databases are deleted after their
# summaries are written (gpurun copies back <= 64 MiB of gpurun_out/).
#   PYTEST_SEL="tests/test_gpu_parity.py" PYTEST_K="reverb or dct" BENCH_CONFIGS="reverb wsj" TRACE=reverb PMC=1 TAG=r03c
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03x}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "${PYTEST_SEL:-}" ]; then
  timeout -k 10 900 python -u -m pytest $PYTEST_SEL ${PYTEST_K:+-k "$PYTEST_K"} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20
  [ $rc -ge 1 ] && exit $rc
fi
for c in ${BENCH_CONFIGS:-}; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline ${BENCH_EXTRA:-} > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -30 $O/bench_$c.log; exit 4; }
  tail -1 $O/bench_$c.log > $O/bench_$c.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), r['stage'], round(r['frac'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})" $O/bench_$c.json $c
done
if [ -n "${TRACE:-}" ]; then
  export TMPDIR=/tmp
  BARGS="--config $TRACE --steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py $BARGS > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 5; }
  python3 scripts/rocpd_summary.py $O/trace/run_results.db $O/kernel_trace_stats.csv > /dev/null || true
  python3 -c "import csv,sys; [print(r[0][:56].ljust(56), *r[1:4]) for r in csv.reader(open(sys.argv[1]))]" $O/kernel_trace_stats.csv | head -14
  if [ -n "${PMC:-}" ]; then
    i=0
    for pmc in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE"; do
      i=$((i+1))
      timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc -d $O/pmc_$i -o run -- python3 bench.py $BARGS > $O/pmc_$i.log 2>&1 || { echo "pmc $pmc failed"; tail -20 $O/pmc_$i.log; exit 6; }
    done
    python3 scripts/pmc_report.py "$O/pmc_*/*.db" $O/pmc.json > $O/pmc.txt 2>&1 || true
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
for k,m in d.items():
    if 'fdlp' not in k: continue
    w = m.get('SQ_WAVE_CYCLES', 0) or 1
    print('%-50s %6.3f ms valu %5.1f%% mfma %5.1f%% lds %.3g conf %.3g waitlds %.2f waitany %.2f GB %.2f' % (k.replace('void ','')[:50], m.get('avg_ms',0), m.get('valu_active_pct_per_simd',0), m.get('mfma_busy_pct',0), m.get('SQ_INSTS_LDS',0), m.get('SQ_LDS_BANK_CONFLICT',0), m.get('SQ_WAIT_INST_LDS',0)/w, m.get('SQ_WAIT_ANY',0)/w, (m.get('fetch_bytes_x2',0)+m.get('write_bytes',0))/1e9))
" $O/pmc.json
  fi
  find $O -name "*.db" -delete; find $O -type d -empty -delete
fi
