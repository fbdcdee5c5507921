#!/usr/bin/env bash
# GPU session: parity tests of the current tree, short bench lines, then a kernel trace + PMC passes of the
# REVERB and WSJ bench commands (one batch in flight) -> gpurun_out/evidence_<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest_gpu.log | tail -3; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
[ $rc -ge 1 ] && exit $rc
for c in ${BENCH_CONFIGS:-wsj reverb}; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -30 $O/bench_$c.log; exit 4; }
  tail -1 $O/bench_$c.log > $O/bench_$c.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), r['stage'], round(r['frac'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})" $O/bench_$c.json $c
done
[ -n "${NO_PMC:-}" ] && exit 0
export SKIP_BENCH=1 EXTRA_PMC="SQ_WAIT_INST_LDS+SQ_INSTS_SALU+SQ_WAIT_ANY+SQ_BUSY_CYCLES+SQ_WAVE_CYCLES+SQ_LDS_IDX_ACTIVE"
TAG=${TAG_PREFIX:-r03b}_reverb BENCH_ARGS="--config reverb --steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers" bash scripts/round_evidence.sh || exit 5
TAG=${TAG_PREFIX:-r03b} BENCH_ARGS="--steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers" bash scripts/round_evidence.sh || exit 6
for t in ${TAG_PREFIX:-r03b}_reverb ${TAG_PREFIX:-r03b}; do
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
for k,m in d.items():
    if not k.startswith('void fdlp') and not k.startswith('fdlp'): continue
    print('%-52s %6.3f ms valu %5.1f%% mfma %5.1f%% lds %.3g conf %.3g GB %.2f' % (k.replace('void ','')[:52], m.get('avg_ms',0), m.get('valu_active_pct_per_simd',0), m.get('mfma_busy_pct',0), m.get('SQ_INSTS_LDS',0), m.get('SQ_LDS_BANK_CONFLICT',0), (m.get('fetch_bytes_x2',0)+m.get('write_bytes',0))/1e9))
" gpurun_out/evidence_$t/pmc.json
done
