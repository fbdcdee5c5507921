#!/usr/bin/env bash
# Full round evidence on one GPU box, every GPU step under its own time limit, stopping at the first
# failure: pytest -m gpu, the smoke, a kernel trace + PMC passes of the WSJ bench command (one batch in
# flight), the default bench line (CPU baseline included, its roofline traffic from the PMC summary just
# written), then the REVERB and CHiME4 lines.  Outputs under gpurun_out/$TAG/.
#   TAG=r03d bash scripts/gpu_round.sh        (NO_PYTEST=1 / NO_PMC=1 / CONFIGS="reverb chime4")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03x}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "${NO_PYTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest_gpu.log | tail -2; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
  tail -1 $O/smoke.log
fi
if [ -z "${NO_PMC:-}" ]; then
  export SKIP_BENCH=1 EXTRA_PMC="SQ_WAIT_INST_LDS+SQ_WAIT_ANY+SQ_BUSY_CYCLES+SQ_WAVE_CYCLES"
  TAG=$TAG BENCH_ARGS="--steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers" bash scripts/round_evidence.sh || exit 4
  unset SKIP_BENCH
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
for k,m in d.items():
    if 'fdlp' not in k and 'dct' not in k and 'ac_' not in k: continue
    w = m.get('SQ_WAVE_CYCLES', 0) or 1
    print('%-50s %6.3f ms valu %5.1f%% mfma %5.1f%% lds %.3g conf %.3g GB %.2f' % (k.replace('void ','')[:50], m.get('avg_ms',0), m.get('valu_active_pct_per_simd',0), m.get('mfma_busy_pct',0), m.get('SQ_INSTS_LDS',0), m.get('SQ_LDS_BANK_CONFLICT',0), (m.get('fetch_bytes_x2',0)+m.get('write_bytes',0))/1e9))
" gpurun_out/evidence_$TAG/pmc.json
fi
if [ -z "${NO_WSJ_BENCH:-}" ]; then
  timeout -k 10 600 python3 bench.py > $O/bench_full.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_full.log; exit 5; }
  tail -1 $O/bench_full.log > $O/bench_full.json
fi
if [ -n "${REVERB_PMC:-}" ]; then  # the REVERB trace + PMC passes -> profiles/${TAG}_reverb_pmc.json (the REVERB line's traffic)
  SKIP_BENCH=1 EXTRA_PMC="SQ_WAIT_INST_LDS+SQ_WAIT_ANY+SQ_BUSY_CYCLES+SQ_WAVE_CYCLES" TAG=${TAG}_reverb \
    BENCH_ARGS="--config reverb --steps 3 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers" bash scripts/round_evidence.sh || exit 7
fi
if [ -n "${LIBRI:-}" ]; then
  timeout -k 10 400 python3 bench.py --workload librispeech --no-cpu-baseline > $O/bench_librispeech.log 2>&1 || { echo "bench librispeech failed"; tail -30 $O/bench_librispeech.log; exit 8; }
  tail -1 $O/bench_librispeech.log > $O/bench_librispeech.json
fi
for c in ${CONFIGS-reverb chime4}; do
  timeout -k 10 400 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -30 $O/bench_$c.log; exit 6; }
  tail -1 $O/bench_$c.log > $O/bench_$c.json
done
for f in $O/bench_*.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; t=d.get('with_transfers') or {}; print(sys.argv[1].split('/')[-1], round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), 'xfer', round(t.get('value',0) or 0,1), r['stage'], round(r['frac'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})" $f
done
