#!/usr/bin/env bash
# PCIe copy-rate probes (split copies, SDMA vs blit, host allocation kinds), then the WSJ kernel trace and
# PMC passes of the bench command (one batch in flight).  Outputs under gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03x}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 180 python3 benchmarks/transfer_probe.py --split-probe > $O/split_sdma.json 2> $O/split_sdma.err || { echo "split probe failed"; tail $O/split_sdma.err; exit 2; }
cat $O/split_sdma.json
timeout -k 10 180 env HSA_ENABLE_SDMA=0 python3 benchmarks/transfer_probe.py --split-probe > $O/split_blit.json 2> $O/split_blit.err || { echo "split blit probe failed"; tail $O/split_blit.err; exit 3; }
cat $O/split_blit.json
timeout -k 10 180 python3 benchmarks/transfer_probe.py --d2h-variants > $O/d2h_variants.json 2> $O/d2h_variants.err || { echo "variants failed"; tail $O/d2h_variants.err; exit 4; }
cat $O/d2h_variants.json
if [ -z "${NO_PMC:-}" ]; then
  export SKIP_BENCH=1 EXTRA_PMC="SQ_WAIT_INST_LDS+SQ_WAIT_ANY+SQ_BUSY_CYCLES+SQ_WAVE_CYCLES"
  TAG=$TAG BENCH_ARGS="--steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers" bash scripts/round_evidence.sh || exit 5
  cp gpurun_out/evidence_$TAG/kernel_trace_stats.csv $O/ 2>/dev/null
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
for k,m in d.items():
    if 'fdlp' not in k: continue
    w = m.get('SQ_WAVE_CYCLES', 0) or 1
    print('%-50s %6.3f ms valu %5.1f%% mfma %5.1f%% lds %.3g conf %.3g waitlds %.2f GB %.2f' % (k.replace('void ','')[:50], m.get('avg_ms',0), m.get('valu_active_pct_per_simd',0), m.get('mfma_busy_pct',0), m.get('SQ_INSTS_LDS',0), m.get('SQ_LDS_BANK_CONFLICT',0), m.get('SQ_WAIT_INST_LDS',0)/w, (m.get('fetch_bytes_x2',0)+m.get('write_bytes',0))/1e9))
" gpurun_out/evidence_$TAG/pmc.json
  find gpurun_out/evidence_$TAG -name "*.db" -delete
fi
