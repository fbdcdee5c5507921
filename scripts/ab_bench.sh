#!/usr/bin/env bash
# Alternating A/B of two bench.py argument sets on one box (same build): A B A B, default bench lines
# without the CPU baseline and PCIe pass.   A="" B="--dct-path four_step" TAG=ab bash scripts/ab_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-ab}
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for v in A B; do
    args=${!v}
    timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-transfers $args > $O/$v$i.log 2>&1 || { echo "$v$i failed"; tail -5 $O/$v$i.log; exit 3; }
    tail -1 $O/$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v$i', '$args', round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), {k: round(x,3) for k,x in d['stage_ms_per_step'].items()})"
  done
done
