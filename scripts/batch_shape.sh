#!/usr/bin/env bash
# Headline vs batch shape (utterances per batch x batches in flight), one box, no CPU baseline / PCIe pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-bs}
O=gpurun_out/$TAG
mkdir -p $O
for cfg in "1024 4" "2048 2" "2048 4" "512 8" "1024 6" "1024 4"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-transfers --utts $1 --inflight $2 > $O/u$1_i$2.log 2>&1 || { echo "u$1 i$2 failed"; tail -5 $O/u$1_i$2.log; exit 3; }
  tail -1 $O/u$1_i$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('utts', $1, 'inflight', $2, round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), round(d['ms_per_step'],2), 'ms/step')"
done
