#!/usr/bin/env bash
# Recipe stage 1 (nj 20, 10 audio-hours, one GPU) with warm JOB chains at 2 / 4 / 8 slots per GPU (at most 16
# processes may use a GPU box's GPU),
# alternating twice.  Output: gpurun_out/$TAG/slots.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-slots}; mkdir -p $O; : > $O/slots.jsonl
for round in 1 2; do
  for k in ${SLOTS:-2 4 8}; do
    timeout -k 10 600 python3 benchmarks/driver_e2e.py --utts ${UTTS:-4500} --lengths 2 14 --nj 20 --jobs-per-gpu $k \
      >> $O/slots.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
print('slots', d['jobs_per_gpu'], round(d['value'],2), 'audio-h/s', round(d['wall_s'],2), 's')" $O/slots.jsonl
  done
done
