#!/usr/bin/env bash
# Recipe-scale stage 1 on one GPU box: the drop-in driver with the recipes' --nj 20 over
# >= 10 audio-hours of page-cached 16 kHz WAVs (U(2,14) s), cold JOBs, then the same data dir with --nj 1 as
# the cross-check.  Output: gpurun_out/$TAG/driver_e2e.jsonl
#   TAG=r06e [UTTS=4500] bash scripts/gpu_e2e.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-e2e}; mkdir -p $O
echo "# benchmarks/driver_e2e.py --utts ${UTTS:-4500} --lengths 2 14 --nj 20 --jobs-per-gpu 4 --check-single --chain-jobs {true,false,true,false}" > $O/driver_e2e.jsonl
for ch in ${CHAINS:-true false true false}; do
  timeout -k 10 900 python3 benchmarks/driver_e2e.py --utts ${UTTS:-4500} --lengths 2 14 --nj 20 --jobs-per-gpu 4 \
    --check-single --chain-jobs $ch >> $O/driver_e2e.jsonl 2> $O/driver_e2e.err || { tail -30 $O/driver_e2e.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
print('chain', d['chain_jobs'], round(d['value'],2), 'audio-h/s', round(d['audio_hours'],2), 'h in', round(d['wall_s'],2), 's; JOB exec mean', d['job_execution_s_mean'], '; single:', d['single_job_check'])" $O/driver_e2e.jsonl
done
