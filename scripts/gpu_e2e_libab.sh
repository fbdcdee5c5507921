#!/usr/bin/env bash
# Recipe stage 1 (nj 20, 10 audio-hours, one GPU, chains) with two builds of the library, alternating:
#   LIB_A=path LIB_B=path TAG=x bash scripts/gpu_e2e_libab.sh     -> gpurun_out/$TAG/e2e_ab.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-e2eab}; mkdir -p $O; : > $O/e2e_ab.jsonl
for round in $(seq ${ROUNDS:-2}); do
  for lib in "$(realpath "$LIB_A")" "$(realpath "$LIB_B")"; do
    FDLP_LIB=$lib timeout -k 10 600 python3 benchmarks/driver_e2e.py --utts ${UTTS:-4500} --lengths 2 14 --nj 20 \
      --jobs-per-gpu ${SLOTS:-4} >> $O/e2e_ab.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); s=d['job_stats_mean']
print(sys.argv[2].split('/')[-1], round(d['value'],2), 'audio-h/s', round(d['wall_s'],2), 's; JOB s', round(s['seconds'],4), 'd2h_wait', round(s['d2h_wait_seconds'],4))" $O/e2e_ab.jsonl $lib
  done
done
