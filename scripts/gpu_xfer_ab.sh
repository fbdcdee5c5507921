#!/usr/bin/env bash
# A/B of PCIe-pass variants (bench.py with transfers), alternating on one box: the device-resident value and the
# first-H2D-to-last-D2H rate of each.  AB_ARGS="--xfer-d2h-issue stream|--xfer-d2h-issue host" [BENCH_EXTRA=...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-xferab}; mkdir -p $O; : > $O/ab.txt
IFS='|' read -ra VARS <<< "${AB_ARGS}"
for round in $(seq ${ROUNDS:-3}); do
  for v in "${VARS[@]}"; do
    timeout -k 10 400 python3 bench.py --no-cpu-baseline ${BENCH_EXTRA:-} $v > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 2; }
    python3 -c "
import json,sys; d=json.loads(open('$O/run.log').read().strip().splitlines()[-1]); x=d['with_transfers']
print(sys.argv[1], 'value', round(d['value'],1), 'xfer', round(x['value'],1), 'ratio', round(x['value']/d['value'],3))" "$v" >> $O/ab.txt
  done
done
cat $O/ab.txt
