#!/usr/bin/env bash
# PMC passes of a short bench run, one counter group per rocprofv3 run: pmc_kernel.sh "C1 C2" "C3" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${PMC_TAG:-pmck}
mkdir -p $O
BARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers"}
i=0
for pmc in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc -d $O/p$i -o run -- python3 bench.py $BARGS > $O/p$i.log 2>&1 || { echo "pmc $pmc failed"; tail -20 $O/p$i.log; exit 4; }
done
python3 scripts/pmc_report.py "$O/p*/*.db" $O/pmc.json
