#!/usr/bin/env bash
# PMC pass (one counter group) over standalone benchmark binaries: pmc_bin.sh "<counters>" bin1 bin2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmcbin
mkdir -p $O
ctr=$1; shift
for b in "$@"; do
  n=$(basename $b)
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $ctr -d $O/$n -o run -- $b > $O/$n.log 2>&1 || { echo "pmc $n failed"; tail $O/$n.log; exit 1; }
  echo "== $n"; python3 scripts/pmc_report.py "$O/$n/*.db"
done
