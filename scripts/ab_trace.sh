#!/usr/bin/env bash
# A/B kernel-trace of bench.py under environment variants: ab_trace.sh "VAR=1" "VAR2=1 VAR3=0" ...
# ("-" = no extra variable).  Prints the bench value and per-kernel avg ms of each variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
BARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline"}
i=0
for v in "$@"; do
  i=$((i+1))
  (
    if [ "$v" != "-" ]; then for kv in $v; do export "$kv"; done; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/v$i -o run -- python3 bench.py $BARGS \
      > gpurun_out/ab/v$i.log 2>&1
  ) || { echo "variant $v failed"; tail -20 gpurun_out/ab/v$i.log; exit 3; }
  echo "== $v  $(grep -o '"value": [0-9.]*' gpurun_out/ab/v$i.log | head -1)"
  python3 - "$(find gpurun_out/ab/v$i -name '*.db' | head -1)" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
for n, k, a in c.execute("select name, count(*), avg(duration) from kernels group by name order by sum(duration) desc"):
    print("   %-60s %4d %9.3f ms" % (n[:60], k, a / 1e6))
PY
done
