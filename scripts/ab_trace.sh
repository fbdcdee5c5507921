#!/usr/bin/env bash
# A/B kernel traces of bench.py variants, alternating on one box: ab_trace.sh "<variant>" "<variant>" ...
# A variant is a list of tokens: NAME=VALUE sets an environment variable (FDLP_LIB=... loads an A/B build),
# anything else is passed to bench.py ("-" = the default).  Prints the bench value and per-kernel avg ms.
#   ROUNDS=2 bash scripts/ab_trace.sh - "--lpc-path lattice8"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
BARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers"}
for round in $(seq 1 ${ROUNDS:-1}); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    envs=(); args=()
    if [ "$v" != "-" ]; then
      for t in $v; do
        if [[ "$t" == *=* && "$t" != --* ]]; then envs+=("$t"); else args+=("$t"); fi
      done
    fi
    d=gpurun_out/ab/r${round}v$i
    env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py $BARGS "${args[@]}" \
      > $d.log 2>&1 || { echo "variant $v failed"; tail -20 $d.log; exit 3; }
    echo "== [$round] $v  $(grep -o '"value": [0-9.]*' $d.log | head -1)"
    python3 - "$(find $d -name '*.db' | head -1)" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
for n, k, a in c.execute("select name, count(*), avg(duration) from kernels group by name order by sum(duration) desc"):
    print("   %-60s %4d %9.3f ms" % (n[:60], k, a / 1e6))
PY
    find $d -name '*.db' -delete
  done
done
