# A/B of bench variants on one box, alternating: AB_ARGS="--lpc-path auto|--lpc-path lattice8" TAG=x bash scripts/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}; mkdir -p $O
IFS='|' read -ra VARS <<< "${AB_ARGS}"
: > $O/ab.txt
for round in 1 2; do
  for v in "${VARS[@]}"; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-transfers ${BENCH_EXTRA:-} $v > $O/ab_run.log 2>&1 || { tail -20 $O/ab_run.log; exit 2; }
    python3 -c "
import json,sys; d=json.loads(open('$O/ab_run.log').read().strip().splitlines()[-1])
print(sys.argv[1], round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})" "$v" >> $O/ab.txt
  done
done
cat $O/ab.txt
if [ -n "${TRACE:-}" ]; then
  for v in "${VARS[@]}"; do
    n=$(echo $v | tr -c 'a-z0-9' '_')
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$n -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers $v > $O/tr_$n.log 2>&1 || { tail -5 $O/tr_$n.log; exit 3; }
    python3 scripts/rocpd_summary.py $O/tr_$n/run_results.db $O/trace_$n.csv > /dev/null || true
    rm -rf $O/tr_$n
    echo "== $v"; cut -c1-60,200- $O/trace_$n.csv | head -12
  done
fi
