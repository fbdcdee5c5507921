# A/B of two builds of the library on one box, alternating (FDLP_LIB selects the build):
#   LIB_A=path LIB_B=path TAG=x [PYTEST="tests/..."] bash scripts/gpu_libab.sh
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-libab}; mkdir -p $O
if [ -n "${PYTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
: > $O/ab.txt
for round in $(seq ${ROUNDS:-2}); do
  for lib in "$LIB_A" "$LIB_B"; do
    FDLP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-transfers ${BENCH_EXTRA:-} > $O/ab_run.log 2>&1 || { tail -20 $O/ab_run.log; exit 2; }
    python3 -c "
import json,sys; d=json.loads(open('$O/ab_run.log').read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), {k.replace('fdlp::','').replace('_kernel',''): round(v,3) for k,v in d.get('kernel_ms_per_launch', d['stage_ms_per_step']).items()})" "$lib" >> $O/ab.txt
  done
done
cat $O/ab.txt
for lib in "$LIB_A" "$LIB_B"; do
  n=$(basename $lib .so)
  FDLP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$n -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers ${BENCH_EXTRA:-} > $O/tr_$n.log 2>&1 || { tail -5 $O/tr_$n.log; exit 3; }
  python3 scripts/rocpd_summary.py $O/tr_$n/run_results.db $O/trace_$n.csv > /dev/null || true
  rm -rf $O/tr_$n
  echo "== $n"; cut -c1-60,200- $O/trace_$n.csv | head -12
done
