# A/B of two builds of the library for the drop-in JOB path and the transfer-inclusive bench line,
# alternating on one box (FDLP_LIB selects the build):
#   LIB_A=path LIB_B=path TAG=x bash scripts/gpu_jobab.sh
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-jobab}; mkdir -p $O
LIB_A=$(realpath "$LIB_A"); LIB_B=$(realpath "$LIB_B")  # the JOB processes run elsewhere
: > $O/ab.txt
for round in 1 2; do
  for lib in "$LIB_A" "$LIB_B"; do
    n=$(basename $lib .so)
    FDLP_LIB=$lib timeout -k 10 200 python3 -u benchmarks/driver_e2e.py --utts 1800 --nj 8 --jobs-per-gpu 4 --trace-dir $O/tr_${n}_$round > $O/e2e_${n}_$round.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 2; }
    FDLP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_EXTRA:-} > $O/bench_run.log 2>&1 || { tail -20 $O/bench_run.log; exit 3; }
    python3 -c "
import json,sys
e=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
t=d.get('with_transfers') or {}
print(sys.argv[1], 'e2e', round(e['value'],3), 'cold_job_wall', e['one_cold_job']['process_wall_s'], 'exec', e['one_cold_job']['execution_time_s'], '| bench', round(d['value'],1), 'xfer', round(t.get('value',0) or 0,1))" $n $O/e2e_${n}_$round.json $O/bench_run.log >> $O/ab.txt
  done
done
cat $O/ab.txt
