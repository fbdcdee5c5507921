#!/usr/bin/env bash
# rocprofv3 kernel-trace stats of a short bench run, then PMC passes (separate runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd_root=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
BARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py $BARGS > gpurun_out/prof/trace.log 2>&1 || { echo "trace run failed"; tail -20 gpurun_out/prof/trace.log; exit 3; }
tail -2 gpurun_out/prof/trace.log
for pmc in "${PMC_SETS[@]:-FETCH_SIZE}"; do :; done
i=0
for pmc in ${PMC_LIST:-"FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"}; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $pmc -d gpurun_out/prof/pmc_$i -o run -- python3 bench.py $BARGS > gpurun_out/prof/pmc_$i.log 2>&1 || { echo "pmc $pmc failed"; tail -20 gpurun_out/prof/pmc_$i.log; exit 4; }
done
find gpurun_out/prof -name "*.csv" | head -50
