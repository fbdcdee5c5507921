#!/usr/bin/env bash
# PMC passes (one counter group per run) over a short bench; writes rocpd dbs under gpurun_out/pmc_*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
BARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
i=0
for grp in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_$i -o run -- python3 bench.py $BARGS > gpurun_out/pmc_$i.log 2>&1 || { echo "pmc group $i failed"; tail -5 gpurun_out/pmc_$i.log; exit 4; }
done
echo pmc done
