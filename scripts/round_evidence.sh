#!/usr/bin/env bash
# Round evidence on one GPU box: rocprofv3 kernel-trace stats and separate PMC passes (FETCH_SIZE /
# WRITE_SIZE / clocks+MFMA busy / VALU / LDS) of the same bench command, then the full bench (with CPU
# baseline), which reads its roofline traffic from the PMC summary written here first.
# Outputs under gpurun_out/evidence/; copy what is judged into profiles/ (see DESIGN.md).
# TAG (default r01x) names that summary: profiles/${TAG}_pmc.json (box-local copy for the bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01x}
O=gpurun_out/evidence_$TAG
mkdir -p $O
# one batch in flight for the trace and PMC passes: the kernels alone, as in the bench line's roofline pass
BARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py $BARGS > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 3; }
python3 scripts/rocpd_summary.py $O/trace/run_results.db $O/kernel_trace_stats.csv > /dev/null || true
# the trace run's own bench line (its HIP-event stage times come from the same process as the kernel trace)
# and the dominant stage's frac recomputed from the trace's kernel durations beside the HIP-event one
grep '"roofline"' $O/trace.log | tail -1 > $O/trace_bench_line.json
python3 scripts/frac_check.py $O/trace_bench_line.json $O/kernel_trace_stats.csv > $O/frac_check.json || true
cp $O/frac_check.json profiles/${TAG}_frac_check.json 2>/dev/null || true
i=0
for pmc in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc ${pmc//+/ } -d $O/pmc_$i -o run -- python3 bench.py $BARGS > $O/pmc_$i.log 2>&1 || { echo "pmc $pmc failed"; tail -20 $O/pmc_$i.log; exit 4; }
done
python3 scripts/pmc_report.py "$O/pmc_*/*.db" $O/pmc.json > $O/pmc.txt 2>&1 || true
cp $O/pmc.json profiles/${TAG}_pmc.json
# the raw databases stay on the box (gpurun copies back at most 64 MiB of gpurun_out/); KEEP_DB=1 keeps them
[ -z "${KEEP_DB:-}" ] && rm -rf $O/trace $O/pmc_*/
[ -n "${SKIP_BENCH:-}" ] && exit 0
timeout -k 10 600 python3 bench.py > $O/bench_full.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_full.log; exit 2; }
tail -1 $O/bench_full.log
