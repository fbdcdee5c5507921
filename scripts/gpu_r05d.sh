set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_ola.py tests/test_bench_shape.py tests/test_compact_output.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1
rc=$?; tail -3 $O/pytest_fused.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest_fused.log | head -30; exit $rc; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --xfer-variants none > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 2; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); x=d['with_transfers']
print('value', round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), 'xfer', round(x['value'],1), 'ratio', round(x['value']/d['value'],3), {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 3; }
python3 scripts/rocpd_summary.py $O/trace/run_results.db $O/kernel_trace_stats.csv > /dev/null || true
rm -rf $O/trace
cat $O/kernel_trace_stats.csv | head -20
