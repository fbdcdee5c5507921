set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
true || timeout -k 10 300 python -u -m pytest tests/test_compact_output.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
true
true || timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 2; }
true
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl -o run -- python3 bench.py --xfer-only --no-cpu-baseline --steps 6 --warmup 2 --xfer-d2h-streams 2 --xfer-variants none > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 3; }
python3 scripts/xfer_timeline.py $O/tl/run_results.db 80 > $O/timeline.txt 2>&1 || true
ls -la $O/tl; du -sh $O/tl
