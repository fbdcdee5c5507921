set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 400 python3 -u benchmarks/durbin4_accuracy.py > $O/durbin4_accuracy.jsonl 2> $O/durbin4_accuracy.err || { tail -20 $O/durbin4_accuracy.err; exit 1; }
cat $O/durbin4_accuracy.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
