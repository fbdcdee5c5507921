set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for bf in 4096 8192 2048; do
timeout -k 10 600 python -u benchmarks/cli_throughput.py --utts 9000 --workers 8 --runners native --batch-frames $bf \
  --variants keep_warm --repeat 3 --trace-dir $O/traces_$bf >> $O/cli.jsonl 2>> $O/cli.err || { tail -20 $O/cli.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05t/cli.jsonl"):
    r = json.loads(l); s = r["job_stats"]
    print(r["batch_frames"], r["variant"], r["repeat"], round(r["value"], 1), round(r["seconds"], 3), {k: round(v, 4) if isinstance(v, float) else v for k, v in s.items() if k in ("setup_seconds", "write_seconds", "widen_seconds", "slot_wait_seconds", "read_wait_seconds", "warm")})
PY
