set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for bf in 8192 4096; do
timeout -k 10 600 python -u benchmarks/cli_throughput.py --utts 9000 --workers 8 --runners native --batch-frames $bf \
  --variants - keep_warm d2h_codes=off --repeat 2 --trace-dir $O/traces_$bf >> $O/cli.jsonl 2>> $O/cli.err || { tail -20 $O/cli.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05j/cli.jsonl"):
    r = json.loads(l); s = r["job_stats"]
    print(r["batch_frames"], r["variant"], r["repeat"], round(r["value"], 1), round(r["seconds"], 3), {k: round(v, 4) if isinstance(v, float) else v for k, v in s.items() if k in ("setup_seconds", "plan_seconds", "write_seconds", "widen_seconds", "d2h_wait_seconds", "slot_wait_seconds", "read_wait_seconds", "warm", "codes")})
PY
timeout -k 10 300 python -u benchmarks/driver_e2e.py --utts 1800 --nj 8 > $O/driver.json 2> $O/driver.err || { tail -20 $O/driver.err; exit 1; }
cat $O/driver.json
