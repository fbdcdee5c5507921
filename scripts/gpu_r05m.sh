set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 120 ./benchmarks/write_probe /tmp 1100 > $O/write.jsonl || exit 1
grep -E "piece|\"write\"" $O/write.jsonl
for bf in 4096 8192; do
timeout -k 10 600 python -u benchmarks/cli_throughput.py --utts 9000 --workers 8 --runners native --batch-frames $bf \
  --variants keep_warm --repeat 3 --trace-dir $O/traces_$bf >> $O/cli.jsonl 2>> $O/cli.err || { tail -20 $O/cli.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05m/cli.jsonl"):
    r = json.loads(l); s = r["job_stats"]
    print(r["batch_frames"], r["variant"], r["repeat"], round(r["value"], 1), round(r["seconds"], 3), {k: round(v, 4) if isinstance(v, float) else v for k, v in s.items() if k in ("setup_seconds", "write_seconds", "widen_seconds", "d2h_wait_seconds", "slot_wait_seconds", "read_wait_seconds", "warm")})
PY
