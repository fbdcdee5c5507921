#!/usr/bin/env bash
# End-to-end measurements on one GPU box: CLI tests, in-process CLI throughput (native runner with the D2H
# copy and with mapped output), the recipe-level driver run with cold JOBs, and the full default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-e2e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_cli.log 2>&1 || { echo "cli tests failed"; tail -30 $O/pytest_cli.log; exit 2; }
tail -1 $O/pytest_cli.log
timeout -k 10 600 python benchmarks/cli_throughput.py --utts ${CLI_UTTS:-4096} --workers 4 --batch-frames 2048 --runners native native_mapped > $O/cli_throughput.jsonl 2> $O/cli_throughput.err || { echo "cli_throughput failed"; tail -20 $O/cli_throughput.err; exit 3; }
python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print('cli', d['host_runner'], round(d['value'],1), 'audio-h/s', round(d['seconds'],3), 's')" $O/cli_throughput.jsonl
timeout -k 10 900 python benchmarks/driver_e2e.py --utts ${E2E_UTTS:-1800} --nj ${E2E_NJ:-8} > $O/driver_e2e.json 2> $O/driver_e2e.err || { echo "driver_e2e failed"; tail -30 $O/driver_e2e.err; exit 4; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); print('driver_e2e', round(d['value'],2), 'audio-h/s wall', round(d['wall_s'],2), 's jobs', d['job_execution_s'])" $O/driver_e2e.json
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 600 python bench.py > $O/bench_full.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_full.log; exit 5; }
tail -1 $O/bench_full.log > $O/bench_full.json
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); x=d['with_transfers']; print('bench', round(d['value'],1), 'xfer', round(x['value'],1), 'mapped', round(x['mapped_output']['value'],1), 'cpu', d['cpu_baseline'])" $O/bench_full.json
