set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
df -h /tmp > $O/df.txt 2>&1; nproc >> $O/df.txt; free -g >> $O/df.txt
timeout -k 10 120 python -u benchmarks/cold_start_probe.py > $O/cold.json 2> $O/cold.err || exit 1
cat $O/cold.json
timeout -k 10 600 python -u benchmarks/cli_throughput.py --utts 9000 --workers 4 8 16 --runners native --batch-frames 8192 > $O/cli.jsonl 2> $O/cli.err || { tail -20 $O/cli.err; exit 1; }
cat $O/cli.jsonl
timeout -k 10 300 python -u benchmarks/driver_e2e.py --utts 1800 --nj 8 > $O/driver.json 2> $O/driver.err || { tail -20 $O/driver.err; exit 1; }
cat $O/driver.json
