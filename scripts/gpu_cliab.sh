# Warm CLI (10 audio-hours of WAVs -> ark) and the cold 8-JOB driver with two builds of the library,
# alternating on one box (FDLP_LIB):  LIB_A=path LIB_B=path TAG=x bash scripts/gpu_cliab.sh
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-cliab}; mkdir -p $O; : > $O/ab.txt
LIB_A=$(realpath "$LIB_A"); LIB_B=$(realpath "$LIB_B")
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_cli.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for round in 1 2; do
  for lib in "$LIB_A" "$LIB_B"; do
    n=$(basename $lib .so)
    FDLP_LIB=$lib timeout -k 10 300 python3 -u benchmarks/cli_throughput.py --utts 9000 --workers 8 --runners native --variants keep_warm --repeat 2 --batch-frames 4096 > $O/cli_${n}_$round.jsonl 2> $O/cli.err || { tail -20 $O/cli.err; exit 2; }
    FDLP_LIB=$lib timeout -k 10 200 python3 -u benchmarks/driver_e2e.py --utts 1800 --nj 8 --jobs-per-gpu 4 > $O/e2e_${n}_$round.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 3; }
    python3 -c "
import json,sys
c=[json.loads(l) for l in open(sys.argv[2]) if l.startswith('{')]
e=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1], 'cli', [round(x['value'],1) for x in c], 'setup', [round(x['job_stats']['setup_seconds'],3) for x in c], '| e2e', round(e['value'],3), 'cold_wall', e['one_cold_job']['process_wall_s'])" $n $O/cli_${n}_$round.jsonl $O/e2e_${n}_$round.json >> $O/ab.txt
  done
done
cat $O/ab.txt
