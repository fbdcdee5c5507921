set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06i; mkdir -p $O; : > $O/ab.txt
for round in 1 2; do
for v in "--utts 1024 --inflight 4" "--utts 2048 --inflight 4" "--utts 2048 --inflight 2" "--utts 512 --inflight 8" "--utts 4096 --inflight 2"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-transfers $v > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 2; }
  python3 -c "
import json,sys; d=json.loads(open('$O/run.log').read().strip().splitlines()[-1])
print(sys.argv[1], round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1))" "$v" >> $O/ab.txt
done; done
cat $O/ab.txt
