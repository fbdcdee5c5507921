# Batches in flight 4 / 6 / 8 alternating on one box, device-resident and PCIe-inclusive:
#   TAG=x bash scripts/gpu_inflight.sh
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${TAG:-inflight}; mkdir -p $O; : > $O/ab.txt
for round in 1 2; do
  for n in ${INFLIGHT:-4 6 8}; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --xfer-variants "" --inflight $n ${BENCH_EXTRA:-} > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 3; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); t=d.get('with_transfers') or {}
print('inflight', sys.argv[1], round(d['value'],1), 'xfer', round(t.get('value',0) or 0,1), 'ratio', round((t.get('value',0) or 0)/d['value'],3))" $n $O/run.log >> $O/ab.txt
  done
done
cat $O/ab.txt
