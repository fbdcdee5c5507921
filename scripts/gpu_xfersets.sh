# The PCIe pass with 2 / 3 / 4 device buffer sets per batch in flight, alternating on one box:
#   TAG=x bash scripts/gpu_xfersets.sh
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${TAG:-xfersets}; mkdir -p $O; : > $O/ab.txt
for round in 1 2; do
  for S in ${SETS:-2 3 4}; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --xfer-variants "" --xfer-sets $S ${BENCH_EXTRA:-} > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 3; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); t=d.get('with_transfers') or {}
print('sets', sys.argv[1], round(d['value'],1), 'xfer', round(t.get('value',0) or 0,1), 'ratio', round((t.get('value',0) or 0)/d['value'],3))" $S $O/run.log >> $O/ab.txt
  done
done
cat $O/ab.txt
