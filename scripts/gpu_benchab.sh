# bench.py variants alternating on one box (device-resident and PCIe-inclusive lines):
#   TAG=x VARIANTS="--xfer-threads 1|--xfer-threads 2" ROUNDS=2 bash scripts/gpu_benchab.sh
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${TAG:-benchab}; mkdir -p $O; : > $O/ab.txt
IFS='|' read -ra VS <<< "$VARIANTS"
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --xfer-variants "" $v > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 3; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); t=d.get('with_transfers') or {}
print(repr(sys.argv[1]), round(d['value'],1), 'xfer', round(t.get('value',0) or 0,1), 'ratio', round((t.get('value',0) or 0)/d['value'],3), 'bitid', t.get('codes_widen_bit_identical'))" "$v" $O/run.log >> $O/ab.txt
  done
done
cat $O/ab.txt
