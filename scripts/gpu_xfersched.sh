# The PCIe pass's copy schedules alternating on one box: streams (H2D stream + D2H streams) vs grouped
# (one copy stream, next step's copy-ins then this step's copy-outs):  TAG=x bash scripts/gpu_xfersched.sh
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${TAG:-xfersched}; mkdir -p $O; : > $O/ab.txt
for round in 1 2 3; do
  for sch in streams grouped; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --xfer-variants "" --xfer-schedule $sch ${BENCH_EXTRA:-} > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 3; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); t=d.get('with_transfers') or {}
print(sys.argv[1], round(d['value'],1), 'xfer', round(t.get('value',0) or 0,1), 'ratio', round((t.get('value',0) or 0)/d['value'],3), 'flagged', t.get('codes_flagged_batches'), 'bitid', t.get('codes_widen_bit_identical'))" $sch $O/run.log >> $O/ab.txt
  done
done
cat $O/ab.txt
