set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_ola.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -30 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
AB_ARGS="--ola-path auto|--ola-path separate" TAG=r05f TRACE=1 bash scripts/gpu_ab.sh || exit 2
for v in auto separate; do
  BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --inflight 1 --no-transfers --ola-path $v" PMC_TAG=r05f/pmc_$v bash scripts/pmc_kernel.sh FETCH_SIZE WRITE_SIZE "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" || exit 3
  python3 -c "
import json
d=json.load(open('gpurun_out/r05f/pmc_$v/pmc.json'))
for k,m in d.items():
    if 'lattice' in k or 'ola' in k: print('$v', k.split('(')[0][-40:], {c: '%.4g' % x for c,x in m.items()})"
done
find gpurun_out/r05f -name "*.db" -delete
