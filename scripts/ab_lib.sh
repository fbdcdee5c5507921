#!/usr/bin/env bash
# A/B of the default library against a variant build (FDLP_LIB=ablib/<name>.so): parity subset on the
# variant, then alternating bench lines and one kernel trace each.   VAR=libfdlp_sb TAG=x bash scripts/ab_lib.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abl}
mkdir -p $O
VL=$PWD/ablib/$VAR.so
FDLP_LIB=$VL timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_shape.py -k "${PYTEST_K:-golden or wsj or reverb or lpc}" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_var.log 2>&1 || { tail -30 $O/pytest_var.log; exit 2; }
tail -1 $O/pytest_var.log
for i in 1 2; do
  for v in base var; do
    lib=$PWD/speech_recognition_tools_amd/lib/libfdlp_hip.so; [ $v = var ] && lib=$VL
    FDLP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-transfers ${BENCH_EXTRA:-} > $O/$v$i.log 2>&1 || { tail -5 $O/$v$i.log; exit 3; }
    grep "^{" $O/$v$i.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v$i', round(d['value'],1), 'one', round(d['one_batch_in_flight']['value'],1), {k: round(x,3) for k,x in d['stage_ms_per_step'].items()})"
  done
done
