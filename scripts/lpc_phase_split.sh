#!/usr/bin/env bash
# Time the cepstrum/envelope kernel of a config with phases masked out (timing builds under ablib/,
# -DFDLP_LPC_PHASES: bit 1 cepstrum, bit 2 envelope; results of those builds are not features).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-reverb}
O=gpurun_out/${TAG:-lps}
mkdir -p $O
for v in full ph3 ph5 ph1; do
  lib=$PWD/speech_recognition_tools_amd/lib/libfdlp_hip.so
  [ $v != full ] && lib=$PWD/ablib/libfdlp_$v.so
  FDLP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-transfers --inflight 1 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 3; }
  python3 scripts/rocpd_summary.py $O/$v/run_results.db $O/$v.csv > /dev/null
  echo "$v $(grep -E 'lattice' $O/$v.csv | cut -d, -f1,4 | cut -c1-120)"
  find $O/$v -name "*.db" -delete
done
