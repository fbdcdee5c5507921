#!/usr/bin/env bash
# D2H event spans in bench.py's PCIe pass (benchmarks/d2h_probe.py --pipeline) at 1, 2 and 4 batches in flight:
# does a batch's 65.5 MB copy run slowly, or wait behind the other batches' copies on the copy engine?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-d2hk}; mkdir -p $O; : > $O/d2h_k.jsonl
for k in ${KS:-1 2 4}; do
  echo "# --k=$k ${EXTRA:-}" >> $O/d2h_k.jsonl
  timeout -k 10 300 python3 benchmarks/d2h_probe.py --pipeline --k=$k ${EXTRA:-} ${VARIANTS:-stream} >> $O/d2h_k.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
cat $O/d2h_k.jsonl
