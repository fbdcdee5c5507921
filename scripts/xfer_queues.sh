#!/usr/bin/env bash
# PCIe-inclusive bench pass vs the stream / hardware-queue layout (GPU_MAX_HW_QUEUES is 4 per process on
# the box; 4 compute streams + the H2D and D2H streams share them).  Outputs under gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-xq}
D=gpurun_out/$TAG
mkdir -p $D
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); x=d['with_transfers']; print(sys.argv[2], round(d['value'],1), 'xfer', round(x['value'],1), round(x['ms_per_step'],2), 'mapped', round(x['mapped_output']['value'],1))" "$1" "$2"; }
run() { name=$1; shift; timeout -k 10 240 "$@" > $D/$name.log 2>&1 || { echo "$name failed"; tail -5 $D/$name.log; exit 3; }; summ $D/$name.log $name; }
run base python3 bench.py --no-cpu-baseline --steps 10
run c2 python3 bench.py --no-cpu-baseline --steps 10 --xfer-compute-streams 2
run c3 python3 bench.py --no-cpu-baseline --steps 10 --xfer-compute-streams 3
run q8 env GPU_MAX_HW_QUEUES=8 python3 bench.py --no-cpu-baseline --steps 10
run q8d2 env GPU_MAX_HW_QUEUES=8 python3 bench.py --no-cpu-baseline --steps 10 --xfer-d2h-streams 2
