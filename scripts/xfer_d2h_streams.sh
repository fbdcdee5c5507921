#!/usr/bin/env bash
# PCIe pass (double-buffered) vs device-to-host copy streams and hardware queues per process, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-xds}
D=gpurun_out/$TAG
mkdir -p $D
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); x=d['with_transfers']; print(sys.argv[2], round(d['value'],1), 'xfer', round(x['value'],1), round(x['ms_per_step'],2))" "$1" "$2"; }
run() { name=$1; shift; timeout -k 10 240 "$@" > $D/$name.log 2>&1 || { echo "$name failed"; tail -5 $D/$name.log; exit 3; }; summ $D/$name.log $name; }
run d1 python3 bench.py --no-cpu-baseline --steps 10
run q8d1 env GPU_MAX_HW_QUEUES=8 python3 bench.py --no-cpu-baseline --steps 10
run q8d2 env GPU_MAX_HW_QUEUES=8 python3 bench.py --no-cpu-baseline --steps 10 --xfer-d2h-streams 2
run q8d4 env GPU_MAX_HW_QUEUES=8 python3 bench.py --no-cpu-baseline --steps 10 --xfer-d2h-streams 4
run q12d4 env GPU_MAX_HW_QUEUES=12 python3 bench.py --no-cpu-baseline --steps 10 --xfer-d2h-streams 4
run q16d8 env GPU_MAX_HW_QUEUES=16 python3 bench.py --no-cpu-baseline --steps 10 --xfer-d2h-streams 8
run q8d4b env GPU_MAX_HW_QUEUES=8 python3 bench.py --no-cpu-baseline --steps 10 --xfer-d2h-streams 4
