#!/bin/bash
# A/B of the PCIe-inclusive bench pass: stream layout and SDMA vs blit-kernel copies.
# Usage (GPU box): bash scripts/xfer_ab.sh [TAG]
set -e
export TMPDIR=/tmp
TAG=${1:-xab}
D=gpurun_out/$TAG
mkdir -p $D
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); x=d['with_transfers']; print(sys.argv[2], round(d['value'],1), round(x['value'],1), round(x['ms_per_step'],2), round(x['mapped_output']['value'],1))" "$1" "$2"; }
run() { name=$1; shift; timeout -k 10 240 "$@" > $D/$name.log 2>&1; summ $D/$name.log $name; }
run base python bench.py --no-cpu-baseline --steps 10
run c2 python bench.py --no-cpu-baseline --steps 10 --xfer-compute-streams 2
run c2d2 python bench.py --no-cpu-baseline --steps 10 --xfer-compute-streams 2 --xfer-d2h-streams 2
run blit env HSA_ENABLE_SDMA=0 python bench.py --no-cpu-baseline --steps 10
run blit_c2 env HSA_ENABLE_SDMA=0 python bench.py --no-cpu-baseline --steps 10 --xfer-compute-streams 2
