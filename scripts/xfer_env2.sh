#!/usr/bin/env bash
# PCIe-inclusive bench pass under SDMA engine-selection settings (ROCr environment), one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-xe2}
D=gpurun_out/$TAG
mkdir -p $D
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); x=d['with_transfers']; print(sys.argv[2], round(d['value'],1), 'xfer', round(x['value'],1), round(x['ms_per_step'],2))" "$1" "$2"; }
run() { name=$1; shift; timeout -k 10 240 "$@" > $D/$name.log 2>&1 || { echo "$name failed"; tail -5 $D/$name.log; exit 3; }; summ $D/$name.log $name; }
run base python3 bench.py --no-cpu-baseline --steps 10
run receng0 env HSA_ENABLE_SDMA_RECOMMENDED_ENG=0 python3 bench.py --no-cpu-baseline --steps 10
run receng1 env HSA_ENABLE_SDMA_RECOMMENDED_ENG=1 python3 bench.py --no-cpu-baseline --steps 10
run gang1 env HSA_ENABLE_SDMA_GANG=1 python3 bench.py --no-cpu-baseline --steps 10
run hdp0 env HSA_ENABLE_SDMA_HDP_FLUSH=0 python3 bench.py --no-cpu-baseline --steps 10
