#!/usr/bin/env bash
# PCIe-inclusive bench pass under copy-engine settings (ROCclr / ROCr environment), one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-xe}
D=gpurun_out/$TAG
mkdir -p $D
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); x=d['with_transfers']; print(sys.argv[2], round(d['value'],1), 'xfer', round(x['value'],1), round(x['ms_per_step'],2), 'mapped', round(x['mapped_output']['value'],1))" "$1" "$2"; }
run() { name=$1; shift; timeout -k 10 240 "$@" > $D/$name.log 2>&1 || { echo "$name failed"; tail -5 $D/$name.log; exit 3; }; summ $D/$name.log $name; }
run base python3 bench.py --no-cpu-baseline --steps 10
run nosdma env HSA_ENABLE_SDMA=0 python3 bench.py --no-cpu-baseline --steps 10
run forceblit env GPU_FORCE_BLIT_COPY_SIZE=1048576 python3 bench.py --no-cpu-baseline --steps 10
run nosdma_wg64 env HSA_ENABLE_SDMA=0 DEBUG_CLR_LIMIT_BLIT_WG=64 python3 bench.py --no-cpu-baseline --steps 10
run base2 python3 bench.py --no-cpu-baseline --steps 10
