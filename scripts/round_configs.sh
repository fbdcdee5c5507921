#!/usr/bin/env bash
# Bench lines of the other BASELINE.json configurations on one GPU box (REVERB M=450, LibriSpeech-scale
# lengths, two ranks sharing the GPU as a launcher check) -> gpurun_out/configs/<name>.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/configs
mkdir -p $O
timeout -k 10 300 python bench.py --config reverb > $O/reverb.log 2>&1 || { tail -20 $O/reverb.log; exit 3; }
tail -1 $O/reverb.log > $O/reverb.json
timeout -k 10 300 python bench.py --workload librispeech > $O/librispeech.log 2>&1 || { tail -20 $O/librispeech.log; exit 4; }
tail -1 $O/librispeech.log > $O/librispeech.json
timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline > $O/2rank_1gpu.log 2>&1 || { tail -20 $O/2rank_1gpu.log; exit 5; }
tail -1 $O/2rank_1gpu.log > $O/2rank_1gpu.json
for n in reverb librispeech 2rank_1gpu; do grep -o '"value": [0-9.]*' $O/$n.json | head -1 | sed "s/^/$n /"; done
