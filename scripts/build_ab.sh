#!/usr/bin/env bash
# Build two library variants for an on-box A/B (scripts/gpu_libab.sh): the committed tree (REF, default HEAD)
# and the working tree, as speech_recognition_tools_amd/lib/ab/{base,new}.so.
#   [REF=HEAD] bash scripts/build_ab.sh
set -eu
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/speech_recognition_tools_amd/lib/ab
mkdir -p $OUT
WT=/tmp/fdlp_ab_base
rm -rf $WT; git worktree prune
git worktree add -f --detach $WT ${REF:-HEAD} > /dev/null
python3 -c "
import importlib.util, sys
for root, out in (('$WT', '$OUT/base.so'), ('$ROOT', '$OUT/new.so')):
    spec = importlib.util.spec_from_file_location('b', root + '/speech_recognition_tools_amd/_build.py')
    m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
    m.build(force=True, out=out)
    print('built', out)
"
git worktree remove --force $WT
