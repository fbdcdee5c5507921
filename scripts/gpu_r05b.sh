set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
: > $O/sdma_env.jsonl
for v in base gang rec0 rec1 gangrec1 base; do
  case $v in
    base) E="";;
    gang) E="HSA_ENABLE_SDMA_GANG=1";;
    rec0) E="HSA_ENABLE_SDMA_RECOMMENDED_ENG=0";;
    rec1) E="HSA_ENABLE_SDMA_RECOMMENDED_ENG=1";;
    gangrec1) E="HSA_ENABLE_SDMA_GANG=1 HSA_ENABLE_SDMA_RECOMMENDED_ENG=1";;
  esac
  env GPU_MAX_HW_QUEUES=8 $E timeout -k 10 200 python3 benchmarks/d2h_probe.py --pipeline stream2 > $O/sdma_env_$v.out 2> $O/sdma_env.err || { tail -5 $O/sdma_env.err; exit 1; }
  sed "s/^{/{\"env\": \"$v\", /" $O/sdma_env_$v.out >> $O/sdma_env.jsonl
done
cat $O/sdma_env.jsonl
