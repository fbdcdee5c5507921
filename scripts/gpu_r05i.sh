set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05i; mkdir -p $O
for s in cmhhpakPds cmpaahhkPds csmkkh cPmhh cmsfkk cmhh; do
  timeout -k 10 60 ./benchmarks/hip_init_probe $s >> $O/init.jsonl 2>&1 || exit 1
done
cat $O/init.jsonl
