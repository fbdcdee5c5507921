set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05l; mkdir -p $O
run() { echo "== $*" >> $O/init_env.txt; for k in 1 2 3; do env "$@" timeout -k 10 60 ./benchmarks/hip_init_probe cmhs >> $O/init_env.txt 2>&1 || return 1; done; }
run A=1 && run GPU_MAX_HW_QUEUES=1 && run GPU_MAX_HW_QUEUES=2 && run AMD_DIRECT_DISPATCH=0 && run HIP_LAZY=1 && run AMD_SERIALIZE_KERNEL=0 HSA_ENABLE_INTERRUPT=0 && run HSA_CU_MASK_SKIP_INIT=1 && run ROCR_VISIBLE_DEVICES=0 && run HSA_ENABLE_IPC_MODE_LEGACY=0 HIP_INITIAL_DM_SIZE=0
which strace ltrace perf > $O/tools.txt 2>&1 || true
cat $O/init_env.txt
