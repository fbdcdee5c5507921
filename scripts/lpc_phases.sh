set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ph
for b in 1 6 7; do
  timeout -k 5 60 ./benchmarks/lpc_env_p$b 2>&1 | grep -v amdgpu.ids || exit 3
done
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/ph/pmc -o run -- ./benchmarks/lpc_env_p1 > gpurun_out/ph/pmc.log 2>&1 || exit 4
