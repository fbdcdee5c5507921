set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ph
for b in 1 6 7; do
  for v in "" 1; do
    FDLP_LPC_SLOTMAJOR=$v timeout -k 5 60 ./benchmarks/lpc_env_p$b 2>&1 | grep -v amdgpu.ids | sed "s/^/slotmajor=$v /" || exit 3
  done
done
for v in "" 1; do
  if [ -n "$v" ]; then export FDLP_LPC_SLOTMAJOR=1; fi
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/ph/pmc$v -o run -- ./benchmarks/lpc_env_p1 > gpurun_out/ph/pmc$v.log 2>&1 || exit 4
done
