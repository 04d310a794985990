# recurrence phase trace with the libm cell and the hardware-exp cell (diagnostic)
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/rec_trace.py > gpurun_out/rt_libm.txt 2>&1 || exit 1
CASR_REC_FASTCELL=1 timeout -k 10 200 python tools/rec_trace.py > gpurun_out/rt_fast.txt 2>&1 || exit 1
cat gpurun_out/rt_libm.txt gpurun_out/rt_fast.txt | grep -v amdgpu.ids
