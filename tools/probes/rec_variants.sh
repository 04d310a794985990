# recurrence phase traces under the tuning knobs (diagnostic)
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/rec_trace.py > gpurun_out/rt_base.txt 2>&1 || exit 1
CASR_REC_RG=16 timeout -k 10 200 python tools/rec_trace.py > gpurun_out/rt_rg16.txt 2>&1 || exit 1
CASR_REC_RG=16 CASR_REC_FASTCELL=1 timeout -k 10 200 python tools/rec_trace.py > gpurun_out/rt_rg16f.txt 2>&1 || exit 1
for f in base rg16 rg16f; do echo "== $f"; grep -v amdgpu.ids gpurun_out/rt_$f.txt; done
