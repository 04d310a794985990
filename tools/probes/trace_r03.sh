cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/probes/dg_trace.py > gpurun_out/trace_greedy.txt 2>&1 || { tail gpurun_out/trace_greedy.txt; exit 1; }
BEAM=1 BB=256 timeout -k 10 120 python tools/probes/dg_trace.py > gpurun_out/trace_beam256.txt 2>&1 || { tail gpurun_out/trace_beam256.txt; exit 1; }
cat gpurun_out/trace_greedy.txt gpurun_out/trace_beam256.txt
