cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06l
B=32 timeout -k 10 200 python tools/probes/dg_trace.py > gpurun_out/r06l/trace_b32.txt 2>&1 || exit $?
B=256 timeout -k 10 200 python tools/probes/dg_trace.py > gpurun_out/r06l/trace_b256.txt 2>&1 || exit $?
OUT=gpurun_out/r06l STAGES='profbeam' PROF_BEAM=16 PROF_BATCHES='256 128' PROF_STEPS=4 bash tools/gpu_session.sh
