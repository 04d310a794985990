#!/bin/bash
# Round-4 pass q: input-GEMM probe ablations on the round-4 code (persistent kernel: full, no k-loop
# DMA, no MFMA, no epilogue stores, DMA only), three reps, bitwise check of persist vs per-tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 200 ./tools/probes/gemm16_probe > $O/gemm16_probe.txt 2>&1 || { tail -5 $O/gemm16_probe.txt; exit 1; }
cat $O/gemm16_probe.txt
timeout -k 10 200 ./tools/probes/gemm16_pipe > $O/gemm16_pipe.txt 2>&1 || { tail -5 $O/gemm16_pipe.txt; exit 1; }
cat $O/gemm16_pipe.txt
