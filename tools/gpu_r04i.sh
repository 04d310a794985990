#!/bin/bash
# Round-4 pass i: ablation phase traces. Beam fused-GEMM epilogue without its row partials (d16),
# logits stores (d32), tile maxima (d64), all three (d112); greedy attention prologue without its
# W_hidden loads (a1), its gate-row gather (a2), both (a3). Results are wrong in these builds:
# timing only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
L=chinese-asr_amd/casr
cp $L/libcasr_hip.so /tmp/casr_base.so
restore() { cp /tmp/casr_base.so $L/libcasr_hip.so; touch $L/libcasr_hip.so; }
for n in base d16 d32 d64 d112 base2; do
  case $n in base*) cp /tmp/casr_base.so $L/libcasr_hip.so;; *) cp $L/libcasr_hip_$n.so $L/libcasr_hip.so;; esac
  touch $L/libcasr_hip.so
  BEAM=1 BB=256 K=8 timeout -k 10 150 python tools/probes/dg_trace.py > $O/beam_$n.txt 2>&1 || { tail -5 $O/beam_$n.txt; restore; exit 1; }
  echo "== $n"; grep -A6 "^proj (beam)" $O/beam_$n.txt | grep "proj\|k loop\|epilogue\|block "
done
for n in base a1 a2 a3 base2; do
  case $n in base*) cp /tmp/casr_base.so $L/libcasr_hip.so;; *) cp $L/libcasr_hip_$n.so $L/libcasr_hip.so;; esac
  touch $L/libcasr_hip.so
  timeout -k 10 150 python tools/probes/dg_trace.py > $O/greedy_$n.txt 2>&1 || { tail -5 $O/greedy_$n.txt; restore; exit 1; }
  echo "== $n"; grep -A10 "^attention (greedy)" $O/greedy_$n.txt
done
restore
timeout -k 10 120 ./tools/probes/logmel_variants_ni > $O/logmel_variants_ni.txt 2>&1 || { tail -5 $O/logmel_variants_ni.txt; exit 1; }
cat $O/logmel_variants_ni.txt
