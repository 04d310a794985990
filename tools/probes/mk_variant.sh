#!/bin/bash
# mk_variant.sh NAME SOURCE FLAGS...: relink libcasr_hip.so's objects with SOURCE (a csrc .hip file
# name) recompiled under FLAGS (ablation macros) as chinese-asr_amd/casr/libcasr_hip_NAME.so
set -e
cd "$(dirname "$0")/../.."
L=chinese-asr_amd/casr
name=$1; src=$2; shift 2
mkdir -p /tmp/casr_var
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Iinclude \
  -Ichinese-asr_amd/csrc "$@" -c chinese-asr_amd/csrc/$src -o /tmp/casr_var/$name.o
objs=$(ls $L/_obj/*.o | grep -v "/${src%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/libcasr_hip_$name.so $objs /tmp/casr_var/$name.o
echo $L/libcasr_hip_$name.so
