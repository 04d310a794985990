#!/bin/bash
# mk_variant.sh NAME SOURCE [FLAGS...]: relink libcasr_hip.so's objects with one source recompiled
# (SOURCE: a csrc .hip file name under FLAGS such as ablation macros, or a path to an edited copy
# of one, which replaces the csrc object of the same base name up to its first '_' or '.') as
# chinese-asr_amd/casr/libcasr_hip_NAME.so
set -e
cd "$(dirname "$0")/../.."
L=chinese-asr_amd/casr
name=$1; src=$2; shift 2
if [ -f "$src" ]; then path=$src; else path=chinese-asr_amd/csrc/$src; fi
base=$(basename "$src"); base=${base%%.*}; base=${base%%_*}
mkdir -p /tmp/casr_var
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Iinclude \
  -Ichinese-asr_amd/csrc "$@" -c "$path" -o /tmp/casr_var/$name.o
objs=$(ls $L/_obj/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/libcasr_hip_$name.so $objs /tmp/casr_var/$name.o
echo $L/libcasr_hip_$name.so
