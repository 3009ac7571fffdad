#!/bin/bash
# Developer tool: builds tools/variants/libkbg_tools_<name>.so, the kernel
# benchmark library with kbg_kernels.hip compiled under experiment macros
# (name=flags pairs), for tools/ff_bench.py (TOOLS_LIB=...). Not shipped.
set -e
cd "$(dirname "$0")/.."
make -s tools
for spec in "$@"; do
  name=${spec%%=*}
  flags=${spec#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC -ffp-contract=off -fno-fast-math -I../include $flags --offload-arch=gfx950 \
    -c csrc/kbg_kernels.hip -o build/kern_$name.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/variants/libkbg_tools_$name.so build/engine_bench.o \
    build/kern_$name.o build/kbg_static.o build/kbg_affinity.o build/kbg_comm.o -L/opt/rocm/lib -lrccl -lpthread
  echo "built $name ($flags)"
done
