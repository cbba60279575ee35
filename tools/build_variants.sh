#!/bin/bash
# Developer tool: build compile-time variants of the verify library for GPU
# A/B timing (tools/ab_variants.py).  Usage: build_variants.sh name "-DFLAG=1" [name "-D..."]...
set -e
cd "$(dirname "$0")/.."
mkdir -p variants/build
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c stellar-core_amd/csrc/sv_kernels.hip \
      -o variants/build/k_$name.o &
done
wait
for o in variants/build/k_*.o; do
  name=${o#variants/build/k_}; name=${name%.o}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libsv_$name.so $o \
      stellar-core_amd/build/sv_api.o stellar-core_amd/build/sv_comb.o stellar-core_amd/build/sv_hash.o stellar-core_amd/build/sv_cpu.o -Wl,-rpath,/opt/rocm/lib -lpthread
done
ls -la variants/*.so
