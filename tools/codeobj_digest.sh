#!/bin/bash
# Developer tool: digest of the gfx950 device assembly of every product kernel
# file (comments and blank lines dropped), to show that a source refactor
# leaves the shipped code objects unchanged.  Usage: codeobj_digest.sh [out dir]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=${1:-/tmp/codeobj}
mkdir -p $O
for f in sv_kernels sv_comb sv_hash; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S \
      $R/stellar-core_amd/csrc/$f.hip -o $O/$f.s
  grep -v '^\s*;' $O/$f.s | grep -v '^\s*$' | grep -v '\.file\|\.ident\|amdhsa.target\|^\s*\.loc\|__hip_cuid' > $O/$f.clean.s
  echo "$f $(sha256sum < $O/$f.clean.s | cut -c1-16) $(wc -l < $O/$f.clean.s) lines"
done
