#!/bin/bash
# Build the float64 mesh stamp tool for the library's source and for alternative sources
# (A/B on the box with tools/gpu_r05_ab.sh).  Usage: tools/build_stamps_ab.sh [alt.hip ...]
set -eu
cd "$(dirname "$0")/.."
CS=ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc
mkdir -p tools/bin
F="-O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -DOTF_M64_STAMPS -I include -I $CS"
/opt/rocm/bin/hipcc $F tools/stamps_mesh64.hip -o tools/bin/stamps_tree -ldl &
for a in "$@"; do
  n=$(basename $a .hip)
  /opt/rocm/bin/hipcc $F "-DOTF_M64_ALT=\"$PWD/$a\"" tools/stamps_mesh64.hip -o tools/bin/stamps_$n -ldl &
done
wait
ls -la tools/bin
