#!/bin/bash
# EXPERIMENT: mesh column hops with plain stores (column tile = XCD under round-robin).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=2000
timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/st_mesh_sc1.txt 2>&1; rc=$?; cat gpurun_out/st_mesh_sc1.txt
[ $rc -eq 0 ] || exit $rc
OTF_MESH_PLAIN=1 timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/st_mesh_plain.txt 2>&1; rc=$?; cat gpurun_out/st_mesh_plain.txt
[ $rc -eq 0 ] || exit $rc
OTF_MESH_PLAIN=1 OTF_MESH_XCD_ROWS=1 timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/st_mesh_plainx.txt 2>&1; rc=$?; cat gpurun_out/st_mesh_plainx.txt
