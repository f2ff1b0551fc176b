#!/bin/bash
# Phase stamps of the final engines (mesh at the metric shape, gather at config 2, tiled for
# comparison) and the config-3 split probe, for profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OTF_STALL_MS=3000
timeout -k 10 60 ./tools/stamps_resident 4096 mesh > gpurun_out/ev_mesh.txt 2>&1 || exit 1
timeout -k 10 60 ./tools/stamps_resident 4096 tiled > gpurun_out/ev_tiled.txt 2>&1 || exit 1
timeout -k 10 60 ./tools/stamps_resident 512 gather double > gpurun_out/ev_gather.txt 2>&1 || exit 1
timeout -k 10 200 python tools/c3_probe.py > gpurun_out/ev_c3.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-gw --no-config5 --no-cpu-baseline --no-hbm-probe > gpurun_out/ev_bench_b.log 2>&1 || exit 1
echo done
