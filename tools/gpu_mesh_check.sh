#!/bin/bash
# Mesh engine: stamps of the given variants, then the mesh / parity GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_mesh_stamps.sh "$@" || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mesh_tests.log 2>&1
rc=$?; tail -5 gpurun_out/mesh_tests.log; echo "pytest rc=$rc"; exit $rc
