#!/bin/bash
# r05 evidence in one call: targeted tests, the fused-vs-two-call probe, float64 mesh
# phase stamps (fused and plain), the whole -m gpu suite, the default bench, then the
# rocprofv3 kernel traces + PMC passes (tools/gpu_r05_prof.sh).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05f}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # $1 = name, $2 = limit, rest = command
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-4} $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step first 300 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_mesh64.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider
step probe 200 python tools/pw_probe.py
if [ -x tools/st_pw ]; then
  export LD_LIBRARY_PATH=$PWD/ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/otfuse/lib:${LD_LIBRARY_PATH:-}
  TAILN=16 step stamps_pw 120 ./tools/st_pw 4096 100 pw
  TAILN=16 step stamps_plain 120 ./tools/st_pw 4096 100
fi
if [ "${FULL:-1}" = "1" ]; then
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider
fi
if [ "${BENCH:-1}" = "1" ]; then
  cp /dev/null $OUT/bench.log
  step bench 600 python bench.py
fi
if [ "${PROF:-1}" = "1" ]; then
  bash tools/gpu_r05_prof.sh || exit $?
fi
echo all done
