#!/bin/bash
# r05 profiles for profiles/: rocprofv3 kernel traces of the float64 headline step, the
# float32 leg and the config-5 sweep (bench.py --profile-only ...), then one PMC pass per
# counter (FETCH_SIZE, WRITE_SIZE) for each (counters in their own runs, kernel trace only).
# Summarise afterwards here: python tools/summarize_profile.py r05
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --profile-only --steps ${PSTEPS:-5} --warmup 1"
run() {  # $1 = dir, $2 = limit, rest = rocprofv3 options before --, then bench flags after ::
  local dir=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > gpurun_out/$dir.log 2>&1
  local rc=$?; echo "$dir rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$dir.log; exit $rc; fi
}
run prof 300 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- $B
run prof_f32 300 --kernel-trace --stats -d gpurun_out/prof_f32 -o run --output-format csv -- $B --profile-f32
run prof_c5 300 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- $B --profile-config5
for c in FETCH_SIZE WRITE_SIZE; do
  run pmc_${c}_auto 240 --pmc $c --kernel-trace -d gpurun_out/pmc_${c}_auto -o run --output-format csv -- $B
  run pmc_${c}_f32 240 --pmc $c --kernel-trace -d gpurun_out/pmc_${c}_f32 -o run --output-format csv -- $B --profile-f32
  run pmc_${c}_c5 240 --pmc $c --kernel-trace -d gpurun_out/pmc_${c}_c5 -o run --output-format csv -- $B --profile-config5
done
run pmc_MFMA_auto 240 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_MFMA_auto -o run --output-format csv -- $B
echo done
