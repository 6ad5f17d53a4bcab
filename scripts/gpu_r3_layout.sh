#!/bin/bash
# GPU box job (round 3): parity of each alpha-scratch layout variant (libvar_*.so via TD_LIB_PATH),
# then the placement spread of each with plain allocations, interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${LAYOUTS:-a_grp b_win c_step}; do
  TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode.py tests/test_gpu_handle.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { echo "pytest $v failed rc=$?"; tail -40 gpurun_out/pytest_$v.log; exit 1; }
  echo "== parity $v: $(tail -1 gpurun_out/pytest_$v.log)"
done
export TD_PLACEMENT_TRIALS=1
for r in 1 2; do
  for v in ${LAYOUTS:-a_grp b_win c_step}; do
    TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_$v.so timeout -k 10 300 python scripts/spread_probe.py 6 2 4 > gpurun_out/spread_${v}_$r.log 2>&1 || { echo "$v failed rc=$?"; tail -20 gpurun_out/spread_${v}_$r.log; exit 1; }
    echo "== round $r $v"; grep instance gpurun_out/spread_${v}_$r.log | sed 's/placement.*//'
  done
done
