#!/bin/bash
# round 5: windowed-kernel parity (tests/test_gpu_window.py + the compat schedule) then config-5
# A/B of the libvar_*.so builds in interleaved rounds (TESTS=0 skips the tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/w5
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTSEL:-tests/test_gpu_window.py tests/test_gpu_decode.py::test_compat_window_schedule} > gpurun_out/w5/pytest.txt 2>&1
  rc=$?; tail -15 gpurun_out/w5/pytest.txt; [ $rc = 0 ] || exit $rc
fi
WB="--window 64 --batch 32768 --steps ${STEPS:-3} --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0 ${EXTRA:-}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in turbo_decoder_cuda_amd/libvar_*.so; do
    TD_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py $WB > gpurun_out/w5/v.json 2> gpurun_out/w5/v.err || { echo "$lib rc=$?"; tail -20 gpurun_out/w5/v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/w5/v.json')); print('round $r', '$lib'.split('/')[-1].ljust(24), d['value'], d['roofline']['kernel_ms_avg'], d['roofline'].get('demux_ms_avg'), d['ber']['bit_errors'])"
  done
done
