# round 4: the full GPU suite on the in-tree build, then the parity subset on each libvar_*.so given in PARITY_LIBS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r4/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "FAILED|Error" gpurun_out/r4/pytest_gpu.log | head -20; fi
[ $rc -le 1 ] || exit $rc
for v in $PARITY_LIBS; do
  TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_decode.py > gpurun_out/r4/parity_$v.log 2>&1
  rc=$?
  echo "parity $v rc=$rc: $(tail -1 gpurun_out/r4/parity_$v.log)"
  [ $rc -le 1 ] || exit $rc
done
