set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo | grep -m1 gfx950 > gpurun_out/arch.txt || true
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/t1.log 2>&1
