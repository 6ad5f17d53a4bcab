# round 4: the window-residue parity tests (and the reference's golden frames) on the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py "tests/test_gpu_decode.py::test_window_edge_residues_vs_oracle" \
  "tests/test_gpu_decode.py::test_four_per_cu_w12_residues" > gpurun_out/r4/residues.log 2>&1
