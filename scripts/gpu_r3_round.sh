#!/bin/bash
# GPU box job (round 3): parity suite, smoke, the default bench line, the config-4 shard on one GPU,
# and the two-rank torchrun rehearsal of config 4 (both ranks on the one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
[ -n "$SKIP_BENCH" ] && exit 0
echo "== bench"
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-600 gpurun_out/bench.json
echo "== config-4 shard"
timeout -k 10 600 python bench.py --batch 32768 --steps 4 --warmup 1 --cpu-sample 0 --no-variants > gpurun_out/bench_b32768.json 2> gpurun_out/bench_b32768.err || { echo "bench32768 failed rc=$?"; tail -30 gpurun_out/bench_b32768.err; exit 1; }
cut -c1-400 gpurun_out/bench_b32768.json
echo "== torchrun 2 ranks"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { echo "torchrun failed rc=$?"; tail -30 gpurun_out/bench_n2.err; exit 1; }
cut -c1-400 gpurun_out/bench_n2.json
