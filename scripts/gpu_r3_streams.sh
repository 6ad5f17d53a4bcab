#!/bin/bash
# GPU box job: PMC check of the per-stream traffic model with two diagnostic builds (wrong results,
# timing/traffic only): d_sparse stores alpha at one step in three (WRITE_SIZE drops by 2/3 of the
# alpha stores), d_noconv skips the F pass's input staging (FETCH_SIZE drops by the F-pass inputs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PB="--steps 4 --warmup 1 --cpu-sample 0 --no-variants"
TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_d_sparse.so timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/streams -o sparse_write --output-format csv -- python3 bench.py $PB > gpurun_out/streams1.log 2>&1 || { echo "sparse failed"; tail -20 gpurun_out/streams1.log; exit 1; }
TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_d_noconv.so timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/streams -o noconv_fetch --output-format csv -- python3 bench.py $PB > gpurun_out/streams2.log 2>&1 || { echo "noconv failed"; tail -20 gpurun_out/streams2.log; exit 1; }
ls gpurun_out/streams
