cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-variants > gpurun_out/sp.json 2> gpurun_out/sp.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sp.json')); print('run $r', d['value'], d['roofline']['kernel_ms_avg'])"
done
