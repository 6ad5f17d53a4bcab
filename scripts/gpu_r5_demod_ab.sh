set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for lib in turbo_decoder_cuda_amd/libvar_a_head.so turbo_decoder_cuda_amd/libturbo_mi355x.so; do
TD_LIB_PATH=$PWD/$lib timeout -k 10 120 python -c "
import bench, torch, json
class A: batch = 4096; K = 6144
r = bench.demod_rates(A, torch.device('cuda:0'))
print('$r', '$lib'.split('/')[-1], json.dumps({k: (v['ms'], v['hbm_frac']) for k, v in r.items()}))
" || exit 1
done; done
