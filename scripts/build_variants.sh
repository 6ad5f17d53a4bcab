#!/bin/bash
# Build kernel variants for an on-box A/B (scripts/variant_ab.sh): one
# turbo_decoder_cuda_amd/libvar_<name>.so per "name:flags" word of VARIANTS, e.g.
#   VARIANTS="a_base: b_diag:-DTD_DIAG=1" scripts/build_variants.sh
# Flags are comma-separated (-DX=1,-DY=2).  Old libvar_*.so are removed first.
set -e
cd "$(dirname "$0")/.."
PKG=turbo_decoder_cuda_amd
rm -f $PKG/libvar_*.so
for v in $VARIANTS; do
  name=${v%%:*}
  flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-honor-nans \
    -Iinclude -I$PKG/csrc ${flags//,/ } -shared -o $PKG/libvar_$name.so \
    $PKG/csrc/td_kernels.hip $PKG/csrc/td_kernels_w12.hip $PKG/csrc/td_synth.hip $PKG/csrc/td_api.cpp &
done
wait
ls -la $PKG/libvar_*.so
