#!/bin/bash
# Build kernel variants for an on-box A/B (scripts/variant_ab.sh): one
# turbo_decoder_cuda_amd/libvar_<name>.so per "name:flags" word of VARIANTS, e.g.
#   VARIANTS="a_base: b_diag:-DTD_DIAG=1" scripts/build_variants.sh
# Flags are comma-separated (-DX=1,-DY=2).  Old libvar_*.so are removed first.
set -e
cd "$(dirname "$0")/.."
PKG=turbo_decoder_cuda_amd
rm -rf $PKG/libvar_*.so $PKG/libvar_*.so.objs
for v in $VARIANTS; do
  name=${v%%:*}
  flags=${v#*:}
  python -c "import sys; from turbo_decoder_cuda_amd import build; build.build_lib(sys.argv[1], sys.argv[2:])" \
    $PKG/libvar_$name.so ${flags//,/ } > /dev/null &
done
wait
ls -la $PKG/libvar_*.so
