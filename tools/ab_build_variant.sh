#!/bin/bash
# ab_build_variant.sh NAME FILE=SOURCE ... — build the product sources into
# datamining_recblr_amd/lib/ab_NAME.so with some csrc files replaced (e.g.
# conv_silu.hip=/tmp/conv_old.hip), for A/B runs selected with RECBLR_LIB.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
tmp=$(mktemp -d)
mkdir -p "$tmp/pkg/csrc" "$tmp/include"
cp include/* "$tmp/include/"
cp datamining_recblr_amd/csrc/* "$tmp/pkg/csrc/"
for kv in "$@"; do cp "${kv#*=}" "$tmp/pkg/csrc/${kv%%=*}"; done
/opt/rocm/bin/hipcc -parallel-jobs=8 -O3 -std=c++20 -shared -fPIC --offload-arch=gfx950 \
  -ffp-contract=off -Wno-unused-function -I "$tmp/include" \
  -o datamining_recblr_amd/lib/ab_$name.so "$tmp"/pkg/csrc/*.hip
rm -rf "$tmp"
