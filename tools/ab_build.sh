#!/bin/bash
# ab_build.sh NAME "-DFOO=1 ..." — build the extension sources with extra
# defines into datamining_recblr_amd/lib/ab_NAME.so, for A/B runs selected
# with RECBLR_LIB=datamining_recblr_amd/lib/ab_NAME.so (e.g. bench.py).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc -parallel-jobs=4 -O3 -std=c++20 -shared -fPIC --offload-arch=gfx950 \
  -ffp-contract=off -Wno-unused-function "$@" -I include \
  -o datamining_recblr_amd/lib/ab_$name.so datamining_recblr_amd/csrc/*.hip
