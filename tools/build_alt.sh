#!/bin/bash
# Build libaccunet_hip.so of git revision $1 into _ab/$2/ (A/B runs: ACCUNET_LIB_OVERRIDE)
set -e -o pipefail
cd "$(dirname "$0")/.."
REV=${1:-HEAD}; NAME=${2:-prev}
rm -rf _ab/${NAME}_src && mkdir -p _ab/${NAME}_src _ab/$NAME
git archive "$REV" acc-unet-unext_amd/csrc include | tar -x -C _ab/${NAME}_src
cd _ab/${NAME}_src/acc-unet-unext_amd/csrc
ls *.hip | xargs -P 8 -I{} sh -c '/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -I../../include -I. -c {} -o {}.o'
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared *.o -o ../../../$NAME/libaccunet_hip.so
cd ../../.. && rm -rf ${NAME}_src
ls -la $NAME
