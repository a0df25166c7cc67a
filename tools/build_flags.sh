#!/bin/bash
# Build libaccunet_hip.so of the WORKING TREE with extra compiler flags into _ab/$1/
# (A/B runs of compile-time knobs: ACCUNET_LIB_OVERRIDE=_ab/$1/libaccunet_hip.so for
# python, LD_LIBRARY_PATH=_ab/$1 for tools/gbench and tools/kbench, whose RUNPATH
# yields to it). Usage: tools/build_flags.sh NAME -DKNOB=VALUE ...
set -e -o pipefail
cd "$(dirname "$0")/.."
NAME=$1; shift
rm -rf _ab/${NAME}_src && mkdir -p _ab/${NAME}_src/acc-unet-unext_amd _ab/$NAME
cp -r acc-unet-unext_amd/csrc _ab/${NAME}_src/acc-unet-unext_amd/csrc
cp -r include _ab/${NAME}_src/include
ABI=0x$(sha256sum include/accunet.h | cut -c1-15)
cd _ab/${NAME}_src/acc-unet-unext_amd/csrc
rm -f *.hipfb
ls *.hip | xargs -P 8 -I{} /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -DACCUNET_ABI_HASH=${ABI}LL -I../../include -I. -c {} -o {}.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared *.o -o ../../../$NAME/libaccunet_hip.so
cd ../../.. && rm -rf ${NAME}_src
ls -la $NAME
