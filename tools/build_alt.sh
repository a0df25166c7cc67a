#!/bin/bash
# Build libaccunet_hip.so of git revision $1 into _ab/$2/ (A/B runs: ACCUNET_LIB_OVERRIDE,
# or LD_LIBRARY_PATH for the tools/ binaries). REV "WORKTREE" takes the working tree;
# EXTRA_FLAGS adds compile definitions (e.g. -DGEMM_PYR_EC=2).
set -e -o pipefail
cd "$(dirname "$0")/.."
REV=${1:-HEAD}; NAME=${2:-prev}
rm -rf _ab/${NAME}_src && mkdir -p _ab/${NAME}_src _ab/$NAME
if [ "$REV" = WORKTREE ]; then
  tar -c acc-unet-unext_amd/csrc include | tar -x -C _ab/${NAME}_src
else
  git archive "$REV" acc-unet-unext_amd/csrc include | tar -x -C _ab/${NAME}_src
fi
# ABI_HEADER=WORKTREE: stamp the working tree's header hash (a revision whose header
# differs only in comments still loads under the current binding)
if [ "${ABI_HEADER:-}" = WORKTREE ]; then cp include/accunet.h _ab/${NAME}_src/include/accunet.h; fi
ABI=0x$(sha256sum _ab/${NAME}_src/include/accunet.h | cut -c1-15)
cd _ab/${NAME}_src/acc-unet-unext_amd/csrc
ls *.hip | xargs -P 8 -I{} sh -c "/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result ${EXTRA_FLAGS:-} -DACCUNET_ABI_HASH=${ABI}LL -I../../include -I. -c {} -o {}.o"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared *.o -o ../../../$NAME/libaccunet_hip.so
cd ../../.. && rm -rf ${NAME}_src
ls -la $NAME
