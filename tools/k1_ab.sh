#!/bin/bash
# A/B of K1 builds in one box session: current tree vs the library in $1 (default _exp/head)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ALT=${1:-_exp/head}
for i in 1 2; do
  timeout -k 5 120 tools/kbench 40 > gpurun_out/kb_cur$i.txt 2>&1
  LD_LIBRARY_PATH=$PWD/$ALT timeout -k 5 120 tools/kbench 40 > gpurun_out/kb_alt$i.txt 2>&1
done
for f in cur1 alt1 cur2 alt2; do echo "== $f"; grep -E "K1|flat|x4/thread nt|K3|bn_bwd" gpurun_out/kb_$f.txt; done
