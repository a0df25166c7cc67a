#!/bin/bash
# GEMM raster / epilogue cache-policy lab on the wide-B shapes (cnv72 conv1 forward,
# x-branch data gradient, pyramid data gradient: 65536 x 4352 x 128): tools/gbench per
# library variant in $VARS (cur = the tree's, else _ab/NAME from tools/build_flags.sh)
# x raster group size $KBS (ACCUNET_GEMM_NGRP_KB), then FETCH_SIZE / WRITE_SIZE passes
# (separate runs) of the pyramid shape for the variants in $PMC ("var:kb" pairs).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/glab
for v in ${VARS:-cur}; do
  LP=""; [ "$v" != cur ] && LP="$PWD/_ab/$v"
  for g in ${KBS:-0}; do
    echo "== $v ngrp_kb=$g"
    LD_LIBRARY_PATH=$LP ACCUNET_GEMM_NGRP_KB=$g GB_ONLY=${GB_ONLY:-65536x4352} timeout -k 10 120 tools/gbench 20
  done
done
for vk in ${PMC:-}; do
  v=${vk%%:*}; g=${vk##*:}
  LP=""; [ "$v" != cur ] && LP="$PWD/_ab/$v"
  for c in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/glab/pmc_${v}_${g}_$c
    rm -rf $d
    LD_LIBRARY_PATH=$LP ACCUNET_GEMM_NGRP_KB=$g GB_ONLY="pyr dgrad" timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $d -o run -- tools/gbench 5 > $d.log 2>&1
    python - "$d" "$v:$g $c" <<'PY'
import csv, glob, sys, statistics
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    if "gemm" in r["Kernel_Name"]:
        per.setdefault(int(r["Dispatch_Id"]), 0.0)
        per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
v = sorted(per.values())
print(sys.argv[2], "dispatches", len(v), "median KiB", statistics.median(v), "-> MB", statistics.median(v) * 1024 / 1e6)
PY
  done
done
