#!/bin/bash
# rocprofv3 kernel trace of a short fp32 bench per library variant (single stream, so
# per-kernel durations are not inflated by the side stream), then per-family step tables.
#   VARIANTS="name:libdir ..." (libdir "-" = in-tree)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export ACCUNET_WGRAD_STREAM=${ACCUNET_WGRAD_STREAM:-0}
for v in $VARIANTS; do
  IFS=: read -r name lib envs <<< "$v"
  if [ "$lib" = "-" ]; then unset ACCUNET_LIB_OVERRIDE; else export ACCUNET_LIB_OVERRIDE=$PWD/$lib/libaccunet_hip.so; fi
  rm -rf gpurun_out/pa_$name
  timeout -k 10 300 env ${envs//,/ } rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pa_$name -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe --dtype ${DT:-fp32} ${BENCH_ARGS:-} > gpurun_out/pa_$name.log 2>&1
  python tools/step_profile.py gpurun_out/pa_$name --last 4 --top ${TOP:-60} > gpurun_out/step_$name.txt
  python tools/kstats.py gpurun_out/pa_$name --steps 7 --top 80 > gpurun_out/kstats_$name.txt
  python tools/splitk_census.py gpurun_out/pa_$name --steps 7 > gpurun_out/splitk_$name.txt
  for fam in ${KGRID:-}; do python tools/kgrid.py gpurun_out/pa_$name $fam > gpurun_out/kgrid_${name}_$fam.txt; done
  if [ -n "${SEQ:-}" ]; then python tools/step_seq.py gpurun_out/pa_$name $SEQ > gpurun_out/seq_$name.txt; fi
  rm -rf gpurun_out/pa_$name
  echo "== $name"; head -24 gpurun_out/step_$name.txt
done
