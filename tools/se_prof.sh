#!/bin/bash
# kernel-trace stats of a short bench run (SE kernels), fused and unfused middle step
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 1 0; do
  rm -rf gpurun_out/se_prof_$f
  ACCUNET_SE_FUSED=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/se_prof_$f -o run -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/se_prof_$f.log 2>&1
  find gpurun_out/se_prof_$f -name '*kernel_stats.csv' -exec cp {} gpurun_out/se_stats_$f.csv \;
  find gpurun_out/se_prof_$f -name '*kernel_trace.csv' -exec cp {} gpurun_out/se_trace_$f.csv \;
  rm -rf gpurun_out/se_prof_$f
  echo "== fused=$f"; grep -i '"se_\|se_' gpurun_out/se_stats_$f.csv | cut -d, -f1-5 | cut -c1-160
done
