#!/bin/bash
# rocprofv3 kernel trace (+ stats) of a short bench run per activation dtype, then the
# per-step breakdown (tools/step_profile.py) and per-kernel totals (tools/kstats.py).
#   DTYPES="fp32 bf16" bash tools/gpu_prof.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for dt in ${DTYPES:-fp32 bf16}; do
  rm -rf gpurun_out/prof_$dt
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$dt -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype $dt > gpurun_out/prof_$dt.log 2>&1
  grep '^{"metric' gpurun_out/prof_$dt.log | cut -c1-160
  python tools/step_profile.py gpurun_out/prof_$dt --last 4 --top 45 > gpurun_out/step_$dt.txt
  python tools/kstats.py gpurun_out/prof_$dt --top 60 > gpurun_out/kstats_$dt.txt
  head -3 gpurun_out/step_$dt.txt
done
