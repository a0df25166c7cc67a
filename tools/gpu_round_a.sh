#!/bin/bash
# First half of the round profile pass (tools/gpu_round.sh split under one call's limit):
# the bench lines and the rocprofv3 kernel traces of the fp32 and bf16 bench
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1
grep '^{"metric' gpurun_out/bench_full.log | cut -c1-300
timeout -k 10 400 python bench.py --dp-path --no-cpu-baseline --no-parity > gpurun_out/bench_dp32.log 2>&1
grep '^{"metric' gpurun_out/bench_dp32.log | grep -o '"dp_path": {[^}]*}'
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline --dp-path > gpurun_out/bench_bf16.log 2>&1
grep '^{"metric' gpurun_out/bench_bf16.log | cut -c1-300
timeout -k 10 300 python bench.py --model unext > gpurun_out/bench_unext.log 2>&1
grep '^{"metric' gpurun_out/bench_unext.log | cut -c1-200
timeout -k 10 300 python bench.py --variant w --size 512 --batch 4 --no-cpu-baseline > gpurun_out/bench_w512.log 2>&1
grep '^{"metric' gpurun_out/bench_w512.log | cut -c1-200
for dt in fp32 bf16; do
  d=prof_bench; [ $dt = bf16 ] && d=prof_bench_bf16
  rm -rf gpurun_out/$d
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$d -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --dtype $dt > gpurun_out/$d.log 2>&1
  python tools/step_profile.py gpurun_out/$d --last 4 --top 45 > gpurun_out/step_$dt.txt
  head -n 3 gpurun_out/step_$dt.txt
done
echo "kernel traces done"
