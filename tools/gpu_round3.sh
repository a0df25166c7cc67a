#!/bin/bash
# Round-3 profile pass, part A: parity tests, the bench lines (fp32 headline + bf16),
# a rocprofv3 kernel trace (+ stats) of the bench, the FETCH_SIZE / WRITE_SIZE passes
# (separate runs) that give K1's and K3's HBM traffic, and tools/kbench.
# Part B (tools/pmc_gemm.sh + the GEMM census) runs as its own call.
# Every GPU step has its own time limit; the first failure ends the pass.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
  tail -1 gpurun_out/gputests.log
fi
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1
grep '^{"metric' gpurun_out/bench_full.log | cut -c1-200
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/bench_bf16.log 2>&1
grep '^{"metric' gpurun_out/bench_bf16.log | cut -c1-200
timeout -k 10 300 python bench.py --model unext > gpurun_out/bench_unext.log 2>&1
grep '^{"metric' gpurun_out/bench_unext.log | cut -c1-200
timeout -k 10 300 python bench.py --variant w --size 512 --batch 4 --no-cpu-baseline > gpurun_out/bench_w512.log 2>&1
grep '^{"metric' gpurun_out/bench_w512.log | cut -c1-200
rm -rf gpurun_out/prof_bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo "kernel trace done"
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
# keep only the probe dispatches (the last 60 dispatch ids cover K1, K3 and the GEMM probe)
python tools/save_profiles.py --shrink-pmc gpurun_out/pmc_fetch gpurun_out/pmc_write
echo "pmc done"
timeout -k 10 120 tools/kbench 20 > gpurun_out/kbench.txt 2>&1
echo "kbench done"
