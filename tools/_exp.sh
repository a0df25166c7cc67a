set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 300 python tools/gemm_exp.py > gpurun_out/exp.txt 2>&1
timeout -k 10 300 python tools/gemm_census.py --top 200 > gpurun_out/census.txt 2>&1
head -2 gpurun_out/census.txt | tail -1
timeout -k 10 400 python bench.py --no-cpu-baseline --no-probe > gpurun_out/bench_iter.log 2>&1
grep '^{"metric' gpurun_out/bench_iter.log | cut -c1-200
