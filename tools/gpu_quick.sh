# Quick GPU pass: parity tests, microbench, bench line (no CPU baseline).
set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 60 tools/kbench 20 > gpurun_out/kbench.txt 2>&1
grep K3 gpurun_out/kbench.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_iter.log 2>&1
grep '^{"metric' gpurun_out/bench_iter.log | cut -c1-200
