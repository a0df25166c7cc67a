#!/bin/bash
# Round profile pass (the final-source pass of a round): parity tests, the bench lines (fp32 headline, bf16, UNeXt,
# ACC_UNet_W at 512^2), a rocprofv3 kernel trace (+ stats) of the fp32 bench and of the
# bf16 bench, the FETCH_SIZE / WRITE_SIZE passes (separate runs) that give K1's and K3's
# HBM traffic, and tools/kbench. Every GPU step has its own time limit; the first
# failure ends the pass. SKIP_TESTS=1 skips the suite.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
  tail -n 1 gpurun_out/gputests.log
fi
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
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
# keep only the probe dispatches (the last 300 dispatch ids cover K1, K3 and the GEMM probe)
python tools/save_profiles.py --shrink-pmc gpurun_out/pmc_fetch gpurun_out/pmc_write
echo "pmc done"
timeout -k 10 120 tools/kbench 20 > gpurun_out/kbench.txt 2>&1
echo "kbench done"
# K1 instruction-level PMC beside the lab structures, and a single-stream trace of the
# step (split-K reduce census, depthwise per-grid table: no cross-stream stretch)
timeout -k 10 600 bash tools/pmc_k1.sh > gpurun_out/pmc_k1.log 2>&1
KGRID="splitk dw3x3" VARIANTS="ss:-" timeout -k 10 600 bash tools/prof_ab.sh > gpurun_out/prof_ss.log 2>&1
echo "pmc_k1 / single-stream trace done"
if [ -n "${DPTRACE:-}" ]; then
  # the data-parallel step (world-1 RCCL group) beside the plain step, bf16, two streams:
  # one step's dispatch sequence each (tools/step_seq.py)
  DT=bf16 ACCUNET_WGRAD_STREAM=1 SEQ="--step -2" VARIANTS="b16plain:-" timeout -k 10 300 bash tools/prof_ab.sh > gpurun_out/prof_dp.log 2>&1
  DT=bf16 ACCUNET_WGRAD_STREAM=1 BENCH_ARGS=--dp-world1 SEQ="--step -2" VARIANTS="b16dp:-" timeout -k 10 300 bash tools/prof_ab.sh >> gpurun_out/prof_dp.log 2>&1
  timeout -k 10 200 python tools/dp_host.py --dtype bf16 > gpurun_out/dp_host_bf16.txt 2>&1
  timeout -k 10 200 python tools/dp_host.py --dtype fp32 > gpurun_out/dp_host_fp32.txt 2>&1
  echo "dp traces done"
fi
if [ -n "${PMC_GEMM:-}" ]; then
  # GEMM census of one step and the PMC passes of the ResPath 3x3 (halo kernels) and the
  # pyramid data gradient at the final sources
  timeout -k 10 300 python tools/gemm_census.py --top 200 > gpurun_out/census_full.txt 2>&1
  head -n 3 gpurun_out/census_full.txt
  KEYS="32,288,1048576,1,2 1048576,32,288,2,0 64,576,262144,1,2 65536,4352,128,0,1" timeout -k 10 900 bash tools/pmc_gemm.sh > gpurun_out/pmc_gemm.log 2>&1
  cat gpurun_out/pmc_gemm/report.txt
fi
