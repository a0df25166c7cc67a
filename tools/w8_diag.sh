#!/bin/bash
# world-8 gloo rehearsal: the world-4 / world-8 tests, then eager bf16 diagnostics
# ((1) one backward stream, (2) default) -- rc 1 there is the worker's own assertion
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_dist_gpu.py -x -v -s -m gpu -k "world8 or world4_buckets" --timeout 600 --timeout-method thread > gpurun_out/w8.log 2>&1
rc=$?
grep -E "fp64 mean|PASSED|FAILED|passed|failed" gpurun_out/w8.log | sort | uniq | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
export ACCUNET_DIST_BACKEND=gloo OMP_NUM_THREADS=2
run() {  # $1: tag, rest: env assignments
  tag=$1; shift
  env "$@" timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) tests/dist_worker.py > gpurun_out/w8_$tag.log 2>&1
  rc=$?
  echo "== $tag rc=$rc"
  grep -E "eager_bf16: losses" gpurun_out/w8_$tag.log | sort | head -10
  return $rc
}
run e16_1stream DIST_MODES=eager_bf16 ACCUNET_WGRAD_STREAM=0
rc2=$?
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit 1
run e16_default DIST_MODES=eager_bf16
exit 0
