#!/bin/bash
# world-8 eager-bf16 sequence diagnostics: does a preceding graph-mode bf16 run (same
# process) leave state that the eager hook reducer in bf16 trips over?
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
export ACCUNET_DIST_BACKEND=gloo OMP_NUM_THREADS=2
run() {  # $1: tag, rest: env assignments
  tag=$1; shift
  env "$@" timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) tests/dist_worker.py > gpurun_out/w8s_$tag.log 2>&1
  rc=$?
  echo "== $tag rc=$rc"
  grep -E "eager_bf16: losses" gpurun_out/w8s_$tag.log | sort | head -8
  return $rc
}
run gb_eb DIST_MODES=graph_bf16,eager_bf16
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run all5_1stream DIST_MODES=graph,eager,trainer,graph_bf16,eager_bf16 ACCUNET_WGRAD_STREAM=0
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run all5 DIST_MODES=graph,eager,trainer,graph_bf16,eager_bf16
exit 0
