set -e -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 120 tools/kbench 20 > gpurun_out/kb_u4_$r.txt 2>&1
  ACCUNET_BN_APPLY_U=8 timeout -k 10 120 tools/kbench 20 > gpurun_out/kb_u8_$r.txt 2>&1
  grep "bn_bwd" gpurun_out/kb_u4_$r.txt | sed 's/^/u4 /'
  grep "bn_bwd" gpurun_out/kb_u8_$r.txt | sed 's/^/u8 /'
done
REPS="1 2" BENCH_ARGS="--no-parity" VARIANTS="u4:-: u8:-:ACCUNET_BN_APPLY_U=8" bash tools/gpu_ab.sh
DT=bf16 REPS="1 2" BENCH_ARGS="--no-parity" VARIANTS="b4:-: b8:-:ACCUNET_BN_APPLY_U=8" bash tools/gpu_ab.sh
