# the 8-GPU driver launch rehearsed on ONE GPU (8 ranks,
# every rank and daemon on GPU 0) at the driver's --max-bytes 1 GiB (2x1 GiB+1
# pairs: ~32 GiB of HBM in all), with autotune and the control-plane extra.
# The ranks start from a shell loop, not torchrun: its Python parent would be a
# 17th process with the GPU open (the box allows 16).
set -o pipefail
OUT=${OUT:-gpurun_out/share8}
mkdir -p $OUT
timeout -k 10 900 env OCM_BENCH_SHARE_GPU=1 RANKLOG_DIR=$OUT bash tools/launch_ranks.sh 8 ${PORT:-29551} bench.py --gpus 8 --steps 3 --warmup 1 --json-out $OUT/bench_share8.json > $OUT/share8.log 2>&1
rc=$?; tail -c 400 $OUT/share8.log; echo; grep -c "\[ocm W" $OUT/share8.log $OUT/rank*.log; exit $rc
