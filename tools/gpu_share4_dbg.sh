# The 4-rank shared-GPU rehearsal at 64 MiB (tests/test_gpu_share.py's command), logged.
set -o pipefail
OUT=${OUT:-gpurun_out/share4dbg}
mkdir -p $OUT
timeout -k 10 240 env OCM_BENCH_SHARE_GPU=1 OCM_BENCH_TIMEOUT_S=180 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29681 bench.py --gpus 4 --steps 2 --warmup 1 --max-bytes 67108864 --alloc-samples 50 --no-ctrl-extra --no-hw-baseline --no-optim-extra --json-out $OUT/share4.json > $OUT/share4.log 2>&1
rc=$?; tail -c 3000 $OUT/share4.log; exit $rc
