# N=4 rehearsal on one GPU (every rank and daemon on GPU 0) with every extra, after the hardware-queue fix.
set -o pipefail
mkdir -p gpurun_out
OCM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 --max-bytes 268435456 --json-out gpurun_out/bench_share4.json > gpurun_out/bench_share4.log 2>&1
rc=$?; tail -c 600 gpurun_out/bench_share4.log; exit $rc
