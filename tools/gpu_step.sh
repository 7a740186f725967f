set -o pipefail
mkdir -p gpurun_out
export OCM_BENCH_SHARE_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29701 bench.py --gpus 4 --steps 2 --warmup 1 --max-bytes 268435456 > gpurun_out/bench_share4.log 2>&1 && \
unset OCM_BENCH_SHARE_GPU && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_soak.log 2>&1
rc=$?; grep '^{' gpurun_out/bench_share4.log | tail -1 | cut -c1-600; tail -2 gpurun_out/pytest_gpu_soak.log; exit $rc
