# Quiesce before device-wide syncs: service tests, loopback bench (HBM ops leave the service resident), N=1 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py tests/test_optim_offload.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_quiesce.log 2>&1 && \
timeout -k 10 200 python -u bench.py --remote loopback --no-optim-extra --json-out gpurun_out/bench_loop_quiesce.json > gpurun_out/bench_loop_quiesce.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_n1.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_quiesce.log; exit $rc
