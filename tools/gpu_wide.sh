# 128-wide service gang: service tests, probe vs the 32-wide configuration, loopback bench A/B (large HBM copies with the service resident).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_runtime.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1 && \
timeout -k 10 600 python -u tools/svc_probe.py --tiers hbm,host --configs default,prev32 --repeat 2 --out gpurun_out/svc_wide.json > gpurun_out/svc_wide.log 2>&1 && \
timeout -k 10 200 python -u bench.py --remote loopback --no-optim-extra --json-out gpurun_out/bench_loop_wide.json > gpurun_out/bench_loop_wide.log 2>&1 && \
OCM_SERVICE_BLOCKS=32 OCM_SERVICE_MAX_LOCAL=4194304 timeout -k 10 200 python -u bench.py --remote loopback --no-optim-extra --json-out gpurun_out/bench_loop_prev32.json > gpurun_out/bench_loop_prev32.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_wide.log; exit $rc
