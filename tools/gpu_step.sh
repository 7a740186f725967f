# One GPU call: targeted tests, then probes; each step bounded, chained with &&.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ctrl_tick.py tests/test_gpu_multi.py tests/test_net_tier.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 && \
timeout -k 10 240 python -u tools/ctrl_probe.py --out gpurun_out/ctrl_probe.json > gpurun_out/ctrl_probe.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -v --timeout 200 --timeout-method thread -k "bench" > gpurun_out/pytest_bench.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_step.log; tail -c 1500 gpurun_out/ctrl_probe.log; tail -3 gpurun_out/pytest_bench.log; exit $rc
