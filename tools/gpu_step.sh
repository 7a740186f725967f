# One GPU call: targeted tests, then probes; each step bounded, chained with &&.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_runtime.py tests/test_optim_offload.py tests/test_gpu_multi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 && \
timeout -k 10 240 python -u tools/ctrl_probe.py --out gpurun_out/ctrl_probe.json > gpurun_out/ctrl_probe.log 2>&1 && \
timeout -k 10 300 python -u tools/svc_park_probe.py --out gpurun_out/svc_park.json > gpurun_out/svc_park.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_step.log; tail -c 1500 gpurun_out/ctrl_probe.log; tail -c 1500 gpurun_out/svc_park.log; exit $rc
