set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py tests/test_examples.py -m gpu -x -v --timeout 120 --timeout-method thread -k "torch_ or remote_weights" > gpurun_out/pytest_step.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_step.log | head -20; exit $rc
