set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_n1.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -c 600 gpurun_out/bench_n1.log; exit $rc
