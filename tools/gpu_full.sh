# Full GPU check: suite, smoke, N=1 bench, rocprofv3 kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_n1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-optim-extra > gpurun_out/rocprof_bench.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -c 400 gpurun_out/bench_n1.log; tail -3 gpurun_out/rocprof_bench.log; exit $rc
