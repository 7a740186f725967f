# Copy-service protocol change: full GPU suite on the new default, then the
# service probe (new default vs the round-2 relay protocol), then the N=1 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python -u tools/svc_probe.py --tiers host,hbm --configs default,relay,wcreq --repeat 2 --out gpurun_out/svc_hybrid.json > gpurun_out/svc_hybrid.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_n1.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; tail -c 300 gpurun_out/bench_n1.log; exit $rc
