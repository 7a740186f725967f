# Round 4: a gang op's extra idle window after its completion. The service tests,
# then the driver's N=1 bench twice (8-16 MiB rows: relaunches and p99).
set -o pipefail
OUT=${OUT:-gpurun_out/r04o}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1_a.json > $OUT/bench_n1_a.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1_b.json > $OUT/bench_n1_b.log 2>&1
rc=$?; tail -2 $OUT/pytest_service.log; grep -E "FAILED|ERROR" $OUT/pytest_service.log | head; tail -c 200 $OUT/bench_n1_a.log; echo; tail -c 200 $OUT/bench_n1_b.log; echo; exit $rc
