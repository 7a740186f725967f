# Round 4: the 2 ms lone window; the service suite, the idle-gap probe, smoke, the N=1 bench.
set -o pipefail
OUT=${OUT:-gpurun_out/r04l}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service.log 2>&1 &&
timeout -k 10 300 python3 -u tools/idle_gap_probe.py --variants default --repeat 2 --out $OUT/idle_gap.json > $OUT/idle_gap.log 2>&1 &&
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1.json > $OUT/bench_n1.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $OUT/pytest_service.log | tail -5; cut -c1-300 $OUT/idle_gap.log; tail -1 $OUT/smoke.log; tail -c 700 $OUT/bench_n1.log; exit $rc
