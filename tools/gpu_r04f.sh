# Round 4: the copy service on the library's own AQL queue with a lone lead.
# AQL probe, the service suite, the idle-gap probe (AQL vs HIP lanes), smoke, N=1 bench.
set -o pipefail
OUT=${OUT:-gpurun_out/r04f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 build/bin/hsa_dispatch_probe build/bin/hsa_dispatch_probe.co > $OUT/hsa_probe.json 2> $OUT/hsa_probe.err &&
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service.log 2>&1 &&
timeout -k 10 300 env OCM_IDLE_GAP_QUEUES=1 python3 -u tools/idle_gap_probe.py --variants default,hip --repeat 1 --out $OUT/idle_gap.json > $OUT/idle_gap.log 2>&1 &&
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1.json > $OUT/bench_n1.log 2>&1
rc=$?; cat $OUT/hsa_probe.json; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest_service.log | tail -40; cat $OUT/idle_gap.log | cut -c1-400; tail -2 $OUT/smoke.log; tail -c 600 $OUT/bench_n1.log; exit $rc
