# Round 4, final check at the end-of-round code: the whole GPU suite, smoke, the
# driver's N=1 bench twice, the N=1 bench under rocprofv3, the 4-thread fuzz.
set -o pipefail
OUT=${OUT:-gpurun_out/final4}
mkdir -p $OUT $OUT/prof
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1_a.json > $OUT/bench_n1_a.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1_b.json > $OUT/bench_n1_b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 -u bench.py --steps 5 --warmup 2 --json-out $OUT/prof/bench.json > $OUT/prof/bench.log 2>&1 &&
timeout -k 10 300 python3 -u tools/gpu_fuzz.py --seconds 45 --seed 53 --threads 4 --configs hbm,stripe,host,net --out $OUT/fuzz_t4.json > $OUT/fuzz_t4.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head; tail -1 $OUT/smoke.log; tail -c 200 $OUT/bench_n1_a.log; echo; tail -c 200 $OUT/bench_n1_b.log; echo; tail -1 $OUT/fuzz_t4.log | cut -c1-200; grep -c "copy service failed" $OUT/fuzz_t4.log; exit $rc
