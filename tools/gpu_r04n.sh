# Round 4, validation at the current code: the whole GPU suite, the 4-thread fuzz,
# smoke and the N=1 bench (the 8-rank rehearsal runs in a call of its own: 16 GPU processes).
set -o pipefail
OUT=${OUT:-gpurun_out/r04n}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -u tools/gpu_fuzz.py --seconds 45 --seed 47 --threads 4 --configs hbm,stripe,host,net --out $OUT/fuzz_t4.json > $OUT/fuzz_t4.log 2>&1 &&
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1.json > $OUT/bench_n1.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head; tail -1 $OUT/fuzz_t4.log | cut -c1-300; grep -c "copy service failed" $OUT/fuzz_t4.log; tail -1 $OUT/smoke.log; tail -c 400 $OUT/bench_n1.log; exit $rc
