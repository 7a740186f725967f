# Longer GPU fuzz at new seeds: every config, one thread and four threads.
set -o pipefail
OUT=${OUT:-gpurun_out/fuzzlong}
mkdir -p $OUT
timeout -k 10 420 python3 -u tools/gpu_fuzz.py --seconds 45 --seed ${SEED1:-17} --configs hbm,stripe,host,copy,net --out $OUT/fuzz_t1.json > $OUT/fuzz_t1.log 2>&1 &&
timeout -k 10 420 python3 -u tools/gpu_fuzz.py --seconds 45 --seed ${SEED2:-23} --threads 4 --configs hbm,stripe,host,net --out $OUT/fuzz_t4.json > $OUT/fuzz_t4.log 2>&1
rc=$?; tail -3 $OUT/fuzz_t1.log; tail -3 $OUT/fuzz_t4.log; exit $rc
