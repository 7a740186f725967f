# Round 4: the whole GPU suite at the AQL-service code, the 4-thread fuzz, then
# the 8-GPU driver launch rehearsed on ONE GPU at 1 GiB.
set -o pipefail
OUT=${OUT:-gpurun_out/r04g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -u tools/gpu_fuzz.py --seconds 45 --seed 43 --threads 4 --configs hbm,stripe,host,net --out $OUT/fuzz_t4.json > $OUT/fuzz_t4.log 2>&1 &&
OUT=$OUT/share8 timeout -k 10 900 bash tools/gpu_share8.sh > $OUT/share8_wrapper.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head; tail -2 $OUT/fuzz_t4.log | cut -c1-300; grep -c "copy service failed" $OUT/*.log $OUT/share8/*.log; tail -c 600 $OUT/share8_wrapper.log; exit $rc
