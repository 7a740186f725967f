# Round 4: AQL vs HIP copy-service lanes, interleaved (hot path per size, gang op after
# 1 ms idle), the service suite, then the 8-rank 1 GiB rehearsal.
set -o pipefail
OUT=${OUT:-gpurun_out/r04h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/svc_queue_ab.py --repeat 3 --out $OUT/svc_queue_ab.json > $OUT/svc_queue_ab.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service.log 2>&1 &&
ps -eo pid,ppid,comm > $OUT/ps_before_share8.txt &&
OUT=$OUT/share8 timeout -k 10 900 bash tools/gpu_share8.sh > $OUT/share8_wrapper.log 2>&1
rc=$?; cut -c1-600 $OUT/svc_queue_ab.log; tail -2 $OUT/pytest_service.log; tail -c 800 $OUT/share8_wrapper.log; exit $rc
