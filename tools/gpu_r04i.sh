# Round 4: same-lane promotions on the AQL queue: the service suite twice, the queue A/B.
set -o pipefail
OUT=${OUT:-gpurun_out/r04i}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service1.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service2.log 2>&1 &&
timeout -k 10 400 python3 -u tools/svc_queue_ab.py --repeat 2 --out $OUT/svc_queue_ab.json > $OUT/svc_queue_ab.log 2>&1
rc=$?; grep -h -E "most_cus|passed|failed" $OUT/pytest_service*.log | cut -c1-900; cut -c1-700 $OUT/svc_queue_ab.log; exit $rc
