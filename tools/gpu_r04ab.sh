# Round 4: small-op modes with gpu_ticks moved off the `done` cache line (12 rounds),
# then the service tests.
set -o pipefail
OUT=${OUT:-gpurun_out/r04ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 12 --sizes 4096,65536 --variants "ticksline:" \
  --out $OUT/ticksline.json > $OUT/ticksline.log 2>&1 &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service.log 2>&1
rc=$?; cut -c1-200 $OUT/ticksline.log; tail -2 $OUT/pytest_service.log; exit $rc
