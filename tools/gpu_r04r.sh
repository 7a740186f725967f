# Round 4: the new host-tier defaults (16 KiB put tiles for 64-256 KiB, 12-member gets
# from 1 MiB) against the old ones, gets of 8-16 MiB at other widths; then the service
# tests and the driver's N=1 bench.
set -o pipefail
OUT=${OUT:-gpurun_out/r04r}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 3 --sizes 65536,131072,262144,1048576,4194304,8388608,16777216 \
  --variants "new:;old:OCM_SERVICE_HOST_TILE_SHIFT_PUT=0,OCM_SERVICE_HOST_GET_WIDTH=1024;w8:OCM_SERVICE_HOST_GET_WIDTH=8;w16:OCM_SERVICE_HOST_GET_WIDTH=16;w24:OCM_SERVICE_HOST_GET_WIDTH=24" \
  --out $OUT/host_defaults_ab.json > $OUT/host_defaults_ab.log 2>&1 &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_n1_a.json > $OUT/bench_n1_a.log 2>&1
rc=$?; cut -c1-600 $OUT/host_defaults_ab.log; tail -2 $OUT/pytest_service.log; grep -E "FAILED|ERROR" $OUT/pytest_service.log | head; tail -c 200 $OUT/bench_n1_a.log; echo; exit $rc
