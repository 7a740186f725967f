# Round 4: WGDONE words on a cache line each (WGDLINE, proto 15+128) against packed (15),
# interleaved in fresh processes, host tier and HBM; then the service tests with it on.
set -o pipefail
OUT=${OUT:-gpurun_out/r04ad}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 6 --sizes 4096,65536,131072,262144,524288,1048576,4194304 \
  --variants "packed:OCM_SERVICE_PROTO=15;line:OCM_SERVICE_PROTO=143" --out $OUT/wgdline_host.json > $OUT/wgdline_host.log 2>&1 &&
HOST_MID_TIER=hbm timeout -k 10 600 python3 -u tools/host_mid_ab.py --rounds 4 --sizes 65536,262144,1048576 \
  --variants "packed:OCM_SERVICE_PROTO=15;line:OCM_SERVICE_PROTO=143" --out $OUT/wgdline_hbm.json > $OUT/wgdline_hbm.log 2>&1 &&
OCM_SERVICE_PROTO=143 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service_wgdline.log 2>&1
rc=$?; cut -c1-400 $OUT/wgdline_host.log; cut -c1-300 $OUT/wgdline_hbm.log; tail -2 $OUT/pytest_service_wgdline.log; exit $rc
