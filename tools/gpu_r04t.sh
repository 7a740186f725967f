# Round 4: one gang record per direct poller (OCM_SERVICE_PROTO bit COPIES): the
# service tests with it on, then A/B against the round-3 protocol on both tiers.
set -o pipefail
OUT=${OUT:-gpurun_out/r04t}
mkdir -p $OUT
export TMPDIR=/tmp
OCM_SERVICE_PROTO=79 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service_copies.log 2>&1 &&
timeout -k 10 600 python3 -u tools/host_mid_ab.py --rounds 3 --sizes 4096,16384,65536,131072,262144,524288,1048576,4194304 \
  --variants "p15:OCM_SERVICE_PROTO=15;p79:OCM_SERVICE_PROTO=79" --out $OUT/copies_ab_host.json > $OUT/copies_ab_host.log 2>&1 &&
HOST_MID_TIER=hbm timeout -k 10 600 python3 -u tools/host_mid_ab.py --rounds 3 --sizes 4096,65536,262144,524288,1048576 \
  --variants "p15:OCM_SERVICE_PROTO=15;p79:OCM_SERVICE_PROTO=79" --out $OUT/copies_ab_hbm.json > $OUT/copies_ab_hbm.log 2>&1
rc=$?; tail -2 $OUT/pytest_service_copies.log; grep -E "FAILED|ERROR" $OUT/pytest_service_copies.log | head; cut -c1-700 $OUT/copies_ab_host.log; cut -c1-500 $OUT/copies_ab_hbm.log; exit $rc
