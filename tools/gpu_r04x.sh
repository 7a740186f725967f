# Round 4: does the lead's poll wait behind the 15 other direct pollers' reads of the
# shared gang record? 4 KiB-1 MiB host-tier ops in fresh processes, 8 rounds: the
# default protocol, LEADREC (the lead reads its own copy), no GANGREC, one direct poller.
set -o pipefail
OUT=${OUT:-gpurun_out/r04x}
mkdir -p $OUT
export TMPDIR=/tmp
OCM_SERVICE_PROTO=143 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_service.py -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_service_leadrec.log 2>&1 &&
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 8 --sizes 4096,65536,262144,1048576 \
  --variants "p15:OCM_SERVICE_PROTO=15;leadrec:OCM_SERVICE_PROTO=143;p13:OCM_SERVICE_PROTO=13;direct1:OCM_SERVICE_DIRECT=1" \
  --out $OUT/leadrec_ab.json > $OUT/leadrec_ab.log 2>&1
rc=$?; tail -2 $OUT/pytest_service_leadrec.log; grep -E "FAILED|ERROR" $OUT/pytest_service_leadrec.log | head; cut -c1-330 $OUT/leadrec_ab.log; exit $rc
