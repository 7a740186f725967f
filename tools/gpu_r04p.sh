# Round 4: the gang relaunch regression test, then host-tier mid sizes under tuning variants.
set -o pipefail
OUT=${OUT:-gpurun_out/r04p}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_service.py::test_back_to_back_gang_ops_never_relaunch" -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_relaunch.log 2>&1 &&
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 3 --out $OUT/host_mid_ab.json > $OUT/host_mid_ab.log 2>&1
rc=$?; grep -E "passed|failed|relaunches" $OUT/pytest_relaunch.log | tail -10; cat $OUT/host_mid_ab.log | cut -c1-400; exit $rc
