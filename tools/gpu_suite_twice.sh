# The GPU suite twice in a row on one box: a flaky test shows before the driver's round-end run.
set -o pipefail
OUT=${OUT:-gpurun_out/twice}
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$i.log 2>&1 || { tail -30 $OUT/pytest_$i.log; exit 1; }
  tail -1 $OUT/pytest_$i.log
done
