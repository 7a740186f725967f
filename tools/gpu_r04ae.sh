# Round 4: the whole GPU suite once more at HEAD (stability of the late tests).
set -o pipefail
OUT=${OUT:-gpurun_out/r04ae}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head; exit $rc
