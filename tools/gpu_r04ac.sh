# Round 4: A/B, interleaved: gpu_ticks on its own cache line (15) against the done line (143, experiment).
set -o pipefail
OUT=${OUT:-gpurun_out/r04ac}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 10 --sizes 4096 --variants "own_line:OCM_SERVICE_PROTO=15;done_line:OCM_SERVICE_PROTO=143" \
  --out $OUT/ticks_ab.json > $OUT/ticks_ab.log 2>&1
rc=$?; cut -c1-200 $OUT/ticks_ab.log; exit $rc
