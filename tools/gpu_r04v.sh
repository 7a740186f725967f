# Round 4: host <-> resident kernel ping-pong per CPU, doorbell kind and spin style.
set -o pipefail
OUT=${OUT:-gpurun_out/r04v}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/pingpong_sweep.py --rounds 2 --out $OUT/pingpong.json > $OUT/pingpong.log 2>&1
rc=$?; cut -c1-200 $OUT/pingpong.log; exit $rc
