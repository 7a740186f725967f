# Round 4: the ping-pong with a 4 KiB copy per answer (get: host -> HBM, put: HBM -> host),
# on 16 CPUs, 3 rounds, 20000 round trips per process (~0.1-0.2 s, long enough to see a
# mode that lasts that long).
set -o pipefail
OUT=${OUT:-gpurun_out/r04aa}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/pingpong_sweep.py --data --rounds 3 --n 20000 --cpus 0,1,2,3,4,5,6,7,64,65,66,67,128,129,192,193 --out $OUT/pingpong_data.json > $OUT/pingpong_data.log 2>&1
rc=$?; cut -c1-200 $OUT/pingpong_data.log | tail -60; exit $rc
