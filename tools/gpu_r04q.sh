# Round 4: host-tier gang width for 512 KiB - 4 MiB ops, and put tiles for 64-256 KiB.
set -o pipefail
OUT=${OUT:-gpurun_out/r04q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 3 --sizes 524288,1048576,2097152,4194304 \
  --variants "default:;direct4:OCM_SERVICE_DIRECT=4;direct8:OCM_SERVICE_DIRECT=8;direct12:OCM_SERVICE_DIRECT=12" \
  --out $OUT/host_wide_ab.json > $OUT/host_wide_ab.log 2>&1 &&
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 3 --sizes 16384,32768,65536,131072,262144 \
  --variants "default:;put_tile14:OCM_SERVICE_HOST_TILE_SHIFT_PUT=14;put_tile13:OCM_SERVICE_HOST_TILE_SHIFT_PUT=13;put_tile14_min32k:OCM_SERVICE_HOST_TILE_SHIFT_PUT=14,OCM_SERVICE_HOST_TILE_MIN=32768" \
  --out $OUT/host_put_ab.json > $OUT/host_put_ab.log 2>&1
rc=$?; cut -c1-400 $OUT/host_wide_ab.log; cut -c1-400 $OUT/host_put_ab.log; exit $rc
