# Round 4: small-op modes against the size of the resident grid (OCM_SERVICE_BLOCKS).
set -o pipefail
OUT=${OUT:-gpurun_out/r04z}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/host_mid_ab.py --rounds 8 --sizes 4096 \
  --variants "b128:;b1:OCM_SERVICE_BLOCKS=1;b16:OCM_SERVICE_BLOCKS=16;b32:OCM_SERVICE_BLOCKS=32" \
  --out $OUT/blocks_ab.json > $OUT/blocks_ab.log 2>&1
rc=$?; cut -c1-200 $OUT/blocks_ab.log; exit $rc
