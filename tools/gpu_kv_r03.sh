# Host-tier batch launches (KV-cache swaps to a pinned host pool): the batch
# and KV GPU tests, then the swap probe over launch shapes (grid cap and
# write-through puts), each in its own process.
set -o pipefail
OUT=gpurun_out/kv_r03
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_batch.py tests/test_kv_offload.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2; do
  for cfg in "0 0" "1 0" "1 128" "1 256" "1 512" "0 256"; do
    set -- $cfg
    timeout -k 10 200 env OCM_BATCH_HOST_SC1=$1 OCM_BATCH_HOST_GRID=$2 python3 -u tools/kv_swap_probe.py --host-only --out $OUT/sc1_$1_g$2_$r.json > $OUT/sc1_$1_g$2_$r.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/kv_r03/sc1_*.json')):
    rows = json.load(open(f))
    print(f.split('/')[-1], [(r['blocks'], r['swap_out_GiBps'], r['swap_in_GiBps']) for r in rows])
PY
