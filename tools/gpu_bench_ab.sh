# bench.py A/B of copy-service protocols (interleaved, N=1).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for p in 7 1; do
    OCM_SERVICE_PROTO=$p timeout -k 10 200 python -u bench.py --no-optim-extra --json-out gpurun_out/bench_ab_p${p}_$i.json > gpurun_out/bench_ab_p${p}_$i.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json
for i in (1, 2):
    for p in (7, 1):
        b = json.load(open(f"gpurun_out/bench_ab_p{p}_{i}.json"))
        print(p, i, b["value"], b["alloc_p50_us"], " ".join(f"{int(s)//1024}K:{b['sweep'][s]['put_us']}/{b['sweep'][s]['get_us']}" for s in ["4096", "65536", "262144", "1048576", "4194304", "16777216"]))
PY
