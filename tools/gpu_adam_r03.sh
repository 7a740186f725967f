# Fused remote Adam with host-tier state: the optimizer GPU tests (host-tier
# kernel variant included), then the launch-shape probe.
set -o pipefail
OUT=gpurun_out/adam_r03
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_optim_offload.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 &&
timeout -k 10 600 python3 -u tools/adam_host_probe.py --configs ${CONFIGS:-generic,host_g64,host_g96,host_g128,host_g160,host_g192,host_g128_v2,host_g256_v2,host_g64_v8,host_g128_v8} --repeat 2 --out $OUT/adam_host_probe.json > $OUT/probe.log 2>&1
rc=$?; tail -16 $OUT/pytest.log; cat $OUT/probe.log; exit $rc
