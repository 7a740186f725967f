# RCCL tick latency after the one-round-trip seal: the rccl tick test, then the
# control-plane probe (1 daemon, leases off, records to itself through the ticks).
set -o pipefail
OUT=gpurun_out/ctrl_r03
mkdir -p $OUT
timeout -k 10 200 python3 -u -m pytest tests/test_ctrl_tick.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ctrl_probe.py --variants rccl_spec_ccd,rccl_spec_ccd_spin300 --repeat 4 --out $OUT/ctrl_probe.json > $OUT/ctrl_probe.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; tail -40 $OUT/ctrl_probe.log; exit $rc
