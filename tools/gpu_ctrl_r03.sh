# RCCL tick latency: the rccl tick tests (every mode), then the control-plane
# probe (1 daemon, leases off, records to itself through the ticks) over the
# done-kernel / tagged-slot completion and seal-wait variants.
set -o pipefail
OUT=gpurun_out/ctrl_r03
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_ctrl_tick.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 &&
timeout -k 10 700 python3 -u tools/ctrl_probe.py --variants ${VARIANTS:-rccl_spec_ccd,rccl_tagged,rccl_wait6,rccl_tagged_wait3,rccl_tagged_wait6,rccl_tagged_wait10,rccl_tagged_wait6_d1,rccl_tagged_wait6_d3} --repeat ${REPEAT:-3} --out $OUT/ctrl_probe.json > $OUT/ctrl_probe.log 2>&1
rc=$?; tail -8 $OUT/pytest.log; tail -40 $OUT/ctrl_probe.log; exit $rc
