# Graph-batched RCCL ticks (OCM_TICK_GRAPH=K): the rccl tick GPU tests (every
# mode, graphs included), then the control-plane probe (1 daemon, leases off,
# records to itself) over K = 0 / 4 / 8 / 16 and the seal wait, interleaved.
set -o pipefail
OUT=${OUT:-gpurun_out/tickgraph}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_ctrl_tick.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 &&
timeout -k 10 600 python3 -u tools/ctrl_probe.py --variants ${VARIANTS:-rccl_nograph,rccl_graph4,rccl_graph8,rccl_graph16,rccl_graph8_nowait,rccl_graph8_w3} --repeat ${REPEAT:-2} --out $OUT/ctrl_probe.json > $OUT/ctrl_probe.log 2>&1
rc=$?; tail -14 $OUT/pytest.log; python3 -c "
import json,sys
d=json.load(open('$OUT/ctrl_probe.json'))
for k,v in d.items(): print(k, v['alloc_p50_us'], v['alloc_p99_us'], v['free_p50_us'], (v.get('tick_stats') or [''])[0][:200])
" || tail -30 $OUT/ctrl_probe.log; exit $rc
