# One GPU call: tick variants with repeats, then a kernel trace of the ticks (daemon included).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ctrl_probe.py --variants rccl_tick_sealed_depth1,rccl_tick_sealed_depth2,rccl_tick_sealed_depth3 --repeat 2 --out gpurun_out/ctrl_probe_rep.json > gpurun_out/ctrl_probe_rep.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tick -o tick -- python3 tools/ctrl_probe.py --variants rccl_tick_sealed_depth3 > gpurun_out/prof_tick.log 2>&1
rc=$?; tail -c 2500 gpurun_out/ctrl_probe_rep.log; tail -3 gpurun_out/prof_tick.log; exit $rc
