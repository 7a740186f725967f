# A/B of the CPU placement modes (OCM_PIN: default = daemon on its own core of
# the GPU's L3 complex and apps on the others; ccd = both on the whole complex;
# 0 = unpinned): remote ocm_alloc / ocm_free latency and 4 KiB put/get, from
# Python (tools/runtime_probe.py) and from the native ocm_bench (tools/spin_probe.py).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for mode in core ccd 0; do
  OCM_PIN=$mode timeout -k 10 200 python -u tools/runtime_probe.py --modes torch_first --repeat 1 > gpurun_out/pin_py_${mode}_${rep}.log 2>&1 || exit $?
  OCM_PIN=$mode timeout -k 10 120 python -u tools/spin_probe.py --gpu --meshes 1 --modes poll > gpurun_out/pin_c_${mode}_${rep}.log 2>&1 || exit $?
done; done
