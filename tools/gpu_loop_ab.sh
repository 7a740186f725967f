# Loopback bench step time under service variants (which part of the step is not in the per-op times).
set -o pipefail
mkdir -p gpurun_out
for v in default proto1 nosvc idle200; do
  case $v in
    default) e="";; proto1) e="OCM_SERVICE_PROTO=1";; nosvc) e="OCM_SERVICE_MAX=0";; idle200) e="OCM_SERVICE_IDLE_US=200";;
  esac
  env $e timeout -k 10 200 python -u bench.py --remote loopback --no-optim-extra --no-characterize --json-out gpurun_out/loop_$v.json > gpurun_out/loop_$v.log 2>&1 || exit $?
done
python3 -c "
import json
for v in ['default','proto1','nosvc','idle200']:
    b=json.load(open(f'gpurun_out/loop_{v}.json')); print(v, b['value'], b['ms_per_step'])
"
