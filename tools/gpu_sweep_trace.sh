# Which bench.py setup step makes every sweep step wait ~2 ms (the copy service's idle exit)?
set -o pipefail
mkdir -p gpurun_out
for v in plain torch verify both; do
  case $v in plain) f="";; torch) f="--torch";; verify) f="--verify";; both) f="--torch --verify";; esac
  timeout -k 10 200 python -u tools/sweep_trace.py --remote loopback $f > gpurun_out/st_$v.json 2> gpurun_out/st_$v.err || exit $?
done
python3 -c "
import json
for v in ['plain','torch','verify','both']:
    d=json.load(open(f'gpurun_out/st_{v}.json')); print(v, [s['step_ms'] for s in d['steps']])
"
