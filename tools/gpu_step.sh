set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/svc_probe.py --tiers host,hbm --configs default,dbhbm --out gpurun_out/svc_dbhbm.json > gpurun_out/svc_dbhbm.log 2>&1
rc=$?; python3 -c "
import json; d=json.load(open('gpurun_out/svc_dbhbm.json'))
for k,v in d.items(): print(k, v['breakdown_4k_put']['doorbell'], {s:(v[s]['get_us'],v[s]['put_us']) for s in ['4096','65536','262144','1048576']})
"; grep -i warn gpurun_out/svc_dbhbm.log | head -3; exit $rc
