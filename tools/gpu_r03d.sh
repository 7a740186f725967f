# Round-3 GPU check of the shared-memory app link: N=1 bench with the link and
# with the mailbox alone (OCM_SHM_LINK=0), then the GPU suite and smoke. Every
# step has its own time limit; a fault, abort, segfault or time limit ends the
# script.
set -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if fatal $rc; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
step bench_link 300 python3 -u bench.py --steps 20 --warmup 5 --json-out $OUT/bench_link.json
step bench_nolink 300 env OCM_SHM_LINK=0 python3 -u bench.py --steps 20 --warmup 5 --no-optim-extra --json-out $OUT/bench_nolink.json
step bench_link2 300 python3 -u bench.py --steps 20 --warmup 5 --no-optim-extra --json-out $OUT/bench_link2.json
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()"
tail -3 $OUT/pytest_gpu.log
