#!/bin/bash
# One GPU call for an iteration: GPU parity tests, smoke, the default bench
# (C2 1M, with the oracle parity sample), a rocprofv3 kernel-trace of a short
# bench, and the C3 bench.  TAG names the outputs (gpurun_out/<TAG>_*).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
TAG=${TAG:-r02q}
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
step smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
step bench
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_bench.json')); print(d['value'], d['ms_per_step'], d.get('parity_sample',{}).get('mismatches'))"
step c3
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_bench.json')); print(d['value'], d['ms_per_step'], d['gb_per_s_scanned'])"
step c4
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c4_bench.json 2> gpurun_out/${TAG}_c4.err || { tail -20 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_bench.json')); print(d['value'], d['ms_per_step'], d['gb_per_s_scanned'])"
[ "${PROF:-0}" = "0" ] && exit 0
export TMPDIR=/tmp
step rocprof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_prof_bench.json 2>$R/gpurun_out/${TAG}_prof_bench.err) || { tail -5 gpurun_out/${TAG}_prof_bench.err; exit 1; }
echo done
