#!/bin/bash
# One GPU call: parity tests, smoke, the default bench (JSON line), a
# rocprofv3 kernel-trace/stats profile of the bench, the PMC traffic passes
# for the roofline kernel and the PMC occupancy passes.  Stops at the first
# failing step.  TAG names the outputs (gpurun_out/<TAG>_*).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
TAG=${TAG:-r03}
STEPS=${STEPS:-all}
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
step smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
step bench
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_c2_bench.json
[ "$STEPS" = "bench" ] && exit 0
export TMPDIR=/tmp
step rocprof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_prof_bench.json 2>$R/gpurun_out/${TAG}_prof_bench.err) || { tail -5 gpurun_out/${TAG}_prof_bench.err; exit 1; }
step traffic
timeout -k 10 400 python -u tools/pmc_traffic.py --config c2 --n-req 1000000 --tag ${TAG} --out gpurun_out/${TAG}_traffic_c2.json > gpurun_out/${TAG}_traffic.log 2>&1 || { tail -20 gpurun_out/${TAG}_traffic.log; exit 1; }
tail -1 gpurun_out/${TAG}_traffic.log
step occupancy
timeout -k 10 400 python -u tools/pmc_occupancy.py --config c2 --n-req 1000000 --out gpurun_out/${TAG}_pmc_c2.json > gpurun_out/${TAG}_occ.log 2>&1 || { tail -20 gpurun_out/${TAG}_occ.log; exit 1; }
cat gpurun_out/${TAG}_occ.log
[ "${CONFIGS:-1}" = "0" ] && exit 0
step c3
timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 --e2e-iters 0 > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
cat gpurun_out/${TAG}_c3_bench.json
step c4
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 --e2e-iters 0 > gpurun_out/${TAG}_c4_bench.json 2> gpurun_out/${TAG}_c4.err || { tail -20 gpurun_out/${TAG}_c4.err; exit 1; }
cat gpurun_out/${TAG}_c4_bench.json
step c5
timeout -k 10 500 python -u bench.py --config c5 --steps 3 --warmup 1 --e2e-iters 0 > gpurun_out/${TAG}_c5_bench.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
cat gpurun_out/${TAG}_c5_bench.json
