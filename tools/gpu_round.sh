#!/bin/bash
# One GPU call: parity tests, smoke, the default bench (JSON line), a
# rocprofv3 kernel-trace/stats profile of the bench, and the PMC traffic
# passes for the roofline kernel.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u tools/pmc_traffic.py --config c2 --n-req 1000000 --out gpurun_out/traffic_c2.json > gpurun_out/traffic.log 2>&1 || { tail -20 gpurun_out/traffic.log; exit 1; }
tail -1 gpurun_out/traffic.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2>$R/gpurun_out/prof_bench.err) || { tail -5 gpurun_out/prof_bench.err; exit 1; }
cat gpurun_out/prof_bench.json
