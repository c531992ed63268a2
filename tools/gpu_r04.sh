#!/bin/bash
# Round-4 GPU iteration: the tests named in FIRST (fail fast), the whole GPU
# suite, the tally fixture re-record (RECORD=1), the default bench (C2 1M, with
# the oracle parity sample) and optionally C3/C4 (CONFIGS=1) and a rocprofv3
# kernel-trace of a short bench (PROF=1).  TAG names gpurun_out/<TAG>_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
TAG=${TAG:-r04}
step() { echo "== $1 $(date +%T)"; }
if [ -n "${FIRST:-}" ]; then
  step first
  timeout -k 10 300 python -u -m pytest $FIRST ${FIRST_K:+-k "$FIRST_K"} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_first.log 2>&1 || { tail -40 gpurun_out/${TAG}_first.log; exit 1; }
  tail -1 gpurun_out/${TAG}_first.log
fi
if [ "${SUITE:-1}" = "1" ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest_gpu.log
  step smoke
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
if [ "${RECORD:-0}" = "1" ]; then
  step record_tally
  timeout -k 10 200 python -u tools/record_tally.py > gpurun_out/${TAG}_record.log 2>&1 || { tail -20 gpurun_out/${TAG}_record.log; exit 1; }
  cp tests/golden/tally_crs_pl1_world2.json gpurun_out/${TAG}_tally_crs_pl1_world2.json
  tail -1 gpurun_out/${TAG}_record.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_bench.json')); print(d['value'], d['ms_per_step'], d.get('parity_sample',{}).get('mismatches'), {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items()}, d['tally']['score_hist_nonzero'])"
fi
if [ "${CONFIGS:-0}" = "1" ]; then
  for c in c3 c4 c5; do
    step $c
    timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --e2e-iters 0 > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}.err || { tail -20 gpurun_out/${TAG}_${c}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_bench.json')); print(d['value'], d['ms_per_step'], d.get('gb_per_s_scanned'), d.get('parity_sample',{}).get('mismatches'))"
  done
fi
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  step rocprof
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_prof_bench.json 2>$R/gpurun_out/${TAG}_prof_bench.err) || { tail -5 gpurun_out/${TAG}_prof_bench.err; exit 1; }
fi
echo done
if [ "${TRAFFIC:-0}" = "1" ]; then
  step traffic
  timeout -k 10 400 python -u tools/pmc_traffic.py --config c2 --n-req 1000000 --tag ${TAG} --out gpurun_out/${TAG}_traffic_c2.json > gpurun_out/${TAG}_traffic.log 2>&1 || { tail -20 gpurun_out/${TAG}_traffic.log; exit 1; }
  tail -3 gpurun_out/${TAG}_traffic.log
fi
if [ "${OCC:-0}" = "1" ]; then
  step occupancy
  timeout -k 10 400 python -u tools/pmc_occupancy.py --config c2 --n-req 1000000 --out gpurun_out/${TAG}_pmc_c2.json > gpurun_out/${TAG}_occ.log 2>&1 || { tail -20 gpurun_out/${TAG}_occ.log; exit 1; }
  cat gpurun_out/${TAG}_occ.log
fi
echo done2
