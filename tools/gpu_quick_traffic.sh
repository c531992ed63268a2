#!/bin/bash
# quick check: a few parity tests, the C2 bench, PMC traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-qt}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "crs_pl1 or crs_pl4 or edge_uris" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_first.log 2>&1 || { tail -30 gpurun_out/${TAG}_first.log; exit 1; }
tail -1 gpurun_out/${TAG}_first.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_c2_bench.json')); print(d['value'], d['ms_per_step'], d['parity_sample']['mismatches'], {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 1})"
timeout -k 10 400 python -u tools/pmc_traffic.py --config c2 --n-req 1000000 --tag ${TAG} --out gpurun_out/${TAG}_traffic_c2.json > gpurun_out/${TAG}_traffic.log 2>&1 || { tail -20 gpurun_out/${TAG}_traffic.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_traffic_c2.json'))['kernels']; print({k: (round(v['fetch_size_kb_raw']*2/1e6,2), round(v['write_size_kb']/1e6,2)) for k, v in d.items() if 'scan' in k or 'eval' in k})"
