#!/bin/bash
# k_scan traffic under GI_SCAN_MODE diagnostics (8: no value_end commit) --
# where k_scan's writes come from.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in ${MODES:-8}; do
  echo "== mode $m $(date +%T)"
  GI_SCAN_MODE=$m timeout -k 10 400 python -u tools/pmc_traffic.py --config c2 --n-req 1000000 --tag scanmode$m --out gpurun_out/scanmode${m}_traffic_c2.json > gpurun_out/scanmode${m}.log 2>&1 || { tail -20 gpurun_out/scanmode${m}.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/scanmode${m}_traffic_c2.json'))['kernels']; print({k: (round(v['fetch_size_kb_raw']*2/1e6,2), round(v['write_size_kb']/1e6,2)) for k, v in d.items() if 'scan' in k})"
done
