#!/bin/bash
# One GPU call: C2 and C3 benches with GI_DIAG=1 (queue / slow / detect list
# usage on stderr).  TAG names the outputs (gpurun_out/<TAG>_*).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-diag}
echo "== c2 $(date +%T)"
GI_DIAG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_c2.err || { tail -20 gpurun_out/${TAG}_c2.err; exit 1; }
grep GI_DIAG gpurun_out/${TAG}_c2.err | tail -2
echo "== c3 $(date +%T)"
GI_DIAG=1 timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
grep GI_DIAG gpurun_out/${TAG}_c3.err | tail -2
python - <<PY
import json
for c in ("c2", "c3"):
    d = json.load(open("gpurun_out/${TAG}_%s_bench.json" % c))
    print(c, d["value"], d["ms_per_step"], {k: v["ms"] for k, v in d["roofline"]["secondary"]["launches"].items()})
PY
