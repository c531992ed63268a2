#!/bin/bash
# A/B timing of ab/<variant>/libgpuinspect.so builds (tools/ab_build.sh) on
# C2: bench (no CPU baseline / e2e) per variant, then optionally the PMC
# traffic of the variants in TRAFFIC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  echo "== $v $(date +%T)"
  L=$PWD/ab/$v/libgpuinspect.so
  [ "$v" = "main" ] && L=$PWD/coraza-kubernetes-operator_amd/libgpuinspect.so
  GI_LIB=$L timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --e2e-iters 0 ${BENCH_ARGS:-} > gpurun_out/ab_${v}.json 2> gpurun_out/ab_${v}.err || { tail -20 gpurun_out/ab_${v}.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_${v}.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['roofline']['secondary']['launches'].items() if v['ms'] > 0.5})"
done
for v in ${TRAFFIC:-}; do
  echo "== traffic $v $(date +%T)"
  L=$PWD/ab/$v/libgpuinspect.so
  [ "$v" = "main" ] && L=$PWD/coraza-kubernetes-operator_amd/libgpuinspect.so
  GI_LIB=$L timeout -k 10 400 python -u tools/pmc_traffic.py --config c2 --n-req 1000000 --tag ab_$v --out gpurun_out/ab_${v}_traffic_c2.json > gpurun_out/ab_${v}_traffic.log 2>&1 || { tail -20 gpurun_out/ab_${v}_traffic.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_${v}_traffic_c2.json'))['kernels']; print({k: (round(v['fetch_size_kb_raw']*2/1e6,2), round(v['write_size_kb']/1e6,2)) for k, v in d.items() if v['hbm_bytes_per_launch'] > 3e8})"
done
