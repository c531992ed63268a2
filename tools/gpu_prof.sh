#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench run (args passed to bench.py).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/prof"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/prof_bench.log" 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 "$R/gpurun_out/prof_bench.log"
find "$R/gpurun_out/prof" -name "*stats*" | head
exit $rc
