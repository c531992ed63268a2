#!/bin/bash
# k_body LDS-tiled transformations: parity with the tiles off, then on (the
# original bodies, then the tile-edge bodies), then the C3 cycle profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05body}
T="timeout -k 10 150 python -u -m pytest tests/test_body_chunks.py -m gpu -x -q --timeout 120 --timeout-method thread"
echo "== tiles off $(date +%T)"
GI_BODY_TILES=0 $T > gpurun_out/${TAG}_off.log 2>&1 || { tail -30 gpurun_out/${TAG}_off.log; exit 1; }
tail -1 gpurun_out/${TAG}_off.log
echo "== tiles on, original bodies $(date +%T)"
$T -k "parity" > gpurun_out/${TAG}_on.log 2>&1 || { tail -30 gpurun_out/${TAG}_on.log; exit 1; }
tail -1 gpurun_out/${TAG}_on.log
echo "== tiles on, tile edges $(date +%T)"
$T -k "tile_edges" > gpurun_out/${TAG}_edges.log 2>&1 || { tail -30 gpurun_out/${TAG}_edges.log; exit 1; }
tail -1 gpurun_out/${TAG}_edges.log
if [ "${PROF:-0}" = "1" ]; then
  TAG=${TAG} CONFIGS="c3" ARGS="--n-req 50000 --e2e-iters 0" bash tools/gpu_prof.sh
fi
echo done
