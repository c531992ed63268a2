#!/bin/bash
# rocprofv3 PMC passes over one command (args = the python command line after
# `python3`).  Each pass is its own run (gfx950 counter-slot limits); output
# under gpurun_out/pmc/<pass>/.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
i=0
script="$1"; shift
case "$script" in /*) ;; *) script="$R/$script" ;; esac
NPASS=${PMC_NPASS:-4}  # 2: the SQ passes only
PASSES=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
        "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
        "FETCH_SIZE"
        "WRITE_SIZE")
for pmc in "${PASSES[@]:0:$NPASS}"; do
  i=$((i+1))
  mkdir -p "$R/gpurun_out/pmc/p$i"
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python3 "$script" "$@" > "$R/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc ($pmc)"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc/p$i.log"; exit $rc; fi
done
