#!/bin/bash
# Round 5: FW bulk PMC passes with the FW after the H2D (the bulk launches the bench times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r05final}; mkdir -p $out
timeout -k 10 900 bash tools/pmc_fw.sh $out/pmc_fw_ov0 --fw-overlap 0 --no-ri --no-verify > $out/pmc_fw_ov0.log 2>&1 || { echo "pmc_fw failed"; tail -20 $out/pmc_fw_ov0.log; exit 1; }
echo done
