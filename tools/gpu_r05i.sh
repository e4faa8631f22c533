#!/bin/bash
# Round 5: PMC of tight_v6 vs tight_v5 (one C3 step each)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05i}; mkdir -p $O
export SRG_STREAM_HOPS=events; ./tools/pmc_scan.sh $O/v6 --no-ri --no-verify --fw-overlap 0 --scan-kernel 6 && ./tools/pmc_scan.sh $O/v5 --no-ri --no-verify --fw-overlap 0 --scan-kernel 5 || exit 1
python3 tools/pmc_kernel.py $O/v6 tight_v6; python3 tools/pmc_kernel.py $O/v5 tight_v5
