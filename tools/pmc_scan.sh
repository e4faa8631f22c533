#!/bin/bash
# PMC passes over one C3 bench step for the tight scan kernel (one pass per counter group).
# usage: tools/pmc_scan.sh OUTDIR [bench args...]
set -e
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
cd /tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d "$R/$out/sq" -o run -- python3 -u $R/bench.py --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$R/$out/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d "$R/$out/lds" -o run -- python3 -u $R/bench.py --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$R/$out/lds.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$out/fetch" -o run -- python3 -u $R/bench.py --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$R/$out/fetch.log" 2>&1
echo pmc done
