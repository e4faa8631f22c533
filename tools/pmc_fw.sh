#!/bin/bash
# PMC passes over one C3 bench step (each pass its own run, as rocprofv3 does not split passes).
# usage: tools/pmc_fw.sh OUTDIR [bench args...]
set -e
out=$1; shift
export TMPDIR=/tmp
# rocprofv3 --pmc serialises dispatches: the FW cross-stream hops must be events (routing.hip stream_hop)
export SRG_STREAM_HOPS=events
mkdir -p "$out"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu --no-profile "$@" > "$out/stats.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/write.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$out/sq" -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/sq.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d "$out/lds" -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/lds.log" 2>&1
echo pmc done
