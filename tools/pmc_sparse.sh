#!/bin/bash
# PMC passes over one C4 (--graph ba) bench step for the sparse kernel (k_sparse_ds), each pass its
# own run (rocprofv3 does not split passes).  usage: tools/pmc_sparse.sh OUTDIR [bench args...]
set -e
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
timeout -k 10 240 python3 -u bench.py --graph ba --steps 2 --warmup 1 --no-cpu "$@" > "$out/c4_bench.json" 2> "$out/c4_bench.err"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- python3 -u bench.py --graph ba --steps 1 --warmup 1 --no-cpu --no-profile "$@" > "$out/stats.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 -u bench.py --graph ba --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 -u bench.py --graph ba --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/write.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$out/sq" -o run -- python3 -u bench.py --graph ba --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/sq.log" 2>&1
echo pmc done
