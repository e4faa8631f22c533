#!/bin/bash
# fused FW step phase traces (SRG_FW_TRACE) for simulated ranks and one rank, several chain sizes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-trace}
mkdir -p $out
run() {  # tag, env..., -- bench args
  tag=$1; shift
  env "$@" SRG_FW_TRACE=1 timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 1 --no-cpu --no-verify --fw-step 1 $BARGS > $out/$tag.json 2> $out/$tag.err || { echo "$tag failed"; tail -5 $out/$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; d=json.load(open('$out/$tag.json')); print(d['ms_per_step'], d['breakdown_ms']['ms_fw'])") $(grep 'fw_step mean' $out/$tag.err | tail -1)"
}
BARGS="--simulate-rank 8:0"
run s8_def A=1 && run s8_ch128 SRG_FW_CH=128 && run s8_ch64 SRG_FW_CH=64 && run s8_sb1 SRG_FW_SB=1 && run s8_sb1_ch128 SRG_FW_SB=1 SRG_FW_CH=128 && \
run s8_flag0 SRG_SIM_FLAG_US=0 SRG_SIM_LINK_GBPS=1e9 && \
BARGS="--simulate-rank 4:0" run s4_def A=1 && BARGS="--simulate-rank 2:0" run s2_def A=1 && \
BARGS="" run c3_def A=1 && BARGS="" run c3_ch128 SRG_FW_CH=128 && BARGS="--config c2" run c2_def A=1 && BARGS="--config c2" run c2_ch64 SRG_FW_CH=64
