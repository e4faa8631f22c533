#!/bin/bash
# round 4 pass m: the chain as one launch (SRG_CHAIN_ONE): rank tests, sims A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04m}
mkdir -p $out
for sr in 8:0 4:0 2:0; do
for cfg in "base:" "one256:SRG_CHAIN_ONE=1 SRG_FW_CH=256" "one512:SRG_CHAIN_ONE=1 SRG_FW_CH=512" "one128:SRG_CHAIN_ONE=1 SRG_FW_CH=128"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr > $out/sim_${sr/:/_}_$name.json 2> $out/sim_${sr/:/_}_$name.err || { echo "sim $sr $name failed"; tail -10 $out/sim_${sr/:/_}_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/sim_${sr/:/_}_$name.json')); b=d['breakdown_ms']; print('$sr $name', d['ms_per_step'], 'fw', b['ms_fw'], 'total', b['ms_total'])"
done
done
