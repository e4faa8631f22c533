#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/cuts
mkdir -p $out
for cuts in "24,56" "32,64,72" "40,72" "24,56" "32,64,72" "40,72" "24,48,72" "24,56"; do
SRG_SCAN_CUTS=$cuts timeout -k 10 200 python -u bench.py --no-cpu --entry host --steps 10 > $out/c3.json 2>$out/c3.err || { tail -20 $out/c3.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3.json'));b=d['breakdown_ms'];print('cuts $cuts', d['ms_per_step'], 'h2d',b['ms_h2d'],'fw',b['ms_fw'],'scan',b['ms_scan'],'d2h',b['ms_d2h'])"
done
