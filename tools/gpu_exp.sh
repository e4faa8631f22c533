# experiments: symmetric FW + scan variant 5 (parity + C3 timing), sparse lane masks / split labels (parity + C4 timing)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/exp
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_sparse_gpu.py -m gpu -x -q -k "scan_variants or golden or scan_v5 or lane_masks or variants_c4 or fw_symmetric or fw_kernels or random_vs_oracle" --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -2 $out/t.log
for cfg in "2 0" "2 1" "5 1"; do set -- $cfg; timeout -k 10 120 python -u bench.py --entry device --steps 5 --no-cpu --scan-variant $1 --fw-symmetric $2 > $out/b$1_s$2.json 2>$out/b$1_s$2.err && python -c "
import json;d=json.load(open('$out/b$1_s$2.json'));r=d['roofline'];print('scan v$1 sym$2', d['ms_per_step'], d['breakdown_ms'], r['frac'], r['avg_launch_ms'])" || exit 1; done
for cfg in "0 0" "1 0" "0 1" "1 1"; do set -- $cfg; SRG_DEBUG_SPARSE=1 timeout -k 10 200 python -u bench.py --graph ba --steps 2 --warmup 1 --no-cpu --sparse-lane-masks $1 --sparse-split-labels $2 > $out/c4_lm$1_sl$2.json 2>$out/c4_lm$1_sl$2.err && python -c "
import json;d=json.load(open('$out/c4_lm$1_sl$2.json'));r=d['roofline'];print('c4 lm$1 sl$2', d['ms_per_step'], r['frac'])" && grep "^sparse:" $out/c4_lm$1_sl$2.err | tail -1 || exit 1; done
