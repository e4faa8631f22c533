#!/bin/bash
# Round 5: fused one-pass codec encoder -- codec / overlap parity, then C3 with 8 / 12 / 16 codec threads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05o}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fw_overlap.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "codec or overlap or early or late or seq" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do for t in 8 12 16; do
  SRG_CODEC_THREADS=$t SRG_DEBUG_CODEC=1 timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --no-verify > $O/c3_t${t}_$i.json 2> $O/c3_t${t}_$i.err || { tail $O/c3_t${t}_$i.err; exit 1; }
done; done
python3 - "$O" <<'PY'
import json,glob,sys,re,statistics
O=sys.argv[1]
for f in sorted(glob.glob(O+"/c3_t*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); b=d["breakdown_ms"]
    cl=[l for l in open(f.replace(".json",".err")) if l.startswith("codec:") and "convert" in l]
    conv=[float(re.search(r"convert ([0-9.]+)",l).group(1)) for l in cl]
    print(f, d["ms_per_step"], "h2d", b["ms_h2d"], "conv med", statistics.median(conv) if conv else None)
PY
