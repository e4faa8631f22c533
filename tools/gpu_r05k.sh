#!/bin/bash
# Round 5: H2D codec threads A/B on C3 (8 default / 12 / 16), codec timing lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k}; mkdir -p $O
for i in 1 2; do for t in 8 16 12; do
  SRG_CODEC_THREADS=$t SRG_DEBUG_CODEC=1 timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri --no-verify > $O/c3_t${t}_$i.json 2> $O/c3_t${t}_$i.err || { tail $O/c3_t${t}_$i.err; exit 1; }
done; done
python3 - "$O" <<'PY'
import json,glob,sys,re
O=sys.argv[1]
for f in sorted(glob.glob(O+"/c3_t*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); b=d["breakdown_ms"]
    cl=[l for l in open(f.replace(".json",".err")) if l.startswith("codec:")]
    conv=[float(re.search(r"convert ([0-9.]+)",l).group(1)) for l in cl]
    wait=[float(re.search(r"slot waits ([0-9.]+)",l).group(1)) for l in cl]
    print(f, d["ms_per_step"], "h2d", b["ms_h2d"], "conv med", sorted(conv)[len(conv)//2] if conv else None, "wait med", sorted(wait)[len(wait)//2] if wait else None)
PY
