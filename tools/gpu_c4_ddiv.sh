cd $GRAFT_REPO_ROOT; O=gpurun_out/ddiv; mkdir -p $O
for i in 1 2; do for d in 1 0 2; do
timeout -k 10 300 python -u bench.py --config c4 --entry device --steps 3 --no-cpu --no-ri --sparse-delta-div $d > $O/c4_${d}_$i.json 2> $O/c4_${d}_$i.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c4_${d}_$i.json').read().strip().splitlines()[-1]); print('div $d', d['ms_per_step'], d['verified_rows'])"
done; done
