cd $GRAFT_REPO_ROOT; O=gpurun_out/c5rs; mkdir -p $O
for v in 12 16; do SRG_LIB_PATH=$GRAFT_REPO_ROOT/ab/librs$v.so timeout -k 10 300 python -u -m pytest tests/test_events.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }; echo "rs$v $(tail -1 $O/pytest_$v.log)"; done
for i in 1 2 3; do for v in 8 12 16; do
  if [ $v = 8 ]; then L=; else L=$GRAFT_REPO_ROOT/ab/librs$v.so; fi
  SRG_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config c5 --steps 20 --no-cpu > $O/c5_${v}_$i.json 2> $O/c5_${v}_$i.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/c5_${v}_$i.json').read().strip().splitlines()[-1]); print('rounds $v', d['ms_per_step'])"
done; done
