set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03q2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "codec or late_loss or golden" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -3 $o/t.log
for i in 1 2; do
for sq in 1 0; do
SRG_CODEC_SEQ=$sq timeout -k 10 200 python -u bench.py --steps 5 --no-cpu --no-verify > $o/seq$sq.$i.json 2>$o/seq$sq.$i.err || exit 1
done; done
SRG_CODEC_SEQ=1 SRG_DEBUG_CODEC=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-verify > $o/dbg.json 2>$o/dbg.err || exit 1
echo ok
