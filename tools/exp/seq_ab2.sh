set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03q4; mkdir -p $o
for i in 1 2 3 4; do
for sq in 1 0; do
SRG_DEBUG_CODEC=1 SRG_CODEC_SEQ=$sq timeout -k 10 200 python -u bench.py --steps 5 --no-cpu --no-verify > $o/seq$sq.$i.json 2>$o/seq$sq.$i.err || exit 1
done; done
echo ok
