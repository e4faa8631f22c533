set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03k2; mkdir -p $o
for i in 1 2; do
for t in 8 12 4; do
SRG_CODEC_THREADS=$t timeout -k 10 200 python -u bench.py --steps 5 --no-cpu --no-verify > $o/t$t.$i.json 2>$o/t$t.$i.err || exit 1
done; done
echo ok
