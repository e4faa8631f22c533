set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03x; mkdir -p $o
for cfg in c2 c1; do
for s in 1 2 4; do
timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --no-cpu --fw-line-split $s > $o/${cfg}_s$s.json 2>$o/${cfg}_s$s.err || exit 1
timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --no-cpu --fw-line-split $s --entry device > $o/${cfg}_s${s}_dev.json 2>$o/${cfg}_s${s}_dev.err || exit 1
done; done
echo ok
