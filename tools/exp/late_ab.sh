set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03q; mkdir -p $o
for i in 1 2; do
for ll in 1 0; do
timeout -k 10 200 python -u bench.py --steps 5 --no-cpu --no-verify --late-loss $ll > $o/ll$ll.$i.json 2>$o/ll$ll.$i.err || exit 1
done; done
echo ok
