set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03r; mkdir -p $o
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 5 --no-cpu --no-verify > $o/reg.$i.json 2>$o/reg.$i.err || exit 1
SRG_EXP_NO_EARLY=1 timeout -k 10 200 python -u bench.py --steps 5 --no-cpu --no-verify > $o/noreg.$i.json 2>$o/noreg.$i.err || exit 1
done
echo ok
