set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r03c2; mkdir -p $o
run() { timeout -k 10 120 python -u bench.py --config c2 --steps 10 --no-cpu --no-verify "$@" > $o/$1$2_$3$4.json 2>/dev/null || exit 1; }
for i in 1 2; do
timeout -k 10 120 python -u bench.py --config c2 --steps 10 --no-cpu --no-verify > $o/base.$i.json 2>/dev/null || exit 1
timeout -k 10 120 python -u bench.py --config c2 --steps 10 --no-cpu --no-verify --scan-groups 1 > $o/sg1.$i.json 2>/dev/null || exit 1
timeout -k 10 120 python -u bench.py --config c2 --steps 10 --no-cpu --no-verify --scan-groups 6 > $o/sg6.$i.json 2>/dev/null || exit 1
timeout -k 10 120 python -u bench.py --config c2 --steps 10 --no-cpu --no-verify --loss-chunks 16 > $o/lc16.$i.json 2>/dev/null || exit 1
timeout -k 10 120 python -u bench.py --config c2 --steps 10 --no-cpu --no-verify --d2h-mode 0 > $o/d2h0.$i.json 2>/dev/null || exit 1
done
echo ok
