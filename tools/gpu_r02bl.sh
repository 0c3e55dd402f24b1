# HBM traffic of the refraction kernel with the first refraction frame's state in LDS (anim120).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for PMC in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/r02blanim_pmc_$PMC -o run -- python3 bench.py --config anim120 --steps 1 --warmup 0 --settle-ms 0 --no-cpu-baseline > /dev/null 2> $O/r02bl.err || { tail $O/r02bl.err; exit 1; }
done
echo ok
