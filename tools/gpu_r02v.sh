set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --output-format csv -d $O/r02v_pcs -o run -- python3 tools/render_loop.py 30 > $O/r02v_pcs.out 2> $O/r02v_pcs.err || { tail -20 $O/r02v_pcs.err; exit 1; }
ls -la $O/r02v_pcs
