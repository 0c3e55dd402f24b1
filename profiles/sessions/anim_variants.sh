#!/bin/bash
# anim120 (BASELINE config 5) throughput and HBM traffic per variant library: one bench line and two
# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) each.  usage: TAG=x bash profiles/sessions/anim_variants.sh LIB...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r03x}
for LIBP in "$@"; do
  N=$(basename $LIBP .so)
  RT_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --config anim120 --steps 3 --warmup 2 --no-cpu-baseline > $O/${T}_${N}_anim.json 2> $O/${T}_${N}_anim.err || { tail $O/${T}_${N}_anim.err; exit 1; }
  for P in FETCH_SIZE WRITE_SIZE; do
    RT_LIB_PATH=$LIBP timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/${T}_${N}_pmc_$P -o run -- python3 bench.py --steps 1 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-extra --config anim120 > /dev/null 2> $O/${T}_${N}_pmc_$P.err || { echo "pmc $P failed for $N"; exit 1; }
  done
  python3 - "$O" "$T" "$N" <<'PY'
import csv, glob, json, re, sys
O, T, N = sys.argv[1:]
v = json.load(open(f"{O}/{T}_{N}_anim.json"))["value"]
res = {}
for P in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = []
    for f in glob.glob(f"{O}/{T}_{N}_pmc_{P}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            m = re.search(r"render_rows_kernel<([^>]*)>", r["Kernel_Name"])
            if m and m.group(1).split(",")[2].strip() == "false":
                vals.append(float(r["Counter_Value"]))
    res[P] = sum(vals) / max(1, len(vals))
mb = (2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024 / 1e6
print(f"{N}: anim120 {v} Mrays/s, HBM traffic {mb:.1f} MB per frame launch (fetch {res['FETCH_SIZE']:.0f} KB x2, write {res['WRITE_SIZE']:.0f} KB)")
PY
done
