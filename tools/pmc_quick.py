"""Print the mean PMC counters of the product row kernel over gpurun_out/<prefix>*/run_counter_collection.csv
(no profiles/ update: for A/B passes of diagnostic libraries).
usage: python tools/pmc_quick.py PREFIX [KERNEL]   (KERNEL default rt_spec_rows_00)"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import _is_render   # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(prefix, kernel="rt_spec_rows_00"):
    agg = defaultdict(list)
    for f in glob.glob(os.path.join(ROOT, "gpurun_out", prefix + "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if _is_render(r["Kernel_Name"], kernel):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{prefix} {k}: mean {sum(v) / len(v):.1f} over {len(v)} dispatches")
    if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
        fe, wr = (sum(agg[k]) / len(agg[k]) for k in ("FETCH_SIZE", "WRITE_SIZE"))
        print(f"{prefix} HBM per launch (2 FETCH + WRITE): {(2 * fe + wr) * 1024 / 1e6:.1f} MB (write {wr / 1024:.1f} MiB)")


if __name__ == "__main__":
    main(*sys.argv[1:])
