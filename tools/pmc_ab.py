"""Summarise rocprofv3 --pmc passes of several variants (diagnostic): for each
gpurun_out/<tag>_<variant>_pmc_*/run_counter_collection.csv, the mean of every counter over the
product dispatches of the render kernels (the calibration instantiation, template argument CAL =
`true`, excluded), per kernel name.  usage: python tools/pmc_ab.py TAG [OUT.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, out=None):
    res = {}
    for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"{tag}_*_pmc_*"))):
        variant = os.path.basename(d)[len(tag) + 1:].split("_pmc_")[0]
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                m = re.search(r"(render_rows\w*kernel)<([^>]*)>", name)
                if not m:
                    continue
                targs = [t.strip() for t in m.group(2).split(",")]
                cal_pos = 1 if "deferred" in m.group(1) else 2      # <REFR, F64, CAL, FC> / <F64, CAL, FC>
                if len(targs) > cal_pos and targs[cal_pos] == "true":
                    continue                                        # the calibration instantiation
                key = f"{m.group(1)}<{m.group(2)}>"
                res.setdefault(variant, {}).setdefault(key, defaultdict(list))[r["Counter_Name"]].append(
                    float(r["Counter_Value"]))
    summ = {}
    for v, ks in res.items():
        for k, cs in ks.items():
            mean = {c: sum(x) / len(x) for c, x in cs.items()}
            if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
                mean["hbm_bytes_per_launch"] = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
            if "SQ_INSTS_VALU" in mean and "SQ_WAVES" in mean:
                mean["valu_per_wave"] = mean["SQ_INSTS_VALU"] / mean["SQ_WAVES"]
            summ[f"{v}/{k}"] = mean
    print(json.dumps(summ, indent=1))
    if out:
        json.dump(summ, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
