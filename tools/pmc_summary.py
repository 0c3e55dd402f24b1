"""Summarise a GPU round's rocprofv3 output (gpurun_out/<tag>_*) into profiles/.

* copies the kernel-trace stats CSV to profiles/<tag>_kernel_stats.csv;
* averages every PMC counter over the render kernel's dispatches and writes
  profiles/<tag>_pmc_render_kernel.json;
* updates profiles/pmc_summary.json[<config>/n1/contiguous] with the HBM traffic per launch:
  (2 * FETCH_SIZE + WRITE_SIZE) * 1024 B -- FETCH_SIZE doubled per MI355X_MICROARCH.md "HBM"
  (gfx950 tallies 128-B read requests at 64 B); both counters are KB per dispatch.
"""
import csv
import re
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _is_render(name, kernel):
    """The product row kernel of a dispatch: the generic render_rows_kernel<MODE, F64, CAL, FC> with
    CAL = false, or the scene-specialised rt_spec_rows_ / rt_spec_prim_<f64><cal> with cal = 0 (the one calibration
    launch per geometry is excluded)."""
    if kernel != "render_rows_kernel":
        return kernel in name
    m = re.search(r"render_rows_kernel<([^>]*)>", name)
    if m:
        a = [x.strip() for x in m.group(1).split(",")]
        return not (len(a) >= 3 and a[2] == "true")
    m = re.match(r"rt_spec_(rows|prim)_(\d)(\d)", name)
    return bool(m) and m.group(3) == "0"


def main(tag="r01", config="globes4k", kernel="render_rows_kernel"):
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    ks = os.path.join(out, f"{tag}_kt", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    agg = defaultdict(list)
    names = set()
    for f in glob.glob(os.path.join(out, f"{tag}_pmc_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if _is_render(r["Kernel_Name"], kernel):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                names.add(r["Kernel_Name"])
    mean = {k: sum(v) / len(v) for k, v in agg.items()}
    res = {"kernel": kernel, "dispatches_per_counter": {k: len(v) for k, v in agg.items()}, "mean": mean}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        res["hbm_bytes_per_launch"] = int((2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024)
    f64 = [mean.get(k) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64")]
    if all(v is not None for v in f64):
        res["executed_fp64_flops_per_launch"] = int((f64[0] + f64[1] + 2 * f64[2]) * 64)
        res["executed_fp64_flops_note"] = "(ADD + MUL + 2*FMA) wave-instructions x 64 lanes (inactive lanes included)"
    with open(os.path.join(prof, f"{tag}_pmc_render_kernel.json"), "w") as f:
        json.dump(res, f, indent=1)
    summ_path = os.path.join(prof, "pmc_summary.json")
    summ = json.load(open(summ_path)) if os.path.exists(summ_path) else {}
    if "hbm_bytes_per_launch" in res:
        sha_path = os.path.join(out, f"{tag}_so_sha16.txt")
        summ[f"{config}/n1/contiguous"] = {"tag": tag, "hbm_bytes_per_launch": res["hbm_bytes_per_launch"],
                                           "fetch_kb": mean["FETCH_SIZE"], "write_kb": mean["WRITE_SIZE"],
                                           "so_sha16": open(sha_path).read().strip() if os.path.exists(sha_path) else None,
                                           "variant": "spec" if any(n.startswith("rt_spec_") for n in names) else "generic",
                                           "kernels": sorted(names)}
        if "executed_fp64_flops_per_launch" in res:
            summ[f"{config}/n1/contiguous"]["executed_fp64_flops_per_launch"] = res["executed_fp64_flops_per_launch"]
        if "SQ_INSTS_VALU" in mean and "SQ_WAVES" in mean:
            summ[f"{config}/n1/contiguous"]["valu_insts_per_wave"] = round(mean["SQ_INSTS_VALU"] / mean["SQ_WAVES"], 1)
        # the per-launch counters bench.py's roofline.issue block is derived from
        keep = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                "SQ_INSTS_VALU_TRANS_F64", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE", "GRBM_COUNT")
        summ[f"{config}/n1/contiguous"]["counters"] = {k: mean[k] for k in keep if k in mean}
        with open(summ_path, "w") as f:
            json.dump(summ, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
