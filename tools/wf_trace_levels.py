"""Per-level time of the last wavefront frame in a rocprofv3 kernel trace (gpurun_out/<dir>/run_kernel_trace.csv):
the kernels from the last wf_trace_kernel to the following wf_fixup_kernel, grouped into levels at every
candidate walk of the nearest pass.  usage: python tools/wf_trace_levels.py DIR [--all]"""
import csv
import re
import sys


def short(n):
    return re.sub(r"\(anonymous namespace\)::", "", n).split("(")[0].replace("void ", "")[:34]


def main(d, all_kernels=False):
    rows = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
    s = [i for i, r in enumerate(rows) if "wf_trace_kernel" in r["Kernel_Name"]][-1]
    e = [i for i, r in enumerate(rows) if "wf_fixup" in r["Kernel_Name"] and i > s][0]
    t0 = int(rows[s]["Start_Timestamp"])
    levels, cur = [], None
    for r in rows[s:e + 1]:
        n = short(r["Kernel_Name"])
        if n.startswith("wfp_cand_kernel<false") or cur is None or (n.startswith("wf_fold") and cur[0] != "fold"):
            cur = ["fold" if n.startswith("wf_fold") else f"L{len(levels)}", [], int(r["Start_Timestamp"])]
            levels.append(cur)
        cur[1].append((n, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000))
    for name, ks, st in levels:
        tot = sum(k[1] for k in ks)
        print(f"{name:5} at {(st - t0) / 1000:8.1f} us: {tot:7.1f} us in {len(ks):2d} kernels" +
              ("" if not all_kernels else "  " + ", ".join(f"{k} {v:.1f}" for k, v in ks)))
    print(f"frame {(int(rows[e]['End_Timestamp']) - t0) / 1000:.1f} us, {e - s + 1} kernels")


if __name__ == "__main__":
    main(sys.argv[1], "--all" in sys.argv)
