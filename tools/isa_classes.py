"""Static instruction-class histogram of one kernel in an assembly listing (hipcc -S, or a code
object disassembled by llvm-objdump): what the specialised megakernel's instructions are, by class
(VERDICT round 4, item 4).  Static counts (each instruction once), not executed counts.
usage: python tools/isa_classes.py FILE.s KERNEL_NAME"""
import collections
import re
import sys

CLASSES = [
    ("fp64 add/mul/fma", r"^v_(add|mul|fma|fmac)_f64"),
    ("fp64 div helpers (div_scale/fmas/fixup, ldexp, frexp, class)", r"^v_(div_scale|div_fmas|div_fixup|ldexp|frexp_\w+|cmp_class)_f64"),
    ("fp64 min/max", r"^v_(min|max)_f64"),
    ("fp64 compare", r"^v_cmpx?_\w+_f64"),
    ("fp64 transcendental (rcp/rsq/sqrt)", r"^v_(rcp|rsq|sqrt)_f64"),
    ("select (v_cndmask)", r"^v_cndmask"),
    ("move (v_mov, readfirstlane/readlane/writelane)", r"^v_(mov|readfirstlane|readlane|writelane|accvgpr)"),
    ("int / bit ops", r"^v_(add|sub|subrev|mul|mad|lshl|lshr|ashr|and|or|xor|bfi|bfe|alignbit|not|cmp\w*_[iu]\d+|min_[iu]|max_[iu]|bcnt|mbcnt|perm|lshlrev|lshrrev|ashrrev|cmpx?_\w+_[iu]\d+)"),
    ("convert", r"^v_cvt"),
    ("other VALU", r"^v_"),
    ("scalar ALU", r"^s_(?!waitcnt|nop|cbranch|branch|load|buffer|store|setprio|endpgm|getpc|swappc|setpc|sleep|barrier)"),
    ("scalar memory", r"^s_(load|buffer|store)"),
    ("branch", r"^s_(cbranch|branch|setpc|swappc|getpc)"),
    ("s_waitcnt / s_nop", r"^s_(waitcnt|nop)"),
    ("vector memory (global/buffer/scratch/flat)", r"^(global|buffer|scratch|flat)_"),
    ("LDS", r"^ds_"),
]


def main(path, kernel):
    s = open(path).read()
    m = re.search(r"^(%s[^:\n]*):" % re.escape(kernel), s, re.M)
    i = m.end()
    j = s.index(".Lfunc_end", i)
    c = collections.Counter()
    total = 0
    for line in s[i:j].splitlines():
        line = line.strip()
        if not line or line.startswith((".", ";")) or line.endswith(":"):
            continue
        op = line.split()[0]
        total += 1
        for name, pat in CLASSES:
            if re.match(pat, op):
                c[name] += 1
                break
        else:
            c["unclassified"] += 1
    valu = sum(v for k, v in c.items() if k.startswith(("fp64", "select", "move", "int", "convert", "other VALU")))
    print(f"{kernel}: {total} static instructions, {valu} VALU")
    for name, _ in CLASSES + [("unclassified", "")]:
        if c[name]:
            share = f"{100.0 * c[name] / valu:5.1f} % of VALU" if name.startswith(("fp64", "select", "move", "int", "convert", "other VALU")) else ""
            print(f"  {name:62s} {c[name]:6d}  {share}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
