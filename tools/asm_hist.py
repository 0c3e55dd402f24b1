"""Static instruction histogram of one kernel in the hipcc -S output (diagnostic)."""
import collections, re, sys
path, pat = sys.argv[1], sys.argv[2]
s = open(path).read()
m = re.search(r"^(%s[^:\n]*):" % pat, s, re.M)
i = m.end(); j = s.index(".Lfunc_end", i)
c = collections.Counter()
for l in s[i:j].splitlines():
    l = l.strip()
    if not l or l.startswith((".", ";")) or l.endswith(":"): continue
    c[l.split()[0]] += 1
print(m.group(1)[:70], "static instrs", sum(c.values()))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 50): print(f"  {k:30s}{v}")
