"""Summarise an ab.sh / ab_env.sh log: mean per (layer, pass) for the two arms, A vs B."""
import collections
import sys

cur = None
d = collections.defaultdict(list)
order = []
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = "A" if ("(default)" in line or "libducosy_hip.so" in line) else "B"
        continue
    p = line.split()
    if len(p) == 4:
        d[(p[0], p[1], cur)].append(float(p[2]))
        if (p[0], p[1]) not in order:
            order.append((p[0], p[1]))
for a, b in order:
    A = sum(d[(a, b, "A")]) / max(len(d[(a, b, "A")]), 1)
    B = sum(d[(a, b, "B")]) / max(len(d[(a, b, "B")]), 1)
    print(f"{a:6s} {b:6s} A {A:7.3f}  B {B:7.3f}  A/B-1 {100 * (A / B - 1):+5.1f}%")
