"""Side-by-side table of a tools/kb_ab.sh log: python tools/kb_cmp.py gpurun_out/kab_TAG.log"""
import re, sys
cur, data, order = None, {}, []
for l in open(sys.argv[1]):
    if l.startswith("=="):
        cur = l[3:].strip(); order.append(cur); continue
    m = re.match(r"(\S+)\s+(.*?)\s+([\d.]+) us\s+floor\s+([\d.]+) us", l)
    if m:
        data.setdefault((m.group(1), m.group(2)), {})[cur] = (float(m.group(3)), float(m.group(4)))
tot = {o: 0.0 for o in order}
for k, v in data.items():
    xs = [v.get(o, (float("nan"), 0))[0] for o in order]
    for o, x in zip(order, xs): tot[o] += x
    print(f"{k[0]:12s} {k[1]:30s} " + " ".join(f"{x:8.1f}" for x in xs) + f"   {xs[-1] - xs[0]:+7.1f}")
print("total", {o: round(t, 1) for o, t in tot.items()})
