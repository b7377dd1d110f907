"""Compare per-class kernel time per step between two rocprof kernel_stats.csv runs.
usage: python tools/stats_cmp.py DIR_A DIR_B [steps]"""
import csv, re, sys
n = float(sys.argv[3]) if len(sys.argv) > 3 else 13


def load(d):
    rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    out = {}
    for r in rows:
        k = re.sub(r"^void ", "", r["Name"])
        k = re.sub(r"\(.*", "", k)[:90]
        c = out.setdefault(k, [0.0, 0.0])
        c[0] += int(r["Calls"]) / n
        c[1] += float(r["TotalDurationNs"]) / n / 1e3
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
keys = sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, [0, 0])[1] - a.get(k, [0, 0])[1]))
print(f"total {sum(v[1] for v in a.values()):9.1f} {sum(v[1] for v in b.values()):9.1f} us/step")
for k in keys[:25]:
    x, y = a.get(k, [0, 0]), b.get(k, [0, 0])
    print(f"{x[1]:8.1f} {y[1]:8.1f} {y[1]-x[1]:+8.1f}  {x[0]:5.1f} {y[0]:5.1f}  {k}")
