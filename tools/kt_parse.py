"""Parse tools/r03/tiles.sh output: per site, default time and best forced config."""
import re, sys
cur = None
data = {}
for line in open(sys.argv[1]):
    m = re.match(r"== (\S+)( (\d+))?", line)
    if m:
        cur = m.group(1) if m.group(1) == "default" else int(m.group(3)) if m.group(3) else m.group(1)
        if cur != "default":
            cur = int(line.split()[-1])
        continue
    m = re.match(r"(\S+)\s+(b\d+ \w+ \d+x\d+x\d+)\s+([\d.]+) us", line)
    if m:
        data.setdefault((m.group(1), m.group(2)), {})[cur] = float(m.group(3))
maxm = int(sys.argv[2]) if len(sys.argv) > 2 else 60000
tot_d = tot_b = 0
for (k, n), v in data.items():
    M = int(n.split()[2].split("x")[0])
    if M > maxm or "wgrad" in k or k.startswith("pwlG"):
        continue
    d = v.get("default")
    best = min((t, c) for c, t in v.items() if c != "default")
    tot_d += d; tot_b += min(best[0], d)
    print(f"{k:10s} {n:28s} default {d:7.1f}  best cfg {best[1]:>2} {best[0]:7.1f}  " +
          " ".join(f"{c}:{v.get(c, 0):.0f}" for c in range(13)))
print(f"sum default {tot_d:.1f} us, best {tot_b:.1f} us")
