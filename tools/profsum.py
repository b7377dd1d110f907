"""Summarise a rocprofv3 kernel_stats.csv per training step: tools/profsum.py <csv> <steps> [top]."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]); top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
tot = sum(float(r['TotalDurationNs']) for r in rows)
print("GPU kernel time per step: %.3f ms" % (tot / steps / 1e6))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
    print("%7.3f %5d %8.1f  %s" % (float(r['TotalDurationNs']) / steps / 1e6, int(r['Calls']), float(r['AverageNs']) / 1e3,
                                   r['Name'][:100]))
