"""Per-kernel PMC summary from tools/pmc_kb.sh output: python3 tools/pmc_table.py DIR [name-filter]

FETCH MB is the raw FETCH_SIZE (KiB -> MB): exact for 64-B read requests, HALF the bytes of wide
128-B-request streams on gfx950 (MI355X_MICROARCH.md §HBM); WR MB is WRITE_SIZE."""
import collections
import csv
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
disp = collections.OrderedDict()
for p in ("p1", "p2", "p3", "p4"):
    try:
        rows = csv.DictReader(open(f"{d}/{p}/run_counter_collection.csv"))
    except FileNotFoundError:
        continue
    for r in rows:
        key = (p, int(r["Dispatch_Id"]))
        e = disp.setdefault(key, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                                  "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "vgpr": r["VGPR_Count"]})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
# group all dispatches of one (name, grid, workgroup) within each pass, in first-seen order
def groups(p):
    out = collections.OrderedDict()
    for (pp, _), e in disp.items():
        if pp == p:
            out.setdefault((e["name"], e["grid"], e["wg"]), []).append(e)
    return out
g = {p: groups(p) for p in ("p1", "p2", "p3", "p4")}
print(f"{'kernel':58s} {'grid':>8s} {'n':>3s} {'us':>7s} {'wait%':>5s} {'winst%':>6s} {'valu%':>5s} {'lds%':>5s} {'ldsconf%':>8s} {'valuI/w':>7s} {'ldsI/w':>6s} {'FETCH MB':>8s} {'WR MB':>6s}")
for key, e1 in g["p1"].items():
    nm = key[0]
    if flt and flt not in nm:
        continue
    def avg(p, k):
        grp = g[p].get(key)
        if not grp:
            return float("nan")
        return sum(x.get(k, 0.0) for x in grp) / len(grp)
    wc = avg("p1", "SQ_WAVE_CYCLES")
    waves = max(1.0, avg("p1", "SQ_WAVES"))
    short = nm.replace("void dfd::", "").replace("dfd::", "")[:58]
    print(f"{short:58s} {key[1]:8d} {len(e1):3d} {avg('p1','dur'):7.1f} {100*avg('p1','SQ_WAIT_ANY')/wc:5.0f} {100*avg('p1','SQ_WAIT_INST_ANY')/wc:6.0f} "
          f"{100*avg('p1','SQ_ACTIVE_INST_VALU')/wc:5.0f} {100*avg('p1','SQ_ACTIVE_INST_LDS')/wc:5.0f} "
          f"{avg('p2','SQ_LDS_BANK_CONFLICT')/max(1,avg('p2','SQ_LDS_IDX_ACTIVE'))*100:8.1f} "
          f"{avg('p2','SQ_INSTS_VALU')/waves:7.0f} {avg('p2','SQ_INSTS_LDS')/waves:6.0f} "
          f"{avg('p3','FETCH_SIZE')/1024:8.1f} {avg('p4','WRITE_SIZE')/1024:6.1f}")
