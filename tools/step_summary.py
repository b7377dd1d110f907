"""Per-training-step summary of a rocprofv3 kernel trace of bench.py.

usage: python tools/step_summary.py <run_kernel_trace.csv> [probe-name-substring] [--order]

A step is the span between two launches of the stem forward kernel (the first kernel of every
B0 step).  Prints, for the median step: GPU-busy time, launches, time per kernel class and the
largest kernels; then the probe kernel's average duration over the whole trace (to compare with
bench.py's HIP-event ``roofline.avg_us``)."""
import csv
import re
import statistics
import sys

CLASSES = [("fused 7x7 MBConv fwd", r"mbconv7"), ("fused 1x1 backward", r"pwl_bwd|pw_fold_bwd"), ("depthwise fwd", r"dw_fwd"), ("depthwise bwd", r"dw_bwd|dw_dgrad|dw_wgrad"),
           ("1x1 conv fwd/dgrad", r"pw_gemm|pw_stream_kernel|pw_sk_kernel"), ("1x1 conv wgrad", r"pw_wgrad|col_sums"),
           ("stem", r"stem_"), ("BN glue", r"bn_|frame_reduce_kernel<[^,]+, 2>"),
           ("SE", r"se_|frame_sum|frame_reduce|mfma_small|sum_parts"),
           ("slab reductions", r"slabs"), ("head / loss", r"linear_|ce_|attn|relu_drop|pool"),
           ("optimizer", r"adam|sumsq|norm_fin|cast_params"), ("other", r".")]


def base(name):
    """kernel name without its argument list (anonymous-namespace qualifiers dropped first)"""
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def klass(name):
    n = base(name)
    for k, pat in CLASSES:
        if re.search(pat, n):
            return k
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    args = [a for a in sys.argv[2:] if not a.startswith("--")]
    probe = args[0] if args else None
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    starts = [i for i, r in enumerate(rows) if "stem_fwd" in r["Kernel_Name"]]
    steps = [rows[a:b] for a, b in zip(starts, starts[1:])]
    busy = [sum(dur(r) for r in s) for s in steps]
    med = steps[sorted(range(len(steps)), key=lambda i: busy[i])[len(steps) // 2]]
    print(f"steps in trace: {len(steps)}; median step: GPU busy {sum(dur(r) for r in med) / 1e3:.3f} ms, "
          f"{len(med)} launches")
    cls = {}
    for r in med:
        c = cls.setdefault(klass(r["Kernel_Name"]), [0.0, 0])
        c[0] += dur(r)
        c[1] += 1
    print("\nclass                  us/step  launches")
    for k, (t, n) in sorted(cls.items(), key=lambda x: -x[1][0]):
        print(f"{k:20s} {t:9.1f} {n:9d}")
    per = {}
    for r in med:
        p = per.setdefault(base(r["Kernel_Name"]), [0.0, 0])
        p[0] += dur(r)
        p[1] += 1
    print("\nlargest kernels (us/step, launches, avg us)")
    for k, (t, n) in sorted(per.items(), key=lambda x: -x[1][0])[:40]:
        print(f"{t:8.1f} {n:4d} {t / n:8.1f}  {k[:110]}")
    if "--order" in sys.argv:  # every launch of the median step in issue order
        print("\nlaunch order (us)")
        for i, r in enumerate(med):
            print(f"{i:4d} {dur(r):8.1f}  {base(r['Kernel_Name'])[:110]}")
    if probe:
        v = [dur(r) for r in rows if probe in r["Kernel_Name"]]
        if v:
            print(f"\nprobe '{probe}': {len(v)} launches, average {statistics.mean(v):.2f} us, "
                  f"median {statistics.median(v):.2f} us")


if __name__ == "__main__":
    main()
