#!/usr/bin/env python
"""GPU busy fraction from a rocprofv3 kernel_trace.csv: over the window spanning the last N launches of a
marker kernel (default k_gbm_step = one per tree), sum of kernel durations (union of intervals) vs wall span,
and the largest idle gaps (host-side launch / decode stalls)."""
import csv
import sys


def main(path, marker="k_gbm_step", last=10):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    marks = [i for i, k in enumerate(ks) if k[2].startswith(marker)]
    i0 = marks[-last - 1] if len(marks) > last else 0
    i1 = marks[-1]
    win = ks[i0:i1]
    t0, t1 = win[0][0], win[-1][0] if len(win) > 1 else win[0][1]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, n in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t1 - t0
    trees = len([k for k in win if k[2].startswith(marker)])
    print(f"trees={trees} wall/tree={span / trees / 1e3:.1f} us busy/tree={busy / trees / 1e3:.1f} us "
          f"busy={100 * busy / span:.1f}% launches/tree={len(win) / trees:.1f}")
    gaps.sort(reverse=True)
    print("largest gaps (us, next kernel):")
    for g, n in gaps[:12]:
        print(f"  {g / 1e3:8.1f}  {n[:70]}")
    print(f"sum of gaps/tree: {sum(g for g, _ in gaps) / trees / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))
