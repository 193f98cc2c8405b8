#!/usr/bin/env python
"""Kernel statistics table from a rocprofv3 rocpd database (ROCm 7.2 default output, ``*_results.db``).

usage: python scripts/rocpd_stats.py gpurun_out/c1/prof_xgb/run_results.db [--top 30] [--md]
"""
import argparse
import sqlite3


def stats(db_path: str):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                      "from kernels group by name order by sum(end - start) desc").fetchall()
    span = db.execute("select min(start), max(end) from kernels").fetchone()
    return rows, span


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--md", action="store_true")
    ap.add_argument("--timeline", default=None, help="kernel-name substring marking one step (e.g. k_gbm_step): "
                    "print every step's wall span and GPU-busy fraction")
    ap.add_argument("--sequence", default=None, help="kernel-name substring marking one step: print the dispatch "
                    "sequence (name, duration, gap before it) of the step after its 10th occurrence")
    ap.add_argument("--gaps", default=None, help="kernel-name substring marking the start of the window (its LAST "
                    "occurrence; e.g. k_num_stats for a DL fit): list the idle gaps > --min-gap us up to the trace end")
    ap.add_argument("--min-gap", type=float, default=50.0)
    ap.add_argument("--window", default=None, help="kernel-name substring marking the start of the window (its LAST "
                    "occurrence): per-kernel table of that window, then every dispatch in order with its gap")
    a = ap.parse_args()
    if a.window:
        db = sqlite3.connect(a.db)
        ks = db.execute("select name, start, end from kernels order by start").fetchall()
        idx = [i for i, k in enumerate(ks) if a.window in k[0]]
        if not idx:
            print("marker not found")
            return
        w = ks[idx[-1]:]
        t0, t1 = w[0][1], max(k[2] for k in w)
        agg = {}
        for nm, st, en in w:
            c, tt = agg.get(nm, (0, 0))
            agg[nm] = (c + 1, tt + en - st)
        busy = sum(v[1] for v in agg.values())
        short = lambda n: n if len(n) < 70 else n[:67] + "..."
        print(f"window {(t1 - t0) / 1e3:.1f} us, {len(w)} dispatches, busy {busy / 1e3:.1f} us\n"
              "| kernel | calls | total us | % |\n|---|---|---|---|")
        for nm, (c, tt) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
            print(f"| `{short(nm)}` | {c} | {tt / 1e3:.1f} | {100 * tt / max(busy, 1):.1f} |")
        print("\n| # | kernel | us | gap us |\n|---|---|---|---|")
        for j, (nm, st, en) in enumerate(w):
            gap = (st - w[j - 1][2]) / 1e3 if j else 0.0
            print(f"| {j} | `{short(nm)}` | {(en - st) / 1e3:.1f} | {gap:.1f} |")
        return
    if a.gaps:
        db = sqlite3.connect(a.db)
        ks = db.execute("select name, start, end from kernels order by start").fetchall()
        idx = [i for i, k in enumerate(ks) if a.gaps in k[0]]
        if not idx:
            print("marker not found")
            return
        i0 = idx[-1]
        t0, t1 = ks[i0][1], max(k[2] for k in ks[i0:])
        busy, last_end, gaps, prev = 0, t0, [], ""
        for nm, st, en in ks[i0:]:
            if st > last_end and (st - last_end) / 1e3 >= a.min_gap:
                gaps.append(((st - last_end) / 1e3, prev, nm))
            busy += max(0, en - max(st, last_end))
            last_end = max(last_end, en)
            prev = nm
        print(f"window {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us; "
              f"gaps >= {a.min_gap:g} us: {len(gaps)}, {sum(g[0] for g in gaps):.1f} us")
        print("| gap us | after | before |\n|---|---|---|")
        short = lambda n: n if len(n) < 50 else n[:47] + "..."
        for g, p_, n in gaps:
            print(f"| {g:.1f} | `{short(p_)}` | `{short(n)}` |")
        return
    if a.sequence:
        db = sqlite3.connect(a.db)
        ks = db.execute("select name, start, end from kernels order by start").fetchall()
        idx = [i for i, k in enumerate(ks) if a.sequence in k[0]]
        if len(idx) < 12:
            print("not enough steps")
            return
        i0, i1 = idx[10], idx[11]
        print(f"step span {(ks[i1][1] - ks[i0][1]) / 1e3:.1f} us, {i1 - i0} dispatches\n| # | kernel | us | gap us |\n|---|---|---|---|")
        for j in range(i0, i1):
            nm = ks[j][0] if len(ks[j][0]) < 60 else ks[j][0][:57] + "..."
            print(f"| {j - i0} | `{nm}` | {(ks[j][2] - ks[j][1]) / 1e3:.1f} | {(ks[j][1] - ks[j - 1][2]) / 1e3:.1f} |")
        return
    if a.timeline:
        db = sqlite3.connect(a.db)
        ks = db.execute("select name, start, end from kernels order by start").fetchall()
        marks = [k[1] for k in ks if a.timeline in k[0]]
        print(f"| step | span us | busy us | busy % |\n|---|---|---|---|")
        for i in range(len(marks) - 1):
            t0, t1 = marks[i], marks[i + 1]
            busy = sum(min(e, t1) - max(s_, t0) for _, s_, e in ks if e > t0 and s_ < t1)
            print(f"| {i} | {(t1 - t0) / 1e3:.1f} | {busy / 1e3:.1f} | {100 * busy / max(t1 - t0, 1):.0f} |")
        return
    rows, span = stats(a.db)
    tot = sum(r[2] for r in rows)
    print(f"kernels: {sum(r[1] for r in rows)} dispatches, {tot / 1e6:.2f} ms busy, first->last {(span[1] - span[0]) / 1e6:.2f} ms")
    if a.md:
        print("| kernel | calls | total ms | avg us | min us | max us | % |\n|---|---|---|---|---|---|---|")
    for name, n, s, avg, mn, mx in rows[: a.top]:
        nm = name if len(name) < 70 else name[:67] + "..."
        if a.md:
            print(f"| `{nm}` | {n} | {s / 1e6:.2f} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | {100 * s / tot:.1f} |")
        else:
            print(f"{nm:70s} {n:6d} {s / 1e6:9.2f} ms {avg / 1e3:9.1f} us {100 * s / tot:5.1f} %")


if __name__ == "__main__":
    main()
