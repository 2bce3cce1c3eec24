"""Busy/idle analysis of a rocprofv3 kernel trace (one stream).
Usage: python tools/trace_gaps.py <kernel_trace.csv> [skip_first_n_dispatches]
Prints total span, summed kernel time, the gap histogram between
consecutive dispatches and the kernels that most often follow large gaps."""
import collections
import csv
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r["Kernel_Name"].split("(")[0].replace("void ocffm::", "")[:40]))
    rows.sort()
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = rows[skip:]
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in rows) / 1e3
    gaps = []
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        gaps.append(((s1 - e0) / 1e3, n0, n1))
    print(f"dispatches {len(rows)}  span {span/1e3:.3f} ms  kernel-busy {busy/1e3:.3f} ms  idle {100*(1-busy/span):.1f}%")
    edges = [0, 1, 2, 4, 8, 16, 32, 64, 1e9]
    hist = collections.Counter()
    tot = collections.Counter()
    for g, _, _ in gaps:
        for lo, hi in zip(edges, edges[1:]):
            if lo <= g < hi or (g < 0 and lo == 0):
                hist[lo] += 1
                tot[lo] += max(g, 0)
    for lo, hi in zip(edges, edges[1:]):
        print(f"gap [{lo:>3}, {hi:>5}) us: n {hist[lo]:6d} total {tot[lo]/1e3:8.3f} ms")
    big = collections.Counter()
    bigt = collections.Counter()
    for g, n0, n1 in gaps:
        if g >= 4:
            big[(n0, n1)] += 1
            bigt[(n0, n1)] += g
    print("largest gap sources (prev -> next): n, total ms")
    for k, v in sorted(bigt.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {k[0]:40s} -> {k[1]:40s} {big[k]:5d} {v/1e3:8.3f}")


if __name__ == "__main__":
    main()
