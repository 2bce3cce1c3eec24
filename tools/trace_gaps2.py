"""Per-epoch busy/span and the largest inter-kernel gap classes of a
rocprofv3 kernel trace of bench.py (epochs end at k_colsum_multi).
Usage: python tools/trace_gaps2.py <kernel_trace.csv> [epoch index]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "colsum_multi" in r["Kernel_Name"]]
ends = idx[1::2]
for a, b in zip(ends[:-1], ends[1:]):
    seg = rows[a + 1:b + 1]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    print(f"kernels {len(seg)} busy {busy:.0f} us span {span:.0f} us gaps {span - busy:.0f}")
e = int(sys.argv[2]) if len(sys.argv) > 2 else len(ends) // 2
seg = rows[ends[e] + 1:ends[e + 1] + 1]
gaps = collections.defaultdict(list)
prev = pn = None
for r in seg:
    n = r["Kernel_Name"].split("(")[0].replace("void ocffm::", "").split("<")[0]
    if prev is not None:
        gaps[(pn, n)].append((int(r["Start_Timestamp"]) - prev) / 1e3)
    prev, pn = int(r["End_Timestamp"]), n
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:14]:
    print(f"{k[0]:22s} -> {k[1]:22s} n {len(v):4d} avg {sum(v) / len(v):6.2f} tot {sum(v):7.1f}")
