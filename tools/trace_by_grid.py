"""Group a rocprofv3 kernel trace by (kernel, grid size): launches, avg and
total duration.  Usage: python tools/trace_by_grid.py <kernel_trace.csv> [substr ...]"""
import collections
import csv
import sys


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if keys and not any(k in n for k in keys):
            continue
        key = (n.split("(")[0].replace("void ocffm::", ""), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]))
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in d.values())
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[0]:45s} grid {k[1]:8d} n {len(v):5d} avg {sum(v)/len(v):8.1f} us  total {sum(v)/1e3:8.3f} ms "
              f"({100*sum(v)/tot:4.1f}%)")


if __name__ == "__main__":
    main()
