"""Kernel sequence of a rocprofv3 kernel trace: start offset, gap before,
duration, grid size and short name of every dispatch from the n-th last
`k_init`-free window.  Usage: python tools/epoch_timeline.py <kernel_trace.csv> [first] [count]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    count = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows)
    t0 = int(rows[first]["Start_Timestamp"]) if rows else 0
    prev = t0
    for r in rows[first:first + count]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ocffm::", "").replace("ocffm::", "")
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{(s - t0) / 1e3:10.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f} grid {grid:6d} {name}")
        prev = e


if __name__ == "__main__":
    main()
