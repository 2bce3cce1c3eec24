"""Average PMC counters per dispatch, grouped by kernel (template args kept)
and grid size, over one or more rocprofv3 counter_collection.csv files.
Usage: python tools/pmc_kernels.py <csv> [<csv> ...]"""
import collections
import csv
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = (r["Kernel_Name"].split("(")[0].replace("void ocffm::", ""), int(r["Grid_Size"]))
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items(), key=lambda kv: kv[0]):
        n = max(len(v) for v in cs.values())
        print(f"{k[0]} grid={k[1]} dispatches={n}")
        for c, v in sorted(cs.items()):
            print(f"    {c:32s} {sum(v)/len(v):16.1f}")


if __name__ == "__main__":
    main()
