"""Summarise rocprofv3 output into profiles/ (run on the build box).

  python tools/pmc_summary.py stats  <kernel_stats.csv> <out.json>
  python tools/pmc_summary.py traffic <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
  python tools/pmc_summary.py variants <kernel_stats.csv> <fetch.csv> <write.csv> <regex> <out.json>

`traffic` follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are
collected in separate --pmc passes (kB units), FETCH_SIZE is doubled (gfx950
tallies 128-B requests at 64 B for wide 16-B/lane loads, which is what every
kernel here issues), and the result is reported per launch, per kernel family.
Infinity-Cache hits are counted by these counters, not excluded.
"""
import csv
import json
import re
import sys
from collections import defaultdict

FAMILY = [  # (regex on the demangled kernel name, family as named by the library's profiler)
    (r"k_hs_cross_seg", "hs_cross_row"), (r"k_hs_side_row", "hs_side_row"),
    (r"k_feat<\w+, \d+, 1\b", "feat_hv"), (r"k_feat<\w+, \d+, 0\b", "feat_grad"),
    (r"k_feat<\w+, \d+, 2\b", "csc_scatter"), (r"k_fin<\w+, \d+, 0\b", "grad_fin"),
    (r"k_fin<\w+, \d+, 1\b", "hv_fin"), (r"k_gd_cross_seg", "gd_cross_row"), (r"k_gd_side_seg", "gd_side_row"),
    (r"k_update_cross_seg", "update_cross_row"), (r"k_update_side_row", "update_side_row"),
    (r"k_gather_pos", "refresh_base"), (r"k_gram_part", "aggregates"), (r"k_reduce_parts", "aggr_reduce"),
    (r"k_gram_mfma32|k_gram_mfma64|k_gram_mfma_f64", "aggregates"), (r"k_rows_T", "rows_T"), (r"k_vec_sum", "bias_sum"), (r"k_pos_gram32|k_gram_rows", "aggregates"),
    (r"k_hs_cross_rc", "hs_cross_row"), (r"k_col_gram", "col_gram"), (r"k_hv_cgram", "hv_cgram"),
    (r"k_apply", "apply_step"), (r"k_rowdot_multi", "rowdot_multi"), (r"k_colsum_multi", "aggregates"),
    (r"k_cg_step", "cg_step"), (r"k_cg_r2", "cg_r2"), (r"k_hot_gram|k_gram_add_tau|k_hot_slot_sum", "ccg_build"),
    (r"k_hot_seg", "hot_seg"), (r"k_mask_rows", "mask_rows"), (r"k_sgd<", "k_sgd"), (r"k_phi<", "k_phi"),
    (r"k_feat_col<\w+, \d+, 1\b", "feat_hv"), (r"k_feat_col<\w+, \d+, 0\b", "feat_grad"),
    (r"k_feat_col<\w+, \d+, 2\b", "csc_scatter"), (r"k_cg_cgram", "cg_cgram"), (r"k_pg_step", "pg_step"),
]


def family(name):
    for key, fam in FAMILY:
        if re.search(key, name):
            return fam
    return re.sub(r"\(.*", "", name)


def stats(path, out):
    res = {}
    for r in csv.DictReader(open(path)):
        fam = family(r["Name"])
        d = res.setdefault(fam, dict(calls=0, total_ns=0))
        d["calls"] += int(r["Calls"])
        d["total_ns"] += int(r["TotalDurationNs"])
    for d in res.values():
        d["avg_us"] = d["total_ns"] / max(1, d["calls"]) / 1e3
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["total_ns"]):
        print(f"{k:20s} calls {v['calls']:6d} avg {v['avg_us']:9.1f} us total {v['total_ns']/1e6:9.3f} ms")


def _per_dispatch(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        vals[family(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def traffic(fetch_csv, write_csv, out):
    f = _per_dispatch(fetch_csv, "FETCH_SIZE")
    w = _per_dispatch(write_csv, "WRITE_SIZE")
    res = {}
    for fam in set(f) | set(w):
        fb = 2.0 * 1024 * sum(f.get(fam, [])) / max(1, len(f.get(fam, [])))
        wb = 1024 * sum(w.get(fam, [])) / max(1, len(w.get(fam, [])))
        res[fam] = {"bytes_per_launch": fb + wb, "fetch_bytes_x2": fb, "write_bytes": wb,
                    "launches": max(len(f.get(fam, [])), len(w.get(fam, [])))}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["bytes_per_launch"]):
        print(f"{k:20s} {v['bytes_per_launch']/1e6:10.2f} MB/launch  (fetch x2 {v['fetch_bytes_x2']/1e6:.2f}, "
              f"write {v['write_bytes']/1e6:.2f})")


def _variant(name):
    """k_gd_cross_seg<float, 32, true, 2, false>(...) -> 'k_gd_cross_seg<float, 32, true, 2, false>'."""
    m = re.search(r"(k_\w+<[^()]*>)", name)
    return m.group(1) if m else re.sub(r"\(.*", "", name)


def variants(stats_csv, fetch_csv, write_csv, regex, out):
    """Per template instantiation (not per family) of the kernels matching
    regex: calls, average duration (kernel trace) and FETCH_SIZE x2 +
    WRITE_SIZE per launch (separate --pmc passes)."""
    res = {}
    for r in csv.DictReader(open(stats_csv)):
        if not re.search(regex, r["Name"]):
            continue
        d = res.setdefault(_variant(r["Name"]), dict(calls=0, total_ns=0))
        d["calls"] += int(r["Calls"])
        d["total_ns"] += int(r["TotalDurationNs"])
    for path, counter, key, mul in ((fetch_csv, "FETCH_SIZE", "fetch_bytes_x2", 2.0), (write_csv, "WRITE_SIZE",
                                                                                         "write_bytes", 1.0)):
        vals = defaultdict(list)
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") == counter and re.search(regex, r["Kernel_Name"]):
                vals[_variant(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for v, xs in vals.items():
            res.setdefault(v, dict(calls=0, total_ns=0))[key] = mul * 1024 * sum(xs) / len(xs)
    for v, d in res.items():
        d["avg_us"] = d["total_ns"] / max(1, d["calls"]) / 1e3
        d["bytes_per_launch"] = d.get("fetch_bytes_x2", 0.0) + d.get("write_bytes", 0.0)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["total_ns"]):
        print(f"{k:60s} calls {v['calls']:5d} avg {v['avg_us']:8.1f} us  PMC {v['bytes_per_launch'] / 1e6:8.1f} MB/launch")


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "variants":
        variants(*sys.argv[2:7])
    else:
        traffic(sys.argv[2], sys.argv[3], sys.argv[4])
