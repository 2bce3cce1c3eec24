import sys, os
sys.path.insert(0, '/root/repo/one-class-ffm_amd')
import ocffm, synth
for n in (100000, 25000, 12500):
    ds = synth.kkbox(n=n)
    g = ocffm.problem_from_dataset(ds, precision=ocffm.FP32, with_test=False)
    ocffm.srand(1); g.init()
    for _ in range(3): g.one_epoch()
    g.sync(); g.reset_stats(); g.set_profiling(True)
    for _ in range(5): g.one_epoch()
    g.sync()
    ks = g.kernel_stats()
    pos = ds.n_positives
    out = []
    for k in ("gd_cross_row", "hs_cross_row", "feat_hv", "feat_grad"):
        v = ks.get(k)
        if v: out.append(f"{k} {v['total_ms']/5:.3f}ms/ep {v['total_ms']/v['launches']*1e3:.1f}us/launch")
    print(f"n={n} pos={pos} cg={g.cg_log().sum()/8:.1f}", *out, flush=True)
    g.close()
