"""Attribute the decode-step launch outliers beside the vocoder.

Input: a rocprofv3 --kernel-trace CSV of the bench (the vocoder of batch s runs on its own stream
beside the decode of batch s + 1). For every decode-step launch class (k_att_persist, k_ffn_persist,
k_advance, the head GEMM, ln_out) it reports the median duration alone (no vocoder kernel overlapping)
and beside the vocoder, and for the launches longer than K x the class median it names the vocoder
kernel classes whose execution overlaps them (class = kernel symbol + grid), with the excess time
(duration - median) charged to the vocoder class with the largest overlap. The longest outliers are
listed with every overlapping vocoder kernel and its own duration.
Usage: outlier_attrib.py kernel_trace.csv [K=4] [top=15]"""
import csv
import statistics
import sys
from collections import defaultdict

DECODE = ("k_att_persist", "k_ffn_persist", "k_advance", "k_gemm2", "k_ln1024", "k_ln_mix")
CODEC = ("k_conv", "k_dw_ln", "k_gemv", "k_fvq", "k_fsq", "k_f32_split")


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("rwkvtts::", "")
    return n[:56]


def grid(r):
    g = r.get("Grid_Size")
    if g:
        return g
    return str(int(r.get("Grid_Size_X", 1) or 1) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1))


def main():
    path = sys.argv[1]
    K = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    dec, voc = [], []
    for r in csv.DictReader(open(path)):
        n = short(r["Kernel_Name"])
        e = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, grid(r))
        if n.startswith(CODEC):
            voc.append(e)
        elif n.startswith(DECODE):
            dec.append(e)
    voc.sort()
    dec.sort()
    # vocoder intervals sorted by start; for each decode launch scan the overlapping ones
    starts = [v[0] for v in voc]
    import bisect

    def overlaps(s, e):
        out = []
        i = bisect.bisect_left(starts, e)
        j = i - 1
        while j >= 0 and len(out) < 64:
            v = voc[j]
            if v[1] > s:
                out.append(v)
            if s - v[0] > 5e7:  # 50 ms back: no vocoder kernel runs that long
                break
            j -= 1
        return out

    by_cls = defaultdict(list)
    for d in dec:
        by_cls[(d[2], d[3])].append(d)
    print(f"{len(dec)} decode-step launches, {len(voc)} vocoder launches; outliers: > {K:g} x class median")
    print(f"{'class':62s} {'n':>7s} {'med_us':>7s} {'alone':>7s} {'beside':>7s} {'mean':>7s} {'max':>9s} {'outl':>6s} {'excess_ms':>9s}")
    charge = defaultdict(lambda: [0, 0.0])
    tax = defaultdict(lambda: [0, 0.0])  # every launch beside the vocoder: duration - the class's median alone
    worst = []
    for (n, g), ds in sorted(by_cls.items(), key=lambda kv: -len(kv[1])):
        if len(ds) < 20:
            continue
        du = [(d[1] - d[0]) / 1e3 for d in ds]
        med = statistics.median(du)
        alone, beside, nout, excess = [], [], 0, 0.0
        ovs = [overlaps(d[0], d[1]) for d in ds]
        med_alone = statistics.median([t for t, ov in zip(du, ovs) if not ov] or du)
        for d, t, ov in zip(ds, du, ovs):
            (beside if ov else alone).append(t)
            if ov:
                best = max(ov, key=lambda v: min(v[1], d[1]) - max(v[0], d[0]))
                e = tax[(best[2], best[3])]
                e[0] += 1
                e[1] += t - med_alone
            if t > K * med:
                nout += 1
                excess += t - med
                if ov:
                    best = max(ov, key=lambda v: min(v[1], d[1]) - max(v[0], d[0]))
                    c = charge[(best[2], best[3])]
                    c[0] += 1
                    c[1] += t - med
                else:
                    charge[("(no vocoder kernel overlapping)", "")][0] += 1
                    charge[("(no vocoder kernel overlapping)", "")][1] += t - med
                worst.append((t, n, g, d, ov))
        fm = lambda x: f"{statistics.median(x):7.2f}" if x else "      -"
        print(f"{(n + ' g' + g)[:62]:62s} {len(ds):7d} {med:7.2f} {fm(alone)} {fm(beside)} {statistics.fmean(du):7.2f} "
              f"{max(du):9.1f} {nout:6d} {excess / 1e3:9.2f}")
    print("\nthe decode tax: every decode-step launch overlapping a vocoder kernel, its duration minus its class's "
          "median alone, charged to the vocoder class with the largest overlap:")
    tot = sum(ex for _, ex in tax.values())
    for (n, g), (c, ex) in sorted(tax.items(), key=lambda kv: -kv[1][1]):
        print(f"  {c:7d} launches {ex / 1e3:9.2f} ms ({100 * ex / max(tot, 1e-9):5.1f} %)  {(n + ' g' + g)[:70]}")
    print(f"  total {tot / 1e3:.2f} ms")
    print("\nexcess time of the outliers charged to the overlapping vocoder kernel class (largest overlap):")
    for (n, g), (c, ex) in sorted(charge.items(), key=lambda kv: -kv[1][1]):
        vd = [(v[1] - v[0]) / 1e3 for v in voc if v[2] == n and v[3] == g]
        vs = f"its launches: {len(vd)} x median {statistics.median(vd):8.1f} us" if vd else ""
        print(f"  {c:6d} outliers {ex / 1e3:9.2f} ms  {(n + ' g' + g)[:70]:70s} {vs}")
    worst.sort(key=lambda w: -w[0])
    print(f"\nthe {top} longest decode-step launches and the vocoder kernels overlapping them:")
    for t, n, g, d, ov in worst[:top]:
        print(f"  {t:9.1f} us  {n} g{g}")
        for v in sorted(ov):
            print(f"      {(v[1] - v[0]) / 1e3:9.1f} us  {v[2]} g{v[3]}  (starts {(v[0] - d[0]) / 1e3:+9.1f} us)")


if __name__ == "__main__":
    main()
