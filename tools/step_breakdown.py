"""Breakdown of one step of a rocprofv3 kernel trace of bench.py, the step chosen by index among the
spans between successive adam_rec_k launches: span, busy/idle, largest gaps, per-kernel totals.
usage: python tools/step_breakdown.py <trace dir> <step index> [n_top] [--gemm]
--gemm: also every GEMM launch of the step in issue order (kernel, workgroups, duration)."""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_groups import dispatches  # noqa: E402


def main():
    d, j = sys.argv[1], int(sys.argv[2])
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ntop = int(args[2]) if len(args) > 2 else 30
    ks = sorted(dispatches(d), key=lambda r: r[3])
    ad = [i for i, k in enumerate(ks) if "adam_rec_k" in k[0] or "adam_gated_k" in k[0]]
    ad = [a for n, a in enumerate(ad) if n == 0 or a - ad[n - 1] > 4]
    a, b = ad[j] + 1, ad[j + 1] + 1
    step = ks[a:b]
    t0, t1 = step[0][3], max(k[3] + k[4] for k in step)
    busy, cur, gaps, prev = 0, t0, [], None
    for k in step:
        s, e = k[3], k[3] + k[4]
        if s > cur:
            gaps.append((s - cur, prev, k[0]))
        busy += max(0, e - max(s, cur))
        if e > cur:
            cur, prev = e, k[0]
    print(f"step {j}: span {(t1 - t0) / 1e6:.3f} ms, {len(step)} kernels, kernel sum "
          f"{sum(k[4] for k in step) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms "
          f"in {len(gaps)} gaps")
    for g, p, n in sorted(gaps, key=lambda x: -x[0])[:10]:
        print(f"  gap {g / 1e3:8.1f} us  after {str(p).replace('(anonymous namespace)::', '')[:55]}  "
              f"before {n.replace('(anonymous namespace)::', '')[:55]}")
    # the torch kernels of the step with their neighbours (what launched them)
    for i, k in enumerate(step):
        if "at::native" in k[0] or "rocclr" in k[0]:
            nb = lambda x: x.replace("(anonymous namespace)::", "")[:48]
            print(f"  torch: {nb(k[0])}  after {nb(step[i - 1][0]) if i else '-'}  before "
                  f"{nb(step[i + 1][0]) if i + 1 < len(step) else '-'}")
    agg = {}
    for k in step:
        n = k[0].replace("(anonymous namespace)::", "")
        t, c = agg.get(n, (0, 0))
        agg[n] = (t + k[4], c + 1)
    tot = sum(k[4] for k in step)
    for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:ntop]:
        print(f"  {t / 1e3:8.1f} us {c:4d}x {100 * t / tot:5.1f}%  {n[:100]}")
    if "--gemm" in sys.argv:
        print("GEMM launches in issue order (start offset us, duration us, workgroups, kernel):")
        for k in step:
            if "gemm" in k[0] and "splitk" not in k[0]:
                n = k[0].replace("(anonymous namespace)::", "").split("(")[0]
                print(f"  {(k[3] - t0) / 1e3:9.1f} {k[4] / 1e3:8.1f} {k[1] // max(k[2], 1):6d}  {n[:90]}")


if __name__ == "__main__":
    main()
