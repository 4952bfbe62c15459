"""Compare the kernels of two timed regions of one kernel trace (tools/nested_probe.py conf_twice: the
same Conformer step run twice in one process). The two regions are the two longest runs of grumc_fwd
launches' neighbourhood: split at the largest idle gap between dispatches. Prints per-kernel mean
durations and counts in each half, the largest differences first.
usage: python tools/two_run_compare.py <trace dir> [top]"""
import collections
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_groups import dispatches  # noqa: E402


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    ks = sorted(dispatches(d), key=lambda r: r[3])
    gaps = [(ks[i + 1][3] - (ks[i][3] + ks[i][4]), i) for i in range(len(ks) - 1)]
    g, cut = max(gaps)
    halves = [ks[:cut + 1], ks[cut + 1:]]
    print(f"split at the largest gap ({g / 1e6:.1f} ms): {len(halves[0])} / {len(halves[1])} dispatches")
    stats = []
    for h in halves:
        s = collections.defaultdict(list)
        for name, _, _, _, dur in h:
            s[name.replace("(anonymous namespace)::", "")[:80]].append(dur / 1e3)
        span = (h[-1][3] + h[-1][4] - h[0][3]) / 1e6
        stats.append((s, span, sum(x[4] for x in h) / 1e6))
    for i, (s, span, tot) in enumerate(stats):
        print(f"half {i}: span {span:.1f} ms, kernel sum {tot:.1f} ms")
    names = set(stats[0][0]) | set(stats[1][0])
    rows = []
    for n in names:
        a, b = stats[0][0].get(n, []), stats[1][0].get(n, [])
        ta, tb = sum(a), sum(b)
        rows.append((tb - ta, n, len(a), ta / max(len(a), 1), len(b), tb / max(len(b), 1), ta, tb))
    for diff, n, ca, ma, cb, mb, ta, tb in sorted(rows, key=lambda r: -abs(r[0]))[:top]:
        print(f"{diff / 1e3:+9.2f} ms  first {ca:5d} x {ma:8.1f} us = {ta / 1e3:8.2f} ms   second {cb:5d} x {mb:8.1f} us "
              f"= {tb / 1e3:8.2f} ms  {n}")


if __name__ == "__main__":
    main()
