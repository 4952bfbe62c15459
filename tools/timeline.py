"""Per-step timeline of a rocprofv3 kernel trace of bench.py: the span of the last complete step
(between two Adam launches), busy time (union of kernel intervals over all streams), the idle gaps
(no kernel running anywhere) and the largest gaps with the kernels around them.
usage: python tools/timeline.py <dir with the trace .db or *kernel_trace.csv> [marker-substring] [steps back]"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_groups import dispatches  # noqa: E402


def main():
    d = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "adam"
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 1   # which step, counted from the last
    ks = sorted(dispatches(d), key=lambda r: r[3])
    marks = [i for i, k in enumerate(ks) if marker in k[0]]
    # one multi-tensor Adam launch (or a few) per step: step boundaries = first marker of each run
    firsts = [m for j, m in enumerate(marks) if j == 0 or m != marks[j - 1] + 1]
    if len(firsts) < 3:
        print("not enough steps in the trace")
        return
    a, b = firsts[-1 - back] + 1, firsts[-back] + 1   # a complete step: after one Adam run up to the next
    while b < len(ks) and marker in ks[b][0]:
        b += 1
    step = ks[a:b]
    t0 = step[0][3]
    t1 = max(k[3] + k[4] for k in step)
    busy, gaps, cur_end, prev = 0, [], t0, None
    for k in step:
        s, e = k[3], k[3] + k[4]
        if s > cur_end:
            gaps.append((s - cur_end, prev, k[0]))
            busy += 0
        busy += max(0, e - max(s, cur_end))
        if e > cur_end:
            cur_end, prev = e, k[0]
    span = t1 - t0
    ksum = sum(k[4] for k in step)
    print(f"step span {span / 1e6:.3f} ms, {len(step)} kernels, kernel-time sum {ksum / 1e6:.3f} ms, "
          f"busy (union) {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms in {len(gaps)} gaps")
    for g, p, n in sorted(gaps, key=lambda x: -x[0])[:8]:
        print(f"  gap {g / 1e3:8.1f} us  after {str(p)[:60]}  before {n[:60]}")
    agg = {}
    for k in step:
        n = k[0].replace("(anonymous namespace)::", "")
        t, c = agg.get(n, (0, 0))
        agg[n] = (t + k[4], c + 1)
    print("top kernels of this step:")
    for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:28]:
        print(f"  {t / 1e3:8.1f} us {c:4d}x {100 * t / ksum:5.1f}%  {n[:100]}")


if __name__ == "__main__":
    main()
