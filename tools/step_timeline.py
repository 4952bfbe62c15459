"""Timeline of one step of a rocprofv3 kernel trace of bench.py (the step chosen as in step_breakdown.py):
every kernel of at least min_us with its start offset from the step start, duration and the number of
kernels overlapping it, and the main-stream stretches where only one kernel ran (what the critical path
is made of). usage: python tools/step_timeline.py <trace dir> <step index> [min_us]"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_groups import dispatches  # noqa: E402


def main():
    d, j = sys.argv[1], int(sys.argv[2])
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    ks = sorted(dispatches(d), key=lambda r: r[3])
    ad = [i for i, k in enumerate(ks) if "adam_rec_k" in k[0] or "adam_gated_k" in k[0]]
    ad = [a for n, a in enumerate(ad) if n == 0 or a - ad[n - 1] > 4]
    step = ks[ad[j] + 1:ad[j + 1] + 1]
    t0 = step[0][3]
    t1 = max(k[3] + k[4] for k in step)
    print(f"step {j}: span {(t1 - t0) / 1e6:.3f} ms, {len(step)} kernels")
    iv = [(k[3], k[3] + k[4]) for k in step]
    solo = 0
    for i, k in enumerate(step):
        s, e = iv[i]
        over = sum(1 for a, b in iv if a < e and b > s) - 1
        if over == 0:
            solo += e - s
        if k[4] / 1e3 >= min_us:
            n = k[0].replace("(anonymous namespace)::", "")
            print(f"  {(s - t0) / 1e6:7.3f} ms  {k[4] / 1e3:8.1f} us  ov {over:2d}  grid {k[1] // max(k[2], 1):6d}  {n[:80]}")
    print(f"time with one kernel alone: {solo / 1e6:.3f} ms of {(t1 - t0) / 1e6:.3f}")


if __name__ == "__main__":
    main()
