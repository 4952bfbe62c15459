"""Kernels of one replayed step of a rocprofv3 --kernel-trace run of bench.py, in launch order, with the
neighbours of every kernel whose name matches a pattern (to find which host op launches it).
usage: python tools/step_dump.py <trace dir> <pattern>[,<pattern>...] [context] [step index, default -1]"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from replay_summary import step_spans  # noqa: E402
from trace_groups import dispatches  # noqa: E402


def main():
    d, pats = sys.argv[1], sys.argv[2].split(",")
    ctxn = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    j = int(sys.argv[4]) if len(sys.argv) > 4 else -1
    ks = sorted(dispatches(d), key=lambda r: r[3])
    a, b = step_spans(ks)[j]
    step = ks[a:b]
    t0 = step[0][3]
    hit = [i for i, k in enumerate(step) if any(p in k[0] for p in pats)]
    show = sorted({i + o for i in hit for o in range(-ctxn, ctxn + 1) if 0 <= i + o < len(step)})
    prev = None
    for i in show:
        if prev is not None and i != prev + 1:
            print("   ...")
        k = step[i]
        name = k[0].replace("(anonymous namespace)::", "")
        print(f"{'>' if i in hit else ' '} {i:5d} {(k[3] - t0) / 1e3:9.1f} us {k[4] / 1e3:8.1f} us grid {k[1] // max(k[2], 1):6d}  {name[:100]}")
        prev = i


if __name__ == "__main__":
    main()
