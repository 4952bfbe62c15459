"""Per-step kernel summary of the REPLAYED steps of a rocprofv3 --kernel-trace run of bench.py (VERDICT
r4 "what's weak" 8: a summary that divides the whole run's kernel time by a guessed step count mixes in
eager warm-up, capture and GEMM-timing steps). The steps are the spans between successive optimizer
launches (adam_rec_k / adam_gated_k); the last `n` of them are the timed replays. Prints the mean span,
busy and idle time per step, and every kernel's time and calls per step.
usage: python tools/replay_summary.py <trace dir> <n replayed steps> [top] [bench ms_per_step]"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_groups import dispatches  # noqa: E402


def step_spans(ks):
    ad = [i for i, k in enumerate(ks) if "adam_rec_k" in k[0] or "adam_gated_k" in k[0]]
    ad = [a for n, a in enumerate(ad) if n == 0 or a - ad[n - 1] > 4]
    return [(ad[j] + 1, ad[j + 1] + 1) for j in range(len(ad) - 1)]


def main():
    d, n = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    bench_ms = float(sys.argv[4]) if len(sys.argv) > 4 else None
    ks = sorted(dispatches(d), key=lambda r: r[3])
    spans = step_spans(ks)[-n:]
    agg, span_t, busy_t, nk = {}, 0.0, 0.0, 0
    for a, b in spans:
        step = ks[a:b]
        t0, t1 = step[0][3], max(k[3] + k[4] for k in step)
        span_t += t1 - t0
        cur = t0
        for k in step:
            s, e = k[3], k[3] + k[4]
            busy_t += max(0, e - max(s, cur))
            cur = max(cur, e)
            name = k[0].replace("(anonymous namespace)::", "")
            t, c = agg.get(name, (0, 0))
            agg[name] = (t + k[4], c + 1)
        nk += len(step)
    m = len(spans)
    tot = sum(t for t, _ in agg.values())
    print(f"{m} replayed steps: span {span_t / m / 1e6:.3f} ms/step (traced), busy {busy_t / m / 1e6:.3f}, idle "
          f"{(span_t - busy_t) / m / 1e6:.3f}, kernel sum {tot / m / 1e6:.3f} ms/step (> span where the side "
          f"stream overlaps), {nk / m:.0f} kernels/step"
          + (f"; untraced bench ms_per_step {bench_ms:.3f}" if bench_ms else ""))
    torch_t = sum(t for name, (t, _) in agg.items() if "at::native" in name or "rocclr" in name)
    print(f"torch / runtime kernels: {torch_t / m / 1e3:.1f} us/step")
    for name, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
        print(f"{t / m / 1e3:9.1f} us/step {c / m:6.1f} calls/step {t / c / 1e3:8.1f} us avg {100 * t / tot:5.1f}%  "
              f"{name[:100]}")


if __name__ == "__main__":
    main()
