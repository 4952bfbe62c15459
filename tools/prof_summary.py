"""Summarise a rocprofv3 --kernel-trace --stats run: top kernels by total time.
usage: python tools/prof_summary.py <dir with *kernel_stats.csv or *.db> [steps] [top]"""
import csv
import glob
import sqlite3
import sys


def rows_from(d):
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
    if f:
        return [(r['Name'], int(r['Calls']), float(r['TotalDurationNs']), float(r['AverageNs']))
                for r in csv.DictReader(open(f[0]))]
    db = glob.glob(f"{d}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    # top_kernels durations are in microseconds
    return [(n, int(k), float(t) * 1e3, float(a) * 1e3)
            for n, k, t, a, _ in c.execute("select * from top_kernels")]


def main():
    d = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = rows_from(d)
    tot = sum(r[2] for r in rows)
    print(f"total kernel time {tot/1e6:.2f} ms ({tot/1e6/steps:.2f} ms per step over {steps:g} steps)")
    for name, calls, total, avg in sorted(rows, key=lambda r: -r[2])[:top]:
        name = name.replace('(anonymous namespace)::', '')
        print(f"{total/1e6/steps:8.3f} ms/step {calls/steps:7.1f} calls/step {avg/1e3:8.1f} us avg "
              f"{100*total/tot:5.1f}%  {name[:100]}")


if __name__ == "__main__":
    main()
