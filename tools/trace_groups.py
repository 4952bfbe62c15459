"""Group a rocprofv3 kernel trace into runs of consecutive dispatches of the same kernel and grid
(a microbenchmark's timed loops) and print each run's median kernel duration.
usage: python tools/trace_groups.py <dir with *kernel_trace.csv> [min_run]"""
import csv
import glob
import sqlite3
import statistics
import sys


def dispatches(d):
    """(name, grid_x, workgroup_x, start_ns, duration_ns) per dispatch, from the CSV or the rocpd db."""
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if f:
        return [(r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]), int(r["Start_Timestamp"]),
                 int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(f[0]))]
    db = glob.glob(f"{d}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    return list(c.execute("select name, grid_x, workgroup_x, start, duration from kernels"))


def main():
    d = sys.argv[1]
    min_run = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    runs = []
    for name, gx, wx, _, dns in sorted(dispatches(d), key=lambda r: r[3]):
        key = (name, gx, wx)
        dur = dns / 1e3
        if runs and runs[-1][0] == key:
            runs[-1][1].append(dur)
        else:
            runs.append((key, [dur]))
    for (name, grid, wg), durs in runs:
        if len(durs) < min_run:
            continue
        name = name.replace("(anonymous namespace)::", "")
        print(f"{statistics.median(durs):9.1f} us  x{len(durs):<4d} grid {grid // wg:6d} wg {wg:4d}  {name[:90]}")


if __name__ == "__main__":
    main()
