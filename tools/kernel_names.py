"""Median duration per distinct kernel name of a rocprofv3 --kernel-trace run, full names (e.g. the
hipBLASLt / Tensile kernels torch.matmul picked on the yardstick shapes).
usage: python tools/kernel_names.py <trace dir> [name substring]"""
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_groups import dispatches  # noqa: E402


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    by = {}
    for name, gx, wx, _, dns in dispatches(d):
        if pat in name:
            by.setdefault((name, gx // max(wx, 1), wx), []).append(dns / 1e3)
    for (name, grid, wg), durs in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{statistics.median(durs):9.1f} us x{len(durs):<4d} grid {grid:6d} wg {wg:4d}  {name}")


if __name__ == "__main__":
    main()
