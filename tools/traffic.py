"""HBM traffic of the GEMM family from two rocprofv3 --pmc passes over bench.py (FETCH_SIZE, then
WRITE_SIZE; gfx950 correction per MI355X_MICROARCH.md 'HBM': FETCH_SIZE counts half the bytes of wide
16-B/lane reads, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores). Both counters are in KB.
Writes <out.json> with mean bytes per GEMM launch, used by bench.py's roofline "traffic" field.
usage: python tools/traffic.py <fetch.db> <write.db> <out.json>"""
import json
import sqlite3
import sys


def per_kernel(db, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, sum(value) from counters_collection "
                     "where counter_name = ? group by dispatch_id", (counter,)).fetchall()
    return rows


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    # our GEMM kernels
    isg = lambda n: ("gemm16_kernel<" in n or "gemm_kernel<" in n or "gemm16_pp_kernel<" in n or "gemm16_pn_kernel<" in n
                     or n.startswith("Cijk_"))
    f = [v for _, n, v in fetch if isg(n)]
    w = [v for _, n, v in write if isg(n)]
    fb = 2.0 * 1024.0 * sum(f) / max(len(f), 1)
    wb = 1024.0 * sum(w) / max(len(w), 1)
    out = {"kernel": "b2p_gemm (all GEMM launches of bench.py steps)", "launches_fetch": len(f),
           "launches_write": len(w), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
           "traffic_bytes_per_launch": fb + wb,
           "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 wide-read correction) + --pmc WRITE_SIZE, separate passes"
                     + ("; side-stream work serialised (B2P_SERIAL_SIDE=1)" if __import__("os").environ.get("B2P_SERIAL_SIDE") == "1" else "")}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
