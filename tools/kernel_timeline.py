"""Per-kernel totals and a start/end timeline (ms from the first kernel) from a rocprofv3
--kernel-trace CSV: python3 tools/kernel_timeline.py <run_kernel_trace.csv> [min_ms]."""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
           r.get("Queue_Id", "")) for r in rows]
    ks.sort()
    t0 = ks[0][0]
    tot, cnt = defaultdict(float), defaultdict(int)
    for s, e, n, _ in ks:
        tot[n] += (e - s) / 1e6
        cnt[n] += 1
    for n in sorted(tot, key=lambda k: -tot[k]):
        print(f"{n[:40]:40s} {tot[n]:9.2f} ms  x{cnt[n]}")
    print(f"--- timeline (ms from first), kernels >= {min_ms:g} ms")
    for s, e, n, q in ks:
        if (e - s) / 1e6 >= min_ms:
            print(f"{(s - t0) / 1e6:8.1f} {(e - t0) / 1e6:8.1f} {(e - s) / 1e6:7.1f} q{q} {n[:40]}")
    print(f"span {(max(e for _, e, _, _ in ks) - t0) / 1e6:.6f}")


if __name__ == "__main__":
    main()
