"""Idle gaps between consecutive kernels on each queue, from a rocprofv3 --kernel-trace CSV
(--output-format csv): how much of a phase's wall time is launch boundaries rather than
kernels.  python tools/kernel_gaps.py <kernel_trace.csv> [name-substring ...]"""
import csv
import sys
from collections import defaultdict


def main(path, keys):
    rows = list(csv.DictReader(open(path)))
    q = defaultdict(list)
    for r in rows:
        qid = (r.get("Queue_Id") or r.get("Queue_ID") or "0", r.get("Stream_Id") or r.get("Stream_ID") or "0")
        q[qid].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for qid, ks in sorted(q.items()):
        ks.sort()
        busy = sum(e - s for s, e, _ in ks)
        gaps = [(ks[i + 1][0] - ks[i][1], ks[i][2], ks[i + 1][2]) for i in range(len(ks) - 1)]
        small = [g for g, _, _ in gaps if 0 <= g < 20000]   # gaps under 20 us: back-to-back launches
        print(f"queue {qid}: {len(ks)} kernels, busy {busy / 1e6:.2f} ms, "
              f"back-to-back gaps {len(small)}: median {sorted(small)[len(small) // 2] / 1e3 if small else 0:.2f} us, "
              f"sum {sum(small) / 1e6:.3f} ms")
        for k in keys:
            sel = [g for g, a, b in gaps if 0 <= g < 20000 and (k in a or k in b)]
            if sel:
                print(f"   touching '{k}': {len(sel)} gaps, median {sorted(sel)[len(sel) // 2] / 1e3:.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
