"""GPU idle time inside device-inflate calls with the default lanes: the
kernel trace (rocprofv3 --kernel-trace of scripts/inflate_probe.py N 2, two
lanes) split into calls by gaps of > 20 ms, and per call the wall span
of its kernels and the time no kernel ran (host-side waits of both lanes).
usage: python scripts/lane_gaps.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows)
calls, cur = [], [iv[0]]
for x in iv[1:]:
    if x[0] - max(e for _, e, _ in cur) > 20_000_000:
        calls.append(cur)
        cur = [x]
    else:
        cur.append(x)
calls.append(cur)
for c in calls:
    t0, t1 = c[0][0], max(e for _, e, _ in c)
    busy, end = 0, t0
    for s, e, _ in c:
        if e <= end:
            continue
        busy += e - max(s, end)
        end = e
    print("call: span %.2f ms, kernels busy %.2f ms, idle %.2f ms, %d kernels" % ((t1 - t0) / 1e6, busy / 1e6,
                                                                                  (t1 - t0 - busy) / 1e6, len(c)))
