"""Per-kernel-class ms per call from scripts/ktrace_ab.sh output directories
(rocprofv3 --kernel-trace --stats; inflate_probe.py runs a warm-up call and
the timed ones: CALLS calls per run).  usage: python scripts/ktrace_sum.py DIR [CALLS]"""
import csv
import glob
import os
import sys

CLASSES = (("slot_upload", "upload"), ("inflate_search", "search"), ("inflate_decode", "decode"),
           ("inflate_expand", "expand"), ("inflate_resolve", "resolve"), ("inflate_crc", "crc"),
           ("parse_", "parse"), ("sketch_candidates", "k1"), ("sketch_finalize", "k1"))
root = sys.argv[1]
calls = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
for d in sorted(glob.glob(os.path.join(root, "*")), key=os.path.getmtime):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        continue
    ms = {}
    for r in csv.DictReader(open(f[0])):
        for key, cls in CLASSES:
            if key in r["Name"]:
                ms[cls] = ms.get(cls, 0.0) + float(r["TotalDurationNs"]) / 1e6 / calls
                break
    dev = sum(v for k, v in ms.items() if k != "upload")
    print("%-14s " % os.path.basename(d) + " ".join("%s %.2f" % (k, ms[k]) for k in sorted(ms)) + "  | device %.2f" % dev)
