"""bench.py's files leg alone in a fresh process (no headline context, no
CPU-baseline threads before it): the same function, data and timing.
usage: python scripts/files_leg_fresh.py > out.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [os.path.join(ROOT, "bench.py")]
import bench  # noqa: E402

a = bench.parse()
files, plain = bench.files_leg(a, 0, 9)
files.pop("roofline_ingest", None)
print(json.dumps({"files": files, "files_plain": plain}))
