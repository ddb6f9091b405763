"""Per-kernel PMC summary of the device-inflate ingest (one C2 file list
through gg_precluster_files, one lane) -> profiles/r06/ingest_pmc.json.

Input: the directory scripts/ingest_pmc.sh wrote, one rocprofv3 run per
pass over `scripts/inflate_probe.py 1000 1` (a warm-up call and a timed one:
every value below is per call, the two calls' dispatches summed and halved):
p1 SQ instruction counters, p2 FETCH_SIZE, p3 WRITE_SIZE.

Per kernel class (cycles = GRBM_GUI_ACTIVE / 8, the per-XCD busy cycles):
  ms_per_call      dispatch time (rocprofv3 timestamps of pass 1)
  valu_frac_guide  VALU wave-instructions / (1024 SIMDs x cycles / 2): the
                   share of the issue slots at MI355X_MICROARCH.md's 2 cycles
                   per wave64 VALU instruction
  valu_per_wave, salu_per_wave, waves, wait_frac (SQ_WAIT_INST_ANY /
                   SQ_WAVE_CYCLES: the share of wave time waiting on a
                   dependency), lds_conflict_per_instr
  hbm_bytes        FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024 (the guide's
                   HBM section: gfx950 FETCH_SIZE counts half of a wide read)
  hbm_frac         hbm_bytes / time against 8 TB/s

Usage: python scripts/ingest_pmc_model.py <pmc-dir> [--out=file]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import k2_pmc_model as km  # noqa: E402

CLASSES = (("slot_upload", "upload"), ("inflate_search", "search"), ("inflate_decode_kernel<true>", "decode_staged"),
           ("inflate_decode_kernel<false>", "decode_global"), ("inflate_expand", "expand"),
           ("inflate_resolve", "resolve"), ("inflate_crc", "crc"), ("parse_", "parse"),
           ("sketch_candidates", "k1"), ("sketch_finalize", "k1_finalize"))
CALLS = 2


def short(name):
    for key, cls in CLASSES:
        if key in name:
            return cls
    return "other: " + name[:40]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--out")]
    out_path = os.path.join(km.ROOT, "profiles", "r06", "ingest_pmc.json")
    for a in sys.argv[1:]:
        if a.startswith("--out="):
            out_path = a.split("=", 1)[1]
    km.short = short
    per = km.load(args[0])
    ks = km.summarise(per)
    res = {"note": __doc__.split("\n\n")[1].replace("\n", " "), "source": os.path.relpath(args[0], km.ROOT),
           "calls": CALLS, "kernels": {}}
    for k, e in ks.items():
        c1 = per[k]["p1"]["counters"]
        waves = c1.get("SQ_WAVES", 0.0)
        x = {"dispatches_per_call": e["dispatches"] / CALLS, "ms_per_call": e["ms"] / CALLS,
             "valu_frac_guide": e.get("valu_frac_guide", 0.0), "waves_per_call": waves / CALLS,
             "valu_per_wave": c1.get("SQ_INSTS_VALU", 0.0) / waves if waves else 0.0,
             "salu_per_wave": c1.get("SQ_INSTS_SALU", 0.0) / waves if waves else 0.0,
             "lds_per_wave": c1.get("SQ_INSTS_LDS", 0.0) / waves if waves else 0.0,
             "wait_frac": (c1.get("SQ_WAIT_INST_ANY", 0.0) / c1["SQ_WAVE_CYCLES"]) if c1.get("SQ_WAVE_CYCLES") else 0.0,
             "lds_conflict_per_instr": e.get("lds_conflict_per_instr", 0.0)}
        if "hbm_bytes" in e:
            x["hbm_bytes_per_call"] = e["hbm_bytes"] / CALLS
            x["hbm_GBps"] = e["hbm_GBps"]
            x["hbm_frac"] = e["hbm_frac"]
        fr = {"valu": x["valu_frac_guide"], "hbm": x.get("hbm_frac", 0.0)}
        x["bound"] = max(fr, key=fr.get)
        x["bound_frac"] = fr[x["bound"]]
        res["kernels"][k] = {a: (round(v, 6) if isinstance(v, float) else v) for a, v in x.items()}
    ing = [e for k, e in res["kernels"].items() if not k.startswith("other") and not k.startswith("k1")]
    res["ingest_ms_per_call"] = round(sum(e["ms_per_call"] for e in ing), 4)
    res["ingest_hbm_bytes_per_call"] = round(sum(e.get("hbm_bytes_per_call", 0.0) for e in ing))
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print("ingest kernels %.2f ms per call, %.2f GB HBM" % (res["ingest_ms_per_call"], res["ingest_hbm_bytes_per_call"] / 1e9))
    for k, e in sorted(res["kernels"].items(), key=lambda kv: -kv[1]["ms_per_call"]):
        print("  %-15s %6.1f disp  %8.3f ms  valu %.3f  wait %.2f  VALU/wave %8.0f  hbm %.3f (%.0f GB/s)"
              % (k, e["dispatches_per_call"], e["ms_per_call"], e["valu_frac_guide"], e["wait_frac"],
                 e["valu_per_wave"], e.get("hbm_frac", 0), e.get("hbm_GBps", 0)))


if __name__ == "__main__":
    main()
