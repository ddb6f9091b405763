"""Per-kernel PMC summary of K2 (the bucketed inverted index and the passing
pairs' device sort) over one bench step -> profiles/r05_k2_pmc.json.

Input: the directory scripts/k2_pmc.sh wrote for one config, one rocprofv3
run per pass over `bench.py --steps 1 --warmup 0`: p1 SQ instruction and LDS
counters, p2 FETCH_SIZE, p3 WRITE_SIZE, p4 TCC_HIT/MISS.

Per kernel (the dispatches of one pass summed; cycles = GRBM_GUI_ACTIVE / 8,
the per-XCD busy cycles):
  ms              kernel time of the pass (rocprofv3 dispatch timestamps)
  valu_ipc        VALU wave-instructions per SIMD-cycle (1024 SIMDs)
  valu_frac_guide valu_ipc x 2: the share of a SIMD's issue slots at the
                  guide's 2 cycles per wave64 VALU instruction
  lds_util        SQ_LDS_IDX_ACTIVE / (256 CUs x cycles): LDS-array busy share
  lds_conflict_per_instr  SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS
  fetch_bytes     FETCH_SIZE x 1024 x 2 (KB; MI355X_MICROARCH.md HBM section:
                  gfx950 FETCH_SIZE reports half the bytes of a wide read)
  write_bytes     WRITE_SIZE x 1024
  hbm_GBps        (fetch + write) / time, and hbm_frac against 8 TB/s
  l2_hit          TCC_HIT / (TCC_HIT + TCC_MISS)

Usage: python scripts/k2_pmc_model.py <config>=<pmc-dir> [...] [--out=file]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_SIMD, N_CU = 1024, 256
HBM_PEAK = 8.0e12
NAMES = ("index_scan", "bucket_hist", "bucket_base", "index_fill_range", "index_fill", "bucket_bounds", "split_keys",
         "split_scatter", "superbin_count", "superbin_place",
         "index_bucket", "index_pairs", "index_runs", "index_mixed", "pair_keys", "pair_gather", "bloom_build")


def short(name):
    for k in NAMES:
        if k + "_kernel" in name:
            return k
    if "ROCPRIM_400200" in name:  # the library's rocPRIM (ROCm 7.2); torch's is ROCPRIM_400001
        if "onesweep" in name and "unsigned short" in name:
            return "index_sort"  # the bucketed build's 16-bit key sort (histogram, scan, 2 passes)
        if "onesweep" in name:
            return "index_sort_full"  # the full build's 32-bit sort (fallback)
        if "scan" in name and "unsigned int" in name:
            return "split_scan"  # the split build's scan of the per-row super-bin counts (u32)
        if "scan" in name:
            return "not_k2: u64 scan (K1 run index)"
        return "pair_sort"  # the passing pairs' sort (merge-sort path below 2^20 items)
    return "not_k2: " + name[:40]  # torch kernels of bench.py's own analysis (torch.unique)


def load(pdir):
    per = {}
    for f in sorted(glob.glob(os.path.join(pdir, "p*", "*counter_collection.csv"))):
        pas = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            d = per.setdefault(k, {}).setdefault(pas, {"counters": {}, "dispatch_s": {}, "names": set()})
            c = d["counters"]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["dispatch_s"][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            d["names"].add(r["Kernel_Name"][:120])
    return per


def summarise(per):
    out = {}
    empty = {"counters": {}, "dispatch_s": {}, "names": set()}
    for k, passes in per.items():
        p1 = passes.get("p1", empty)
        c1 = p1["counters"]
        t = sum(p1["dispatch_s"].values())
        cyc = c1.get("GRBM_GUI_ACTIVE", 0.0) / 8
        e = {"dispatches": len(p1["dispatch_s"]), "ms": t * 1e3, "valu_instr": c1.get("SQ_INSTS_VALU", 0.0),
             "kernel_names": sorted(set().union(*[p["names"] for p in passes.values()]))[:3]}
        if cyc > 0 and t > 0:
            e["effective_clock_ghz"] = cyc / t / 1e9
            e["valu_ipc"] = e["valu_instr"] / (N_SIMD * cyc)
            e["valu_frac_guide"] = e["valu_ipc"] * 2.0
            e["lds_util"] = c1.get("SQ_LDS_IDX_ACTIVE", 0.0) / (N_CU * cyc)
            e["lds_conflict_per_instr"] = (c1.get("SQ_LDS_BANK_CONFLICT", 0.0) / c1["SQ_INSTS_LDS"]
                                           if c1.get("SQ_INSTS_LDS") else 0.0)
        p2, p3, p4 = passes.get("p2", empty), passes.get("p3", empty), passes.get("p4", empty)
        fb = p2["counters"].get("FETCH_SIZE")
        wb = p3["counters"].get("WRITE_SIZE")
        if fb is not None:
            e["fetch_bytes"] = fb * 1024 * 2
            e["fetch_ms"] = sum(p2["dispatch_s"].values()) * 1e3
        if wb is not None:
            e["write_bytes"] = wb * 1024
            e["write_ms"] = sum(p3["dispatch_s"].values()) * 1e3
        if fb is not None and wb is not None and t > 0:
            e["hbm_bytes"] = e["fetch_bytes"] + e["write_bytes"]
            e["hbm_GBps"] = e["hbm_bytes"] / t / 1e9
            e["hbm_frac"] = e["hbm_GBps"] * 1e9 / HBM_PEAK
        h, m = p4["counters"].get("TCC_HIT_sum"), p4["counters"].get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            e["l2_hit"] = h / (h + m)
        fr = {"valu": e.get("valu_frac_guide", 0.0), "lds": e.get("lds_util", 0.0), "hbm": e.get("hbm_frac", 0.0)}
        e["bound"] = max(fr, key=fr.get)
        e["bound_frac"] = fr[e["bound"]]
        out[k] = {x: (round(v, 6) if isinstance(v, float) else v) for x, v in e.items()}
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--out")]
    out_path = os.path.join(ROOT, "profiles", "r05_k2_pmc.json")
    for a in sys.argv[1:]:
        if a.startswith("--out="):
            out_path = a.split("=", 1)[1]
    res = {"note": __doc__.split("\n\n")[1].replace("\n", " ")}
    for a in args:
        cfg, pdir = a.split("=", 1)
        res[cfg] = {"source": os.path.relpath(pdir, ROOT), "kernels": summarise(load(pdir))}
        ks = res[cfg]["kernels"]
        k2 = [e for k, e in ks.items() if not k.startswith("not_k2")]
        res[cfg]["K2_total_ms"] = round(sum(e["ms"] for e in k2), 5)
        res[cfg]["K2_hbm_bytes"] = round(sum(e.get("hbm_bytes", 0.0) for e in k2))
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    for cfg in res:
        if cfg == "note":
            continue
        print(cfg, "K2 total %.3f ms, %.3f GB HBM" % (res[cfg]["K2_total_ms"], res[cfg]["K2_hbm_bytes"] / 1e9))
        for k, e in res[cfg]["kernels"].items():
            print("  %-16s %3d x %8.3f ms  valu %.2f  lds %.2f  hbm %.3f (%.0f GB/s)  l2hit %.2f -> %s"
                  % (k, e["dispatches"], e["ms"], e.get("valu_frac_guide", 0), e.get("lds_util", 0),
                     e.get("hbm_frac", 0), e.get("hbm_GBps", 0), e.get("l2_hit", 0), e["bound"]))


if __name__ == "__main__":
    main()
