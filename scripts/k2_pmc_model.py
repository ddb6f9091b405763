"""Per-kernel PMC summary of one bench step (K1 and the K2 kernels) ->
profiles/r02_k2_pmc.json (achieved VALU / LDS / HBM throughput
of the pair kernel against gfx950 peaks).

Input: the directory scripts/k2_pmc.sh wrote for one config (p1: SQ
instruction and LDS counters, p2: L2->fabric read requests by size, p3: write
requests, p4: FETCH_SIZE), one rocprofv3 run per pass over `bench.py
--steps 1 --warmup 0` (one launch set of every kernel).

Per kernel (dispatches of one pass summed; cycles = GRBM_GUI_ACTIVE / 8, the
per-XCD busy cycles):
  valu_ipc        VALU wave-instructions per SIMD-cycle (1024 SIMDs)
  valu_frac_full  valu_ipc x 4.21: the fraction of a SIMD's issue slots at the
                  measured cost of full-rate 32-bit ops (dual-issued simple
                  ops cost 2.30, 64-bit ops 4.99: profiles/r02_ubench_dual_8wps.txt)
  lds_util        SQ_LDS_IDX_ACTIVE / (256 CUs x cycles): LDS-array busy share
  lds_GBps        SQ_INSTS_LDS_LOAD_BANDWIDTH x 64 B / time (peak 256 B/clk/CU)
  hbm_read_GBps   128 / 64 / 32 B x TCC_EA0_RDREQ_{128B,64B,32B} / time: the
                  L2's fabric reads (calibrated: K1's 7.5 GB of packed words
                  read at C3 show as 7.9 GB); hbm_write_GBps likewise from
                  TCC_EA0_WRREQ (64 B) and the rest of WRREQ (32 B)
  bound           the largest of valu_frac_full, lds_util, hbm fraction of 8 TB/s

Usage: python scripts/k2_pmc_model.py <config>=<pmc-dir> [...] [--out file]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLK = 2.4e9
N_SIMD, N_CU = 1024, 256
FULL_COST = 4.21
HBM_PEAK = 8.0e12
LDS_PEAK = 256 * N_CU * CLK


def short(name):
    for k in ("sketch_candidates", "index_scan", "index_fill", "index_runs", "index_pairs", "pairs_gate",
              "gate_build", "gate_lo32"):
        if k in name:
            return k
    if "onesweep_iteration" in name:
        return "sort_pass"
    if "onesweep" in name:
        return "sort_histogram"
    return name[:40]


def load(pdir):
    per = {}
    for f in sorted(glob.glob(os.path.join(pdir, "p*", "*counter_collection.csv"))):
        pas = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            d = per.setdefault(k, {}).setdefault(pas, {"counters": {}, "dispatch_s": {}})
            c = d["counters"]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["dispatch_s"][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return per


def summarise(per):
    out = {}
    for k, passes in per.items():
        p1 = passes.get("p1", {"counters": {}, "dispatch_s": {}})
        c1 = p1["counters"]
        t = sum(p1["dispatch_s"].values())
        cyc = c1.get("GRBM_GUI_ACTIVE", 0.0) / 8
        rd = passes.get("p2", {"counters": {}})["counters"]
        wr = passes.get("p3", {"counters": {}})["counters"]
        n128, n64, n32 = rd.get("TCC_EA0_RDREQ_128B_sum", 0.0), rd.get("TCC_EA0_RDREQ_64B_sum", 0.0), \
            rd.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        rbytes = 128 * n128 + 64 * n64 + 32 * n32
        w64 = wr.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        wbytes = 64 * w64 + 32 * max(0.0, wr.get("TCC_EA0_WRREQ_sum", 0.0) - w64)
        e = {"dispatches": len(p1["dispatch_s"]), "ms": t * 1e3, "valu_instr": c1.get("SQ_INSTS_VALU", 0.0)}
        if cyc > 0 and t > 0:
            e["effective_clock_ghz"] = cyc / t / 1e9
            e["valu_ipc"] = e["valu_instr"] / (N_SIMD * cyc)
            e["valu_frac_full"] = e["valu_ipc"] * FULL_COST
            e["lds_util"] = c1.get("SQ_LDS_IDX_ACTIVE", 0.0) / (N_CU * cyc)
            e["lds_bank_conflict_share"] = (c1.get("SQ_LDS_BANK_CONFLICT", 0.0) / c1["SQ_LDS_IDX_ACTIVE"]
                                            if c1.get("SQ_LDS_IDX_ACTIVE") else 0.0)
            e["lds_GBps"] = c1.get("SQ_INSTS_LDS_LOAD_BANDWIDTH", 0.0) * 64 / t / 1e9
            e["lds_frac_of_peak_bytes"] = e["lds_GBps"] * 1e9 / LDS_PEAK
        tr = sum(passes.get(p, {"dispatch_s": {}})["dispatch_s"].get(d, 0.0)
                 for p in ("p2",) for d in passes.get(p, {"dispatch_s": {}})["dispatch_s"])
        tw = sum(passes.get("p3", {"dispatch_s": {}})["dispatch_s"].values())
        e["hbm_read_bytes"] = rbytes
        e["hbm_write_bytes"] = wbytes
        if tr > 0:
            e["hbm_read_GBps"] = rbytes / tr / 1e9
        if tw > 0:
            e["hbm_write_GBps"] = wbytes / tw / 1e9
        if tr > 0 and tw > 0:
            e["hbm_frac"] = (rbytes / tr + wbytes / tw) / HBM_PEAK
        fr = {"valu": e.get("valu_frac_full", 0.0), "lds": e.get("lds_util", 0.0), "hbm": e.get("hbm_frac", 0.0)}
        e["bound"] = max(fr, key=fr.get)
        e["bound_frac"] = fr[e["bound"]]
        out[k] = {x: (round(v, 5) if isinstance(v, float) else v) for x, v in e.items()}
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--out")]
    out_path = os.path.join(ROOT, "profiles", "r02_k2_pmc.json")
    for a in sys.argv[1:]:
        if a.startswith("--out="):
            out_path = a.split("=", 1)[1]
    res = {"note": __doc__.split("\n\n")[1].replace("\n", " ")}
    for a in args:
        cfg, pdir = a.split("=", 1)
        res[cfg] = summarise(load(pdir))
        k2 = [k for k in res[cfg] if k != "sketch_candidates"]
        res[cfg]["K2_total_ms"] = round(sum(res[cfg][k]["ms"] for k in k2), 4)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    for cfg in res:
        if cfg == "note":
            continue
        print(cfg, "K2 total %.3f ms" % res[cfg]["K2_total_ms"])
        for k, e in res[cfg].items():
            if isinstance(e, dict):
                print("  %-18s %8.3f ms  valu %.2f  lds %.2f  hbm %.3f  rd %.0f GB/s  wr %.0f GB/s  -> %s"
                      % (k, e["ms"], e.get("valu_frac_full", 0), e.get("lds_util", 0), e.get("hbm_frac", 0),
                         e.get("hbm_read_GBps", 0), e.get("hbm_write_GBps", 0), e["bound"]))


if __name__ == "__main__":
    main()
