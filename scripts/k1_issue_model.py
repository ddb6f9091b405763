"""K1's VALU-issue ceiling at HEAD -> profiles/r04_k1_issue_model.json.

Inputs (all measured on the MI355X, committed under profiles/):
  * a rocprofv3 --pmc pass over one K1 launch at C3 (scripts/pmc_head.sh):
    SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU2, GRBM_GUI_ACTIVE, FETCH_SIZE, ...
  * the issue cost of each instruction class from scripts/ubench_dual.hip's
    PMC pass (cycles per wave64 instruction per SIMD at the effective clock,
    GRBM_GUI_ACTIVE / 8, 8 waves per SIMD, independent chains):
      dual ~2.3 (pairs co-issue), full ~4.2, wide (64-bit) ~5.0
  * K1's machine code in the library (scripts/k1_isa.py): the share of each
    class among the VALU instructions of its hot path (one segment of the
    unrolled hashing loop with no candidate branch taken, k1_isa.hot_path;
    the whole-kernel static shares are recorded beside it).

floor (cycles per wave of 64 k-mers) = VALU per wave-k-mer (PMC) x
    sum_class share_class x cost_class
peak (Gkmer/s) = 1024 SIMDs x 2.4 GHz x 64 / floor
The floor is a lower bound on issue time: it assumes every dual-class
instruction finds a partner and nothing else stalls.

Usage: python scripts/k1_issue_model.py <pmc-dir> [out.json]
"""
import csv
import glob
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import k1_isa  # noqa: E402

# ubench_dual variants by class (scripts/ubench_dual.hip numbering)
DUAL_V = [0, 2, 3, 4, 5, 7, 9, 13, 17, 18]
FULL_V = [10, 11, 12, 14, 15, 16, 31, 32]
WIDE_V = [20, 21, 22, 23]
C3_KMERS = 10000 * (3000000 - 21 + 1)


def counters(pmc_dir, regex):
    """{counter: value} of the first dispatch whose kernel name contains regex, over every CSV in pmc_dir."""
    out, dur = {}, None
    for f in sorted(glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)):
        first = None
        for r in csv.DictReader(open(f)):
            if regex not in r["Kernel_Name"]:
                continue
            if first is None:
                first = r["Dispatch_Id"]
            if r["Dispatch_Id"] != first:
                continue
            out[r["Counter_Name"]] = float(r["Counter_Value"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return out, dur


def class_costs(ubench_csv):
    by = {}
    for r in csv.DictReader(open(ubench_csv)):
        v = int(r["Kernel_Name"].split("<")[1].split(">")[0])
        by.setdefault((v, r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    cyc = {}
    for (v, _d), c in by.items():
        if "GRBM_GUI_ACTIVE" in c and "SQ_INSTS_VALU" in c:
            cyc.setdefault(v, []).append((c["GRBM_GUI_ACTIVE"] / 8) / (c["SQ_INSTS_VALU"] / 1024))
    med = {v: statistics.median(x) for v, x in cyc.items()}
    return {"dual": statistics.median(med[v] for v in DUAL_V), "full": statistics.median(med[v] for v in FULL_V),
            "wide": statistics.median(med[v] for v in WIDE_V)}


def main():
    pmc_dir = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r04_k1_issue_model.json")
    lib = os.path.join(ROOT, "galah_amd", "lib", "libgalahgpu.so")
    c, dur = counters(pmc_dir, "sketch_candidates_kernel<21")
    costs = class_costs(os.path.join(ROOT, "profiles", "ubench", "r02_pmc_ubench_dual.csv"))
    listing = k1_isa.kernel_listing(lib)
    hs = k1_isa.histogram(listing)
    h = k1_isa.histogram(k1_isa.hot_path(k1_isa.kernel_listing(lib, with_addr=True)))
    nv = h["dual"] + h["full"] + h["wide"]
    share = {k: h[k] / nv for k in ("dual", "full", "wide")}
    nvs = hs["dual"] + hs["full"] + hs["wide"]
    share_static = {k: hs[k] / nvs for k in ("dual", "full", "wide")}
    waves = C3_KMERS / 64.0
    valu = c["SQ_INSTS_VALU"] / waves
    per_instr = sum(share[k] * costs[k] for k in share)
    floor = valu * per_instr
    cyc_simd = c["GRBM_GUI_ACTIVE"] / 8
    measured = cyc_simd * 1024 / waves
    peak = 1024 * 2.4e9 * 64 / floor / 1e9
    model = {
        "note": ("floor = %.2f VALU per wave-k-mer (PMC, C3 launch) x %.3f cycles (hot-path class shares dual %.3f / "
                 "full %.3f / wide %.3f at %.2f / %.2f / %.2f cycles, ubench_dual PMC) = %.1f cycles; peak = 1024 "
                 "SIMDs x 2.4 GHz x 64 / floor" % (valu, per_instr, share["dual"], share["full"], share["wide"],
                                                   costs["dual"], costs["full"], costs["wide"], floor)),
        "k1_fingerprint": k1_isa.fingerprint(listing),
        "valu_per_wave_kmer": valu,
        "class_share_hot_path": share,
        "hot_path_valu_per_kmer": nv / 44.0,
        "class_share_static": share_static,
        "class_cost_cycles": costs,
        "floor_cycles_per_wave_kmer": floor,
        "peak_gkmer_per_s": peak,
        "pmc_launch_s": dur,
        "pmc_cycles_per_wave_kmer": measured,
        "pmc_effective_clock_ghz": cyc_simd / dur / 1e9 if dur else None,
        "pmc_issue_frac": floor / measured,
        "valu2_share": c.get("SQ_ACTIVE_INST_VALU2", 0.0) / c["SQ_INSTS_VALU"],
        "lds_bank_conflict_per_lds_instr": (c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_INSTS_LDS"]
                                            if c.get("SQ_INSTS_LDS") else None),
        "hbm_bytes_per_kmer_pmc": (c["FETCH_SIZE"] * 1024 / C3_KMERS) if "FETCH_SIZE" in c else None,
        "counters": c,
    }
    with open(out, "w") as f:
        json.dump(model, f, indent=1)
    print(json.dumps({k: v for k, v in model.items() if k != "counters"}, indent=1))


if __name__ == "__main__":
    main()
