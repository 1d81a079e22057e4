#!/usr/bin/env python3
"""Fold a tools/profile_round.sh / profile_modes.sh output directory into committed summaries under profiles/.

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-kernel averages of the PMC passes
  profiles/pmc_traffic.json         HBM bytes per k_spectra launch, keyed "<config>_mode<m>",
                                    read by bench.py for roofline.traffic
  profiles/pmc_valu.json            k_spectra executed-work counters (VALU instructions, the FP64
                                    ADD/MUL/FMA/TRANS mix, FP64 flops, issue fraction, clock), same
                                    keys, read by bench.py for the executed roofline (roofline.achieved)

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B): on gfx950 FETCH_SIZE counts
half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact
for 16-B-per-lane stores, which is what k_spectra's slab stores are.
usage: summarize_profile.py <prof_dir> <tag> <config> <df_mode>
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    for k in ("k_spectra", "k_dndx", "k_phitab", "k_reduce", "k_prep", "k_aniso", "k_chain_pass", "k_famod_b", "k_renorm", "k_df_eval"):
        if k in name:
            return name[name.index(k):].split("(")[0]
    return name.split("(")[0][:60]


def counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    seen = set()
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Dispatch_Id"] not in seen:
            seen.add(r["Dispatch_Id"])
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return acc, dur


def build_id(d):
    """Identity of the library the profiled run loaded: bench.py prints it on stderr as 'build_id <id>' (the
    trace pass log); falls back to the in-tree library (the same file the snapshot carried)."""
    for log in (os.path.join(d, "trace.log"), os.path.join(d, "trace", "trace.log")):
        if os.path.exists(log):
            for ln in open(log, errors="replace"):
                if ln.startswith("build_id "):
                    return ln.split()[1]
    sys.path.insert(0, ROOT)
    from is3d2_amd import _lib
    return _lib.build_id()


def main():
    d, tag, config, mode = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    bid = build_id(d)
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(d, "trace", "run_kernel_stats.csv"), os.path.join(prof, "%s_kernel_stats.csv" % tag))
    out = {}
    for sub in ("pmcA", "pmcB", "pmcC", "pmcD", "pmcE", "pmcK"):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        acc, dur = counters(p)
        for k, cs in acc.items():
            e = out.setdefault(k, {})
            for c, v in cs.items():
                e[c] = sum(v) / len(v)
            e.setdefault("launches", len(dur[k]))
            e.setdefault("avg_ns_pmc_pass", sum(dur[k]) / len(dur[k]))
    for k, e in out.items():
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_per_launch"] = (2.0 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024.0
    for k, e in out.items():
        # executed-work view: the effective clock is GRBM_GUI_ACTIVE / 8 XCDs over the dispatch, and
        # SQ_ACTIVE_INST_VALU counts quad-cycles in which a wave issued VALU, summed over waves, so
        # valu_issue_frac = 4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x cycles): the share of SIMD cycles
        # the VALU pipes were issuing (MI355X_MICROARCH.md, PMC and DVFS sections)
        if "GRBM_GUI_ACTIVE" in e and "SQ_ACTIVE_INST_VALU" in e:
            cyc = e["GRBM_GUI_ACTIVE"] / 8.0
            e["clock_ghz"] = cyc / e["avg_ns_pmc_pass"]
            e["valu_issue_frac"] = 4.0 * e["SQ_ACTIVE_INST_VALU"] / (1024.0 * cyc)
    # the raw per-kernel summary names the library it was taken on, so bench.py's roofline can be recomputed from it
    out["_meta"] = {"build_id": bid, "tag": tag, "config": config, "df_mode": mode,
                    "note": "per-kernel averages over the launches of each rocprofv3 --pmc pass (one process per pass)"}
    json.dump(out, open(os.path.join(prof, "%s_pmc.json" % tag), "w"), indent=1, sort_keys=True)
    meta = out.pop("_meta")
    # the dominant k_spectra kernel (the modified modes also run the short F_FB fallback launch); an F_TS launch
    # over a surface whose tables exceed one chunk runs it several times per pass (engine.hip): per-pass totals =
    # per-launch averages x launches per pass, passes = the record prepass launches (k_prep, one per pass: since
    # round 5 a Grad / RTA-CE pass also enqueues the gated fallback plan's k_spectra / k_reduce, which return at once)
    # (operation 0: k_dndx, its main launch once per pass beside the F_FB one)
    dom = "k_dndx" if any(k.startswith("k_dndx") for k in out) else "k_spectra"
    spec = sorted((k for k in out if k.startswith(dom)), key=lambda k: -out[k].get("avg_ns_pmc_pass", 0.0))
    passes = sum(out[k].get("launches", 0) for k in out if k.startswith("k_prep"))
    key = "%s_mode%d" % (config, mode)
    lpp = 1.0
    if spec and passes:
        lpp = out[spec[0]]["launches"] / float(passes)
    if spec and "hbm_bytes_per_launch" in out[spec[0]]:
        tp = os.path.join(prof, "pmc_traffic.json")
        t = json.load(open(tp)) if os.path.exists(tp) else {}
        t[key] = {"hbm_bytes_per_launch": out[spec[0]]["hbm_bytes_per_launch"], "launches_per_pass": lpp,
                  "hbm_bytes_per_pass": out[spec[0]]["hbm_bytes_per_launch"] * lpp, "tag": tag, "build_id": bid}
        json.dump(t, open(tp, "w"), indent=1, sort_keys=True)
    if spec and "valu_issue_frac" in out[spec[0]]:
        vp = os.path.join(prof, "pmc_valu.json")
        v = json.load(open(vp)) if os.path.exists(vp) else {}
        e = out[spec[0]]
        v[key] = {"tag": tag, "build_id": bid, "valu_insts_per_launch": e["SQ_INSTS_VALU"], "valu_issue_frac": e["valu_issue_frac"],
                  "clock_ghz": e["clock_ghz"]}
        for c in ("ADD_F64", "MUL_F64", "FMA_F64", "TRANS_F64", "INT32", "INT64", "CVT"):
            if "SQ_INSTS_VALU_" + c in e:
                v[key][c.lower() + "_insts_per_launch"] = e["SQ_INSTS_VALU_" + c]
        if "SQ_INSTS_VALU_FLOPS_FP64" in e:
            # the counter adds FMA x 2 + ADD + MUL + TRANS per WAVE-instruction (it equals that sum of the
            # per-type counters); x 64 lanes = flops (rocprofv3's derived FLOP metrics scale it the same way)
            v[key]["fp64_flops_per_launch"] = 64.0 * e["SQ_INSTS_VALU_FLOPS_FP64"]
            v[key]["fp64_flops_per_pass"] = 64.0 * e["SQ_INSTS_VALU_FLOPS_FP64"] * lpp
        if "SQ_LDS_BANK_CONFLICT" in e:
            v[key]["lds_bank_conflict_cycles"] = e["SQ_LDS_BANK_CONFLICT"]
        if "SQ_LDS_IDX_ACTIVE" in e and "clock_ghz" in e:
            # LDS-array cycles summed over the 256 CUs / (256 x kernel cycles)
            v[key]["lds_busy_frac"] = e["SQ_LDS_IDX_ACTIVE"] / (256.0 * e["avg_ns_pmc_pass"] * e["clock_ghz"])
        if "SQC_DCACHE_REQ" in e and e["SQC_DCACHE_REQ"] > 0:
            v[key]["scalar_cache_miss_frac"] = e.get("SQC_DCACHE_MISSES", 0.0) / e["SQC_DCACHE_REQ"]
        v[key]["kernel_ns_pmc_pass"] = e["avg_ns_pmc_pass"]
        v[key]["launches_per_pass"] = lpp
        json.dump(v, open(vp, "w"), indent=1, sort_keys=True)
    for k, e in sorted(out.items()):
        print(k, {c: round(v, 3) for c, v in e.items()})
    print("_meta", meta)


if __name__ == "__main__":
    main()
