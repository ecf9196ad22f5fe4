"""Per-kernel counter summary of a tools/pmc_c4.sh directory (C3 / C4 / SWEEP
config kernels of tools/bench_configs.py): per launch and per sample VALU /
SALU / VMEM / LDS wave-instructions, lane utilisation
(SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)), VALU busy per wave
(SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES), SQ_WAIT_ANY share and L2 hit rate.
Usage: python tools/summarize_cfg_pmc.py gpurun_out/<tag>/pmc_bvh SAMPLES_PER_LAUNCH... > summary.json
(samples given per kernel-name substring as NAME=SAMPLES)."""
import csv
import json
import os
import statistics
import sys

src = sys.argv[1]
spl = dict(a.split("=") for a in sys.argv[2:])


def rows(d):
    p = os.path.join(src, d, "run_counter_collection.csv")
    return list(csv.DictReader(open(p))) if os.path.exists(p) else []


out = {}
for key, samples in spl.items():
    samples = float(samples)
    acc = {}
    for d in ("sq", "sq2", "mem"):
        for r in rows(d):
            if key not in r["Kernel_Name"]:
                continue
            acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    c = {k: statistics.mean(v.values()) for k, v in acc.items()}
    ks = [k for k in csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))) if key in k["Name"]]
    rec = {"kernel": ks[0]["Name"] if ks else key, "avg_ms": float(ks[0]["AverageNs"]) / 1e6 if ks else None,
           "samples_per_launch": samples, "counters_per_launch": c}
    if ks:
        rec["msamples_per_s"] = samples / (rec["avg_ms"] * 1e-3) / 1e6
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
        if k in c:
            rec[k.lower() + "_per_sample"] = c[k] / samples
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
        rec["valu_lane_utilization"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_VALU" in c:
        rec["valu_active_frac_of_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
    if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
        rec["wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        rec["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    out[key] = rec
print(json.dumps(out, indent=1))
