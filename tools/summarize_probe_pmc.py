"""Per-scene counter summary of a tools/pmc_probe.sh directory: the render
kernel's dispatches in launch order are grouped per scene (3 per scene:
warm-up + 2 timed, tools/probes/nonopq_scenes.py).  Usage:
python tools/summarize_probe_pmc.py gpurun_out/<dir> SPP > summary.json"""
import csv, json, os, sys
src, spp = sys.argv[1], int(sys.argv[2])
SCENES = ("nature", "mineways", "tree_water_ao")
PX = 1200 * 900


def per_dispatch(d):
    acc = {}
    for r in csv.DictReader(open(os.path.join(src, d, "run_counter_collection.csv"))):
        if "render_kernel_q" not in r["Kernel_Name"]:
            continue
        acc.setdefault(int(r["Dispatch_Id"]), {}).setdefault(r["Counter_Name"], 0.0)
        acc[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return [acc[k] for k in sorted(acc)]


rows = {}
for d in ("sq", "sq2", "mem"):
    for i, c in enumerate(per_dispatch(d)):
        rows.setdefault(i, {}).update(c)
out = {}
n = len(rows) // len(SCENES)
for si, name in enumerate(SCENES):
    ds = [rows[i] for i in range(si * n + 1, si * n + n)]      # timed dispatches (skip the warm-up)
    c = {k: sum(x[k] for x in ds) / len(ds) for k in ds[0]}
    S = PX * spp
    out[name] = {"valu_per_sample": c["SQ_INSTS_VALU"] / S, "salu_per_sample": c["SQ_INSTS_SALU"] / S,
                 "vmem_per_sample": c["SQ_INSTS_VMEM"] / S,
                 "valu_lane_utilization": c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]),
                 "wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
                 "l2_hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])}
print(json.dumps(out, indent=1))
