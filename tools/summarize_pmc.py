"""Summarize a rocprofv3 measurement directory (gpurun_out/<tag>) for the
render kernel: mean duration, HBM traffic per launch (FETCH_SIZE x2 gfx950
correction + WRITE_SIZE, both KiB units), instruction mix, VALU activity.
Writes profiles/<tag>/summary.json and profiles/pmc_traffic.json."""
import csv, json, os, statistics, sys
tag = sys.argv[1]
src = os.path.join("gpurun_out", tag)
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)
def rows(d):
    p = os.path.join(src, d, "run_counter_collection.csv")
    return list(csv.DictReader(open(p))) if os.path.exists(p) else []
KNAME = os.environ.get("KNAME", "render_kernel_q<false, 0, -2, false>")     # the C2 hot kernel (r03: <false, 0, 0>; r01: render_kernel<false, false, false>)
def per_dispatch(d, counter, kname=KNAME):
    acc = {}
    for r in rows(d):
        if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
            acc[r["Dispatch_Id"]] = acc.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return statistics.mean(acc.values()) if acc else None
ks = list(csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))))
render = [k for k in ks if KNAME in k["Name"]][0]
fetch_kib = per_dispatch("fetch", "FETCH_SIZE")
write_kib = per_dispatch("write", "WRITE_SIZE")
hbm = (2 * fetch_kib + write_kib) * 1024 if fetch_kib is not None else None
s = {c: per_dispatch("sq", c) for c in ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM",
                                       "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"]}
s.update({c: per_dispatch("sq2", c) for c in ["SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                             "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE"]})
mix = {c: per_dispatch("mix", c) for c in ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                           "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64",
                                           "SQ_INSTS_VALU_CVT", "SQ_INSTS_BRANCH"]}
fl = {c: per_dispatch("flops", c) for c in ["SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU_FLOPS_FP64_TRANS",
                                           "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU"]}
s.update({k: v for k, v in mix.items() if v is not None})
s.update({k + ("@flops_pass" if k == "SQ_ACTIVE_INST_VALU" else ""): v for k, v in fl.items() if v is not None})
dur_ns = float(render["AverageNs"])
out = {"kernel": render["Name"], "calls": int(render["Calls"]), "avg_ms": dur_ns / 1e6,
       "fetch_kib_raw": fetch_kib, "write_kib": write_kib,
       "hbm_bytes_per_launch": hbm, "counters_per_launch": s,
       "effective_clock_ghz": s["GRBM_GUI_ACTIVE"] / 8 / (dur_ns * 1e-9) / 1e9 if s["GRBM_GUI_ACTIVE"] else None,
       "valu_active_frac_of_wave_cycles": s["SQ_ACTIVE_INST_VALU"] / s["SQ_WAVE_CYCLES"] if s["SQ_WAVE_CYCLES"] else None,
       "wait_any_frac": s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"] if s["SQ_WAVE_CYCLES"] else None,
       "wait_inst_any_frac": s["SQ_WAIT_INST_ANY"] / s["SQ_WAVE_CYCLES"] if s["SQ_WAVE_CYCLES"] else None,
       "valu_lane_utilization": (fl["SQ_THREAD_CYCLES_VALU"] / (fl["SQ_ACTIVE_INST_VALU"] * 64)
                                 if fl["SQ_THREAD_CYCLES_VALU"] and fl["SQ_ACTIVE_INST_VALU"] else None),
       # SQ_INSTS_VALU_FLOPS_FP64 counts per wave instruction (FMA = 2): it equals
       # ADD_F64 + MUL_F64 + 2*FMA_F64 + TRANS_F64 exactly, so lane FLOPs are x64,
       # scaled by the measured lane utilization.
       "hw_fp64_tflops": (fl["SQ_INSTS_VALU_FLOPS_FP64"] * 64 * (fl["SQ_THREAD_CYCLES_VALU"] / (fl["SQ_ACTIVE_INST_VALU"] * 64))
                          / (dur_ns * 1e-9) / 1e12
                          if fl["SQ_INSTS_VALU_FLOPS_FP64"] and fl["SQ_ACTIVE_INST_VALU"] else None),
       "note": "FETCH_SIZE doubled (gfx950 reports half of wide-load bytes, MI355X_MICROARCH.md HBM); "
               "units KiB; per " + KNAME + " launch; PMC runs are separate rocprofv3 passes"}
json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
for f in ["kt/run_kernel_stats.csv"]:
    os.system("cp %s %s" % (os.path.join(src, f), os.path.join(dst, "kernel_stats.csv")))
for d in ["fetch", "write", "sq", "sq2", "mix", "flops"]:
    p = os.path.join(src, d, "run_counter_collection.csv")
    if os.path.exists(p):
        os.system("cp %s %s" % (p, os.path.join(dst, "pmc_%s.csv" % d)))
for f in ["bench.json", "host_path.json", "pytest_gpu.log", "demo.log"]:
    p = os.path.join(src, f)
    if os.path.exists(p):
        os.system("cp %s %s" % (p, os.path.join(dst, f)))
import subprocess
commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
json.dump({"render_kernel_hbm_bytes_per_launch": hbm, "source": dst + "/summary.json",
           "workload": "C2 1200x900 1000spp 6 bounces, spp_chunks 32", "kernel": KNAME,
           "measured_at_commit": commit,
           "note": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, separate passes; a committed profile "
                   "value, re-measured by tools/profile_run.sh + tools/summarize_pmc.py"},
          open(os.path.join("profiles", "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
