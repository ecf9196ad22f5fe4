"""Kernel timeline of the rt_fill_canva x 12 pthreads drop-in (bench.py
end_to_end) for rocprofv3 --kernel-trace; with --analyze DIR, per-frame
span, kernel busy time (union of dispatch intervals) and the idle gaps.
Usage: rocprofv3 --kernel-trace -d gpurun_out/ft -o run --output-format csv -- python3 tools/fill_trace.py
       python3 tools/fill_trace.py --analyze gpurun_out/ft"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def analyze(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ks = [k for k in ks if "render_kernel" in k[2] or "combine" in k[2]]
    # frames: 13 fill_call()s (1 untimed + reps) of 12 bands; split where the gap exceeds 2 ms
    frames, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - max(e for _, e, _ in cur) > 2_000_000:
            frames.append(cur)
            cur = [k]
        else:
            cur.append(k)
    frames.append(cur)
    for fr in frames:
        span = max(e for _, e, _ in fr) - fr[0][0]
        busy, end = 0, 0
        for s, e, _ in fr:
            if e > end:
                busy += e - max(s, end)
                end = e
        rk = [k for k in fr if "render_kernel" in k[2]]
        durs = sorted((e - s) / 1e6 for s, e, _ in rk)
        print("frame: %d dispatches, span %.2f ms, busy %.2f ms, render kernels %d (%.2f..%.2f ms each)"
              % (len(fr), span / 1e6, busy / 1e6, len(rk), durs[0], durs[-1]))


def main():
    import numpy as np  # noqa: F401
    import bench
    import tipe_rt
    from tipe_rt import scenes
    spheres = scenes.cornell_spheres()
    scene = tipe_rt.make_scene(spheres)
    cam = tipe_rt.init_camera(**{k: scenes.README_CAMERA[k] for k in ("origin", "target", "up", "vfov", "ratio")})
    print(bench.end_to_end(scene, spheres, cam, reps=2))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        main()
