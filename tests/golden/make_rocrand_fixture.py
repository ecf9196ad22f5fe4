"""Regenerate tests/golden/rocrand_stream.json: the first 12 draws of
rocRAND's own Philox4x32-10 engine (rocrand_init(seed, (s << 32) | p, 0),
rocrand()) for a few (seed, pixel, sample) streams, from
/opt/rocm/include/rocrand/rocrand_philox4x32_10.h compiled host-side by
hipcc (src/rocrand_stream.cpp).  Pins the RT_RNG_PHILOX stream spec (rt.h)
to hiprand/rocrand's generator."""
import json, os, subprocess, tempfile
HERE = os.path.dirname(os.path.abspath(__file__))
exe = os.path.join(tempfile.mkdtemp(), "rocrand_stream")
subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-w", "-o", exe, os.path.join(HERE, "src", "rocrand_stream.cpp")], check=True)
rows = []
for line in subprocess.run([exe], check=True, capture_output=True, text=True).stdout.splitlines():
    v = [int(x) for x in line.split()]
    rows.append({"seed": v[0], "pixel": v[1], "sample": v[2], "draws": v[3:]})
with open(os.path.join(HERE, "rocrand_stream.json"), "w") as f:
    json.dump(rows, f, indent=1)
print("wrote", len(rows), "streams")
