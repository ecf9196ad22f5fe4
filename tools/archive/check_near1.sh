#!/bin/bash
# Exhaustive CPU check of sqrt_rcp_near1 + div_core0 (rt_device_math.h): every
# double in [1 - 2^-18, 1 + 2^-18] (5.2e10 values) in 8 slices, with the
# program tests/test_near1_sqrt.py builds from the header's own source.
# Usage: bash tools/check_near1.sh   (about 4 minutes on 8 cores)
set -e -o pipefail
D=$(mktemp -d)
python3 - "$D" <<'EOF'
import pathlib, sys
sys.path.insert(0, "tests")
import test_near1_sqrt as t
print(t.build(pathlib.Path(sys.argv[1])))
EOF
python3 - "$D" <<'EOF'
import struct, subprocess, sys
d = sys.argv[1]
ub = lambda x: struct.unpack("<Q", struct.pack("<d", x))[0]
bd = lambda u: struct.unpack("<d", struct.pack("<Q", u))[0]
lo, hi = ub(1.0 - 2.0 ** -18), ub(1.0 + 2.0 ** -18)
cuts = [lo + (hi - lo + 1) * k // 8 for k in range(9)]
ps = [subprocess.Popen([d + "/near1", repr(bd(cuts[k])), repr(bd(cuts[k + 1] - 1 if k < 7 else hi)), "1"],
                       stdout=subprocess.PIPE, text=True) for k in range(8)]
tot = 0
for p in ps:
    out = p.communicate()[0].strip().splitlines()[-1]
    print(out)
    f = out.split()
    tot += int(f[1])
    assert f[3] == "0" and f[5] == "0", out
print("all", tot, "doubles: sqrt and div_core0 exact")
EOF
rm -rf "$D"
