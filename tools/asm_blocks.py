"""Per-basic-block instruction census of a kernel in rt_kernels.s (make -C
tipe-raytracer_amd asm).  Usage: [KERNEL=sym] python tools/asm_blocks.py [min_valu] [asm]
Default kernel: render_kernel<false, false, false> (the sphere-scene render)."""
import collections
import os
import re
import sys

path = sys.argv[2] if len(sys.argv) > 2 else "tipe-raytracer_amd/rt_kernels.s"
s = open(path).read()
KERNEL = os.environ.get("KERNEL", "_ZN2rt13render_kernelILb0ELb0ELb0EEEvNS_7KParamsE")
start = s.index(KERNEL + ":")
body = s[start:s.index("s_endpgm", start)].splitlines()
blocks, cur = [], ["entry", [], ""]
for line in body:
    m = re.match(r"^(\.LBB\S+):(.*)", line)
    if m:
        blocks.append(cur)
        cur = [m.group(1), [], m.group(2).strip(" ;")]
        continue
    t = line.strip()
    if t and not t.startswith(";") and not t.startswith("."):
        cur[1].append(t.split()[0])
blocks.append(cur)
lim = int(sys.argv[1]) if len(sys.argv) > 1 else 0
keys = ["v_readlane_b32", "v_writelane_b32", "v_mov_b32_e32", "v_mov_b64_e32", "v_cndmask_b32_e32",
        "v_rsq_f64_e32", "v_rcp_f64_e32", "v_div_scale_f64", "v_mad_u64_u32", "scratch_load_dwordx2",
        "s_load_dwordx16", "s_load_dwordx2"]
short = ["rl", "wl", "mov", "mov64", "cnd", "rsq", "rcp", "dsc", "mad", "scr", "sl16", "sl2"]
for name, ins, loop in blocks:
    c = collections.Counter(ins)
    v = sum(n for k, n in c.items() if k.startswith("v_"))
    if v < lim:
        continue
    tags = " ".join(f"{sh}:{c[k]}" for k, sh in zip(keys, short) if c[k])
    print(f"{name:12s} v={v:4d} s={sum(n for k, n in c.items() if k.startswith('s_')):3d} {tags:60s} {loop[:40]}")
