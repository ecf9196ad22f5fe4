"""Instruction-class histogram of a render kernel's round loop, by phase and by
source function (where the non-arithmetic VALU issue is).

    make -C tipe-raytracer_amd asm-lines        # rt_kernels_g.s with .loc line tables
    python tools/isa_hist.py [KERNEL_SYMBOL] [asm] > profiles/<tag>/isa_hist.txt

Static counts: every instruction of the loop body (basic blocks the compiler
marks as inside a loop) once, attributed through its .loc inline chain to
  * the phase of render_kernel_q it was inlined into (the kernel's own
    "// ---- N." section markers, rt_kernels.hip), and
  * the innermost source function (rt_kernels.hip / rt_device_math.h).
Costs use the measured gfx950 issue rates (tools/probes/op_rates2/3, SIMD
cycles per wave64 instruction at 4-8 waves/SIMD), so the "cycles" columns are
the static issue cost of one pass over each block, not a dynamic profile: a
block's share of run time also depends on how often the round takes it (the
census, tools/census.sh, gives the phase time shares).
"""
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYM = sys.argv[1] if len(sys.argv) > 1 else "_ZN2rt15render_kernel_qILb0ELi0ELin2ELb0EEEvNS_7KParamsE"
ASM = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "tipe-raytracer_amd", "rt_kernels_g.s")
SRC = {"rt_kernels.hip": os.path.join(ROOT, "tipe-raytracer_amd", "csrc", "rt_kernels.hip"),
       "rt_device_math.h": os.path.join(ROOT, "tipe-raytracer_amd", "csrc", "rt_device_math.h")}

# measured issue cost (SIMD cycles per wave64 instruction, 8 waves/SIMD; op_rates2/3)
COST = {"f64 add/mul/fma": 4.75, "f64 cmp/class": 4.7, "f64 trans": 16.3, "f64 other": 4.8, "f32 fma/mul/add": 2.75,
        "f32 cmp/minmax": 4.7, "f32 trans": 8.3, "cvt": 4.7, "int32 alu": 3.0, "int64/mad64": 5.1, "cndmask": 3.0,
        "mov": 3.0, "lane xfer": 4.0, "lds": 0.0, "vmem": 0.0, "smem": 0.0, "salu": 0.0, "branch": 0.0, "other": 0.0}


SHORT = {"f64 add/mul/fma": "f64a", "f64 cmp/class": "f64c", "f64 trans": "f64t", "f64 other": "f64o",
         "f32 fma/mul/add": "f32a", "f32 cmp/minmax": "f32c", "f32 trans": "f32t", "cvt": "cvt", "int32 alu": "i32",
         "int64/mad64": "i64", "cndmask": "cnd", "mov": "mov", "lane xfer": "lane", "lds": "lds", "vmem": "vmem",
         "smem": "smem", "salu": "salu", "branch": "br", "other": "oth"}


def classify(op):
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_getpc")):
        return "branch"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if not op.startswith("v_"):
        return "other"
    o = op.split("_e32")[0].split("_e64")[0]
    if o.startswith("v_cndmask"):
        return "cndmask"
    if o.startswith(("v_mov", "v_accvgpr")):
        return "mov"
    if o.startswith(("v_readlane", "v_writelane", "v_readfirstlane", "v_permlane", "v_mov_dpp")):
        return "lane xfer"
    if o.startswith("v_cvt"):
        return "cvt"
    if o.endswith("_f64"):
        if o.startswith("v_cmp"):
            return "f64 cmp/class"
        if o.startswith(("v_rsq", "v_rcp", "v_sqrt")):
            return "f64 trans"
        if o.startswith(("v_add_f64", "v_mul_f64", "v_fma_f64", "v_fmac_f64")):
            return "f64 add/mul/fma"
        return "f64 other"
    if o.endswith(("_f32", "_f16")) or "fma_mix" in o:
        if o.startswith(("v_cmp", "v_min", "v_max", "v_med")):
            return "f32 cmp/minmax"
        if o.startswith(("v_rsq", "v_rcp", "v_sqrt", "v_exp", "v_log", "v_sin", "v_cos")):
            return "f32 trans"
        return "f32 fma/mul/add"
    if o.startswith(("v_mad_u64", "v_mad_i64", "v_lshl_add_u64", "v_add_co", "v_addc", "v_sub_co", "v_subb", "v_mul_hi",
                     "v_mul_lo", "v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64", "v_cmp_lt_i64", "v_cmp_gt_i64",
                     "v_cmp_eq_u64", "v_cmp_ne_u64")):
        return "int64/mad64"
    return "int32 alu"


def functions(path):
    """line -> enclosing function name (a crude scan of definitions)."""
    names = {}
    cur = "?"
    pat = re.compile(r"^\s{0,4}(?:__device__|__global__|static|template|__host__)[^;]*?\b([A-Za-z_][A-Za-z0-9_]*)\s*\(")
    for i, line in enumerate(open(path), 1):
        m = pat.match(line)
        if m and m.group(1) not in ("__launch_bounds__", "if", "for", "while", "sizeof"):
            cur = m.group(1)
        names[i] = cur
    return names


FUN = {k: functions(v) for k, v in SRC.items()}
kern_lines = open(SRC["rt_kernels.hip"]).read().splitlines()


def phase_of_line(ln):
    """render_kernel_q's section ('// ---- N.' marker) containing line ln."""
    best = "setup"
    for i in range(min(ln, len(kern_lines)) - 1, -1, -1):
        m = re.search(r"// ---- (\d\.[^-]*)", kern_lines[i])
        if m:
            return m.group(1).strip()
        if re.search(r"void render_kernel_q\(", kern_lines[i]):
            return best
    return best


def main():
    s = open(ASM).read()
    i0 = s.index(SYM + ":")
    body = s[i0:s.index("s_endpgm", i0)].splitlines()
    kfun_lo = next(i for i, l in enumerate(kern_lines, 1) if "void render_kernel_q(" in l)
    kfun_hi = next(i for i, l in enumerate(kern_lines, 1) if i > kfun_lo and l.startswith("}"))
    in_loop = False
    loc = ""
    by_phase = collections.defaultdict(collections.Counter)
    by_fun = collections.defaultdict(collections.Counter)
    total = collections.Counter()
    for line in body:
        t = line.strip()
        m = re.match(r"^(\.LBB\S+):(.*)", t)
        if m:
            in_loop = "Loop" in m.group(2) or "Depth" in m.group(2)
            continue
        if t.startswith(".loc"):
            loc = t.split(";", 1)[1].strip() if ";" in t else ""
            continue
        if not t or t.startswith((";", ".")) or not in_loop:
            continue
        op = t.split()[0]
        cls = classify(op)
        chain = re.findall(r"([\w./-]+):(\d+):\d+", loc)
        inner = "?"
        phase = "setup"
        if chain:
            f, ln = chain[0]
            base = os.path.basename(f)
            inner = FUN[base].get(int(ln), "?") if base in FUN else base
            for f2, ln2 in chain:
                if os.path.basename(f2) == "rt_kernels.hip" and kfun_lo <= int(ln2) <= kfun_hi:
                    phase = phase_of_line(int(ln2))
                    break
        by_phase[phase][cls] += 1
        by_fun[inner][cls] += 1
        total[cls] += 1
    classes = [c for c in COST if total[c]]

    def row(name, c):
        v = sum(n for k, n in c.items() if COST.get(k, 0) > 0)
        cyc = sum(n * COST.get(k, 0) for k, n in c.items())
        na = sum(n for k, n in c.items() if k in ("f64 cmp/class", "cndmask", "mov", "int32 alu", "int64/mad64", "cvt",
                                                  "lane xfer", "f32 cmp/minmax"))
        return "%-34s valu %4d  cyc %6.0f  non-arith %4d (%3.0f%%)  " % (name[:34], v, cyc, na, 100.0 * na / max(v, 1)) + \
               " ".join("%s:%d" % (SHORT[k], c[k]) for k in classes if c[k])
    print("kernel %s, loop blocks only (static counts; issue cycles from measured gfx950 rates)" % SYM)
    print("classes: " + ", ".join("%s = %s" % (v, k) for k, v in SHORT.items()))
    print(row("TOTAL", total))
    print("\n-- by phase of the round --")
    for p, c in sorted(by_phase.items(), key=lambda kv: -sum(kv[1].values())):
        print(row(p, c))
    print("\n-- by innermost source function --")
    for p, c in sorted(by_fun.items(), key=lambda kv: -sum(kv[1].values()))[:30]:
        print(row(p, c))


if __name__ == "__main__":
    main()
