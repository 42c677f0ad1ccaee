#!/usr/bin/env python3
"""Per-phase ISA census of the BVH megakernel (render_kernel<1,true,false,false,false,true,5>).

Builds tray_kernel.hip for gfx950 with the product flags plus -g (debug line
tables do not change the generated code: the census checks the instruction
count against the product build's assembly), disassembles the kernel, and
symbolises every instruction with its inline stack. The frame of
render_kernel gives the source line of the kernel loop the instruction belongs
to; the TRAY_MARK anchors in tray_kernel.hip (no-ops in every build but
-DTRAY_CENSUS) divide the loop into phases: refill (item assignment, camera
ray, candidate tests, shading of candidate-answered camera rays), node steps,
leaf tests, shading. Each VALU instruction is classed as the SQ_INSTS_VALU_*
counters class it (FP64 add/mul/fma, FP32, transcendental, INT32, INT64,
conversion) or, for the ~42 % those counters do not cover, by what it is
(moves, v_cndmask, compares, min/max, lane ops, bit ops that are not INT32
arithmetic).

Static counts are per pass through a phase's code. With --phase (a
tools/phase_profile.py record: phase executions per frame) the tool also
weights them into an estimate of dynamic wave-instructions per frame, to set
against SQ_INSTS_VALU of the same build (profiles/pmc_mix_c2.json, per launch
of --frames frames). Rare paths (blocks holding a full FP64 division or sqrt,
the fallbacks of the Markstein quotient and sqrt_core range checks) are
counted separately as cold.

    python tools/isa_census.py [--phase profiles/r2h_phase_c2.json] [--pmc profiles/pmc_mix_c2.json]
           [--json out.json] [--markdown]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tray_amd", "csrc", "tray_kernel.hip")
KERNEL = "_ZN4tray13render_kernelILi1ELb1ELb0ELb0ELb0ELi1ELi5EEEvNS_12KernelParamsE"  # --layout 2: ...ILi2E...
LLVM = "/opt/rocm/lib/llvm/bin"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "-mllvm",
         "-amdgpu-atomic-optimizer-strategy=None"]

# VALU classes the SQ_INSTS_VALU_* counters report (MI355X), then the rest.
COUNTED = ("fp64_add", "fp64_mul", "fp64_fma", "trans", "fp32_fma", "fp32_mul", "fp32_add", "int32", "int64", "cvt")
UNCOUNTED = ("mov", "cndmask", "cmp", "minmax", "lane", "bitop", "fp64_other", "other")


def valu_class(m: str) -> str:
    """The class of VALU mnemonic m (e.g. 'v_fma_f64')."""
    m = re.sub(r"_e(32|64|64_dpp|32_dpp|_sdwa)$", "", m)
    if m.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "lane"
    if m.startswith("v_mov") or m in ("v_swap_b32", "v_accvgpr_read_b32", "v_accvgpr_write_b32", "v_accvgpr_mov_b32"):
        return "mov"
    if m.startswith("v_cndmask"):
        return "cndmask"
    if m.startswith(("v_cmp", "v_cmpx")):
        return "cmp"
    if m.startswith(("v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos", "v_exp", "v_log")):
        return "trans"
    if m.startswith("v_cvt"):
        return "cvt"
    if re.match(r"v_(min|max|med)3?_(f32|f64|u32|i32|f16)|v_pk_(min|max)", m):
        return "minmax"
    if m in ("v_add_f64", "v_add_f64_e64"):
        return "fp64_add"
    if m == "v_mul_f64":
        return "fp64_mul"
    if m in ("v_fma_f64", "v_fmac_f64"):
        return "fp64_fma"
    if m.endswith("_f64"):  # div_scale / div_fmas / div_fixup / ldexp / frexp / class
        return "fp64_other"
    if re.match(r"v_(pk_)?(fma|fmac|fmaak|fmamk|mad|mac)_(f32|legacy)", m) or m.startswith("v_pk_fma"):
        return "fp32_fma"
    if re.match(r"v_(pk_)?mul_f32", m):
        return "fp32_mul"
    if re.match(r"v_(pk_)?(add|sub|subrev)_f32", m):
        return "fp32_add"
    if m.startswith(("v_mad_u64", "v_mad_i64", "v_lshl_add_u64", "v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64",
                     "v_add_co", "v_addc_co", "v_sub_co", "v_subb_co", "v_subrev_co", "v_subbrev_co", "v_add_u64",
                     "v_sub_u64")):
        return "int64"
    if re.match(r"v_(add|sub|subrev|add3|mul_lo|mul_hi|mad_u32|mad_i32|mul_u32|mul_i32|lshl_add|add_lshl|"
                r"lshlrev|lshrrev|ashrrev|lshl_or|and_or|or3|xad|mbcnt|bcnt)_", m):
        return "int32"
    if re.match(r"v_(and|or|xor|not|bfe|bfi|alignbit|alignbyte|perm|bfrev|ffbh|ffbl)_", m):
        return "bitop"
    return "other"


def unit_of(m: str) -> str:
    if m.startswith("v_"):
        return "valu"
    if m.startswith("s_waitcnt") or m in ("s_nop", "s_sleep", "s_barrier", "s_setprio"):
        return "wait"
    if m.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc", "s_endpgm")):
        return "branch"
    if m.startswith(("s_load", "s_buffer_load", "s_store", "s_memtime", "s_memrealtime", "s_dcache")):
        return "smem"
    if m.startswith("s_"):
        return "salu"
    if m.startswith("ds_"):
        return "lds"
    if m.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def build(work: str) -> str:
    os.makedirs(work, exist_ok=True)
    obj = os.path.join(work, "k.o")
    co = os.path.join(work, "k.co")
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-g", "--cuda-device-only", "-c", "-o", obj, SRC], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={obj}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def product_count(work: str) -> int:
    """VALU+SALU+... instruction count of the kernel in the product build's assembly (no -g)."""
    s = os.path.join(work, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "--cuda-device-only", "-S", "-o", s, SRC], check=True)
    n, inside = 0, False
    for line in open(s):
        if line.startswith(KERNEL + ":"):
            inside = True
            continue
        if inside and line.startswith(".Lfunc_end"):
            break
        if inside and re.match(r"\s+[sv]_|\s+(ds|global|buffer|flat|scratch)_", line):
            n += 1
    return n


def disassemble(co: str):
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    insts, inside = [], False
    for line in out.splitlines():
        if line.endswith(f"<{KERNEL}>:"):
            inside = True
            continue
        if inside:
            if not line.strip():
                break
            m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", line)
            if m:
                tgt = re.search(r"<" + re.escape(KERNEL) + r"\+0x([0-9a-f]+)>", line)
                insts.append({"addr": int(m.group(3), 16), "mn": m.group(1), "ops": m.group(2),
                              "target": int(tgt.group(1), 16) if tgt else None})
    return insts


def symbolize(co: str, insts):
    """Inline stack (innermost first) of every instruction: [(function, line), ...]."""
    q = "\n".join(hex(i["addr"]) for i in insts) + "\n"
    out = subprocess.run([f"{LLVM}/llvm-symbolizer", f"--obj={co}", "--inlining", "--functions=short",
                          "--output-style=JSON"], input=q, check=True, capture_output=True, text=True).stdout
    stacks = []
    for line in out.splitlines():
        rec = json.loads(line)
        stacks.append([(f["FunctionName"], int(f["Line"])) for f in rec["Symbol"]])
    assert len(stacks) == len(insts)
    return stacks


def phase_anchors():
    """(line, phase) of every TRAY_MARK in the kernel loop, in source order."""
    marks = []
    for k, line in enumerate(open(SRC), 1):
        m = re.search(r'TRAY_MARK\("(\w+)"\)', line)
        if m and "#define" not in line:
            marks.append((k, m.group(1)))
    return marks


def phase_of(line: int, marks) -> str:
    ph = "prologue"
    for ln, name in marks:
        if line >= ln:
            ph = name
    return ph


# Which phase-profile counter counts the executions of each phase (per frame).
WEIGHT = {"refill_assign": "loop_iters", "refill_cam": "refill_phases", "refill_cand": "refill_phases",
          "refill_shade": "refill_phases", "refill_end": "loop_iters", "node_ctl": "node_iters", "node": "node_iters",
          "leaf_decide": "loop_iters", "leaf_ctl": "leaf_phases", "leaf": "leaf_phases",
          "shade_ctl": "shade_phases", "shade": "shade_phases", "shade_end": "shade_phases"}
GROUP = {"refill_assign": "refill", "refill_cam": "refill", "refill_cand": "refill", "refill_shade": "refill",
         "refill_end": "loop", "node_ctl": "node", "node": "node", "leaf_decide": "loop", "leaf_ctl": "leaf",
         "leaf": "leaf", "shade_ctl": "shade", "shade": "shade", "shade_end": "shade"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work", default=os.path.join(ROOT, "tray_amd", "build", "census"))
    ap.add_argument("--phase", default=os.path.join(ROOT, "profiles", "r2h_phase_c2.json"))
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_mix_c2.json"))
    ap.add_argument("--json", default=None)
    ap.add_argument("--markdown", action="store_true")
    ap.add_argument("--layout", type=int, default=1, help="LDS layout instance (1: book cover; 2: dense C5)")
    ap.add_argument("--list", default=None, metavar="PHASE",
                    help="print the hot instructions of one phase (address, instruction, innermost function:line)")
    args = ap.parse_args()
    global KERNEL
    KERNEL = KERNEL.replace("ILi1E", f"ILi{args.layout}E")

    co = build(args.work)
    insts = disassemble(co)
    stacks = symbolize(co, insts)
    marks = phase_anchors()
    kernel_fn = "render_kernel"

    # Basic blocks: leaders are branch targets and instructions after a branch.
    leaders = {insts[0]["addr"]}
    base = insts[0]["addr"]
    for k, i in enumerate(insts):
        if i["target"] is not None:
            leaders.add(base + i["target"])
        if i["mn"].startswith(("s_cbranch", "s_branch")) and k + 1 < len(insts):
            leaders.add(insts[k + 1]["addr"])
    block, bid = [], -1
    for i in insts:
        if i["addr"] in leaders:
            bid += 1
        block.append(bid)
    # Rare paths: the full-division and full-sqrt lowerings behind the Markstein / sqrt_core range checks
    # (v_div_scale_f64 and v_cmp_class_f64 appear only there).
    cold_blocks = {block[k] for k, i in enumerate(insts) if i["mn"].startswith(("v_div_scale_f64", "v_cmp_class_f64"))}

    static = collections.defaultdict(lambda: collections.Counter())
    inner = collections.defaultdict(lambda: collections.Counter())
    ph = "prologue"
    for k, (i, st) in enumerate(zip(insts, stacks)):
        line = next((ln for fn, ln in st if fn.startswith(kernel_fn)), 0)
        if line:  # line 0: compiler-generated (merged) code, kept with the instructions before it
            ph = phase_of(line, marks)
        hot = block[k] not in cold_blocks
        u = unit_of(i["mn"])
        key = ph if hot else ph + ":cold"
        if args.list == key:
            print(f"{i['addr']:6x}  {i['mn']:<24} {i['ops'][:48]:<48} {st[0][0][:40]}:{st[0][1]}")
        static[key]["inst"] += 1
        static[key]["unit:" + u] += 1
        if u == "valu":
            static[key]["valu"] += 1
            static[key]["c:" + valu_class(i["mn"])] += 1
            if hot:
                inner[ph][st[0][0] if st[0][0] != kernel_fn else "(loop)"] += 1

    rec = {"kernel": KERNEL, "build": "product flags + -g (tray_amd/Makefile HIPFLAGS)",
           "instructions": len(insts), "product_asm_instructions": product_count(args.work),
           "valu_classes_counted_by_pmc": COUNTED, "valu_classes_not_counted": UNCOUNTED,
           "phases": {}, "inner_functions_valu": {}}
    order = [m for _, m in marks]
    for ph in ["prologue"] + order + [p + ":cold" for p in ["prologue"] + order]:
        if ph in static:
            c = static[ph]
            rec["phases"][ph] = {"inst": c["inst"], "valu": c["valu"],
                                 "units": {k[5:]: v for k, v in sorted(c.items()) if k.startswith("unit:")},
                                 "valu_classes": {k[2:]: v for k, v in sorted(c.items()) if k.startswith("c:")}}
    for ph, c in inner.items():
        rec["inner_functions_valu"][ph] = dict(c.most_common(8))

    # Dynamic estimate per frame from the phase profile.
    if args.phase and os.path.exists(args.phase):
        pr = json.load(open(args.phase))
        dyn = collections.Counter()
        dyn_group = collections.defaultdict(collections.Counter)
        for ph, w in WEIGHT.items():
            if ph not in static:
                continue
            n = pr.get(w, 0)
            for k, v in static[ph].items():
                if k == "valu" or k.startswith("c:"):
                    dyn[k] += v * n
                    dyn_group[GROUP[ph]][k] += v * n
        est = {"source": os.path.relpath(args.phase, ROOT), "weights": {ph: WEIGHT[ph] for ph in WEIGHT},
               "valu_per_frame": dyn["valu"],
               "classes_per_frame": {k[2:]: v for k, v in sorted(dyn.items()) if k.startswith("c:")},
               "by_group": {g: {"valu": c["valu"], **{k[2:]: v for k, v in sorted(c.items()) if k.startswith("c:")}}
                            for g, c in dyn_group.items()}}
        tot = max(1, dyn["valu"])
        est["uncounted_share"] = round(sum(dyn["c:" + c] for c in UNCOUNTED) / tot, 3)
        est["uncounted_split"] = {c: round(dyn["c:" + c] / tot, 3) for c in UNCOUNTED}
        if args.pmc and os.path.exists(args.pmc):
            pm = json.load(open(args.pmc))
            f = pm.get("frames_per_launch", 1)
            c = pm["counters"]
            est["pmc_valu_per_frame"] = c["SQ_INSTS_VALU"] / f
            est["pmc_uncounted_share"] = round(1 - sum(c[k] for k in (
                "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32",
                "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
                "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT")) / c["SQ_INSTS_VALU"], 3)
            est["estimate_over_pmc"] = round(dyn["valu"] / est["pmc_valu_per_frame"], 3)
        rec["dynamic_estimate"] = est

    js = json.dumps(rec, indent=1)
    if args.list:
        return
    if args.json:
        open(args.json, "w").write(js + "\n")
    if args.markdown:
        print_markdown(rec)
    else:
        print(js)


def print_markdown(rec):
    cls = COUNTED + UNCOUNTED
    print(f"instructions: {rec['instructions']} (product asm: {rec['product_asm_instructions']})\n")
    print("| phase | inst | VALU | " + " | ".join(cls) + " | LDS | VMEM | SALU | branch | wait |")
    print("|---" * (8 + len(cls)) + "|")
    for ph, c in rec["phases"].items():
        v = c["valu_classes"]
        u = c["units"]
        print(f"| {ph} | {c['inst']} | {c['valu']} | " + " | ".join(str(v.get(k, 0)) for k in cls) +
              f" | {u.get('lds', 0)} | {u.get('vmem', 0)} | {u.get('salu', 0)} | {u.get('branch', 0)} | {u.get('wait', 0)} |")
    if "dynamic_estimate" in rec:
        e = rec["dynamic_estimate"]
        print("\ndynamic estimate per frame:", json.dumps({k: e[k] for k in e if k not in ("weights", "by_group")}))
        for g, c in e["by_group"].items():
            print(g, json.dumps(c))
    print("\ninner functions (VALU):")
    for ph, c in rec["inner_functions_valu"].items():
        print(ph, json.dumps(c))


if __name__ == "__main__":
    sys.exit(main())
