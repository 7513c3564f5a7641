"""VALU issue classes of a kernel's instruction mix (profiling aid, CPU only).

Disassembles a kernel of libskml's device code (hipcc --cuda-device-only, llvm-objdump) and splits
its VALU instructions into the two issue classes tools/ubench/issue.hip measured on gfx950
(profiles/r06_ubench_issue.txt, 8 waves per SIMD of independent chains):

- 2-cycle class (~2.6 SIMD cycles per wave-instruction measured): v_add/v_sub/v_and/v_or/v_xor,
  the shifts, v_mul_f32, v_fma_f32, v_mov_b32 (e32 encodings);
- 4-cycle class (~4.4 measured): v_min/v_max/v_med3/v_min3/v_max3 (f32, u32, i32), every DPP
  move or DPP-fused op, v_cmp/v_cndmask, v_bfi/v_perm/v_sad and the other VOP3 forms.

Anything not in the 2-cycle list counts as 4-cycle (the conservative side).  The mix-weighted issue
ceiling of the kernel is then 1 wave-instruction per clock per CU x 4 / (4 - 2 f2), f2 = the
2-cycle share.  The share is static (instructions in the code, not executed); the leaf's code is
one unrolled round, so the two agree up to the exact-merge and partial-tile paths.

usage: python tools/valu_mix.py [SOURCE.hip] [KERNEL_SUBSTRING] > profiles/r06_leaf_valu_mix.json
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TWO_CYCLE = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|and_b32|or_b32|xor_b32|lshlrev_b32|lshrrev_b32|ashrrev_i32|"
                       r"mul_f32|fma_f32|add_f32|mov_b32)_e32$")


def disassemble(src):
    tmp = tempfile.mkdtemp()
    co, elf = os.path.join(tmp, "k.co"), os.path.join(tmp, "k.elf")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "--cuda-device-only", "-c", src, "-o", co], stderr=subprocess.DEVNULL)
    subprocess.check_call(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + co,
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + elf])
    return subprocess.check_output(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", elf],
                                   text=True).split("\n")


def mix(lines, kernel):
    heads = [i for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <", l)]
    start = next(i for i in heads if kernel in lines[i])
    end = next((i for i in heads if i > start), len(lines))
    ops = collections.Counter()
    for l in lines[start + 1:end]:
        m = re.match(r"\s*(v_[a-z0-9_]+)", l)
        if m:
            ops[m.group(1)] += 1
    total = sum(ops.values())
    two = sum(c for k, c in ops.items() if TWO_CYCLE.match(k))
    f2 = two / total
    return {"kernel": lines[start].split("<")[1].rstrip(">:"), "valu_static": total, "two_cycle": two,
            "two_cycle_share": round(f2, 4), "ceiling_factor": round(4.0 / (4.0 - 2.0 * f2), 4),
            "top": dict(ops.most_common(20))}


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "sketchml_amd", "csrc", "skml_sketch.hip")
    kern = sys.argv[2] if len(sys.argv) > 2 else "k_leaf64ILi1E"
    res = mix(disassemble(src), kern)
    res["source"] = os.path.relpath(src, ROOT)
    res["classes"] = "profiles/r06_ubench_issue.txt (tools/ubench/issue.hip): 2-cycle ~2.6, 4-cycle ~4.4 SIMD cycles"
    print(json.dumps(res, indent=1))
