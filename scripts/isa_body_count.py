"""Static instruction counts per basic block of the C3 fused kernel's chunk loop.

Compiles bo_predict_d2.hip as the library build does (hipcc --save-temps, gfx950, max-ILP
scheduler), takes cm_predict_kernel<2, GRID, UPPER, !GROWS, 16, !PART> (the C3 headline kernel)
and prints, for every basic block holding MFMAs, the count of each instruction class: MFMA,
VALU (other v_ instructions), v_accvgpr reads/writes, LDS (ds_), VMEM (buffer_/global_),
s_waitcnt, s_nop, s_barrier, other SALU.  The SEP chunk loop is the second group of MFMA blocks
(the first is the non-separable path of the same kernel, with its lockstep barrier per body).

    python scripts/isa_body_count.py [out.txt]          (CPU only; ~30 s)
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
KERNEL = "_ZN12_GLOBAL__N_117cm_predict_kernelILi2ELb1ELb1ELb0ELi16ELb0EEEvN2bo9FusedArgsE"


def classify(ins):
    op = ins.split()[0] if ins else ""
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "acc"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def blocks(asm, kname):
    i = asm.index(kname + ":")
    j = asm.index(".Lfunc_end", i)
    out, cur = [], ["entry", []]
    for ln in asm[i:j].split("\n"):
        t = ln.strip()
        if re.match(r"^\.LBB\d+_\d+:", t):
            out.append(cur)
            cur = [t.split(":")[0], []]
            continue
        if not t or t.startswith((";", ".")):
            continue
        cur[1].append(t.split(";")[0].strip())
    out.append(cur)
    return out


def main():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(ROOT, "bayesopt_smart_amd", "csrc", "bo_predict_d2.hip")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "-I", os.path.join(ROOT, "include"), "-mllvm", "-amdgpu-sched-strategy=max-ilp",
                        "-c", src, "-o", os.path.join(d, "d2.o"), "--save-temps"], cwd=d, check=True,
                       capture_output=True)
        asm = open(os.path.join(d, "bo_predict_d2-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    lines = [f"# static counts per MFMA-holding basic block of {KERNEL}", "# label: " +
             " ".join(["mfma", "valu", "acc", "lds", "vmem", "wait", "nop", "barrier", "salu"])]
    for label, ins in blocks(asm, KERNEL):
        c = {}
        for x in ins:
            k = classify(x)
            c[k] = c.get(k, 0) + 1
        if c.get("mfma", 0) >= 8:
            lines.append(f"{label}: " + " ".join(str(c.get(k, 0)) for k in
                                                  ("mfma", "valu", "acc", "lds", "vmem", "wait", "nop", "barrier", "salu")))
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
