"""Instruction histogram of one kernel's loops, from hipcc -S output.

    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S kernels.hip -o k.s
    python3 tools/isa_hist.py k.s _ZN3cpz13k_verify_eachENS_10VerifyArgsE

Splits the kernel into basic blocks, finds the back edges (a branch to a label at or above
it), and prints for every loop body (label .. back edge) its instruction count and mnemonic
histogram, innermost loops first.  Used to see where a kernel's non-MAD VALU work goes.
"""
import collections
import re
import sys


def kernel_lines(path, name):
    out, on = [], False
    for line in open(path):
        if line.startswith(name + ":"):
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end") or line.strip().startswith(".size") and name in line:
                break
            out.append(line.rstrip("\n"))
    return out


def parse(path, name):
    """(instructions [(mnemonic, text)], loops [(first, last, label)] innermost first)."""
    lines = kernel_lines(path, name)
    labels = {}
    insts = []
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            m = re.match(r"^(\.LBB[0-9_]+):", s)
            if m:
                labels[m.group(1)] = len(insts)
            continue
        insts.append((s.split()[0], s))
    loops = []
    for idx, (mn, s) in enumerate(insts):
        if mn.startswith("s_cbranch") or mn == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= idx:
                loops.append((labels[tgt], idx, tgt))
    loops.sort(key=lambda t: t[1] - t[0])
    return insts, loops


def loop_bodies(path, name):
    """[(label, Counter of mnemonics)] per loop body, innermost first."""
    insts, loops = parse(path, name)
    return [(tgt, collections.Counter(mn for mn, _ in insts[lo:hi + 1])) for lo, hi, tgt in loops]


def main():
    path, name = sys.argv[1], sys.argv[2]
    insts, loops = parse(path, name)
    total = collections.Counter(mn for mn, _ in insts)
    print("kernel %s: %d instructions" % (name, len(insts)))
    for lo, hi, tgt in loops:
        body = collections.Counter(mn for mn, _ in insts[lo:hi + 1])
        n = hi + 1 - lo
        valu = sum(v for k, v in body.items() if k.startswith("v_"))
        mad = body.get("v_mad_i64_i32", 0) + body.get("v_mad_u64_u32", 0)
        print("\nloop %s [%d..%d]: %d instructions, %d VALU, %d MAD (%.0f%%)" % (tgt, lo, hi, n, valu, mad,
                                                                              100.0 * mad / max(valu, 1)))
        for k, v in body.most_common(24):
            print("   %6d %s" % (v, k))
    print("\nwhole kernel:")
    for k, v in total.most_common(30):
        print("   %6d %s" % (v, k))


if __name__ == "__main__":
    main()
