"""ISA check of the MFMA kernels (build/jpgx_mx-gfx950.s): no memory load may write a VGPR that an
earlier MFMA still has to read.

Why: a chained MFMA (SrcC = an earlier product) whose destination differs from its SrcC leaves
the SrcC registers dead to the register allocator right after issue, and the scheduler may give
them to an LDS / global load issued a few instructions later.  The load's data can land before
the MFMA has read its last 16-lane group of SrcC (C rows 12..15) when the matrix pipe is backed
up -- nondeterministic wrong rows 12..15 (Y blocks 3 / 7 of a step), seen in k_mx422 / k_mx420
(profiles/r03_mfma_war.txt).  The compiler's wait states cover VALU writes, not this.

Rule checked: on every control-flow path from an MFMA (fall-through, taken branches and loop
back-edges: a walk over the .LBB basic blocks) up to the first non-MFMA instruction that reads its
result or the result of a later MFMA (which waits for it; a wave's MFMAs complete in issue order,
so then this one has read every operand), no instruction that writes VGPRs
from memory -- LDS reads, permutes / swizzles, LDS or global atomics with return, global /
buffer / flat / scratch / image loads -- may write any of its SrcA / SrcB / SrcC registers (VGPRs
or AGPRs).  With --valu-srcc, no VALU instruction may write its SrcC registers either (round 4:
a VALU write into the C input of a chained product 3 wait states after its issue -- the count
hipcc's hazard recognizer pads for this gfx950 form -- gave nondeterministic wrong C rows 12..15;
profiles/r04_mfma_valu_war.txt).  A path is followed for at most LIMIT instructions.
With --valu-all, for a product that may start late -- a chained one (C input from a register: it
waits for its producer in the matrix pipe) or one issued behind it in the same burst -- no VALU
instruction may write ANY of its operands (A, B or C) either: such a product reads them late, after
hipcc's hazard padding, which counts from issue (profiles/r04_mfma_valu_war.txt).
With --no-pk (round 5, the root cause of the rows-12..15 fault): no packed-fp32 VALU arithmetic
(v_pk_add_f32, v_pk_mul_f32, v_pk_fma_f32) anywhere in a kernel that issues MFMAs.  On gfx950 such
an instruction intermittently writes wrong values in lanes 48..63 when the same wave issues
v_mfma_f32_16x16x32_f16 products (tools/probes/pk_hazard4.hip reproduces it in isolation: 0 wrong
without MFMAs in the wave, ~1.7e-4 of packed 8-point DCTs with them; pk_hazard5.hip: an op_sel
swap of a source's halves suffices).  Lanes 48..63 of k_mxs's column pass are blocks 3 / 7 of a
step -- the "C rows 12..15" of rounds 3-5, which every earlier rule only moved around
(DESIGN.md 4.3f).
Usage: python tools/mfma_war_check.py [--valu-srcc | --valu-all] [--no-pk] FILE.s [kernel ...]
(exit 1 on a violation)
"""
import re
import sys

LIMIT = 400
BRANCH = re.compile(r"^s_(c?branch\w*|setpc\w*|cbranch\w*)$")


def regs(s):
    """the register names an operand list mentions: ('v', n) and ('a', n)"""
    out = set()
    for k, a, b in re.findall(r"\b([va])\[(\d+):(\d+)\]", s):
        out |= {(k, i) for i in range(int(a), int(b) + 1)}
    for k, a in re.findall(r"\b([va])(\d+)\b", s):
        out.add((k, int(a)))
    return out


def operands(t):
    p = t.split(None, 1)
    if len(p) < 2:
        return p[0], []
    return p[0], [o.strip() for o in re.split(r",(?![^\[]*\])", p[1])]


def writes_from_memory(op):
    """instructions whose VGPR destination is written when memory returns (asynchronously)"""
    if op.startswith("ds_"):
        return (op.startswith(("ds_read", "ds_bpermute", "ds_permute", "ds_swizzle", "ds_consume",
                               "ds_append")) or "_rtn" in op)
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "load" in op or "atomic" in op
    return op.startswith("image_")


def kernel_body(text, name):
    """(instructions, label -> index) of one kernel"""
    m = re.search(r"^(_Z[^\s:]*\d%sE[^\s:]*):" % re.escape(name), text, re.M)
    if not m:
        return None, None
    end = text.find(".Lfunc_end", m.end())
    ins, labels = [], {}
    for ln in text[m.end():end].splitlines():
        t = ln.split(";")[0].strip()
        if not t:
            continue
        lm = re.match(r"^(\.LBB\w+):", t)
        if lm:
            labels[lm.group(1)] = len(ins)
            continue
        if t.startswith("."):
            continue
        ins.append(t)
    return ins, labels


def successors(ins, labels, j):
    """next instruction indices after ins[j] on any path"""
    op, ops = operands(ins[j])
    if op == "s_endpgm" or op.startswith("s_setpc") or op == "s_trap":
        return []
    if op == "s_branch":
        return [labels[ops[0]]] if ops and ops[0] in labels else []
    out = [j + 1] if j + 1 < len(ins) else []
    if op.startswith("s_cbranch") and ops and ops[0] in labels:
        out.append(labels[ops[0]])
    return out


def delayed(ins, i):
    """MFMA i may start late: it takes its C input from a register (a chained product, which waits
    for its producer in the matrix pipe), or follows one in the same burst of products (no VALU read
    of a product result in between; a wave's products execute in order)"""
    def chained(t):
        _, o = operands(t)
        return len(o) > 3 and bool(regs(o[3]))
    if chained(ins[i]):
        return True
    for j in range(i - 1, max(i - 64, -1), -1):
        t = ins[j]
        op, o = operands(t)
        if op.startswith("v_mfma"):
            if chained(t):
                return True
            continue
        if t.startswith(".LBB") or op.startswith(("s_cbranch", "s_branch", "s_endpgm")):
            return False
        if op.startswith("v_") and o:
            # a VALU read of an earlier product's result ends the burst
            for k in range(j - 1, max(j - 64, -1), -1):
                pk, ok = operands(ins[k])
                if pk.startswith("v_mfma") and regs(ok[0]) & regs(",".join(o[1:])):
                    return False
    return False


def check(ins, labels, valu_srcc=False, valu_all=False):
    bad = []
    for i, t in enumerate(ins):
        op, ops = operands(t)
        if not op.startswith("v_mfma"):
            continue
        src = regs(",".join(ops[1:]))
        srcc = regs(ops[3]) if len(ops) > 3 else set()
        if valu_all and delayed(ins, i):
            srcc = src                     # every operand of a product that may start late
        # paths: (next index, registers whose read implies completion, steps taken)
        stack = [(k, frozenset(regs(ops[0])), 1) for k in successors(ins, labels, i)]
        seen = set()
        found = {}
        while stack:
            j, dst, n = stack.pop()
            if n > LIMIT or (j, dst) in seen:
                continue
            seen.add((j, dst))
            u = ins[j]
            uop, uops = operands(u)
            done = False
            if uop.startswith("v_mfma"):
                # a later product: the matrix pipe completes a wave's MFMAs in issue order, so
                # a read of ITS result implies this one is done too (mx_fence relies on it)
                dst = dst | frozenset(regs(uops[0]))
            elif uops and writes_from_memory(uop):
                hit = regs(uops[0]) & src
                if hit and j not in found:
                    found[j] = (i, j, t, u, sorted(hit))
            elif uop.startswith(("v_", "ds_write", "global_store", "buffer_store", "flat_store",
                                 "scratch_store")) and uops:
                reads = regs(",".join(uops[1:])) if uop.startswith("v_") else regs(",".join(uops))
                done = bool(reads & dst)          # the result is read: the MFMA has completed
                if not done and valu_srcc and uop.startswith("v_") and not uop.startswith("v_readfirstlane"):
                    hit = regs(uops[0]) & srcc
                    if hit and j not in found:
                        found[j] = (i, j, t, u, sorted(hit))
            if not done:
                stack.extend((k, dst, n + 1) for k in successors(ins, labels, j))
        bad.extend(found[j] for j in sorted(found))
    return bad


# every packed VALU operation but the plain move (round 6): the probes showed the fault with
# v_pk_{add,mul,fma}_f32; the 16-bit packed forms were never probed, so they are refused as well
PK_F32 = re.compile(r"^v_pk_(?!mov_b32$)\w+$")


def packed_f32(ins):
    """indices of packed VALU arithmetic instructions (any v_pk_* but v_pk_mov_b32), if the kernel
    issues MFMAs"""
    if not any(t.startswith("v_mfma") for t in ins):
        return []
    return [i for i, t in enumerate(ins) if PK_F32.match(operands(t)[0])]


def main():
    args = sys.argv[1:]
    valu_all = "--valu-all" in args
    valu_srcc = "--valu-srcc" in args or valu_all
    no_pk = "--no-pk" in args
    args = [a for a in args if a not in ("--valu-srcc", "--valu-all", "--no-pk")]
    path = args[0]
    names = args[1:] or ["k_mx", "k_mx422", "k_mx420"]
    text = open(path).read()
    rc = 0
    for n in names:
        ins, labels = kernel_body(text, n)
        if ins is None:
            print(f"{n}: not found")
            rc = 1
            continue
        if no_pk:
            pk = packed_f32(ins)
            print(f"{n}: {sum(1 for x in ins if x.startswith('v_mfma'))} MFMAs, {len(pk)} packed VALU instruction(s)")
            for i in pk[:12]:
                print(f"   at {i}: {ins[i][:72]}")
            rc |= 1 if pk else 0
            continue
        bad = check(ins, labels, valu_srcc, valu_all)
        what = ("load(s) or VALU write(s)" if valu_all else
                "load(s) or VALU write(s) of C inputs" if valu_srcc else "load(s)")
        print(f"{n}: {sum(1 for x in ins if x.startswith('v_mfma'))} MFMAs, {len(bad)} {what} into live MFMA operands")
        for i, j, t, u, hit in bad[:12]:
            print(f"   at {j} after the MFMA at {i}: {t[:64]}\n         {u[:64]}  -> {hit}")
        rc |= 1 if bad else 0
    sys.exit(rc)


if __name__ == "__main__":
    main()
