"""ISA-level checks of the built MFMA kernels (CPU: hipcc cross-compiles gfx950 here).

The MFMA operand rule (jpgx_mx.hip, mx_fence; tools/mfma_war_check.py): no load may write a VGPR
that an issued MFMA may still read.  A chained product whose SrcC registers the allocator reuses
for an LDS read gave nondeterministic wrong C rows 12..15 (profiles/r03_mfma_war.txt), which
parity tests only catch by luck -- so the property is checked on the ISA of every build."""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "jpeg-encoder-and-decoder_amd")


def test_mfma_operand_rule(tmp_path):
    asm = tmp_path / "jpgx_mx-gfx950.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-slp-vectorize", "-I" + os.path.join(REPO, "include"), "--cuda-device-only", "-S",
                    os.path.join(PKG, "csrc", "jpgx_mx.hip"), "-o", str(asm)],
                   check=True, capture_output=True)
    names = ["k_mxs", "k_mxs422", "k_mxs420"]     # every __global__ MFMA kernel of the product
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "mfma_war_check.py"), str(asm)] + names,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count(" 0 load(s) into live MFMA operands") == len(names), r.stdout
    # the launched (short-wave) kernels: no VALU write into the C input of a product in flight either
    short = ["k_mxs", "k_mxs422", "k_mxs420"]
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "mfma_war_check.py"), "--valu-all", str(asm)]
                       + short, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count(" 0 load(s) or VALU write(s) into live MFMA operands") == len(short), r.stdout
    # the root cause of the rows-12..15 fault: no packed-fp32 VALU arithmetic in a
    # kernel that issues MFMAs
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "mfma_war_check.py"), "--no-pk", str(asm)]
                       + names, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count(" 0 packed VALU instruction(s)") == len(names), r.stdout
    # and no scratch, no VGPR / SGPR spills
    text = asm.read_text()
    for n in ("k_mxs", "k_mxs422", "k_mxs420"):
        m = re.search(r"\.name:\s+_ZN12_GLOBAL__N_1\d+%sE13jx_xform_args\s*\n(.*?)\.vgpr_spill_count:\s+(\d+)" % n,
                      text, re.S)
        assert m, n
        meta = m.group(1)
        assert int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", meta).group(1)) == 0, n
        assert int(re.search(r"\.sgpr_spill_count:\s+(\d+)", meta).group(1)) == 0, n
        assert int(m.group(2)) == 0, n
    # k_mxs420 issues its fourth step's LDS-DMA from inline asm that sets M0, a register the
    # compiler treats as reserved: every compiler-emitted reader of M0 (a builtin LDS-DMA, or an
    # instruction naming m0 as a source) must follow its own M0 write in the same basic block, with
    # no inline asm in between
    for n in ("k_mxs", "k_mxs422", "k_mxs420"):
        assert _m0_readers_unsafe(text, n) == [], n


def _m0_readers_unsafe(text, kernel):
    m = re.search(r"^(_Z[^\s:]*\d%sE[^\s:]*):" % kernel, text, re.M)
    body = text[m.end():text.find(".Lfunc_end", m.end())].splitlines()
    bad, m0_set, in_asm = [], False, False
    for ln in body:
        t = ln.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm, m0_set = True, False
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if in_asm or not t or t.startswith(";") or t.startswith("."):
            if re.match(r"^\.LBB\w+:", t):
                m0_set = False                 # a new basic block: M0 unknown again
            continue
        ops = t.split(None, 1)
        op, rest = ops[0], (ops[1] if len(ops) > 1 else "")
        dst = rest.split(",")[0].strip()
        if dst == "m0" and op.startswith("s_"):
            m0_set = True
            continue
        reads_m0 = "_lds_" in op or op.endswith("_lds") or re.search(r"\bm0\b", rest) is not None
        if reads_m0 and not m0_set:
            bad.append(t)
    return bad


def test_mfma_operand_rule_catches_a_violation(tmp_path):
    """the checker itself: an LDS read into the SrcC of a chained MFMA before its result is read"""
    s = tmp_path / "fake.s"
    s.write_text("\n".join([
        "_ZN12_GLOBAL__N_14k_mxE13jx_xform_args:",
        "\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0",
        "\tv_mfma_f32_16x16x32_f16 v[12:15], v[0:3], v[4:7], v[8:11]",
        "\tds_read_b64 v[8:9], v20",
        "\tv_add_f32_e32 v30, v12, v13",
        ".Lfunc_end0:", ""]))
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "mfma_war_check.py"), str(s), "k_mx"],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "1 load(s)" in r.stdout, r.stdout


def _check_fake(tmp_path, lines):
    s = tmp_path / "fake.s"
    s.write_text("\n".join(["_ZN12_GLOBAL__N_14k_mxE13jx_xform_args:"] + lines + [".Lfunc_end0:", ""]))
    return subprocess.run([sys.executable, os.path.join(REPO, "tools", "mfma_war_check.py"), str(s), "k_mx"],
                          capture_output=True, text=True)


def test_mfma_operand_rule_follows_branches_and_back_edges(tmp_path):
    """the checker walks the control-flow graph: a load reached only through a taken branch, or
    only around the loop back-edge (the next iteration's first loads into the previous MFMA's
    operands), is a violation; the same load after a read of the result is not"""
    taken = _check_fake(tmp_path, [
        "\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0",
        "\ts_cbranch_vccnz .LBB0_2",
        "\tv_add_f32_e32 v30, v8, v9",
        "\ts_endpgm",
        ".LBB0_2:",
        "\tds_bpermute_b32 v4, v20, v21",
        "\ts_endpgm"])
    assert taken.returncode == 1 and "1 load(s)" in taken.stdout, taken.stdout
    back = _check_fake(tmp_path, [
        ".LBB0_1:",
        "\tds_read_b128 v[0:3], v40",
        "\ts_waitcnt lgkmcnt(0)",
        "\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0",
        "\ts_add_u32 s0, s0, 1",
        "\ts_cbranch_scc1 .LBB0_1",
        "\tv_add_f32_e32 v30, v8, v9",
        "\ts_endpgm"])
    assert back.returncode == 1 and "1 load(s)" in back.stdout, back.stdout
    ok = _check_fake(tmp_path, [
        ".LBB0_1:",
        "\tds_read_b128 v[0:3], v40",
        "\ts_waitcnt lgkmcnt(0)",
        "\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0",
        "\tv_mfma_f32_16x16x32_f16 v[12:15], v[0:3], v[4:7], 0",
        "\tv_readfirstlane_b32 s2, v15",
        "\ts_cbranch_scc1 .LBB0_1",
        "\ts_endpgm"])
    assert ok.returncode == 0, ok.stdout


def test_mfma_operand_rule_covers_agprs_and_returning_atomics(tmp_path):
    r = _check_fake(tmp_path, [
        "\tv_mfma_f32_16x16x32_f16 a[8:11], v[0:3], v[4:7], a[8:11]",
        "\tglobal_atomic_add_f32 a8, v[20:21], v22, off sc0",
        "\tv_accvgpr_read_b32 v30, a8"])
    assert r.returncode == 1 and "1 load(s)" in r.stdout, r.stdout


def test_mfma_valu_srcc_rule(tmp_path):
    """--valu-srcc: a VALU write into the C input of a chained product before its result (or a
    later product's) is read is a violation (the round-4 rows-12..15 fault,
    profiles/r04_mfma_valu_war.txt); the same write after the read is not; without the flag the
    load-only rule ignores it"""
    lines = [
        "\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0",
        "\tv_mfma_f32_16x16x32_f16 v[12:15], v[0:3], v[4:7], v[8:11]",
        "\ts_nop 0",
        "\tv_pk_add_f32 v[8:9], v[20:21], v[22:23]",
        "\tv_add_f32_e32 v30, v12, v13"]
    s = tmp_path / "fake.s"
    s.write_text("\n".join(["_ZN12_GLOBAL__N_14k_mxE13jx_xform_args:"] + lines + [".Lfunc_end0:", ""]))
    tool = os.path.join(REPO, "tools", "mfma_war_check.py")
    bad = subprocess.run([sys.executable, tool, "--valu-srcc", str(s), "k_mx"], capture_output=True, text=True)
    assert bad.returncode == 1 and " 1 load(s) or VALU write(s)" in bad.stdout, bad.stdout
    plain = subprocess.run([sys.executable, tool, str(s), "k_mx"], capture_output=True, text=True)
    assert plain.returncode == 0, plain.stdout
    lines[2:4] = ["\tv_add_f32_e32 v30, v12, v13", "\tv_pk_add_f32 v[8:9], v[20:21], v[22:23]"]
    s.write_text("\n".join(["_ZN12_GLOBAL__N_14k_mxE13jx_xform_args:"] + lines + [".Lfunc_end0:", ""]))
    ok = subprocess.run([sys.executable, tool, "--valu-srcc", str(s), "k_mx"], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stdout


def test_mfma_chained_operand_rule(tmp_path):
    """--valu-all: a chained product (C input from a register) may start late, so a VALU write into
    its A operand before a result is read is a violation; the same write after an independent
    product (C = 0) is not (hipcc's padding holds for it)"""
    tool = os.path.join(REPO, "tools", "mfma_war_check.py")
    s = tmp_path / "fake.s"

    def run(lines):
        s.write_text("\n".join(["_ZN12_GLOBAL__N_14k_mxE13jx_xform_args:"] + lines + [".Lfunc_end0:", ""]))
        return subprocess.run([sys.executable, tool, "--valu-all", str(s), "k_mx"], capture_output=True, text=True)

    chained = run([
        "\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0",
        "\tv_mfma_f32_16x16x32_f16 v[12:15], v[16:19], v[4:7], v[8:11]",
        "\ts_nop 2",
        "\tv_perm_b32 v16, s0, v20, v21",
        "\tv_add_f32_e32 v30, v12, v13"])
    assert chained.returncode == 1 and " 1 load(s) or VALU write(s)" in chained.stdout, chained.stdout
    independent = run([
        "\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0",
        "\ts_nop 2",
        "\tv_perm_b32 v0, s0, v20, v21",
        "\tv_add_f32_e32 v30, v8, v9"])
    assert independent.returncode == 0, independent.stdout


# The acc[1] column pass right after the Cr products of the round-4b "bgl" reproducer (B operands from
# global memory at the wave's top: 20/20 launches wrong, gpurun_out/r6a), k_mxs step 0 -- every build
# of rounds 3-5 that showed the rows-12..15 fault had this form (packed fp32 after the wave's MFMAs).
_BGL_EXCERPT = [
    "\tv_mfma_f32_16x16x32_f16 v[74:77], v[46:49], v[2:5], 0",
    "\tv_mfma_f32_16x16x32_f16 v[42:45], v[42:45], v[6:9], 0",
    "\tv_mfma_f32_16x16x32_f16 v[38:41], v[46:49], v[6:9], 0",
    "\tv_add_f32_e64 v0, v60, v64",
    "\tv_add_f32_e64 v1, v61, v65",
    "\tv_pk_add_f32 v[46:47], v[58:59], v[62:63]",
    "\tv_pk_add_f32 v[48:49], v[52:53], v[56:57]",
    "\tv_pk_add_f32 v[50:51], v[50:51], v[54:55]",
    "\tv_pk_add_f32 v[52:53], v[46:47], v[48:49] op_sel:[0,1] op_sel_hi:[1,0]",
    "\tv_pk_fma_f32 v[52:53], v[46:47], s[12:13], v[46:47] op_sel:[1,0,0] op_sel_hi:[1,1,0]",
    "\ts_endpgm"]


def test_no_packed_fp32_rule(tmp_path):
    """--no-pk: packed-fp32 arithmetic in a kernel that issues MFMAs is rejected (the recorded failing
    build's column pass is), its scalar form passes, and a kernel without MFMAs may use packed fp32"""
    tool = os.path.join(REPO, "tools", "mfma_war_check.py")
    s = tmp_path / "fake.s"

    def run(lines):
        s.write_text("\n".join(["_ZN12_GLOBAL__N_14k_mxE13jx_xform_args:"] + lines + [".Lfunc_end0:", ""]))
        return subprocess.run([sys.executable, tool, "--no-pk", str(s), "k_mx"], capture_output=True, text=True)

    bad = run(_BGL_EXCERPT)
    assert bad.returncode == 1 and " 5 packed VALU instruction(s)" in bad.stdout, bad.stdout
    scalar = run(_BGL_EXCERPT[:5] + ["\tv_add_f32_e32 v46, v58, v62", "\tv_add_f32_e32 v47, v59, v63",
                                     "\tv_fmac_f32_e32 v52, 0x3f5906bd, v46", "\ts_endpgm"])
    assert scalar.returncode == 0, scalar.stdout
    no_mfma = run(["\tv_pk_fma_f32 v[0:1], v[2:3], v[4:5], v[6:7] op_sel_hi:[0,1,1]", "\ts_endpgm"])
    assert no_mfma.returncode == 0, no_mfma.stdout
    moves = run(["\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0",
                 "\tv_pk_mov_b32 v[20:21], v[22:23], v[22:23] op_sel:[1,0]", "\ts_endpgm"])
    assert moves.returncode == 0, moves.stdout


def test_no_packed_fp32_rule_rejects_recorded_failing_builds():
    """every recorded failing build of the MFMA kernels fails --no-pk, whatever the other rules said
    of it.  Committed excerpts (tests/isa_fixtures/: k_mxs of the round-4b variants bgl -- B from
    global memory --, w1 -- one-wave workgroups -- and ucc -- the compact-table exact pass without
    its lgkmcnt(0) --, from 40 lines before the first MFMA to 200 after the first packed op) always
    run; the whole variant ISA (build/variants, gitignored, tools/build_variants.sh over
    tools/probes/jpgx_mx_r5_knobs.patch (git history: 63924df)) is checked too where this checkout has it."""
    tool = os.path.join(REPO, "tools", "mfma_war_check.py")
    fix = os.path.join(REPO, "tests", "isa_fixtures")
    for name in ("bgl", "w1", "ucc"):
        f = os.path.join(fix, name + "_k_mxs.isa")
        r = subprocess.run([sys.executable, tool, "--no-pk", f, "k_mxs"], capture_output=True, text=True)
        assert r.returncode == 1 and "16 MFMAs" in r.stdout and "packed VALU" in r.stdout, (name, r.stdout)
    vdir = os.path.join(PKG, "build", "variants")
    for name in ("bgl", "bglpad", "w1", "ucc", "dump3"):
        f = os.path.join(vdir, name + ".s")
        if os.path.exists(f):
            r = subprocess.run([sys.executable, tool, "--no-pk", f, "k_mxs"], capture_output=True, text=True)
            assert r.returncode == 1 and "packed VALU" in r.stdout, (name, r.stdout)


def test_no_packed_rule_covers_16bit_packed_forms(tmp_path):
    """the 16-bit packed VALU forms were never probed after MFMAs, so --no-pk refuses
    them too; only v_pk_mov_b32 (a move, used by the compiler to pair registers) passes"""
    tool = os.path.join(REPO, "tools", "mfma_war_check.py")
    s = tmp_path / "fake.s"
    mfma = "\tv_mfma_f32_16x16x32_f16 v[8:11], v[0:3], v[4:7], 0"
    for op in ("v_pk_add_f16 v20, v21, v22", "v_pk_fma_f16 v20, v21, v22, v23", "v_pk_mul_lo_u16 v20, v21, v22",
               "v_pk_add_u16 v20, v21, v22", "v_pk_mul_f32 v[20:21], v[22:23], v[24:25]"):
        s.write_text("\n".join(["_ZN12_GLOBAL__N_14k_mxE13jx_xform_args:", mfma, "\t" + op, "\ts_endpgm",
                                ".Lfunc_end0:", ""]))
        r = subprocess.run([sys.executable, tool, "--no-pk", str(s), "k_mx"], capture_output=True, text=True)
        assert r.returncode == 1 and " 1 packed VALU" in r.stdout, (op, r.stdout)


def test_m0_rule_catches_a_reader_after_asm():
    fake = """_ZN12_GLOBAL__N_18k_fakeE13jx_xform_args:
\ts_mov_b32 m0, s4
\tglobal_load_lds_dwordx4 v[2:3], off
\t;;#ASMSTART
\ts_mov_b32 m0, s9
\tglobal_load_lds_dwordx4 v[4:5], off
\t;;#ASMEND
\tglobal_load_lds_dwordx4 v[6:7], off
\ts_add_i32 m0, s4, 0x400
\tglobal_load_lds_dwordx4 v[6:7], off
.LBB0_1:
\tglobal_load_lds_dword v[8:9], off
\tv_readlane_b32 s2, v1, m0
.Lfunc_end0:
"""
    bad = _m0_readers_unsafe(fake, "k_fake")
    assert bad == ["global_load_lds_dwordx4 v[6:7], off", "global_load_lds_dword v[8:9], off",
                   "v_readlane_b32 s2, v1, m0"], bad
