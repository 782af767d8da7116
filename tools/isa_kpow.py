"""Instruction budget of k_pow (the dominant kernel) from its compiled gfx950 ISA.

Compiles eg_capi.hip exactly as __graft_entry__.build() does, plus --save-temps, takes the device
assembly of k_pow<true, false> (the Montgomery-friendly, variable-time instantiation every verify /
encrypt launch runs), splits it into basic blocks and finds its loops (a backward branch to a label
closes a loop).  The Montgomery multiply and squaring are mont_mul_impl (eg_bignum.hpp:230): a peeled
first CIOS step, then kT = 8 trips of a `#pragma unroll 1` loop whose body is 18 CIOS steps (17 + the
next trip's step 0), then two carry passes.  The two loop bodies with the most v_mad_u64_u32 are the
multiply's and the squaring's trip; this prints their instruction counts by class, per trip and per
CIOS step, and the whole function's counts, so the glue (everything that is not a MAC) can be
attacked class by class.

    python tools/isa_kpow.py [--asm FILE] [--kernel k_powILb1ELb0E]  > profiles/r05_isa_kpow.txt
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

CLASSES = [
    ("mac v_mad_u64_u32", lambda op, line: op == "v_mad_u64_u32"),
    ("dpp moves / ops", lambda op, line: "_dpp" in op or " row_" in line or "quad_perm" in line or "row_newbcast" in line),
    ("64-bit add (v_add_co / v_addc)", lambda op, line: op.startswith(("v_add_co_u32", "v_addc_co_u32", "v_add_co_ci_u32",
                                                                        "v_lshl_add_u64", "v_add_u64"))),
    ("64-bit shift / align (carry split)", lambda op, line: op.startswith(("v_lshrrev_b64", "v_alignbit_b32",
                                                                           "v_lshlrev_b64", "v_lshl_or_b32"))),
    ("32-bit and / bfe / or / shift", lambda op, line: op.startswith(("v_and_b32", "v_bfe_u32", "v_or_b32", "v_lshrrev_b32",
                                                                      "v_lshlrev_b32", "v_and_or_b32", "v_or3_b32",
                                                                      "v_and3_b32", "v_bfi_b32"))),
    ("32-bit add / sub / mul", lambda op, line: op.startswith(("v_add_u32", "v_sub_u32", "v_mul_lo_u32", "v_add3_u32",
                                                               "v_mul_u32_u24", "v_mad_u32_u24", "v_subrev_u32",
                                                               "v_sub_co_u32", "v_subb_co_u32"))),
    ("v_mov / cndmask / readlane", lambda op, line: op.startswith(("v_mov_b32", "v_mov_b64", "v_cndmask", "v_readfirstlane",
                                                                   "v_readlane", "v_writelane", "v_accvgpr", "v_pk_mov"))),
    ("other VALU", lambda op, line: op.startswith("v_")),
    ("LDS (ds_*)", lambda op, line: op.startswith("ds_")),
    ("global / buffer / scalar memory", lambda op, line: op.startswith(("global_", "buffer_", "s_load", "s_buffer", "flat_"))),
    ("s_waitcnt / s_nop / barriers", lambda op, line: op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep"))),
    ("other SALU / branch", lambda op, line: op.startswith("s_")),
]


def classify(op, line):
    for name, f in CLASSES:
        if f(op, line):
            return name
    return "other"


def compile_asm(tmp: Path) -> Path:
    import __graft_entry__ as g
    flags = [f for f in g.HIP_FLAGS if f != "-shared"]
    cmd = [g.HIPCC, *flags, "--save-temps", "-I", str(ROOT / "include"), "-c", "-o", str(tmp / "x.o"),
           str(g.CSRC / "eg_capi.hip")]
    subprocess.run(cmd, check=True, cwd=tmp)
    return next(tmp.glob("*gfx950*.s"))


def function_body(asm: str, key: str):
    m = re.search(r"^(_Z\w*%s\w*):" % re.escape(key), asm, flags=re.M)
    if not m:
        sys.exit(f"no function matching {key}")
    name = m.group(1)
    end = asm.index(".Lfunc_end", m.end())
    return name, asm[m.end():end].splitlines()


def blocks(lines):
    """-> list of (label, [(op, line)]) basic blocks (a block starts at a label)."""
    out, cur, lab = [], [], "entry"
    for ln in lines:
        s = ln.split(";")[0].strip()
        if not s:
            continue
        if re.match(r"^\.?L\w+:", s) or re.match(r"^\w+:", s):
            out.append((lab, cur))
            lab, cur = s[:-1], []
            continue
        if s.startswith("."):
            continue
        cur.append((s.split()[0], s))
    out.append((lab, cur))
    return out


def count(instrs):
    c = collections.Counter(classify(op, line) for op, line in instrs)
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", help="an existing gfx950 .s (default: compile eg_capi.hip)")
    ap.add_argument("--kernel", default="k_powILb1ELb0E")
    a = ap.parse_args()
    if a.asm:
        asm_path = Path(a.asm)
    else:
        tmp = Path(tempfile.mkdtemp(prefix="isa_kpow_"))
        asm_path = compile_asm(tmp)
    asm = asm_path.read_text()
    name, lines = function_body(asm, a.kernel)
    bl = blocks(lines)
    labels = {lab: i for i, (lab, _) in enumerate(bl)}
    # loops: a block whose branch targets a label at or before it
    # loops: a block whose branch targets a label at or before it; the trip loops of mont_mul_impl
    # (`#pragma unroll 1` over the kT = 8 trips) compile to SELF-loops whose body is 17 CIOS steps
    # (steps 1..17 of a trip); the trip's step 0 (the previous trip's tail, `if (s + 1 < kT)`) is the
    # block the loop is entered from
    selfloops = []
    for i, (lab, ins) in enumerate(bl):
        for op, line in ins:
            if (op.startswith("s_cbranch") or op == "s_branch") and line.split()[-1] == lab:
                selfloops.append(i)
    whole = count([x for _, ins in bl for x in ins])
    print(f"k_pow instruction budget: {name}")
    print(f"source: {asm_path.name} (hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize, eg_bignum.hpp kT = 8 lanes x "
          f"kL = 18 limbs of 2^29 per element)")
    print(f"whole function: {sum(whole.values())} static instructions")
    for k, _ in CLASSES:
        if whole[k]:
            print(f"  {k:38s} {whole[k]:6d}")
    print()
    trips = []
    for i in selfloops:
        body = bl[i][1]
        c = count(body)
        if c["mac v_mad_u64_u32"] < 400:
            continue
        kind = "multiply" if c["mac v_mad_u64_u32"] >= 600 else "squaring"
        trips.append((kind, i, c, body))
    valu_keys = [k for k, _ in CLASSES if k not in ("LDS (ds_*)", "global / buffer / scalar memory",
                                                      "s_waitcnt / s_nop / barriers", "other SALU / branch")]
    per_step = {}
    for kind, i, c, body in trips:
        steps = 17
        valu = sum(c[k] for k in valu_keys)
        print(f"{kind}: trip loop {bl[i][0]} = 17 CIOS steps ({len(body)} instructions, {valu} VALU)")
        for k, _ in CLASSES:
            if c[k]:
                print(f"  {k:38s} {c[k]:5d} per 17 steps  {c[k] / steps:7.2f} per step")
        glue = valu - c["mac v_mad_u64_u32"]
        print(f"  VALU per step {valu / steps:.2f}: {c['mac v_mad_u64_u32'] / steps:.2f} MAC + {glue / steps:.2f} glue "
              f"({glue / valu:.1%} of the step's VALU)")
        per_step[kind] = {k: c[k] / steps for k, _ in CLASSES}
        print()
    if "multiply" in per_step and "squaring" in per_step:
        f_sqr = float(os.environ.get("SQR_FRAC", "0.5898"))  # BENCH_r04 squaring_frac
        print(f"per Montgomery op per lane, 144 CIOS steps, squaring fraction {f_sqr} (BENCH_r04):")
        tot = 0.0
        for k in valu_keys:
            v = 144 * ((1 - f_sqr) * per_step["multiply"][k] + f_sqr * per_step["squaring"][k])
            tot += v
            if v:
                print(f"  {k:38s} {v:8.0f}")
        print(f"  {'VALU in the CIOS steps':38s} {tot:8.0f}   (PMC r04o: 5,447 VALU per op per lane in total: the rest")
        print("   is the per-op epilogue -- two carry passes, SQR pre-doubling -- the table / LDS moves and the op")
        print("   program interpreter)")


if __name__ == "__main__":
    main()
