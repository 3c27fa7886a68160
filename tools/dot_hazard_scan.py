#!/usr/bin/env python3
"""Dot-product result hazard check for the gfx950 kernels (no GPU needed).

gfx950 runs the v_dot* instructions like the matrix-core ones: another VALU instruction may read
a dot's destination only three wait states after the dot.  The compiler pads the instructions it
emits, but not the ones inside inline assembly, which is how the gather's int8 facing prefilter
issues its v_dot4_i32_i8 (orx_kernels.hip sdot4x4: four dots and an s_nop 2 in one block).  A
read that comes too early sees the old register value (measured: the two-hit-point gather variant,
whose schedule read a dot one instruction later, dropped photons; profiles/r05h_*).

    python tools/dot_hazard_scan.py FILE.s|FILE.dis ...     # gfx950 assembly or llvm-objdump -d text
    python tools/dot_hazard_scan.py --build                 # compile the csrc sources that issue dots

Prints every dot whose destination is read, or whose block branches, within fewer than three wait
states (each instruction one, s_nop N N + 1), and exits 1 if there is one."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "oppositerenderer_amd", "csrc")
WAIT = 3
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-fno-fast-math", "-fno-slp-vectorize", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
         "--offload-device-only", "-S"]
DOT = re.compile(r"^(v_dot\w*)\s+(v\d+),")


def _instructions(lines):
    """(line number, mnemonic, operand text) of every instruction, comments and labels dropped"""
    for i, line in enumerate(lines):
        t = line.split("//")[0].split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        parts = t.split(None, 1)
        yield i, parts[0], parts[1] if len(parts) > 1 else ""


def _reads(operands, reg):
    """does an instruction's source list name VGPR `reg` (alone or inside a v[a:b] range)"""
    n = int(reg[1:])
    srcs = operands.split(",")[1:]
    for s in srcs:
        for m in re.finditer(r"\bv(\d+)\b", s):
            if int(m.group(1)) == n:
                return True
        for m in re.finditer(r"\bv\[(\d+):(\d+)\]", s):
            if int(m.group(1)) <= n <= int(m.group(2)):
                return True
    return False


def scan_text(text):
    """[(line, dot instruction, offending instruction, wait states)] of one assembly text"""
    lines = text.splitlines()
    ins = list(_instructions(lines))
    bad, ndots = [], 0
    for k, (ln, mnem, ops) in enumerate(ins):
        m = DOT.match(mnem + " " + ops)
        if not m or mnem.startswith("v_dot4c") or mnem.startswith("v_dot2c"):
            continue  # the accumulator (VOP2) forms are compiler-emitted and padded by it
        ndots += 1
        dst, ws = m.group(2), 0
        for ln2, mnem2, ops2 in ins[k + 1:]:
            if ws >= WAIT:
                break
            if mnem2.startswith("s_branch") or mnem2.startswith("s_cbranch") or mnem2.startswith("s_setpc") or \
                    mnem2 == "s_endpgm" or _reads(ops2, dst):
                bad.append((ln + 1, (mnem + " " + ops).strip(), (mnem2 + " " + ops2).strip(), ws))
                break
            ws += int(ops2, 0) + 1 if mnem2 == "s_nop" else 1
    return ndots, bad


def build_and_scan():
    """compile every csrc source whose text issues a v_dot to gfx950 assembly and scan it"""
    results = {}
    for name in sorted(os.listdir(CSRC)):
        if not name.endswith(".hip"):
            continue
        src = os.path.join(CSRC, name)
        if "v_dot" not in open(src).read():
            continue
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "k.s")
            subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + ["-o", out, src], check=True, capture_output=True)
            results[name] = scan_text(open(out).read())
    return results


def main(argv):
    if argv[:1] == ["--build"]:
        results = build_and_scan()
    else:
        results = {f: scan_text(open(f).read()) for f in argv}
    worst = 0
    for f, (ndots, bad) in results.items():
        print("%s: %d inline dots, %d read or left before %d wait states" % (f, ndots, len(bad), WAIT))
        for b in bad[:20]:
            print("  line %d: %s -> %s (%d)" % b)
        worst = max(worst, len(bad))
    return 1 if worst else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
