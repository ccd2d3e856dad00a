#!/usr/bin/env python3
"""Static check of the transposing LDS reads in a gfx950 assembly listing (hipcc -S --cuda-device-only, or
``llvm-objdump -d`` of a code object extracted with ``llvm-objdump --offloading``).

``ds_read_b64_tr_b16`` is issued from inline asm (csrc/include/ddpx_pipe.h frag_tr), which the compiler's
waitcnt pass cannot see.  Every read's destination VGPRs must not be read or written by any instruction
before the next ``s_waitcnt lgkmcnt(0)`` on that path (straight-line scan; basic-block ends stop the scan).

    hipcc -O3 -S --cuda-device-only --offload-arch=gfx950 -Icsrc/include -o x.s csrc/kernels/gemm_pipe.hip
    python tools/check_tr_reads.py x.s
(tests/test_tr_reads.py runs it on the disassembly of the built libddpx_kernels.so.)
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(operand_text):
    out = set()
    for m in REG.finditer(operand_text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main(path):
    lines = open(path).read().splitlines()
    bad, checked = [], 0
    for i, ln in enumerate(lines):
        t = ln.strip()
        if not t.startswith("ds_read_b64_tr_b16"):
            continue
        dst = regs(t.split(None, 1)[1].split(",")[0])
        checked += 1
        for j in range(i + 1, min(i + 400, len(lines))):
            u = lines[j].strip()
            if not u or u.startswith(";") or u.startswith("."):
                continue
            if u.endswith(":") and not u.startswith("0"):  # a label: control may join here, stop
                break
            if u.startswith("s_waitcnt") and "lgkmcnt(0)" in u:
                break
            if u.startswith("ds_read_b64_tr_b16") or u.startswith("s_"):
                continue
            ops = u.split(None, 1)
            if len(ops) < 2:
                continue
            if regs(ops[1]) & dst:
                bad.append((i + 1, j + 1, t, u))
                break
    for b in bad:
        print(f"line {b[0]}: {b[2]}\n  touched at line {b[1]} before lgkmcnt(0): {b[3]}")
    print(f"{checked} transposing reads checked, {len(bad)} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
