"""Disassemble one kernel of a built object and count its instructions by mnemonic (speed work:
static VALU counts of a kernel variant before any GPU run).

usage: python tools/isa_dump.py OBJ_OR_LIB 'demangled-name substring' [--asm OUT.s]
Prints the matching kernel names, then for the first match: total instructions, VALU / SALU /
LDS / VMEM counts and the 25 most frequent mnemonics.
"""
import collections
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_resources import LLVM, code_objects  # noqa: E402


def disasm(co):
    out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--demangle", "--no-show-raw-insn", co],
                         capture_output=True, text=True).stdout
    funcs, cur, name = {}, [], None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            if name:
                funcs[name] = cur
            name, cur = m.group(1), []
            continue
        s = line.strip()
        if name and s and not s.startswith(";") and not s.startswith("Disassembly"):
            cur.append(s)
    if name:
        funcs[name] = cur
    return funcs


def classify(mn):
    if mn.startswith("v_"):
        return "valu"
    if mn.startswith("s_"):
        return "salu"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    asm_out = sys.argv[sys.argv.index("--asm") + 1] if "--asm" in sys.argv else None
    for co in code_objects(path):
        funcs = disasm(co)
        hits = [n for n in funcs if pat in n]
        for n in hits:
            print("match:", n, len(funcs[n]))
        if not hits:
            continue
        body = funcs[hits[0]]
        if asm_out:
            open(asm_out, "w").write("\n".join(body) + "\n")
        mns = [b.split()[0] for b in body]
        cls = collections.Counter(classify(m) for m in mns)
        print("total", len(mns), dict(cls))
        for mn, c in collections.Counter(mns).most_common(25):
            print("%6d %s" % (c, mn))
        return


if __name__ == "__main__":
    main()
