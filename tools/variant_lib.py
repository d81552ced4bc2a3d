"""A/B helper: libvbf_var.so = the product objects with some translation units recompiled with extra
compiler flags (e.g. an LLVM scheduler strategy), for tools/ab_lib.sh (AB_LIB=velarixdb_amd/libvbf_var.so).

usage: python tools/variant_lib.py "FLAGS" TU.hip [TU.hip ...]
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "velarixdb_amd"))
import build  # noqa: E402


def main():
    flags, tus = sys.argv[1].split(), sys.argv[2:]
    src_obj = os.path.join(ROOT, "build", "obj")
    var_obj = os.path.join(ROOT, "build", "obj_var")
    os.makedirs(var_obj, exist_ok=True)
    for f in os.listdir(src_obj):
        shutil.copy2(os.path.join(src_obj, f), var_obj)
    procs = []
    for tu in tus:
        cmd = [build._hipcc(), "--offload-arch=" + build.ARCH, "-O3", "-std=c++20", "-fPIC", "-Wall"] + flags + [
            "-c", os.path.join(build.CSRC, tu), "-o", os.path.join(var_obj, tu.replace(".hip", ".o"))]
        print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd, cwd=build.CSRC))
    if any(p.wait() for p in procs):
        raise SystemExit("compile failed")
    out = os.path.join(ROOT, "velarixdb_amd", "libvbf_var.so")
    objs = [os.path.join(var_obj, s.replace(".hip", ".o")) for s in build.SOURCES]
    subprocess.check_call([build._hipcc(), "--offload-arch=" + build.ARCH, "-shared", "-fPIC", "-o", out] + objs)
    print(out)


if __name__ == "__main__":
    main()
