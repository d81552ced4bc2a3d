"""Per-kernel register / scratch / LDS usage of a built object or library (speed work: a stash that
spilled to scratch, or a VGPR count that drops occupancy, shows here before any GPU run).

usage: python tools/kernel_resources.py [build/obj/vbf_partition.o | velarixdb_amd/libvbf.so] [name filter]

Unbundles the gfx950 code object with clang-offload-bundler and reads the AMDGPU metadata notes
(llvm-readelf --notes): .vgpr_count, .agpr_count, .sgpr_count, .private_segment_fixed_size
(scratch bytes per lane), .group_segment_fixed_size (static LDS).
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(path):
    # host objects / libraries carry the device code as a clang offload bundle in .hip_fatbin
    fd, fb = tempfile.mkstemp(suffix=".fatbin")
    os.close(fd)
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fb, path,
                           os.devnull])
    path = fb
    out = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--list", "--type=o", "--input=" + path],
                         capture_output=True, text=True)
    targets = [t for t in out.stdout.split() if "gfx950" in t]
    for t in targets:
        fd, co = tempfile.mkstemp(suffix=".co")
        os.close(fd)
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--input=" + path, "--output=" + co, "--targets=" + t])
        yield co


def kernels(co):
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True,
                           text=True).stdout
    cur = {}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == "agpr_count" and cur:
            yield cur
            cur = {}
        cur[k] = v
    if cur:
        yield cur


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "velarixdb_amd/libvbf.so"
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for co in code_objects(path):
        for k in kernels(co):
            name = k.get("name", "?")
            if filt and filt not in name:
                continue
            print("vgpr %4s agpr %3s sgpr %3s scratch %4s lds %6s  %s" % (
                k.get("vgpr_count"), k.get("agpr_count"), k.get("sgpr_count"),
                k.get("private_segment_fixed_size"), k.get("group_segment_fixed_size"), name))
        os.unlink(co)


if __name__ == "__main__":
    main()
