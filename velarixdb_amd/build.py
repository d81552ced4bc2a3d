"""Build libvbf.so in-tree for gfx950 (explicit hipcc; the .so travels with the repo snapshot)."""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["vbf_kernels.hip", "vbf_partition.hip", "vbf_partition_rk_a.hip", "vbf_partition_rk_b.hip", "vbf_partition_rk_c.hip", "vbf_partition_rk_d.hip", "vbf_partition_sat.hip", "vbf_partition_k1_a.hip", "vbf_partition_k1_b.hip", "vbf_partition_k1_c.hip", "vbf_probe_part.hip", "vbf_probe_part_rk_a.hip", "vbf_probe_part_rk_b.hip", "vbf_probe_part_rk_c.hip", "vbf_probe_part_rk_d.hip", "vbf_probe_pu.hip", "vbf_probe_pu_rk_a.hip", "vbf_probe_pu_rk_b.hip", "vbf_sst.hip", "vbf_multi.hip", "vbf_multi_part.hip", "vbf_compact.hip", "vbf_api.hip"]
OUT = os.path.join(HERE, "libvbf.so")
ARCH = os.environ.get("VBF_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(path, seen=None):
    """The file and every quoted include it reaches in csrc/ or include/."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path, errors="replace") as f:
        text = f.read()
    for name in _INC.findall(text):
        for d in (os.path.dirname(path), CSRC, os.path.join(HERE, "..", "include")):
            cand = os.path.normpath(os.path.join(d, name))
            if os.path.exists(cand):
                _deps(cand, seen)
                break
    return seen


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [
        os.path.join(HERE, "..", "include", "vbf.h"), __file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, out=OUT, defines=()):
    """One hipcc per translation unit, in parallel, then one link.  `defines` (e.g.
    VBF_ABLATION_BUILD=1 for tools/ablate.py, written to velarixdb_amd/libvbf_ablate.so) build a
    variant library for VBF_LIB; the product is libvbf.so without any."""
    tag = "_".join(d.replace("=", "") for d in defines)
    objdir = os.path.join(HERE, "..", "build", "obj" + ("_" + tag if tag else ""))
    os.makedirs(objdir, exist_ok=True)
    flags = ["--offload-arch=" + ARCH, "-O3", "-std=c++20", "-fPIC", "-Wall"] + ["-D" + d for d in defines]
    procs, objs = [], []
    # an object is current when newer than its source and the headers it includes (transitively,
    # csrc/ and include/); build(force=True) after changing the flags
    for s in SOURCES:
        obj = os.path.join(objdir, s.replace(".hip", ".o"))
        objs.append(obj)
        src = os.path.join(CSRC, s)
        t_dep = max(os.path.getmtime(d) for d in _deps(src))
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > t_dep:
            continue
        cmd = [_hipcc()] + flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((s, subprocess.Popen(cmd, cwd=CSRC)))
    failed = [s for s, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError("hipcc failed for " + ", ".join(failed))
    # every object current (against its own sources, so a header edited while an earlier build ran
    # still recompiles what includes it) and the library newer than all of them: nothing to link
    if not procs and not force and os.path.exists(out) and \
            os.path.getmtime(out) > max(os.path.getmtime(o) for o in objs):
        return out
    cmd = [_hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(out + ".tmp", out)
    return out


EXAMPLES = ("c_host", "memtable_latency", "rust_replay")


def build_examples(verbose=False):
    """examples/*.c: the C ABI from a plain C host (gcc, no Python/torch in that process)."""
    root = os.path.dirname(HERE)
    outs = []
    for name in EXAMPLES:
        src = os.path.join(root, "examples", name + ".c")
        out = os.path.join(root, "examples", name)
        cmd = ["gcc", "-std=c11", "-D_POSIX_C_SOURCE=200809L", "-O2", "-Wall", "-Wextra", "-I",
               os.path.join(root, "include"), src, "-L", HERE, "-lvbf", "-Wl,-rpath,$ORIGIN/../velarixdb_amd",
               "-o", out]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        outs.append(out)
    return outs


ABLATION_LIB = os.path.join(HERE, "libvbf_ablate.so")

if __name__ == "__main__":
    if "--ablation" in sys.argv:
        print(build(verbose=True, out=ABLATION_LIB, defines=("VBF_ABLATION_BUILD=1",)))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
