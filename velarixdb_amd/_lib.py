"""ctypes binding of the C ABI in include/vbf.h (libvbf.so, built in-tree for gfx950).

There is no fallback: if the shared library is missing or fails to load, importing this
module raises, so no product path can silently run on the CPU.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# VBF_LIB selects an alternative in-tree build (A/B of compile-time variants); default libvbf.so
LIB_PATH = os.environ.get("VBF_LIB") or os.path.join(_HERE, "libvbf.so")

VBF_OK = 0
VBF_EINVAL = -1
VBF_EHIP = -2
VBF_ENOMEM = -3
VBF_ENODEV = -4
VBF_EDIVZERO = -5
VBF_DEVICE_HOST = -1
VBF_DEVICE_AUTO = -2  # the library places the filter (round-robin over the devices)
VBF_MIRROR_OFF, VBF_MIRROR_LAZY, VBF_MIRROR_EAGER = 0, 1, 2
VBF_EXT_NONE = 0xFFFFFFFFFFFFFFFF  # vbf_filter_serialize_ext: the reference's 16 bytes only

VBF_BUILD_AUTO = 0
VBF_BUILD_ATOMIC = 1
VBF_BUILD_PARTITIONED = 2
VBF_BUILD_FRESH = 0x100  # OR into a build strategy: BloomFilter::new fused with the build (vbf.h)

_u8p = ctypes.c_void_p  # raw pointers (host or device) travel as integers
_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_int = ctypes.c_int
_dbl = ctypes.c_double
_vp = ctypes.c_void_p

# name -> (restype, argtypes); must cover every function declared in include/vbf.h
SIGNATURES = {
    "vbf_version": (ctypes.c_char_p, []),
    "vbf_last_error": (ctypes.c_char_p, []),
    "vbf_device_count": (_int, [ctypes.POINTER(_int)]),
    "vbf_profile_enable": (_int, [_int]),
    "vbf_profile_read": (_int, [_vp, _vp, _int]),
    "vbf_num_bits": (_u32, [_u64, _dbl]),
    "vbf_num_hash_functions": (_u32, [_u32, _u32]),
    "vbf_size": (_int, [_dbl, _u64, ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "vbf_meta_serialize": (None, [_u32, _u32, _dbl, _vp]),
    "vbf_meta_parse": (_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_u32), ctypes.POINTER(_u32),
                              ctypes.POINTER(_dbl)]),
    "vbf_build_dev": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _u32, _vp, _vp]),
    "vbf_build_dev_ex": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _u32, _vp, _int, _vp]),
    "vbf_build_workspace_bytes": (_u64, [_u64, _u32, _u32]),
    "vbf_release_workspaces": (_int, []),
    "vbf_probe_dev": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _u32, _vp, _vp, _vp]),
    "vbf_probe_count_dev": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _u32, _vp, _vp, _vp]),
    "vbf_probe_dev_ex": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _u32, _vp, _vp, _int, _vp]),
    "vbf_probe_count_dev_ex": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _u32, _vp, _vp, _int, _vp]),
    "vbf_hashes_dev": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _vp, _vp]),
    "vbf_or_words_dev": (_int, [_vp, _vp, _u64, _vp]),
    "vbf_or_fold_dev": (_int, [_vp, _vp, _u64, _u32, _u64, _vp]),
    "vbf_popcount_dev": (_int, [_vp, _u64, _vp, _vp]),
    "vbf_gen_fixed_dev": (_int, [_u64, _u64, _u64, _u32, _vp, _vp]),
    "vbf_gen_var_dev": (_int, [_u64, _u64, _u64, _vp, _vp, _vp]),
    "vbf_build_host": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _u32, _vp, _u64, _int]),
    "vbf_probe_host": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _u32, _vp, _u64, _vp, _int]),
    "vbf_build_shards_host": (_int, [_vp, _u64, _vp, _int]),
    "vbf_filter_new": (_int, [_dbl, _u64, _int, ctypes.POINTER(_vp)]),
    "vbf_filter_default": (_int, [_int, ctypes.POINTER(_vp)]),
    "vbf_filter_new_sized": (_int, [_u32, _u32, _dbl, _int, ctypes.POINTER(_vp)]),
    "vbf_filter_recover": (_int, [_vp, ctypes.c_size_t, _int, ctypes.POINTER(_vp)]),
    "vbf_filter_clone": (_int, [_vp, ctypes.POINTER(_vp)]),
    "vbf_filter_free": (None, [_vp]),
    "vbf_filter_set_host": (_int, [_vp, _vp, _vp, _u64, _u64, _int]),
    "vbf_filter_set_dev": (_int, [_vp, _vp, _vp, _u64, _u64, _int, _vp]),
    "vbf_filter_set_host_async": (_int, [_vp, _vp, _vp, _u64, _u64, _int, _vp, _vp]),
    "vbf_filter_sync": (_int, [_vp]),
    "vbf_filter_busy": (_int, [_vp]),
    "vbf_filter_stream_wait": (_int, [_vp, _vp]),
    "vbf_filter_stream_record": (_int, [_vp, _vp]),
    "vbf_filter_set_mirror": (_int, [_vp, _int]),
    "vbf_filter_serialize_ext": (_int, [_vp, _vp, _vp, _u64, _u64, _int, _vp, _u64, ctypes.POINTER(_u64)]),
    "vbf_filter_recover_ext": (_int, [_vp, _u64, _int, ctypes.POINTER(_vp), ctypes.POINTER(_int)]),
    "vbf_filter_contains_host": (_int, [_vp, _vp, _vp, _u64, _u64, _int, _vp]),
    "vbf_filter_contains_dev": (_int, [_vp, _vp, _vp, _u64, _u64, _int, _vp, _vp]),
    "vbf_filter_num_bits": (_u32, [_vp]),
    "vbf_filter_num_elements": (_u32, [_vp]),
    "vbf_filter_num_hash_functions": (_u32, [_vp]),
    "vbf_filter_false_positive_rate": (_dbl, [_vp]),
    "vbf_filter_device": (_int, [_vp]),
    "vbf_filter_host_bytes": (_u64, [_vp]),
    "vbf_filter_words_dev": (_vp, [_vp]),
    "vbf_filter_words_dev_read": (_vp, [_vp]),
    "vbf_filter_set_sst_entries": (_int, [_vp, _u64]),
    "vbf_filter_sst_entries": (_u64, [_vp]),
    "vbf_filter_take_restored": (_int, [_vp]),
    "vbf_filter_set_num_elements": (_int, [_vp, _u32]),
    "vbf_filter_migrate": (_int, [_vp, _int]),
    "vbf_filter_serialize": (_int, [_vp, _vp]),
    "vbf_filter_clear": (_int, [_vp, ctypes.POINTER(_vp)]),
    "vbf_filter_words_to_host": (_int, [_vp, _vp, _u64]),
    "vbf_filter_words_from_host": (_int, [_vp, _vp, _u64]),
    "vbf_gen_sst_fixed_dev": (_int, [_u64, _u64, _u64, _u32, _vp, _vp, _vp]),
    "vbf_multi_probe_dev": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _vp, _vp, _vp, _vp, _vp]),
    "vbf_multi_probe_host": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _vp, _vp, _vp, _vp]),
    "vbf_multi_probe_host_grouped": (_int, [_vp, _vp, _u64, _u64, _int, _u32, _vp, _vp, _vp, _vp, _vp]),
    "vbf_compact_merge_dev": (_int, [_vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _u64, _int, _u64, _u64, _u64,
                                      _vp, _vp, _vp, _vp, _vp, _vp]),
    "vbf_compact_merge_host": (_int, [_vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _u64, _int, _u64, _u64, _u64,
                                       _vp, _vp, _vp, _vp, _vp, _int]),
    "vbf_gather_entries_dev": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _u64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "vbf_sst_index_blocks": (_int, [_vp, _u64, _vp, _u64, _vp]),
    "vbf_sst_decode_dev": (_int, [_vp, _u64, _vp, _u64, _vp, _u64, _vp, _vp, _vp, _vp, _u64, _vp, _vp]),
    "vbf_sst_decode_host": (_int, [_vp, _u64, _vp, _u64, _vp, _u64, _vp, _vp, _vp, _vp, _u64, _vp, _int]),
    "vbf_filter_rebuild_from_sst_dev": (_int, [_vp, _vp, _u64, _vp, _u64, _vp, _vp]),
    "vbf_filter_rebuild_from_sst_host": (_int, [_vp, _vp, _u64, _vp, _u64, _vp]),
}


class VbfError(RuntimeError):
    """A nonzero status from the C ABI, carrying vbf_last_error()."""

    def __init__(self, fn, code, msg):
        super().__init__("%s failed (%d): %s" % (fn, code, msg))
        self.code = code


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("velarixdb_amd: %s is missing; run __graft_entry__.build() "
                          "(hipcc --offload-arch=gfx950). There is no CPU fallback." % LIB_PATH)
    # One HIP runtime per process.  libvbf.so needs libamdhip64.so.7; PyTorch-ROCm ships its own
    # copy under that soname.  Loaded after torch, libvbf binds to torch's copy; loaded first,
    # it pulls in /opt/rocm's and a later `import torch` binds to that one and finds no GPU.
    # So when torch is installed it is imported (not initialised) first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(fn_name, rc):
    if rc != VBF_OK:
        raise VbfError(fn_name, rc, lib.vbf_last_error().decode(errors="replace"))
    return rc


def call(fn_name, *args):
    return check(fn_name, getattr(lib, fn_name)(*args))


def device_count():
    c = _int(0)
    rc = lib.vbf_device_count(ctypes.byref(c))
    return c.value if rc == VBF_OK else 0


PHASES = ("tile_sort", "transpose", "seg_or", "atomic_build", "probe", "sst_walk", "sst_scan", "sst_emit",
          "merge_levels", "fold", "select", "probe_pack", "probe_seg", "probe_out")


def profile_read():
    """{phase: (total_ms, launches)} since the last read (needs vbf_profile_enable(1))."""
    n = len(PHASES)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_uint64 * n)()
    call("vbf_profile_read", ms, cnt, n)
    return {p: (ms[i], cnt[i]) for i, p in enumerate(PHASES)}
