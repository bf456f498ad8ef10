"""ctypes binding of libsyncfast_amd.so (the C-ABI in include/syncfast_amd.h).

The library is built in-tree (``syncfast_amd/lib/libsyncfast_amd.so``) by
``__graft_entry__.build()`` / ``make -C syncfast_amd/csrc``.  There is no
Python or CPU fallback: if the library is missing, importing the compute
entry points raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SF_LIB overrides the library path (tuning builds, scripts/tune*.py only).
LIB_PATH = os.environ.get("SF_LIB") or os.path.join(_HERE, "lib", "libsyncfast_amd.so")

SF_OK = 0
SF_EIO = -5
SF_EAGAIN = -11
SF_ENOMEM = -12
SF_ENODEV = -19
SF_EINVAL = -22
SF_ENOSPC = -28
SF_ERANGE = -34
SF_ETIMEDOUT = -110

HASH_DIGEST_LEN = 20
MAX_BLOCK_SIZE = 32 << 20

# Every symbol include/syncfast_amd.h declares (checked by the CPU tests).
EXPORTED = (
    "sf_version", "sf_strerror", "sf_device_count", "sf_set_device", "sf_release_host_cache",
    "sf_index_device_fixed", "sf_index_device_blocks", "sf_index_device_batch",
    "sf_index_device_fixed_weak", "sf_index_device_blocks_weak", "sf_index_device_batch_chained",
    "sf_index_device_batch_chained_cols",
    "sf_fill_splitmix_device", "sf_wire_file_blocks_device", "sf_wire_blocks_device", "sf_wire_blocks_fd", "sf_wire_file_blocks_fd", "sf_index_buffer", "sf_index_buffer_blocks", "sf_index_file_blocks", "sf_file_stamp_fd", "sf_index_fd_blocks", "sf_index_fd_fixed", "sf_index_file", "sf_index_file_range", "sf_index_fd", "sf_free_rows", "sf_index_files",
    "sf_index_fds_blocks", "sf_cut_fd", "sf_free_cuts", "sf_index_fd_cut", "sf_shard_range", "sf_index_file_multi",
    "sf_index_device_multi", "sf_index_device_multi_ex",
    "sf_blocks_hash", "sf_blocks_hash_sigs", "sf_sha1_host",
    "sf_block_set_build", "sf_block_set_lookup", "sf_block_set_free",
)
# Test hooks (include/syncfast_amd_test.h): knobs latched at load, route counters,
# the explicit-list processing order.
EXPORTED_TEST = ("sf_test_set_knob", "sf_test_get_knob", "sf_test_get_stat", "sf_test_table_order",
                 "sf_test_table_order_bits",
                 "sf_test_set_read_hook", "sf_test_xcd_litmus", "sf_test_multi_plan")


class SfError(OSError):
    """A negative SF_E* return code (maps to the reference's Error::Io)."""

    def __init__(self, code: int, what: str = ""):
        msg = _strerror(code)
        super().__init__(-code, f"{what}: {msg}" if what else msg)
        self.code = code


class BlockSig(ctypes.Structure):
    """sf_block_sig: (offset, size, sha1[20]) -- 32 bytes."""
    _fields_ = [("offset", ctypes.c_uint64), ("size", ctypes.c_uint32),
                ("sha1", ctypes.c_uint8 * 20)]


class ChainJob(ctypes.Structure):
    """sf_chain_job: one blocks_hash chain job of an earlier batch."""
    _fields_ = [("d_digests", ctypes.c_void_p), ("n_files", ctypes.c_uint32), ("part", ctypes.c_uint32),
                ("blocks", ctypes.c_uint64), ("d_state", ctypes.c_void_p), ("d_hashes", ctypes.c_void_p)]


class FileStamp(ctypes.Structure):
    """sf_file_stamp: fstat's identity of an open file's contents."""
    _fields_ = [("dev", ctypes.c_uint64), ("ino", ctypes.c_uint64), ("size", ctypes.c_uint64),
                ("nlink", ctypes.c_uint64), ("mtime_sec", ctypes.c_int64), ("mtime_nsec", ctypes.c_int64),
                ("ctime_sec", ctypes.c_int64), ("ctime_nsec", ctypes.c_int64)]


def same_stamp(a: FileStamp, b: FileStamp) -> bool:
    """The library's stamp comparison (include/syncfast_amd.h): dev, ino, size
    and mtime equal, and ctime too unless the link count changed."""
    return (a.dev, a.ino, a.size, a.mtime_sec, a.mtime_nsec) == (b.dev, b.ino, b.size, b.mtime_sec, b.mtime_nsec) \
        and (a.nlink != b.nlink or (a.ctime_sec, a.ctime_nsec) == (b.ctime_sec, b.ctime_nsec))


# sf_test_read_hook_fn: void (*)(void* arg, uint64_t window)
READ_HOOK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64)


class FileDesc(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("len", ctypes.c_uint64)]


_lib = None


def _declare(L: ctypes.CDLL) -> None:
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    L.sf_version.restype = ctypes.c_char_p
    L.sf_version.argtypes = []
    L.sf_strerror.restype = ctypes.c_char_p
    L.sf_strerror.argtypes = [i32]
    L.sf_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    L.sf_set_device.argtypes = [i32]
    L.sf_release_host_cache.argtypes = []
    L.sf_index_device_fixed.argtypes = [vp, u64, u32, vp, u64, pu64, vp]
    L.sf_index_device_blocks.argtypes = [vp, u64, vp, vp, u64, vp, vp, vp]
    L.sf_index_device_fixed_weak.argtypes = [vp, u64, u32, vp, vp, u64, pu64, vp]
    L.sf_index_device_blocks_weak.argtypes = [vp, u64, vp, vp, u64, vp, vp, vp, vp]
    L.sf_index_device_batch_chained.argtypes = [vp, u32, u64, u32, vp, ctypes.POINTER(ChainJob), u32, vp]
    L.sf_index_device_batch_chained_cols.argtypes = [vp, u32, u64, u32, u64, u64, vp, ctypes.POINTER(ChainJob), u32,
                                                     vp]
    L.sf_index_device_batch.argtypes = [vp, u64, ctypes.POINTER(FileDesc), u32, u32, vp, u64, vp, vp, pu64, vp, vp]
    L.sf_fill_splitmix_device.argtypes = [vp, u64, u64, u64, vp]
    L.sf_wire_file_blocks_device.argtypes = [vp, u64, u32, u64, vp, u64, pu64, vp]
    L.sf_wire_blocks_device.argtypes = [vp, vp, u64, vp, u64, pu64, vp]
    L.sf_wire_blocks_fd.argtypes = [vp, vp, u64, i32, pu64, vp]
    L.sf_wire_file_blocks_fd.argtypes = [vp, u64, u32, u64, i32, pu64, vp]
    L.sf_index_buffer.argtypes = [vp, u64, u32, ctypes.POINTER(BlockSig), u64, pu64]
    L.sf_index_buffer_blocks.argtypes = [vp, u64, vp, vp, u64, ctypes.POINTER(BlockSig), vp]
    L.sf_index_file_blocks.argtypes = [ctypes.c_char_p, vp, vp, u64, ctypes.POINTER(BlockSig), vp]
    L.sf_file_stamp_fd.argtypes = [i32, ctypes.POINTER(FileStamp)]
    L.sf_index_fd_blocks.argtypes = [i32, ctypes.POINTER(FileStamp), vp, vp, u64, ctypes.POINTER(BlockSig), vp]
    L.sf_index_fd_fixed.argtypes = [i32, ctypes.POINTER(FileStamp), u32, ctypes.POINTER(BlockSig), u64, pu64, vp]
    L.sf_index_file.argtypes = [ctypes.c_char_p, u32, ctypes.POINTER(BlockSig), u64, pu64, vp]
    L.sf_index_file_range.argtypes = [ctypes.c_char_p, u64, u64, u32, ctypes.POINTER(BlockSig), u64, pu64]
    L.sf_index_fd.argtypes = [i32, u32, ctypes.POINTER(ctypes.POINTER(BlockSig)), pu64, vp]
    L.sf_free_rows.argtypes = [ctypes.POINTER(BlockSig)]
    L.sf_index_files.argtypes = [ctypes.POINTER(ctypes.c_char_p), u32, u32, u64, ctypes.POINTER(BlockSig), u64,
                                 pu64, vp, pu64, ctypes.POINTER(ctypes.c_uint32)]
    L.sf_index_fds_blocks.argtypes = [vp, vp, u32, vp, vp, vp, u64, ctypes.POINTER(BlockSig), u64, pu64, vp, vp,
                                      ctypes.POINTER(ctypes.c_uint32)]
    L.sf_cut_fd.argtypes = [i32, vp, vp, u32, ctypes.POINTER(vp), ctypes.POINTER(vp), pu64]
    L.sf_free_cuts.argtypes = [vp]
    L.sf_free_cuts.restype = None
    L.sf_index_fd_cut.argtypes = [i32, vp, vp, u32, ctypes.POINTER(ctypes.POINTER(BlockSig)), pu64, vp]
    L.sf_shard_range.argtypes = [u64, u32, u32, u32, pu64, pu64]
    L.sf_index_file_multi.argtypes = [ctypes.c_char_p, u32, u32, ctypes.POINTER(BlockSig), u64, pu64, vp]
    L.sf_index_device_multi.argtypes = [u32, vp, u64, u32, vp, u32, vp, vp]
    L.sf_index_device_multi_ex.argtypes = [u32, vp, u64, u32, vp, u32, vp, vp, vp]
    L.sf_blocks_hash.argtypes = [vp, u64, vp]
    L.sf_blocks_hash_sigs.argtypes = [ctypes.POINTER(BlockSig), u64, vp]
    L.sf_sha1_host.argtypes = [vp, u64, vp]
    L.sf_block_set_build.argtypes = [vp, vp, u64, ctypes.POINTER(vp), vp]
    L.sf_block_set_lookup.argtypes = [vp, vp, u64, vp, vp]
    L.sf_block_set_free.argtypes = [vp, vp]
    pi64 = ctypes.POINTER(ctypes.c_int64)
    L.sf_test_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_int64, pi64]
    L.sf_test_get_knob.argtypes = [ctypes.c_char_p, pi64]
    L.sf_test_get_stat.argtypes = [ctypes.c_char_p, pi64]
    L.sf_test_table_order.argtypes = [vp, u64, vp, vp]
    L.sf_test_table_order_bits.argtypes = [vp, u64, ctypes.c_uint32, vp, vp]
    L.sf_test_set_read_hook.argtypes = [READ_HOOK, vp]
    L.sf_test_xcd_litmus.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
    L.sf_test_multi_plan.argtypes = [u64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, vp, vp, vp]
    for name in EXPORTED + EXPORTED_TEST:
        if name not in ("sf_version", "sf_strerror", "sf_free_rows"):
            getattr(L, name).restype = ctypes.c_int
    L.sf_free_rows.restype = None


def lib() -> ctypes.CDLL:
    """Load the HIP library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(syncfast_amd has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def _strerror(code: int) -> str:
    try:
        return lib().sf_strerror(code).decode()
    except ImportError:
        return f"error {code}"


def check(rc: int, what: str = "") -> None:
    if rc != SF_OK:
        raise SfError(rc, what)


def get_knob(name: str) -> int:
    """Current value of a library knob (latched from the environment when the
    library was loaded; include/syncfast_amd_test.h)."""
    v = ctypes.c_int64()
    check(lib().sf_test_get_knob(name.encode(), ctypes.byref(v)), name)
    return v.value


def set_knob(name: str, value: int) -> int:
    """Set a library knob (test hook); returns the previous value."""
    old = ctypes.c_int64()
    check(lib().sf_test_set_knob(name.encode(), int(value), ctypes.byref(old)), name)
    return old.value


def get_stat(name: str) -> int:
    """A route counter of the host entry points ("pages_locked",
    "not_anon_refused")."""
    v = ctypes.c_int64()
    check(lib().sf_test_get_stat(name.encode(), ctypes.byref(v)), name)
    return v.value


_read_hook_ref = None  # keeps the ctypes thunk alive while the library holds it


def set_read_hook(fn) -> None:
    """Test hook (sf_test_set_read_hook): fn(window) runs after each window a
    pread route of the library has read, on the calling thread; None removes
    it."""
    global _read_hook_ref
    if fn is None:
        check(lib().sf_test_set_read_hook(READ_HOOK(), None), "sf_test_set_read_hook")
        _read_hook_ref = None
        return
    thunk = READ_HOOK(lambda _arg, window: fn(int(window)))
    check(lib().sf_test_set_read_hook(thunk, None), "sf_test_set_read_hook")
    _read_hook_ref = thunk


def _code_objects(path: str):
    """(triple, bytes) of every gfx950 code object in the library's
    .hip_fatbin section (one clang offload bundle per GPU translation unit)."""
    import struct
    with open(path or LIB_PATH, "rb") as f:
        b = f.read()
    if b[:4] != b"\x7fELF" or b[4] != 2:
        raise ValueError("not an ELF64 library")
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    stro = secs[shstrndx][4]
    fat = None
    for sec in secs:
        name = b[stro + sec[0]: b.index(b"\0", stro + sec[0])]
        if name == b".hip_fatbin":
            fat = b[sec[4]: sec[4] + sec[5]]
    if fat is None:
        raise ValueError("no .hip_fatbin section")
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = fat.find(magic)
    while pos >= 0:  # bundle: magic, u64 entries, then (u64 offset, u64 size, u64 triple length, triple)
        n, = struct.unpack_from("<Q", fat, pos + len(magic))
        p = pos + len(magic) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24: p + 24 + tlen]
            p += 24 + tlen
            if triple.startswith(b"hipv4-amdgcn"):
                yield triple, fat[pos + off: pos + off + size]
        pos = fat.find(magic, pos + 1)


FIXED_KERNEL = "_ZN2sf17sha1_fixed_kernelILi128ELi1ELb0EEEvPKhmjmPhNS_11PadScheduleEPj"
CHAINED_KERNEL = "_ZN2sf25sha1_fixed_chained_kernelILi128EEEvPKhmjmPhNS_11PadScheduleENS_8ChainJobES5_jjj"
TABLE_KERNEL = "_ZN2sf17sha1_table_kernelILi128ELb0EEEvPKhmPKmPKjmPhPiPjS6_"


def kernel_code_sha256(path: str = None, symbol: str = FIXED_KERNEL) -> str:
    """SHA-256 of one kernel's machine code (its bytes in the gfx950 code
    object's .text, located through .symtab): what the GPU runs for that
    kernel.  Other kernels of the same translation unit can change without
    changing it.  bench.py keys the PMC traffic of profiles/traffic.json on it
    for the headline kernel (sha1_fixed_kernel<128, 1, false>); config 3's
    line names sha1_fixed_chained_kernel<128>'s (CHAINED_KERNEL), whose
    block rate depends on how its block part was compiled (DESIGN.md
    section 3.3b)."""
    import hashlib
    import struct
    for _, co in _code_objects(path):
        if co[:4] != b"\x7fELF":
            continue
        shoff, = struct.unpack_from("<Q", co, 0x28)
        shentsize, shnum, shstrndx = struct.unpack_from("<HHH", co, 0x3A)
        secs = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + i * shentsize) for i in range(shnum)]
        stro = secs[shstrndx][4]
        names = [co[stro + s[0]: co.index(b"\0", stro + s[0])] for s in secs]
        if b".symtab" not in names:
            continue
        symtab = secs[names.index(b".symtab")]
        strtab = secs[symtab[6]]  # sh_link
        for i in range(symtab[5] // 24):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", co, symtab[4] + 24 * i)
            nm = co[strtab[4] + st_name: co.index(b"\0", strtab[4] + st_name)]
            if nm == symbol.encode() and st_size:
                sec = secs[st_shndx]  # (name, type, flags, addr, offset, size, ...)
                start = sec[4] + (st_value - sec[3])
                return hashlib.sha256(co[start: start + st_size]).hexdigest()
    raise ValueError(f"no code object defines {symbol}")


def code_object_sha256(path: str = None, kernel: bytes = b"sha1_fixed_kernel") -> str:
    """SHA-256 of the gfx950 code object that holds `kernel` (the library's
    ``.hip_fatbin`` section holds one clang offload bundle per GPU translation
    unit; the SHA-1 kernels are in sf_capi.hip's).  What the GPU runs for that
    kernel: host-only changes, and changes to other translation units' kernels,
    leave it unchanged; any change to the SHA-1 kernels alters it.  bench.py
    keys the PMC traffic of profiles/traffic.json on it."""
    import hashlib
    import struct
    with open(path or LIB_PATH, "rb") as f:
        b = f.read()
    if b[:4] != b"\x7fELF" or b[4] != 2:
        raise ValueError("not an ELF64 library")
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    stro = secs[shstrndx][4]
    fat = None
    for sec in secs:
        name = b[stro + sec[0]: b.index(b"\0", stro + sec[0])]
        if name == b".hip_fatbin":
            fat = b[sec[4]: sec[4] + sec[5]]
    if fat is None:
        raise ValueError("no .hip_fatbin section")
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = fat.find(magic)
    while pos >= 0:  # bundle: magic, u64 entries, then (u64 offset, u64 size, u64 triple length, triple)
        n, = struct.unpack_from("<Q", fat, pos + len(magic))
        p = pos + len(magic) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24: p + 24 + tlen]
            p += 24 + tlen
            co = fat[pos + off: pos + off + size]
            if triple.startswith(b"hipv4-amdgcn") and kernel in co:
                return hashlib.sha256(co).hexdigest()
        pos = fat.find(magic, pos + 1)
    raise ValueError(f"no code object holds {kernel!r}")


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib().sf_device_count(ctypes.byref(n)), "sf_device_count")
    return n.value
