"""ctypes binding of libbwtmi.so (C ABI in include/bwtmi.h).

The shared library is built in-tree (``make -C bwt-algorithm_amd``) and loaded
from the package's parent directory.  There is deliberately no fallback: if
the library or a gfx950 device is missing, the calls below raise.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import threading
from typing import Dict, Optional

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("BWTMI_LIB", os.path.join(_PKG_ROOT, "libbwtmi.so"))

FMT = {"strfinder": 0, "bed": 1, "vcf": 2, "trf_table": 3, "trf_dat": 4}


class BwtmiError(RuntimeError):
    pass


class Hit(C.Structure):
    _fields_ = [("start", C.c_int64), ("end", C.c_int64), ("unit_len", C.c_int32),
                ("prim_len", C.c_int32), ("copies", C.c_int64)]


class Params(C.Structure):
    _fields_ = [("min_copies", C.c_int32), ("max_unit_len", C.c_int32),
                ("show_progress", C.c_int32), ("tier2", C.c_int32), ("threads", C.c_int32),
                ("build_index", C.c_int32), ("sa_sample", C.c_int32), ("reserved", C.c_int32)]


class LibParams(C.Structure):
    _fields_ = [("min_period", C.c_int32), ("max_period", C.c_int32), ("max_short_motif", C.c_int32),
                ("min_copies", C.c_int32), ("min_array_length", C.c_int32), ("allow_mismatches", C.c_int32),
                ("min_entropy", C.c_double)]


_lib = None
_lock = threading.RLock()    # ctx() -> lib() re-enters

# name -> (restype, argtypes)
_P = C.c_void_p
_SIGS = {
    "bwtmi_last_error": (C.c_char_p, []),
    "bwtmi_version": (C.c_char_p, []),
    "bwtmi_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "bwtmi_open": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "bwtmi_close": (C.c_int, [_P]),
    "bwtmi_free": (None, [_P]),
    "bwtmi_last_timing": (C.c_int, [_P, C.POINTER(C.c_double)]),
    "bwtmi_kernel_stats": (C.c_int, [_P, C.c_int, C.c_int, C.c_char_p, C.c_int64]),
    "bwtmi_kernel_stats_filter": (C.c_int, [_P, C.c_char_p]),
    "bwtmi_strict_scan": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                    C.POINTER(C.POINTER(Hit)), C.POINTER(C.c_int64)]),
    "bwtmi_index_build": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int32, C.c_uint32, C.POINTER(_P)]),
    "bwtmi_index_free": (C.c_int, [_P]),
    "bwtmi_index_size": (C.c_int64, [_P]),
    "bwtmi_index_get_sa": (C.c_int, [_P, _P]),
    "bwtmi_index_get_bwt": (C.c_int, [_P, _P]),
    "bwtmi_index_get_counts": (C.c_int, [_P, _P, _P]),
    "bwtmi_index_occ_len": (C.c_int64, [_P]),
    "bwtmi_index_get_occ": (C.c_int, [_P, C.c_uint8, _P]),
    "bwtmi_index_sampled_len": (C.c_int64, [_P]),
    "bwtmi_index_get_sampled": (C.c_int, [_P, _P]),
    "bwtmi_index_kmer_count": (C.c_int64, [_P]),
    "bwtmi_index_get_kmer": (C.c_int, [_P, _P, _P]),
    "bwtmi_index_lcp": (C.c_int, [_P, _P, _P]),
    "bwtmi_backward_search_batch": (C.c_int, [_P, _P, _P, _P, C.c_int64, _P]),
    "bwtmi_index_lcp_plateaus": (C.c_int, [_P, _P, C.POINTER(LibParams), C.POINTER(C.c_void_p),
                                           C.POINTER(C.c_int64)]),
    "bwtmi_index_short_imperfect": (C.c_int, [_P, _P, C.POINTER(LibParams), _P, C.c_int64, _P, C.c_int32]),
    "bwtmi_job_tier1": (C.c_int, [_P, _P, C.c_int32, C.c_int32]),
    "bwtmi_index_long_repeats": (C.c_int, [_P, _P, C.POINTER(LibParams), _P, C.c_int64, _P, C.c_int32]),
    "bwtmi_index_tier3": (C.c_int, [_P, _P, _P, _P, C.c_int64, _P, C.c_int32, C.c_int32]),
    "bwtmi_job_create": (C.c_int, [C.POINTER(Params), C.POINTER(_P)]),
    "bwtmi_job_free": (C.c_int, [_P]),
    "bwtmi_job_add_contig": (C.c_int, [_P, C.c_char_p, _P, C.c_int64, C.c_int64, C.c_int64,
                                       C.POINTER(C.c_int32)]),
    "bwtmi_job_scan": (C.c_int, [_P, _P]),
    "bwtmi_job_wait": (C.c_int, [_P, _P]),
    "bwtmi_job_upload": (C.c_int, [_P, _P]),
    "bwtmi_job_reset": (C.c_int, [_P]),
    "bwtmi_job_set_params": (C.c_int, [_P, C.POINTER(Params)]),
    "bwtmi_job_select": (C.c_int, [_P, _P, C.c_int32]),
    "bwtmi_job_add_hits": (C.c_int, [_P, C.c_int32, _P, C.c_int64]),
    "bwtmi_job_raw_count": (C.c_int64, [_P]),
    "bwtmi_job_postprocess": (C.c_int, [_P]),
    "bwtmi_job_count": (C.c_int64, [_P]),
    "bwtmi_job_render": (C.c_int, [_P, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]),
    "bwtmi_job_write": (C.c_int, [_P, C.c_int, C.c_char_p]),
    "bwtmi_job_write_async": (C.c_int, [_P, C.c_int, C.c_char_p]),
    "bwtmi_job_write_join": (C.c_int, [_P]),
    "bwtmi_job_unit_count": (C.c_int32, [_P]),
    "bwtmi_job_unit_rows": (C.c_int, [_P, _P]),
    "bwtmi_job_render_units": (C.c_int, [_P, C.c_int, _P, _P]),
    "bwtmi_job_write_units": (C.c_int, [_P, C.c_char_p, _P, C.c_int]),
    "bwtmi_job_write_units_async": (C.c_int, [_P, C.c_char_p, _P, C.c_int]),
    "bwtmi_job_get_records": (C.c_int, [_P, _P, _P]),
    "bwtmi_job_get_string": (C.c_int64, [_P, C.c_int64, C.c_int, _P, C.c_int64]),
    "bwtmi_job_get_strings": (C.c_int64, [_P, C.c_int, _P, C.c_int64, _P]),
    "bwtmi_fasta_count_records": (C.c_int64, [C.c_char_p, C.c_int64]),
    "bwtmi_job_export": (C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]),
    "bwtmi_job_import": (C.c_int, [_P, _P, C.c_int64]),
    "bwtmi_job_stage_ms": (C.c_int, [_P, C.POINTER(C.c_double)]),
    "bwtmi_align_region": (C.c_int, [C.c_char_p, C.c_int64, C.c_int64, C.c_int64, C.c_char_p, C.c_int64,
                                     C.c_double, C.c_int64, C.c_int64, _P, C.POINTER(C.c_double), _P,
                                     C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "bwtmi_job_load_fasta": (C.c_int, [_P, C.c_char_p, C.c_int32]),
    "bwtmi_job_load_fasta_dev": (C.c_int, [_P, _P, C.c_char_p, C.c_int32]),
    "bwtmi_job_device_text": (C.c_int, [_P, _P, C.c_int32, C.c_void_p]),
    "bwtmi_job_contig_count": (C.c_int32, [_P]),
    "bwtmi_job_contig_info": (C.c_int64, [_P, C.c_int32, C.c_char_p, C.c_int64, C.POINTER(C.c_int64),
                                          C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "bwtmi_job_contig_seq": (C.c_int, [_P, C.c_int32, _P]),
    "bwtmi_job_load_fasta_shard": (C.c_int, [_P, C.c_char_p, C.c_int32, C.c_int32, C.c_int32]),
    "bwtmi_job_fasta_scan_part": (C.c_int, [_P, C.c_char_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p),
                                            C.POINTER(C.c_int64)]),
    "bwtmi_job_fasta_scan_part_dev": (C.c_int, [_P, _P, C.c_char_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p),
                                                C.POINTER(C.c_int64)]),
    "bwtmi_job_load_fasta_parts": (C.c_int, [_P, C.c_char_p, C.c_int32, C.c_int32, C.c_int32, _P, C.c_int64]),
    "bwtmi_job_load_fasta_parts_dev": (C.c_int, [_P, _P, C.c_char_p, C.c_int32, C.c_int32, C.c_int32, _P, C.c_int64]),
    "bwtmi_job_contig_weight": (C.c_int64, [_P, C.c_int32]),
    "bwtmi_job_select_shard": (C.c_int, [_P, C.c_int32, C.c_int32, _P, _P]),
    "bwtmi_host_info": (C.c_int, [C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "bwtmi_comm_unique_id": (C.c_int, [_P]),
    "bwtmi_comm_init": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, _P, C.POINTER(_P)]),
    "bwtmi_comm_allreduce": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int32]),
    "bwtmi_comm_free": (C.c_int, [_P]),
    "bwtmi_device_sync": (C.c_int, [C.c_int32]),
    "bwtmi_job_set_records": (C.c_int, [_P, _P, C.c_int64]),
    "bwtmi_wire_record_size": (C.c_int, []),
    "bwtmi_job_contig_error": (C.c_int64, [_P, C.c_int32, C.c_char_p, C.c_int64]),
    "bwtmi_source_hash": (C.c_char_p, []),
    "bwtmi_trace_push": (C.c_int, [C.c_char_p]),
    "bwtmi_trace_pop": (C.c_int, []),
    "bwtmi_knob_set": (C.c_int, [C.c_char_p, C.c_int64]),
    "bwtmi_knob_get": (C.c_int, [C.c_char_p, C.POINTER(C.c_int64)]),
    "bwtmi_knob_default": (C.c_int, [C.c_char_p, C.POINTER(C.c_int64)]),
    "bwtmi_knob_names": (C.c_char_p, []),
    "bwtmi_bind_host": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int)]),
    "bwtmi_host_binding_plan": (C.c_int, [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, C.c_char_p,
                                          C.c_char_p, C.c_int64, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
}
EXPORTED = tuple(_SIGS)


def lib():
    """Load libbwtmi.so (raises BwtmiError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise BwtmiError(f"{LIB_PATH} not found: build it with `make -C {_PKG_ROOT}` "
                                 "(there is no CPU fallback)")
            L = C.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().bwtmi_last_error()
        raise BwtmiError(f"libbwtmi error {rc}: {msg.decode(errors='replace') if msg else ''}")


_ctxs: Dict[int, C.c_void_p] = {}


def device_count() -> int:
    n = C.c_int(0)
    check(lib().bwtmi_device_count(C.byref(n)))
    return n.value


def ctx(device: Optional[int] = None) -> C.c_void_p:
    """Per-process device context (opened once per device, closed at exit)."""
    if device is None:
        device = int(os.environ.get("BWTMI_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    with _lock:
        h = _ctxs.get(device)
        if h is None:
            h = C.c_void_p()
            check(lib().bwtmi_open(device, C.byref(h)))
            _ctxs[device] = h
    return h


@atexit.register
def _close_all():
    if _lib is None:
        return
    for h in list(_ctxs.values()):
        _lib.bwtmi_close(h)
    _ctxs.clear()


def source_hash() -> str:
    """sha256 of csrc/* and include/bwtmi.h embedded when libbwtmi.so was built."""
    return lib().bwtmi_source_hash().decode()


def tree_source_hash() -> str:
    """The same hash computed from the sources in this tree (Makefile SRC_HASH):
    the files in byte order of their paths, concatenated."""
    import glob
    import hashlib
    csrc = os.path.join(_PKG_ROOT, "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.cpp")) + glob.glob(os.path.join(csrc, "*.h")) +
                   glob.glob(os.path.join(csrc, "*.hip")))
    files.append(os.path.join(os.path.dirname(_PKG_ROOT), "include", "bwtmi.h"))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def check_build() -> str:
    """Fails loudly when the loaded library was built from other sources than
    this tree's (a stale or foreign libbwtmi.so); returns the hash."""
    got, want = source_hash(), tree_source_hash()
    if got != want:
        raise BwtmiError(f"{LIB_PATH} was built from sources {got[:16]}..., this tree holds {want[:16]}...: "
                         f"rebuild with `make -C {_PKG_ROOT}`")
    return got


def knob(name: str, value: Optional[int] = None) -> int:
    """Read (and with value, set) a run-time switch BWTMI_<name>;
    returns the value before the call."""
    v = C.c_int64()
    check(lib().bwtmi_knob_get(name.encode(), C.byref(v)))
    if value is not None:
        check(lib().bwtmi_knob_set(name.encode(), int(value)))
    return v.value


def knob_names() -> list:
    return lib().bwtmi_knob_names().decode().split(",")


class knobs:
    """with knobs(RUNS_DENSE=1, ...): set switches for the block, restore after."""

    def __init__(self, **kv):
        self.kv = kv
        self.old = {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = knob(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            knob(k, v)
        return False


def bind_host(h, on: bool = True) -> bool:
    """Move this process's host work onto the CPUs of its GPU's NUMA node (the
    CLI, bench and rank launcher ask for it; the library never does on its own);
    on=False restores the affinity the binding replaced.  True when it changed."""
    b = C.c_int(0)
    check(lib().bwtmi_bind_host(h, int(on), C.byref(b)))
    return bool(b.value)


def binding_plan(sysroot: str, local_rank: int, rank_pci, threads: int, allowed: str, smt: bool = False):
    """(cpulist or '', node, local ranks on that node) the binding would choose,
    from a sysfs tree under sysroot; no affinity change."""
    out = C.create_string_buffer(8192)
    node, peers = C.c_int(-1), C.c_int(0)
    check(lib().bwtmi_host_binding_plan(sysroot.encode(), local_rank, ",".join(rank_pci).encode(), threads, int(smt),
                                        allowed.encode(), out, len(out), C.byref(node), C.byref(peers)))
    return out.value.decode(), node.value, peers.value


def kernel_stats(h, enable: bool = True, reset: bool = True) -> dict:
    """{kernel: (total_ms, launches, algorithmic_bytes)} from HIP events on the ctx stream."""
    buf = C.create_string_buffer(1 << 16)
    check(lib().bwtmi_kernel_stats(h, int(enable), int(reset), buf, len(buf)))
    out = {}
    for line in buf.value.decode().splitlines():
        name, ms, n, b = line.split()
        out[name] = (float(ms), int(n), float(b))
    return out


def kernel_stats_filter(h, name: str = "") -> None:
    """Time only the launches named `name` ("" = every launch)."""
    check(lib().bwtmi_kernel_stats_filter(h, name.encode() if name else None))


def host_info() -> dict:
    """CPUs visible to this process, ranks on the node, post-processing threads per rank."""
    v, lw, t = C.c_int32(), C.c_int32(), C.c_int32()
    check(lib().bwtmi_host_info(C.byref(v), C.byref(lw), C.byref(t)))
    return {"cpus_visible": v.value, "local_world": lw.value, "threads_per_rank": t.value}


def last_timing(h) -> tuple:
    out = (C.c_double * 3)()
    check(lib().bwtmi_last_timing(h, out))
    return tuple(out)
