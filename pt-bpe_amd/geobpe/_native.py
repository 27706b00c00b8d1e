"""ctypes binding of libgeobpe.so (the C-ABI in include/geobpe.h).

The HIP library is the product: there is no CPU fallback.  Importing this
module on a box without the built library raises immediately; calls into a
context raise `GeoBPEError` (or `ValueError` for the reference's ValueError
cases) with the library's message.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GEOBPE_LIB") or os.path.join(HERE, "libgeobpe.so")  # override: kernel A/B builds

E_OK, E_ARG, E_VALUE, E_CAPACITY, E_HIP, E_HASH = range(6)
DELTA_RECORD_BYTES = 40
# geobpe_allgather_fn: (user, host send, host recv, bytes per rank) -> 0 on success
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)


def rccl_path():
    """The RCCL library this process's PyTorch uses (the engine's communicator binds to the
    same instance), or None for the system's librccl.so.1."""
    try:
        import torch
        p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        return p if os.path.exists(p) else None
    except ImportError:  # pragma: no cover
        return None


class GeoBPEError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libgeobpe.so (built by __graft_entry__.build() / geobpe.build)."""
    global _lib
    if _lib is not None:
        return _lib
    # Share ONE HIP runtime with PyTorch: torch bundles its own libamdhip64
    # (soname libamdhip64.so.7); loading torch first makes libgeobpe.so bind to
    # that copy, so torch streams / device pointers are valid in our calls.  A
    # second runtime instance in the process would not see the device.
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover
        pass
    if not os.path.exists(LIB_PATH):
        raise GeoBPEError(
            f"{LIB_PATH} is missing: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')")
    L = ctypes.CDLL(LIB_PATH)
    P, I32, I64, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    pI32, pI64 = ctypes.POINTER(I32), ctypes.POINTER(I64)
    sig = {
        "geobpe_create": (ctypes.c_int, [ctypes.POINTER(P), ctypes.c_int, P, I64]),
        "geobpe_destroy": (None, [P]),
        "geobpe_last_error": (ctypes.c_char_p, [P]),
        "geobpe_load_angles": (ctypes.c_int, [P, I64, P, P]),
        "geobpe_angle_range": (ctypes.c_int, [P, P, P]),
        "geobpe_quantize": (ctypes.c_int, [P, I32, P, D]),
        "geobpe_symbol_first": (ctypes.c_int, [P, I64, P]),
        "geobpe_init_tokens": (ctypes.c_int, [P, P, I32]),
        "geobpe_bin": (ctypes.c_int, [P]),
        "geobpe_set_bin_dense": (ctypes.c_int, [P, ctypes.c_int]),
        "geobpe_step": (ctypes.c_int, [P, pI32, pI32, pI64]),
        "geobpe_run": (ctypes.c_int, [P, I64, pI64]),
        "geobpe_run_log": (ctypes.c_int, [P, I64, pI64, pI64, P, I64]),
        "geobpe_set_tail": (ctypes.c_int, [P, I64]),
        "geobpe_set_mid": (ctypes.c_int, [P, I64]),
        "geobpe_merge_log": (I64, [P, P, I64]),
        "geobpe_key_json": (I64, [P, I32, ctypes.c_char_p, I64]),
        "geobpe_debug_key_less": (ctypes.c_int, [P, P, I32, P]),
        "geobpe_debug_counts": (I64, [P, P, P, I64]),
        "geobpe_debug_state": (I64, [P, P, I64]),
        "geobpe_debug_key": (ctypes.c_int, [P, I32, P]),
        "geobpe_step_select": (ctypes.c_int, [P, pI32, pI32]),
        "geobpe_step_apply": (ctypes.c_int, [P, pI64]),
        "geobpe_delta_export": (ctypes.c_int, [P, P, I64, pI64]),
        "geobpe_delta_import": (ctypes.c_int, [P, P, I64]),
        "geobpe_set_distributed": (ctypes.c_int, [P, ctypes.c_int]),
        "geobpe_set_global_residues": (ctypes.c_int, [P, I64]),
        "geobpe_set_rank": (ctypes.c_int, [P, ctypes.c_int32]),
        "geobpe_token_json": (I64, [P, I32, ctypes.c_char_p, I64]),
        "geobpe_token_content": (I64, [P, I32, P, I64]),
        "geobpe_vocab_count": (I64, [P]),
        "geobpe_num_keys": (I64, [P]),
        "geobpe_num_tokens": (I64, [P]),
        "geobpe_segmentation": (I64, [P, P, P, P]),
        "geobpe_encode": (I64, [P, P, P]),
        "geobpe_verify_counts": (I64, [P]),
        "geobpe_debug_timeline": (I64, [P, ctypes.c_int, P, I64]),
        "geobpe_set_profiling": (ctypes.c_int, [P, ctypes.c_int]),
        "geobpe_set_work_counters": (ctypes.c_int, [P, ctypes.c_int]),
        "geobpe_set_hold": (ctypes.c_int, [P, I64]),
        "geobpe_kernel_ms": (D, [P, ctypes.c_char_p, pI64]),
        "geobpe_set_profiling_filter": (ctypes.c_int, [P, ctypes.c_char_p]),
        "geobpe_marker": (ctypes.c_int, [P, ctypes.c_int32]),
        "geobpe_synchronize": (ctypes.c_int, [P]),
        "geobpe_set_record_events": (ctypes.c_int, [P, ctypes.c_int]),
        "geobpe_replay_load": (ctypes.c_int, [P, P, P, P, P, P, P, I64]),
        "geobpe_delta_export_async": (ctypes.c_int, [P, P, I64, P]),
        "geobpe_delta_import_async": (ctypes.c_int, [P, P, I64]),
        "geobpe_pipeline_begin": (ctypes.c_int, [P]),
        "geobpe_pipeline_iter": (ctypes.c_int, [P, P, I64]),
        "geobpe_pipeline_import": (ctypes.c_int, [P, P, ctypes.c_int32, I64]),
        "geobpe_pipeline_poll": (ctypes.c_int, [P, P]),
        "geobpe_pipeline_resolve": (ctypes.c_int, [P, P, I64]),
        "geobpe_pipeline_end": (ctypes.c_int, [P]),
        "geobpe_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p, P]),
        "geobpe_comm_init_rccl": (ctypes.c_int, [P, ctypes.c_char_p, P, ctypes.c_int32, ctypes.c_int32]),
        "geobpe_comm_error": (ctypes.c_char_p, []),
        "geobpe_comm_set_callback": (ctypes.c_int, [P, P, P, ctypes.c_int32, ctypes.c_int32]),
        "geobpe_comm_set_slot": (ctypes.c_int, [P, I64]),
        "geobpe_run_exchange": (ctypes.c_int, [P, I64, pI64]),
        "geobpe_pdb_backbone": (I64, [ctypes.c_char_p, P, I64]),
        "geobpe_pdb_error": (ctypes.c_char_p, []),
        "geobpe_featurize": (ctypes.c_int, [ctypes.c_int, I64, P, P, P]),
        "geobpe_events": (I64, [P, P, P, P]),
        "geobpe_nerf": (ctypes.c_int, [ctypes.c_int, I64, P, P, P]),
        "geobpe_glue_opt": (ctypes.c_int, [ctypes.c_int, I64, P, P, P, P, P, ctypes.c_int32, ctypes.c_int32, P, P,
                                           ctypes.c_float, ctypes.c_double, ctypes.c_double, P, P, P]),
        "geobpe_rmsd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P, P,
                                       ctypes.c_int, P]),
        "geobpe_arena_release": (ctypes.c_int, [ctypes.c_int]),
        "geobpe_set_collapse": (ctypes.c_int, [P, ctypes.c_int]),
        "geobpe_comm_peer": (ctypes.c_int, [P, ctypes.c_int]),
        "geobpe_run_exchange_log": (ctypes.c_int, [P, I64, pI64, pI64, P, I64]),
        "geobpe_comm_peer_active": (ctypes.c_int, [P]),
        "geobpe_collapsed": (ctypes.c_int, [P]),
    }
    ab = bool(os.environ.get("GEOBPE_LIB"))  # (an older A/B build may lack this round's entry points)
    for name, (res, args) in sig.items():
        if ab and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


EXPORTED_SYMBOLS = [
    "geobpe_create", "geobpe_destroy", "geobpe_last_error", "geobpe_load_angles", "geobpe_angle_range",
    "geobpe_quantize", "geobpe_symbol_first", "geobpe_init_tokens", "geobpe_bin", "geobpe_set_bin_dense", "geobpe_step",
    "geobpe_run", "geobpe_run_log", "geobpe_set_tail", "geobpe_set_mid", "geobpe_merge_log", "geobpe_key_json", "geobpe_debug_key_less", "geobpe_debug_counts", "geobpe_debug_state", "geobpe_debug_key",
    "geobpe_step_select", "geobpe_step_apply", "geobpe_delta_export", "geobpe_delta_import",
    "geobpe_set_distributed", "geobpe_set_global_residues", "geobpe_set_rank", "geobpe_token_json", "geobpe_token_content",
    "geobpe_vocab_count", "geobpe_num_keys", "geobpe_num_tokens", "geobpe_segmentation", "geobpe_encode",
    "geobpe_verify_counts", "geobpe_debug_timeline", "geobpe_set_profiling", "geobpe_set_work_counters", "geobpe_set_hold", "geobpe_set_profiling_filter", "geobpe_kernel_ms", "geobpe_marker", "geobpe_synchronize",
    "geobpe_set_record_events", "geobpe_events", "geobpe_replay_load",
    "geobpe_delta_export_async", "geobpe_delta_import_async", "geobpe_pipeline_begin", "geobpe_pipeline_iter",
    "geobpe_pipeline_import", "geobpe_pipeline_poll", "geobpe_pipeline_resolve", "geobpe_pipeline_end",
    "geobpe_comm_unique_id", "geobpe_comm_init_rccl", "geobpe_comm_error", "geobpe_comm_set_callback",
    "geobpe_comm_set_slot", "geobpe_run_exchange", "geobpe_pdb_backbone", "geobpe_pdb_error",
    "geobpe_featurize", "geobpe_rmsd", "geobpe_nerf", "geobpe_glue_opt", "geobpe_arena_release",
    "geobpe_set_collapse", "geobpe_collapsed", "geobpe_comm_peer", "geobpe_comm_peer_active",
    "geobpe_run_exchange_log",
]


def check(ctx, rc: int) -> None:
    if rc == E_OK:
        return
    msg = lib().geobpe_last_error(ctx)
    msg = msg.decode() if msg else f"error {rc}"
    if rc == E_VALUE:
        raise ValueError(msg)
    raise GeoBPEError(f"libgeobpe: {msg} (code {rc})")
