"""ctypes bindings to the in-tree native libraries.

* ``libomldm_hip.so``  — hand-written CDNA4 kernels (csrc/kernels/*.hip, gfx950).
* ``libomldm_host.so`` — host data plane + CPU reference implementations (csrc/host).

The HIP library is REQUIRED whenever a tensor lives on a GPU: ops never fall back to
PyTorch eager code silently; a missing/stale build raises :class:`NativeMissing`.
Kernel launchers take raw device pointers and the current HIP stream
(``torch.cuda.current_stream().cuda_stream``) so they order correctly with PyTorch
work and RCCL collectives issued on the same stream.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE_DIR = os.path.join(_HERE, "_native")
HIP_LIB_PATH = os.path.join(NATIVE_DIR, "libomldm_hip.so")
HOST_LIB_PATH = os.path.join(NATIVE_DIR, "libomldm_host.so")

_lock = threading.Lock()
_hip = None
_host = None

vp, i32, i64, u32, u64, f32 = C.c_void_p, C.c_int, C.c_longlong, C.c_uint32, C.c_uint64, C.c_float
f64 = C.c_double


class NativeMissing(RuntimeError):
    pass


def _sig(lib, name, res, args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = args
    return fn


# (name, restype, argtypes) for every exported HIP launcher.
HIP_SIGS = [
    ("omldm_linear_round", i32, [vp, i32, vp, i32, i32, vp, i32, vp, i32, i32, i32, i32, vp, i32,
                                 vp,
                                 vp, vp, i32, i32, f32, f32, f32, f32, f32, i32, i32, i32, i32,
                                 i32, i32, f32, vp, i32, vp]),
    ("omldm_spill_words", i64, [i32, i32, i32]),
    ("omldm_linear_reduce_part", i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32,
                                       i32, i32, i32, vp]),
    ("omldm_linear_part_bounds", i32, [i32, i32, i32, vp]),
    ("omldm_linear_table_geom", i32, [i32, i32, vp]),
    ("omldm_linear_predict", i32, [vp, i32, i64, i32, vp, i32, i32, vp, i32, i32, i32, i32, i32,
                                   vp, vp, vp]),
    ("omldm_linear_apply", i32, [vp, vp, vp, i32, vp]),
    ("omldm_linear_apply_multi", i32, [i32, vp, vp, vp, i32, vp]),
    ("omldm_linear_seq_round", i32, [vp, vp, i32, vp, i32, vp, i32, i32, i32, i32, vp, vp, i32,
                                     vp, vp, i32, i32, f32, f32, f32, f32, i32, vp]),
    ("omldm_linear_seq_apply", i32, [vp, vp, i32, vp, i32, vp]),
    ("omldm_linear_seq_broadcast", i32, [vp, vp, i32, i32, vp]),
    ("omldm_hash_raw", i32, [vp, i64, i32, i32, i64, vp, vp]),
    ("omldm_linear_seq_reduce", i32, [vp, vp, i32, i32, vp, f32, vp, vp, vp]),
    ("omldm_scan3_lds_cap", i32, []),
    ("omldm_scan3_set_cap", None, [i32]),
    ("omldm_scan3_set_gram_valu", None, [i32]),
    ("omldm_scan3_set_gram_ablate", i32, [i32]),
    ("omldm_scan3_fits", i32, [i32, i32, i32, i32]),
    ("omldm_scan3_ws_words", i64, [i32, i32, i32, i32, i32, i32, i64, i32]),
    ("omldm_scan3_prepare", i32, [vp, i32, vp, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32,
                                  i32, f32, i64, i32, i32, f32, f32, f32, vp, vp]),
    ("omldm_scan3_run", i32, [vp, i32, i32, vp, i32, i32, i32, i32, vp, i32, vp, i32, i32, f32,
                              f32, f32, f32, i32, i64, vp, i32, i32, i32, u32, vp, i32, f32, f32,
                              vp]),
    ("omldm_scan3_run_multi", i32, [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp,
                                    i32, i32, i32, i32, i32, i32, i32, i32, i64, i32, i32, vp, vp,
                                    vp]),
    ("omldm_scan3_max_pipes", i32, []),
    ("omldm_scan3mc_lds_cap", i32, [i32]),
    ("omldm_scan3mc_spill_floats", i64, [i32, i32, i32]),
    ("omldm_scan3mc_run", i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, vp, i32, vp,
                                i32, f32, i32, vp, vp, vp, vp, vp, vp, vp]),
    ("omldm_scan3_set_comb", None, [i32]),
    ("omldm_scan3_set_form", None, [i32]),
    ("omldm_scan3_set_cns", None, [i32]),
    ("omldm_scan3_set_inscan", None, [i32]),
    ("omldm_scan3_wait_next", None, [vp, C.c_uint64]),
    ("omldm_scan3_signal", i32, [vp, C.c_uint64, vp]),
    ("omldm_scan3_set_prep_split", None, [i32]),
    ("omldm_scan3_get_comb", i32, []),
    ("omldm_scan3_comb_err", i32, []),
    ("omldm_scan3_comb_err_drain", i32, [vp, vp]),
    ("omldm_scan3_teardown", i32, []),
    ("omldm_scan3_set_mode", None, [i32]),
    ("omldm_scan3_get_mode", i32, []),
    ("omldm_scan3_part_bounds", i32, [i32, i32, i32, i64, i32, i32, vp]),
    ("omldm_scan3_stamps", i32, [vp]),
    ("omldm_colstats_update", i32, [vp, i32, i32, C.c_double, vp, vp, vp, vp, i32, vp, i32, vp]),
    ("omldm_scale", i32, [vp, vp, i32, i32, i32, vp, vp, C.c_double, vp, vp, vp]),
    ("omldm_poly", i32, [vp, i32, i32, vp, i32, i32, vp, vp]),
    ("omldm_pull_copy", i32, [vp, vp, i64, i32, vp]),
    ("omldm_pull_copy_set_wt", None, [i32]),
    ("omldm_pull_copy_segs", i32, [vp, i32, i32, vp]),
    ("omldm_h2d_async", i32, [vp, vp, i64, vp]),
    ("omldm_gram_update", i32, [vp, vp, i32, i32, vp, i32, vp, vp, vp]),
    ("omldm_gram_update_poly2", i32, [vp, vp, i32, i32, vp, i32, vp, i32, vp, vp, vp]),
    ("omldm_kmeans_assign", i32, [vp, vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp]),
    ("omldm_kmeans_apply", i32, [vp, vp, i32, i32, vp, vp, vp, vp, vp]),
    ("omldm_multiclass_round", i32, [vp, i32, vp, i32, i32, vp, i32, i32, vp, i32, i32, i32, i32,
                                     i32, i32, i32, f32, i32, vp, vp, i32, vp, vp, vp, i32, vp]),
    ("omldm_multiclass_apply", i32, [vp, vp, i32, i32, vp, i32, i32, vp, vp, vp, i32, vp, vp]),
    ("omldm_mlp_lds_bytes", i64, [i32, vp]),
    ("omldm_mlp_round", i32, [vp, vp, vp, i64, i32, i32, i32, vp, i32, i32, f32, vp, vp, vp, vp,
                              vp]),
    ("omldm_mlp_forward", i32, [vp, vp, i64, i32, vp, i32, vp, vp]),
    ("omldm_ht_update", i32, [vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    ("omldm_ht_update_ws_ints", i64, [i32, i32, i32]),
    ("omldm_ht_split", i32, [i32, i32, i32, i32, f32, f32, f32, vp, vp]),
    ("omldm_ht_predict", i32, [vp, i32, i32, i32, i32, vp, vp, vp]),
    ("omldm_ht_route", i32, [vp, i32, i32, i32, vp, vp, vp]),
    ("omldm_ht_exact", i32, [vp, vp, i32, i32, i32, i32, i32, i32, f32, f32, f32, vp, vp, vp,
                             vp]),
    ("omldm_drift_norms", i32, [vp, vp, i64, f32, vp, vp]),
    ("omldm_fold_reload", i32, [vp, vp, f32, vp, i64, vp]),
    ("omldm_elastic_pre", i32, [vp, vp, vp, vp, i64, vp]),
    ("omldm_elastic_post", i32, [vp, vp, vp, vp, f32, i64, vp]),
    ("omldm_async_push", i32, [vp, vp, vp, vp, vp, i64, vp]),
    ("omldm_async_pull", i32, [vp, vp, vp, vp, vp, f32, i64, vp]),
    ("omldm_gm_local", i32, [vp, f32, vp, vp]),
    ("omldm_fgm_local", i32, [vp, vp, f64, vp, vp]),
    ("omldm_fgm_hub", i32, [vp, vp, f64, i32, vp, vp]),
    ("omldm_fgm_begin", i32, [vp, vp, f64, vp]),
    ("omldm_holdout_route", i32, [vp, vp, vp, i64, vp, vp, vp, i32, vp, vp, vp, i32, i64, i64,
                                  i64, i64, i64, i64, i64, i64, i32, i32, i32, i32, vp]),
    ("omldm_kmeans_seq_fits", i32, [i32, i32]),
    ("omldm_scan3mc_debug", i32, [vp]),
    ("omldm_mlp_form", i32, [i32]),
    ("omldm_kmeans_seq_form", i32, [i32]),
    ("omldm_kmeans_seq", i32, [vp, i32, vp, i32, i32, i32, vp, vp, vp, vp]),
    ("omldm_ipc_alloc", vp, [i64]),
    ("omldm_ipc_free", i32, [vp]),
    ("omldm_ipc_handle", i32, [vp, vp]),
    ("omldm_ipc_handle_size", i32, []),
    ("omldm_ipc_open", vp, [vp]),
    ("omldm_ipc_close", i32, [vp]),
    ("omldm_copy_d2d", i32, [vp, vp, i64, vp]),
    ("omldm_p2p_delta", i32, [vp, vp, vp, vp, i64, vp]),
    ("omldm_p2p_axpy", i32, [vp, vp, f32, i64, vp]),
    ("omldm_p2p_install", i32, [vp, vp, vp, vp, i64, vp]),
    ("omldm_sig_create", vp, [vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, i32]),
    ("omldm_sig_destroy", None, [vp]),
    ("omldm_sig_state_words", i32, [i32]),
    ("omldm_sig_hub", i32, [vp, vp, i64, f32, vp]),
    ("omldm_sig_worker", i32, [vp, i32, vp, vp, vp, i64, i64, vp]),
    ("omldm_holdout_route_spokes", i32, [vp, vp, vp, i64, vp, vp, vp, i32, i32, vp, vp, vp, i64,
                                         vp, vp, i32, i32, i32, i32, vp]),
    ("omldm_json_parse", i32, [vp, vp, i32, i32, i32, i32, i64, i32, vp, vp, vp, vp, vp, vp]),
    ("omldm_copy_engine_create", vp, [i32]),
    ("omldm_copy_engine_destroy", None, [vp]),
    ("omldm_copy_engine_submit", u64, [vp, vp, vp, i64, vp, vp]),
    ("omldm_copy_engine_stream_wait", i32, [vp, u64, vp, vp]),
    ("omldm_event_create", vp, []),
    ("omldm_event_destroy", i32, [vp]),
    ("omldm_event_record", i32, [vp, vp]),
    ("omldm_stream_create_cumask", vp, [i32]),
    ("omldm_stream_create_cumask_ex", vp, [i32, i32, i32]),
    ("omldm_stream_create_cumask_words", vp, [vp, i32]),
    ("omldm_cu_probe", i32, [vp, vp]),
    ("omldm_host_device_ptr", vp, [vp]),
    ("omldm_stream_destroy", i32, [vp]),
    ("omldm_host_register", i32, [vp, i64]),
    ("omldm_host_alloc_thp", vp, [i64]),
    ("omldm_host_free_thp", None, [vp]),
]

HOST_SIGS = [
    ("omldm_cpu_kmeans_seq", i32, [vp, i32, vp, i32, i32, i32, vp, vp, vp]),
    ("omldm_murmur3_32", u32, [C.c_char_p, i64, u32]),
    ("omldm_json_to_dib", i64, [vp, vp, i32, i32, i32, i32, vp, i64, vp, i32]),
    ("omldm_crc32c", u32, [C.c_char_p, i64, u32]),
    ("omldm_hash_cat", C.c_int32, [C.c_char_p, i64, i32, i32, i64]),
    ("omldm_hash_cat16", C.c_int32, [C.c_char_p, i64, i32, i32]),
    ("omldm_parse_instances", i64, [C.c_char_p, vp, i32, i32, i32, i32, i64, i32, vp, vp, vp, vp,
                                    i32]),
    ("omldm_synth_batch", None, [u64, i64, i32, i32, i32, i64, i32, i32, f32, i32, vp, vp, vp,
                                 i32]),
    ("omldm_cpu_linear_round", i32, [vp, i32, vp, i32, vp, i32, vp, i32, i32, i32, vp, i32, vp,
                                     i32, i32, f32, f32, f32, f32, f32, i32, i32, f32, i32]),
    ("omldm_cpu_linear_apply", None, [vp, vp, vp, i32]),
    ("omldm_index_lines", i64, [vp, i64, i64, vp]),
    ("omldm_format_predictions", i64, [vp, vp, vp, i64, i32, vp, vp, i64, vp]),
    ("omldm_read_log", i64, [i32, i64, vp, i64, i64, vp, vp, i64]),
    ("omldm_fcst_lane_start", vp, [vp, vp, i32, vp, i32, i32, i32, i32, i64, i32, vp, vp, i32,
                                   vp, vp, vp, i32, vp]),
    ("omldm_fcst_lane_set_mailbox", None, [vp, vp]),
    ("omldm_fcst_lane_need_wave", i32, [vp]),
    ("omldm_fcst_lane_pause", i32, [vp, i32, i64]),
    ("omldm_fcst_lane_offsets", None, [vp, vp]),
    ("omldm_fcst_lane_stats", None, [vp, vp]),
    ("omldm_fcst_lane_tout", i64, [vp, i64]),
    ("omldm_fcst_lane_wait", i32, [vp, i64, i64]),
    ("omldm_fcst_lane_now_ns", i64, []),
    ("omldm_fcst_lane_latencies", i64, [vp, vp, i64]),
    ("omldm_fcst_lane_stop", None, [vp]),
    ("omldm_fill_regions", i64, [i32, vp, vp, vp, vp, vp, vp, vp, vp, i32]),
    ("omldm_codec_available", i32, [i32]),
    ("omldm_codec_decompress", i32, [i32, C.c_char_p, i64, vp, vp]),
    ("omldm_codec_compress", i32, [i32, C.c_char_p, i64, i32, vp, vp]),
    ("omldm_codec_free", None, [vp]),
    ("omldm_kafka_decode_into", i64, [C.c_char_p, i64, i64, i64, vp, i64, vp, vp, i32]),
    ("omldm_kafka_encode_lines", i32, [vp, vp, i64, i32, i64, i64, i32, i32, vp, vp]),
    ("omldm_cpu_multiclass_round", i32, [vp, vp, i32, vp, i32, vp, i32, i32, i32, i32, i32, i32,
                                         f32, i32, vp, vp]),
    ("omldm_cpu_linear_predict", None, [vp, i64, i32, vp, i32, vp, i32, i32, i32, i32, i32, vp,
                                        vp]),
    ("omldm_synth_raw", None, [u64, i64, i32, i32, i32, i32, i32, f32, f32, vp, vp, vp, i32]),
    ("omldm_cpu_hash_raw", None, [vp, i64, i32, i32, i64, vp, i32]),
    ("omldm_cpu_linear_seq_round", i32, [vp, vp, i32, vp, i32, vp, i32, i32, i32, i32, vp, i32,
                                         vp, i32, i32, f32, f32, f32, f32, i32, i32]),
    ("omldm_cpu_linear_seq_round64", i32, [vp, vp, i32, vp, i32, vp, i32, i32, i32, i32, vp,
                                           i32, vp, i32, i32, f32, f32, f32, f32, i32, i32]),
]


class _Lib:
    def __init__(self, path, sigs):
        self.path = path
        self.cdll = C.CDLL(path, mode=C.RTLD_GLOBAL)
        for name, res, args in sigs:
            try:
                setattr(self, name, _sig(self.cdll, name, res, args))
            except AttributeError:
                pass


def _maybe_build(host_only: bool):
    if os.environ.get("OMLDM_NO_AUTOBUILD"):
        return
    from omldm_amd import _build

    _build.build(host_only=host_only)


def host() -> _Lib:
    global _host
    if _host is None:
        with _lock:
            if _host is None:
                if not os.path.exists(HOST_LIB_PATH):
                    _maybe_build(host_only=True)
                if not os.path.exists(HOST_LIB_PATH):
                    raise NativeMissing(f"{HOST_LIB_PATH} missing: run python -m omldm_amd._build")
                _host = _Lib(HOST_LIB_PATH, HOST_SIGS)
    return _host


def hip() -> _Lib:
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                if not os.path.exists(HIP_LIB_PATH):
                    _maybe_build(host_only=False)
                if not os.path.exists(HIP_LIB_PATH):
                    raise NativeMissing(
                        f"{HIP_LIB_PATH} missing: the HIP kernels are required on GPU; "
                        "run python -m omldm_amd._build")
                _hip = _Lib(HIP_LIB_PATH, HIP_SIGS)
                import atexit

                atexit.register(_hip_teardown)
    return _hip


def _hip_teardown() -> None:
    """Destroy the streams / events the kernel library created on demand while the HIP
    runtime is still up (Python's atexit runs before the shared libraries' finalizers)."""
    lib = _hip
    if lib is not None and getattr(lib, "omldm_scan3_teardown", None) is not None:
        try:
            lib.omldm_scan3_teardown()
        except Exception:  # noqa: BLE001 - best effort at exit
            pass


def check(rc: int, what: str) -> None:
    if rc:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")


def ptr(t) -> int:
    """Raw data pointer of a tensor/ndarray (None → NULL)."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data


def dptr(t) -> int:
    """Pointer usable by a kernel: device tensors as-is, pinned host tensors through
    their device alias (zero-copy access over PCIe)."""
    if t is None:
        return None
    if getattr(t, "is_cuda", False):
        return t.data_ptr()
    if t.is_pinned():
        p = hip().omldm_host_device_ptr(t.data_ptr())
        if not p:
            raise RuntimeError("pinned host tensor has no device mapping")
        return p
    raise ValueError("kernel argument must be a device tensor or pinned host memory")


def stream_of(t) -> int:
    import torch

    if t is not None and getattr(t, "is_cuda", False):
        return torch.cuda.current_stream(t.device).cuda_stream
    return 0
