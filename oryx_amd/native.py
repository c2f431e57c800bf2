"""Loading of the in-tree native libraries (built by :mod:`oryx_amd._build`).

``runtime()`` returns the host C++ runtime (log transport etc.); ``kernels()`` the HIP kernel
library.  The kernel library must be loaded after ``torch`` so it binds to the same HIP
runtime instance (torch ships ``libamdhip64.so.7``; the dynamic linker reuses it by soname).

On a GPU box the HIP path is mandatory: :func:`require_kernels` raises if the library is
missing or fails to load (``oryx.gpu.require-native``), so a silent eager fallback can never
masquerade as the native path.
"""

from __future__ import annotations

import ctypes
import os
import threading

from . import _build

__all__ = ["runtime", "kernels", "require_kernels", "kernels_available", "stream_ptr"]

_lock = threading.Lock()
_runtime = None
_kernels = None
_kernels_error = None

# must equal oryx_kernels_version() in csrc/kernels/als.hip; bump both whenever an exported
# kernel entry point's signature or semantics change
KERNELS_ABI_VERSION = 29

c_vp = ctypes.c_void_p
c_i = ctypes.c_int
c_ll = ctypes.c_longlong
c_f = ctypes.c_float
c_cp = ctypes.c_char_p


def _sig(lib, name, restype, argtypes):
    fn = getattr(lib, name)
    fn.restype = restype
    fn.argtypes = argtypes
    return fn


def _load_runtime():
    path = _build.RUNTIME_SO
    if not os.path.exists(path) or _build._stale(path, _runtime_sources()):
        try:
            _build.build_runtime()
        except Exception:
            if not os.path.exists(path):
                raise
    lib = ctypes.CDLL(path)
    _sig(lib, "oryx_log_last_error", c_cp, [])
    _sig(lib, "oryx_log_open", c_vp, [c_cp, c_cp, c_i, c_ll, c_ll])
    _sig(lib, "oryx_log_exists", c_i, [c_cp, c_cp])
    _sig(lib, "oryx_log_close", None, [c_vp])
    _sig(lib, "oryx_log_num_partitions", c_i, [c_vp])
    _sig(lib, "oryx_log_max_message", c_ll, [c_vp])
    _sig(lib, "oryx_log_partition_for", c_i, [c_vp, c_cp, c_i])
    _sig(lib, "oryx_log_append_batch", c_ll, [c_vp, c_i, c_cp, c_ll, c_i, c_ll, c_i, c_vp])
    _sig(lib, "oryx_log_append_values", c_ll, [c_vp, c_i, c_cp, c_i, c_cp, c_vp, c_i, c_ll,
                                                c_i])
    # h, partition, key, key_len, blob, lens, n, gap, ts, fsync
    _sig(lib, "oryx_log_append_values_gap", c_ll, [c_vp, c_i, c_cp, c_i, c_vp, c_vp, c_i, c_i,
                                                    c_ll, c_i])
    _sig(lib, "oryx_log_begin_offset", c_ll, [c_vp, c_i])
    _sig(lib, "oryx_log_end_offset", c_ll, [c_vp, c_i])
    _sig(lib, "oryx_log_retain", c_i, [c_vp, c_ll])
    _sig(lib, "oryx_reader_open", c_vp, [c_vp, c_i, c_ll])
    _sig(lib, "oryx_reader_close", None, [c_vp])
    _sig(lib, "oryx_reader_position", c_ll, [c_vp])
    _sig(lib, "oryx_reader_seek", None, [c_vp, c_ll])
    _sig(lib, "oryx_reader_read_text", c_ll, [c_vp, c_ll, c_vp, c_ll, ctypes.POINTER(c_ll),
                                              ctypes.POINTER(c_i)])
    _sig(lib, "oryx_reader_poll", c_ll, [c_vp, c_vp, c_ll, c_i, c_i, ctypes.POINTER(c_ll)])
    _sig(lib, "oryx_offsets_set", c_i, [c_cp, c_cp, c_cp, c_i, ctypes.POINTER(c_i),
                                         ctypes.POINTER(c_ll)])
    _sig(lib, "oryx_offsets_get", c_ll, [c_cp, c_cp, c_cp, c_i])
    _register_runtime_extras(lib)
    return lib


def _register_runtime_extras(lib):
    c_dp = ctypes.POINTER(ctypes.c_double)
    _sig(lib, "oryx_dict_new", c_vp, [])
    _sig(lib, "oryx_dict_free", None, [c_vp])
    _sig(lib, "oryx_dict_size", c_ll, [c_vp])
    _sig(lib, "oryx_dict_clear", None, [c_vp])
    _sig(lib, "oryx_dict_encode", c_ll, [c_vp, c_cp, c_ll, c_i, c_vp])
    _sig(lib, "oryx_dict_get", c_ll, [c_vp, c_cp, c_ll])
    _sig(lib, "oryx_dict_merge", c_ll, [c_vp, c_vp, c_vp])
    _sig(lib, "oryx_dict_key", c_ll, [c_vp, c_ll, c_vp, c_ll])
    _sig(lib, "oryx_line_ends", c_ll, [c_vp, c_ll, c_vp, c_ll])
    _sig(lib, "oryx_hostbuf_alloc", c_vp, [c_ll])
    _sig(lib, "oryx_hostbuf_free", None, [c_vp, c_ll])
    _sig(lib, "oryx_hostbuf_stats", None, [c_vp])
    _sig(lib, "oryx_hostbuf_quiesce", c_ll, [c_ll])
    _sig(lib, "oryx_read_file_parallel", c_ll, [c_cp, c_vp, c_ll, c_i])
    _sig(lib, "oryx_hostbuf_prefault", None, [c_vp, c_ll, c_i])
    _sig(lib, "oryx_encode_spans", c_ll, [c_vp, c_vp, c_vp, c_ll, c_ll, c_vp, c_vp])
    _sig(lib, "oryx_gather_lines", c_ll, [c_vp, c_vp, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_concat_buffers", c_ll, [c_vp, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_reader_poll_frames", c_ll, [c_vp, c_vp, c_ll, ctypes.c_int,
                                                ctypes.POINTER(c_ll)])
    _sig(lib, "oryx_parse_up_frames", c_ll, [c_vp, c_ll, c_ll, ctypes.c_int, c_ll, c_vp, c_vp,
                                             c_vp, c_vp, ctypes.POINTER(c_ll)])
    _sig(lib, "oryx_aggregate_scores", c_ll, [c_vp, c_vp, c_vp, c_vp, c_ll, ctypes.c_int,
                                              c_vp, c_vp, c_vp])
    _sig(lib, "oryx_reader_text_bound", c_ll, [c_vp, c_ll])
    _sig(lib, "oryx_parse_ratings", c_ll, [c_cp, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_ll, c_ll, c_i])
    _sig(lib, "oryx_format_float_rows", c_ll, [c_vp, c_ll, c_i, c_ll, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_rowmap_new", c_vp, [])
    _sig(lib, "oryx_rowmap_free", None, [c_vp])
    _sig(lib, "oryx_rowmap_size", c_ll, [c_vp])
    _sig(lib, "oryx_rowmap_set", None, [c_vp, c_vp, c_vp, c_vp, c_ll])
    _sig(lib, "oryx_rowmap_remove", None, [c_vp, c_vp, c_vp, c_ll])
    _sig(lib, "oryx_rowmap_translate", c_ll, [c_vp, c_vp, c_vp])
    # buf, len, F, is_num, out, span_off, span_len, max_rows
    _sig(lib, "oryx_csv_numeric_block", c_ll, [c_cp, c_ll, c_i, c_vp, c_vp, c_vp, c_vp,
                                               c_ll])
    _sig(lib, "oryx_dict_keys_blob", c_ll, [c_vp, c_ll, c_ll, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_dict_owners", c_ll, [c_vp, c_ll, c_i, c_vp])
    _sig(lib, "oryx_ts_range", c_ll, [c_vp, c_ll, c_ll, c_vp, c_vp])
    _sig(lib, "oryx_csv_to_f32", c_ll, [c_vp, c_ll, c_i, c_vp, c_vp, c_i, c_vp, c_vp, c_vp,
                                        c_ll])
    _sig(lib, "oryx_csv_to_f64", c_ll, [c_vp, c_ll, c_i, c_vp, c_vp, c_i, c_vp, c_vp, c_vp,
                                        c_ll])
    _sig(lib, "oryx_speed_new", c_vp, [])
    _sig(lib, "oryx_speed_free", None, [c_vp])
    _sig(lib, "oryx_speed_parse", c_ll, [c_vp, c_vp, c_ll, c_vp, c_vp, c_ll])
    _sig(lib, "oryx_speed_counts", c_ll, [c_vp, c_vp])
    _sig(lib, "oryx_speed_aggregate", c_ll, [c_vp, c_i, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_speed_new_keys", c_ll, [c_vp, c_i, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_speed_assemble", c_ll, [c_vp, c_ll, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_vp, c_i, c_vp, c_ll, c_vp, c_vp])
    _sig(lib, "oryx_rowmap_key_suffixes", c_ll, [c_vp, c_vp, c_ll])
    _sig(lib, "oryx_format_leaf_updates", c_ll, [c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_i,
                                                 c_vp, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_format_cluster_updates", c_ll, [c_vp, c_vp, c_vp, c_ll, c_i, c_vp, c_ll,
                                                    c_vp])
    _sig(lib, "oryx_format_cluster_updates_slots", c_ll, [c_vp, c_vp, c_vp, c_vp, c_ll, c_i,
                                                          c_vp, c_ll, c_vp])
    _sig(lib, "oryx_format_f64_repr_host", None, [c_vp, c_ll, c_vp, c_vp])
    # nq, k, kp, max_batch, targets, cand_ptr, cand, cand_all, num_buckets, words,
    # bucket_start, n_rows, ex_ptr, ex_rows, pos_of_row, n_pos, delta_lo, delta_hi, out,
    # out_cap, info
    _sig(lib, "oryx_topn_prep", c_ll, [c_i, c_i, c_i, c_i, c_vp, c_vp, c_vp, c_vp, c_i, c_i,
                                       c_vp, c_ll, c_vp, c_vp, c_vp, c_ll, c_ll, c_ll, c_vp,
                                       c_ll, c_vp])
    _sig(lib, "oryx_digest128", None, [c_vp, c_ll, c_vp])
    _sig(lib, "oryx_blob_hash64", None, [c_vp, c_vp, c_ll, ctypes.c_ulonglong, c_vp])
    _sig(lib, "oryx_http_start", c_vp, [c_cp, c_i, c_i, c_ll])
    _sig(lib, "oryx_http_port", c_i, [c_vp])
    _sig(lib, "oryx_http_served", c_ll, [c_vp])
    _sig(lib, "oryx_http_next", c_ll, [c_vp, c_vp, c_ll, c_i])
    _sig(lib, "oryx_http_respond", c_i, [c_vp, ctypes.c_ulonglong, c_cp, c_ll, c_i])
    _sig(lib, "oryx_http_stop", None, [c_vp])
    _sig(lib, "oryx_http_free", None, [c_vp])
    _sig(lib, "oryx_http_tls", c_i, [c_vp, c_cp, c_cp, c_cp])
    _sig(lib, "oryx_http_tls_error", c_cp, [])
    # path, password, alias, cert_pem*, cert_len*, key_pem*, key_len*
    _sig(lib, "oryx_keystore_to_pem", c_i, [c_cp, c_cp, c_cp, c_vp, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_keystore_free", None, [c_vp])
    _sig(lib, "oryx_keystore_error", c_cp, [])
    _sig(lib, "oryx_speed_append", c_ll, [c_vp, c_vp, c_i, c_ll, c_ll, c_vp, c_vp, c_vp, c_vp,
                                          c_vp, c_vp, c_i, c_ll, c_i, c_vp])
    _sig(lib, "oryx_split_by_time", c_ll, [c_vp, c_ll, c_ll, c_ll, c_vp, c_vp, c_vp, c_vp,
                                           c_vp, c_vp])
    _sig(lib, "oryx_dict_encode_nums", c_ll, [c_vp, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_dict_encode_blob", c_ll, [c_vp, c_vp, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_dict_find_blob", c_ll, [c_vp, c_vp, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_dict_keys_blob_sel", c_ll, [c_vp, c_vp, c_ll, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_parse_up_batch", c_ll, [c_cp, c_vp, c_ll, c_i, c_vp, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_up_texts", c_ll, [c_vp, c_ll, c_vp, c_ll])
    _sig(lib, "oryx_up_ids", c_ll, [c_vp, c_ll])
    _sig(lib, "oryx_up_known_codes", c_ll, [c_vp, c_vp, c_ll])
    # raw, used, nrec, k, max_n, kinds, vecs, id_ends, known_cnt, consumed_bytes
    _sig(lib, "oryx_parse_up_records", c_ll, [c_vp, c_ll, c_ll, c_i, c_ll, c_vp, c_vp, c_vp,
                                              c_vp, c_vp])
    # users, items, u, i, nx, ny, vx, vy, n, k, with_known, out, cap
    _sig(lib, "oryx_format_als_updates", c_ll, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                c_ll, c_i, c_i, c_vp, c_ll])
    # users, items, u, i, xtext, xends, ytext, yends, vx, vy, n, with_known, out, cap,
    # msg_ends, n_msgs
    _sig(lib, "oryx_assemble_als_updates", c_ll, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                  c_vp, c_vp, c_vp, c_ll, c_i, c_vp, c_ll,
                                                  c_vp, c_vp])
    # kind, ids, id_ends, rows, row_ends, n, known, known_ends, kidx, out, cap, msg_ends, n_msgs
    _sig(lib, "oryx_assemble_row_messages", c_ll, [c_i, c_vp, c_vp, c_vp, c_vp, c_ll, c_vp,
                                                   c_vp, c_vp, c_vp, c_ll, c_vp, c_vp])
    # items, uu, ii, m, n_users, out, cap, ends
    _sig(lib, "oryx_known_items_text", c_ll, [c_vp, c_vp, c_vp, c_ll, c_ll, c_vp, c_ll, c_vp])
    _sig(lib, "oryx_write_gzip", c_i, [c_cp, c_vp, c_ll, c_i])
    _sig(lib, "oryx_gzip_indexed_size", c_ll, [c_vp, c_ll])
    _sig(lib, "oryx_gzip_indexed_inflate", c_ll, [c_vp, c_ll, c_vp, c_ll])
    # buf, len, k, max_n, vecs, id_ends
    _sig(lib, "oryx_parse_feature_lines", c_ll, [c_vp, c_ll, c_i, c_ll, c_vp, c_vp])


def _runtime_sources():
    import glob
    return glob.glob(os.path.join(_build.CSRC, "runtime", "*"))


def runtime():
    global _runtime
    if _runtime is None:
        with _lock:
            if _runtime is None:
                _runtime = _load_runtime()
    return _runtime


def _load_kernels():
    import torch  # noqa: F401  (bind to torch's HIP runtime first)
    # ORYX_KERNELS_SO: load another build of the kernel library (same-box A/B of kernel changes)
    path = os.environ.get("ORYX_KERNELS_SO") or _build.KERNELS_SO
    if path == _build.KERNELS_SO:
        # incremental: a no-op when the library is newer than every kernel source, so a
        # library left over from before a kernel change is never loaded silently
        _build.build_kernels()
    lib = ctypes.CDLL(path)
    _sig(lib, "oryx_kernels_version", c_i, [])
    got = lib.oryx_kernels_version()
    if got != KERNELS_ABI_VERSION:
        raise RuntimeError("%s has kernel ABI version %d, this package expects %d (stale "
                           "build: rebuild with python -m oryx_amd._build --force)"
                           % (path, got, KERNELS_ABI_VERSION))
    # ORYX_ALS_VARIANT selects the KP<=64 solve kernel for A/B runs (csrc/kernels/als.hip:
    # 5 = four rows per wave, batched block LDL^T (als_batch.hip), 3 = panel Cholesky at
    # raised priority, 2 = panel + 3-deep gather ring, 0 = panel + 1-deep, 1 = register)
    _sig(lib, "oryx_als_set_variant", c_i, [c_i])
    _sig(lib, "oryx_als_get_variant", c_i, [])
    _sig(lib, "oryx_als_batch_profile", c_i, [c_vp])
    rc_variant = lib.oryx_als_set_variant(int(os.environ.get("ORYX_ALS_VARIANT", "5")))
    if rc_variant != 0:
        raise RuntimeError("ORYX_ALS_VARIANT=%s needs the tuning build of the kernels "
                           "(python -m oryx_amd._build --tuning; ORYX_KERNELS_SO=%s)"
                           % (os.environ.get("ORYX_ALS_VARIANT"), _build.TUNING_SO))
    # ORYX_ALS_WIDE_VARIANT: 64 < k <= 128 and fp32-mode solve (2 = als_solve_batch_gl,
    # 0 = als_solve_wide / als_solve_wave, 1 = als_solve_block)
    _sig(lib, "oryx_als_set_wide_variant", c_i, [c_i])
    _sig(lib, "oryx_als_get_wide_variant", c_i, [])
    if lib.oryx_als_set_wide_variant(int(os.environ.get("ORYX_ALS_WIDE_VARIANT", "2"))) != 0:
        raise RuntimeError("ORYX_ALS_WIDE_VARIANT=%s needs the tuning build of the kernels "
                           "(python -m oryx_amd._build --tuning; ORYX_KERNELS_SO=%s)"
                           % (os.environ.get("ORYX_ALS_WIDE_VARIANT"), _build.TUNING_SO))
    # ..., n_long, ws, split (fp32 factors as bf16 hi|lo rows of 2*kp), nnz, epoch (long
    # rows' partial sums beside the solve; 0 = before it), stream
    _sig(lib, "oryx_als_solve", c_i, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i,
                                      c_i, c_f, c_f, c_i, c_vp, c_vp, c_vp, c_i, c_i, c_vp,
                                      c_i, c_ll, ctypes.c_uint, c_vp])
    _sig(lib, "oryx_als_ws_stride", c_i, [c_i])
    _sig(lib, "oryx_gramian_ws_floats", c_i, [c_i])
    _sig(lib, "oryx_als_tuning_available", c_i, [])
    if lib.oryx_als_tuning_available():
        # superseded kernels and their analysis entry points: the tuning build only
        # (python -m oryx_amd._build --tuning; csrc/kernels/tuning/als_variants.hip)
        _sig(lib, "oryx_als_solve_profile64", c_i, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                    c_i, c_i, c_f, c_f, c_i, c_i, c_vp, c_vp])
        _sig(lib, "oryx_als_debug_gram", c_i, [c_vp, c_vp, c_vp, c_vp, c_i, c_f, c_i, c_ll,
                                               c_ll, c_vp, c_i, c_vp])
    _sig(lib, "oryx_gramian_f32", c_i, [c_vp, c_ll, c_i, c_i, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_kmeans_nearest_chunks", c_i, [c_ll, c_i])
    _sig(lib, "oryx_kmeans_nearest_f64", c_i, [c_vp, c_ll, c_i, c_vp, c_i, c_vp, c_vp, c_vp, c_vp,
                                               c_vp])
    _sig(lib, "oryx_spd_inverse_pair", c_i, [c_vp, c_vp, c_i, c_vp, c_vp, ctypes.c_double,
                                             c_vp, c_vp])
    _sig(lib, "oryx_pair_dots", c_i, [c_vp, c_vp, c_vp, c_vp, c_ll, c_i, c_vp, c_vp])
    # one-shot IPC all-reduce (ipc_allreduce.hip; parallel/ipc.py)
    _sig(lib, "oryx_ipc_alloc", c_i, [c_ll, c_vp])
    _sig(lib, "oryx_ipc_free", c_i, [c_vp])
    _sig(lib, "oryx_ipc_handle_size", c_i, [])
    _sig(lib, "oryx_ipc_handle", c_i, [c_vp, c_vp])
    _sig(lib, "oryx_ipc_open", c_i, [c_vp, c_vp])
    _sig(lib, "oryx_ipc_close", c_i, [c_vp])
    _sig(lib, "oryx_ipc_allreduce_f32", c_i, [c_vp, c_ll, c_vp, c_i, c_i, ctypes.c_uint, c_ll,
                                              ctypes.c_double, c_vp, c_vp])
    _sig(lib, "oryx_ipc_header_floats", c_ll, [])
    # numeric CSV lines -> feature matrix on the device (csv.hip; models/features.py)
    # buf, starts, ends, n, default_ts, out_u, out_i, out_s, out_ts, bad, n_bad, stream
    _sig(lib, "oryx_rating_lines", c_i, [c_vp, c_vp, c_vp, c_ll, c_ll, c_vp, c_vp, c_vp, c_vp,
                                         c_vp, c_vp, c_vp])
    _sig(lib, "oryx_csv_lines_to_matrix", c_i, [c_vp, c_vp, c_vp, c_ll, c_i, c_vp, c_vp, c_i,
                                                c_vp, c_i, c_vp, c_vp, c_i, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_format_f64_slots", c_i, [c_vp, c_ll, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_csv_wide_lines_to_matrix", c_i, [c_vp, c_vp, c_vp, c_ll, c_i, c_vp, c_i,
                                                     c_vp, c_i, c_vp, c_vp, c_vp, c_i, c_vp,
                                                     c_vp, c_vp])
    # peer-push all-gather (ipc_allgather.hip; parallel/ipc.py IpcAllGather)
    _sig(lib, "oryx_ipc_xcd_probe", c_i, [c_vp, c_vp, c_ll, c_vp, c_vp])
    _sig(lib, "oryx_ipc_gather_flag_bytes", c_ll, [])
    _sig(lib, "oryx_ipc_gather_limits", c_i, [c_vp])
    _sig(lib, "oryx_ipc_handle_range", c_i, [c_vp, c_vp, c_vp])
    _sig(lib, "oryx_ipc_gather_ready", c_i, [c_vp, c_i, ctypes.c_uint, c_vp])
    _sig(lib, "oryx_ipc_gather_push", c_i, [c_vp, c_ll, c_vp, c_ll, c_vp, c_i, c_i, c_i, c_i,
                                            c_i, c_i, ctypes.c_uint, ctypes.c_double, c_vp,
                                            c_vp])
    _sig(lib, "oryx_ipc_gather_wait", c_i, [c_vp, c_i, c_i, c_i, c_i, ctypes.c_uint,
                                            ctypes.c_double, c_vp, c_vp])
    _sig(lib, "oryx_kmeans_assign", c_i, [c_vp, c_vp, c_vp, c_ll, c_i, c_i, c_vp, c_vp, c_vp,
                                          c_vp])
    # X, xnorm, C, n, d_pad, k_pad, cnorm, Xf, ldx, d, Cf, CT2, k, cmax, assign, mind, idx2,
    # flags, stats, list2, defer_full, stream
    _sig(lib, "oryx_kmeans_assign_cert", c_i, [c_vp, c_vp, c_vp, c_ll, c_i, c_i, c_vp, c_vp, c_i,
                                               c_i, c_vp, c_vp, c_i, c_f, c_vp, c_vp, c_vp, c_vp,
                                               c_vp, c_vp, c_i, c_vp])
    _sig(lib, "oryx_kmeans_rescore_list", c_i, [c_vp, c_i, c_i, c_vp, c_i, c_vp, c_ll, c_vp,
                                                c_vp, c_vp])
    # x, xT, cl, csize, s, d, partial, stream
    _sig(lib, "oryx_kmeans_silhouette_mfma_rows", c_i, [c_i])
    # xp, xn, cl, csize, s, ks, bounds, nsplit, work, partial, stream
    _sig(lib, "oryx_kmeans_silhouette_mfma", c_i, [c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_vp, c_i,
                                                   c_vp, c_vp, c_vp])
    _sig(lib, "oryx_kmeans_silhouette", c_i, [c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_vp, c_i, c_vp,
                                              c_vp, c_vp])
    # X, Y, k, xrow, yrow, vals, xinv, yinv, implicit, n, new_x, new_y, vx, vy, stream
    _sig(lib, "oryx_als_foldin", c_i, [c_vp, c_vp, c_i, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_ll,
                                       c_vp, c_vp, c_vp, c_vp, c_vp])
    # M, n, k, ld, row_len, stream / M, n, k, ld, row_end, row_len, out, stream
    _sig(lib, "oryx_format_rows_len", c_i, [c_vp, c_ll, c_i, c_ll, c_vp, c_vp])
    _sig(lib, "oryx_format_rows_text", c_i, [c_vp, c_ll, c_i, c_ll, c_vp, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_format_csv_len", c_i, [c_vp, c_ll, c_i, c_ll, c_vp, c_vp])
    _sig(lib, "oryx_format_csv_text", c_i, [c_vp, c_ll, c_i, c_ll, c_vp, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_topn_waves", c_ll, [c_ll])
    # Y, inv_norm, Q, kp, nq, bucket_of, cand_bits, words, ranges, tile0, n_ranges, n_tiles,
    # excl_ptr, excl_rows, out_score, out_row, stream
    # Y, perm, ld, Q, kp, nq, cosine, kl, bucket_of, cand_bits, words, ranges, tile0,
    # n_ranges, n_tiles, excl_ptr, excl_rows, out_score, out_row, stream
    _sig(lib, "oryx_topn_scan2", c_i, [c_vp, c_vp, c_ll, c_vp, c_i, c_i, c_i, c_i, c_vp, c_vp,
                                       c_i, c_vp, c_vp, c_i, c_ll, c_vp, c_vp, c_vp, c_vp,
                                       c_vp])
    _sig(lib, "oryx_topn_scan3", c_i, [c_vp, c_vp, c_ll, c_vp, c_ll, c_vp, c_i, c_i, c_i, c_i,
                                       c_vp, c_vp, c_i, c_vp, c_vp, c_i, c_ll, c_vp, c_vp,
                                       c_vp, c_vp, c_vp])
    _sig(lib, "oryx_topn_waves_kl", c_ll, [c_ll, c_i])
    _sig(lib, "oryx_topn_max_queries", c_i, [c_i])
    _sig(lib, "oryx_counting_sort", c_i, [c_vp, c_ll, c_i, c_vp, c_vp, c_vp, c_vp])
    # ..., hist, n_live (device piece count, nullable), stream
    _sig(lib, "oryx_rdf_histogram_pieces", c_i, [c_vp, c_i, c_ll, c_i, c_i, c_vp, c_vp, c_i, c_i,
                                                 c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i,
                                                 c_vp, c_i, c_i, c_vp, c_vp, c_vp])
    # seed, total, out, stream
    _sig(lib, "oryx_rdf_poisson_weights", c_i, [ctypes.c_ulonglong, c_ll, c_vp, c_vp])
    # Xb, bin_bytes, n, P, p_used, T, node_of, nodes, feat, bin, cat_left, B, child_base,
    # weight, width, keys, stream
    _sig(lib, "oryx_rdf_route_keys", c_i, [c_vp, c_i, c_ll, c_i, c_i, c_i, c_vp, c_i, c_vp, c_vp,
                                           c_vp, c_i, c_vp, c_vp, c_i, c_vp, c_vp])
    # node_of, weight, label, y, S, cls, T, n, width, hist, visits, stream
    _sig(lib, "oryx_rdf_node_totals", c_i, [c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_ll, c_i,
                                            c_vp, c_vp, c_vp])
    # X, n, F, T, roots, feat, thr, cat_off, cat_bits, cat_len, left, right, leaf_value, C,
    # weights, vote, stream
    _sig(lib, "oryx_rdf_forest_vote", c_i, [c_vp, c_ll, c_i, c_i, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_vp, c_vp, c_vp, c_vp, c_i, c_vp, c_vp, c_vp])
    # counts, T, W, lo, hi, piece, max_pieces, ptree, pnode, pbeg, pend, n_live, stream
    _sig(lib, "oryx_rdf_expand_pieces", c_i, [c_vp, c_i, c_i, c_i, c_i, c_ll, c_i, c_vp, c_vp,
                                              c_vp, c_vp, c_vp, c_vp])
    # hist, feats, is_cat, T, W, Fs, B, S, kind, force_leaf, feat, bin, tot, gain, cat_left,
    # err, stream
    _sig(lib, "oryx_rdf_best_split", c_i, [c_vp, c_vp, c_vp, c_i, c_i, c_i, c_i, c_i, c_i, c_i,
                                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_kmeans_sorted_ws_bytes", c_ll, [c_ll, c_i])
    _sig(lib, "oryx_kmeans_pp", c_i, [c_vp, c_vp, c_vp, c_ll, c_i, c_i, c_vp, c_vp, c_vp, c_vp,
                                      c_vp])
    _sig(lib, "oryx_kmeans_accumulate_sorted", c_i, [c_vp, c_vp, c_vp, c_ll, c_i, c_i, c_i,
                                                     c_vp, c_vp, c_vp, c_vp, c_vp])
    _sig(lib, "oryx_kmeans_accumulate", c_i, [c_vp, c_vp, c_vp, c_ll, c_i, c_i, c_i, c_vp,
                                              c_vp, c_vp, c_vp])
    # Xb, bin_bytes, n, P, label, y, S, cls, weight, T, node_of, node_lo, nodes, feats, Fs, B,
    # hist, stream
    _sig(lib, "oryx_rdf_histogram", c_i, [c_vp, c_i, c_ll, c_i, c_vp, c_vp, c_i, c_i, c_vp, c_i,
                                          c_vp, c_i, c_i, c_vp, c_i, c_i, c_vp, c_vp])
    # Xb, bin_bytes, n, P (row pitch), p_used (bytes of a row in use), T, node_of, nodes,
    # split_feat, split_bin, cat_left, B, child_base, visits, stream
    _sig(lib, "oryx_rdf_sort_keys", c_i, [c_vp, c_vp, c_i, c_ll, c_i, c_vp, c_vp])
    _sig(lib, "oryx_rdf_route", c_i, [c_vp, c_i, c_ll, c_i, c_i, c_i, c_vp, c_i, c_vp, c_vp,
                                      c_vp, c_i, c_vp, c_vp, c_vp])
    # X, n, F, T, roots, feat, thr, cat_off, cat_bits, cat_len, left, right, leaf, stream
    _sig(lib, "oryx_rdf_forest_leaf", c_i, [c_vp, c_ll, c_i, c_i, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_vp, c_vp, c_vp, c_vp, c_vp])
    return lib


def kernels():
    global _kernels, _kernels_error
    if _kernels is None and _kernels_error is None:
        with _lock:
            if _kernels is None and _kernels_error is None:
                try:
                    _kernels = _load_kernels()
                except Exception as e:  # recorded; require_kernels() re-raises
                    _kernels_error = e
    if _kernels is None:
        raise RuntimeError("oryx_amd HIP kernels unavailable: %r" % (_kernels_error,))
    return _kernels


def kernels_available() -> bool:
    try:
        kernels()
        return True
    except Exception:
        return False


def require_kernels():
    """Fail loudly when the HIP kernels cannot be used on a GPU device."""
    return kernels()


def stream_ptr(device=None) -> int:
    """The calling thread's current HIP stream on ``device`` (raw pointer): one cheap
    runtime query per launch -- ``torch.cuda.current_stream`` costs ~8 us of Python, a
    visible share of a small serving request's launches."""
    import torch
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:
        idx = getattr(device, "index", None) if device is not None else None
        if idx is None:
            idx = device if isinstance(device, int) else torch.cuda.current_device()
        return raw(idx)
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError("%s failed (native error %d)" % (what, rc))
