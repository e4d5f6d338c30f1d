"""ctypes binding of dccrg_amd/libdccrgx.so (C ABI declared in include/dccrgx.h).

The product path is the HIP library; there is no CPU fallback.  Importing
this module fails loudly if the library has not been built.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# DCCRGX_LIB: another in-tree build of the same library (a paired A/B of two
# builds, dccrg_amd/build.py `out=`); the default is the product build
LIB_PATH = os.path.join(HERE, os.path.basename(os.environ.get("DCCRGX_LIB", "libdccrgx.so")))
HEADER = os.path.join(os.path.dirname(HERE), "include", "dccrgx.h")

_lib = None

# int (*)(void* ctx, const void* const* send, const size_t* send_bytes,
#         void* const* recv, const size_t* recv_bytes)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_void_p),
                          C.POINTER(C.c_size_t))

u64 = C.c_uint64
i64 = C.c_int64
i32 = C.c_int32
sz = C.c_size_t
vp = C.c_void_p
P = C.POINTER

_SIGS = {
    "dccrgx_last_error": (C.c_char_p, []),
    "dccrgx_abi_version": (C.c_int, []),
    "dccrgx_get_unique_id": (C.c_int, [vp]),
    "dccrgx_create": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, P(vp)]),
    "dccrgx_create_with_exchange": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, vp, P(vp)]),
    "dccrgx_destroy": (C.c_int, [vp]),
    "dccrgx_device_count": (C.c_int, [P(C.c_int)]),
    "dccrgx_get_cells_by_criteria": (C.c_int, [vp, vp, sz, C.c_int, C.c_int, vp, sz, P(sz)]),
    "dccrgx_get_slots": (C.c_int, [vp, vp, sz, vp]),
    "dccrgx_download_user_csr": (C.c_int, [vp, C.c_int, C.c_int, vp, vp, vp, sz, P(sz)]),
    "dccrgx_set_initial_length": (C.c_int, [vp, P(u64)]),
    "dccrgx_set_maximum_refinement_level": (C.c_int, [vp, C.c_int]),
    "dccrgx_get_maximum_refinement_level": (C.c_int, [vp, P(C.c_int)]),
    "dccrgx_get_neighborhood_length": (C.c_int, [vp, P(C.c_uint)]),
    "dccrgx_get_initial_length": (C.c_int, [vp, vp]),
    "dccrgx_get_periodic": (C.c_int, [vp, vp]),
    "dccrgx_get_geometry": (C.c_int, [vp, vp, vp]),
    "dccrgx_set_geometry_block": (C.c_int, [vp, vp, sz]),
    "dccrgx_get_geometry_block": (C.c_int, [vp, vp, sz, P(sz)]),
    "dccrgx_set_periodic": (C.c_int, [vp, C.c_int, C.c_int, C.c_int]),
    "dccrgx_set_neighborhood_length": (C.c_int, [vp, C.c_uint]),
    "dccrgx_initialize": (C.c_int, [vp]),
    "dccrgx_set_geometry": (C.c_int, [vp, P(C.c_double), P(C.c_double)]),
    "dccrgx_geometry_batch": (C.c_int, [vp, vp, sz, vp, vp]),
    "dccrgx_get_cell_from_indices": (u64, [vp, P(u64), C.c_int]),
    "dccrgx_get_indices": (C.c_int, [vp, u64, P(u64)]),
    "dccrgx_get_refinement_level": (C.c_int, [vp, u64]),
    "dccrgx_get_last_cell": (u64, [vp]),
    "dccrgx_mapping_batch": (C.c_int, [vp, vp, sz, vp, vp]),
    "dccrgx_get_cells": (C.c_int, [vp, C.c_int, vp, sz, P(sz)]),
    "dccrgx_get_counts": (C.c_int, [vp, P(sz), P(sz), P(sz), P(sz)]),
    "dccrgx_get_neighbors_of": (C.c_int, [vp, u64, vp, vp, sz, P(sz)]),
    "dccrgx_get_slot_ids": (C.c_int, [vp, vp, sz, P(sz)]),
    "dccrgx_download_csr": (C.c_int, [vp, C.c_int, vp, vp, vp, sz, P(sz)]),
    "dccrgx_get_neighbors_to": (C.c_int, [vp, u64, vp, sz, P(sz)]),
    "dccrgx_get_face_neighbors_of": (C.c_int, [vp, u64, vp, vp, sz, P(sz)]),
    "dccrgx_is_local": (C.c_int, [vp, u64]),
    "dccrgx_get_process": (C.c_int, [vp, u64]),
    "dccrgx_get_slot": (i64, [vp, u64]),
    "dccrgx_get_peers": (C.c_int, [vp, vp, sz, P(sz)]),
    "dccrgx_get_cells_to_send": (C.c_int, [vp, C.c_int, vp, sz, P(sz)]),
    "dccrgx_get_cells_to_receive": (C.c_int, [vp, C.c_int, vp, sz, P(sz)]),
    "dccrgx_get_number_of_update_cells": (C.c_int, [vp, P(u64), P(u64)]),
    "dccrgx_refine_completely": (C.c_int, [vp, u64]),
    "dccrgx_unrefine_completely": (C.c_int, [vp, u64]),
    "dccrgx_dont_unrefine": (C.c_int, [vp, u64]),
    "dccrgx_dont_refine": (C.c_int, [vp, u64]),
    "dccrgx_get_removed_cells": (C.c_int, [vp, vp, sz, P(sz)]),
    "dccrgx_removed_field_download": (C.c_int, [vp, C.c_int, vp, sz]),
    "dccrgx_removed_field_device_ptr": (C.c_int, [vp, C.c_int, P(vp)]),
    "dccrgx_stop_refining": (C.c_int, [vp, vp, sz, P(sz)]),
    "dccrgx_get_new_cells": (C.c_int, [vp, vp, sz, P(sz)]),
    "dccrgx_set_cells": (C.c_int, [vp, vp, vp, sz]),
    "dccrgx_pin": (C.c_int, [vp, u64, C.c_int]),
    "dccrgx_unpin": (C.c_int, [vp, u64]),
    "dccrgx_balance_load": (C.c_int, [vp, C.c_int]),
    "dccrgx_balance_load_to": (C.c_int, [vp, vp, vp, sz]),
    "dccrgx_initialize_balance_load": (C.c_int, [vp, C.c_int, vp, vp, sz]),
    "dccrgx_make_new_partition": (C.c_int, [vp, vp, vp, sz, P(sz)]),
    "dccrgx_set_load_balancing_method": (C.c_int, [vp, C.c_char_p]),
    "dccrgx_get_load_balancing_method": (C.c_int, [vp, C.c_char_p, sz]),
    "dccrgx_set_cell_weight": (C.c_int, [vp, u64, C.c_double]),
    "dccrgx_get_cell_weight": (C.c_double, [vp, u64]),
    "dccrgx_continue_balance_load": (C.c_int, [vp]),
    "dccrgx_get_migration_cells": (C.c_int, [vp, C.c_int, C.c_int, vp, sz, P(sz)]),
    "dccrgx_finish_balance_load": (C.c_int, [vp]),
    "dccrgx_migration_message_size": (C.c_int, [vp, C.c_int, P(sz), P(sz)]),
    "dccrgx_migration_pack": (C.c_int, [vp, C.c_int, vp, sz]),
    "dccrgx_migration_place": (C.c_int, [vp, C.c_int, vp, sz]),
    "dccrgx_halo_message_size": (C.c_int, [vp, C.c_int, C.c_int, P(sz), P(sz)]),
    "dccrgx_halo_pack": (C.c_int, [vp, C.c_int, C.c_int, vp, sz]),
    "dccrgx_halo_place": (C.c_int, [vp, C.c_int, C.c_int, vp, sz]),
    "dccrgx_save_grid_data": (C.c_int, [vp, C.c_char_p, C.c_uint64, vp, sz]),
    "dccrgx_load_grid_data": (C.c_int, [vp, C.c_char_p, C.c_uint64, sz]),
    "dccrgx_start_loading_grid_data": (C.c_int, [vp, C.c_char_p, C.c_uint64, sz]),
    "dccrgx_continue_loading_grid_data": (C.c_int, [vp, C.c_int, vp]),
    "dccrgx_finish_loading_grid_data": (C.c_int, [vp]),
    "dccrgx_grid_file_bytes_left": (C.c_int, [vp, vp]),
    "dccrgx_add_neighborhood": (C.c_int, [vp, C.c_int, vp, sz]),
    "dccrgx_remove_neighborhood": (C.c_int, [vp, C.c_int]),
    "dccrgx_get_user_neighbors": (C.c_int, [vp, C.c_int, C.c_uint64, C.c_int, vp, vp, sz, P(sz)]),
    "dccrgx_get_user_update_list": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, sz, P(sz)]),
    "dccrgx_update_copies_of_remote_neighbors_hood": (C.c_int, [vp, C.c_int]),
    "dccrgx_get_cell_process": (C.c_int, [vp, vp, vp, sz, P(sz)]),
    "dccrgx_find_neighbors_of": (C.c_int, [vp, u64, vp, sz, vp, vp, sz, P(sz)]),
    "dccrgx_get_face_cache": (C.c_int, [vp, vp, vp, sz, P(sz)]),
    "dccrgx_unpin_all_cells": (C.c_int, [vp]),
    "dccrgx_add_field": (C.c_int, [vp, C.c_char_p, sz, C.c_int, P(C.c_int)]),
    "dccrgx_set_field_transfer": (C.c_int, [vp, C.c_int, C.c_int]),
    "dccrgx_add_variable_field": (C.c_int, [vp, C.c_char_p, C.c_int, P(C.c_int)]),
    "dccrgx_variable_field_sizes": (C.c_int, [vp, C.c_int, sz, sz, vp]),
    "dccrgx_variable_field_resize": (C.c_int, [vp, C.c_int, sz, sz, vp]),
    "dccrgx_variable_field_upload": (C.c_int, [vp, C.c_int, sz, sz, vp, sz]),
    "dccrgx_variable_field_download": (C.c_int, [vp, C.c_int, sz, sz, vp, sz, P(sz)]),
    "dccrgx_variable_field_device_ptr": (C.c_int, [vp, C.c_int, P(vp), P(vp)]),
    "dccrgx_removed_variable_field_download": (C.c_int, [vp, C.c_int, vp, vp, sz, P(sz)]),
    "dccrgx_set_send_single_cells": (C.c_int, [vp, C.c_int]),
    "dccrgx_get_send_single_cells": (C.c_int, [vp, P(C.c_int)]),
    "dccrgx_set_field_window": (C.c_int, [vp, C.c_int, sz, sz]),
    "dccrgx_field_device_ptr": (C.c_int, [vp, C.c_int, P(vp)]),
    "dccrgx_field_upload": (C.c_int, [vp, C.c_int, sz, sz, vp]),
    "dccrgx_field_download": (C.c_int, [vp, C.c_int, sz, sz, vp]),
    "dccrgx_update_copies_of_remote_neighbors": (C.c_int, [vp]),
    "dccrgx_start_remote_neighbor_copy_updates": (C.c_int, [vp]),
    "dccrgx_wait_remote_neighbor_copy_update_receives": (C.c_int, [vp]),
    "dccrgx_wait_remote_neighbor_copy_update_sends": (C.c_int, [vp]),
    "dccrgx_wait_remote_neighbor_copy_updates": (C.c_int, [vp]),
    "dccrgx_gol_step": (C.c_int, [vp, C.c_int, C.c_int]),
    "dccrgx_gol_commit": (C.c_int, [vp, C.c_int]),
    "dccrgx_gol_amr": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int]),
    "dccrgx_get_live_neighbors": (C.c_int, [vp, C.c_int, C.c_int]),
    "dccrgx_advection_step": (C.c_int, [vp, P(C.c_int), C.c_double, C.c_int]),
    "dccrgx_advection_commit": (C.c_int, [vp, C.c_int]),
    "dccrgx_advection_initialize": (C.c_int, [vp, P(C.c_int)]),
    "dccrgx_advection_max_time_step": (C.c_int, [vp, P(C.c_int), P(C.c_double)]),
    "dccrgx_advection_max_time_step_device": (C.c_int, [vp, P(C.c_int), vp]),
    "dccrgx_advection_check_adaptation": (C.c_int, [vp, C.c_int, C.c_double, C.c_double, C.c_double, vp]),
    "dccrgx_advection_adapt": (C.c_int, [vp, vp, vp]),
    "dccrgx_advection_refine_candidates": (C.c_int, [vp, C.c_int, C.c_double, C.c_double, vp, sz, P(sz)]),
    "dccrgx_advection_layout": (C.c_int, [vp, P(u64)]),
    "dccrgx_poisson_cache": (C.c_int, [vp, C.c_int, C.c_int, vp, sz, vp, sz]),
    "dccrgx_poisson_solve": (C.c_int, [vp, C.c_uint, C.c_uint, C.c_double, C.c_double, C.c_double, C.c_int,
                                       P(C.c_uint), P(C.c_double)]),
    "dccrgx_poisson_field": (C.c_int, [vp, C.c_char_p, P(C.c_int)]),
    "dccrgx_allreduce_f64": (C.c_int, [vp, P(C.c_double), C.c_int, C.c_int]),
    "dccrgx_allreduce_f64_device": (C.c_int, [vp, vp, vp, C.c_int, C.c_int]),
    "dccrgx_barrier": (C.c_int, [vp]),
    "dccrgx_get_transport": (C.c_int, [vp, P(C.c_int), P(C.c_int)]),
    "dccrgx_comm_loopback": (C.c_int, [vp, C.c_int, sz, sz, sz]),
    "dccrgx_synchronize": (C.c_int, [vp]),
    "dccrgx_compute_stream": (vp, [vp]),
    "dccrgx_kernel_timing": (C.c_int, [vp, C.c_int, P(C.c_double), P(i64)]),
}


def header_symbols():
    """Every function the C header declares."""
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(dccrgx_[a-z0-9_]+)\s*\(", txt)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"dccrg_amd native library missing: {LIB_PATH} (run python -m dccrg_amd.build)")
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class DccrgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"dccrgx error {code}: {msg}")
        self.code = code


OK, EINVAL, EHIP, ECOMM, ERANGE, ENOTFOUND = 0, -1, -2, -3, -4, -5


def check(rc):
    if rc != 0:
        raise DccrgError(rc, lib().dccrgx_last_error().decode())
    return rc
