"""ctypes binding of libkodr_rlnc.so (include/kodr_rlnc.h).

The shared library is built in-tree by kodr_amd/build.sh (or
``__graft_entry__.build()``).  There is no pure-Python fallback: if the library
is missing or no HIP device is usable, data-plane calls raise.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# rlnc_hook_fn (rlnc_decoders_add_pieces_gpu_hook): keep the wrapped object alive for the call
HOOK_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p)
LIB_PATH = os.environ.get("KODR_RLNC_LIB", os.path.join(_HERE, "libkodr_rlnc.so"))

_u8p = ctypes.POINTER(ctypes.c_uint8)
_sz = ctypes.c_size_t
_szp = ctypes.POINTER(ctypes.c_size_t)
_vp = ctypes.c_void_p
_vpp = ctypes.POINTER(ctypes.c_void_p)
_int = ctypes.c_int

# name -> (restype, argtypes); mirrors include/kodr_rlnc.h one to one
SIGNATURES = {
    "rlnc_version": (ctypes.c_char_p, []),
    "rlnc_status_string": (ctypes.c_char_p, [_int]),
    "rlnc_last_hip_error": (ctypes.c_char_p, []),
    "rlnc_device_count": (_int, [ctypes.POINTER(_int)]),
    "rlnc_ctx_create": (_int, [_int, _vp, _vpp]),
    "rlnc_ctx_destroy": (_int, [_vp]),
    "rlnc_ctx_synchronize": (_int, [_vp]),
    "rlnc_ctx_stream": (_vp, [_vp]),
    "rlnc_ctx_set_route_min_k": (_int, [_vp, _sz]),
    "rlnc_ctx_elim_stats": (_int, [_vp, _szp, _szp, _szp, _szp]),
    "rlnc_random_bytes": (_int, [_u8p, _sz]),
    "rlnc_device_pool_trim": (_int, [_int, _sz]),
    "rlnc_device_pool_cached": (_sz, [_int]),
    "rlnc_dev_alloc": (_int, [_vp, _sz, _vpp]),
    "rlnc_dev_free": (_int, [_vp, _vp]),
    "rlnc_memcpy_h2d": (_int, [_vp, _vp, _vp, _sz]),
    "rlnc_memcpy_d2h": (_int, [_vp, _vp, _vp, _sz]),
    "rlnc_memcpy_d2d_async": (_int, [_vp, _vp, _vp, _sz]),
    "rlnc_host_register": (_int, [_vp, _vp, _sz]),
    "rlnc_host_unregister": (_int, [_vp, _vp]),
    "rlnc_event_create": (_int, [_vp, _vpp]),
    "rlnc_event_record": (_int, [_vp, _vp]),
    "rlnc_event_elapsed_ms": (_int, [_vp, _vp, ctypes.POINTER(ctypes.c_float)]),
    "rlnc_ctx_wait_event": (_int, [_vp, _vp]),
    "rlnc_event_destroy": (_int, [_vp]),
    "rlnc_split_by_piece_count": (_int, [_sz, _sz, _szp, _szp]),
    "rlnc_split_by_piece_size": (_int, [_sz, _sz, _szp, _szp]),
    "rlnc_coded_pieces_for_recoding": (_int, [_sz, _sz, _sz, _szp]),
    "rlnc_is_systematic": (_int, [_u8p, _sz]),
    "rlnc_encoder_create_with_piece_count": (_int, [_vp, _int, _u8p, _sz, _sz, _vpp]),
    "rlnc_encoder_create_with_piece_size": (_int, [_vp, _int, _u8p, _sz, _sz, _vpp]),
    "rlnc_encoder_create": (_int, [_vp, _int, _u8p, _sz, _sz, _vpp]),
    "rlnc_encoder_create_device": (_int, [_vp, _int, _vp, _sz, _sz, _sz, _vpp]),
    "rlnc_encoder_destroy": (_int, [_vp]),
    "rlnc_encoder_piece_count": (_sz, [_vp]),
    "rlnc_encoder_piece_size": (_sz, [_vp]),
    "rlnc_encoder_decodable_len": (_sz, [_vp]),
    "rlnc_encoder_coded_piece_len": (_sz, [_vp]),
    "rlnc_encoder_padding": (_sz, [_vp]),
    "rlnc_encoder_device_pieces": (_vp, [_vp, _szp]),
    "rlnc_encoder_systematic_remaining": (_sz, [_vp]),
    "rlnc_encoder_coded_pieces": (_int, [_vp, _u8p, _sz, _u8p]),
    "rlnc_encoder_coded_pieces_device": (_int, [_vp, _vp, _sz, _vp, _sz]),
    "rlnc_encoder_coded_wire_device": (_int, [_vp, _sz, _vp, _sz]),
    "rlnc_encoder_seed": (_int, [_vp, ctypes.c_uint64]),
    "rlnc_encoder_prepare": (_int, [_vp]),
    "rlnc_encoder_compact": (_int, [_vp]),
    "rlnc_encoder_group_coded_pieces_device": (_int, [_vpp, _sz, _vp, _sz, _vp, _sz]),
    "rlnc_encoder_group_coded_wire_device": (_int, [_vpp, _sz, _sz, _vp, _sz]),
    "rlnc_recoder_create": (_int, [_vp, _u8p, _sz, _sz, _sz, _vpp]),
    "rlnc_recoder_create_device": (_int, [_vp, _vp, _sz, _sz, _sz, _sz, _vpp]),
    "rlnc_recoder_destroy": (_int, [_vp]),
    "rlnc_recoder_prepare": (_int, [_vp]),
    "rlnc_recoder_compact": (_int, [_vp]),
    "rlnc_recoder_piece_count": (_sz, [_vp]),
    "rlnc_recoder_coded_piece_len": (_sz, [_vp]),
    "rlnc_recoder_coded_pieces": (_int, [_vp, _u8p, _sz, _u8p]),
    "rlnc_recoder_coded_pieces_device": (_int, [_vp, _vp, _sz, _vp, _sz]),
    "rlnc_decoder_create": (_int, [_vp, _sz, _vpp]),
    "rlnc_decoder_destroy": (_int, [_vp]),
    "rlnc_decoder_add_piece": (_int, [_vp, _u8p, _sz, _u8p, _sz]),
    "rlnc_decoder_add_piece_device": (_int, [_vp, _u8p, _sz, _vp, _sz]),
    "rlnc_decoder_add_piece_device_borrowed": (_int, [_vp, _u8p, _sz, _vp, _sz]),
    "rlnc_decoder_add_pieces": (_int, [_vp, _vp, _sz, _sz, _sz, _int, _szp]),
    "rlnc_decoder_add_pieces_gpu": (_int, [_vp, _vp, _sz, _sz, _sz, _szp]),
    "rlnc_decoder_set_policy": (_int, [_vp, _int]),
    "rlnc_decoder_decoded_mask": (_sz, [_vp, _u8p]),
    "rlnc_decoder_get_decoded": (_int, [_vp, _sz, _vp, _int]),
    "rlnc_decoder_bind_output": (_int, [_vp, _vp, _sz]),
    "rlnc_decoders_add_pieces_gpu": (_int, [_vp, _sz, _vp, _vp, _sz, _sz, _vp, _vp]),
    "rlnc_decoders_add_pieces_gpu_hook": (_int, [_vp, _sz, _vp, _vp, _sz, _sz, _vp, _vp, _vp, _vp]),
    "rlnc_decoders_flush_gpu": (_int, [_vp, _sz]),
    "rlnc_decoders_get_pieces_device": (_int, [_vp, _sz, _vp, _sz]),
    "rlnc_recoder_group_coded_pieces_device": (_int, [_vpp, _sz, _vp, _sz, _vp, _sz]),
    "rlnc_decoder_is_decoded": (_int, [_vp]),
    "rlnc_decoder_required": (_sz, [_vp]),
    "rlnc_decoder_useful": (_sz, [_vp]),
    "rlnc_decoder_received": (_sz, [_vp]),
    "rlnc_decoder_piece_length": (_sz, [_vp]),
    "rlnc_decoder_piece_count": (_sz, [_vp]),
    "rlnc_decoder_get_piece": (_int, [_vp, _sz, _u8p]),
    "rlnc_decoder_get_pieces": (_int, [_vp, _u8p]),
    "rlnc_decoder_get_pieces_device": (_int, [_vp, _vp, _sz]),
    "rlnc_decoder_coefficients": (_int, [_vp, _u8p]),
    "rlnc_decoder_apply_stats": (_int, [_vp, _szp, _szp]),
    "rlnc_decoder_last_apply_bitsliced": (_int, [_vp]),
    "rlnc_decoder_elim_stats": (_int, [_vp, _szp, _szp, _szp, _szp]),
    "rlnc_decoder_transform": (_int, [_vp, _u8p]),
    "rlnc_gf_matmul_device": (_int, [_vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, _sz, _sz]),
    "rlnc_bitslice_device": (_int, [_vp, _vp, _sz, _sz, _sz]),
    "rlnc_bs_body_offsets": (_int, [_vp, _vp]),
    "rlnc_gf_matmul_bs_device": (_int, [_vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, _sz, _sz]),
    "rlnc_last_launch_plan": (_int, [_vp]),
}


class LaunchPlan(ctypes.Structure):
    """rlnc_launch_plan (include/kodr_rlnc.h): the last product launch of this thread."""
    _fields_ = [(n, ctypes.c_int) for n in ("kernel", "tile_rows", "waves", "lane_groups", "ring",
                                            "rows_per_wave", "generations", "workgroups")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


def last_launch_plan():
    p = LaunchPlan()
    rc = lib().rlnc_last_launch_plan(ctypes.byref(p))
    if rc != 0:
        raise RuntimeError(f"rlnc_last_launch_plan: {rc}")
    return p.as_dict()

_lib = None
_lock = threading.Lock()


class LibraryMissing(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes handle of libkodr_rlnc.so."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise LibraryMissing(
                    f"{LIB_PATH} not built: run kodr_amd/build.sh (or __graft_entry__.build())")
            h = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            _lib = h
    return _lib


def u8(buf):
    """Borrow a pointer to a bytes-like / numpy uint8 buffer (no copy when writable)."""
    import numpy as np
    arr = buf if isinstance(buf, np.ndarray) else np.frombuffer(bytes(buf), dtype=np.uint8)
    if arr.dtype != np.uint8 or not arr.flags["C_CONTIGUOUS"]:
        arr = np.ascontiguousarray(arr, dtype=np.uint8)
    return arr, arr.ctypes.data_as(_u8p)
