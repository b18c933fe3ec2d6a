"""ctypes binding of librtmi.so (include/rtmi.h).

The product path is the HIP library; there is no Python or CPU fallback.  If
the library is missing, `lib()` raises so a caller can never silently run
something else.
"""
from __future__ import annotations

import ctypes
import os

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RTMI_LIB: another build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("RTMI_LIB", os.path.join(_PKG_DIR, "build", "librtmi.so"))

RT_OK = 0
RT_E_INVALID = -1
RT_E_HIP = -2
RT_E_NOMEM = -3
RT_E_INTERNAL = -6
RT_E_IO = -4
RT_E_UNSUPPORTED = -5

RT_PRESET_CPU = 0
RT_PRESET_GPU = 1
RT_HIT_RULE_CPU = 0
RT_HIT_RULE_GPU = 1
RT_SAMPLER_UNIFORM = 0
RT_SAMPLER_COSINE = 1
RT_HIT_NONE = -1
RT_HIT_TYPE_LIGHT = 1
RT_HIT_TYPE_SURFACE = 2

# kernel families of rt_ktime_read
RT_KT_RENDER_PS = 0
RT_KT_RENDER = 1
RT_KT_SARSA_RENDER = 2
RT_KT_SARSA_APPLY = 3
RT_KT_DQN_MLP = 4
RT_KT_DQN_BOUNCE = 5
RT_KT_DQN_CAMERA = 6
RT_KT_COUNT = 7

# every symbol include/rtmi.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "rt_params_default", "rt_ctx_create", "rt_ctx_destroy", "rt_last_error",
    "rt_cornell_counts", "rt_cornell_geometry", "rt_obj_geometry",
    "rt_scene_create", "rt_scene_destroy", "rt_scene_normals",
    "rt_intersect", "rt_intersect_device", "rt_intersect_method", "rt_render", "rt_render_tiles_device",
    "rt_pack_argb", "rt_save_bmp", "rt_save_png", "rt_selftest", "rt_filter_build", "rt_rect_candidates", "rt_cull_masks_device",
    "rt_ctab_candidates",
    "rt_dynet_read", "rt_dynet_write", "rt_dqn_create", "rt_dqn_destroy", "rt_dqn_set_mlp", "rt_dqn_forward", "rt_dqn_forward_device",
    "rt_dqn_sample",
    "rt_render_dqn", "rt_render_dqn_tiles_device",
    "rt_sarsa_create", "rt_sarsa_create_density", "rt_sarsa_destroy", "rt_sarsa_info", "rt_sarsa_volumes", "rt_sarsa_read",
    "rt_sarsa_nearest", "rt_render_sarsa", "rt_render_sarsa_tiles_device", "rt_sarsa_td_device",
    "rt_sarsa_apply", "rt_sarsa_set_search", "rt_sarsa_search_stats", "rt_sarsa_save_q",
    "rt_neuralq_create", "rt_neuralq_destroy", "rt_neuralq_epsilon", "rt_neuralq_render_frame",
    "rt_sarsa_save_selected", "rt_sarsa_load_q", "rt_sarsa_set_sampling", "rt_sarsa_set_td_mode", "rt_sarsa_get_td_mode", "rt_sarsa_set_inframe_lanes", "rt_sarsa_frame_stats",
    "rt_dqn_save_selected",
    "rt_dqn_trainer_create", "rt_dqn_trainer_destroy", "rt_dqn_trainer_params", "rt_dqn_train_step_device",
    "rt_dqn_td_targets_device",
    "rt_scene_set_accel", "rt_scene_accel_info", "rt_scene_ctab_info", "rt_bvh_check",
    "rt_ktime_enable", "rt_ktime_read", "rt_ktime_name",
)


class RtCamera(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_float * 4), ("yaw_y", ctypes.c_float), ("yaw_x", ctypes.c_float)]


class RtParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
        ("max_bounces", ctypes.c_int32), ("sampler", ctypes.c_int32), ("preset", ctypes.c_int32),
        ("hit_rule", ctypes.c_int32), ("spp_split", ctypes.c_int32), ("seed", ctypes.c_uint64),
        ("env_light", ctypes.c_float), ("t_scale", ctypes.c_float),
    ]

    def to_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class RtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rtmi error {code}: {msg}")
        self.code = code


_LIB = None
_P = ctypes.c_void_p
_FP = ctypes.POINTER(ctypes.c_float)
_IP = ctypes.POINTER(ctypes.c_int32)
_UP = ctypes.POINTER(ctypes.c_uint32)
_U64P = ctypes.POINTER(ctypes.c_uint64)


def _declare(lib):
    i, f = ctypes.c_int, ctypes.c_float
    sig = {
        "rt_params_default": (i, [i, ctypes.POINTER(RtParams)]),
        "rt_ctx_create": (i, [i, ctypes.POINTER(_P)]),
        "rt_ctx_destroy": (i, [_P]),
        "rt_last_error": (ctypes.c_char_p, []),
        "rt_cornell_counts": (i, [ctypes.POINTER(i), ctypes.POINTER(i)]),
        "rt_cornell_geometry": (i, [i, _FP, _FP, _FP, _FP, _IP]),
        "rt_obj_geometry": (i, [ctypes.c_char_p, i, _FP, _FP, ctypes.POINTER(i), _FP, _FP, _IP,
                                ctypes.POINTER(i), _FP, ctypes.POINTER(i)]),
        "rt_scene_create": (i, [_P, _FP, _FP, i, _FP, _FP, _IP, i, ctypes.POINTER(_P)]),
        "rt_scene_destroy": (i, [_P]),
        "rt_scene_normals": (i, [_P, _FP]),
        "rt_intersect": (i, [_P, _P, _FP, _FP, i, f, i, _FP, _IP]),
        "rt_intersect_device": (i, [_P, _P, _P, _P, i, f, i, _P, _P, _P]),
        "rt_intersect_method": (i, [_P, _P, _FP, _FP, i, f, i, i, _FP, _IP, _IP]),
        "rt_scene_set_accel": (i, [_P, i]),
        "rt_scene_accel_info": (i, [_P, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(ctypes.c_int64)]),
        "rt_scene_ctab_info": (i, [_P, i, ctypes.POINTER(i), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_uint64)]),
        "rt_bvh_check": (i, [_FP, i, ctypes.POINTER(ctypes.c_int64)]),
        "rt_render": (i, [_P, _P, ctypes.POINTER(RtCamera), ctypes.POINTER(RtParams), i, i, i, i,
                          _FP, _U64P]),
        "rt_render_tiles_device": (i, [_P, _P, ctypes.POINTER(RtCamera), ctypes.POINTER(RtParams),
                                       _IP, i, i, _P, _P, _P]),
        "rt_pack_argb": (i, [_FP, i, _UP]),
        "rt_save_bmp": (i, [ctypes.c_char_p, _UP, i, i]),
        "rt_save_png": (i, [ctypes.c_char_p, _UP, i, i]),
        "rt_selftest": (i, [_P, i, _U64P]),
        "rt_filter_build": (i, [_FP, i, _FP]),
        "rt_cull_masks_device": (i, [_P, _P, ctypes.POINTER(RtCamera), ctypes.POINTER(RtParams), i, i, i, i,
                                     _U64P, ctypes.POINTER(ctypes.c_int64)]),
        "rt_rect_candidates": (i, [_FP, i, ctypes.POINTER(RtCamera), ctypes.POINTER(RtParams), i, i, i, i,
                                   _U64P]),
        "rt_ctab_candidates": (i, [_FP, i, i, i, _IP, _FP, _FP, i, _U64P, ctypes.POINTER(ctypes.c_int64)]),
        "rt_dynet_read": (i, [ctypes.c_char_p, i, _IP, _IP, _FP, ctypes.POINTER(i),
                              ctypes.POINTER(ctypes.c_int64)]),
        "rt_dynet_write": (i, [ctypes.c_char_p, i, _IP, _IP, _FP]),
        "rt_dqn_set_mlp": (i, [_P, i]),
        "rt_dqn_create": (i, [_P, _FP, i, _IP, i, ctypes.POINTER(_FP), ctypes.POINTER(_FP),
                              ctypes.POINTER(_P)]),
        "rt_dqn_destroy": (i, [_P]),
        "rt_dqn_trainer_create": (i, [_P, _FP, i, _IP, i, ctypes.POINTER(_FP), ctypes.POINTER(_FP), f,
                                      ctypes.POINTER(_P)]),
        "rt_dqn_trainer_destroy": (i, [_P]),
        "rt_dqn_trainer_params": (i, [_P, ctypes.POINTER(_FP), ctypes.POINTER(_FP)]),
        "rt_dqn_train_step_device": (i, [_P, _P, _P, _P, _P, i, _FP, _FP, _P]),
        "rt_dqn_td_targets_device": (i, [_P, ctypes.c_uint64, _P, _P, _P, _P, _P, i, i, i, _P, _P]),
        "rt_dqn_forward": (i, [_P, _P, _FP, i, _FP]),
        "rt_dqn_forward_device": (i, [_P, _P, _P, i, _P, _P]),
        "rt_dqn_sample": (i, [_P, _P, ctypes.c_uint64, _FP, _FP, _IP, _UP, i, i, i, _FP, _FP, _IP]),
        "rt_render_dqn": (i, [_P, _P, _P, ctypes.POINTER(RtCamera), ctypes.POINTER(RtParams), i, i,
                              i, i, _FP, _U64P]),
        "rt_render_dqn_tiles_device": (i, [_P, _P, _P, ctypes.POINTER(RtCamera),
                                           ctypes.POINTER(RtParams), _IP, i, i, _P, _P, _P]),
        "rt_sarsa_create": (i, [_P, _P, ctypes.c_uint64, ctypes.POINTER(_P)]),
        "rt_sarsa_create_density": (i, [_P, _P, ctypes.c_uint64, ctypes.c_float, ctypes.POINTER(_P)]),
        "rt_sarsa_destroy": (i, [_P]),
        "rt_sarsa_info": (i, [_P, _IP, _IP, _UP]),
        "rt_sarsa_set_search": (i, [_P, i]),
        "rt_sarsa_set_sampling": (i, [_P, i]),
        "rt_sarsa_set_td_mode": (i, [_P, i]),
        "rt_sarsa_set_inframe_lanes": (i, [_P, i]),
        "rt_sarsa_get_td_mode": (i, [_P, _IP]),
        "rt_neuralq_create": (i, [_P, _P, _P, i, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                  ctypes.POINTER(_P)]),
        "rt_neuralq_destroy": (i, [_P]),
        "rt_neuralq_epsilon": (i, [_P, _FP]),
        "rt_neuralq_render_frame": (i, [_P, _P, _P, _P, _FP, _FP, _U64P]),
        "rt_sarsa_load_q": (i, [_P, ctypes.c_char_p]),
        "rt_sarsa_frame_stats": (i, [_P, _U64P, _U64P]),
        "rt_sarsa_save_q": (i, [_P, ctypes.c_char_p]),
        "rt_dqn_save_selected": (i, [_P, _P, ctypes.c_char_p, ctypes.c_char_p]),
        "rt_sarsa_save_selected": (i, [_P, _P, ctypes.c_char_p, ctypes.c_char_p]),
        "rt_sarsa_search_stats": (i, [_P, _IP, _IP, ctypes.POINTER(ctypes.c_int64), _U64P]),
        "rt_sarsa_volumes": (i, [_P, _FP, _FP, _IP, _P]),
        "rt_sarsa_read": (i, [_P, _FP, _FP, _UP, _FP]),
        "rt_sarsa_nearest": (i, [_P, _P, _FP, _FP, i, _IP]),
        "rt_render_sarsa": (i, [_P, _P, _P, ctypes.POINTER(RtCamera), ctypes.POINTER(RtParams), i, _FP,
                                _U64P]),
        "rt_render_sarsa_tiles_device": (i, [_P, _P, _P, ctypes.POINTER(RtCamera), ctypes.POINTER(RtParams),
                                             _IP, i, i, _P, _P, i, _P]),
        "rt_sarsa_td_device": (i, [_P, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_int64)]),
        "rt_sarsa_apply": (i, [_P, _P]),
        "rt_ktime_enable": (i, [i]),
        "rt_ktime_read": (i, [i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
        "rt_ktime_name": (ctypes.c_char_p, [i]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name):  # an older A/B variant build; EXPORTS is checked by tests
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """The loaded librtmi.so; raises if it has not been built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C {_PKG_DIR}` "
                "(or __graft_entry__.build()); there is no fallback path")
        handle = ctypes.CDLL(LIB_PATH)
        _declare(handle)
        _LIB = handle
    return _LIB


def check(rc: int) -> None:
    if rc != RT_OK:
        raise RtError(rc, lib().rt_last_error().decode(errors="replace"))
