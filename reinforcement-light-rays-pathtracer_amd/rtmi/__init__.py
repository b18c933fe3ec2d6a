"""rtmi — MI355X-native Monte Carlo path tracer (Python binding).

The compute path is librtmi.so (hand-written HIP kernels for gfx950 behind
the C ABI in include/rtmi.h); this package only binds it.  Importing rtmi
does not touch the GPU.
"""
from ._lib import (LIB_PATH, RT_HIT_NONE, RT_HIT_RULE_CPU, RT_HIT_RULE_GPU, RT_HIT_TYPE_LIGHT,
                   RT_HIT_TYPE_SURFACE, RT_PRESET_CPU, RT_PRESET_GPU, RT_SAMPLER_COSINE,
                   RT_SAMPLER_UNIFORM, RT_KT_RENDER_PS, RT_KT_RENDER, RT_KT_SARSA_RENDER, RT_KT_SARSA_APPLY,
                   RT_KT_DQN_MLP, RT_KT_DQN_BOUNCE, RT_KT_DQN_CAMERA, RT_KT_COUNT, RtCamera, RtError,
                   RtParams, check, lib)
from .api import (CAMERAS, OBJ_KINDS, Context, Geometry, Scene, camera, cornell_geometry,
                  default_params, filter_records, intersect, intersect_device, intersect_method, ISECT_SCAN,
                  ISECT_FILTER, ISECT_MFMA, ISECT_BVH, ACCEL_AUTO, ACCEL_SCAN, ACCEL_BVH,
                  obj_geometry, pack_argb,
                  rect_candidates, ctab_candidates, render, render_tiles_device, save_bmp, save_png,
                  ktime_enable, ktime_read, ktime_name)
from . import dist, dqn, metrics, sarsa, tiles

__all__ = [
    "LIB_PATH", "RT_HIT_NONE", "RT_HIT_RULE_CPU", "RT_HIT_RULE_GPU", "RT_HIT_TYPE_LIGHT",
    "RT_HIT_TYPE_SURFACE", "RT_PRESET_CPU", "RT_PRESET_GPU", "RT_SAMPLER_COSINE",
    "RT_SAMPLER_UNIFORM", "RtCamera", "RtError", "RtParams", "lib", "CAMERAS", "OBJ_KINDS",
    "Context", "Geometry", "Scene", "camera", "cornell_geometry", "default_params", "filter_records", "intersect",
    "intersect_device", "obj_geometry", "pack_argb", "rect_candidates", "ctab_candidates", "render", "render_tiles_device", "save_bmp", "save_png",
    "dist", "dqn", "metrics", "sarsa", "tiles", "check", "ktime_enable", "ktime_read", "ktime_name",
    "RT_KT_RENDER_PS", "RT_KT_RENDER", "RT_KT_SARSA_RENDER", "RT_KT_SARSA_APPLY", "RT_KT_DQN_MLP",
    "RT_KT_DQN_BOUNCE", "RT_KT_DQN_CAMERA", "RT_KT_COUNT",
]
