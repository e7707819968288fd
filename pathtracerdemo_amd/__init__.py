"""MI355X-native path tracer: the per-pixel compute path of hdm0922/PathTracerDemo.

``Renderer`` mirrors the reference's ``Renderer`` (Renderer_TEST.ts) over libptx.so,
the HIP/gfx950 implementation behind the C ABI of ``include/ptx.h``.
"""
from .scene.world import World, compile_scene, serialize_world  # noqa: F401


def Renderer(*args, **kwargs):  # lazy: importing the package must not require a GPU
    from .renderer import Renderer as _R
    return _R(*args, **kwargs)
