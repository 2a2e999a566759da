"""Alias of pertrenderer_amd.random_rasterizer (drop-in import path randomras.random_rasterizer)."""
import sys as _sys

import pertrenderer_amd.random_rasterizer as _impl

_sys.modules[__name__] = _impl
