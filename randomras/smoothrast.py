"""Alias of pertrenderer_amd.smoothrast (drop-in import path randomras.smoothrast)."""
import sys as _sys

import pertrenderer_amd.smoothrast as _impl

_sys.modules[__name__] = _impl
