"""Alias of pertrenderer_amd.smoothagg (drop-in import path randomras.smoothagg)."""
import sys as _sys

import pertrenderer_amd.smoothagg as _impl

_sys.modules[__name__] = _impl
