"""Import alias so code written against quentinll/pertrenderer (``import randomras``,
randomras/__init__.py:1-3) runs unchanged on pertrenderer_amd."""
from pertrenderer_amd.random_rasterizer import RandomSimpleShader, SimpleShader  # noqa: F401
from pertrenderer_amd.smoothagg import CauchyAgg, GaussianAgg, SoftAgg  # noqa: F401
from pertrenderer_amd.smoothrast import AffineRast, ArctanRast, GaussianRast, SoftRast  # noqa: F401
