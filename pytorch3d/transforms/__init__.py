"""pytorch3d.transforms (shim; experiments/eval.py:47-53)."""
from pertrenderer_amd.renderer.transforms import (Rotate, random_rotations, so3_exp_map,  # noqa: F401
                                                  so3_exponential_map, so3_log_map, so3_relative_angle)
