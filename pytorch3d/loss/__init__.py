"""pytorch3d.loss (shim; experiments/eval.py:26-31)."""
from pertrenderer_amd.renderer.loss import (chamfer_distance, mesh_edge_loss,  # noqa: F401
                                            mesh_laplacian_smoothing, mesh_normal_consistency)
