"""Scratch: the kept-graph regression test with the old one-pass mean restored (expected to fail)."""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from pertrenderer_amd import pose_opt
from pertrenderer_amd.renderer.transforms import Rotate, so3_exponential_map
import test_gpu_pose_opt as T

def old_forward(self):
    mesh = self.scene.meshes
    R = so3_exponential_map(self.log_rot)
    predicted = mesh.update_padded(Rotate(R).transform_points(mesh.verts_padded()))
    images = self.renderer(predicted, cameras=self.scene.cameras[0], lights=self.scene.lights)
    return ((images[..., :3] - self.target) ** 2).mean()

pose_opt._CapturedIteration._forward = old_forward
dev = torch.device("cuda:0")
try:
    T.test_kept_graphs_record_each_problems_losses(dev)
    print("OLD MEAN: test passed")
except AssertionError as e:
    print("OLD MEAN: test failed as expected:", str(e)[:300])
