"""Hand-computed known-answer cases for the K-nearest-face rasterizer (PyTorch3D 0.4.0
rasterize_meshes semantics) — shared by tests/test_rast_oracle.py (the C
oracle) and tests/test_gpu_rast_kat.py (the HIP kernel).

Every expected number below was worked out by hand (derivations in the comments), not
produced by either implementation.

Pixel centres (PyTorch3D NDC, +X left, +Y up, pixel (0, 0) top-left):
  H = W = 4:  col -> x = 0.75, 0.25, -0.25, -0.75 ;  row -> y = 0.75, 0.25, -0.25, -0.75.
Triangle A = v0 (0,0), v1 (1,0), v2 (0,1): for a point (x, y) its barycentrics are
  w = (1 - x - y, x, y); signed area edge(v0, v1, v2) = -1 (a back face under cull_backfaces).
"""
import numpy as np

A_XY = [(0.0, 0.0), (1.0, 0.0), (0.0, 1.0)]


def tri(xy, z):
    return [[x, y, zz] for (x, y), zz in zip(xy, z)]


def _case(name, faces, H=4, W=4, K=1, blur=0.0, persp=False, clip=False, cull=False, first=None, nfaces=None,
          p2f=None, values=None):
    fv = np.asarray(faces, np.float64)
    if first is None:
        first, nfaces = [0], [fv.shape[0]]
    N = len(first)
    full = -np.ones((N, H, W, K), np.int64)
    for (n, r, c), ids in (p2f or {}).items():
        full[n, r, c, :len(ids)] = ids
    return dict(name=name, fv=fv, first=np.asarray(first, np.int64), nfaces=np.asarray(nfaces, np.int64), H=H,
                W=W, K=K, blur=blur, persp=persp, clip=clip, cull=cull, p2f=full, values=values or {})


# slot values: (n, row, col, k) -> (zbuf, (bary0, bary1, bary2), signed squared distance)
BLUR_KEPT_P2F = {(0, 0, 1): [0], (0, 0, 2): [0], (0, 1, 0): [0], (0, 1, 1): [0], (0, 1, 2): [0],
                 (0, 2, 0): [0], (0, 2, 1): [0]}

CASES = [
    # blur 0.0626: sqrt(blur) = 0.2502 widens A's box [0,1]^2 to include x = -0.25 / y = -0.25.
    #  (0,1) (0.25,0.75) on edge v1v2: w = (0,.25,.75), outside (w0 not > 0), d = 0  -> kept, dist +0
    #  (0,2) (-0.25,0.75): w = (.5,-.25,.75), z = .5 - .5 + 2.25 = 2.25, nearest edge x=0: d = .0625
    #  (1,0) (0.75,0.25) on edge v1v2: w = (0,.75,.25), z = 1.5 + .75 = 2.25, d = 0
    #  (1,1) (0.25,0.25) inside: w = (.5,.25,.25), z = .5 + .5 + .75 = 1.75, dist = -.0625
    #  (1,2) (-0.25,0.25): w = (1,-.25,.25), z = 1 - .5 + .75 = 1.25, d = .0625
    #  (2,0) (0.75,-0.25): w = (.5,.75,-.25), z = .5 + 1.5 - .75 = 1.25, d = .0625 (edge y=0)
    #  (2,1) (0.25,-0.25): w = (1,.25,-.25), z = 1 + .5 - .75 = .75, d = .0625
    #  (0,0) (0.75,0.75): nearest point (.5,.5): d = .125 >= blur -> culled; (2,2): d to v0 = .125 -> culled
    #  column 3 / row 3 (|coord| .75 beyond the widened box) -> culled by the box
    _case("blur_kept", [tri(A_XY, (1, 2, 3))], blur=0.0626, p2f=BLUR_KEPT_P2F, values={
        (0, 0, 1, 0): (2.75, (0.0, 0.25, 0.75), 0.0),
        (0, 0, 2, 0): (2.25, (0.5, -0.25, 0.75), 0.0625),
        (0, 1, 0, 0): (2.25, (0.0, 0.75, 0.25), 0.0),
        (0, 1, 1, 0): (1.75, (0.5, 0.25, 0.25), -0.0625),
        (0, 1, 2, 0): (1.25, (1.0, -0.25, 0.25), 0.0625),
        (0, 2, 0, 0): (1.25, (0.5, 0.75, -0.25), 0.0625),
        (0, 2, 1, 0): (0.75, (1.0, 0.25, -0.25), 0.0625)}),
    # blur 0.0624: sqrt = 0.2498 < 0.25, so the box drops x = -0.25 and y = -0.25 although
    # d = .0625 would pass a box grown by blur itself; only the d = 0 edge pixels and (1,1) remain
    _case("blur_box_is_sqrt", [tri(A_XY, (1, 2, 3))], blur=0.0624,
          p2f={(0, 0, 1): [0], (0, 1, 0): [0], (0, 1, 1): [0]}),
    # blur 0: the test is `!inside && d >= blur` -> on-edge pixels (d = 0) are dropped
    _case("hard_edges_excluded", [tri(A_XY, (1, 2, 3))], blur=0.0, p2f={(0, 1, 1): [0]},
          values={(0, 1, 1, 0): (1.75, (0.5, 0.25, 0.25), -0.0625)}),
    # clip_barycentric_coords: negative weights -> 0, renormalised; pz from the clipped weights,
    # `inside` and the distance from the unclipped ones
    #  (0,2): (.5,0,.75)/1.25 = (.4,0,.6), z = .4 + 1.8 = 2.2
    #  (1,2): (1,0,.25)/1.25 = (.8,0,.2), z = .8 + .6 = 1.4
    #  (2,0): (.5,.75,0)/1.25 = (.4,.6,0), z = .4 + 1.2 = 1.6
    #  (2,1): (1,.25,0)/1.25 = (.8,.2,0), z = .8 + .4 = 1.2
    _case("clip", [tri(A_XY, (1, 2, 3))], blur=0.0626, clip=True, p2f=BLUR_KEPT_P2F, values={
        (0, 0, 2, 0): (2.2, (0.4, 0.0, 0.6), 0.0625),
        (0, 1, 1, 0): (1.75, (0.5, 0.25, 0.25), -0.0625),
        (0, 1, 2, 0): (1.4, (0.8, 0.0, 0.2), 0.0625),
        (0, 2, 0, 0): (1.6, (0.4, 0.6, 0.0), 0.0625),
        (0, 2, 1, 0): (1.2, (0.8, 0.2, 0.0), 0.0625)}),
    # perspective_correct: b_i ~ w_i * prod_{j != i} z_j.  (1,1): (.5*2*3, 1*.25*3, 1*2*.25) = (3,.75,.5),
    # sum 4.25 -> (12/17, 3/17, 2/17), z = 24/17 (= 1 / sum(w_i / z_i))
    _case("perspective", [tri(A_XY, (1, 2, 3))], blur=0.0, persp=True, p2f={(0, 1, 1): [0]},
          values={(0, 1, 1, 0): (24 / 17, (12 / 17, 3 / 17, 2 / 17), -0.0625)}),
    # perspective then clip: (1,2) w = (1,-.25,.25) -> (6,-.75,.5)/5.75 = (24,-3,2)/23 -> clip (12/13,0,1/13),
    # z = 15/13; (0,2) w = (.5,-.25,.75) -> (3,-.75,1.5)/3.75 = (.8,-.2,.4) -> clip (2/3,0,1/3), z = 5/3
    _case("perspective_clip", [tri(A_XY, (1, 2, 3))], blur=0.0626, persp=True, clip=True, p2f=BLUR_KEPT_P2F,
          values={(0, 1, 2, 0): (15 / 13, (12 / 13, 0.0, 1 / 13), 0.0625),
                  (0, 0, 2, 0): (5 / 3, (2 / 3, 0.0, 1 / 3), 0.0625),
                  (0, 1, 1, 0): (24 / 17, (12 / 17, 3 / 17, 2 / 17), -0.0625)}),
    # zmax < 0: the face is behind the camera and skipped everywhere, although at (1,2)
    # pz = 1*(-1) + (-.25)*(-5) + .25*(-.5) = .125 >= 0 would pass the pz test
    _case("cull_zmax", [tri(A_XY, (-1, -5, -0.5))], blur=0.0626),
    # pz < 0 per pixel (zmax = 1 >= 0): only (1,0) w = (0,.75,.25) has pz = .75 - .25 = .5 >= 0
    _case("cull_pz", [tri(A_XY, (-3, 1, -1))], blur=0.0626, p2f={(0, 1, 0): [0]},
          values={(0, 1, 0, 0): (0.5, (0.0, 0.75, 0.25), 0.0)}),
    # |area| <= 1e-8: a collinear face is skipped even with a huge blur; the next face renders
    _case("degenerate_area", [tri([(0, 0), (1, 1), (0.5, 0.5)], (1, 1, 1)), tri(A_XY, (1, 2, 3))], K=2,
          blur=0.0, p2f={(0, 1, 1): [1]}),
    # A (area -1) and A with reversed winding (area +1) on the same plane: equal pz 1.75 ->
    # ascending face index breaks the tie; cull_backfaces removes face 0 (area < 0)
    _case("tie_order", [tri(A_XY, (1, 2, 3)), tri([A_XY[0], A_XY[2], A_XY[1]], (1, 3, 2))], K=2, blur=0.0,
          p2f={(0, 1, 1): [0, 1]}, values={(0, 1, 1, 1): (1.75, (0.5, 0.25, 0.25), -0.0625)}),
    _case("cull_backfaces", [tri(A_XY, (1, 2, 3)), tri([A_XY[0], A_XY[2], A_XY[1]], (1, 3, 2))], K=2, blur=0.0,
          cull=True, p2f={(0, 1, 1): [1]}),
    # K truncation: four coplanar copies at z = 2 and one at z = 1; K = 3 keeps z = 1 then the
    # lowest two indices of the tie
    _case("k_truncation", [tri(A_XY, (2, 2, 2))] * 4 + [tri(A_XY, (1, 1, 1))], K=3, blur=0.0,
          p2f={(0, 1, 1): [4, 0, 1]}, values={(0, 1, 1, 0): (1.0, (0.5, 0.25, 0.25), -0.0625),
                                               (0, 1, 1, 2): (2.0, (0.5, 0.25, 0.25), -0.0625)}),
    # two meshes in one packed batch: face ids are global, each image sees only its own faces
    _case("two_meshes", [tri(A_XY, (2, 2, 2))] * 4 + [tri(A_XY, (1, 1, 1))], K=2, blur=0.0,
          first=[0, 3], nfaces=[3, 2], p2f={(0, 1, 1): [0, 1], (1, 1, 1): [4, 3]}),
    # non-square W > H: x spans the widened range W/H * 2 -> x = -1.5, -.5, .5, 1.5 (col 3..0),
    # y = .5, -.5 (row 0, 1).  Small triangles around (1.5, .5), (-1.5, -.5), (.5, -.5)
    _case("nonsquare_wide",
          [tri([(1.4, 0.4), (1.6, 0.4), (1.5, 0.6)], (2, 2, 2)),
           tri([(-1.6, -0.6), (-1.4, -0.6), (-1.5, -0.4)], (2, 2, 2)),
           tri([(0.4, -0.6), (0.6, -0.6), (0.5, -0.4)], (2, 2, 2))],
          H=2, W=4, p2f={(0, 0, 0): [0], (0, 1, 3): [1], (0, 1, 1): [2]}),
    # non-square H > W: y spans +-2 -> y = 1.5, .5, -.5, -1.5 (row 0..3), x = .5, -.5 (col 0, 1)
    _case("nonsquare_tall",
          [tri([(0.4, 1.4), (0.6, 1.4), (0.5, 1.6)], (2, 2, 2)),
           tri([(-0.6, -1.6), (-0.4, -1.6), (-0.5, -1.4)], (2, 2, 2))],
          H=4, W=2, p2f={(0, 0, 0): [0], (0, 3, 1): [1]}),
]


def check(case, p2f, zbuf, bary, dists, tol=2e-6):
    """Compare rasterizer outputs (numpy) with a case's hand-computed expectation."""
    name = case["name"]
    np.testing.assert_array_equal(p2f, case["p2f"], err_msg=f"{name}: pix_to_face")
    pad = case["p2f"] < 0
    assert np.all(zbuf[pad] == -1) and np.all(dists[pad] == -1) and np.all(bary[pad] == -1), f"{name}: padding"
    for (n, r, c, k), (z, b, d) in case["values"].items():
        np.testing.assert_allclose(zbuf[n, r, c, k], z, rtol=0, atol=tol, err_msg=f"{name}: zbuf at {(n, r, c, k)}")
        np.testing.assert_allclose(bary[n, r, c, k], b, rtol=0, atol=tol, err_msg=f"{name}: bary at {(n, r, c, k)}")
        np.testing.assert_allclose(dists[n, r, c, k], d, rtol=0, atol=tol, err_msg=f"{name}: dists at {(n, r, c, k)}")
        if d < 0:
            assert dists[n, r, c, k] < 0, f"{name}: inside pixel must have a negative distance"


def soup(F, seed, spread=0.9, size=0.5, zmin=1.0, zmax=5.0):
    """Random overlapping faces for the finite-difference checks of the backward."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-spread, spread, (F, 1, 2))
    xy = c + rng.uniform(-size, size, (F, 3, 2))
    z = rng.uniform(zmin, zmax, (F, 3, 1))
    return np.concatenate([xy, z], -1)


def persp_denominator(fv, p2f, H, W):
    """sum_i w_i * prod_{j != i} z_j of each slot (square images: NDC centre -1 + (2i+1)/S)."""
    x = -1 + (2 * (W - 1 - np.arange(W)) + 1) / W
    y = -1 + (2 * (H - 1 - np.arange(H)) + 1) / H
    px = np.broadcast_to(x[None, None, :, None], p2f.shape)
    py = np.broadcast_to(y[None, :, None, None], p2f.shape)
    v = fv[np.where(p2f >= 0, p2f, 0)]  # (...,3,3)
    (x0, y0, z0), (x1, y1, z1), (x2, y2, z2) = [np.moveaxis(v[..., i, :], -1, 0) for i in range(3)]
    area = (x2 - x0) * (y1 - y0) - (y2 - y0) * (x1 - x0)
    w0 = ((px - x1) * (y2 - y1) - (py - y1) * (x2 - x1)) / area
    w1 = ((px - x2) * (y0 - y2) - (py - y2) * (x0 - x2)) / area
    w2 = ((px - x0) * (y1 - y0) - (py - y0) * (x1 - x0)) / area
    return w0 * z1 * z2 + w1 * z0 * z2 + w2 * z0 * z1
