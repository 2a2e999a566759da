"""Synthetic meshes for the rasterizer tests: the reference's sphere_642 (tests/golden, a copy of
the reference's data file) subdivided k times (each face into 4, new vertices pushed to the unit
sphere), so that 3 levels give 81 920 faces -- the scanned-mesh scale at which the coarse bins
matter."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_sphere():
    v, f = [], []
    with open(os.path.join(ROOT, "tests", "golden", "sphere_642.obj")) as fh:
        for line in fh:
            t = line.split()
            if t and t[0] == "v":
                v.append([float(x) for x in t[1:4]])
            elif t and t[0] == "f":
                f.append([int(x.split("/")[0]) - 1 for x in t[1:4]])
    return np.asarray(v, np.float32), np.asarray(f, np.int64)


def subdivide(verts, faces, levels):
    verts = [tuple(x) for x in verts.tolist()]
    for _ in range(levels):
        mid, out = {}, []

        def midpoint(a, b):
            key = (min(a, b), max(a, b))
            if key not in mid:
                p = (np.asarray(verts[a]) + np.asarray(verts[b])) / 2.0
                verts.append(tuple((p / np.linalg.norm(p)).tolist()))
                mid[key] = len(verts) - 1
            return mid[key]

        for a, b, c in faces.tolist():
            ab, bc, ca = midpoint(a, b), midpoint(b, c), midpoint(c, a)
            out += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        faces = np.asarray(out, np.int64)
    return np.asarray(verts, np.float32), faces


def fine_sphere(levels=3):
    return subdivide(*load_sphere(), levels)
