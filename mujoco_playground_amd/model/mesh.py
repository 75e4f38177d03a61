"""Mesh assets for the model compiler: binary STL reader, MuJoCo-style mesh inertia,
re-centring to the inertial frame, and the convex hull used for collision.

Restates the MuJoCo compiler's mesh processing [ext: mujoco user_mesh.cc, not vendored
in /root/reference] for the two meshes the reference loads
(`models/ackermann_robot_v2.xml:8-14`, `CAD Models/Base.stl`, `CAD Models/Ceiling.stl`).

Inertia modes (MuJoCo `mesh/inertia` attribute):
  * "legacy"  -- the MuJoCo <=3.3 default: pyramids from the area-weighted face centre with
                 ABSOLUTE volumes (over-counts non-convex meshes, such as these holed plates);
  * "exact"   -- signed-volume divergence-theorem integrals (correct for watertight meshes);
  * "convex"  -- exact integrals over the convex hull.
The reference pins only `mujoco>=3.0.0` (`requirements.txt:4`), so the mode in effect is
unrecorded; we default to "legacy" and document it in DESIGN.md (parity risk).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

from .mathutil import mat_to_quat


def read_binary_stl(path: str) -> np.ndarray:
    """Return float32 triangles [ntri, 3, 3]."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 84:
        raise ValueError(f"{path}: too short for a binary STL")
    (ntri,) = struct.unpack_from("<I", data, 80)
    if 84 + 50 * ntri != len(data):
        raise ValueError(f"{path}: size does not match {ntri} binary triangles")
    rec = np.frombuffer(data, dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]),
                        count=ntri, offset=84)
    return np.array(rec["v"], dtype=np.float32)


def dedupe(tris: np.ndarray):
    """Shared-vertex representation (MuJoCo removes repeated STL vertices)."""
    flat = tris.reshape(-1, 3)
    verts, inv = np.unique(flat, axis=0, return_inverse=True)
    faces = inv.reshape(-1, 3).astype(np.int32)
    return verts.astype(np.float32), faces


def _tri_area_normal(a, b, c):
    cr = np.cross(b - a, c - a)
    n2 = np.linalg.norm(cr, axis=-1)
    area = 0.5 * n2
    with np.errstate(invalid="ignore", divide="ignore"):
        nrm = np.where(n2[:, None] > 0, cr / np.maximum(n2, 1e-300)[:, None], 0.0)
    return area, nrm


def _second_moments(D, E, F, vol):
    """Sum over tetrahedra (0, D, E, F) of vol/20*(2ΣVᵢVᵢᵀ + cross terms) -> 3x3 P."""
    P = np.zeros((3, 3))
    for j in range(3):
        for k in range(3):
            P[j, k] = np.sum(vol / 20.0 * (
                2 * (D[:, j] * D[:, k] + E[:, j] * E[:, k] + F[:, j] * F[:, k])
                + D[:, j] * E[:, k] + D[:, k] * E[:, j]
                + D[:, j] * F[:, k] + D[:, k] * F[:, j]
                + E[:, j] * F[:, k] + E[:, k] * F[:, j]))
    return P


def mesh_inertia(verts: np.ndarray, faces: np.ndarray, mode: str = "legacy"):
    """Volume, centre of mass and unit-density inertia tensor (about the CoM).

    Returns (volume, com[3], I[3,3]).
    """
    v = verts.astype(np.float64)
    if mode == "convex":
        from scipy.spatial import ConvexHull
        h = ConvexHull(v)
        faces = _oriented_hull_faces(v, h)
        mode = "exact"
    a, b, c = v[faces[:, 0]], v[faces[:, 1]], v[faces[:, 2]]
    area, nrm = _tri_area_normal(a, b, c)
    if mode == "legacy":
        facecen = np.sum(area[:, None] * (a + b + c) / 3.0, axis=0) / np.sum(area)
        vol = np.abs(np.einsum("ij,ij->i", a - facecen, nrm) * area / 3.0)
        volume = vol.sum()
        com = np.sum(vol[:, None] * (a + b + c + facecen) / 4.0, axis=0) / volume
        D, E, F = a - com, b - com, c - com
        tvol = np.abs(np.einsum("ij,ij->i", D, np.cross(E, F)) / 6.0)
    elif mode == "exact":
        vol = np.einsum("ij,ij->i", a, np.cross(b, c)) / 6.0
        volume = vol.sum()
        if volume < 0:  # inward-facing winding
            vol, volume = -vol, -volume
            b, c = c, b
        com = np.sum(vol[:, None] * (a + b + c) / 4.0, axis=0) / volume
        D, E, F = a - com, b - com, c - com
        tvol = np.einsum("ij,ij->i", D, np.cross(E, F)) / 6.0
    else:
        raise ValueError(mode)
    P = _second_moments(D, E, F, tvol)
    I = np.array([
        [P[1, 1] + P[2, 2], -P[0, 1], -P[0, 2]],
        [-P[0, 1], P[0, 0] + P[2, 2], -P[1, 2]],
        [-P[0, 2], -P[1, 2], P[0, 0] + P[1, 1]],
    ])
    return float(volume), com, I


def _oriented_hull_faces(v, hull):
    faces = hull.simplices.copy()
    cen = v[hull.vertices].mean(axis=0)
    for i, f in enumerate(faces):
        n = np.cross(v[f[1]] - v[f[0]], v[f[2]] - v[f[0]])
        if np.dot(n, v[f[0]] - cen) < 0:
            faces[i] = f[[0, 2, 1]]
    return faces


@dataclass
class CompiledMesh:
    name: str
    vert: np.ndarray        # float32 [nv,3], in the mesh inertial frame
    face: np.ndarray        # int32 [nf,3]
    hull_vert: np.ndarray   # float32 [nh,3] convex-hull vertices (inertial frame)
    hull_face: np.ndarray   # int32 [nhf,3] indices into hull_vert (outward winding)
    hull_adj: list          # hull vertex adjacency (graph), list of int lists
    volume: float
    pos: np.ndarray         # CoM in the STL frame
    quat: np.ndarray        # principal-axes rotation, STL frame <- inertial frame
    inertia: np.ndarray     # unit-density principal moments [3]
    rbound: float           # bounding-sphere radius about the inertial-frame origin


def compile_mesh(name: str, path: str, mode: str = "legacy") -> CompiledMesh:
    from scipy.spatial import ConvexHull

    tris = read_binary_stl(path)
    verts, faces = dedupe(tris)
    volume, com, I = mesh_inertia(verts, faces, mode)
    if volume <= 1e-15:
        raise ValueError(f"mesh {name}: volume too small")
    evals, evecs = np.linalg.eigh(I)
    order = np.argsort(-evals)            # MuJoCo lists principal moments largest first
    evals, evecs = evals[order], evecs[:, order]
    if np.linalg.det(evecs) < 0:
        evecs[:, 2] = -evecs[:, 2]
    quat = mat_to_quat(evecs)
    # vertices expressed in the inertial frame: R^T (v - com)
    vloc = ((verts.astype(np.float64) - com) @ evecs).astype(np.float32)
    hull = ConvexHull(vloc.astype(np.float64))
    hidx = np.array(sorted(hull.vertices), dtype=np.int32)
    remap = {int(g): i for i, g in enumerate(hidx)}
    hf = _oriented_hull_faces(vloc.astype(np.float64), hull)
    hull_face = np.array([[remap[int(x)] for x in f] for f in hf], dtype=np.int32)
    adj = [set() for _ in hidx]
    for f in hull_face:
        for i in range(3):
            a, b = int(f[i]), int(f[(i + 1) % 3])
            adj[a].add(b)
            adj[b].add(a)
    rbound = float(np.max(np.linalg.norm(vloc.astype(np.float64), axis=1)))
    return CompiledMesh(name=name, vert=vloc, face=faces, hull_vert=vloc[hidx].copy(),
                        hull_face=hull_face, hull_adj=[sorted(s) for s in adj], volume=volume,
                        pos=com, quat=quat, inertia=evals, rbound=rbound)
