#!/usr/bin/env python
"""Marching-cubes case tables, generated (not transcribed) for the mesh path.

The reference extracts its mesh with PyMCubes ``mcubes.marching_cubes(cube, cfg.mesh_th)``
(``lib/networks/renderer/aninerf_mesh_renderer.py:45``). PyMCubes (a third-party C++ extension) is
not installed here, so its case table cannot be pinned; this module derives a table from one rule
and the mesh path (``csrc/anr_mesh.hip``) and the oracle (``oracle/mcubes.py``) both use it.

Conventions (Lorensen & Cline numbering): corners
    c0 (0,0,0) c1 (1,0,0) c2 (1,1,0) c3 (0,1,0) c4 (0,0,1) c5 (1,0,1) c6 (1,1,1) c7 (0,1,1)
edges e0 c0-c1, e1 c1-c2, e2 c2-c3, e3 c3-c0, e4 c4-c5, e5 c5-c6, e6 c6-c7, e7 c7-c4,
e8 c0-c4, e9 c1-c5, e10 c2-c6, e11 c3-c7. Bit m of the case index is set when corner m is
outside (value <= iso); inside = value > iso (the body, high density).
Rule: on every cube face the crossing edges are joined by segments; a face with two diagonal
inside corners (the ambiguous face) separates the inside corners. Both cubes sharing a face
derive the same segments from the same four corners, so the surface is closed across cubes.
Segments are oriented with the inside corner on their left seen from outside the cube; the
chained loops are fanned from their first point, giving triangles whose right-hand normal
points from the inside (high) region to the outside (low) region.

Run as a script to regenerate ``animatable_nerf_amd/csrc/anr_mc_table.h``.
"""
import os

import numpy as np

CORNERS = np.array([(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)], float)
EDGES = [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 7), (7, 4), (0, 4), (1, 5), (2, 6), (3, 7)]
# faces as cyclic corner lists + outward normal
FACES = [((0, 3, 2, 1), (0, 0, -1)), ((4, 5, 6, 7), (0, 0, 1)), ((0, 1, 5, 4), (0, -1, 0)),
         ((3, 7, 6, 2), (0, 1, 0)), ((0, 4, 7, 3), (-1, 0, 0)), ((1, 2, 6, 5), (1, 0, 0))]
# edge (grid-point corner, axis): the vertex of edge e belongs to the lower corner of the edge and
# runs along one axis — the owner used by the vertex numbering of the mesh kernels
EDGE_OWNER = []
for a, b in EDGES:
    lo = a if CORNERS[a].sum() < CORNERS[b].sum() else b
    axis = int(np.argmax(np.abs(CORNERS[b] - CORNERS[a])))
    EDGE_OWNER.append((tuple(int(v) for v in CORNERS[lo]), axis))


def _edge_index(a, b):
    for i, (p, q) in enumerate(EDGES):
        if (p, q) == (a, b) or (q, p) == (a, b):
            return i
    raise KeyError((a, b))


def case_triangles(case):
    inside = [not (case >> m) & 1 for m in range(8)]
    mid = {e: (CORNERS[a] + CORNERS[b]) / 2 for e, (a, b) in enumerate(EDGES)}
    succ = {}
    for cyc, nrm in FACES:
        n = np.array(nrm, float)
        ins = [inside[c] for c in cyc]
        cross = [_edge_index(cyc[k], cyc[(k + 1) % 4]) for k in range(4) if ins[k] != ins[(k + 1) % 4]]
        if not cross:
            continue
        if len(cross) == 2:
            inner = [cyc[k] for k in range(4) if ins[k]]
            segs = [(cross[0], cross[1], inner[0])]
        else:  # ambiguous face: cut off each inside corner separately
            segs = []
            for k in range(4):
                if ins[k]:
                    segs.append((_edge_index(cyc[(k - 1) % 4], cyc[k]), _edge_index(cyc[k], cyc[(k + 1) % 4]), cyc[k]))
        for p, q, ic in segs:
            P, Q, I = mid[p], mid[q], CORNERS[ic]
            if np.dot(np.cross(Q - P, I - P), n) < 0:
                p, q = q, p
            assert p not in succ, (case, p)
            succ[p] = q
    assert sorted(succ) == sorted(succ.values())
    tris = []
    todo = sorted(succ)
    seen = set()
    for start in todo:
        if start in seen:
            continue
        loop = [start]
        seen.add(start)
        e = succ[start]
        while e != start:
            loop.append(e)
            seen.add(e)
            e = succ[e]
        for a, b, c in _triangulate(loop):
            tris.append((a, c, b))  # winding flipped to the outward normal
    return tris


def _faces_of_edge(e):
    a, b = EDGES[e]
    return {f for f, (cyc, _) in enumerate(FACES) if a in cyc and b in cyc}


def _triangulations(poly):
    """all triangulations of a convex-position polygon (vertex lists), deterministic order"""
    if len(poly) < 3:
        yield []
        return
    if len(poly) == 3:
        yield [tuple(poly)]
        return
    a, b = poly[0], poly[-1]
    for k in range(1, len(poly) - 1):
        for left in _triangulations(poly[:k + 1]):
            for right in _triangulations(poly[k:]):
                yield left + [(a, poly[k], b)] + right


def _triangulate(loop):
    """Triangles of a loop whose interior diagonals never lie on a cube face: a diagonal between two
    vertices on a common face could coincide with the neighbouring cube's surface and make the
    mesh non-manifold. The first such triangulation (fans from each apex first) is used."""
    n = len(loop)
    cands = []
    for r in range(n):  # fans first
        rot = loop[r:] + loop[:r]
        cands.append([(rot[0], rot[k], rot[k + 1]) for k in range(1, n - 1)])
    cands += list(_triangulations(list(loop)))
    adj = {frozenset((loop[k], loop[(k + 1) % n])) for k in range(n)}
    for tris in cands:
        ok = True
        for t in tris:
            for u, w in ((t[0], t[1]), (t[1], t[2]), (t[2], t[0])):
                if frozenset((u, w)) not in adj and _faces_of_edge(u) & _faces_of_edge(w):
                    ok = False
        if ok:
            return tris
    raise AssertionError(f'no face-free triangulation for loop {loop}')


def mc_tables():
    """-> (count (256,) int, table (256, 3*MAXT) int with -1 padding)."""
    all_t = [case_triangles(c) for c in range(256)]
    maxt = max(len(t) for t in all_t)
    table = -np.ones((256, 3 * maxt), np.int32)
    count = np.zeros(256, np.int32)
    for c, t in enumerate(all_t):
        count[c] = len(t)
        for k, tri in enumerate(t):
            table[c, 3 * k:3 * k + 3] = tri
    return count, table


def _check_orientation():
    # single inside corner c0: the triangle's normal must point away from c0 (towards the outside)
    (t,) = case_triangles(0xFE)
    mid = [(CORNERS[a] + CORNERS[b]) / 2 for a, b in EDGES]
    nrm = np.cross(mid[t[1]] - mid[t[0]], mid[t[2]] - mid[t[0]])
    assert np.dot(nrm, mid[t[0]] - CORNERS[0]) > 0, 'outward orientation'


def write_header(path):
    _check_orientation()
    count, table = mc_tables()
    lines = ['// anr_mc_table.h — GENERATED by tools/gen_mc_table.py (rule in its docstring); do not edit.',
             '#pragma once', '', 'namespace anr {', '',
             f'#define ANR_MC_MAXT {table.shape[1] // 3}',
             '// triangles per case', '__device__ __constant__ static const unsigned char kMcCount[256] = {']
    for r in range(0, 256, 32):
        lines.append('    ' + ', '.join(str(int(v)) for v in count[r:r + 32]) + ',')
    lines.append('};')
    lines.append('// edge indices of the triangles of each case (-1 padded)')
    lines.append(f'__device__ __constant__ static const signed char kMcTris[256][{table.shape[1]}] = {{')
    for r in range(256):
        lines.append('    {' + ', '.join(str(int(v)) for v in table[r]) + '},')
    lines.append('};')
    lines.append('// owner of each edge\'s vertex: lower corner offset (x, y, z) and axis')
    own = ', '.join('{%d, %d, %d, %d}' % (o[0][0], o[0][1], o[0][2], o[1]) for o in EDGE_OWNER)
    lines.append('__device__ __constant__ static const signed char kMcEdgeOwner[12][4] = {' + own + '};')
    lines += ['', '}  // namespace anr', '']
    with open(path, 'w') as f:
        f.write('\n'.join(lines))


if __name__ == '__main__':
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    write_header(os.path.join(root, 'animatable_nerf_amd', 'csrc', 'anr_mc_table.h'))
    c, t = mc_tables()
    print('max triangles per case', t.shape[1] // 3, 'total', int(c.sum()))
