"""Shape "loopsubdiv" (src/shapes/loopsubdiv.cpp:137-437) through the loader.

The reference's loopsubdiv.cpp cannot be built here on its own (it includes
pbrt.h, which needs the absent glog submodule), and the reference's tests hold
no Loop-subdivision vectors, so the refined meshes are checked against an
independent float64 restatement of Loop's rules written below (edge-face
adjacency instead of the reference's pointer half-edges; the same vertex and
face numbering) -- positions to 1e-5 of the mesh size, normal directions to
1e-4 -- plus exact properties: counts (V + E, 4F per level), planar meshes stay
exactly planar with normals exactly along the plane normal, and the CTM is
applied after subdivision.  Bit-level parity with the reference is unpinned."""
import math
import os

import numpy as np
import pytest

import ptgpu
import pyoracle

HEADER = """LookAt 0 0 -6  0 0 0  0 1 0
Camera "perspective" "float fov" [40]
PixelFilter "box" "float xwidth" [0.5] "float ywidth" [0.5]
Film "image" "integer xresolution" [24] "integer yresolution" [16]
Sampler "halton" "integer pixelsamples" [4]
Integrator "path" "integer maxdepth" [3]
WorldBegin
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [4 4 4]
  Shape "trianglemesh" "point P" [-1 3 -1  1 3 -1  0 3 1] "integer indices" [0 1 2]
AttributeEnd
"""


def _scene(tmp_path, P, idx, levels, xform="", material='Material "matte" "rgb Kd" [0.5 0.4 0.3]', extra=""):
    lv = "" if levels is None else '"integer levels" [%d]' % levels
    shape = ('Shape "loopsubdiv" %s "integer indices" [%s] "point P" [%s] %s' %
             (lv, " ".join(map(str, np.asarray(idx).reshape(-1))),
              " ".join(repr(float(x)) for x in np.asarray(P, np.float32).reshape(-1)), extra))
    txt = HEADER + f"AttributeBegin\n  {xform}\n  {material}\n  {shape}\nAttributeEnd\nWorldEnd\n"
    p = os.path.join(str(tmp_path), "loop_%s_%d.pbrt" % (levels, len(idx)))
    with open(p, "w") as f:
        f.write(txt)
    return p


def _subdiv_mesh(tmp_path, P, idx, levels, **kw):
    hs = ptgpu.HostScene(_scene(tmp_path, P, idx, levels, **kw))
    m = hs.mesh()
    tri = m["tri"][1:]                        # triangle 0 is the light
    base = tri[:, :3].min()
    return m["P"][base:], m["N"][base:], tri[:, :3] - base, hs


# ---- independent restatement (float64) ---------------------------------------------------------

def _loop_ref(P, idx, levels):
    V = [np.array(p, np.float64) for p in np.asarray(P, np.float64)]
    F = [tuple(int(i) for i in f) for f in np.asarray(idx).reshape(-1, 3)]

    def analyse(V, F):
        ef = {}
        for fi, f in enumerate(F):
            for k in range(3):
                ef.setdefault(frozenset((f[k], f[(k + 1) % 3])), []).append(fi)
        nb = [set() for _ in V]
        bnb = [[] for _ in V]
        for e, fs in ef.items():
            a, b = tuple(e)
            nb[a].add(b)
            nb[b].add(a)
            if len(fs) == 1:
                bnb[a].append(b)
                bnb[b].append(a)
        return ef, nb, bnb

    def beta(n):
        return 3.0 / 16.0 if n == 3 else 3.0 / (8.0 * n)

    for _ in range(levels):
        ef, nb, bnb = analyse(V, F)
        newV = []
        for i, v in enumerate(V):
            if bnb[i]:
                newV.append(0.75 * v + 0.125 * (V[bnb[i][0]] + V[bnb[i][1]]))
            else:
                n = len(nb[i])
                newV.append((1 - n * beta(n)) * v + beta(n) * sum(V[j] for j in nb[i]))
        eidx = {}
        for fi, f in enumerate(F):
            for k in range(3):
                a, b = f[k], f[(k + 1) % 3]
                key = frozenset((a, b))
                if key in eidx:
                    continue
                fs = ef[key]
                if len(fs) == 1:
                    p = 0.5 * (V[a] + V[b])
                else:
                    opp = [next(x for x in F[g] if x != a and x != b) for g in fs[:2]]
                    p = 0.375 * (V[a] + V[b]) + 0.125 * (V[opp[0]] + V[opp[1]])
                eidx[key] = len(V) + len(eidx)
                newV.append(p)
        newF = []
        for a, b, c in F:
            eab, ebc, eca = eidx[frozenset((a, b))], eidx[frozenset((b, c))], eidx[frozenset((c, a))]
            newF += [(a, eab, eca), (eab, b, ebc), (eca, ebc, c), (eab, ebc, eca)]
        V, F = newV, newF
    ef, nb, bnb = analyse(V, F)
    lim = []
    for i, v in enumerate(V):
        if bnb[i]:
            lim.append(0.6 * v + 0.2 * (V[bnb[i][0]] + V[bnb[i][1]]))
        else:
            n = len(nb[i])
            g = 1.0 / (n + 3.0 / (8.0 * beta(n)))
            lim.append((1 - n * g) * v + g * sum(V[j] for j in nb[i]))
    # ordered one-rings: per incident face (prev, next) in winding order
    inc = [[] for _ in V]
    for f in F:
        for k in range(3):
            inc[f[k]].append((f[(k + 2) % 3], f[(k + 1) % 3]))
    N = []
    for i, v in enumerate(lim):
        pairs = inc[i]
        if not bnb[i]:
            ring = [pairs[0][1]]
            while len(ring) < len(pairs):
                ring.append(next(nx for pv, nx in pairs if pv == ring[-1]))
            n = len(ring)
            S = sum(math.cos(2 * math.pi * j / n) * lim[r] for j, r in enumerate(ring))
            T = sum(math.sin(2 * math.pi * j / n) * lim[r] for j, r in enumerate(ring))
        else:
            prevs = {pv for pv, _ in pairs}
            fend = next((pv, nx) for pv, nx in pairs if nx not in prevs)   # its (v, next) edge is on the boundary
            ring = [fend[1], fend[0]]
            cur = fend
            while True:
                nxt = [(pv, nx) for pv, nx in pairs if nx == cur[0]]
                if not nxt:
                    break
                cur = nxt[0]
                ring.append(cur[0])
            n = len(ring)
            S = lim[ring[-1]] - lim[ring[0]]
            R = [lim[r] for r in ring]
            if n == 2:
                T = R[0] + R[1] - 2 * v
            elif n == 3:
                T = R[1] - v
            elif n == 4:
                T = -R[0] + 2 * R[1] + 2 * R[2] - R[3] - 2 * v
            else:
                th = math.pi / (n - 1)
                T = math.sin(th) * (R[0] + R[-1])
                for k in range(1, n - 1):
                    T = T + (2 * math.cos(th) - 2) * math.sin(k * th) * R[k]
                T = -T
        N.append(np.cross(S, T))
    return np.array(lim), np.array(N), np.array(F)


# ---- meshes ------------------------------------------------------------------------------------

def tetra():
    P = [[1, 1, 1], [1, -1, -1], [-1, 1, -1], [-1, -1, 1]]
    return P, [0, 1, 2, 0, 3, 1, 0, 2, 3, 1, 3, 2]


def icosa():
    t = (1 + 5 ** 0.5) / 2
    P = [[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
         [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]]
    F = [0, 11, 5, 0, 5, 1, 0, 1, 7, 0, 7, 10, 0, 10, 11, 1, 5, 9, 5, 11, 4, 11, 10, 2, 10, 7, 6, 7, 1, 8,
         3, 9, 4, 3, 4, 2, 3, 2, 6, 3, 6, 8, 3, 8, 9, 4, 9, 5, 2, 4, 11, 6, 2, 10, 8, 6, 7, 9, 8, 1]
    return P, F


def grid(n=3):
    P = [[x - n / 2, y - n / 2, 0.0] for y in range(n + 1) for x in range(n + 1)]
    F = []
    for y in range(n):
        for x in range(n):
            a = y * (n + 1) + x
            F += [a, a + 1, a + n + 2, a, a + n + 2, a + n + 1]
    return P, F


def open_box():
    P = [[-1, -1, -1], [1, -1, -1], [1, 1, -1], [-1, 1, -1], [-1, -1, 1], [1, -1, 1], [1, 1, 1], [-1, 1, 1]]
    F = [0, 2, 1, 0, 3, 2, 0, 1, 5, 0, 5, 4, 3, 7, 6, 3, 6, 2, 0, 4, 7, 0, 7, 3, 1, 2, 6, 1, 6, 5]
    return P, F


def fan(k=6):
    # boundary vertex 0 of valence k+1 (the general boundary tangent rule)
    P = [[0, 0, 0.2]] + [[math.cos(math.pi * i / k), math.sin(math.pi * i / k), 0.1 * (i % 2)] for i in range(k + 1)]
    F = []
    for i in range(k):
        F += [0, i + 1, i + 2]
    return P, F


MESHES = {"tetra": tetra, "icosa": icosa, "grid": grid, "open_box": open_box, "fan": fan}


@pytest.mark.parametrize("name", sorted(MESHES))
@pytest.mark.parametrize("levels", [0, 1, 2])
def test_loopsubdiv_matches_restatement(tmp_path, name, levels):
    P, idx = MESHES[name]()
    gp, gn, gt, _ = _subdiv_mesh(tmp_path, P, idx, levels)
    rp, rn, rt = _loop_ref(np.asarray(P, np.float32), idx, levels)
    assert np.array_equal(gt, rt)
    size = float(np.abs(rp).max())
    np.testing.assert_allclose(gp, rp, atol=1e-5 * size, rtol=0)
    gnn = gn / np.linalg.norm(gn, axis=1, keepdims=True)
    rnn = rn / np.linalg.norm(rn, axis=1, keepdims=True)
    np.testing.assert_allclose(gnn, rnn, atol=1e-4, rtol=0)


@pytest.mark.parametrize("name", ["tetra", "icosa", "open_box"])
def test_loopsubdiv_counts(tmp_path, name):
    P, idx = MESHES[name]()
    nv, nf = len(P), len(idx) // 3
    ne = len({frozenset((idx[3 * f + k], idx[3 * f + (k + 1) % 3])) for f in range(nf) for k in range(3)})
    for levels in (1, 2, 3):
        gp, gn, gt, _ = _subdiv_mesh(tmp_path, P, idx, levels)
        assert len(gt) == 4 * nf
        assert len(gp) == nv + ne           # V' = V + E, E' = 2E + 3F
        nv, ne = nv + ne, 2 * ne + 3 * nf
        nf = 4 * nf


def test_loopsubdiv_planar_stays_planar(tmp_path):
    P, idx = grid(4)
    gp, gn, gt, _ = _subdiv_mesh(tmp_path, P, idx, 3)
    assert np.all(gp[:, 2] == 0)
    assert np.all(gn[:, :2] == 0) and np.all(gn[:, 2] != 0)


def test_loopsubdiv_default_levels_and_transform(tmp_path):
    """levels defaults to "nlevels", then 3 (loopsubdiv.cpp:404-405); the CTM
    maps the refined object-space mesh (TriangleMesh ctor, triangle.cpp:75)."""
    P, idx = icosa()
    a, an, at, _ = _subdiv_mesh(tmp_path, P, idx, 3)
    assert len(at) == 20 * 64
    (tmp_path / "b").mkdir()
    b, _, bt, _ = _subdiv_mesh(tmp_path / "b", P, idx, None)
    assert np.array_equal(b, a) and np.array_equal(bt, at)
    (tmp_path / "n").mkdir()
    n, _, nt, _ = _subdiv_mesh(tmp_path / "n", P, idx, None, extra='"integer nlevels" [1]')
    assert len(nt) == 20 * 4
    (tmp_path / "c").mkdir()
    c, cn, ct, _ = _subdiv_mesh(tmp_path / "c", P, idx, 3, xform="Translate 1 2 3")
    np.testing.assert_allclose(c, a + np.array([1, 2, 3], np.float32), atol=1e-5)
    assert np.array_equal(cn, an)


def test_loopsubdiv_missing_data_is_an_error_not_fatal(tmp_path, capfd):
    txt = HEADER + 'Shape "loopsubdiv" "point P" [0 0 0 1 0 0 0 1 0]\nWorldEnd\n'
    p = tmp_path / "bad.pbrt"
    p.write_text(txt)
    hs = ptgpu.HostScene(str(p))
    assert len(hs.mesh()["tri"]) == 1         # the light only: no shapes made
    assert "indices" in capfd.readouterr().err


def test_loopsubdiv_renders(tmp_path):
    """The refined mesh (limit positions, shading normals) through the oracle
    renderer: finite, lit."""
    P, idx = icosa()
    hs = ptgpu.HostScene(_scene(tmp_path, P, idx, 2, material='Material "plastic" "rgb Kd" [0.4 0.2 0.2]'))
    img, st = pyoracle.render(hs.desc, nthreads=4)
    assert np.isfinite(img).all() and img.mean() > 0


def test_killeroo_simple_shape_count():
    """BASELINE config 1 scene (reference scenes/killeroo-simple.pbrt): two
    `loopsubdiv nlevels 1` killeroos + 4 quad triangles + 1 sphere.  The
    reference's own run counted 66,533 shapes (SURVEY.md §8(d) C5 [probe]),
    which pins the subdivided topology: 2 x 33,264 triangles."""
    from conftest import REPO
    hs = ptgpu.HostScene(os.path.join(REPO, "scenes", "killeroo-simple.pbrt"))
    d = ptgpu._desc_prefix.from_address(hs.desc)
    assert d.n_prims == 66533 and d.n_triangles == 66532
    it = ptgpu.integrator_desc(hs)
    assert it.kind == 0 and it.rr_threshold == float("-inf")  # "mypath": PathIntegrator without RR
