// loopsubdiv.cpp -- Shape "loopsubdiv" (host side of the boundary).
//
// Behaviour of LoopSubdivide / CreateLoopSubdiv (src/shapes/loopsubdiv.cpp:
// 137-437): a manifold-with-boundary triangle mesh is refined `levels` times
// (even vertices by the one-ring / boundary rules, odd vertices from their
// edge's two or four neighbours), pushed to the limit surface, and given the
// limit-surface tangent cross product as a per-vertex shading normal.  The
// result is an ordinary triangle mesh (P in object space, N, indices) that the
// loader hands to the trianglemesh path.
//
// The half-edge graph is index-based here (the reference links heap records by
// pointer), but every quantity is formed in the reference's order: the vertex
// numbering of each level (children of the old vertices, then edge vertices in
// first-encounter face order), each vertex's start face (which fixes where its
// one-ring begins, and so the float summation order), and the float
// expressions themselves.
#include <cmath>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "host_common.h"

namespace pt {

namespace {

constexpr float kPiF = 3.14159265358979323846f;

inline int next3(int i) { return (i + 1) % 3; }
inline int prev3(int i) { return (i + 2) % 3; }

struct P3 {
    float x, y, z;
};
inline P3 operator+(P3 a, P3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline P3 operator-(P3 a, P3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline P3 operator*(float s, P3 a) { return {a.x * s, a.y * s, a.z * s}; }
inline P3& operator+=(P3& a, P3 b) { a = a + b; return a; }

struct SdVert {
    P3 p{0, 0, 0};
    int startFace = -1;
    int child = -1;
    bool regular = false, boundary = false;
};

struct SdFace {
    int v[3] = {-1, -1, -1};
    int f[3] = {-1, -1, -1};
    int children[4] = {-1, -1, -1, -1};
};

struct Mesh {
    std::vector<SdVert> V;
    std::vector<SdFace> F;

    int vnum(int face, int vert) const {
        const SdFace& f = F[face];
        for (int i = 0; i < 3; ++i)
            if (f.v[i] == vert) return i;
        throw PtError(PT_ERR_PARSE, "loopsubdiv: inconsistent mesh (vertex not on its face)");
    }
    int nextFace(int face, int vert) const { return F[face].f[vnum(face, vert)]; }
    int prevFace(int face, int vert) const { return F[face].f[prev3(vnum(face, vert))]; }
    int nextVert(int face, int vert) const { return F[face].v[next3(vnum(face, vert))]; }
    int prevVert(int face, int vert) const { return F[face].v[prev3(vnum(face, vert))]; }
    int otherVert(int face, int v0, int v1) const {
        const SdFace& f = F[face];
        for (int i = 0; i < 3; ++i)
            if (f.v[i] != v0 && f.v[i] != v1) return f.v[i];
        throw PtError(PT_ERR_PARSE, "loopsubdiv: degenerate face");
    }

    // SDVertex::valence (loopsubdiv.cpp:104-121)
    int valence(int vi) const {
        const SdVert& v = V[vi];
        int f = v.startFace;
        int nf = 1;
        if (!v.boundary) {
            while ((f = nextFace(f, vi)) != v.startFace) {
                if (f < 0) throw PtError(PT_ERR_PARSE, "loopsubdiv: non-manifold vertex");
                ++nf;
            }
            return nf;
        }
        while ((f = nextFace(f, vi)) != -1) ++nf;
        f = v.startFace;
        while ((f = prevFace(f, vi)) != -1) ++nf;
        return nf + 1;
    }
    // SDVertex::oneRing (loopsubdiv.cpp:413-429)
    void oneRing(int vi, std::vector<P3>* ring) const {
        ring->clear();
        const SdVert& v = V[vi];
        if (!v.boundary) {
            int face = v.startFace;
            do {
                ring->push_back(V[nextVert(face, vi)].p);
                face = nextFace(face, vi);
            } while (face != v.startFace);
        } else {
            int face = v.startFace, f2;
            while ((f2 = nextFace(face, vi)) != -1) face = f2;
            ring->push_back(V[nextVert(face, vi)].p);
            do {
                ring->push_back(V[prevVert(face, vi)].p);
                face = prevFace(face, vi);
            } while (face != -1);
        }
    }
};

inline float loop_beta(int valence) { return valence == 3 ? 3.f / 16.f : 3.f / (8.f * valence); }  // :123-128
inline float loop_gamma(int valence) { return 1.f / (valence + 3.f / (8.f * loop_beta(valence))); }  // :130-132

// weightOneRing / weightBoundary (loopsubdiv.cpp:403-411, 431-441)
P3 weight_one_ring(const Mesh& m, int vi, float beta, std::vector<P3>& ring) {
    const int valence = m.valence(vi);
    m.oneRing(vi, &ring);
    P3 p = (1 - valence * beta) * m.V[vi].p;
    for (int i = 0; i < valence; ++i) p += beta * ring[i];
    return p;
}
P3 weight_boundary(const Mesh& m, int vi, float beta, std::vector<P3>& ring) {
    const int valence = m.valence(vi);
    m.oneRing(vi, &ring);
    P3 p = (1 - 2 * beta) * m.V[vi].p;
    p += beta * ring[0];
    p += beta * ring[valence - 1];
    return p;
}

inline uint64_t edge_key(int a, int b) {
    const uint32_t lo = (uint32_t)(a < b ? a : b), hi = (uint32_t)(a < b ? b : a);
    return (uint64_t)lo << 32 | hi;
}

}  // namespace

void loop_subdivide(int levels, const std::vector<int>& indices, const std::vector<float>& P,
                    std::vector<float>* outP, std::vector<float>* outN, std::vector<int>* outIdx) {
    const int nVertices = (int)P.size() / 3;
    if (indices.size() % 3 != 0) throw PtError(PT_ERR_PARSE, "loopsubdiv: indices not a multiple of 3");
    const int nFaces = (int)indices.size() / 3;
    Mesh m;
    m.V.resize(nVertices);
    for (int i = 0; i < nVertices; ++i) m.V[i].p = P3{P[3 * i], P[3 * i + 1], P[3 * i + 2]};
    m.F.resize(nFaces);
    for (int i = 0; i < nFaces; ++i)
        for (int j = 0; j < 3; ++j) {
            const int v = indices[3 * i + j];
            if (v < 0 || v >= nVertices) throw PtError(PT_ERR_PARSE, "loopsubdiv: vertex index out of range");
            m.F[i].v[j] = v;
            m.V[v].startFace = i;  // the last face listing the vertex (loopsubdiv.cpp:160-167)
        }
    for (int i = 0; i < nVertices; ++i)
        if (m.V[i].startFace < 0) throw PtError(PT_ERR_PARSE, "loopsubdiv: vertex not referenced by any face");
    // adjacency (loopsubdiv.cpp:169-190): the first face of an edge waits in the
    // set; the second links to it and removes it (a third would start over)
    {
        struct Pending { int face, edgeNum; };
        std::unordered_map<uint64_t, Pending> open;
        open.reserve((size_t)nFaces * 2);
        for (int i = 0; i < nFaces; ++i)
            for (int e = 0; e < 3; ++e) {
                const uint64_t k = edge_key(m.F[i].v[e], m.F[i].v[next3(e)]);
                auto it = open.find(k);
                if (it == open.end()) {
                    open.emplace(k, Pending{i, e});
                } else {
                    m.F[it->second.face].f[it->second.edgeNum] = i;
                    m.F[i].f[e] = it->second.face;
                    open.erase(it);
                }
            }
    }
    // boundary / regular flags (loopsubdiv.cpp:192-206)
    for (int i = 0; i < nVertices; ++i) {
        SdVert& v = m.V[i];
        int f = v.startFace;
        do {
            f = m.nextFace(f, i);
        } while (f != -1 && f != v.startFace);
        v.boundary = f == -1;
        const int val = m.valence(i);
        v.regular = (!v.boundary && val == 6) || (v.boundary && val == 4);
    }

    std::vector<int> f(nFaces), v(nVertices);
    for (int i = 0; i < nFaces; ++i) f[i] = i;
    for (int i = 0; i < nVertices; ++i) v[i] = i;
    std::vector<P3> ring;
    for (int level = 0; level < levels; ++level) {
        std::vector<int> newFaces, newVertices;
        newFaces.reserve(4 * f.size());
        newVertices.reserve(v.size() + 3 * f.size() / 2 + 16);
        // children of the old vertices and faces (loopsubdiv.cpp:219-233)
        for (int vi : v) {
            const int c = (int)m.V.size();
            SdVert cv;
            cv.regular = m.V[vi].regular;
            cv.boundary = m.V[vi].boundary;
            m.V.push_back(cv);
            m.V[vi].child = c;
            newVertices.push_back(c);
        }
        for (int fi : f)
            for (int k = 0; k < 4; ++k) {
                const int c = (int)m.F.size();
                m.F.push_back(SdFace());
                m.F[fi].children[k] = c;
                newFaces.push_back(c);
            }
        // even vertices (loopsubdiv.cpp:237-251)
        for (int vi : v) {
            const SdVert& sv = m.V[vi];
            P3 p;
            if (!sv.boundary) p = weight_one_ring(m, vi, sv.regular ? 1.f / 16.f : loop_beta(m.valence(vi)), ring);
            else p = weight_boundary(m, vi, 1.f / 8.f, ring);
            m.V[sv.child].p = p;
        }
        // odd (edge) vertices (loopsubdiv.cpp:253-285)
        std::unordered_map<uint64_t, int> edgeVerts;
        edgeVerts.reserve(f.size() * 2);
        for (int fi : f)
            for (int k = 0; k < 3; ++k) {
                const int a = m.F[fi].v[k], b = m.F[fi].v[next3(k)];
                const uint64_t key = edge_key(a, b);
                if (edgeVerts.count(key)) continue;
                const int nvi = (int)m.V.size();
                SdVert ev;
                ev.regular = true;
                ev.boundary = m.F[fi].f[k] == -1;
                ev.startFace = m.F[fi].children[3];
                // edge.v[0] / v[1] are the pointer-ordered endpoints; both sums
                // below are two-term and therefore order-independent
                const P3 pa = m.V[a].p, pb = m.V[b].p;
                if (ev.boundary) {
                    ev.p = 0.5f * pa;
                    ev.p += 0.5f * pb;
                } else {
                    ev.p = 3.f / 8.f * pa;
                    ev.p += 3.f / 8.f * pb;
                    ev.p += 1.f / 8.f * m.V[m.otherVert(fi, a, b)].p;
                    ev.p += 1.f / 8.f * m.V[m.otherVert(m.F[fi].f[k], a, b)].p;
                }
                m.V.push_back(ev);
                newVertices.push_back(nvi);
                edgeVerts.emplace(key, nvi);
            }
        // start faces of the even vertices (loopsubdiv.cpp:290-294)
        for (int vi : v) {
            const int vn = m.vnum(m.V[vi].startFace, vi);
            m.V[m.V[vi].child].startFace = m.F[m.V[vi].startFace].children[vn];
        }
        // child face neighbours (loopsubdiv.cpp:296-311)
        for (int fi : f) {
            for (int j = 0; j < 3; ++j) {
                const SdFace& face = m.F[fi];
                m.F[face.children[3]].f[j] = face.children[next3(j)];
                m.F[face.children[j]].f[next3(j)] = face.children[3];
                int f2 = face.f[j];
                m.F[face.children[j]].f[j] = f2 >= 0 ? m.F[f2].children[m.vnum(f2, face.v[j])] : -1;
                f2 = face.f[prev3(j)];
                m.F[face.children[j]].f[prev3(j)] = f2 >= 0 ? m.F[f2].children[m.vnum(f2, face.v[j])] : -1;
            }
        }
        // child face vertices (loopsubdiv.cpp:313-326)
        for (int fi : f) {
            for (int j = 0; j < 3; ++j) {
                const SdFace& face = m.F[fi];
                m.F[face.children[j]].v[j] = m.V[face.v[j]].child;
                const int ev = edgeVerts.at(edge_key(face.v[j], face.v[next3(j)]));
                m.F[face.children[j]].v[next3(j)] = ev;
                m.F[face.children[next3(j)]].v[j] = ev;
                m.F[face.children[3]].v[j] = ev;
            }
        }
        f.swap(newFaces);
        v.swap(newVertices);
    }

    // limit positions (loopsubdiv.cpp:331-341)
    std::vector<P3> pLimit(v.size());
    for (size_t i = 0; i < v.size(); ++i)
        pLimit[i] = m.V[v[i]].boundary ? weight_boundary(m, v[i], 1.f / 5.f, ring)
                                       : weight_one_ring(m, v[i], loop_gamma(m.valence(v[i])), ring);
    for (size_t i = 0; i < v.size(); ++i) m.V[v[i]].p = pLimit[i];

    // limit-surface tangents -> shading normals (loopsubdiv.cpp:343-380)
    outN->clear();
    outN->reserve(3 * v.size());
    for (int vi : v) {
        P3 S{0, 0, 0}, T{0, 0, 0};
        const int valence = m.valence(vi);
        m.oneRing(vi, &ring);
        const P3 vp = m.V[vi].p;
        if (!m.V[vi].boundary) {
            for (int j = 0; j < valence; ++j) {
                S += std::cos(2 * kPiF * j / valence) * ring[j];
                T += std::sin(2 * kPiF * j / valence) * ring[j];
            }
        } else {
            S = ring[valence - 1] - ring[0];
            if (valence == 2) T = (ring[0] + ring[1]) - 2 * vp;
            else if (valence == 3) T = ring[1] - vp;
            else if (valence == 4)
                T = -1 * ring[0] + 2 * ring[1] + 2 * ring[2] + -1 * ring[3] + -2 * vp;
            else {
                const float theta = kPiF / float(valence - 1);
                T = std::sin(theta) * (ring[0] + ring[valence - 1]);
                for (int k = 1; k < valence - 1; ++k) {
                    const float wt = (2 * std::cos(theta) - 2) * std::sin((k) * theta);
                    T += wt * ring[k];
                }
                T = P3{-T.x, -T.y, -T.z};
            }
        }
        // Cross (geometry.h) in double, rounded to float
        const double sx = S.x, sy = S.y, sz = S.z, tx = T.x, ty = T.y, tz = T.z;
        outN->push_back((float)((sy * tz) - (sz * ty)));
        outN->push_back((float)((sz * tx) - (sx * tz)));
        outN->push_back((float)((sx * ty) - (sy * tx)));
    }
    outP->clear();
    outP->reserve(3 * v.size());
    for (const P3& p : pLimit) { outP->push_back(p.x); outP->push_back(p.y); outP->push_back(p.z); }
    // triangle indices: position of each face vertex in the final level (loopsubdiv.cpp:382-398)
    std::unordered_map<int, int> used;
    used.reserve(v.size() * 2);
    for (size_t i = 0; i < v.size(); ++i) used[v[i]] = (int)i;
    outIdx->clear();
    outIdx->reserve(3 * f.size());
    for (int fi : f)
        for (int j = 0; j < 3; ++j) outIdx->push_back(used.at(m.F[fi].v[j]));
}

}  // namespace pt
