// bvh_build.cpp -- host SAH BVH construction, restating BVHAccel
// (src/accelerators/bvh.cpp:190-402 recursiveBuild, 640-658 flattenBVHTree)
// so that node order, bounds and primitive order equal the reference's: same
// 12-bucket SAH, same leaf rule, and the same libstdc++ std::partition /
// std::nth_element on the primitives in scene order.  The device traverses
// the resulting 32-byte nodes.
//
// Parallel build, same tree: the two children of a node partition disjoint
// ranges [start, mid) and [mid, end) of the primitive-info array, so the top
// subtrees run on their own threads without changing any partition.  The
// reference appends a leaf's primitives to orderedPrims in creation order
// (depth first, left child first), which visits the leaf ranges in increasing
// order -- so orderedPrims is simply the final info array, and a leaf's
// firstPrimOffset is its range start.  Node creation order does not matter:
// flattenBVHTree numbers the nodes depth first.
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>

#include "host_common.h"

namespace pt {

namespace {

BBox bb_empty() {
    BBox b;
    b.pmin = v3(FLT_MAX, FLT_MAX, FLT_MAX);
    b.pmax = v3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    return b;
}
BBox bb_points(V3 a, V3 b) { return BBox{vmin(a, b), vmax(a, b)}; }
BBox bb_union(const BBox& a, const BBox& b) { return BBox{vmin(a.pmin, b.pmin), vmax(a.pmax, b.pmax)}; }
BBox bb_union(const BBox& a, V3 p) { return BBox{vmin(a.pmin, p), vmax(a.pmax, p)}; }
float bb_area(const BBox& b) {
    V3 d = b.pmax - b.pmin;
    return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
}
int bb_max_extent(const BBox& b) {
    V3 d = b.pmax - b.pmin;
    if (d.x > d.y && d.x > d.z) return 0;
    if (d.y > d.z) return 1;
    return 2;
}
V3 bb_offset(const BBox& b, V3 p) {
    V3 o = p - b.pmin;
    if (b.pmax.x > b.pmin.x) o.x /= b.pmax.x - b.pmin.x;
    if (b.pmax.y > b.pmin.y) o.y /= b.pmax.y - b.pmin.y;
    if (b.pmax.z > b.pmin.z) o.z /= b.pmax.z - b.pmin.z;
    return o;
}

struct PrimInfo {
    size_t primitiveNumber;
    BBox bounds;
    V3 centroid;
};

struct BuildNode {
    BBox bounds;
    BuildNode* children[2];
    int splitAxis, firstPrimOffset, nPrimitives;
};

constexpr int kParallelMin = 1 << 15;  // subtrees smaller than this stay on their thread

struct Builder {
    int maxPrimsInNode;
    std::vector<PrimInfo>& info;
    std::atomic<int> totalNodes{0};
    std::mutex mu;
    std::vector<std::unique_ptr<std::deque<BuildNode>>> pools;  // one per build thread

    std::deque<BuildNode>* new_pool() {
        std::lock_guard<std::mutex> lk(mu);
        pools.emplace_back(new std::deque<BuildNode>());
        return pools.back().get();
    }
    void leaf(BuildNode* node, int start, int end, const BBox& bounds) {
        node->firstPrimOffset = start;  // orderedPrims == info after the build (see above)
        node->nPrimitives = end - start;
        node->bounds = bounds;
        node->children[0] = node->children[1] = nullptr;
    }

    BuildNode* build(int start, int end, std::deque<BuildNode>* pool, int par) {
        pool->emplace_back();
        BuildNode* node = &pool->back();
        ++totalNodes;
        BBox bounds = bb_empty();
        for (int i = start; i < end; ++i) bounds = bb_union(bounds, info[i].bounds);
        int nPrimitives = end - start;
        if (nPrimitives == 1) {
            leaf(node, start, end, bounds);
            return node;
        }
        BBox cb = bb_empty();
        for (int i = start; i < end; ++i) cb = bb_union(cb, info[i].centroid);
        int dim = bb_max_extent(cb);
        int mid = (start + end) / 2;
        if (cb.pmax[dim] == cb.pmin[dim]) {
            leaf(node, start, end, bounds);
            return node;
        }
        if (nPrimitives <= 2) {
            mid = (start + end) / 2;
            std::nth_element(&info[start], &info[mid], &info[end - 1] + 1,
                             [dim](const PrimInfo& a, const PrimInfo& b) { return a.centroid[dim] < b.centroid[dim]; });
        } else {
            constexpr int nBuckets = 12;
            int count[nBuckets] = {0};
            BBox bb[nBuckets];
            for (int i = 0; i < nBuckets; ++i) bb[i] = bb_empty();
            auto bucket = [&](V3 c) {
                int b = (int)(nBuckets * bb_offset(cb, c)[dim]);
                if (b == nBuckets) b = nBuckets - 1;
                return b;
            };
            for (int i = start; i < end; ++i) {
                int b = bucket(info[i].centroid);
                count[b]++;
                bb[b] = bb_union(bb[b], info[i].bounds);
            }
            float cost[nBuckets - 1];
            for (int i = 0; i < nBuckets - 1; ++i) {
                BBox b0 = bb_empty(), b1 = bb_empty();
                int c0 = 0, c1 = 0;
                for (int j = 0; j <= i; ++j) { b0 = bb_union(b0, bb[j]); c0 += count[j]; }
                for (int j = i + 1; j < nBuckets; ++j) { b1 = bb_union(b1, bb[j]); c1 += count[j]; }
                cost[i] = 1 + (c0 * bb_area(b0) + c1 * bb_area(b1)) / bb_area(bounds);
            }
            float minCost = cost[0];
            int split = 0;
            for (int i = 1; i < nBuckets - 1; ++i)
                if (cost[i] < minCost) { minCost = cost[i]; split = i; }
            float leafCost = (float)nPrimitives;
            if (nPrimitives > maxPrimsInNode || minCost < leafCost) {
                PrimInfo* pm = std::partition(&info[start], &info[end - 1] + 1,
                                              [&](const PrimInfo& pi) { return bucket(pi.centroid) <= split; });
                mid = (int)(pm - &info[0]);
            } else {
                leaf(node, start, end, bounds);
                return node;
            }
        }
        BuildNode *c0 = nullptr, *c1 = nullptr;
        if (par > 0 && nPrimitives >= kParallelMin) {  // left subtree on its own thread
            std::deque<BuildNode>* lp = new_pool();
            std::thread t([&] { c0 = build(start, mid, lp, par - 1); });
            c1 = build(mid, end, pool, par - 1);
            t.join();
        } else {
            c0 = build(start, mid, pool, 0);
            c1 = build(mid, end, pool, 0);
        }
        node->children[0] = c0;
        node->children[1] = c1;
        node->bounds = bb_union(c0->bounds, c1->bounds);
        node->splitAxis = dim;
        node->nPrimitives = 0;
        return node;
    }
};

int flatten(BuildNode* n, std::vector<LinearNode>& out, int* offset) {
    LinearNode& ln = out[*offset];
    ln.bmin[0] = n->bounds.pmin.x; ln.bmin[1] = n->bounds.pmin.y; ln.bmin[2] = n->bounds.pmin.z;
    ln.bmax[0] = n->bounds.pmax.x; ln.bmax[1] = n->bounds.pmax.y; ln.bmax[2] = n->bounds.pmax.z;
    ln.pad = 0;
    int my = (*offset)++;
    if (n->nPrimitives > 0) {
        if (n->nPrimitives >= 65536) throw PtError(PT_ERR_UNSUPPORTED, "BVH leaf with >= 65536 primitives");
        out[my].offset = n->firstPrimOffset;
        out[my].nprims = (uint16_t)n->nPrimitives;
        out[my].axis = 0;
    } else {
        out[my].axis = (uint8_t)n->splitAxis;
        out[my].nprims = 0;
        flatten(n->children[0], out, offset);
        int second = flatten(n->children[1], out, offset);
        out[my].offset = second;
    }
    return my;
}

}  // namespace

BBox prim_world_bound(const pt_scene_desc* d, int i) {
    const pt_prim& p = d->prims[i];
    if (p.kind == PT_PRIM_TRIANGLE) {  // Triangle::WorldBound (triangle.cpp:180-187)
        const pt_triangle& t = d->triangles[p.index];
        auto P = [&](int k) { return v3(d->P[3 * k], d->P[3 * k + 1], d->P[3 * k + 2]); };
        return bb_union(bb_points(P(t.v[0]), P(t.v[1])), P(t.v[2]));
    }
    // Shape::WorldBound = ObjectToWorld(ObjectBound()) (shape.cpp:52, transform.cpp:238-249)
    BBox ob;
    M4 m;
    if (p.kind == PT_PRIM_SPHERE) {  // Sphere::ObjectBound (sphere.cpp:44-47)
        const pt_sphere& sp = d->spheres[p.index];
        const SphereMembers sm = sphere_members(sp);
        ob = bb_points(v3(-sm.radius, -sm.radius, sm.zmin), v3(sm.radius, sm.radius, sm.zmax));
        std::memcpy(m.m, sp.object_to_world.m, 64);
    } else {
        const pt_aaplane& pl = d->planes[p.index];
        ob = bb_points(v3(pl.lo[0], pl.lo[1], pl.lo[2]), v3(pl.hi[0], pl.hi[1], pl.hi[2]));
        std::memcpy(m.m, pl.object_to_world.m, 64);
    }
    V3 a = ob.pmin, b = ob.pmax;
    V3 q = xf_point(m, v3(a.x, a.y, a.z));
    BBox r{q, q};
    r = bb_union(r, xf_point(m, v3(b.x, a.y, a.z)));
    r = bb_union(r, xf_point(m, v3(a.x, b.y, a.z)));
    r = bb_union(r, xf_point(m, v3(a.x, a.y, b.z)));
    r = bb_union(r, xf_point(m, v3(a.x, b.y, b.z)));
    r = bb_union(r, xf_point(m, v3(b.x, b.y, a.z)));
    r = bb_union(r, xf_point(m, v3(b.x, a.y, b.z)));
    r = bb_union(r, xf_point(m, v3(b.x, b.y, b.z)));
    return r;
}

void build_bvh(const pt_scene_desc* d, std::vector<LinearNode>* nodes, std::vector<int>* prim_order) {
    nodes->clear();
    prim_order->clear();
    if (d->n_prims <= 0) return;
    const int hw = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<PrimInfo> info((size_t)d->n_prims);
    {   // primitive bounds (BVHPrimitiveInfo, bvh.cpp:206-209), in parallel slices
        std::vector<std::thread> th;
        const int n = d->n_prims, per = (n + hw - 1) / hw;
        for (int t = 0; t < hw; ++t)
            th.emplace_back([&, t] {
                for (int i = t * per; i < std::min(n, (t + 1) * per); ++i) {
                    info[i].primitiveNumber = (size_t)i;
                    info[i].bounds = prim_world_bound(d, i);
                    info[i].centroid = .5f * info[i].bounds.pmin + .5f * info[i].bounds.pmax;
                }
            });
        for (auto& t : th) t.join();
    }
    int maxPrims = d->bvh_max_prims > 0 ? std::min(255, d->bvh_max_prims) : 4;
    Builder b{maxPrims, info};
    int par = 0;
    while ((1 << par) < hw) ++par;
    BuildNode* root = b.build(0, d->n_prims, b.new_pool(), par);
    prim_order->resize((size_t)d->n_prims);
    for (int i = 0; i < d->n_prims; ++i) (*prim_order)[i] = (int)info[i].primitiveNumber;
    nodes->resize((size_t)b.totalNodes.load());
    int off = 0;
    flatten(root, *nodes, &off);
}

}  // namespace pt
