// kernels.hip -- the wavefront path tracer's gfx950 kernels.
//
// One batch = (pixel list) x (consecutive sample indices).  Per bounce the
// host enqueues k_trace over the ray queue (continuation + NEE rays) and
// k_shade over the path queue.  k_shade first resolves the NEE rays of the
// previous vertex (L += beta * Ld, integrator.cpp:122), then shades the new
// hit exactly as PathIntegrator::Li (path.cpp:81-186) and appends the next
// rays / live paths with one wave-aggregated atomic per wave (ballot +
// mbcnt prefix).  k_film adds the finished samples to the film in sample
// order (FilmTile::AddSample, film.h:121-161) by gathering over each pixel's
// filter window -- deterministic, no float atomics.
#pragma once
#include "devfuncs.h"
#include "kernels.h"
#undef PT_FILE_ID
#define PT_FILE_ID 2  // PT_IDX source tag

namespace pt {

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// number of set bits of m below this lane (the mbcnt prefix count)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Reserve `cnt` (0..3) consecutive queue entries per lane with one atomic per
// wave.  Must be reached by every active lane of the wave together.
__device__ __forceinline__ uint32_t wave_reserve(uint32_t* counter, uint32_t cnt) {
    const uint64_t b0 = __ballot((cnt & 1u) != 0);
    const uint64_t b1 = __ballot((cnt & 2u) != 0);
    const uint64_t act = __ballot(1);
    const uint32_t lane = lane_id();
    const uint64_t lower = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t prefix = (uint32_t)__popcll(b0 & lower) + 2u * (uint32_t)__popcll(b1 & lower);
    const uint32_t total = (uint32_t)__popcll(b0) + 2u * (uint32_t)__popcll(b1);
    const int leader = __ffsll((unsigned long long)act) - 1;
    uint32_t base = 0;
    if ((int)lane == leader && total) base = atomicAdd(counter, total);
    base = (uint32_t)__shfl((int)base, leader);
    return base + prefix;
}

// Queue appends of one wave, staged in LDS across grid-stride iterations and
// published with ONE packed 64-bit atomic per flush that reserves room in both
// output queues (counts[2] = rays in the low word, counts[3] = paths in the
// high word).  Same-address atomics serialise in one L2 channel: two per wave
// per iteration bounded the shading kernels (doubling them doubled k_shade's
// time), so a wave now flushes once per several hundred queue entries.
#ifndef PT_WQR
#define PT_WQR 448
#define PT_WQP 192
#endif
constexpr uint32_t kWqRays = PT_WQR;   // >= 3 * 64: one iteration always fits after a flush
constexpr uint32_t kWqPaths = PT_WQP;  // >= 64
struct WaveQ {
    uint32_t* r;       // LDS, kWqRays ray-queue entries
    uint32_t* p;       // LDS, kWqPaths path-queue entries
    uint32_t nr, np;   // fill levels (wave-uniform)
};
__device__ __forceinline__ void wq_flush(WaveQ& q, uint32_t* counts2, uint32_t* rq_out, uint32_t* pq_out) {
    if ((q.nr | q.np) == 0) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t lane = lane_id();
    unsigned long long old = 0;
    if (lane == 0)
        old = atomicAdd((unsigned long long*)counts2, (unsigned long long)q.nr | ((unsigned long long)q.np << 32));
    const uint32_t rb = (uint32_t)__shfl((int)(uint32_t)old, 0);
    const uint32_t pb = (uint32_t)__shfl((int)(uint32_t)(old >> 32), 0);
    for (uint32_t k = lane; k < q.nr; k += 64) rq_out[rb + k] = q.r[k];
    for (uint32_t k = lane; k < q.np; k += 64) pq_out[pb + k] = q.p[k];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    q.nr = 0;
    q.np = 0;
}
// A step's 0..3 ray-queue entries in three registers (pushed by selects: a
// dynamically indexed array would live in scratch).
struct RayList {
    uint32_t r0 = 0, r1 = 0, r2 = 0;
    uint32_t n = 0;
    __device__ __forceinline__ void push(uint32_t e) {
        r0 = n == 0 ? e : r0;
        r1 = n == 1 ? e : r1;
        r2 = n == 2 ? e : r2;
        ++n;
    }
};
// Append nrays (0..3) ray entries and, if keep, the path slot.  Reached by
// every lane of the wave together.
__device__ __forceinline__ void wq_push(WaveQ& q, const RayList& rl, bool keep, uint32_t slot, uint32_t* counts2,
                                        uint32_t* rq_out, uint32_t* pq_out) {
    const uint32_t nrays = rl.n;
    const uint64_t b0 = __ballot((nrays & 1u) != 0);
    const uint64_t b1 = __ballot((nrays & 2u) != 0);
    const uint64_t bp = __ballot(keep);
    const uint32_t lane = lane_id();
    const uint64_t lower = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t rtot = (uint32_t)__popcll(b0) + 2u * (uint32_t)__popcll(b1);
    const uint32_t ptot = (uint32_t)__popcll(bp);
    if (q.nr + rtot > kWqRays || q.np + ptot > kWqPaths) wq_flush(q, counts2, rq_out, pq_out);
    const uint32_t rpre = q.nr + (uint32_t)__popcll(b0 & lower) + 2u * (uint32_t)__popcll(b1 & lower);
    if (nrays > 0) q.r[rpre] = rl.r0;
    if (nrays > 1) q.r[rpre + 1] = rl.r1;
    if (nrays > 2) q.r[rpre + 2] = rl.r2;
    if (keep) q.p[q.np + (uint32_t)__popcll(bp & lower)] = slot;
    q.nr += rtot;
    q.np += ptot;
}
#define PT_WAVEQ(q)                                                   \
    __shared__ uint32_t wq_r_[kShadeBlock / 64][kWqRays];             \
    __shared__ uint32_t wq_p_[kShadeBlock / 64][kWqPaths];            \
    WaveQ q{wq_r_[threadIdx.x / 64], wq_p_[threadIdx.x / 64], 0u, 0u}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ void flush_stats(DevStats* s, unsigned long long cl, unsigned long long sh,
                                            unsigned long long nodes, unsigned long long prims) {
    cl = wave_sum_u64(cl);
    sh = wave_sum_u64(sh);
    nodes = wave_sum_u64(nodes);
    prims = wave_sum_u64(prims);
    if (lane_id() == 0) {
        if (cl) atomicAdd(&s->closest, cl);
        if (sh) atomicAdd(&s->shadow, sh);
        if (nodes) atomicAdd(&s->nodes, nodes);
        if (prims) atomicAdd(&s->prims, prims);
    }
}

// ----------------------------------------------------------------------------
// BVH traversal (BVHAccel::Intersect / IntersectP, bvh.cpp:662-738).
// Near-child-first order by dirIsNeg[axis], tMax shrinking on every
// accepted hit (GeometricPrimitive::Intersect, primitive.cpp:116-130).
// The 64-entry node stack lives in LDS (kStackLds entries per lane,
// [entry][lane] layout) with a per-thread global spill for deeper trees.
// ----------------------------------------------------------------------------
template <bool kAny, bool kSph = true>
__device__ __forceinline__ int traverse(const DevScene& sc, const float4* __restrict__ bnodes,
                                        const float4* __restrict__ bprims, Ray ray, int (*stk)[kTraceBlock],
                                        int* spill, unsigned long long* nodes, unsigned long long* prims,
                                        float* tOut = nullptr) {
    const int tid = threadIdx.x;
    const V3 inv = v3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
    const bool n0 = inv.x < 0, n1 = inv.y < 0, n2 = inv.z < 0;
    const float kx = 1 + 2 * gammaf(3);
    int toVisit = 0, cur = 0, hitPrim = -1;
    if (sc.n_nodes == 0) return -1;
    for (;;) {
        const float4 a = bnodes[2 * cur];
        const float4 b = bnodes[2 * cur + 1];
        ++*nodes;
        // Bounds3::IntersectP(ray, invDir, dirIsNeg) (geometry.h:1584-1606)
        float tMin = ((n0 ? a.w : a.x) - ray.o.x) * inv.x;
        float tMax = ((n0 ? a.x : a.w) - ray.o.x) * inv.x;
        float tyMin = ((n1 ? b.x : a.y) - ray.o.y) * inv.y;
        float tyMax = ((n1 ? a.y : b.x) - ray.o.y) * inv.y;
        tMax *= kx;
        tyMax *= kx;
        bool hitb = !(tMin > tyMax || tyMin > tMax);
        if (hitb) {
            if (tyMin > tMin) tMin = tyMin;
            if (tyMax < tMax) tMax = tyMax;
            float tzMin = ((n2 ? b.y : a.z) - ray.o.z) * inv.z;
            float tzMax = ((n2 ? a.z : b.y) - ray.o.z) * inv.z;
            tzMax *= kx;
            hitb = !(tMin > tzMax || tzMin > tMax);
            if (hitb) {
                if (tzMin > tMin) tMin = tzMin;
                if (tzMax < tMax) tMax = tzMax;
                hitb = (tMin < ray.tmax) && (tMax > 0);
            }
        }
        if (hitb) {
            const int off = __float_as_int(b.z);
            const uint32_t npax = __float_as_uint(b.w);
            const int np = (int)(npax & 0xffffu);
            if (np > 0) {
                for (int i = 0; i < np; ++i) {
                    const int pi = off + i;
                    ++*prims;
                    const float4 r0 = bprims[3 * pi];
                    const float4 r1 = bprims[3 * pi + 1];
                    const uint32_t fl = __float_as_uint(r0.w);
                    float t;
                    bool ok;
                    if (fl & kPrimAnalytic) {
                        ok = shape_test<kSph>(sc, fl, __float_as_int(r1.w), ray, &t);
                    } else {
                        const float4 r2 = bprims[3 * pi + 2];
                        float b0, b1, b2;
                        ok = tri_test(v3(r0.x, r0.y, r0.z), v3(r1.x, r1.y, r1.z), v3(r2.x, r2.y, r2.z), ray, &t, &b0,
                                      &b1, &b2);
                        if (!kAny && (fl & kPrimDegenerate)) ok = false;
                    }
                    if (ok) {
                        if (kAny) return pi;
                        ray.tmax = t;
                        hitPrim = pi;
                    }
                }
                if (toVisit == 0) break;
                --toVisit;
                cur = toVisit < kStackLds ? stk[toVisit][tid] : spill[toVisit - kStackLds];
            } else {
                const int axis = (int)(npax >> 16);
                const bool neg = axis == 0 ? n0 : (axis == 1 ? n1 : n2);
                const int far = neg ? cur + 1 : off;
                cur = neg ? off : cur + 1;
                if (toVisit < kStackLds) stk[toVisit][tid] = far;
                else spill[toVisit - kStackLds] = far;
                ++toVisit;
            }
        } else {
            if (toVisit == 0) break;
            --toVisit;
            cur = toVisit < kStackLds ? stk[toVisit][tid] : spill[toVisit - kStackLds];
        }
    }
    if (tOut) *tOut = ray.tmax;  // GeometricPrimitive::Intersect sets ray.tMax = tHit
    return hitPrim;
}

// Ray records (DevPaths::ray / rayA / rayB): 32 B per slot, {o.xyz, d.x} {d.yz, tMax, 0} -- one
// 32-B sector, two 16-B accesses per lane (round 2's SoA fields took six or seven 4-B accesses, each
// its own sector when a queue's slots are spread).  tMax is the shadow ray's bound (ray A of the MIS
// estimator), kInf for closest-hit rays.
__device__ __forceinline__ Ray load_ray(const float* a, uint32_t slot) {
    const float4* r = reinterpret_cast<const float4*>(a) + 2 * (size_t)slot;
    const float4 p = r[0], q = r[1];
    return Ray{v3(p.x, p.y, p.z), v3(p.w, q.x, q.y), q.z};
}
__device__ __forceinline__ Ray load_ray(const float* a, uint32_t slot, float tmax) {
    Ray r = load_ray(a, slot);
    r.tmax = tmax;
    return r;
}
// the traversal's refill: o, d and (shadow rays only) tMax -- one 16-B, one 8-B and one 4-B load,
// no register for the record's pad word
__device__ __forceinline__ Ray load_ray_trace(const float* a, uint32_t slot, bool shadow) {
    const float4* r = reinterpret_cast<const float4*>(a) + 2 * (size_t)slot;
    const float4 p = r[0];
    const float2 q = *reinterpret_cast<const float2*>(r + 1);
    const float t = shadow ? reinterpret_cast<const float*>(r + 1)[2] : kInf;
    return Ray{v3(p.x, p.y, p.z), v3(p.w, q.x, q.y), t};
}
__device__ __forceinline__ void store_ray(float* a, uint32_t slot, const Ray& r) {
    float4* d = reinterpret_cast<float4*>(a) + 2 * (size_t)slot;
    d[0] = make_float4(r.o.x, r.o.y, r.o.z, r.d.x);
    d[1] = make_float4(r.d.y, r.d.z, r.tmax, 0.f);
}

// kLdsScene: small scenes (nodes + prim records <= kLdsSceneMax bytes) are
// staged once per block into LDS, so the dependent node/primitive fetches of
// the traversal are LDS reads instead of L1/L2 round trips.
template <bool kLdsScene, bool kSph>
__global__ __launch_bounds__(kTraceBlock) void k_trace(DevScene sc, DevPaths ps, const uint32_t* __restrict__ rq,
                                                       const uint32_t* __restrict__ rq_count, int* spill,
                                                       DevStats* stats)
#ifdef PT_TU_TRACE
{
    __shared__ int stk[kStackLds][kTraceBlock];
    extern __shared__ float4 lds_scene[];
    const float4* bnodes = sc.nodes;
    const float4* bprims = sc.prims;
    if constexpr (kLdsScene) {
        const int nn = 2 * sc.n_nodes, total = nn + 3 * sc.n_prims;
        for (int i = threadIdx.x; i < total; i += blockDim.x) lds_scene[i] = i < nn ? sc.nodes[i] : sc.prims[i - nn];
        __syncthreads();
        bnodes = lds_scene;
        bprims = lds_scene + nn;
    }
    const uint32_t n = *rq_count;
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    int* myspill = spill + (size_t)gtid * (64 - kStackLds);
    unsigned long long nodes = 0, prims = 0, ncl = 0, nsh = 0;
    for (uint32_t i = gtid; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t e = rq[i];
        const uint32_t slot = e >> 2, kind = e & 3u;
        if (kind == kRayShadow) {
            Ray r = load_ray(ps.rayA, slot);
            int h = traverse<true, kSph>(sc, bnodes, bprims, r, stk, myspill, &nodes, &prims);
            *hit_word(ps, slot, kHdHitA) = h >= 0 ? 1 : 0;
            ++nsh;
        } else {
            Ray r;
            if (kind == kRayCont) r = load_ray(ps.ray, slot, kInf);
            else if (kind == kRayA) r = load_ray(ps.rayA, slot, kInf);
            else r = load_ray(ps.rayB, slot, kInf);
            int h = traverse<false, kSph>(sc, bnodes, bprims, r, stk, myspill, &nodes, &prims);
            if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = h;
            else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = h;
            else *hit_word(ps, slot, kHdHitB) = h;
            ++ncl;
        }
    }
    flush_stats(stats, ncl, nsh, nodes, prims);
}
#else
;
#endif

// ----------------------------------------------------------------------------
// Persistent traversal with per-lane ray refill.  The same traversal as
// traverse<kAny> (same node order, same box and primitive tests, same tMax
// updates, same counters) restated as a one-step-per-iteration state machine:
// each iteration a lane either visits one node or tests one primitive of the
// leaf it reached, and a lane whose ray has finished takes the next ray of
// the queue (one atomic per wave per refill) instead of idling until the
// slowest ray of its wave is done.
// ----------------------------------------------------------------------------
__device__ __forceinline__ bool node_box_hit(float4 a, float4 b, const Ray& ray, V3 inv, bool n0, bool n1, bool n2) {
    // Bounds3::IntersectP(ray, invDir, dirIsNeg) (geometry.h:1584-1606), its
    // early exits folded into one predicate (same values, no branches)
    const float kx = 1 + 2 * gammaf(3);
    float tMin = ((n0 ? a.w : a.x) - ray.o.x) * inv.x;
    float tMax = ((n0 ? a.x : a.w) - ray.o.x) * inv.x;
    const float tyMin = ((n1 ? b.x : a.y) - ray.o.y) * inv.y;
    float tyMax = ((n1 ? a.y : b.x) - ray.o.y) * inv.y;
    const float tzMin = ((n2 ? b.y : a.z) - ray.o.z) * inv.z;
    float tzMax = ((n2 ? a.z : b.y) - ray.o.z) * inv.z;
    tMax *= kx;
    tyMax *= kx;
    tzMax *= kx;
    const bool ok1 = !(tMin > tyMax) & !(tyMin > tMax);
    tMin = tyMin > tMin ? tyMin : tMin;
    tMax = tyMax < tMax ? tyMax : tMax;
    const bool ok2 = !(tMin > tzMax) & !(tzMin > tMax);
    tMin = tzMin > tMin ? tzMin : tMin;
    tMax = tzMax < tMax ? tzMax : tMax;
    return ok1 & ok2 & (tMin < ray.tmax) & (tMax > 0);
}

// 7 waves per SIMD without spheres (72 VGPRs: the one-register stack position below brought the
// kernel from 78 to 74, and the remaining 12 B of spills are reloaded once per primitive test; C5
// isolated 52.7 -> 49.4 ms per launch); PT_TRACE_PT_WAVES (experiment builds) overrides
#ifdef PT_TRACE_PT_WAVES
#define PT_TRACE_PT_ATTR __attribute__((amdgpu_waves_per_eu(PT_TRACE_PT_WAVES)))
#else
#define PT_TRACE_PT_ATTR __attribute__((amdgpu_waves_per_eu(kSph ? 1 : 7)))
#endif
template <bool kLdsScene, bool kSpill, bool kSph>
__global__ __launch_bounds__(kTraceBlock) PT_TRACE_PT_ATTR void k_trace_pt(DevScene sc, DevPaths ps, const uint32_t* __restrict__ rq,
                                                          const uint32_t* __restrict__ rq_count, uint32_t* fetch,
                                                          int refill_min, int leaf_min, int stack_rows, int* spill,
                                                          DevStats* stats)
#ifdef PT_TU_TRACE
{
    // Dynamic LDS: [scene float4s if kLdsScene][stack].  With kSpill the
    // stack is kStackLds entries per lane plus a global spill; without, the
    // BVH is shallow enough that stack_rows entries per lane always suffice.
    extern __shared__ float4 lds_dyn[];
    const float4* bnodes = sc.nodes;
    const float4* bprims = sc.prims;
    const int scene_f4 = kLdsScene ? 2 * sc.n_nodes + 3 * sc.n_prims : 0;
    if constexpr (kLdsScene) {
        const int nn = 2 * sc.n_nodes;
        for (int i = threadIdx.x; i < scene_f4; i += blockDim.x) lds_dyn[i] = i < nn ? sc.nodes[i] : sc.prims[i - nn];
        __syncthreads();
        bnodes = lds_dyn;
        bprims = lds_dyn + nn;
    }
    int* stk = (int*)(lds_dyn + scene_f4);  // [row][kTraceBlock]
    const uint32_t n = *rq_count;
    const uint32_t rmin = (uint32_t)min(max(refill_min, 1), 64);  // idle lanes that trigger a refill
    const uint32_t lmin = (uint32_t)max(leaf_min, 1);             // parked lanes that trigger a leaf step
    const int tid = threadIdx.x;
    const uint32_t lane = lane_id();
    // The stack position as ONE register: so = toVisit * 512 + 4 * tid, the byte offset of the lane's next
    // free LDS stack entry ([row][kTraceBlock] ints, rows 512 bytes apart) -- its depth is so >> 9, its
    // column so & 511 -- instead of the depth plus the thread index (which the 7-wave budget, 72 VGPRs,
    // otherwise spilled).  Entries past the LDS rows go to the lane's spill column, entry v at spill[SPILL(v)].
    static_assert(kTraceBlock * 4 == 512, "k_trace_pt stack rows are 512 bytes apart");
#define SPILL(v) ((blockIdx.x * (uint32_t)kTraceBlock + ((so & 511u) >> 2)) * 64u + (uint32_t)(v))
#define STK(o) (*reinterpret_cast<int*>(reinterpret_cast<char*>(stk) + (o)))
    // The counters as wave totals (uniform: scalar registers).  A lane's node visits and primitive tests of
    // one loop iteration (cst: visits in bits 0-3, tests in bits 8-11) are added at the top of the next,
    // where the wave's lanes are converged, one ballot per bit; rays where the refill takes them.
    static_assert(kNodeSteps < 16 && kLeafSteps < 16, "k_trace_pt step counts are 4-bit fields");
    uint32_t ncl_w = 0, nsh_w = 0, nodes_w = 0, prims_w = 0;
    uint32_t cst = 0;
    uint32_t iters_w = 0;
    bool active = false, exhausted = false, drained = false;
    uint32_t qn = 0, qe = 0;  // the wave's private chunk of the ray queue (as k_trace_nb)
    uint32_t ent = 0;  // the ray-queue entry: slot << 2 | kind (one register for both)
    Ray ray{v3(0, 0, 0), v3(0, 0, 1), 0};
    V3 inv = v3(0, 0, 0);
    TriShear sh{0, 0, 0, 0};
    bool n0 = false, n1 = false, n2 = false;
    const uint32_t so0 = 4u * (uint32_t)tid;  // an empty stack
    uint32_t so = so0;
    const uint32_t soRows = (uint32_t)stack_rows * 512u;
    int cur = 0, hitPrim = -1, leafPos = 0, leafEnd = 0;
    for (;;) {
#pragma unroll
        for (int bit = 0; bit < 4; ++bit) {
            if ((1 << bit) <= kNodeSteps) nodes_w += (uint32_t)__popcll(__ballot((cst >> bit) & 1u)) << bit;
            if ((1 << bit) <= kLeafSteps) prims_w += (uint32_t)__popcll(__ballot((cst >> (8 + bit)) & 1u)) << bit;
        }
        cst = 0;
        if (!exhausted) {
            const uint64_t idle = __ballot(!active);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (nidle >= rmin) {  // rmin in [1, 64]: one scalar compare
                if (qn >= qe && !drained) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(fetch, kTraceChunk);
                    base = __builtin_amdgcn_readlane(base, 0);  // the lane that did the atomic, whatever EXEC holds: in an SGPR
                    qn = base < n ? base : n;
                    qe = base + kTraceChunk < n ? base + kTraceChunk : n;
                    drained = base + kTraceChunk >= n;
                }
                const uint32_t take = qe - qn < nidle ? qe - qn : nidle;
                const uint32_t k = lanes_below(idle);
                const uint32_t i = qn + k;
                qn += take;
                if (drained && qn >= qe) exhausted = true;
                const bool takes = !active && k < take;  // exactly `take` idle lanes
                if (!active) {
                    if (k < take) {
                        const uint32_t e = rq[i];
                        ent = e;
                        const uint32_t slot = e >> 2, kind = e & 3u;
                        ray = load_ray_trace(kind == kRayCont ? ps.ray : (kind == kRayB ? ps.rayB : ps.rayA), slot, kind == kRayShadow);
                        inv = v3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
                        sh = tri_shear(ray.d);
                        n0 = inv.x < 0; n1 = inv.y < 0; n2 = inv.z < 0;
                        cur = 0; so = so & 511u; hitPrim = -1; leafPos = 0; leafEnd = 0;
                        active = sc.n_nodes > 0;  // empty scene: every ray misses
                        if (!active) {
                            if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = 0;
                            else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = -1;
                            else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = -1;
                            else *hit_word(ps, slot, kHdHitB) = -1;
                        }
                    }
                }
                const uint32_t nsh = (uint32_t)__popcll(__ballot(takes && (ent & 3u) == kRayShadow));
                nsh_w += nsh;
                ncl_w += take - nsh;
            }
        }
        if (__ballot(active) == 0) {
            if (exhausted) break;
            continue;
        }
        // One uniform step kind per iteration: primitive tests for the lanes
        // parked at a leaf once at least leaf_min of them are (or no lane has
        // a node to visit), otherwise node visits for the others.  A lane's
        // own sequence of node visits and primitive tests is unchanged.
        const bool wantLeaf = active && leafPos < leafEnd;
        const uint32_t nLeaf = (uint32_t)__popcll(__ballot(wantLeaf));
        const uint32_t nNode = (uint32_t)__popcll(__ballot(active && !wantLeaf));
        const bool leafStep = nLeaf >= (nNode == 0 ? 1u : lmin);  // lmin >= 1
        ++iters_w;
        if (!active || wantLeaf != leafStep) continue;
        bool done = false;
        if (leafStep) {
#pragma unroll
            for (int u = 0; u < kLeafSteps; ++u) {  // up to kLeafSteps primitive tests of the lane's leaf
                if (u > 0 && (done || leafPos >= leafEnd)) continue;
                const int pi = leafPos++;
                cst += 0x100u;
                const float4 r0 = bprims[3 * pi];
                const float4 r1 = bprims[3 * pi + 1];
                const uint32_t fl = __float_as_uint(r0.w);
                float t;
                bool ok;
                if (fl & kPrimAnalytic) {
                    ok = shape_test<kSph>(sc, fl, __float_as_int(r1.w), ray, &t);
                } else {
                    const float4 r2 = bprims[3 * pi + 2];
                    ok = tri_hit(v3(r0.x, r0.y, r0.z), v3(r1.x, r1.y, r1.z), v3(r2.x, r2.y, r2.z), ray, sh, &t);
                    if ((ent & 3u) != kRayShadow && (fl & kPrimDegenerate)) ok = false;
                }
                if (ok) {
                    hitPrim = pi;
                    if ((ent & 3u) == kRayShadow) done = true;
                    else ray.tmax = t;
                }
                if (!done && leafPos == leafEnd) {
                    if (so < 512u) done = true;
                    else {
                        so -= 512u;
                        cur = (!kSpill || so < soRows) ? STK(so) : spill[SPILL((so >> 9) - (uint32_t)stack_rows)];
                    }
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < kNodeSteps; ++u) {  // up to kNodeSteps node visits while in node mode
                if (u > 0 && (done || leafPos < leafEnd)) continue;
                const float4 a = bnodes[2 * cur];
                const float4 b = bnodes[2 * cur + 1];
                ++cst;
                if (node_box_hit(a, b, ray, inv, n0, n1, n2)) {
                    const int off = __float_as_int(b.z);
                    const uint32_t npax = __float_as_uint(b.w);
                    const int np = (int)(npax & 0xffffu);
                    if (np > 0) {
                        leafPos = off;
                        leafEnd = off + np;
                    } else {
                        const int axis = (int)(npax >> 16);
                        const bool neg = axis == 0 ? n0 : (axis == 1 ? n1 : n2);
                        const int far = neg ? cur + 1 : off;
                        cur = neg ? off : cur + 1;
                        if (!kSpill || so < soRows) STK(so) = far;
                        else spill[SPILL((so >> 9) - (uint32_t)stack_rows)] = far;
                        so += 512u;
                    }
                } else if (so < 512u) {
                    done = true;
                } else {
                    so -= 512u;
                    cur = (!kSpill || so < soRows) ? STK(so) : spill[SPILL((so >> 9) - (uint32_t)stack_rows)];
                }
            }
        }
        if (done) {
            const uint32_t slot = ent >> 2, kind = ent & 3u;
            if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = hitPrim >= 0 ? 1 : 0;
            else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = hitPrim;
            else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = hitPrim;
            else *hit_word(ps, slot, kHdHitB) = hitPrim;
            active = false;
        }
    }
    if (lane == 0) {
        if (ncl_w) atomicAdd(&stats->closest, (unsigned long long)ncl_w);
        if (nsh_w) atomicAdd(&stats->shadow, (unsigned long long)nsh_w);
        if (nodes_w) atomicAdd(&stats->nodes, (unsigned long long)nodes_w);
        if (prims_w) atomicAdd(&stats->prims, (unsigned long long)prims_w);
        if (iters_w) atomicAdd(&stats->lane_iters, 64ull * iters_w);
    }
#undef SPILL
#undef STK
}
#else
;
#endif

// ----------------------------------------------------------------------------
// k_trace_nb: k_trace_pt with the per-step control flow replaced by selects
// (the traversal is the same; only which instructions run changes).  The
// stack push is an unconditional LDS store above the top; the pop an
// unconditional LDS load below it.  Only for BVHs whose stack fits in LDS.
// ----------------------------------------------------------------------------
// PT_TRACE_WAVES (experiment builds): force the waves-per-SIMD register budget
#ifdef PT_TRACE_WAVES
#define PT_TRACE_NB_ATTR __attribute__((amdgpu_waves_per_eu(PT_TRACE_WAVES)))
#else
#define PT_TRACE_NB_ATTR
#endif
// The 32-byte node as two ds_read_b128 (4 LDS cycles each per wave; the
// compiler's own split of the two float4 loads into b96 + b32 pieces takes 18)
__device__ __forceinline__ void lds_node(const float4* lds_nodes, int c, float4* a, float4* b) {
    // (C2 k_trace_nb 9.05 -> 8.87 ms per launch).  lds_nodes is the LDS copy: its
    // generic address's low 32 bits are the LDS offset.
    const uint32_t addr = (uint32_t)(uintptr_t)(lds_nodes + 2 * c);
    float4 x, y;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(x), "=v"(y) : "v"(addr) : "memory");
    *a = x;
    *b = y;
}

template <bool kLdsScene, bool kSph>
__global__ __launch_bounds__(kTraceBlock) PT_TRACE_NB_ATTR void k_trace_nb(DevScene sc, DevPaths ps, const uint32_t* __restrict__ rq,
                                                          const uint32_t* __restrict__ rq_count, uint32_t* fetch,
                                                          int refill_min, int leaf_min, DevStats* stats)
#ifdef PT_TU_TRACE
{
    extern __shared__ float4 lds_dyn[];
    const float4* bnodes = sc.nodes;
    const float4* bprims = sc.prims;
    const int scene_f4 = kLdsScene ? 2 * sc.n_nodes + 3 * sc.n_prims : 0;
    if constexpr (kLdsScene) {
        const int nn = 2 * sc.n_nodes;
        for (int i = threadIdx.x; i < scene_f4; i += blockDim.x) lds_dyn[i] = i < nn ? sc.nodes[i] : sc.prims[i - nn];
        __syncthreads();
        bnodes = lds_dyn;
        bprims = lds_dyn + nn;
    }
    int* stk = (int*)(lds_dyn + scene_f4) + threadIdx.x;  // entry k at stk[k * kTraceBlock]
    const uint32_t n = *rq_count;
    const uint32_t rmin = (uint32_t)min(max(refill_min, 1), 64);  // idle lanes that trigger a refill
    const uint32_t lmin = (uint32_t)max(leaf_min, 1);             // parked lanes that trigger a leaf step
    const uint32_t lane = lane_id();
    uint32_t nodes = 0, prims = 0, ncl = 0, nsh = 0, iters = 0;
    bool active = false, exhausted = false, drained = false;
    // The wave takes queue entries kTraceChunk at a time (one atomic) and
    // hands them to its idle lanes from that private chunk, so frequent partial
    // refills do not each hit the one shared counter.
    uint32_t qn = 0, qe = 0;
    uint32_t slot = 0, kind = 0;
    Ray ray{v3(0, 0, 0), v3(0, 0, 1), 0};
    V3 inv = v3(0, 0, 0);
    TriShear sh{0, 0, 0, 0};
    bool n0 = false, n1 = false, n2 = false;
    int cur = 0, toVisit = 0, hitPrim = -1, leafPos = 0, leafEnd = 0;
    for (;;) {
        if (!exhausted) {
            const uint64_t idle = __ballot(!active);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (nidle >= rmin) {  // rmin in [1, 64]: one scalar compare
                if (qn >= qe && !drained) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(fetch, kTraceChunk);
                    base = __builtin_amdgcn_readlane(base, 0);  // the lane that did the atomic, whatever EXEC holds: in an SGPR
                    qn = base < n ? base : n;
                    qe = base + kTraceChunk < n ? base + kTraceChunk : n;
                    drained = base + kTraceChunk >= n;
                }
                const uint32_t take = qe - qn < nidle ? qe - qn : nidle;
                const uint32_t k = lanes_below(idle);
                const uint32_t i = qn + k;
                qn += take;
                if (drained && qn >= qe) exhausted = true;
                if (!active) {
                    if (k < take) {
                        const uint32_t e = rq[i];
                        slot = e >> 2;
                        kind = e & 3u;
                        ray = load_ray_trace(kind == kRayCont ? ps.ray : (kind == kRayB ? ps.rayB : ps.rayA), slot, kind == kRayShadow);
                        inv = v3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
                        sh = tri_shear(ray.d);
                        n0 = inv.x < 0; n1 = inv.y < 0; n2 = inv.z < 0;
                        cur = 0; toVisit = 0; hitPrim = -1; leafPos = 0; leafEnd = 0;
                        active = sc.n_nodes > 0;  // empty scene: every ray misses
                        if (!active) {
                            if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = 0;
                            else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = -1;
                            else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = -1;
                            else *hit_word(ps, slot, kHdHitB) = -1;
                        }
                        if (kind == kRayShadow) ++nsh; else ++ncl;
                    }
                }
            }
        }
        const bool wantLeaf = active && leafPos < leafEnd;
        const uint64_t mLeaf = __ballot(wantLeaf);
        const uint64_t mNode = __ballot(active && !wantLeaf);
        if ((mLeaf | mNode) == 0) {
            if (exhausted) break;
            continue;
        }
        const uint32_t nLeaf = (uint32_t)__popcll(mLeaf);
        const bool leafStep = nLeaf > 0 && (mNode == 0 || nLeaf >= lmin);
        ++iters;
        bool done = false;
        if (leafStep) {
#pragma unroll
            for (int u = 0; u < kLeafSteps; ++u) {  // up to kLeafSteps primitive tests of the lane's leaf
                if (!(active && !done && leafPos < leafEnd)) continue;
                const int pi = leafPos++;
                ++prims;
                const float4 r0 = bprims[3 * pi];
                const float4 r1 = bprims[3 * pi + 1];
                const float4 r2 = bprims[3 * pi + 2];
                const uint32_t fl = __float_as_uint(r0.w);
                float t = 0;
                bool ok;
                if (fl & kPrimAnalytic) {
                    ok = shape_test<kSph>(sc, fl, __float_as_int(r1.w), ray, &t);
                } else {
                    ok = tri_hit(v3(r0.x, r0.y, r0.z), v3(r1.x, r1.y, r1.z), v3(r2.x, r2.y, r2.z), ray, sh, &t);
                    ok &= (kind == kRayShadow) | !(fl & kPrimDegenerate);
                }
                hitPrim = ok ? pi : hitPrim;
                ray.tmax = (ok && kind != kRayShadow) ? t : ray.tmax;
                done = ok && kind == kRayShadow;
                const bool leafDone = !done && leafPos == leafEnd;
                const int popv = stk[max(toVisit - 1, 0) * kTraceBlock];
                done |= leafDone && toVisit == 0;
                const bool pop = leafDone && toVisit > 0;
                cur = pop ? popv : cur;
                toVisit -= pop ? 1 : 0;
            }
        } else if (active && !wantLeaf) {
            // kNodeSteps node visits per loop iteration for lanes that stay in
            // node mode (the loop's refill / step-kind bookkeeping is paid once)
#pragma unroll
            for (int u = 0; u < kNodeSteps; ++u) {
                if (u > 0 && (done || leafPos < leafEnd)) continue;
                const bool go = true;
                const int c = cur;
                float4 a, b;
                if constexpr (kLdsScene) lds_node(bnodes, c, &a, &b);
                else { a = bnodes[2 * c]; b = bnodes[2 * c + 1]; }
                nodes += go ? 1u : 0u;
                const bool hit = node_box_hit(a, b, ray, inv, n0, n1, n2);
                const int off = __float_as_int(b.z);
                const uint32_t npax = __float_as_uint(b.w);
                const int np = (int)(npax & 0xffffu);
                const int axis = (int)(npax >> 16);
                const bool neg = axis == 0 ? n0 : (axis == 1 ? n1 : n2);
                const bool inner = go && hit && np == 0;
                const bool leaf = go && hit && np > 0;
                const bool miss = go && !hit;
                stk[toVisit * kTraceBlock] = neg ? c + 1 : off;  // push slot (kept only for an inner node)
                const int popv = stk[max(toVisit - 1, 0) * kTraceBlock];
                const bool pop = miss && toVisit > 0;
                done = go ? (miss && toVisit == 0) : done;
                cur = inner ? (neg ? off : c + 1) : (pop ? popv : c);
                toVisit += inner ? 1 : (pop ? -1 : 0);
                leafPos = leaf ? off : leafPos;
                leafEnd = leaf ? off + np : leafEnd;
            }
        }
        if (done) {
            if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = hitPrim >= 0 ? 1 : 0;
            else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = hitPrim;
            else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = hitPrim;
            else *hit_word(ps, slot, kHdHitB) = hitPrim;
            active = false;
        }
    }
    flush_stats(stats, ncl, nsh, nodes, prims);
    const unsigned long long it = wave_sum_u64(iters);
    if (lane == 0 && it) atomicAdd(&stats->lane_iters, it);
}
#else
;
#endif

// ----------------------------------------------------------------------------
// k_trace_lds: k_trace_nb for LDS-resident scenes with less work per node
// visit.  The traversal kernel is VALU-issue-bound (C2: ~64 VALU per node
// visit, about half of it bookkeeping around the box test), so:
//  * node records are re-encoded while staged: word 1 .w = primitivesOffset +
//    nPrimitives (the leaf's end) for a leaf, 0x80000000 | 1 << (16 + axis)
//    for an interior node -- "interior?" is a sign test, "the ray runs against
//    the split axis" one AND with the ray's direction sign bits (sgn); nodes
//    are named by LDS byte address (word 1 .z of an interior node = its second
//    child's), so the first child is +32 and a node load needs no address math;
//  * the stack pointer is the LDS byte address of the top entry (row 0 of the
//    lane's column is a dummy an empty stack's pop reads): a push writes 512
//    bytes above it, a pop reads it, together with the node's two loads;
//  * the slab updates are v_max / v_min (box_hit_mm).
// Same visit order, tests, tMax updates and counters as k_trace_nb.
// ----------------------------------------------------------------------------
// Bounds3::IntersectP (geometry.h:1584-1606) as max3 / min3 of the slab
// distances.  The reference's sequence -- reject if tMin > tyMax or tyMin >
// tMax, tMin = max, tMax = min, the same with z, then tMin < ray.tMax and
// tMax > 0 -- gives the same answer:
//  * with every distance a number, its two rejections are the six cross-axis
//    pairs of max(t0) <= min(t1); the three same-axis pairs t0 <= t1 can only
//    fail when that axis' far distance u is negative (t1 = u * gamma-scale <=
//    u), and then tMax <= t1 < 0 fails `tMax > 0` anyway;
//  * a NaN y / z distance constrains nothing there (its comparisons are false,
//    `if (tyMin > tMin)` keeps tMin) and max / min skip it the same way;
//  * a NaN x distance leaves the reference's tMin or tMax NaN to the end,
//    where `NaN < tMax` / `NaN > 0` fail: failed explicitly here.
// Signed zeros only meet comparisons.
__device__ __forceinline__ bool box_hit_mm(float4 a, float4 b, const Ray& ray, V3 inv, bool n0, bool n1, bool n2) {
    const float kx = 1 + 2 * gammaf(3);
    const float tx0 = ((n0 ? a.w : a.x) - ray.o.x) * inv.x;
    float tx1 = ((n0 ? a.x : a.w) - ray.o.x) * inv.x;
    const float ty0 = ((n1 ? b.x : a.y) - ray.o.y) * inv.y;
    float ty1 = ((n1 ? a.y : b.x) - ray.o.y) * inv.y;
    const float tz0 = ((n2 ? b.y : a.z) - ray.o.z) * inv.z;
    float tz1 = ((n2 ? a.z : b.y) - ray.o.z) * inv.z;
    tx1 *= kx;
    ty1 *= kx;
    tz1 *= kx;
    const float f0 = __builtin_fmaxf(__builtin_fmaxf(tx0, ty0), tz0);
    const float f1 = __builtin_fminf(__builtin_fminf(tx1, ty1), tz1);
    return !(f0 > f1) & (f0 < ray.tmax) & (f1 > 0) & !__builtin_isunordered(tx0, tx1);
}

static_assert(kTraceBlock * 4 == 512, "k_trace_lds stack rows are 512 bytes apart");
// 7 waves per SIMD (<= 72 VGPRs; the compiler's own choice lands at 74 = 6 waves)
#ifdef PT_TRACE_WAVES
#define PT_TRACE_LDS_ATTR __attribute__((amdgpu_waves_per_eu(PT_TRACE_WAVES)))
#else
#define PT_TRACE_LDS_ATTR __attribute__((amdgpu_waves_per_eu(kSph ? 1 : 7)))
#endif
// the node at LDS address addr (two ds_read_b128) and the stack's top entry, one wait
__device__ __forceinline__ void lds_node_top(uint32_t addr, uint32_t sp, float4* a, float4* b, int* top) {
    float4 x, y;
    int t;
    asm volatile(
        "ds_read_b128 %0, %3\n\tds_read_b128 %1, %3 offset:16\n\tds_read_b32 %2, %4\n\ts_waitcnt lgkmcnt(0)"
        : "=v"(x), "=v"(y), "=v"(t) : "v"(addr), "v"(sp) : "memory");
    *a = x;
    *b = y;
    *top = t;
}
__device__ __forceinline__ void lds_push(uint32_t sp, int v) {
    asm volatile("ds_write_b32 %0, %1 offset:512" : : "v"(sp), "v"(v) : "memory");
}
__device__ __forceinline__ int lds_top(uint32_t sp) {
    int t;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(sp) : "memory");
    return t;
}

template <bool kSph>
__global__ __launch_bounds__(kTraceBlock) PT_TRACE_LDS_ATTR void k_trace_lds(DevScene sc, DevPaths ps,
                                                                           const uint32_t* __restrict__ rq,
                                                                           const uint32_t* __restrict__ rq_count,
                                                                           uint32_t* fetch, int refill_min,
                                                                           int leaf_min, DevStats* stats)
#ifdef PT_TU_TRACE
{
    extern __shared__ float4 lds_dyn[];
    const int nn = 2 * sc.n_nodes;
    const int scene_f4 = nn + 3 * sc.n_prims;
    const uint32_t node0 = (uint32_t)(uintptr_t)lds_dyn;  // nodes are named by their LDS byte address
    for (int i = threadIdx.x; i < scene_f4; i += blockDim.x) {
        float4 v = i < nn ? sc.nodes[i] : sc.prims[i - nn];
        if (i < nn && (i & 1)) {  // (offset, nPrimitives | axis << 16) -> the encoding above
            const uint32_t npax = __float_as_uint(v.w);
            const uint32_t np = npax & 0xffffu;
            const uint32_t off = (uint32_t)__float_as_int(v.z);
            v.w = __uint_as_float(np ? off + np : 0x80000000u | (1u << (16 + (npax >> 16))));
            if (!np) v.z = __uint_as_float(node0 + 32u * off);  // second child: its LDS address
        }
        lds_dyn[i] = v;
    }
    __syncthreads();
    const float4* bprims = lds_dyn + nn;
    // the lane's stack column: row 0 the dummy, entry k (k >= 1) in row k
    const uint32_t sbase = (uint32_t)(uintptr_t)((int*)(lds_dyn + scene_f4) + threadIdx.x);
    const uint32_t n = *rq_count;
    const uint32_t rmin = (uint32_t)min(max(refill_min, 1), 64);  // idle lanes that trigger a refill
    const uint32_t lmin = (uint32_t)max(leaf_min, 1);             // parked lanes that trigger a leaf step
    const uint32_t lane = lane_id();
    uint32_t nrays = 0, nodes = 0, prims = 0;  // nrays: closest + shadow << 16
    unsigned long long iters_w = 0;  // wave total
    bool active = false, exhausted = false, drained = false;
    uint32_t qn = 0, qe = 0;
    uint32_t slot = 0, kind = 0;
    Ray ray{v3(0, 0, 0), v3(0, 0, 1), 0};
    V3 inv = v3(0, 0, 0);
    TriShear sh{0, 0, 0, 0};
    bool n0 = false, n1 = false, n2 = false;
    uint32_t sgn = 0, sp = sbase, cur = node0;
    int hitPrim = -1, leafPos = 0, leafEnd = 0;
    for (;;) {
        if (!exhausted) {
            const uint64_t idle = __ballot(!active);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (nidle >= rmin) {  // rmin in [1, 64]: one scalar compare
                if (qn >= qe && !drained) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(fetch, kTraceChunk);
                    base = __builtin_amdgcn_readlane(base, 0);  // the lane that did the atomic, whatever EXEC holds: in an SGPR
                    qn = base < n ? base : n;
                    qe = base + kTraceChunk < n ? base + kTraceChunk : n;
                    drained = base + kTraceChunk >= n;
                }
                const uint32_t take = qe - qn < nidle ? qe - qn : nidle;
                const uint32_t k = lanes_below(idle);
                const uint32_t i = qn + k;
                qn += take;
                if (drained && qn >= qe) exhausted = true;
                if (!active && k < take) {
                    const uint32_t e = rq[i];
                    slot = e >> 2;
                    kind = e & 3u;
                    ray = load_ray_trace(kind == kRayCont ? ps.ray : (kind == kRayB ? ps.rayB : ps.rayA), slot, kind == kRayShadow);
                    inv = v3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
                    sh = tri_shear(ray.d);
                    n0 = inv.x < 0; n1 = inv.y < 0; n2 = inv.z < 0;
                    sgn = (n0 ? 1u << 16 : 0u) | (n1 ? 1u << 17 : 0u) | (n2 ? 1u << 18 : 0u);
                    cur = node0; sp = sbase; hitPrim = -1; leafPos = 0; leafEnd = 0;
                    active = sc.n_nodes > 0;  // empty scene: every ray misses
                    if (!active) {
                        if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = 0;
                        else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = -1;
                        else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = -1;
                        else *hit_word(ps, slot, kHdHitB) = -1;
                    }
                    nrays += kind == kRayShadow ? 0x10000u : 1u;
                }
            }
        }
        const bool wantLeaf = active && leafPos < leafEnd;
        const uint64_t mLeaf = __ballot(wantLeaf);
        const uint64_t mNode = __ballot(active && !wantLeaf);
        if ((mLeaf | mNode) == 0) {
            if (exhausted) break;
            continue;
        }
        const uint32_t nLeaf = (uint32_t)__popcll(mLeaf);
        const bool leafStep = nLeaf > 0 && (mNode == 0 || nLeaf >= lmin);
        ++iters_w;
        bool done = false;
        if (leafStep) {
#pragma unroll
            for (int u = 0; u < kLeafSteps; ++u) {  // up to kLeafSteps primitive tests of the lane's leaf
                if (!(active && !done && leafPos < leafEnd)) continue;
                const int pi = leafPos++;
                ++prims;
                const float4 r0 = bprims[3 * pi];
                const float4 r1 = bprims[3 * pi + 1];
                const float4 r2 = bprims[3 * pi + 2];
                const uint32_t fl = __float_as_uint(r0.w);
                float t = 0;
                bool ok;
                if (fl & kPrimAnalytic) {
                    ok = shape_test<kSph>(sc, fl, __float_as_int(r1.w), ray, &t);
                } else {
                    ok = tri_hit(v3(r0.x, r0.y, r0.z), v3(r1.x, r1.y, r1.z), v3(r2.x, r2.y, r2.z), ray, sh, &t);
                    ok &= (kind == kRayShadow) | !(fl & kPrimDegenerate);
                }
                hitPrim = ok ? pi : hitPrim;
                ray.tmax = (ok && kind != kRayShadow) ? t : ray.tmax;
                done = ok && kind == kRayShadow;
                if (!done && leafPos == leafEnd) {  // the leaf is finished: pop
                    const bool empty = sp == sbase;
                    done = empty;
                    if (!empty) {
                        cur = (uint32_t)lds_top(sp);
                        sp -= 512;
                    }
                }
            }
        } else {
            // kNodeSteps node visits per loop iteration for lanes that stay in node mode.  One lane mask,
            // nm, tracks "still in node mode" (an interior node or a pop); done is derived once after the
            // steps -- left node mode without a leaf -- instead of being merged after every step
            const bool nm0 = active & (leafPos >= leafEnd);  // done is false here
            bool nm = nm0;
#pragma unroll
            for (int u = 0; u < kNodeSteps; ++u) {
                if (!nm) continue;
                ++nodes;
                float4 a, b;
                int top;
                lds_node_top(cur, sp, &a, &b, &top);
                const bool hit = box_hit_mm(a, b, ray, inv, n0, n1, n2);
                const uint32_t off = __float_as_uint(b.z);  // leaf: primitivesOffset; interior: second child
                const uint32_t w = __float_as_uint(b.w);
                const bool inner = hit & ((int)w < 0);
                const bool leaf = hit & ((int)w >= 0);
                const bool neg = (w & sgn) != 0;
                const bool empty = sp == sbase;
                lds_push(sp, (int)(neg ? cur + 32u : off));  // the far child (kept only for an interior node)
                const bool pop = !hit & !empty;
                nm = inner | pop;
                cur = inner ? (neg ? off : cur + 32u) : (pop ? (uint32_t)top : cur);
                sp = inner ? sp + 512 : (pop ? sp - 512 : sp);
                leafPos = leaf ? (int)off : leafPos;
                leafEnd = leaf ? (int)w : leafEnd;
            }
            done = nm0 & !nm & (leafPos >= leafEnd);  // the ray left the BVH: stack empty on a miss
        }
        if (done) {
            if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = hitPrim >= 0 ? 1 : 0;
            else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = hitPrim;
            else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = hitPrim;
            else *hit_word(ps, slot, kHdHitB) = hitPrim;
            active = false;
        }
    }
    flush_stats(stats, nrays & 0xffffu, nrays >> 16, nodes, prims);
    if (lane == 0 && iters_w) atomicAdd(&stats->lane_iters, 64ull * iters_w);
}
#else
;
#endif

// ----------------------------------------------------------------------------
// k_trace_oct: k_trace_lds over per-octant node images.  Every box test of the
// reference picks each slab's near and far plane by the ray's direction signs
// (Bounds3::IntersectP with dirIsNeg, geometry.h:1584-1606) and BVHAccel
// visits the near child first by the split axis' sign (bvh.cpp:700-712): both
// choices depend only on the ray's octant.  A block therefore stages the BVH
// eight times, once per octant, with each node's planes stored near/far and
// its children stored near/far, and a ray walks the image of its octant: the
// node step has no per-node selects, and each slab's two distances are one
// packed pair (v_pk_add_f32 / v_pk_mul_f32: the same IEEE operations on both
// halves, in the reference's order).  Node visits, primitive tests, tMax
// updates and the box test's answers (NaN slabs included, as box_hit_mm) are
// k_trace_lds's, so hits and counters are the reference's.
//
// Octant image node (32 B): {x_near, x_far, y_near, y_far} {z_near, z_far, Z, W}
//   interior: Z = LDS address of the near child, W = of the far child (same image)
//   leaf:     Z = 0x80000000 | primitive end, W = first primitive
// Blocks of kOctBlock threads (7 waves: four blocks fill a CU at 7 waves per
// SIMD) share one staging; the stack is k_trace_lds's LDS column of node
// addresses, rows kOctBlock * 4 B apart.
// ----------------------------------------------------------------------------
typedef float pt_f2 __attribute__((ext_vector_type(2)));
static_assert(kOctBlock * 4 == 1792, "k_trace_oct stack rows are 1792 bytes apart");
__device__ __forceinline__ void lds_push_oct(uint32_t sp, int v) {
    asm volatile("ds_write_b32 %0, %1 offset:1792" : : "v"(sp), "v"(v) : "memory");
}
// The box test of box_hit_mm on an octant image node: px/py/pz the slabs' (near,
// far) plane pairs, o / inv the ray's origin and reciprocal direction as splats
__device__ __forceinline__ bool box_hit_oct(pt_f2 px, pt_f2 py, pt_f2 pz, V3 o, V3 inv, float tmax) {
    const pt_f2 kx = {1.f, 1 + 2 * gammaf(3)};  // tMax *= 1 + 2 * gamma(3); the near distance times 1 exactly
    const pt_f2 tx = ((px - o.x) * inv.x) * kx;  // scalar operands splat to both halves
    const pt_f2 ty = ((py - o.y) * inv.y) * kx;
    const pt_f2 tz = ((pz - o.z) * inv.z) * kx;
    const float f0 = __builtin_fmaxf(__builtin_fmaxf(tx.x, ty.x), tz.x);
    const float f1 = __builtin_fminf(__builtin_fminf(tx.y, ty.y), tz.y);
    return !(f0 > f1) & (f0 < tmax) & (f1 > 0) & !__builtin_isunordered(tx.x, tx.y);
}

template <bool kSph>
__global__ __launch_bounds__(kOctBlock) __attribute__((amdgpu_waves_per_eu(kSph ? 1 : 7))) void k_trace_oct(
    DevScene sc, DevPaths ps, const uint32_t* __restrict__ rq, const uint32_t* __restrict__ rq_count,
    uint32_t* fetch, int refill_min, int leaf_min, DevStats* stats)
#ifdef PT_TU_TRACE
{
    extern __shared__ float4 lds_dyn[];
    const int nnodes = sc.n_nodes;
    const int img_f4 = 2 * nnodes;           // float4s of one octant image
    const int nprim_f4 = 3 * sc.n_prims;
    const uint32_t img0 = (uint32_t)(uintptr_t)lds_dyn;
    const uint32_t img_bytes = 32u * (uint32_t)nnodes;
    // the eight octant images, then the primitive records (as k_trace_lds)
    for (int i = threadIdx.x; i < 8 * nnodes; i += blockDim.x) {
        const int o = i / nnodes, k = i - o * nnodes;
        const float4 a = sc.nodes[2 * k], b = sc.nodes[2 * k + 1];
        const bool n0 = o & 1, n1 = (o >> 1) & 1, n2 = (o >> 2) & 1;
        // LinearBVHNode: a = {bmin.xyz, bmax.x}, b = {bmax.yz, offset, nPrimitives | axis << 16}
        float4 A, B;
        A.x = n0 ? a.w : a.x; A.y = n0 ? a.x : a.w;
        A.z = n1 ? b.x : a.y; A.w = n1 ? a.y : b.x;
        B.x = n2 ? b.y : a.z; B.y = n2 ? a.z : b.y;
        const uint32_t npax = __float_as_uint(b.w);
        const uint32_t np = npax & 0xffffu, axis = npax >> 16;
        const uint32_t off = (uint32_t)__float_as_int(b.z);
        const uint32_t base = img0 + (uint32_t)o * img_bytes;
        if (np > 0) {
            B.z = __uint_as_float(0x80000000u | (off + np));
            B.w = __uint_as_float(off);
        } else {
            const bool neg = (o >> axis) & 1;  // dirIsNeg[axis]: the second child first
            const uint32_t first = base + 32u * (uint32_t)(k + 1), second = base + 32u * off;
            B.z = __uint_as_float(neg ? second : first);
            B.w = __uint_as_float(neg ? first : second);
        }
        lds_dyn[(size_t)o * img_f4 + 2 * k] = A;
        lds_dyn[(size_t)o * img_f4 + 2 * k + 1] = B;
    }
    for (int i = threadIdx.x; i < nprim_f4; i += blockDim.x) lds_dyn[8 * img_f4 + i] = sc.prims[i];
    __syncthreads();
    const float4* bprims = lds_dyn + 8 * img_f4;
    // the lane's stack column: row 0 the dummy, entry k (k >= 1) in row k
    const uint32_t sbase = (uint32_t)(uintptr_t)((int*)(lds_dyn + 8 * img_f4 + nprim_f4) + threadIdx.x);
    const uint32_t n = *rq_count;
    const uint32_t rmin = (uint32_t)min(max(refill_min, 1), 64);  // idle lanes that trigger a refill
    const uint32_t lmin = (uint32_t)max(leaf_min, 1);             // parked lanes that trigger a leaf step
    const uint32_t lane = lane_id();
    uint32_t nrays = 0, nodes = 0, prims = 0;  // nrays: closest + shadow << 16
    unsigned long long iters_w = 0;
    bool active = false, exhausted = false, drained = false;
    uint32_t qn = 0, qe = 0;
    uint32_t slot = 0, kind = 0;
    Ray ray{v3(0, 0, 0), v3(0, 0, 1), 0};
    V3 inv = v3(0, 0, 0);
    TriShear sh{0, 0, 0, 0};
    uint32_t sp = sbase, cur = img0;
    int hitPrim = -1, leafPos = 0, leafEnd = 0;
    for (;;) {
        if (!exhausted) {
            const uint64_t idle = __ballot(!active);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (nidle >= rmin) {  // rmin in [1, 64]: one scalar compare
                if (qn >= qe && !drained) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(fetch, kTraceChunk);
                    base = __builtin_amdgcn_readlane(base, 0);  // the lane that did the atomic, whatever EXEC holds: in an SGPR
                    qn = base < n ? base : n;
                    qe = base + kTraceChunk < n ? base + kTraceChunk : n;
                    drained = base + kTraceChunk >= n;
                }
                const uint32_t take = qe - qn < nidle ? qe - qn : nidle;
                const uint32_t k = lanes_below(idle);
                const uint32_t i = qn + k;
                qn += take;
                if (drained && qn >= qe) exhausted = true;
                if (!active && k < take) {
                    const uint32_t e = rq[i];
                    slot = e >> 2;
                    kind = e & 3u;
                    ray = load_ray_trace(kind == kRayCont ? ps.ray : (kind == kRayB ? ps.rayB : ps.rayA), slot, kind == kRayShadow);
                    inv = v3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
                    sh = tri_shear(ray.d);
                    const uint32_t oct = (inv.x < 0 ? 1u : 0u) | (inv.y < 0 ? 2u : 0u) | (inv.z < 0 ? 4u : 0u);
                    cur = img0 + oct * img_bytes; sp = sbase; hitPrim = -1; leafPos = 0; leafEnd = 0;
                    active = nnodes > 0;  // empty scene: every ray misses
                    if (!active) {
                        if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = 0;
                        else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = -1;
                        else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = -1;
                        else *hit_word(ps, slot, kHdHitB) = -1;
                    }
                    nrays += kind == kRayShadow ? 0x10000u : 1u;
                }
            }
        }
        const bool wantLeaf = active && leafPos < leafEnd;
        const uint64_t mLeaf = __ballot(wantLeaf);
        const uint64_t mNode = __ballot(active && !wantLeaf);
        if ((mLeaf | mNode) == 0) {
            if (exhausted) break;
            continue;
        }
        const uint32_t nLeaf = (uint32_t)__popcll(mLeaf);
        const bool leafStep = nLeaf > 0 && (mNode == 0 || nLeaf >= lmin);
        ++iters_w;
        bool done = false;
        if (leafStep) {
#pragma unroll
            for (int u = 0; u < kLeafSteps; ++u) {  // up to kLeafSteps primitive tests of the lane's leaf
                if (!(active && !done && leafPos < leafEnd)) continue;
                const int pi = leafPos++;
                ++prims;
                const float4 r0 = bprims[3 * pi];
                const float4 r1 = bprims[3 * pi + 1];
                const float4 r2 = bprims[3 * pi + 2];
                const uint32_t fl = __float_as_uint(r0.w);
                float t = 0;
                bool ok;
                if (fl & kPrimAnalytic) {
                    ok = shape_test<kSph>(sc, fl, __float_as_int(r1.w), ray, &t);
                } else {
                    ok = tri_hit(v3(r0.x, r0.y, r0.z), v3(r1.x, r1.y, r1.z), v3(r2.x, r2.y, r2.z), ray, sh, &t);
                    ok &= (kind == kRayShadow) | !(fl & kPrimDegenerate);
                }
                hitPrim = ok ? pi : hitPrim;
                ray.tmax = (ok && kind != kRayShadow) ? t : ray.tmax;
                done = ok && kind == kRayShadow;
                if (!done && leafPos == leafEnd) {  // the leaf is finished: pop
                    const bool empty = sp == sbase;
                    done = empty;
                    if (!empty) {
                        cur = (uint32_t)lds_top(sp);
                        sp -= 1792;
                    }
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < kNodeSteps; ++u) {
                if (!(active && !done && leafPos >= leafEnd)) continue;
                ++nodes;
                float4 a, b;
                int top;
                lds_node_top(cur, sp, &a, &b, &top);
                const bool hit = box_hit_oct(pt_f2{a.x, a.y}, pt_f2{a.z, a.w}, pt_f2{b.x, b.y}, ray.o, inv, ray.tmax);
                const int Z = __float_as_int(b.z);
                const uint32_t W = __float_as_uint(b.w);
                const bool inner = hit & (Z >= 0);
                const bool leaf = hit & (Z < 0);
                const bool empty = sp == sbase;
                lds_push_oct(sp, (int)W);  // the far child (kept only for an interior node)
                done = !hit & empty;
                const bool pop = !hit & !empty;
                cur = inner ? (uint32_t)Z : (pop ? (uint32_t)top : cur);
                sp = inner ? sp + 1792 : (pop ? sp - 1792 : sp);
                leafPos = leaf ? (int)W : leafPos;
                leafEnd = leaf ? (Z & 0x7fffffff) : leafEnd;
            }
        }
        if (done) {
            if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = hitPrim >= 0 ? 1 : 0;
            else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = hitPrim;
            else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = hitPrim;
            else *hit_word(ps, slot, kHdHitB) = hitPrim;
            active = false;
        }
    }
    flush_stats(stats, nrays & 0xffffu, nrays >> 16, nodes, prims);
    if (lane == 0 && iters_w) atomicAdd(&stats->lane_iters, 64ull * iters_w);
}
#else
;
#endif

// ----------------------------------------------------------------------------
// k_trace_w: LDS-resident scenes traversed over a 4-wide BVH (round 6).
//
// The host collapses the reference's binary LinearBVHNode tree (bvh.cpp:640-658)
// into nodes of up to four children (render.hip build_wide): a child is a binary
// node of the original tree with its exact bounds -- an interior one becomes
// another wide node, a leaf keeps its primitive range.  A node step loads the
// four child boxes (7 x ds_read_b128), tests all four with the reference's box
// test (Bounds3::IntersectP, geometry.h:1584-1606, the near / far planes picked
// by address from the ray's direction signs), pushes the hit children farthest
// first and continues at the nearest: about three dependent LDS round trips per
// C2 ray instead of the binary walk's ~15.
//
// Same answers as BVHAccel::Intersect / IntersectP (bvh.cpp:662-738):
//  * any-hit: the box test is monotone in the box (IEEE rounding is monotone,
//    a parent's bounds contain its children's), so a primitive's leaf box passes
//    only if every binary ancestor's does, and each leaf box is tested exactly:
//    the primitives reached are the reference's and occlusion is order-free;
//  * closest hit: the reference keeps the LAST accepted primitive, accepted
//    against a tMax that shrinks in its visit order (Triangle::Intersect's
//    scaled test, triangle.cpp:259-261; AAPlaneShape's `t < tMax` in the plane's
//    object space, whose origin the Transform moved forward by its error bound,
//    transform.h:303-316, plane.cpp:15-55), and culls boxes against it.  Every
//    such t carries rounding errors of a few ulps of t plus absolute errors of
//    order 10 eps x the coordinates involved at non-grazing incidence (pbrt's
//    own deltaT bound, triangle.cpp:362-385; the transformed origin's shift).
//    So primitives are accepted against T = tBest + |tBest| 2^-17 + 2A, with
//    A = 2^-18 R (R = the scene's largest |coordinate| + the origin's: 64 eps R,
//    several times those errors), and boxes culled against T + 30A; the smallest
//    t wins and every other accepted t goes to t2.  When no other primitive is
//    accepted within W = tBest + |tBest| 2^-18 + A, the margins exceed the
//    error bounds and the winner is the only primitive the reference can keep
//    whatever its order;
//    otherwise -- a near tie, a hit at t <= 0 (aaplane: no t > 0 test), a NaN
//    t, or a ray with an infinite 1/d component (NaN slabs) -- the ray goes to
//    a retrace queue that the binary k_trace_lds traverses in the reference's
//    order right after this launch.  The one case no margin covers is a
//    triangle whose computed t lies more than 32A = 2^-13 R below its own leaf
//    box's entry distance (incidence within a few mrad of grazing AND a box
//    that starts beyond the winner, where the reference's own answer turns on
//    its visit order).  Its node / primitive
//    counters are not produced (the binary build runs for the counting frame,
//    pt_set_count_bytes).
//
// Wide node image (112 B, 16-B aligned): {lo.x of children 0-3} {hi.x} {lo.y}
// {hi.y} {lo.z} {hi.z} {child words}; a child word is 0x80000000 | the LDS byte
// address of a wide node, or first primitive | count << 24 for a leaf; unused
// slots have inverted bounds (+inf / -inf: never hit) and word 0.
// ----------------------------------------------------------------------------
// the acceptance / culling bound T and the tie window W around the best t (a: the ray's absolute margin A)
__device__ __forceinline__ float wide_accept(float t, float a) { return t + fabsf(t) * (1.0f / 131072.0f) + 2 * a; }
__device__ __forceinline__ float wide_tie(float t, float a) { return t + fabsf(t) * (1.0f / 262144.0f) + a; }

// the wide node at cur (its six plane quads picked by the ray's direction signs: near x at cur + ax, far x at
// cur + 16 - ax, ...) and the stack's top entry, one wait
__device__ __forceinline__ void lds_wnode_top(uint32_t cur, uint32_t axyz, uint32_t sp, float4* nx, float4* fx,
                                              float4* ny, float4* fy, float4* nz, float4* fz, uint4* wd,
                                              uint32_t* top) {
    const uint32_t c16 = cur + 16u;
    const uint32_t ax = axyz & 0xffu, ay = (axyz >> 8) & 0xffu, az = axyz >> 16;
    float4 a, b, c, d, e, f;
    uint4 g;
    uint32_t t;
    asm volatile(
        "ds_read_b128 %0, %8\n\t"
        "ds_read_b128 %1, %9\n\t"
        "ds_read_b128 %2, %10 offset:32\n\t"
        "ds_read_b128 %3, %11 offset:32\n\t"
        "ds_read_b128 %4, %12 offset:64\n\t"
        "ds_read_b128 %5, %13 offset:64\n\t"
        "ds_read_b128 %6, %14 offset:96\n\t"
        "ds_read_b32 %7, %15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d), "=&v"(e), "=&v"(f), "=&v"(g), "=&v"(t)
        : "v"(cur + ax), "v"(c16 - ax), "v"(cur + ay), "v"(c16 - ay), "v"(cur + az), "v"(c16 - az), "v"(cur),
          "v"(sp)
        : "memory");
    *nx = a; *fx = b; *ny = c; *fy = d; *nz = e; *fz = f; *wd = g; *top = t;
}
__device__ __forceinline__ void lds_write1(uint32_t a, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" : : "v"(a), "v"(v) : "memory");
}
// three entries above the top (the node step's pushes; rows past the new top are dead)
__device__ __forceinline__ void lds_push3(uint32_t sp, uint32_t a, uint32_t b, uint32_t c) {
    asm volatile("ds_write_b32 %0, %1 offset:512\n\tds_write_b32 %0, %2 offset:1024\n\tds_write_b32 %0, %3 offset:1536"
                 : : "v"(sp), "v"(a), "v"(b), "v"(c) : "memory");
}

// The reference's box test (box_hit_mm without its NaN-slab term: a ray with an infinite 1/d component is
// retraced by the binary kernel) for two children at once: p*/q* their near / far planes, packed.
struct WideHit2 {
    pt_f2 f0;
    bool h0, h1;
};
// ix / iy / iz: 1/d splatted to both halves (kept per ray: built per step, the splats went through scratch)
__device__ __forceinline__ WideHit2 wide_box2(pt_f2 nx, pt_f2 fx, pt_f2 ny, pt_f2 fy, pt_f2 nz, pt_f2 fz, pt_f2 ox,
                                              pt_f2 oy, pt_f2 oz, pt_f2 ix, pt_f2 iy, pt_f2 iz, float tc) {
    const float kx = 1 + 2 * gammaf(3);
    const pt_f2 tx0 = (nx - ox) * ix, tx1 = ((fx - ox) * ix) * kx;
    const pt_f2 ty0 = (ny - oy) * iy, ty1 = ((fy - oy) * iy) * kx;
    const pt_f2 tz0 = (nz - oz) * iz, tz1 = ((fz - oz) * iz) * kx;
    WideHit2 r;
    r.f0.x = __builtin_fmaxf(__builtin_fmaxf(tx0.x, ty0.x), tz0.x);
    r.f0.y = __builtin_fmaxf(__builtin_fmaxf(tx0.y, ty0.y), tz0.y);
    const float f1a = __builtin_fminf(__builtin_fminf(tx1.x, ty1.x), tz1.x);
    const float f1b = __builtin_fminf(__builtin_fminf(tx1.y, ty1.y), tz1.y);
    r.h0 = !(r.f0.x > f1a) & (r.f0.x < tc) & (f1a > 0);
    r.h1 = !(r.f0.y > f1b) & (r.f0.y < tc) & (f1b > 0);
    return r;
}

// wide-node steps per loop iteration for lanes that stay in node mode (C2: 1 / 2 / 3 -> 8.88 / 8.54 / 8.39 ms
// per launch)
#ifndef PT_WNODE_STEPS
#define PT_WNODE_STEPS 3
#endif
constexpr int kWNodeSteps = PT_WNODE_STEPS;
// 6 waves per SIMD (80 VGPRs, no scratch; the compiler's own choice is 82 = 5 waves, and 7 waves spill 40 B)
#ifdef PT_TRACE_W_WAVES
#define PT_TRACE_W_ATTR __attribute__((amdgpu_waves_per_eu(PT_TRACE_W_WAVES)))
#else
#define PT_TRACE_W_ATTR __attribute__((amdgpu_waves_per_eu(6)))
#endif
constexpr uint32_t kWideStrideLds = 112;  // LDS image: 7 x 16 B per wide node
constexpr uint32_t kWideStrideHbm = 128;  // HBM image: one 128-B line per wide node (7 x 16 B + 16 B pad)

// The HBM image's node loads (k_trace_w<true>): the six plane quads picked by the ray's direction signs and the
// child words, as buffer loads at 32-bit byte offsets from the image base (one 128-B line per node)
__device__ __forceinline__ void hbm_wnode(__amdgpu_buffer_rsrc_t img, uint32_t cur, uint32_t axyz, float4* nx,
                                          float4* fx, float4* ny, float4* fy, float4* nz, float4* fz, uint4* wd) {
    const uint32_t ax = axyz & 0xffu, ay = (axyz >> 8) & 0xffu, az = axyz >> 16;
    auto ld = [&](uint32_t off) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(img, (int)off, 0, 0);
        return __builtin_bit_cast(float4, v);
    };
    *nx = ld(cur + ax);
    *fx = ld(cur + 16u - ax);
    *ny = ld(cur + 32u + ay);
    *fy = ld(cur + 48u - ay);
    *nz = ld(cur + 64u + az);
    *fz = ld(cur + 80u - az);
    *wd = __builtin_bit_cast(uint4, ld(cur + 96u));
}

// k_trace_w<kHbm>: kHbm = false stages the 112-B-node image and the primitive records in LDS (C2-C4);
// kHbm = true reads the 128-B-node image and the records from HBM (C5's ten million primitives), with the
// stack in `stack_rows` LDS rows per lane and its deeper entries in a per-lane global spill column.
template <bool kHbm>
__global__ __launch_bounds__(kTraceBlock) PT_TRACE_W_ATTR void k_trace_w(DevScene sc, DevPaths ps,
                                                                        const uint32_t* __restrict__ rq,
                                                                        const uint32_t* __restrict__ rq_count,
                                                                        uint32_t* fetch, int refill_min, int leaf_min,
                                                                        uint32_t* retrace_q, uint32_t* retrace_n,
                                                                        int stack_rows, uint32_t* spill,
                                                                        DevStats* stats)
#ifdef PT_TU_TRACE
{
    extern __shared__ float4 lds_dyn[];
    const int nw = kHbm ? 0 : 7 * sc.n_wnodes;
    const int scene_f4 = kHbm ? 0 : nw + 3 * sc.n_prims;
    const uint32_t node0 = kHbm ? 0u : (uint32_t)(uintptr_t)lds_dyn;  // LDS: wide nodes named by LDS byte address
    if constexpr (!kHbm) {
        for (int i = threadIdx.x; i < scene_f4; i += blockDim.x) {
            float4 v = i < nw ? sc.wnodes[i] : sc.prims[i - nw];
            if (i < nw && i % 7 == 6) {  // child words: image offsets -> LDS addresses
                uint32_t w[4] = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                                 __float_as_uint(v.w)};
                for (int k = 0; k < 4; ++k)
                    if ((int)w[k] < 0) w[k] = 0x80000000u | (node0 + (w[k] & 0x7fffffffu));
                v = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]),
                                __uint_as_float(w[3]));
            }
            lds_dyn[i] = v;
        }
        __syncthreads();
    }
    const float4* bprims = kHbm ? sc.prims : lds_dyn + nw;
    // the HBM image as a buffer resource (gfx9 dword 3: 32-bit data format), one per launch
    const __amdgpu_buffer_rsrc_t img = __builtin_amdgcn_make_buffer_rsrc((void*)sc.wnodes, (short)0, 0x7fffffff,
                                                                        0x00020000);
    // the lane's stack column: row 0 the dummy, entry k (k >= 1) in row k (LDS byte addresses, rows 512 B apart);
    // kHbm: rows from `stack_rows` on live in the lane's spill column (entry k at spill[col + k - stack_rows])
    const uint32_t sbase = (uint32_t)(uintptr_t)((uint32_t*)(lds_dyn + scene_f4) + threadIdx.x);
    // the LDS rows' end and the spill column, recomputed where used (registers: the 6-wave budget)
    const uint32_t srows = 512u * (uint32_t)stack_rows;
#define PT_SLIM (sbase + srows)
#define PT_SCOL (spill + (size_t)(blockIdx.x * (uint32_t)kTraceBlock + threadIdx.x) * (uint32_t)kSpillWords)
    auto srow = [&](uint32_t a) { return (a - PT_SLIM) >> 9; };  // spill index of a stack address past the LDS rows
    const uint32_t n = *rq_count;
    const uint32_t rmin = (uint32_t)min(max(refill_min, 1), 64);  // idle lanes that trigger a refill
    const uint32_t lmin = (uint32_t)max(leaf_min, 1);             // parked lanes that trigger a leaf step
    const uint32_t lane = lane_id();
    uint32_t nrays = 0, wnp = 0;  // nrays: closest + shadow << 16; wnp: wide nodes + prim tests << 16
    unsigned long long iters_w = 0;
    bool active = false, exhausted = false, drained = false, retr = false;
    uint32_t qn = 0, qe = 0;
    uint32_t ent = 0;  // the ray-queue entry: slot << 2 | kind
    // the ray: its origin and 1/d splatted to both halves of a pair (the packed box tests' operands; .x the
    // scalar), the bound T; the direction itself is reloaded only for analytic shapes (aaplane tests)
    pt_f2 ox = {0, 0}, oy = {0, 0}, oz = {0, 0}, ix = {0, 0}, iy = {0, 0}, iz = {0, 0};
    float tmx = 0;
    TriShear sh{0, 0, 0, 0};
    uint32_t axyz = 0, sp = sbase, cur = node0;  // axyz: the near planes' offsets per axis (bytes 0-2: 0 / 16)
    float tBest = kInf, t2 = kInf;  // closest accepted t and the smallest other accepted t
    int hitPrim = -1;
    uint32_t lf = 0;  // the leaf being tested: next primitive | primitives left << 24 (a leaf child word)
    for (;;) {
        if (!exhausted) {
            const uint64_t idle = __ballot(!active);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (nidle >= rmin) {
                if (qn >= qe && !drained) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(fetch, kTraceChunk);
                    base = __builtin_amdgcn_readlane(base, 0);
                    qn = base < n ? base : n;
                    qe = base + kTraceChunk < n ? base + kTraceChunk : n;
                    drained = base + kTraceChunk >= n;
                }
                const uint32_t take = qe - qn < nidle ? qe - qn : nidle;
                const uint32_t k = lanes_below(idle);
                const uint32_t i = qn + k;
                qn += take;
                if (drained && qn >= qe) exhausted = true;
                if (!active && k < take) {
                    const uint32_t e = rq[i];
                    ent = e;
                    const uint32_t slot = e >> 2, kind = e & 3u;
                    const Ray ray = load_ray_trace(kind == kRayCont ? ps.ray : (kind == kRayB ? ps.rayB : ps.rayA),
                                                   slot, kind == kRayShadow);
                    ox = pt_f2{ray.o.x, ray.o.x};
                    oy = pt_f2{ray.o.y, ray.o.y};
                    oz = pt_f2{ray.o.z, ray.o.z};
                    tmx = ray.tmax;
                    const V3 inv = v3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
                    ix = pt_f2{inv.x, inv.x};
                    iy = pt_f2{inv.y, inv.y};
                    iz = pt_f2{inv.z, inv.z};
                    sh = tri_shear(ray.d);
                    axyz = (inv.x < 0 ? 16u : 0u) | (inv.y < 0 ? 16u << 8 : 0u) | (inv.z < 0 ? 16u << 16 : 0u);
                    // NaN slabs (0 * inf) only arise with an infinite 1/d component: the binary kernel's case
                    retr = !(__builtin_fmaxf(__builtin_fmaxf(fabsf(inv.x), fabsf(inv.y)), fabsf(inv.z)) < kInf);
                    cur = node0; sp = sbase; hitPrim = -1; lf = 0;
                    tBest = kInf; t2 = kInf;
                    active = sc.n_wnodes > 0;  // empty scene: every ray misses
                    if (!active) {
                        if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = 0;
                        else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = -1;
                        else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = -1;
                        else *hit_word(ps, slot, kHdHitB) = -1;
                        nrays += kind == kRayShadow ? 0x10000u : 1u;
                    }
                }
            }
        }
        const bool wantLeaf = active && lf >= (1u << 24);
        const uint64_t mLeaf = __ballot(wantLeaf);
        const uint64_t mNode = __ballot(active && !wantLeaf);
        if ((mLeaf | mNode) == 0) {
            if (exhausted) break;
            continue;
        }
        const uint32_t nLeaf = (uint32_t)__popcll(mLeaf);
        const bool leafStep = nLeaf > 0 && (mNode == 0 || nLeaf >= lmin);
        ++iters_w;
        bool done = false;
        const bool shadow = (ent & 3u) == kRayShadow;
        // the ray's absolute margin A (not kept: one register less)
        const float amarg = (sc.wide_scale + __builtin_fmaxf(__builtin_fmaxf(fabsf(ox.x), fabsf(oy.x)), fabsf(oz.x))) *
                            (1.0f / 262144.0f);
        if (leafStep) {
#pragma unroll
            for (int u = 0; u < kLeafSteps; ++u) {  // up to kLeafSteps primitive tests of the lane's leaf
                if (!(active && !done && lf >= (1u << 24))) continue;
                const int pi = (int)(lf & 0xffffffu);
                lf += 1u - (1u << 24);
                wnp += 0x10000u;
                const float4 r0 = bprims[3 * pi];
                const float4 r1 = bprims[3 * pi + 1];
                const float4 r2 = bprims[3 * pi + 2];
                const uint32_t fl = __float_as_uint(r0.w);
                float t = 0;
                bool ok;
                if (fl & kPrimAnalytic) {
                    const uint32_t kd = ent & 3u;
                    Ray ray = load_ray_trace(kd == kRayCont ? ps.ray : (kd == kRayB ? ps.rayB : ps.rayA), ent >> 2,
                                             false);
                    ray.tmax = tmx;
                    ok = shape_test<false>(sc, fl, __float_as_int(r1.w), ray, &t);
                } else {
                    const Ray ray{v3(ox.x, oy.x, oz.x), v3(0, 0, 0), tmx};  // tri_hit reads o and tMax (+ the shear)
                    ok = tri_hit(v3(r0.x, r0.y, r0.z), v3(r1.x, r1.y, r1.z), v3(r2.x, r2.y, r2.z), ray, sh, &t);
                    ok &= shadow | !(fl & kPrimDegenerate);
                }
                if (shadow) {
                    hitPrim = ok ? pi : hitPrim;
                    done = ok;
                } else if (ok) {
                    const bool better = !(t >= tBest);  // a NaN t is kept (and retraced below)
                    t2 = __builtin_fminf(t2, better ? tBest : t);
                    tBest = better ? t : tBest;
                    hitPrim = better ? pi : hitPrim;
                    tmx = better ? wide_accept(t, amarg) : tmx;
                }
                if (!done && lf < (1u << 24)) {  // the leaf is finished: pop
                    const bool empty = sp == sbase;
                    done = empty;
                    if (!empty) {
                        uint32_t w;
                        if (!kHbm || sp < PT_SLIM) w = (uint32_t)lds_top(sp);
                        else w = PT_SCOL[srow(sp)];
                        sp -= 512;
                        const bool inner = (int)w < 0;
                        cur = inner ? (w & 0x7fffffffu) : cur;
                        lf = inner ? 0u : w;
                    }
                }
            }
        } else {
            const bool nm0 = active & (lf < (1u << 24));
            bool nm = nm0;
#pragma unroll
            for (int u = 0; u < kWNodeSteps; ++u) {
                if (!nm) continue;
                ++wnp;
                float4 nx, fx, ny, fy, nz, fz;
                uint4 wd;
                uint32_t top;
                if constexpr (kHbm) {
                    hbm_wnode(img, cur, axyz, &nx, &fx, &ny, &fy, &nz, &fz, &wd);
                    top = sp < PT_SLIM ? (uint32_t)lds_top(sp) : PT_SCOL[srow(sp)];
                } else {
                    lds_wnode_top(cur, axyz, sp, &nx, &fx, &ny, &fy, &nz, &fz, &wd, &top);
                }
                // box cull: T + 30A for closest-hit rays, a shadow ray's own tMax (any-hit: the reference's set)
                const float tc = shadow ? tmx : tmx + 30 * amarg;
                const WideHit2 h01 = wide_box2(pt_f2{nx.x, nx.y}, pt_f2{fx.x, fx.y}, pt_f2{ny.x, ny.y},
                                               pt_f2{fy.x, fy.y}, pt_f2{nz.x, nz.y}, pt_f2{fz.x, fz.y}, ox, oy, oz,
                                               ix, iy, iz, tc);
                const WideHit2 h23 = wide_box2(pt_f2{nx.z, nx.w}, pt_f2{fx.z, fx.w}, pt_f2{ny.z, ny.w},
                                               pt_f2{fy.z, fy.w}, pt_f2{nz.z, nz.w}, pt_f2{fz.z, fz.w}, ox, oy, oz,
                                               ix, iy, iz, tc);
                // sort keys: a hit child's entry distance (> -inf), a missed one -inf; descending, so the hits
                // come first, farthest to nearest
                const float kHitMin = -3.40282347e38f;
                float k0 = h01.h0 ? __builtin_fmaxf(h01.f0.x, kHitMin) : -kInf;
                float k1 = h01.h1 ? __builtin_fmaxf(h01.f0.y, kHitMin) : -kInf;
                float k2 = h23.h0 ? __builtin_fmaxf(h23.f0.x, kHitMin) : -kInf;
                float k3 = h23.h1 ? __builtin_fmaxf(h23.f0.y, kHitMin) : -kInf;
                uint32_t w0 = wd.x, w1 = wd.y, w2 = wd.z, w3 = wd.w;
#define PT_WCAS(a, b)                                   \
    {                                                   \
        const bool s_ = k##a < k##b;                    \
        const float ka_ = s_ ? k##b : k##a;             \
        k##b = s_ ? k##a : k##b;                        \
        k##a = ka_;                                     \
        const uint32_t wa_ = s_ ? w##b : w##a;          \
        w##b = s_ ? w##a : w##b;                        \
        w##a = wa_;                                     \
    }
                PT_WCAS(0, 1) PT_WCAS(2, 3) PT_WCAS(0, 2) PT_WCAS(1, 3) PT_WCAS(1, 2)
#undef PT_WCAS
                const uint32_t nh = (uint32_t)h01.h0 + (uint32_t)h01.h1 + (uint32_t)h23.h0 + (uint32_t)h23.h1;
                // the hits but the nearest, farthest first (rows past the new top are dead)
                if (!kHbm || sp + 1536u < PT_SLIM) {
                    lds_push3(sp, w0, w1, w2);
                } else {  // the spill's edge: entry by entry
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        const uint32_t a = sp + 512u * (uint32_t)(q + 1), v = q == 0 ? w0 : (q == 1 ? w1 : w2);
                        if (a < PT_SLIM) lds_write1(a, v);
                        else if (srow(a) < (uint32_t)kSpillWords) PT_SCOL[srow(a)] = v;
                    }
                }
                // the nearest hit w[nh - 1] (or the popped top) as three selects: the compiler turned the
                // nested conditional into branches (-13 SALU and 2 branches per node step)
                const bool go = (nh > 0) | (sp != sbase);
                const uint32_t s01 = nh >= 2u ? w1 : w0, s23 = nh >= 4u ? w3 : w2;
                const uint32_t sn = nh >= 3u ? s23 : s01;
                const uint32_t nxt = nh == 0u ? top : sn;
                sp = nh > 0 ? sp + 512u * (nh - 1u) : (go ? sp - 512u : sp);
                const bool inner = go & ((int)nxt < 0);
                const bool leaf = go & ((int)nxt >= 0);
                nm = inner;
                cur = inner ? (nxt & 0x7fffffffu) : cur;
                lf = leaf ? nxt : lf;
            }
            done = nm0 & !nm & (lf < (1u << 24));  // left the BVH: a miss with an empty stack
        }
        if (done) {
            const uint32_t slot = ent >> 2, kind = ent & 3u;
            // closest hit: retrace near ties (another accepted t within W) and hits at t <= 0 / NaN
            const bool tie = !shadow && hitPrim >= 0 && (!(tBest > 0) || t2 <= wide_tie(tBest, amarg));
            if (retr || tie) {  // counted by the retrace launch (its own DevStats)
                retrace_q[atomicAdd(retrace_n, 1u)] = ent;
            } else {
                if (kind == kRayShadow) *hit_word(ps, slot, kHdHitA) = hitPrim >= 0 ? 1 : 0;
                else if (kind == kRayCont) *hit_word(ps, slot, kHdHit) = hitPrim;
                else if (kind == kRayA) *hit_word(ps, slot, kHdHitA) = hitPrim;
                else *hit_word(ps, slot, kHdHitB) = hitPrim;
                nrays += kind == kRayShadow ? 0x10000u : 1u;
            }
            active = false;
        }
    }
    flush_stats(stats, nrays & 0xffffu, nrays >> 16, 0, 0);
    {
        const unsigned long long a = wave_sum_u64(wnp & 0xffffu), b = wave_sum_u64(wnp >> 16);
        if (lane == 0) {
            if (a) atomicAdd(&stats->wnodes, a);
            if (b) atomicAdd(&stats->wprims, b);
            if (iters_w) atomicAdd(&stats->lane_iters, 64ull * iters_w);
        }
    }
#undef PT_SLIM
#undef PT_SCOL
}
#else
;
#endif

// ----------------------------------------------------------------------------
// Camera rays: GetCameraSample (sampler.cpp:46-53) + GenerateRayDifferential
// (perspective.cpp:100-154) + CameraToWorld (transform.h:251-264)
// ----------------------------------------------------------------------------
__device__ __forceinline__ Ray camera_ray(const DevScene& sc, float fx, float fy, float lx, float ly) {
    V3 pc = xf_point(sc.r2c, v3(fx, fy, 0));
    Ray r{v3(0, 0, 0), normalize(v3(pc.x, pc.y, pc.z)), kInf};
    if (sc.lens_radius > 0) {
        float dx, dy;
        concentric_sample_disk(lx, ly, &dx, &dy);
        float plx = sc.lens_radius * dx, ply = sc.lens_radius * dy;
        float ft = sc.focal_distance / r.d.z;
        V3 pFocus = r.o + r.d * ft;
        r.o = v3(plx, ply, 0);
        r.d = normalize(pFocus - r.o);
    }
    return xf_ray(sc.c2w, r);
}

// FilmMeta (kernels.h) of one axis: film pixel q + o - win for o = 0..2win against
// AddSample's bounds and filter-table index (film.h:121-161) -- k_film's
// expressions on the same pFilm coordinate
__device__ __forceinline__ uint32_t film_meta_axis(float f, int q, int win, float r, float inv_r) {
    const float d = f - 0.5f;
    const int t0 = (int)ceilf(d - r), t1 = (int)floorf(d + r) + 1;
    uint32_t m = 0;
    for (int o = 0; o <= 2 * win; ++o) {
        const int t = q + o - win;
        if (t < t0 || t >= t1) continue;
        int i = (int)floorf(fabsf((t - d) * inv_r * 16));
        i = i < 15 ? i : 15;
        m |= (uint32_t)i << (4 * o) | 1u << (20 + o);
    }
    return m;
}

template <bool kMeta>  // FilmMeta records (k_film_sk) instead of pFilm
__global__ __launch_bounds__(256) void k_camera(DevScene sc, DevPaths ps, const int2* __restrict__ pix, int npix,
                                                int s0, int nsamp, HaltonPixelConsts hp, uint32_t* rq,
                                                uint32_t* pq, FilmMeta fm)
#ifdef PT_TU_MISC
{
    const uint32_t N = (uint32_t)ps.n;
    const uint32_t total = (uint32_t)npix * (uint32_t)nsamp;
    for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < total; slot += gridDim.x * blockDim.x) {
        // pixel-major: a pixel's samples are consecutive slots (k_film loads them coalesced)
        const uint32_t p = slot / (uint32_t)nsamp, sl = slot - p * (uint32_t)nsamp;
        const int2 px = pix[p];
        const uint32_t off = halton_pixel_offset(sc, px.x, px.y, hp.exp1, hp.scale0, hp.mi0, hp.mi1);
        const uint32_t idx = off + (uint32_t)(s0 + (int)sl) * sc.hal_stride;
        const float fx = (float)px.x + halton_dim(sc, idx, 0);
        const float fy = (float)px.y + halton_dim(sc, idx, 1);
        float lx = 0.5f, ly = 0.5f;
        if (sc.lens_radius > 0) { lx = halton_dim(sc, idx, 3); ly = halton_dim(sc, idx, 4); }
        const Ray r = camera_ray(sc, fx, fy, lx, ly);
        if (kMeta)
            reinterpret_cast<uint2*>(ps.pfilm)[slot] = make_uint2(film_meta_axis(fx, px.x, fm.win, fm.rx, fm.inv_rx),
                                                                  film_meta_axis(fy, px.y, fm.win, fm.ry, fm.inv_ry));
        else
            ps.pfilm[slot] = make_float2(fx, fy);
        ps.body[2 * (size_t)slot] = make_float4(0.f, 0.f, 0.f, __uint_as_float(idx));  // L = 0, hidx
        ps.body[2 * (size_t)slot + 1] = make_float4(1.f, 1.f, 1.f, 1.f);              // beta = 1, etaScale = 1
        // dims 0-4 (pFilm, time, pLens) and the wvl dimension consumed; with sample
        // arrays Get1D jumps over [5, arrayEndDim) for wvl (sampler.cpp:180-184)
        *st_word(ps, slot) = (uint32_t)(sc.wvl_dim + 1) | kStCont;
        if (ps.dli) {
            ps.dli[kDlD * N + slot] = 0;
            ps.dli[kDlAoff * N + slot] = 0;
            ps.dli[kDlS * N + slot] = s0 + (int)sl;
            ps.dli[kDlPix * N + slot] = (int)off;
        }
        store_ray(ps.ray, slot, r);
        rq[slot] = slot << 2 | kRayCont;
        pq[slot] = slot;
    }
}
#else
;
#endif

// ----------------------------------------------------------------------------
// Shading
// ----------------------------------------------------------------------------
struct Dims {
    const DevScene* sc;
    uint32_t idx;
    int dim;
    bool overflow;
    __device__ __forceinline__ float get1() {
        if (dim >= sc->max_dim) { overflow = true; ++dim; return 0.5f; }
        return halton_dim(*sc, idx, dim++);
    }
};
// The same dimension counter reading the LDS-staged tables (k_shade).
struct DimsL {
    const DevScene* sc;
    const HalLds* hl;
    uint32_t idx;
    int dim;
    bool overflow;
    __device__ __forceinline__ float get1() {
        if (dim >= sc->max_dim) { overflow = true; ++dim; return 0.5f; }
        return halton_dim(*sc, *hl, idx, dim++);
    }
};

__device__ __forceinline__ S3 load_s3(const float* a, uint32_t n, uint32_t slot) {
    return s3(a[slot], a[n + slot], a[2 * n + slot]);
}
__device__ __forceinline__ void store_s3(float* a, uint32_t n, uint32_t slot, S3 v) {
    a[slot] = v.c[0]; a[n + slot] = v.c[1]; a[2 * n + slot] = v.c[2];
}

// Le of whatever area light the primitive carries (SurfaceInteraction::Le,
// interaction.cpp:148-151); the hit normal is only needed for one-sided lights.
template <int kFt>
__device__ __forceinline__ S3 hit_Le(const DevScene& sc, int prim, const Ray& ray, int* lightOut) {
    int mat, light;
    const PrimRec rec = prim_rec(sc, prim);
    prim_info<Ft<kFt>::sph>(sc, rec, &mat, &light);
    *lightOut = light;
    if (light < 0) return s3(0.f);
    const DevLight& l = sc.lights[PT_IDX(light, sc.n_lights)];
    if (l.two_sided) return l.L;
    SurfHit si;
    if (!surface_at<Ft<kFt>::sph>(sc, prim, rec, ray, &si)) return s3(0.f);
    return area_L(l, si.n, -ray.d);
}

// Finish the NEE of the previous vertex: Ld from the traced rays, then
// L += beta * Ld / lightPdf (integrator.cpp:121, path.cpp:122-127).
// EstimateDirect's value from its traced rays (integrator.cpp:124-258,
// portal_arealight.cpp:29-239): the Ld of the previous vertex's NEE.
// The payload fields every resolve reads, and ray A (the portal estimators'
// closest-hit ray); shade_batch loads them one path ahead.
// The payload fields a resolve reads and the traced NEE ray whose hit it
// evaluates (ray A for the portal estimators, ray B for MIS); shade_batch
// loads them one path ahead.
struct NeeIn {
    S3 F, Li, beta;
    float pdf, lpdf;  // pdf: the portal estimators' sample pdf; MIS ray B: the scattering pdf
    float w;          // projection: the portal-selection pdf; MIS ray B: the scattering weight
    int nl;   // MIS: the light the BSDF-sampled ray B must hit
    Ray ray;
};
// Only the fields the resolve of this payload reads (flags fl, the hits hA /
// hB of rays A and B): what nee_value touches under the same conditions.
// The payload is one 64-B record per slot: each quarter a resolve needs is one
// 16-B load.
// kMis: the scene has lights the MIS branch samples (Ft::mis).
template <bool kMis = true>
__device__ __forceinline__ NeeIn nee_load(const DevPaths& ps, uint32_t slot, uint32_t fl, int hA) {
    const float4* q = reinterpret_cast<const float4*>(ps.nee) + 4u * slot;
    NeeIn in{s3(0.f), s3(0.f), s3(0.f), 0.f, 0.f, 1.f, 0, Ray{v3(0, 0, 0), v3(0, 0, 1), kInf}};
    const bool portalA = (fl & kNfPortal) && (fl & kNfA);
    const bool misB = kMis && !(fl & kNfPortal) && (fl & kNfMis) && (fl & kNfB);
    const bool mis = kMis && !(fl & kNfPortal) && (fl & kNfMis);
    const float4 q0 = q[0];  // beta, light-selection pdf
    in.beta = s3(q0.x, q0.y, q0.z);
    in.lpdf = q0.w;
    if (portalA || (mis && (fl & kNfC1) && hA == 0)) {  // F, the portal estimators' pdf
        const float4 q1 = q[1];
        in.F = s3(q1.x, q1.y, q1.z);
        if (portalA) in.pdf = q1.w;
    }
    if ((portalA && hA < 0 && !(fl & kNfLi0)) || misB) {  // Li / f2, the MIS scattering weight
        const float4 q2 = q[2];
        in.Li = s3(q2.x, q2.y, q2.z);
        if (misB) in.w = q2.w;
    }
    if (misB) {  // scattering pdf, MIS light
        const float4 q3 = q[3];
        in.pdf = q3.x;
        in.nl = __float_as_int(q3.z);
    } else if ((fl & kNfPortal) && (fl & kNfDivPortal)) {  // the projection estimator's portal pdf
        in.w = q[3].y;
    }
    if (portalA && hA >= 0) in.ray = load_ray(ps.rayA, slot, kInf);
    if (misB) in.ray = load_ray(ps.rayB, slot, kInf);
    return in;
}
// fl / hA / hB: the payload's flags and the hits of rays A and B.
template <int kFt>
__device__ __forceinline__ S3 nee_value(const DevScene& sc, const DevPaths& ps, uint32_t slot, uint32_t fl,
                                        int hA, int hB, const NeeIn& in) {
    S3 Ld = s3(0.f);
    if (fl & kNfPortal) {
        if (fl & kNfA) {
            S3 Li = in.Li;
            const int h = hA;
            if (h >= 0) {
                int lid;
                Li = hit_Le<kFt>(sc, h, in.ray, &lid);
            }
            const S3 f = in.F;
            if (!is_black(f) && !is_black(Li)) Ld = Ld + (f * Li) / in.pdf;
        }
        if (fl & kNfDivPortal) Ld = Ld / in.w;
    } else if (Ft<kFt>::mis && (fl & kNfMis)) {
        if ((fl & kNfC1) && hA == 0) Ld = Ld + in.F;
        if (fl & kNfB) {
            const int h = hB;
            const int nl = in.nl;
            S3 Li = s3(0.f);
            if (h >= 0) {
                int lid;
                const S3 le = hit_Le<kFt>(sc, h, in.ray, &lid);
                if (lid == nl) Li = le;
            } else if (Ft<kFt>::inf && sc.lights[PT_IDX(nl, sc.n_lights)].kind == PT_LIGHT_INFINITE) {
                Li = inf_Le(sc.lights[PT_IDX(nl, sc.n_lights)], in.ray.d);  // light.Le(ray)
            }
            if (!is_black(Li)) {
                const S3 f2 = in.Li;
                Ld = Ld + (((f2 * Li) * s3(1.f)) * in.w) / in.pdf;
            }
        }
    }
    return Ld;
}
// st: the path's state word (the payload's flags at kStNfShift)
template <int kFt>
__device__ __forceinline__ S3 nee_value(const DevScene& sc, const DevPaths& ps, uint32_t slot, uint32_t st) {
    const uint32_t fl = (st & kStNfMask) >> kStNfShift;
    const int hA = *hit_word(ps, slot, kHdHitA);
    return nee_value<kFt>(sc, ps, slot, fl, hA, *hit_word(ps, slot, kHdHitB), nee_load<Ft<kFt>::mis>(ps, slot, fl, hA));
}
template <int kFt>
__device__ __forceinline__ void resolve_nee(const DevScene& sc, const DevPaths& ps, uint32_t slot, uint32_t fl,
                                            int hA, int hB, const NeeIn& in, S3* L) {
    const S3 Ld = nee_value<kFt>(sc, ps, slot, fl, hA, hB, in);
    *L = *L + in.beta * (Ld / in.lpdf);
}

__device__ __forceinline__ void put_nee(const DevPaths& ps, uint32_t slot, int k, float v) {
    ps.nee[(uint32_t)kNee * slot + (uint32_t)k] = v;
}
__device__ __forceinline__ void put_nee3(const DevPaths& ps, uint32_t slot, int k, S3 v) {
    put_nee(ps, slot, k, v.c[0]); put_nee(ps, slot, k + 1, v.c[1]); put_nee(ps, slot, k + 2, v.c[2]);
}
// one whole 16-B quarter of the payload record in one store (a 4-B store per field made a portal
// step's payload nine store instructions, each addressing 64 lanes' records)
__device__ __forceinline__ void put_nee_q(const DevPaths& ps, uint32_t slot, int q, S3 v, float w) {
    reinterpret_cast<float4*>(ps.nee)[4u * slot + (uint32_t)q] = make_float4(v.c[0], v.c[1], v.c[2], w);
}

// PortalArealight::EstimateDirect set-up (portal_arealight.cpp:29-239).
// u1 = uScattering (argument order at integrator.cpp:132); u2 is unused; the
// selected portal is call-local.  Returns the payload's kNf* flags (kNfA: ray
// A was emitted); the caller keeps them in the path's state word.
template <int kFt>
__device__ __forceinline__ uint32_t portal_nee(const DevScene& sc, const DevPaths& ps, uint32_t slot, int lightIdx,
                                           const SurfHit& it, const Bsdf& bsdf, float u10, float u11,
                                           uint32_t* ab = nullptr) {
    const DevLight& l = sc.lights[PT_IDX(lightIdx, sc.n_lights)];
    const DevPlane& lp = sc.planes[PT_IDX(l.shape, sc.n_planes)];
    uint32_t flags = kNfPortal;
    if (l.strategy != PT_PORTAL_LIGHT) {
        const V3 pObj = xf_point(lp.w2o, it.p);
        // Distribution1D over the portals' visibility (portal_arealight.cpp:38-60),
        // evaluated without arrays: InFrustum() is always true (aaportal.cpp:101-104),
        // so dist[i] is 1 for portals in front of the point and 0 otherwise; the
        // CDF entries are recomputed with the same sequential float sums.
        const int np = l.n_portals;
        if (np > 0 && PT_IDX(l.first_portal + np - 1, sc.n_pplanes) != l.first_portal + np - 1) return 0u;
        const DevPlane* portals = sc.portal_planes + l.first_portal;
        int nvis = 0;
        for (int i = 0; i < np; ++i) nvis += plane_in_front(portals[i], pObj) ? 1 : 0;
        if (nvis > 0) {
            float sum = 0;
            for (int i = 0; i < nvis; ++i) sum += 1.f;
            const float dv = 1.f / sum;            // dist[i] /= sum
            const float inc = dv / (float)np;      // Distribution1D: func[i] / n
            float funcInt = 0;
            for (int i = 0; i < np; ++i) funcInt = funcInt + (plane_in_front(portals[i], pObj) ? inc : 0.f / (float)np);
            // FindInterval over the monotone CDF = number of entries <= u, minus one
            int cnt = 1;  // cdf[0] = 0 <= u
            float c = 0;
            for (int i = 1; i < np + 1; ++i) {
                c = c + (plane_in_front(portals[i - 1], pObj) ? inc : 0.f / (float)np);
                const float ci = funcInt == 0 ? (float)i / (float)np : c / funcInt;
                cnt += ci <= u10 ? 1 : 0;
            }
            int sel = cnt - 1;
            sel = sel < 0 ? 0 : (sel > np - 1 ? np - 1 : sel);
            const float dsel = plane_in_front(portals[sel], pObj) ? dv : 0.f / sum;
            const float portalPdf = (funcInt > 0) ? dsel / (funcInt * np) : 0;
            const DevPlane& pp = sc.portal_planes[PT_IDX(l.first_portal + sel, sc.n_pplanes)];
            if (plane_in_front(pp, pObj)) {
                V3 wi = v3(0, 0, 0);
                float pdf = 0;
                if (l.strategy == PT_PORTAL_UNIFORM) {
                    // AAPortal::SamplePortal (aaportal.cpp:73-83)
                    V3 sp, sn, spe;
                    float areaPdf;
                    plane_sample(pp, u10, u11, &sp, &sn, &spe, &areaPdf);
                    wi = normalize(sp - it.p);
                    pdf = dist2(it.p, sp) / (absdot(plane_normal(pp), -wi) * pp.area);
                } else {
                    // AAPortal::SampleProj (aaportal.cpp:114-159), literal
                    const V3 dLo = normalize(it.p - lp.lo);
                    const V3 dHi = normalize(it.p - lp.hi);
                    if (dLo.z == 0 || dHi.z == 0) pdf = 0;
                    else {
                        const V3 lpLo = lp.lo, lpHi = lp.hi;
                        const float tLo = (pp.lo_a - lpLo[lp.ax]) / dLo[lp.ax];
                        const float tHi = (pp.lo_a - lpHi[lp.ax]) / dHi[lp.ax];
                        const V3 projLo = lp.lo + dLo * tLo;
                        const V3 projHi = lp.hi + dHi * tHi;
                        const V3 isectHi = vmax(pp.lo, projLo);
                        const V3 isectLo = vmin(pp.hi, projHi);
                        const float len0 = isectHi[pp.ax0] - isectLo[pp.ax0];
                        const float len1 = isectHi[pp.ax1] - isectLo[pp.ax1];
                        V3 sampled = v3(0, 0, 0);
                        sampled.set(pp.ax, pp.lo_a);
                        sampled.set(pp.ax0, isectLo[pp.ax0] + u10 * len0);
                        sampled.set(pp.ax1, isectLo[pp.ax1] + u10 * len1);
                        const V3 sampledWorld = xf_point(pp.w2o, sampled);
                        wi = sampledWorld - it.p;
                        pdf = dist2(it.p, sampled) / (absdot(plane_normal(pp), -wi) * (len0 * len1));
                    }
                    flags |= kNfDivPortal;
                    put_nee(ps, slot, kNeePortalPdf, portalPdf);
                    if (ab) *ab += 4;
                }
                if (pdf > 0) {
                    const Ray r{offset_ray_origin(it.p, it.perr, it.n, wi), wi, kInf};
                    store_ray(ps.rayA, slot, r);
                    put_nee_q(ps, slot, kNeeF / 4, bsdf_f<kFt>(bsdf, it.wo, wi, kBxNonSpecular) * absdot(wi, it.sn), pdf);
                    // Li = 0 before the portal ray is traced (portal_arealight.cpp:181), kept on a miss: a flag
                    // instead of a 12-B store and load
                    flags |= kNfA | kNfLi0;
                    if (ab) *ab += 24 + 12 + 4 + 12;  // the algorithmic count keeps Li's 12 B
                }
                return flags;
            }
        }
    }
    // EstimateDirectLight (portal_arealight.cpp:115-156)
    V3 wi, sp, sn, spe;
    float pdf = 0;
    const S3 Li = area_sample_li<kFt>(sc, l, it, u10, u11, &wi, &pdf, &sp, &sn, &spe);
    if (!is_black(Li) && pdf > 0) {
        const Ray r{offset_ray_origin(it.p, it.perr, it.n, wi), wi, kInf};
        store_ray(ps.rayA, slot, r);
        put_nee_q(ps, slot, kNeeF / 4, bsdf_f<kFt>(bsdf, it.wo, wi, kBxNonSpecular) * absdot(wi, it.sn), pdf);
        put_nee_q(ps, slot, kNeeLi / 4, Li, 0.f);  // .w: the MIS weight's word, unread by the portal resolve
        flags |= kNfA;
        if (ab) *ab += 24 + 12 + 4 + 12;
    }
    return flags;
}

// EstimateDirect, MIS branch (integrator.cpp:137-258) for a DiffuseAreaLight.
// Emits ray A (shadow, any-hit) and/or ray B (BSDF-sampled, closest-hit).
template <int kFt>
__device__ __forceinline__ uint32_t mis_nee(const DevScene& sc, const DevPaths& ps, uint32_t slot, int lightIdx,
                                            const SurfHit& it, const Bsdf& bsdf, float ul0, float ul1, float us0,
                                            float us1, uint32_t* ab = nullptr) {
    const DevLight& l = sc.lights[PT_IDX(lightIdx, sc.n_lights)];
    uint32_t flags = kNfMis;
    V3 wi, sp, sn, spe;
    float lightPdf = 0, scatteringPdf = 0;
    const S3 Li = area_sample_li<kFt>(sc, l, it, ul0, ul1, &wi, &lightPdf, &sp, &sn, &spe);
    if (lightPdf > 0 && !is_black(Li)) {
        const S3 f = bsdf_f<kFt>(bsdf, it.wo, wi, kBxNonSpecular) * absdot(wi, it.sn);
        scatteringPdf = bsdf_pdf<kFt>(bsdf, it.wo, wi, kBxNonSpecular);
        if (!is_black(f)) {
            // VisibilityTester::Unoccluded -> SpawnRayTo(Interaction) (light.cpp:59-61, interaction.h:75-80)
            const V3 origin = offset_ray_origin(it.p, it.perr, it.n, sp - it.p);
            const V3 target = offset_ray_origin(sp, spe, sn, origin - sp);
            const V3 d = target - origin;
            store_ray(ps.rayA, slot, Ray{origin, d, 1 - kShadowEps});
            if (l.kind == PT_LIGHT_POINT) {  // IsDeltaLight: no MIS weight (integrator.cpp:186-188)
                put_nee_q(ps, slot, kNeeF / 4, (f * Li) / lightPdf, 0.f);  // .w: the portal pdf's word, unread
            } else {
                const float lightWeight = power_heuristic(lightPdf, scatteringPdf);
                put_nee_q(ps, slot, kNeeF / 4, ((f * Li) * lightWeight) / lightPdf, 0.f);
            }
            flags |= kNfA | kNfC1;
            if (ab) *ab += 28 + 12;
        }
    }
    if (l.kind != PT_LIGHT_POINT) {  // BSDF sampling only for non-delta lights
        float pdf2 = scatteringPdf;
        V3 wi2 = wi;
        int sampledType = 0;
        S3 f = bsdf_sample<kFt>(bsdf, it.wo, &wi2, us0, us1, &pdf2, kBxNonSpecular, &sampledType);
        f = f * absdot(wi2, it.sn);
        if (!is_black(f) && pdf2 > 0) {
            const float lp = area_pdf_li<kFt>(sc, l, it, wi2);
            if (lp != 0) {
                const float sw = power_heuristic(pdf2, lp);
                const Ray r{offset_ray_origin(it.p, it.perr, it.n, wi2), wi2, kInf};
                store_ray(ps.rayB, slot, r);
                put_nee_q(ps, slot, kNeeLi / 4, f, sw);
                // {spdf, portal pdf (unread here), light, -}
                reinterpret_cast<float4*>(ps.nee)[4u * slot + (uint32_t)kNeeSpdf / 4u] =
                    make_float4(pdf2, 0.f, __int_as_float(lightIdx), 0.f);
                flags |= kNfB;
                if (ab) *ab += 24 + 12 + 4 + 4 + 4;
            }
        }
    }
    return flags;
}

// One path step.  Returns the rays to enqueue in rays[] and whether the path
// stays alive.
// The fields every step reads first, loaded for the next path of a lane while
// the current one is shaded (shade_batch): the kernel is bound by the latency
// of its dependent loads, and these are the first two links of the chain.
struct PathPre {
    uint32_t st, hidx;
    int hit, hitA, hitB;
    S3 L, beta;
    Ray ray;
    float eta;    // etaScale (Russian roulette reads it)
};
// What a step reads of its own path only once it starts: the NEE payload
// and the hit primitive's record.  shade_batch issues these loads before the
// next path's body prefetch, so waiting for them (vmcnt counts in issue
// order) does not wait for the prefetch, and they are not carried in
// registers through the previous step (the register budget of 3 waves).
struct PathNow {
    NeeIn nee;
    PrimRec rec;
};
template <int kFt>
__device__ __forceinline__ void path_load_nee(const DevPaths& ps, uint32_t slot, const PathPre& p, PathNow* q) {
    if (p.st & kStNee) q->nee = nee_load<Ft<kFt>::mis>(ps, slot, (p.st & kStNfMask) >> kStNfShift, p.hitA);
}
template <int kFt>
__device__ __forceinline__ void path_load_rec(const DevScene& sc, const PathPre& p, PathNow* q) {
    if ((p.st & kStCont) && p.hit >= 0) q->rec = prim_rec(sc, p.hit);
}
template <int kFt>
__device__ __forceinline__ void path_load_now(const DevScene& sc, const DevPaths& ps, uint32_t slot, const PathPre& p,
                                              PathNow* q) {
    path_load_nee<kFt>(ps, slot, p, q);
    path_load_rec<kFt>(sc, p, q);
}
// Two stages: the head record (state word with the payload flags, hits) two
// paths ahead, the body one path ahead and only what the head says this step
// will read.
// kMis: the scene has lights the MIS branch samples -- only then can ray B (its hit word) be pending
template <bool kMis = true>
__device__ __forceinline__ void path_prefetch_head(const DevPaths& ps, uint32_t slot, PathPre* p) {
    p->st = *st_word(ps, slot);
    p->hit = *hit_word(ps, slot, kHdHit);
    p->hitA = *hit_word(ps, slot, kHdHitA);
    p->hitB = kMis ? *hit_word(ps, slot, kHdHitB) : -1;
}
__device__ __forceinline__ void path_prefetch_body(const DevPaths& ps, uint32_t slot, PathPre* p) {
    const float3 a = *reinterpret_cast<const float3*>(body_word(ps, slot, kBdL));
    p->L = s3(a.x, a.y, a.z);
    if (p->st & kStCont) {
        p->hidx = hidx_of(ps, slot);
        const float4 b = ps.body[2u * slot + 1u];
        p->beta = s3(b.x, b.y, b.z);
        p->eta = b.w;
        p->ray = load_ray(ps.ray, slot, kInf);
    }
}
__device__ __forceinline__ void store_L(const DevPaths& ps, uint32_t slot, S3 L) {
    *reinterpret_cast<float3*>(body_word(ps, slot, kBdL)) = make_float3(L.c[0], L.c[1], L.c[2]);
}
// A finished sample's radiance, pixel-major and dense (the film pass reads it
// for every film pixel its filter footprint reaches)
__device__ __forceinline__ void store_Lfin(const DevPaths& ps, uint32_t slot, S3 L) {
    float* p = ps.Lfin + 3u * slot;
    p[0] = L.c[0]; p[1] = L.c[1]; p[2] = L.c[2];
}
__device__ __forceinline__ S3 load_Lfin(const DevPaths& ps, uint32_t slot) {
    const float* p = ps.Lfin + 3u * slot;
    return s3(p[0], p[1], p[2]);
}

// ab: algorithmic path-state bytes this step reads and writes (the bench's
// k_shade roofline): the SoA fields the reference's Li loop carries from one
// vertex to the next, plus the queue entries (scene tables are not counted).
template <int kFt>
__device__ __forceinline__ void shade_path(const DevScene& sc, const HalLds& hl, const DevPaths& ps, uint32_t slot,
                                           const PathPre& pre, const PathNow& now, RayList* rays,
                                           bool* keep, bool* overflow, uint32_t* ab) {
    rays->n = 0;
    if (PT_IDX((int)slot, ps.n) != (int)slot) return;
    uint32_t st = pre.st;
    S3 L = pre.L;
    if (ab) *ab += 4 + 4 + 12 + 12 + 4;  // queue entry, st + L read, L + st written
    if (st & kStNee) {
        const uint32_t fl = (st & kStNfMask) >> kStNfShift;
        {   // bytes of the NEE payload resolve_nee reads (integrator.cpp:121, portal_arealight.cpp:29-239)
            uint32_t b = 4 + 12 + 4;  // flags, beta, light-selection pdf
            if (fl & kNfPortal) {
                if (fl & kNfA) b += 12 + 4 + 12 + 4 + (pre.hitA >= 0 ? 24 : 0);
                if (fl & kNfDivPortal) b += 4;
            } else if (fl & kNfMis) {
                if (fl & kNfC1) b += 4 + 12;
                if (fl & kNfB) b += 4 + 4 + 12 + 4 + 4 + (pre.hitB >= 0 ? 24 : 0);
            }
            if (ab) *ab += b;
        }
        resolve_nee<kFt>(sc, ps, slot, fl, pre.hitA, pre.hitB, now.nee, &L);
        st &= ~(kStNee | kStNfMask);
    }
    if (st & kStCont) {
        st &= ~kStCont;
        int bounces = (int)((st >> kStBounceShift) & 0xffu);
        const bool specular = (st & kStSpecular) != 0;
        const Ray ray = pre.ray;
        const int hp = pre.hit;
        S3 beta = pre.beta;
        if (ab) *ab += 24 + 4 + 12;
        SurfHit si;
        bool found = hp >= 0 && surface_at<Ft<kFt>::sph>(sc, hp, now.rec, ray, &si);
        int mat = -1, light = -1;
        if (found) prim_info<Ft<kFt>::sph>(sc, now.rec, &mat, &light);
        if (bounces == 0 || specular) {
            if (found) L = L + beta * (light >= 0 ? area_L(sc.lights[PT_IDX(light, sc.n_lights)], si.n, -ray.d) : s3(0.f));
            else if (Ft<kFt>::inf)
                for (int li = 0; li < sc.n_lights; ++li)  // scene.infiniteLights, in light order
                    if (sc.lights[PT_IDX(li, sc.n_lights)].kind == PT_LIGHT_INFINITE) L = L + beta * inf_Le(sc.lights[PT_IDX(li, sc.n_lights)], ray.d);
        }
        if (found && bounces < sc.max_depth) {
            if (sc.mats[PT_IDX(mat, sc.n_mats)].kind == PT_MAT_NONE) {
                // null BSDF: continue through the surface, bounces unchanged (path.cpp:108-113)
                const Ray r{offset_ray_origin(si.p, si.perr, si.n, ray.d), ray.d, kInf};
                store_ray(ps.ray, slot, r);
                if (ab) *ab += 24;
                st |= kStCont;
                rays->push(slot << 2 | kRayCont);
            } else {
                DimsL dm{&sc, &hl, pre.hidx, (int)(st & kStDimMask), false};
                if (ab) *ab += 4;
                Bsdf bsdf;
                // Camera::GenerateWvls (camera.cpp:62-76): wvls[0] from camera dimension 5
                const float wvl0 = Ft<kFt>::spec && sc.mats[PT_IDX(mat, sc.n_mats)].kind == PT_MAT_DISPERSIVE_GLASS
                                       ? (float)400 + (float)300 * halton_dim(sc, dm.idx, sc.wvl_dim) : 550.f;
                make_bsdf<kFt>(&sc.mats[PT_IDX(mat, sc.n_mats)], si, wvl0, &bsdf);
                if (bsdf_num<kFt>(bsdf, kBxNonSpecular) > 0) {
                    // UniformSampleOneLight (integrator.cpp:100-122)
                    bool deferred = false;
                    uint32_t nf = 0;  // the payload's kNf* flags
                    float lightPdf = 0;
                    bool haveLight = false;
                    if (sc.n_lights > 0) {
                        const float ul = dm.get1();
                        const int ln = find_interval(sc.ldist_cdf, sc.n_lights + 1, ul);
                        lightPdf = (sc.ldist_int > 0) ? sc.ldist_func[PT_IDX(ln, sc.n_lights)] / (sc.ldist_int * sc.n_lights) : 0;
                        if (lightPdf != 0) {
                            haveLight = true;
                            const float uL0 = dm.get1(), uL1 = dm.get1();
                            const float uS0 = dm.get1(), uS1 = dm.get1();
                            if (!Ft<kFt>::mis || sc.lights[PT_IDX(ln, sc.n_lights)].kind == PT_LIGHT_PORTAL_AREA) {
                                nf = portal_nee<kFt>(sc, ps, slot, ln, si, bsdf, uS0, uS1, ab);
                                if (nf & kNfA) {
                                    rays->push(slot << 2 | kRayA);
                                    deferred = true;
                                }
                            } else {
                                nf = mis_nee<kFt>(sc, ps, slot, ln, si, bsdf, uL0, uL1, uS0, uS1, ab);
                                if (nf & kNfA) rays->push(slot << 2 | kRayShadow);
                                if (nf & kNfB) rays->push(slot << 2 | kRayB);
                                deferred = (nf & (kNfA | kNfB)) != 0;
                            }
                        }
                    }
                    if (deferred) {
                        put_nee_q(ps, slot, kNeeBeta / 4, beta, lightPdf);
                        if (ab) *ab += 12 + 4;
                        st = (st & ~kStNfMask) | kStNee | (nf << kStNfShift);
                    } else {
                        // no ray: EstimateDirect returned Spectrum(0)
                        L = L + beta * (haveLight ? s3(0.f) / lightPdf : s3(0.f));
                    }
                }
                // BSDF sampling (path.cpp:131-151)
                const float u0 = dm.get1(), u1 = dm.get1();
                V3 wi = v3(0, 0, 0);
                float pdf = 0;
                int sampled = 0;
                const S3 f = bsdf_sample<kFt>(bsdf, -ray.d, &wi, u0, u1, &pdf, kBxAll, &sampled);
                if (!(is_black(f) || pdf == 0.f)) {
                    beta = beta * ((f * absdot(wi, si.sn)) / pdf);
                    if (sampled & kBxSpecular) st |= kStSpecular;
                    else st &= ~kStSpecular;
                    float etaScale = pre.eta;
                    if (Ft<kFt>::spec && (sampled & kBxSpecular) && (sampled & kBxT)) {  // etaScale (path.cpp:144-150)
                        const float eta = bsdf.eta;
                        etaScale *= (dot(-ray.d, si.n) > 0) ? (eta * eta) : 1 / (eta * eta);
                        *body_word(ps, slot, kBdEta) = etaScale;
                        if (ab) *ab += 4;
                    }
                    if (ab) *ab += 4;  // etaScale read for Russian roulette
                    const Ray r{offset_ray_origin(si.p, si.perr, si.n, wi), wi, kInf};
                    bool alive = true;
                    // Russian roulette (path.cpp:177-185)
                    const S3 rrBeta = beta * etaScale;
                    if (max_comp(rrBeta) < sc.rr_threshold && bounces > 3) {
                        const float q = smax(0.05f, 1 - max_comp(rrBeta));
                        if (dm.get1() < q) alive = false;
                        else beta = beta / (1 - q);
                    }
                    if (alive) {
                        store_ray(ps.ray, slot, r);
                        *reinterpret_cast<float3*>(body_word(ps, slot, kBdBeta)) = make_float3(beta.c[0], beta.c[1], beta.c[2]);
                        if (ab) *ab += 24 + 12;
                        ++bounces;
                        st |= kStCont;
                        rays->push(slot << 2 | kRayCont);
                    }
                }
                if (dm.overflow) { st |= kStDimOverflow; *overflow = true; }
                st = (st & ~kStDimMask) | (uint32_t)min(dm.dim, (int)kStDimMask);  // past max_dim only after overflow
                st = (st & ~(0xffu << kStBounceShift)) | ((uint32_t)(bounces & 0xff) << kStBounceShift);
            }
        }
    }
    *st_word(ps, slot) = st;
    *keep = (st & (kStCont | kStNee)) != 0;
    if (*keep) store_L(ps, slot, L);
    else store_Lfin(ps, slot, L);
    if (ab) *ab += 4 * (rays->n + (*keep ? 1u : 0u));  // ray / path queue entries written
}

// Copy n 4-byte words global -> LDS, the whole block.
__device__ __forceinline__ void lds_copy_words(void* dst, const void* src, uint32_t bytes) {
    uint32_t* d = (uint32_t*)dst;
    const uint32_t* g = (const uint32_t*)src;
    for (uint32_t i = threadIdx.x; i < bytes / 4u; i += blockDim.x) d[i] = g[i];
}
// k_shade_tab: the scene tables a path step reads (primitive records,
// materials, lights and their planes, portal planes, the light distribution)
// copied into LDS after the Halton tables, and a scene view whose table
// pointers address the LDS copies -- the step's chains of dependent
// scene-table loads then wait on LDS (lgkmcnt), not behind the path-state
// loads and stores in flight (vmcnt counts in issue order).
__device__ __forceinline__ DevScene stage_tables(const DevScene& sc, uint4* lds) {
    const TabLayout t = tab_layout(sc.n_prims, sc.n_mats, sc.n_lights, sc.n_planes, sc.n_pplanes);
    char* base = (char*)lds + sc.hal_lds_bytes;
    lds_copy_words(base + t.prims, sc.prims, 48u * (uint32_t)sc.n_prims);
    lds_copy_words(base + t.mats, sc.mats, (uint32_t)sizeof(pt_material) * (uint32_t)sc.n_mats);
    lds_copy_words(base + t.lights, sc.lights, (uint32_t)sizeof(DevLight) * (uint32_t)sc.n_lights);
    lds_copy_words(base + t.planes, sc.planes, (uint32_t)sizeof(DevPlane) * (uint32_t)sc.n_planes);
    lds_copy_words(base + t.pplanes, sc.portal_planes, (uint32_t)sizeof(DevPlane) * (uint32_t)sc.n_pplanes);
    lds_copy_words(base + t.lfunc, sc.ldist_func, 4u * (uint32_t)sc.n_lights);
    lds_copy_words(base + t.lcdf, sc.ldist_cdf, 4u * (uint32_t)(sc.n_lights + 1));
    DevScene v = sc;
    v.prims = (const float4*)(base + t.prims);
    v.mats = (const pt_material*)(base + t.mats);
    v.lights = (const DevLight*)(base + t.lights);
    v.planes = (const DevPlane*)(base + t.planes);
    v.portal_planes = (const DevPlane*)(base + t.pplanes);
    v.ldist_func = (const float*)(base + t.lfunc);
    v.ldist_cdf = (const float*)(base + t.lcdf);
    return v;
}

// kLean: the current path's body is loaded at the start of its own step
// (ahead of the next path's head prefetch) instead of one path ahead -- the
// register budget of 3 waves per SIMD for the kernels with the MIS branch.
// kAb: count the algorithmic path-state bytes (shade_path's ab) -- one
// register, which the 3-wave build cannot spare, so the counting build is a
// separate instantiation that the renderer runs only on request
// (pt_set_count_bytes; the bench's one extra frame).
// kAhead 2: the NEE payload and the hit primitive's record (path_load_now) are
// loaded one path ahead as well, with the next path's body, instead of at the
// start of the path's own step -- ≈30 more VGPRs, for the 2-wave MIS kernels
// whose feature set leaves them (ShadeAhead); kAhead 1: the payload alone one
// path ahead, the record at the step's start (the two-lobe sets, C3)
#define PT_ABP (kAb ? &ab : nullptr)
#ifdef PT_NO_AHEAD  // experiment build: the round-4 order
template <int kFt>
constexpr int kShadeAhead = 0;
#else
// two-lobe sets: 256 VGPRs and one wave with both ahead; the payload alone ahead fits 2 waves (PT_AHEAD1=0: off)
#ifndef PT_AHEAD1
#define PT_AHEAD1 1
#endif
template <int kFt>
constexpr int kShadeAhead = !Ft<kFt>::mis ? 0 : (!(Ft<kFt>::micro && Ft<kFt>::spec) ? 2 : PT_AHEAD1);
#endif
template <int kFt, bool kTab, bool kLean = false, bool kAb = false, int kAhead = 0>
__device__ __forceinline__ void shade_batch(const DevScene& sc0, const DevPaths& ps, const uint32_t* __restrict__ pq,
                                            const uint32_t* __restrict__ pq_count, uint32_t* rq_out,
                                            uint32_t* rq_out_count, uint32_t* pq_out, uint32_t* pq_out_count,
                                            DevStats* stats) {
    const uint32_t n = *pq_count;
    bool overflow = false;
    PT_WAVEQ(wq);
    extern __shared__ uint4 pt_shade_lds[];
    const DevScene sc = kTab ? stage_tables(sc0, pt_shade_lds) : sc0;
    const HalLds hl = stage_halton(sc0, pt_shade_lds);  // its __syncthreads also covers the tables
    uint32_t ab = 0;  // this lane's algorithmic path-state bytes
    const uint32_t stride = gridDim.x * blockDim.x;
    // software pipeline over the grid-stride iterations: while this path is
    // shaded, the queue entry three paths ahead, the head of the path two
    // ahead and the body of the next path are in flight (slots in the queue
    // are distinct, so no step writes what a prefetch read)
    uint32_t base = blockIdx.x * blockDim.x;
#if defined(PT_SHADE_PIPE) && PT_SHADE_PIPE == 0
    // experiment build: no prefetch (each path's loads, then its step)
    for (; base < n; base += stride) {
        const uint32_t i = base + threadIdx.x;
        RayList rays;
        bool keep = false;
        uint32_t slot = 0;
        if (i < n) {
            slot = pq[i];
            PathPre pre{};
            PathNow now{};
            path_prefetch_head<Ft<kFt>::mis>(ps, slot, &pre);
            path_prefetch_body(ps, slot, &pre);
            path_load_now<kFt>(sc, ps, slot, pre, &now);
            shade_path<kFt>(sc, hl, ps, slot, pre, now, &rays, &keep, &overflow, PT_ABP);
        }
        wq_push(wq, rays, keep, slot, rq_out_count, rq_out, pq_out);
    }
#else
    if constexpr (kLean) {
        const uint32_t i0 = base + threadIdx.x;
        uint32_t slot = 0, slot1 = 0;
        PathPre pre{};  // this path's head (its body is loaded when its step starts)
        if (i0 < n) {
            slot = pq[i0];
            path_prefetch_head<Ft<kFt>::mis>(ps, slot, &pre);
        }
        if (i0 + stride < n) slot1 = pq[i0 + stride];
        for (; base < n; base += stride) {
            const uint32_t i = base + threadIdx.x;
            PathPre nxt{};
            PathNow now{};
            uint32_t slot2 = 0;
            if (i < n) {
                path_prefetch_body(ps, slot, &pre);
                path_load_now<kFt>(sc, ps, slot, pre, &now);
            }
            if (i + stride < n) path_prefetch_head<Ft<kFt>::mis>(ps, slot1, &nxt);
            if (i + 2 * stride < n) slot2 = pq[i + 2 * stride];
            RayList rays;
            bool keep = false;
            if (i < n) shade_path<kFt>(sc, hl, ps, slot, pre, now, &rays, &keep, &overflow, PT_ABP);
            wq_push(wq, rays, keep, slot, rq_out_count, rq_out, pq_out);
            slot = slot1;
            slot1 = slot2;
            pre = nxt;
        }
    } else {
    const uint32_t i0 = base + threadIdx.x;
    uint32_t slot = 0, slot1 = 0, slot2 = 0;
    PathPre pre{}, nxt{};  // this path (complete) and the next one (head only)
    if (i0 < n) {
        slot = pq[i0];
        path_prefetch_head<Ft<kFt>::mis>(ps, slot, &pre);
        path_prefetch_body(ps, slot, &pre);
    }
    if (i0 + stride < n) {
        slot1 = pq[i0 + stride];
        path_prefetch_head<Ft<kFt>::mis>(ps, slot1, &nxt);
    }
    if (i0 + 2 * stride < n) slot2 = pq[i0 + 2 * stride];
    PathNow now{};  // kAhead: this path's NEE payload (and hit record), loaded one path ahead
    if constexpr (kAhead == 2) {
        if (i0 < n) path_load_now<kFt>(sc, ps, slot, pre, &now);
    } else if constexpr (kAhead == 1) {
        if (i0 < n) path_load_nee<kFt>(ps, slot, pre, &now);
    }
    for (; base < n; base += stride) {
        const uint32_t i = base + threadIdx.x;
        PathPre nn{};
        uint32_t slot3 = 0;
        PathNow nowN{};
        if constexpr (kAhead == 2) {
            if (i + stride < n) {
                path_prefetch_body(ps, slot1, &nxt);  // its head arrived during the last path
                path_load_now<kFt>(sc, ps, slot1, nxt, &nowN);
            }
        } else if constexpr (kAhead == 1) {
            if (i < n) path_load_rec<kFt>(sc, pre, &now);  // issued ahead of the prefetches below
            if (i + stride < n) {
                path_prefetch_body(ps, slot1, &nxt);
                path_load_nee<kFt>(ps, slot1, nxt, &nowN);
            }
        } else {
            now = PathNow{};
            if (i < n) path_load_now<kFt>(sc, ps, slot, pre, &now);  // issued ahead of the prefetches below
            if (i + stride < n) path_prefetch_body(ps, slot1, &nxt);  // its head arrived during the last path
        }
        if (i + 2 * stride < n) path_prefetch_head<Ft<kFt>::mis>(ps, slot2, &nn);
        if (i + 3 * stride < n) slot3 = pq[i + 3 * stride];
        RayList rays;
        bool keep = false;
        if (i < n) shade_path<kFt>(sc, hl, ps, slot, pre, now, &rays, &keep, &overflow, PT_ABP);
        wq_push(wq, rays, keep, slot, rq_out_count, rq_out, pq_out);
        slot = slot1;
        slot1 = slot2;
        slot2 = slot3;
        pre = nxt;
        nxt = nn;
        if constexpr (kAhead != 0) now = nowN;
    }
    }
#endif
    wq_flush(wq, rq_out_count, rq_out, pq_out);
    if (overflow) atomicAdd(&stats->dim_overflow, 1ull);
    if (kAb) {
        const unsigned long long abw = wave_sum_u64((unsigned long long)ab);
        if (lane_id() == 0 && abw) atomicAdd(&stats->shade_bytes, abw);
    }
}

// ----------------------------------------------------------------------------
// k_shade_sort (round 6): the path queue grouped by the material class of each
// path's new hit (kPrimClassShift: matte, specular, microfacet; misses and
// paths with only an NEE resolve pending count as matte), chunk by chunk:
// block b takes entries [4096 b, 4096 (b + 1)) and writes them back to the
// same range with the classes one after the other.  The shading kernel's
// waves take 64 consecutive entries, so almost every wave then holds one class
// and its material branches (make_bsdf, the lobe loops of BSDF::f / Pdf /
// Sample_f) are uniform: a matte wave no longer executes FresnelSpecular or
// the microfacet lobes because one of its lanes hit glass.  Paths are
// independent, so the order of a queue never changes a result.
// ----------------------------------------------------------------------------
constexpr uint32_t kSortChunk = 4096;  // 256 threads x 16 entries
__global__ __launch_bounds__(256) void k_shade_sort(DevScene sc, DevPaths ps, const uint32_t* __restrict__ pq,
                                                    const uint32_t* __restrict__ pq_count, uint32_t* __restrict__ out)
#ifdef PT_TU_MISC
{
    __shared__ uint32_t buf[kSortChunk];
    __shared__ uint32_t cnt[3], run[3];
    const uint32_t n = *pq_count;
    const uint32_t c0 = blockIdx.x * kSortChunk;
    if (c0 >= n) return;
    const uint32_t m = min(kSortChunk, n - c0);
    if (threadIdx.x < 3) { cnt[threadIdx.x] = 0; run[threadIdx.x] = 0; }
    __syncthreads();
    uint32_t slot[16], cls = 0;  // cls: 2 bits per entry, 3 = none
    const uint32_t lane = lane_id();
    const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t i = (uint32_t)k * 256u + threadIdx.x;
        uint32_t c = 3;
        slot[k] = 0;
        if (i < m) {
            const uint32_t s = pq[c0 + i];
            slot[k] = s;
            const uint32_t stw = *st_word(ps, s);
            const int h = *hit_word(ps, s, kHdHit);
            c = ((stw & kStCont) && h >= 0) ? (__float_as_uint(sc.prims[3 * h].w) >> kPrimClassShift) & 3u : 0u;
            c = c > 2 ? 0 : c;
        }
        cls |= c << (2 * k);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // per-class counts: one LDS atomic per wave and class
        const uint32_t c = (cls >> (2 * k)) & 3u;
#pragma unroll
        for (uint32_t q = 0; q < 3; ++q) {
            const uint32_t nq = (uint32_t)__popcll(__ballot(c == q));
            if (lane == 0 && nq) atomicAdd(&cnt[q], nq);
        }
    }
    __syncthreads();
    const uint32_t off1 = cnt[0], off2 = cnt[0] + cnt[1];
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // positions: the class's offset + the wave's block of it + the lane's rank
        const uint32_t c = (cls >> (2 * k)) & 3u;
#pragma unroll
        for (uint32_t q = 0; q < 3; ++q) {
            const uint64_t b = __ballot(c == q);
            uint32_t base = 0;
            if (lane == 0 && b) base = atomicAdd(&run[q], (uint32_t)__popcll(b));
            base = __builtin_amdgcn_readlane(base, 0);
            if (c == q) buf[(q == 0 ? 0u : (q == 1 ? off1 : off2)) + base + (uint32_t)__popcll(b & below)] = slot[k];
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += 256) out[c0 + i] = buf[i];
}
#else
;
#endif

// ----------------------------------------------------------------------------
// DirectLightingIntegrator::Li (directlighting.cpp:58-84) as a resumable
// per-sample state machine.  The reference recurses depth first through
// SpecularReflect / SpecularTransmit (integrator.cpp:639-770) and consumes
// sampler dimensions in that order, and it sums each vertex's radiance before
// its parent scales it (f * Li * |cos| / pdf), so the device keeps an explicit
// stack of frames (DevPaths::dlframe) and resumes a parent when its child's
// subtree returns.  Each EstimateDirect of UniformSampleAllLights (one per
// sample-array entry) or UniformSampleOneLight is one wavefront step: its rays
// are traced, then nee_value() gives its Ld and the sum continues in the
// reference's order.
// ----------------------------------------------------------------------------
enum DlStep { kDlHit, kDlLights, kDlOne, kDlAcc, kDlSpecR, kDlSpecT, kDlReturn, kDlDone };

template <int kFt>
__device__ __forceinline__ void shade_dl(const DevScene& sc, const DevPaths& ps, uint32_t slot, RayList* rays,
                                         bool* keep, bool* overflow) {
    const uint32_t N = (uint32_t)ps.n;
    int* const I = ps.dli;
    float* const Fl = ps.dlf;
    float* const FR = ps.dlframe;
    auto fr = [&](int d, int k) -> float& { return FR[(size_t)(d * kDlFrame + k) * N + slot]; };
    auto fr3 = [&](int d, int k) { return s3(fr(d, k), fr(d, k + 1), fr(d, k + 2)); };
    auto set3 = [&](int d, int k, S3 v) { fr(d, k) = v.c[0]; fr(d, k + 1) = v.c[1]; fr(d, k + 2) = v.c[2]; };
    auto fl3 = [&](int k) { return s3(Fl[k * N + slot], Fl[(k + 1) * N + slot], Fl[(k + 2) * N + slot]); };
    auto setf3 = [&](int k, S3 v) { Fl[k * N + slot] = v.c[0]; Fl[(k + 1) * N + slot] = v.c[1]; Fl[(k + 2) * N + slot] = v.c[2]; };

    uint32_t st = *st_word(ps, slot);
    rays->n = 0;
    int d = I[kDlD * N + slot];
    Dims dm{&sc, hidx_of(ps, slot), (int)(st & kStDimMask), false};
    int step;
    S3 e = s3(0.f), Lc = s3(0.f);
    if (st & kStNee) {
        e = nee_value<kFt>(sc, ps, slot, st);
        st &= ~(kStNee | kStNfMask);
        step = kDlAcc;
    } else {
        st &= ~kStCont;
        step = kDlHit;
    }
    // the current frame's vertex (rebuilt from its stored ray when resuming)
    bool haveV = false;
    SurfHit si{};
    Bsdf bsdf{};
    auto vertex = [&]() {
        if (haveV) return;
        const Ray r{v3(fr(d, kFrRay), fr(d, kFrRay + 1), fr(d, kFrRay + 2)),
                    v3(fr(d, kFrRay + 3), fr(d, kFrRay + 4), fr(d, kFrRay + 5)), kInf};
        const int prim = __float_as_int(fr(d, kFrPrim));
        surface_at<Ft<kFt>::sph>(sc, prim, r, &si);
        int mat, light;
        prim_info<Ft<kFt>::sph>(sc, prim, &mat, &light);
        const float wvl0 = Ft<kFt>::spec && sc.mats[PT_IDX(mat, sc.n_mats)].kind == PT_MAT_DISPERSIVE_GLASS
                               ? (float)400 + (float)300 * halton_dim(sc, dm.idx, sc.wvl_dim) : 550.f;
        make_bsdf<kFt>(&sc.mats[PT_IDX(mat, sc.n_mats)], si, wvl0, &bsdf, false);
        haveV = true;
    };
    // one EstimateDirect: emits its rays, or yields Ld = 0 at once
    auto estimate = [&](int j, float uL0, float uL1, float uS0, float uS1) -> bool {
        vertex();
        uint32_t f;
        if (sc.lights[PT_IDX(j, sc.n_lights)].kind == PT_LIGHT_PORTAL_AREA) {
            f = portal_nee<kFt>(sc, ps, slot, j, si, bsdf, uS0, uS1);
            if (f & kNfA) rays->push(slot << 2 | kRayA);
            f &= (f & kNfA) ? ~0u : 0u;
        } else {
            f = mis_nee<kFt>(sc, ps, slot, j, si, bsdf, uL0, uL1, uS0, uS1);
            if (f & kNfA) rays->push(slot << 2 | kRayShadow);
            if (f & kNfB) rays->push(slot << 2 | kRayB);
            f &= (f & (kNfA | kNfB)) ? ~0u : 0u;
        }
        st = (st & ~kStNfMask) | (f << kStNfShift);  // the payload's flags ride in the state word
        return f != 0;
    };
    // Sampler::Get2DArray entry k of array ai: GetIndexForSample(s * n + k) (sampler.cpp:149-160)
    auto array_u = [&](int ai, int k, int n, float* u0, float* u1) {
        const uint32_t idx = (uint32_t)I[kDlPix * N + slot] +
                             ((uint32_t)I[kDlS * N + slot] * (uint32_t)n + (uint32_t)k) * sc.hal_stride;
        *u0 = halton_dim(sc, idx, 5 + 2 * ai);
        *u1 = halton_dim(sc, idx, 5 + 2 * ai + 1);
    };
    auto spawn_child = [&](S3 f, V3 wi, float pdf, int phase) {
        set3(d, kFrFac, f);
        fr(d, kFrCos) = absdot(wi, si.sn);
        fr(d, kFrPdf) = pdf;
        fr(d, kFrPhase) = __int_as_float(phase);
        const Ray r{offset_ray_origin(si.p, si.perr, si.n, wi), wi, kInf};  // SpawnRay
        store_ray(ps.ray, slot, r);
        ++d;
        haveV = false;
        st |= kStCont;
        rays->push(slot << 2 | kRayCont);
    };
    bool emitted = false;
    while (!emitted && step != kDlDone) {
        switch (step) {
            case kDlHit: {
                const Ray ray = load_ray(ps.ray, slot, kInf);
                const int hp = *hit_word(ps, slot, kHdHit);
                SurfHit h;
                const bool found = hp >= 0 && surface_at<Ft<kFt>::sph>(sc, hp, ray, &h);
                if (!found) {  // Light::Le of every light: only infinite lights emit
                    S3 Lm = s3(0.f);
                    if (Ft<kFt>::inf)
                        for (int li = 0; li < sc.n_lights; ++li)
                            if (sc.lights[PT_IDX(li, sc.n_lights)].kind == PT_LIGHT_INFINITE) Lm = Lm + inf_Le(sc.lights[PT_IDX(li, sc.n_lights)], ray.d);
                    Lc = Lm;
                    step = kDlReturn;
                    break;
                }
                int mat, light;
                prim_info<Ft<kFt>::sph>(sc, hp, &mat, &light);
                if (sc.mats[PT_IDX(mat, sc.n_mats)].kind == PT_MAT_NONE) {  // Li(isect.SpawnRay(ray.d), depth)
                    const Ray r{offset_ray_origin(h.p, h.perr, h.n, ray.d), ray.d, kInf};
                    store_ray(ps.ray, slot, r);
                    st |= kStCont;
                    rays->push(slot << 2 | kRayCont);
                    emitted = true;
                    break;
                }
                for (int c = 0; c < 3; ++c) { fr(d, kFrRay + c) = ray.o[c]; fr(d, kFrRay + 3 + c) = ray.d[c]; }
                fr(d, kFrPrim) = __int_as_float(hp);
                haveV = false;
                vertex();
                const S3 Le = light >= 0 ? area_L(sc.lights[PT_IDX(light, sc.n_lights)], si.n, si.wo) : s3(0.f);  // isect.Le(wo)
                set3(d, kFrL, s3(0.f) + Le);
                if (sc.n_lights > 0) {
                    if (sc.dl_strategy == PT_DIRECT_ALL) {
                        setf3(kDlLnee, s3(0.f));
                        I[kDlJ * N + slot] = 0;
                        step = kDlLights;
                    } else
                        step = kDlOne;
                } else
                    step = kDlSpecR;
                break;
            }
            case kDlLights: {  // UniformSampleAllLights (integrator.cpp:69-98), light j
                const int j = I[kDlJ * N + slot];
                if (j == sc.n_lights) {
                    set3(d, kFrL, fr3(d, kFrL) + fl3(kDlLnee));
                    step = kDlSpecR;
                    break;
                }
                const int n = sc.lights[PT_IDX(j, sc.n_lights)].n_samples;
                int aoff = I[kDlAoff * N + slot];
                const int a1 = aoff < sc.dl_arrays ? aoff++ : -1;
                const int a2 = aoff < sc.dl_arrays ? aoff++ : -1;
                I[kDlAoff * N + slot] = aoff;
                float uL0, uL1, uS0, uS1;
                if (a1 < 0 || a2 < 0) {
                    I[kDlMode * N + slot] = kDlModeSingle;
                    uL0 = dm.get1(); uL1 = dm.get1();
                    uS0 = dm.get1(); uS1 = dm.get1();
                } else {
                    I[kDlMode * N + slot] = kDlModeArray;
                    I[kDlK * N + slot] = 0;
                    I[kDlN * N + slot] = n;
                    I[kDlAi * N + slot] = a1;
                    setf3(kDlLd, s3(0.f));
                    array_u(a1, 0, n, &uL0, &uL1);
                    array_u(a2, 0, n, &uS0, &uS1);
                }
                if (estimate(j, uL0, uL1, uS0, uS1)) { st |= kStNee; emitted = true; }
                else { e = s3(0.f); step = kDlAcc; }
                break;
            }
            case kDlOne: {  // UniformSampleOneLight without a distribution (integrator.cpp:100-122)
                const int nl = sc.n_lights;
                const int ln = min((int)(dm.get1() * nl), nl - 1);
                Fl[kDlLpdf * N + slot] = (float)1 / nl;
                const float uL0 = dm.get1(), uL1 = dm.get1();
                const float uS0 = dm.get1(), uS1 = dm.get1();
                I[kDlMode * N + slot] = kDlModeOne;
                if (estimate(ln, uL0, uL1, uS0, uS1)) { st |= kStNee; emitted = true; }
                else { e = s3(0.f); step = kDlAcc; }
                break;
            }
            case kDlAcc: {
                const int mode = I[kDlMode * N + slot];
                if (mode == kDlModeArray) {
                    const S3 Ld = fl3(kDlLd) + e;
                    const int k = I[kDlK * N + slot] + 1, n = I[kDlN * N + slot];
                    if (k < n) {
                        setf3(kDlLd, Ld);
                        I[kDlK * N + slot] = k;
                        const int ai = I[kDlAi * N + slot];
                        float uL0, uL1, uS0, uS1;
                        array_u(ai, k, n, &uL0, &uL1);
                        array_u(ai + 1, k, n, &uS0, &uS1);
                        if (estimate(I[kDlJ * N + slot], uL0, uL1, uS0, uS1)) { st |= kStNee; emitted = true; }
                        else { e = s3(0.f); step = kDlAcc; }
                    } else {
                        setf3(kDlLnee, fl3(kDlLnee) + Ld / (float)n);
                        I[kDlJ * N + slot] += 1;
                        step = kDlLights;
                    }
                } else if (mode == kDlModeSingle) {
                    setf3(kDlLnee, fl3(kDlLnee) + e);
                    I[kDlJ * N + slot] += 1;
                    step = kDlLights;
                } else {
                    set3(d, kFrL, fr3(d, kFrL) + e / Fl[kDlLpdf * N + slot]);
                    step = kDlSpecR;
                }
                break;
            }
            case kDlSpecR:
            case kDlSpecT: {  // SpecularReflect / SpecularTransmit (integrator.cpp:639-770)
                if (step == kDlSpecR && !(d + 1 < sc.max_depth)) {
                    Lc = fr3(d, kFrL);
                    step = kDlReturn;
                    break;
                }
                const float u0 = dm.get1(), u1 = dm.get1();
                vertex();
                V3 wi = v3(0, 0, 0);
                float pdf = 0;
                int sampled = 0;
                const int type = (step == kDlSpecR ? kBxR : kBxT) | kBxSpecular;
                const S3 f = bsdf_sample<kFt>(bsdf, si.wo, &wi, u0, u1, &pdf, type, &sampled);
                if (pdf > 0.f && !is_black(f) && absdot(wi, si.sn) != 0.f) {
                    spawn_child(f, wi, pdf, step == kDlSpecR ? 0 : 1);
                    emitted = true;
                } else if (step == kDlSpecR) {
                    step = kDlSpecT;
                } else {
                    Lc = fr3(d, kFrL);
                    step = kDlReturn;
                }
                break;
            }
            case kDlReturn: {
                if (d == 0) {
                    store_Lfin(ps, slot, Lc);
                    step = kDlDone;
                    break;
                }
                --d;
                haveV = false;
                set3(d, kFrL, fr3(d, kFrL) + ((fr3(d, kFrFac) * Lc) * fr(d, kFrCos)) / fr(d, kFrPdf));
                if (__float_as_int(fr(d, kFrPhase)) == 0) step = kDlSpecT;
                else { Lc = fr3(d, kFrL); step = kDlReturn; }
                break;
            }
            default: step = kDlDone; break;
        }
    }
    I[kDlD * N + slot] = d;
    if (dm.overflow) { st |= kStDimOverflow; *overflow = true; }
    st = (st & ~kStDimMask) | (uint32_t)min(dm.dim, (int)kStDimMask);  // past max_dim only after overflow
    *st_word(ps, slot) = st;
    *keep = (st & (kStCont | kStNee)) != 0;
}

template <int kFt>
__global__ __launch_bounds__(kShadeBlock) void k_shade_dl(DevScene sc, DevPaths ps, const uint32_t* __restrict__ pq,
                                                          const uint32_t* __restrict__ pq_count, uint32_t* rq_out,
                                                          uint32_t* rq_out_count, uint32_t* pq_out,
                                                          uint32_t* pq_out_count, DevStats* stats)
#ifdef PT_TU_SHADE
{
    const uint32_t n = *pq_count;
    bool overflow = false;
    PT_WAVEQ(wq);
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        RayList rays;
        bool keep = false;
        uint32_t slot = 0;
        if (i < n) {
            slot = pq[i];
            shade_dl<kFt>(sc, ps, slot, &rays, &keep, &overflow);
        }
        wq_push(wq, rays, keep, slot, rq_out_count, rq_out, pq_out);
    }
    wq_flush(wq, rq_out_count, rq_out, pq_out);
    if (overflow) atomicAdd(&stats->dim_overflow, 1ull);
}
#else
;
#endif

// Register-budget variants of the shading kernel (occupancy vs spills), each
// compiled for a scene-feature set kFt; render.hip picks one (PT_SHADE_VARIANT,
// scene_features).
template <int kFt, bool kAb>
__global__ __launch_bounds__(kShadeBlock) void k_shade(DevScene sc, DevPaths ps, const uint32_t* __restrict__ pq,
                                                       const uint32_t* __restrict__ pq_count, uint32_t* rq_out,
                                                       uint32_t* rq_out_count, uint32_t* pq_out,
                                                       uint32_t* pq_out_count, DevStats* stats)
#ifdef PT_TU_SHADE
{
    shade_batch<kFt, false, false, kAb, kShadeAhead<kFt>>(sc, ps, pq, pq_count, rq_out, rq_out_count, pq_out, pq_out_count, stats);
}
#else
;
#endif
// The scene tables in LDS (stage_tables): scenes whose tables fit kTabLdsMax.
template <int kFt, bool kAb>
__global__ __launch_bounds__(kShadeBlock) void k_shade_tab(DevScene sc, DevPaths ps, const uint32_t* __restrict__ pq,
                                                           const uint32_t* __restrict__ pq_count, uint32_t* rq_out,
                                                           uint32_t* rq_out_count, uint32_t* pq_out,
                                                           uint32_t* pq_out_count, DevStats* stats)
#ifdef PT_TU_SHADE
{
    shade_batch<kFt, true, false, kAb, kShadeAhead<kFt>>(sc, ps, pq, pq_count, rq_out, rq_out_count, pq_out, pq_out_count, stats);
}
#else
;
#endif
// k_shade with a 3-waves-per-SIMD register budget (scene tables too large for LDS)
template <int kFt, bool kAb>
__global__ __launch_bounds__(kShadeBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_shade_w3h(
    DevScene sc, DevPaths ps, const uint32_t* __restrict__ pq, const uint32_t* __restrict__ pq_count, uint32_t* rq_out,
    uint32_t* rq_out_count, uint32_t* pq_out, uint32_t* pq_out_count, DevStats* stats)
#ifdef PT_TU_SHADE
{
    shade_batch<kFt, false, Ft<kFt>::mis, kAb>(sc, ps, pq, pq_count, rq_out, rq_out_count, pq_out, pq_out_count, stats);
}
#else
;
#endif
// k_shade_tab with a 3-waves-per-SIMD register budget (PT_SHADE_VARIANT=3)
template <int kFt, bool kAb>
__global__ __launch_bounds__(kShadeBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_shade_w3(
    DevScene sc, DevPaths ps, const uint32_t* __restrict__ pq, const uint32_t* __restrict__ pq_count, uint32_t* rq_out,
    uint32_t* rq_out_count, uint32_t* pq_out, uint32_t* pq_out_count, DevStats* stats)
#ifdef PT_TU_SHADE
{
    shade_batch<kFt, true, Ft<kFt>::mis, kAb>(sc, ps, pq, pq_count, rq_out, rq_out_count, pq_out, pq_out_count, stats);
}
#else
;
#endif


// ----------------------------------------------------------------------------
// Film: for every film pixel of the batch's region, rebuild each FilmTile's
// partial sum in the reference's order -- the tile's pixels in scan order,
// each pixel's samples in order (SamplerIntegrator::Render,
// integrator.cpp:533-560; FilmTile::AddSample film.h:121-161 + the radiance
// sanitiser integrator.cpp:592-613) -- then merge the partials tile by tile
// in tile order as XYZ (Film::MergeFilmTile film.cpp:117-130).  A pure
// gather: deterministic, no float atomics.  Bit-identical to the reference
// whenever a batch holds all samples of its tiles.
//
// One wave per film pixel: the 64 lanes evaluate 64 consecutive samples of a
// source pixel (slots are pixel-major, so the loads coalesce), then the
// touching lanes' contributions are added in lane order with readlane --
// the float sum keeps the reference's sequential association.
// ----------------------------------------------------------------------------
__device__ __forceinline__ float lane_val(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

// The radiance sanitiser of SamplerIntegrator::Render (integrator.cpp:592-613:
// NaN, negative luminance, infinite luminance -> black) and AddSample's
// maxSampleLuminance clamp (film.h:121-161).
__device__ __forceinline__ S3 film_sanitize(S3 L, float max_lum) {
    if (has_nan(L)) L = s3(0.f);
    else if ((double)lum_y(L) < -1e-5) L = s3(0.f);
    else if (__builtin_isinf(lum_y(L))) L = s3(0.f);
    if (lum_y(L) > max_lum) L = L * (max_lum / lum_y(L));
    return L;
}

__global__ __launch_bounds__(256) void k_film(DevPaths ps, FilmConsts fc, const int* __restrict__ pixslot, int p0,
                                              int np, int nsamp, int bx0, int by0, int bw, int bh, float4* accum)
#ifdef PT_TU_MISC
{
    const int cw = fc.crop_x1 - fc.crop_x0;
    const int sbw = fc.sb_x1 - fc.sb_x0;
    const int total = bw * bh;
    const int lane = (int)lane_id();
    const int nwaves = (int)(gridDim.x * blockDim.x) >> 6;
    for (int t = (int)(blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < total; t += nwaves) {
        const int tx = bx0 + t % bw, ty = by0 + t / bw;
        const int wy0 = max(ty - fc.win, fc.sb_y0), wy1 = min(ty + fc.win, fc.sb_y1 - 1);
        const int wx0 = max(tx - fc.win, fc.sb_x0), wx1 = min(tx + fc.win, fc.sb_x1 - 1);
        if (wy0 > wy1 || wx0 > wx1) continue;
        const size_t o = (size_t)(ty - fc.crop_y0) * cw + (tx - fc.crop_x0);
        float4 acc = accum[o];
        bool touched = false;
        const int ty0 = (wy0 - fc.sb_y0) >> 4, ty1 = (wy1 - fc.sb_y0) >> 4;
        const int tx0 = (wx0 - fc.sb_x0) >> 4, tx1 = (wx1 - fc.sb_x0) >> 4;
        for (int tr = ty0; tr <= ty1; ++tr) {
            for (int tc = tx0; tc <= tx1; ++tc) {
                const int qy0 = max(wy0, fc.sb_y0 + 16 * tr), qy1 = min(wy1, fc.sb_y0 + 16 * tr + 15);
                const int qx0 = max(wx0, fc.sb_x0 + 16 * tc), qx1 = min(wx1, fc.sb_x0 + 16 * tc + 15);
                float p0s = 0.f, p1s = 0.f, p2s = 0.f, wsum = 0.f;
                bool any = false;
                for (int qy = qy0; qy <= qy1; ++qy) {
                    for (int qx = qx0; qx <= qx1; ++qx) {
                        const int p = pixslot[(qy - fc.sb_y0) * sbw + (qx - fc.sb_x0)] - p0;
                        if (p < 0 || p >= np) continue;
                        for (int c0 = 0; c0 < nsamp; c0 += 64) {
                            const int sl = c0 + lane;
                            bool touch = false;
                            S3 c = s3(0.f);
                            float w = 0.f;
                            if (sl < nsamp) {
                                const uint32_t slot = (uint32_t)p * (uint32_t)nsamp + (uint32_t)sl;
                                const float2 pf = ps.pfilm[slot];
                                const float dx = pf.x - 0.5f, dy = pf.y - 0.5f;
                                const int x0 = (int)ceilf(dx - fc.rx), x1 = (int)floorf(dx + fc.rx) + 1;
                                const int y0 = (int)ceilf(dy - fc.ry), y1 = (int)floorf(dy + fc.ry) + 1;
                                touch = !(tx < x0 || tx >= x1 || ty < y0 || ty >= y1);
                                if (touch) {
                                    const S3 L = film_sanitize(load_Lfin(ps, slot), fc.max_lum);
                                    const float fxv = fabsf((tx - dx) * fc.inv_rx * 16);
                                    const float fyv = fabsf((ty - dy) * fc.inv_ry * 16);
                                    int ix = (int)floorf(fxv); ix = ix < 15 ? ix : 15;
                                    int iy = (int)floorf(fyv); iy = iy < 15 ? iy : 15;
                                    w = fc.table[iy * 16 + ix];
                                    c = (L * 1.f) * w;
                                }
                            }
                            uint64_t m = __ballot(touch);
                            if (m) any = true;
                            while (m) {
                                const int j = __ffsll((unsigned long long)m) - 1;
                                m &= m - 1;
                                p0s += lane_val(c.c[0], j);
                                p1s += lane_val(c.c[1], j);
                                p2s += lane_val(c.c[2], j);
                                wsum += lane_val(w, j);
                            }
                        }
                    }
                }
                if (!any) continue;
                // RGBSpectrum::ToXYZ (spectrum.h:64-68) of the tile pixel, merged
                acc.x += 0.412453f * p0s + 0.357580f * p1s + 0.180423f * p2s;
                acc.y += 0.212671f * p0s + 0.715160f * p1s + 0.072169f * p2s;
                acc.z += 0.019334f * p0s + 0.119193f * p1s + 0.950227f * p2s;
                acc.w += wsum;
                touched = true;
            }
        }
        if (touched && lane == 0) accum[o] = acc;
    }
}
#else
;
#endif

// k_film_t: k_film with lane = film pixel.  k_film gives a film pixel one wave
// (lane = sample) and folds the touching samples into its FilmTile sums one
// readlane at a time: a serial chain of dependent adds per pixel, ~16 K long
// at 1024 spp with the 2-pixel Gaussian (C3: 20.9 ms per launch).  Here a wave
// owns an 8 x 8 square of film pixels and walks the source pixels their filter
// windows reach -- FilmTile by FilmTile (tile row, tile column), scan order
// within a tile, samples in order -- 64 samples at a time: lane j loads sample
// j, applies the sanitiser and maxSampleLuminance (film.h AddSample's caller,
// integrator.cpp:568-600) and finds its pixel bounds, then the samples that
// reach the square are broadcast one by one and every lane adds the ones
// touching its pixel.  Each film pixel sees its samples in k_film's order and
// does k_film's operations, so the sums are bit-identical; the 64 pixels'
// chains run side by side.
__global__ __launch_bounds__(256) void k_film_t(DevPaths ps, FilmConsts fc, const int* __restrict__ pixslot, int p0,
                                                int np, int nsamp, int bx0, int by0, int bw, int bh, float4* accum)
#ifdef PT_TU_MISC
{
    __shared__ float s_tab[256];
    if (threadIdx.x < 256) s_tab[threadIdx.x] = fc.table[threadIdx.x];
    __syncthreads();
    const int cw = fc.crop_x1 - fc.crop_x0;
    const int sbw = fc.sb_x1 - fc.sb_x0;
    const int lane = (int)lane_id();
    const int nbx = (bw + 7) >> 3, nsq = nbx * ((bh + 7) >> 3);
    const int sq = (int)__builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (sq >= nsq) return;
    const int gx0 = bx0 + (sq % nbx) * 8, gy0 = by0 + (sq / nbx) * 8;
    const int gx1 = min(gx0 + 7, bx0 + bw - 1), gy1 = min(gy0 + 7, by0 + bh - 1);
    const int tx = gx0 + (lane & 7), ty = gy0 + (lane >> 3);
    const bool on = tx <= gx1 && ty <= gy1 && max(ty - fc.win, fc.sb_y0) <= min(ty + fc.win, fc.sb_y1 - 1) &&
                    max(tx - fc.win, fc.sb_x0) <= min(tx + fc.win, fc.sb_x1 - 1);
    const size_t o = (size_t)(ty - fc.crop_y0) * cw + (tx - fc.crop_x0);
    float4 acc = on ? accum[o] : make_float4(0.f, 0.f, 0.f, 0.f);
    bool touched = false;
    const int rx0 = max(gx0 - fc.win, fc.sb_x0), rx1 = min(gx1 + fc.win, fc.sb_x1 - 1);
    const int ry0 = max(gy0 - fc.win, fc.sb_y0), ry1 = min(gy1 + fc.win, fc.sb_y1 - 1);
    if (rx0 <= rx1 && ry0 <= ry1) {
        for (int tr = (ry0 - fc.sb_y0) >> 4; tr <= (ry1 - fc.sb_y0) >> 4; ++tr) {
            for (int tc = (rx0 - fc.sb_x0) >> 4; tc <= (rx1 - fc.sb_x0) >> 4; ++tc) {
                const int qy0 = max(ry0, fc.sb_y0 + 16 * tr), qy1 = min(ry1, fc.sb_y0 + 16 * tr + 15);
                const int qx0 = max(rx0, fc.sb_x0 + 16 * tc), qx1 = min(rx1, fc.sb_x0 + 16 * tc + 15);
                float p0s = 0.f, p1s = 0.f, p2s = 0.f, wsum = 0.f;  // this pixel's FilmTile contribSum
                bool any = false;
                for (int qy = qy0; qy <= qy1; ++qy) {
                    for (int qx = qx0; qx <= qx1; ++qx) {
                        const int p = pixslot[(qy - fc.sb_y0) * sbw + (qx - fc.sb_x0)] - p0;
                        if (p < 0 || p >= np) continue;
                        for (int c0 = 0; c0 < nsamp; c0 += 64) {
                            const int sl = c0 + lane;
                            // lane = sample sl: bounds, sanitised radiance, and whether it reaches the square
                            float dx = 0.f, dy = 0.f;
                            S3 L = s3(0.f);
                            int x0 = 0, x1 = 0, y0 = 0, y1 = 0;
                            bool reach = false;
                            if (sl < nsamp) {
                                const uint32_t slot = (uint32_t)p * (uint32_t)nsamp + (uint32_t)sl;
                                const float2 pf = ps.pfilm[slot];
                                dx = pf.x - 0.5f;
                                dy = pf.y - 0.5f;
                                x0 = (int)ceilf(dx - fc.rx); x1 = (int)floorf(dx + fc.rx) + 1;
                                y0 = (int)ceilf(dy - fc.ry); y1 = (int)floorf(dy + fc.ry) + 1;
                                reach = !(gx1 < x0 || gx0 >= x1 || gy1 < y0 || gy0 >= y1);
                                if (reach) {
                                    L = film_sanitize(load_Lfin(ps, slot), fc.max_lum);
                                }
                            }
                            // the bounds relative to the square's corner, one byte each (|offset| <= 8 + win)
                            const uint32_t bb = (uint32_t)(uint8_t)(x0 - gx0 + 64) | (uint32_t)(uint8_t)(x1 - gx0 + 64) << 8 |
                                                (uint32_t)(uint8_t)(y0 - gy0 + 64) << 16 | (uint32_t)(uint8_t)(y1 - gy0 + 64) << 24;
                            uint64_t m = __ballot(reach);
                            const int lx = (lane & 7) + 64, ly = (lane >> 3) + 64;
                            while (m) {
                                const int j = __ffsll((unsigned long long)m) - 1;
                                m &= m - 1;
                                const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)bb, j);
                                const bool touch = on && !(lx < (int)(b & 255u) || lx >= (int)((b >> 8) & 255u) ||
                                                           ly < (int)((b >> 16) & 255u) || ly >= (int)(b >> 24));
                                if (touch) {
                                    const float sdx = lane_val(dx, j), sdy = lane_val(dy, j);
                                    const float fxv = fabsf((tx - sdx) * fc.inv_rx * 16);
                                    const float fyv = fabsf((ty - sdy) * fc.inv_ry * 16);
                                    int ix = (int)floorf(fxv); ix = ix < 15 ? ix : 15;
                                    int iy = (int)floorf(fyv); iy = iy < 15 ? iy : 15;
                                    const float w = s_tab[iy * 16 + ix];
                                    const S3 c = (s3(lane_val(L.c[0], j), lane_val(L.c[1], j), lane_val(L.c[2], j)) * 1.f) * w;
                                    p0s += c.c[0];
                                    p1s += c.c[1];
                                    p2s += c.c[2];
                                    wsum += w;
                                    any = true;
                                }
                            }
                        }
                    }
                }
                if (!any) continue;
                // RGBSpectrum::ToXYZ (spectrum.h:64-68) of the tile pixel, merged
                acc.x += 0.412453f * p0s + 0.357580f * p1s + 0.180423f * p2s;
                acc.y += 0.212671f * p0s + 0.715160f * p1s + 0.072169f * p2s;
                acc.z += 0.019334f * p0s + 0.119193f * p1s + 0.950227f * p2s;
                acc.w += wsum;
                touched = true;
            }
        }
    }
    if (touched) accum[o] = acc;
}
#else
;
#endif

// k_film_prep: the batch's finished radiance sanitised in place before
// k_film_sk reads it -- once per sample, where the film pass would repeat it
// for every film pixel the sample reaches (film_sanitize, above).
__global__ __launch_bounds__(256) void k_film_prep(DevPaths ps, float max_lum, uint32_t n)
#ifdef PT_TU_MISC
{
    for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < n; slot += gridDim.x * blockDim.x) {
        const S3 L = film_sanitize(load_Lfin(ps, slot), max_lum);
        float* p = ps.Lfin + 3u * slot;
        p[0] = L.c[0]; p[1] = L.c[1]; p[2] = L.c[2];
    }
}
#else
;
#endif

// k_film_sk: the RGB film with one lane per film pixel and the lanes' walks
// skewed so that lanes needing the same source pixel read it together.
//
// A film pixel's FilmTile sum is one serial chain (its window's source pixels
// in scan order, each pixel's samples in order), so a film pass can only
// choose which chains run side by side and when each reads its samples.
// k_film gives a chain a wave (lane = sample, readlane-ordered adds); k_film_t
// gives it a lane but walks every sample that reaches an 8 x 8 square, a
// quarter of the lanes touching each.  Here a wave (one per block) owns
// A x W film pixels (W = 2 win + 1 window rows, A = 64 / W columns: 12 x 5 for
// the 2-pixel Gaussian) and lane (a, b) walks its own window -- step
// k = 0..W^2-1 is source pixel (k mod W, k / W) of the window, all its samples
// -- starting at step t0 of the wave's clock:
//   skew 2: t0 = a + W b.  At clock t lane (a, b) reads source pixel
//     (Fx - win + a + k mod W, Fy - win + b + k / W), k = t - t0, and
//     a + k mod W + W (b + k / W) = t: every lane that needs a source pixel
//     reads it at the same clock step, sample for sample, so the wave reads
//     each source pixel of its region once (at most 64 / W + 1 distinct pixels
//     per load instruction), over A + 2 W^2 - W - 1 steps;
//   skew 1: t0 = a -- a source pixel is read once per window row that needs
//     it, over A + W^2 - 1 steps;
//   skew 0: no skew -- W^2 steps, every lane its own source pixel.
// The kernel is bound by the lanes' serial walks (one wave per SIMD), so the
// step count weighs against the loads shared.
//
// The per-sample footprint comes from k_camera's FilmMeta record (filter-table
// index and reach per offset: AddSample's bounds and weight, film.h:121-161,
// computed from pFilm as k_film computes them), the radiance is sanitised
// beforehand by k_film_prep, and a sample's contribution is
// formed without branches -- a sample that does not reach the lane's pixel
// adds +0, which leaves a sum that starts at +0 bit-identical.  Sums per
// FilmTile of the window (at most 2 x 2 tiles for win <= 2) are merged as XYZ
// in tile order: k_film's operations in k_film's order, bit-identical.
__global__ __launch_bounds__(64) void k_film_sk(DevPaths ps, FilmConsts fc, const int* __restrict__ pixslot, int p0,
                                                int np, int nsamp, int bx0, int by0, int bw, int bh, float4* accum,
                                                int skew)
#ifdef PT_TU_MISC
{
    __shared__ float s_tab[256];
    for (int i = (int)threadIdx.x; i < 256; i += 64) s_tab[i] = fc.table[i];
    __syncthreads();
    const int win = fc.win, W = 2 * win + 1, A = 64 / W;
    const int lane = (int)lane_id();
    const int b = lane / A, a = lane - b * A;
    const int nbx = (bw + A - 1) / A, nby = (bh + W - 1) / W;
    const int wv = (int)blockIdx.x;
    if (wv >= nbx * nby) return;
    const int tx = bx0 + (wv % nbx) * A + a, ty = by0 + (wv / nbx) * W + b;
    const int wx0 = max(tx - win, fc.sb_x0), wx1 = min(tx + win, fc.sb_x1 - 1);
    const int wy0 = max(ty - win, fc.sb_y0), wy1 = min(ty + win, fc.sb_y1 - 1);
    const bool on = b < W && tx < bx0 + bw && ty < by0 + bh && wx0 <= wx1 && wy0 <= wy1;
    const int tc0 = (wx0 - fc.sb_x0) >> 4, tr0 = (wy0 - fc.sb_y0) >> 4;
    const int sbw = fc.sb_x1 - fc.sb_x0;
    const int t0 = (skew >= 1 ? a : 0) + (skew >= 2 ? W * b : 0);
    const int nsteps = W * W + (skew >= 1 ? A - 1 : 0) + (skew >= 2 ? W * (W - 1) : 0);
    const uint2* __restrict__ meta = reinterpret_cast<const uint2*>(ps.pfilm);
    const float* __restrict__ Lf = ps.Lfin;
    float P[4][4];  // per window FilmTile (row-major 2 x 2): contribSum r, g, b, filterWeightSum
#pragma unroll
    for (int i = 0; i < 4; ++i) P[i][0] = P[i][1] = P[i][2] = P[i][3] = 0.f;
    uint32_t anyq = 0;
    for (int t = 0; t < nsteps; ++t) {
        const int k = t - t0;
        const int ky = k >= 0 ? k / W : 0, kx = k - ky * W;
        const int qx = tx + kx - win, qy = ty + ky - win;
        int p = -1;
        if (on && k >= 0 && k < W * W && qx >= wx0 && qx <= wx1 && qy >= wy0 && qy <= wy1)
            p = pixslot[(qy - fc.sb_y0) * sbw + (qx - fc.sb_x0)] - p0;
        if (p >= 0 && p < np) {
            const int quad = (((qy - fc.sb_y0) >> 4) - tr0) * 2 + (((qx - fc.sb_x0) >> 4) - tc0);
            const uint32_t ox = (uint32_t)(tx - qx + win), oy = (uint32_t)(ty - qy + win);
            const uint32_t sx = 4u * ox, sy = 4u * oy, rx = 20u + ox, ry = 20u + oy;
            float c0 = quad == 0 ? P[0][0] : quad == 1 ? P[1][0] : quad == 2 ? P[2][0] : P[3][0];
            float c1 = quad == 0 ? P[0][1] : quad == 1 ? P[1][1] : quad == 2 ? P[2][1] : P[3][1];
            float c2 = quad == 0 ? P[0][2] : quad == 1 ? P[1][2] : quad == 2 ? P[2][2] : P[3][2];
            float cw = quad == 0 ? P[0][3] : quad == 1 ? P[1][3] : quad == 2 ? P[2][3] : P[3][3];
            uint32_t any = 0;
            // sample contribution: L * w and w (L sanitised by k_film_prep), or +0 where the sample does not
            // reach the pixel
            auto contrib = [&](uint2 m, float lr, float lg, float lb, float o[4]) {
                const uint32_t touch = (m.x >> rx) & (m.y >> ry) & 1u;
                const S3 L = s3(lr, lg, lb);
                const float w = s_tab[((m.y >> sy) & 15u) * 16u + ((m.x >> sx) & 15u)];
                const S3 c = L * w;
                o[0] = touch ? c.c[0] : 0.f;
                o[1] = touch ? c.c[1] : 0.f;
                o[2] = touch ? c.c[2] : 0.f;
                o[3] = touch ? w : 0.f;
                any |= touch;
            };
            auto add = [&](const float o[4]) {
                c0 += o[0];
                c1 += o[1];
                c2 += o[2];
                cw += o[3];
            };
            const uint32_t base = (uint32_t)p * (uint32_t)nsamp;
            if ((nsamp & 3) == 0) {
                // four samples per iteration (two 16-B meta loads, three 16-B radiance loads), the next
                // four loaded before this four are formed; the four adds stay in sample order
                const uint4* mp = reinterpret_cast<const uint4*>(meta + base);
                const float4* lp = reinterpret_cast<const float4*>(Lf + 3u * base);
                uint4 m01 = mp[0], m23 = mp[1];
                float4 l0 = lp[0], l1 = lp[1], l2 = lp[2];
                for (int s = 0; s < nsamp; s += 4) {
                    uint4 n01 = m01, n23 = m23;
                    float4 n0 = l0, n1 = l1, n2 = l2;
                    if (s + 4 < nsamp) {
                        const int g = (s >> 2) + 1;
                        n01 = mp[2 * g];
                        n23 = mp[2 * g + 1];
                        n0 = lp[3 * g];
                        n1 = lp[3 * g + 1];
                        n2 = lp[3 * g + 2];
                    }
                    float o0[4], o1[4], o2[4], o3[4];
                    contrib(make_uint2(m01.x, m01.y), l0.x, l0.y, l0.z, o0);
                    contrib(make_uint2(m01.z, m01.w), l0.w, l1.x, l1.y, o1);
                    contrib(make_uint2(m23.x, m23.y), l1.z, l1.w, l2.x, o2);
                    contrib(make_uint2(m23.z, m23.w), l2.y, l2.z, l2.w, o3);
                    add(o0);
                    add(o1);
                    add(o2);
                    add(o3);
                    m01 = n01; m23 = n23;
                    l0 = n0; l1 = n1; l2 = n2;
                }
            } else {
                for (int s = 0; s < nsamp; ++s) {
                    const uint32_t slot = base + (uint32_t)s;
                    float o[4];
                    contrib(meta[slot], Lf[3u * slot], Lf[3u * slot + 1u], Lf[3u * slot + 2u], o);
                    add(o);
                }
            }
            if (any) anyq |= 1u << quad;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (quad == i) {
                    P[i][0] = c0;
                    P[i][1] = c1;
                    P[i][2] = c2;
                    P[i][3] = cw;
                }
            }
        }
        if (on && k == W * W - 1 && anyq) {
            const size_t o = (size_t)(ty - fc.crop_y0) * (fc.crop_x1 - fc.crop_x0) + (tx - fc.crop_x0);
            float4 acc = accum[o];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (!((anyq >> i) & 1u)) continue;
                // RGBSpectrum::ToXYZ (spectrum.h:64-68) of the tile pixel, merged in tile order
                acc.x += 0.412453f * P[i][0] + 0.357580f * P[i][1] + 0.180423f * P[i][2];
                acc.y += 0.212671f * P[i][0] + 0.715160f * P[i][1] + 0.072169f * P[i][2];
                acc.z += 0.019334f * P[i][0] + 0.119193f * P[i][1] + 0.950227f * P[i][2];
                acc.w += P[i][3];
            }
            accum[o] = acc;
        }
    }
}
#else
;
#endif

// ----------------------------------------------------------------------------
// Test hooks (parity unit tests through the C ABI)
// ----------------------------------------------------------------------------
__global__ void k_debug_halton(DevScene sc, const uint32_t* idx, const int* dims, int n, float* out)
#ifdef PT_TU_MISC
{
    // both table paths: the shading kernel's LDS-staged one (two digits per
    // step) is returned; a disagreement with the global-table path is a NaN
    extern __shared__ uint4 dbg_lds[];
    const HalLds hl = stage_halton(sc, dbg_lds);
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (dims[i] >= sc.max_dim) { out[i] = -1.f; return; }
    const float a = halton_dim(sc, hl, idx[i], dims[i]), b = halton_dim(sc, idx[i], dims[i]);
    out[i] = __float_as_uint(a) == __float_as_uint(b) ? a : __uint_as_float(0x7fc00000u);
}
#else
;
#endif
__global__ void k_debug_pixel_offset(DevScene sc, HaltonPixelConsts hp, const int2* pix, int n, uint32_t* out)
#ifdef PT_TU_MISC
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = halton_pixel_offset(sc, pix[i].x, pix[i].y, hp.exp1, hp.scale0, hp.mi0, hp.mi1);
}
#else
;
#endif
__global__ void k_debug_camera(DevScene sc, const float* film, int n, float* out)
#ifdef PT_TU_MISC
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r = camera_ray(sc, film[2 * i], film[2 * i + 1], 0.5f, 0.5f);
    out[6 * i] = r.o.x; out[6 * i + 1] = r.o.y; out[6 * i + 2] = r.o.z;
    out[6 * i + 3] = r.d.x; out[6 * i + 4] = r.d.y; out[6 * i + 5] = r.d.z;
}
#else
;
#endif
__global__ __launch_bounds__(kTraceBlock) void k_debug_trace(DevScene sc, const float* rays, int n, int any,
                                                             int* spill, int* out_prim)
#ifdef PT_TU_MISC
{
    __shared__ int stk[kStackLds][kTraceBlock];
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r{v3(rays[7 * i], rays[7 * i + 1], rays[7 * i + 2]), v3(rays[7 * i + 3], rays[7 * i + 4], rays[7 * i + 5]),
          rays[7 * i + 6]};
    unsigned long long a = 0, b = 0;
    int* sp = spill + (size_t)i * (64 - kStackLds);
    out_prim[i] = any ? traverse<true>(sc, sc.nodes, sc.prims, r, stk, sp, &a, &b)
                      : traverse<false>(sc, sc.nodes, sc.prims, r, stk, sp, &a, &b);
}
#else
;
#endif

// BSDF of scene material `mat` in the local frame n = (0,0,1): for each i,
// in[8i..]: wo(3), wi(3), u0, u1 -> out[8i..]: f(3), pdf, sampled wi(3), sampled pdf
// (sampled f replaces f when in wi is all zero).
__global__ void k_debug_bsdf(DevScene sc, int mat, const float* in, int n, float* out)
#ifdef PT_TU_MISC
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* a = in + 8 * i;
    SurfHit si{};
    si.n = v3(0, 0, 1); si.sn = v3(0, 0, 1); si.sdpdu = v3(1, 0, 0);
    Bsdf b;
    make_bsdf(&sc.mats[PT_IDX(mat, sc.n_mats)], si, 550.f, &b, sc.integrator != PT_INTEGRATOR_DIRECT);
    const V3 wo = v3(a[0], a[1], a[2]), wi = v3(a[3], a[4], a[5]);
    float* o = out + 8 * i;
    S3 f = s3(0.f);
    float pdf = 0;
    if (wi.x != 0 || wi.y != 0 || wi.z != 0) {
        f = bsdf_f(b, wo, wi, kBxAll);
        pdf = bsdf_pdf(b, wo, wi, kBxAll);
    }
    V3 ws = v3(0, 0, 0);
    float spdf = 0;
    int sampled = 0;
    const S3 sf = bsdf_sample(b, wo, &ws, a[6], a[7], &spdf, kBxAll, &sampled);
    if (wi.x == 0 && wi.y == 0 && wi.z == 0) f = sf;
    o[0] = f.c[0]; o[1] = f.c[1]; o[2] = f.c[2]; o[3] = pdf;
    o[4] = ws.x; o[5] = ws.y; o[6] = ws.z; o[7] = spdf;
}
#else
;
#endif

}  // namespace pt
