// fetch_calib -- known-byte access kernels for calibrating rocprofv3's
// FETCH_SIZE / WRITE_SIZE on the access shapes of the shading kernels.
//
// MI355X_MICROARCH.md (HBM section) establishes FETCH_SIZE = 1/2 of the bytes
// only for wide coalesced streaming reads; the shading kernels read and write
// 4-, 12-, 16- and 32-byte pieces of per-slot state at slots spread over a
// 64 M-slot batch (the compacted path queue).  Each kernel here moves a known
// number of bytes in one of those shapes over arrays far larger than the
// Infinity Cache (2 GiB of 32-B records), so the counters' bytes per
// algorithmic byte can be read off per access class:
//
//   k_rd<W, kRand> / k_wr<W, kRand>: every lane reads / writes W bytes
//   (W = 4: a SoA word; 12: a float3 in a 32-B record; 16: a float4 in one;
//   32: the whole record) of slot s = perm(i), i over all 64 M slots, where
//   perm is the identity (kRand = false: coalesced) or i * 0x9E3779B1 mod 2^26
//   (kRand = true: a bijection that spreads a wave's 64 slots over the array).
//
// usage: fetch_calib [reps]  -- prints one JSON line per kernel with its
// algorithmic bytes per launch; rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
// of the same command give the counters (scripts/fetch_calib_summary.py).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                                    \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

constexpr uint32_t kLog2Slots = 26;  // 64 M slots (the default shading batch when calibrated in round 5; 96 M since)
constexpr uint32_t kSlots = 1u << kLog2Slots;

__device__ __forceinline__ uint32_t perm(uint32_t i, bool rnd) {
    return rnd ? (i * 0x9E3779B1u) & (kSlots - 1u) : i;
}

// W-byte read of slot s: from a SoA word array (W = 4) or the 32-B records
template <int W, bool kRand>
__global__ __launch_bounds__(256) void k_rd(const float4* __restrict__ rec, const float* __restrict__ soa,
                                            float* __restrict__ sink) {
    float acc = 0.f;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kSlots; i += gridDim.x * blockDim.x) {
        const uint32_t s = perm(i, kRand);
        if constexpr (W == 4) {
            acc += soa[s];
        } else if constexpr (W == 12) {
            const float3 v = *reinterpret_cast<const float3*>(rec + 2u * s);
            acc += v.x + v.y + v.z;
        } else if constexpr (W == 16) {
            const float4 v = rec[2u * s];
            acc += v.x + v.y + v.z + v.w;
        } else {
            const float4 v = rec[2u * s], u = rec[2u * s + 1u];
            acc += v.x + v.y + v.z + v.w + u.x + u.y + u.z + u.w;
        }
    }
    if (acc == 12345.678f) sink[0] = acc;  // keeps the loads; never true for the zero-filled arrays
}

template <int W, bool kRand>
__global__ __launch_bounds__(256) void k_wr(float4* __restrict__ rec, float* __restrict__ soa, float val) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kSlots; i += gridDim.x * blockDim.x) {
        const uint32_t s = perm(i, kRand);
        const float v = val + (float)(i & 7u);
        if constexpr (W == 4) {
            soa[s] = v;
        } else if constexpr (W == 12) {
            *reinterpret_cast<float3*>(rec + 2u * s) = make_float3(v, v, v);
        } else if constexpr (W == 16) {
            rec[2u * s] = make_float4(v, v, v, v);
        } else {
            rec[2u * s] = make_float4(v, v, v, v);
            rec[2u * s + 1u] = make_float4(v, v, v, v);
        }
    }
}

template <int W, bool kRand>
static void run(const char* name, float4* rec, float* soa, float* sink, int reps, hipEvent_t a, hipEvent_t b) {
    const dim3 grid(256 * 32), block(256);
    float ms = 0;
    for (int r = 0; r < reps; ++r) {
        CHK(hipEventRecord(a));
        if (name[1] == 'r' && name[2] == 'd') hipLaunchKernelGGL((k_rd<W, kRand>), grid, block, 0, 0, rec, soa, sink);
        else hipLaunchKernelGGL((k_wr<W, kRand>), grid, block, 0, 0, rec, soa, 1.f);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float t = 0;
        CHK(hipEventElapsedTime(&t, a, b));
        ms += t;
    }
    const double bytes = (double)W * kSlots;
    std::printf("{\"kernel\": \"k_%s<%d, %s>\", \"width\": %d, \"random\": %s, \"algorithmic_bytes_per_launch\": %.0f, "
                "\"avg_ms\": %.4f, \"GBs\": %.1f}\n",
                name + 1, W, kRand ? "true" : "false", W, kRand ? "true" : "false", bytes, ms / reps,
                bytes / (ms / reps * 1e-3) / 1e9);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
    float4* rec = nullptr;
    float* soa = nullptr;
    float* sink = nullptr;
    CHK(hipMalloc(&rec, (size_t)kSlots * 32));
    CHK(hipMalloc(&soa, (size_t)kSlots * 4));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(rec, 0, (size_t)kSlots * 32));
    CHK(hipMemset(soa, 0, (size_t)kSlots * 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    run<4, false>("_rd", rec, soa, sink, reps, a, b);
    run<4, true>("_rd", rec, soa, sink, reps, a, b);
    run<12, true>("_rd", rec, soa, sink, reps, a, b);
    run<16, true>("_rd", rec, soa, sink, reps, a, b);
    run<32, false>("_rd", rec, soa, sink, reps, a, b);
    run<32, true>("_rd", rec, soa, sink, reps, a, b);
    run<4, false>("_wr", rec, soa, sink, reps, a, b);
    run<4, true>("_wr", rec, soa, sink, reps, a, b);
    run<12, true>("_wr", rec, soa, sink, reps, a, b);
    run<16, true>("_wr", rec, soa, sink, reps, a, b);
    run<32, false>("_wr", rec, soa, sink, reps, a, b);
    run<32, true>("_wr", rec, soa, sink, reps, a, b);
    CHK(hipFree(rec));
    CHK(hipFree(soa));
    CHK(hipFree(sink));
    return 0;
}
