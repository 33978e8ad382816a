// kernels.h -- launch geometry and small constant blocks shared by the
// wavefront kernels and the host driver.
#pragma once

#include "device.h"

namespace pt {

constexpr int kTraceBlock = 128;       // 2 waves; LDS stack = kStackLds * 128 * 4 B
constexpr int kOctBlock = 448;         // k_trace_oct: 7 waves per block, 4 blocks per CU
constexpr uint32_t kTraceChunk = 512;  // ray-queue entries a k_trace_nb wave takes per atomic
// k_trace_nb: node visits / primitive tests per loop iteration for lanes that
// stay in node / leaf mode (the loop's refill and step-kind bookkeeping is paid
// once per iteration); C2: 1/1 -> 6/2 took the kernel from 14.2 to 9.2 ms
#ifndef PT_NODE_STEPS
#define PT_NODE_STEPS 6
#endif
#ifndef PT_LEAF_STEPS
#define PT_LEAF_STEPS 2
#endif
constexpr int kNodeSteps = PT_NODE_STEPS;
constexpr int kLeafSteps = PT_LEAF_STEPS;
constexpr int kStackLds = 20;     // LDS-resident part of the 64-entry BVH stack
constexpr int kSpillWords = 64 - kStackLds;  // k_trace_pt: global spill entries per lane beyond the LDS rows
constexpr int kWideLdsRowsMax = 24;  // k_trace_w<true>: LDS stack rows per lane (12 blocks of 128 lanes per CU)
constexpr int kShadeBlock = 128;
constexpr int kShadeBpcW3 = 36;       // k_shade_w3 blocks per CU (six rounds of its 6 resident blocks; 24: C2 k_shade 5.97 vs 5.88 ms)
constexpr int kMaxPortals = PT_MAX_PORTALS;  // include/pt.h
constexpr int kLdsSceneMax = 16384;  // bytes of BVH nodes + prim records staged in LDS by k_trace<true>
constexpr size_t kTabLdsMax = 8192;   // bytes of scene tables k_shade_tab stages in LDS after the Halton tables
constexpr size_t kHalLdsMax = 28672;  // bytes of Halton tables staged in LDS by k_shade (DevScene::hal_lds_dims)

// HaltonSampler constants for the per-pixel offset (halton.cpp:65-93)
struct HaltonPixelConsts {
    int exp1;
    uint32_t scale0;
    uint32_t mi0, mi1;
};

// Film constants (film.cpp:45-86, film.h:121-161)
struct FilmConsts {
    int crop_x0, crop_y0, crop_x1, crop_y1;
    int sb_x0, sb_y0, sb_x1, sb_y1;
    int win;  // filter window half-size in pixels
    float rx, ry, inv_rx, inv_ry;
    float max_lum;
    float table[256];
};

// k_film_sk's per-sample footprint record, which k_camera stores in place of
// pFilm (DevPaths::pfilm as uint2) when win > 0: per axis, for the film pixel
// offsets o = 0..2win (pixel q + o - win), the filter-table index (4 bits at
// 4o) and whether AddSample's bounds reach it (bit 20 + o).  win <= 2.
struct FilmMeta {
    int win;  // 0: k_camera stores pFilm
    float rx, ry, inv_rx, inv_ry;
};
constexpr int kFilmSkMaxWin = 2;

}  // namespace pt
