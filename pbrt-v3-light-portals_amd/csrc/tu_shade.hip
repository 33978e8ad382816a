// tu_shade.hip -- translation unit of the path-vertex shading kernels
// (kernels.hip), one object per scene-feature set: compiled with
// -DPT_FT=<kFt> (all instantiated feature sets when PT_FT is undefined;
// 99: the DirectLighting kernel).
#define PT_TU_SHADE 1
#include "kernels.hip"

namespace pt {
#define PT_ARGS DevScene, DevPaths, const uint32_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, DevStats*
// each variant with and without the algorithmic-byte count (kAb)
#define PT_SHADE_FT(F)                                       \
    template __global__ void k_shade<F, false>(PT_ARGS);     \
    template __global__ void k_shade_tab<F, false>(PT_ARGS); \
    template __global__ void k_shade_w3<F, false>(PT_ARGS);  \
    template __global__ void k_shade_w3h<F, false>(PT_ARGS); \
    template __global__ void k_shade_w3h<F, true>(PT_ARGS);  \
    template __global__ void k_shade<F, true>(PT_ARGS);      \
    template __global__ void k_shade_tab<F, true>(PT_ARGS);  \
    template __global__ void k_shade_w3<F, true>(PT_ARGS);
#if !defined(PT_FT) || PT_FT == 0
PT_SHADE_FT(0)
#endif
#if !defined(PT_FT) || PT_FT == 4
PT_SHADE_FT(kFtInfinite)
#endif
#if !defined(PT_FT) || PT_FT == 8
PT_SHADE_FT(kFtSphere)
#endif
#if !defined(PT_FT) || PT_FT == 12
PT_SHADE_FT(kFtInfinite | kFtSphere)
#endif
#if !defined(PT_FT) || PT_FT == 7
PT_SHADE_FT(kFtMicro | kFtSpecular | kFtInfinite)
#endif
#if !defined(PT_FT) || PT_FT == 15
PT_SHADE_FT(kFtAll)
#endif
#if !defined(PT_FT) || PT_FT == 16
PT_SHADE_FT(kFtPortalOnly)
#endif
#if !defined(PT_FT) || PT_FT == 99
template __global__ void k_shade_dl<kFtAll>(PT_ARGS);
#endif
#undef PT_SHADE_FT
#undef PT_ARGS
}  // namespace pt
