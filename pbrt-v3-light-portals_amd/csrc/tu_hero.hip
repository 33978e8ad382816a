// tu_hero.hip -- translation unit of the hero-wavelength kernels (hero.hip).
#define PT_TU_HERO 1
#include "hero.hip"

namespace pt {
// hero shading kernels per scene-feature set (devfuncs.h kFt*): matte-only,
// smooth specular (glass, dispersive glass, mirror), specular + an infinite
// light, no spheres, everything
#define PT_ARGS DevScene, DevHero, DevPaths, DevHeroPaths, const uint32_t*, const uint32_t*, uint32_t*, uint32_t*, \
                uint32_t*, uint32_t*, DevStats*
#define PT_HERO_FT(F)                                 \
    template __global__ void k_shade_hero<F>(PT_ARGS);    \
    template __global__ void k_shade_hero_w2<F>(PT_ARGS); \
    template __global__ void k_shade_hero_w4<F>(PT_ARGS);
PT_HERO_FT(0)
PT_HERO_FT(kFtSpecular)
PT_HERO_FT(kFtSpecular | kFtInfinite)
PT_HERO_FT(kFtMicro | kFtSpecular | kFtInfinite)
PT_HERO_FT(kFtAll)
#undef PT_HERO_FT
#undef PT_ARGS
#define PT_FILM_ARGS DevHero, DevPaths, FilmConsts, const int*, int, int, int, int, int, int, int, float4*
template __global__ void k_film_s60_sq<2, 2, 16>(PT_FILM_ARGS);
#undef PT_FILM_ARGS
}  // namespace pt
