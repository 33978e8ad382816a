// tu_misc.hip -- translation unit of the camera, film and debug kernels (kernels.hip).
#define PT_TU_MISC 1
#include "kernels.hip"

namespace pt {
template __global__ void k_camera<false>(DevScene, DevPaths, const int2*, int, int, int, HaltonPixelConsts, uint32_t*,
                                         uint32_t*, FilmMeta);
template __global__ void k_camera<true>(DevScene, DevPaths, const int2*, int, int, int, HaltonPixelConsts, uint32_t*,
                                        uint32_t*, FilmMeta);
}  // namespace pt
